# pool cliff mechanism: heavy-first ray order (SURF_KEY=2) vs ascending (1) across pool sizes and k_extend grids
mkdir -p gpurun_out/r4/cliff
bash tools/ab.sh gpurun_out/r4/cliff 'k1p45|SURF_KEY=1|--pool 4147200' 'k2p45|SURF_KEY=2|--pool 4147200' \
  'k1p50|SURF_KEY=1|' 'k2p50|SURF_KEY=2|' 'k1g56|SURF_KEY=1,SURF_GRID_EXTEND=56|' 'k2g56|SURF_KEY=2,SURF_GRID_EXTEND=56|' \
  'k1g72|SURF_KEY=1,SURF_GRID_EXTEND=72|' 'k2g72|SURF_KEY=2,SURF_GRID_EXTEND=72|' 'k2g36|SURF_KEY=2,SURF_GRID_EXTEND=36|' 'k1p50b|SURF_KEY=1|'
