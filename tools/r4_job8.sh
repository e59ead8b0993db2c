# heavy-first ray order (SURF_KEY=2): pool-size and k_extend-grid sweep
mkdir -p gpurun_out/r4/cliff2
bash tools/ab.sh gpurun_out/r4/cliff2 'k2p35|SURF_KEY=2|--pool 3225600' 'k2p40|SURF_KEY=2|--pool 3686400' \
  'k2p45|SURF_KEY=2|--pool 4147200' 'k2p50|SURF_KEY=2|' 'k2p60|SURF_KEY=2|--pool 5529600' 'k2p70|SURF_KEY=2|--pool 6451200' \
  'k2g52|SURF_KEY=2,SURF_GRID_EXTEND=52|' 'k2g60|SURF_KEY=2,SURF_GRID_EXTEND=60|' 'k1p50|SURF_KEY=1|' 'k2p50b|SURF_KEY=2|'
