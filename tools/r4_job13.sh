mkdir -p gpurun_out/r4/cgrid2
bash tools/ab.sh -r 2 gpurun_out/r4/cgrid2 'g12||' 'g16|SURF_GRID_CONNECT=16|' 'g24|SURF_GRID_CONNECT=24|' 'g32|SURF_GRID_CONNECT=32|'
