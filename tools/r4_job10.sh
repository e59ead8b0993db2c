mkdir -p gpurun_out/r4/skey
bash tools/ab.sh -r 2 gpurun_out/r4/skey 's0||' 's1|SURF_SKEY_REV=1|' 'c1|SURF_KEY=1|--workload C5 --steps 1 --warmup 0' 'c2||--workload C5 --steps 1 --warmup 0'
