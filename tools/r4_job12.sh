mkdir -p gpurun_out/r4/fork
SURF_FORK=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
   -k "ray_order or issue_order or render_64 or spp4 or c3_subset or drain_policies" > gpurun_out/r4/fork/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4/fork/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh -r 2 gpurun_out/r4/fork 'f0||' 'f1|SURF_FORK=1|'
