# XCD work-queue A/B: parity subset with both queues on, then C3 bench lines per SURF_XCDQ
mkdir -p gpurun_out/r4/xcdq
SURF_XCDQ=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
   -k "ray_order or issue_order or render_64 or drain_policies or spp4 or c3_subset" > gpurun_out/r4/xcdq/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4/xcdq/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh gpurun_out/r4/xcdq 'q0|SURF_XCDQ=0|' 'q1|SURF_XCDQ=1|' 'q2|SURF_XCDQ=2|' 'q3|SURF_XCDQ=3|' 'q0b|SURF_XCDQ=0|' 'q3b|SURF_XCDQ=3|'
