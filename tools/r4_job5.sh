mkdir -p gpurun_out/r4/xcdq2
SURF_XCDQ=12 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
   -k "ray_order or issue_order or render_64 or spp4 or c3_subset" > gpurun_out/r4/xcdq2/pytest.log 2>&1
rc=$?; tail -2 gpurun_out/r4/xcdq2/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab.sh gpurun_out/r4/xcdq2 'q0|SURF_XCDQ=0|' 'q4|SURF_XCDQ=4|' 'q8|SURF_XCDQ=8|' 'q12|SURF_XCDQ=12|' 'q0b|SURF_XCDQ=0|' 'q4b|SURF_XCDQ=4|'
for q in q0 q4 q8 q12 q0b q4b; do python3 -c "import json;j=json.load(open('gpurun_out/r4/xcdq2/$q.json'));print('$q', j['kernel_ms_profile_pass'])"; done
