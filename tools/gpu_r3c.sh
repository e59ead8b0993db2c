mkdir -p gpurun_out/r3_c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "closest_hit or any_hit or boundary or drain_policies or general_tlas or c5_deep or render_64" > gpurun_out/r3_c/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r3_c/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/chain_probe2.py > gpurun_out/r3_c/chain.txt 2>&1; cat gpurun_out/r3_c/chain.txt
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r3_c/bench.json 2> gpurun_out/r3_c/bench.err; python -c "import json;j=json.load(open('gpurun_out/r3_c/bench.json'));print(j['value'], j['kernel_ms_profile_pass'])"
