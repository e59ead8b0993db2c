# round-4 checkpoint: -m gpu suite, lone-chain latency, one C3 bench line, k_connect PMC attribution
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4/gputest.log 2>&1
rc=$?
tail -3 gpurun_out/r4/gputest.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 150 python tools/chain_probe.py > gpurun_out/r4/chain.txt 2>&1 || exit 3
tail -1 gpurun_out/r4/chain.txt
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r4/bench_c3.json 2> gpurun_out/r4/bench_c3.err || exit 4
python3 -c "import json;j=json.load(open('gpurun_out/r4/bench_c3.json'));print(j['value'], j['kernel_ms_profile_pass'])"
timeout -k 10 700 bash tools/pmc_variants.sh gpurun_out/r4/connect_pmc k_connect 'FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum' 'def||' 'noshsort|SURF_SORT=2|' > gpurun_out/r4/connect_pmc.txt 2>&1 || exit 5
cat gpurun_out/r4/connect_pmc.txt
exit $rc
