timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_gputest.log 2>&1
rc=$?
tail -3 gpurun_out/r4_gputest.log
if [ $rc -le 1 ]; then
  timeout -k 10 700 bash tools/pmc_variants.sh gpurun_out/r4_connect_pmc k_connect 'FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum' 'def||' 'noshsort|SURF_SORT=2|' > gpurun_out/r4_connect_pmc.txt 2>&1 || exit 3
  cat gpurun_out/r4_connect_pmc.txt
fi
exit $rc
