# pool-size cliff of k_extend: per pool size, k_extend time (profile pass) and its L2 hit rate / fetch
mkdir -p gpurun_out/r4
timeout -k 10 1000 bash tools/pmc_variants.sh gpurun_out/r4/pool_cliff k_extend 'TCC_HIT_sum TCC_MISS_sum;FETCH_SIZE' \
  'p45||--pool 4147200' 'p46||--pool 4239360' 'p47||--pool 4331520' 'p48||--pool 4423680' 'p50||--pool 4608000' > gpurun_out/r4/pool_cliff.txt 2>&1
rc=$?; cat gpurun_out/r4/pool_cliff.txt; exit $rc
