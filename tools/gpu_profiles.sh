#!/bin/bash
# rocprofv3 evidence (kernel trace + FETCH_SIZE + WRITE_SIZE passes) and a bench line per workload.
# usage: tools/gpu_profiles.sh TAG WL:STEPS [WL:STEPS ...]
set -o pipefail
TAG=$1; shift
for spec in "$@"; do
  WL=${spec%%:*}; STEPS=${spec##*:}
  wl=$(echo $WL | tr A-Z a-z)
  OUT=gpurun_out/$TAG/$wl
  mkdir -p $OUT profiles/r2_$wl
  bash tools/profile_round.sh $OUT/prof $WL $STEPS || { echo "profile $WL failed"; exit 1; }
  cp $OUT/prof/summary.json profiles/r2_$wl/summary.json
  cp $OUT/prof/trace/run_kernel_stats.csv $OUT/kernel_stats.csv
  timeout -k 10 400 python bench.py --workload $WL --steps $STEPS --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench $WL failed"; tail $OUT/bench.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench.json')); print('$WL', d['value'], d['ms_per_step'], json.dumps(d['roofline']), json.dumps(d['pipeline_roofline']), (d.get('cpu_baseline') or {}).get('value'), (d.get('parity') or {}).get('bitexact'))"
done
