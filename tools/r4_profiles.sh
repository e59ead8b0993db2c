#!/bin/bash
# Round-4 rocprofv3 evidence: tools/profile_round.sh per workload -> OUT/<wl>/summary.json
# (copied to profiles/r4_<wl>/ and read by bench.py's roofline).  usage: tools/r4_profiles.sh OUT [WORKLOADS...]
OUT=${1:-gpurun_out/r4_prof}; shift
WLS=${@:-C3 C2 C4 C5}
mkdir -p "$OUT"
for wl in $WLS; do
    bash tools/profile_round.sh "$OUT/$wl" "$wl" 2 || { echo "profile $wl failed"; exit 1; }
    python3 -c "import json;s=json.load(open('$OUT/$wl/summary.json'));k=[v for n,v in s['kernels'].items() if n.startswith('k_extend')][0];print('$wl', s.get('bench_value_traced'), 'k_extend avg us', k['avg_us'], s.get('k_extend_pmc'))"
done
