#!/bin/bash
# Round-3 GPU session: rocprofv3 evidence of C2 / C4 / C5 on the current tree
# (tools/profile_round.sh per workload -> profiles/r3_<wl>/), then the C5
# trace-kernel occupancy sweep (SURF_TRACE_WAVES 2/4/6/8, lib/variants/s4t<N>.so).
# usage: tools/r3_profiles.sh OUT [WORKLOADS...]
set -o pipefail
OUT=${1:-gpurun_out/r3_prof}
shift
WLS=${@:-C2 C4 C5}
mkdir -p "$OUT"
for wl in $WLS; do
    bash tools/profile_round.sh "$OUT/$wl" "$wl" 2 || { echo "profile $wl failed"; exit 1; }
    echo "profiled $wl"
done
echo ok
