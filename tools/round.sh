#!/bin/bash
# One GPU session's standard steps, as named presets (replaces the per-round
# r3_*/r4_* wrappers and r4_job*.sh launchers).  Run from the repo root on the
# GPU box; every step has its own time limit and the first failure ends the run.
#
#   tools/round.sh suite    OUT            -m gpu suite (-v log) + smoke()
#   tools/round.sh benches  OUT            bench lines C3 (default) / C2 / C4 / C5, the N = 2 bench
#                                          path rehearsed on one GPU (two ranks on device 0, gloo
#                                          gather, assembled frame checked against the oracle),
#                                          and the 8-shard projections of C3 and C4 (tools/shard_probe.py)
#   tools/round.sh profiles OUT [WL ...]   rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes per
#                                          workload (tools/profile_round.sh -> OUT/<wl>/summary.json,
#                                          copied to profiles/r<N>_<wl>/ and read by bench.py's roofline)
#   tools/round.sh final    OUT            suite, profiles C3 C2 C4 C5, benches
#
# Experiments use tools/ab.sh (same-box A/B of environment knobs / library
# variants) and tools/pmc_variants.sh (per-kernel PMC per variant); MEASUREMENTS.md
# records each experiment's invocation beside its result.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
step=${1:?preset: suite | benches | profiles | final}
OUT=${2:?out dir}
shift 2
mkdir -p "$OUT"

suite() {
    timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
        || { tail -20 "$OUT/pytest_gpu.log"; return 1; }
    tail -1 "$OUT/pytest_gpu.log"
    timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -5 "$OUT/smoke.log"; return 1; }
    tail -1 "$OUT/smoke.log"
}

line() {   # bench JSON -> one summary line
    python3 -c "import json,sys;j=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=j.get('roofline') or {};print(sys.argv[2], j['value'], (j.get('parity') or {}).get('bitexact'), j.get('gpu_vs_cpu'), r.get('frac'))" "$1" "$2"
}

benches() {
    local b=$OUT/bench
    mkdir -p "$b"
    timeout -k 10 400 python bench.py > "$b/bench_c3.json" 2> "$b/bench_c3.err" || { tail -5 "$b/bench_c3.err"; return 1; }
    line "$b/bench_c3.json" C3
    for wl in C2 C4 C5; do
        timeout -k 10 500 python bench.py --workload $wl > "$b/bench_${wl,,}.json" 2> "$b/bench_${wl,,}.err" || { tail -5 "$b/bench_${wl,,}.err"; return 1; }
        line "$b/bench_${wl,,}.json" $wl
    done
    SURF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 > "$b/dist_n2.json" 2> "$b/dist_n2.err" || { tail -5 "$b/dist_n2.err"; return 1; }
    line "$b/dist_n2.json" N2
    timeout -k 10 300 python tools/shard_probe.py 8 > "$b/shards8_c3.txt" 2>&1 || return 1
    tail -1 "$b/shards8_c3.txt"
    W=1920 H=1080 F=1024 timeout -k 10 600 python tools/shard_probe.py 8 > "$b/shards8_c4.txt" 2>&1 || return 1
    tail -1 "$b/shards8_c4.txt"
}

profiles() {
    local wls=${*:-C3 C2 C4 C5}
    for wl in $wls; do
        bash tools/profile_round.sh "$OUT/prof/$wl" "$wl" 2 || { echo "profile $wl failed"; return 1; }
        python3 -c "import json;s=json.load(open('$OUT/prof/$wl/summary.json'));k=[v for n,v in s['kernels'].items() if n.startswith('k_extend')][0];print('$wl', s.get('bench_value_traced'), 'k_extend avg us', k['avg_us'], s.get('k_extend_pmc'))"
    done
}

case $step in
    suite) suite ;;
    benches) benches ;;
    profiles) profiles "$@" ;;
    final) suite && profiles C3 C2 C4 C5 && benches ;;
    *) echo "unknown preset $step"; exit 2 ;;
esac
