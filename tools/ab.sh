#!/bin/bash
# Same-box A/B runner: one measurement set per variant, variants interleaved.
#   tools/ab.sh [-t] [-c] [-s] [-n] [-r REPS] OUT 'name|ENV=V,ENV=V|--bench-opts' ...
#   -t  the -m gpu suite once first (defaults)       -c  lone-chain latency (tools/chain_probe.py)
#   -s  8-shard shard-1 breakdown (tools/shard_breakdown.py 8 1)
#   -n  no bench line (default: one bench.py line without the CPU leg: --steps 3 --warmup 1 + opts)
#   -r  repetitions of the whole variant list (interleaved A B A B ...)
# A library build is a variant too: 'timing|SURF_HIP_LIB=surf-path-tracer_amd/lib/variants/timing.so|'.
# Examples (DESIGN.md cites these): the two-level walk A/B
#   tools/ab.sh -c -s OUT 'w0|SURF_WALK2=0|' 'w1|SURF_WALK2=1|'
# the C5 trace-wave sweep: tools/ab.sh OUT 't4|SURF_HIP_LIB=surf-path-tracer_amd/lib/variants/s4t4.so|--workload C5 --steps 1 --warmup 0'
# the pool A/B: tools/ab.sh OUT 'p5||' 'p45||--pool 4147200'
suite=0; chain=0; shard=0; bench=1; reps=1
while getopts "tcsnr:" o; do
  case $o in t) suite=1;; c) chain=1;; s) shard=1;; n) bench=0;; r) reps=$OPTARG;; *) exit 2;; esac
done
shift $((OPTIND - 1))
OUT=${1:?out dir}; shift
mkdir -p "$OUT"
if [ $suite = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
fi
for rep in $(seq 1 "$reps"); do
  for v in "$@"; do
    IFS='|' read -r name envs opts <<< "$v"
    tag=$name; [ "$reps" -gt 1 ] && tag=${name}_$rep
    line="$tag"
    run() {   # run CMD... in a subshell with the variant's environment
      ( IFS=,; for e in $envs; do [ -n "$e" ] && export "$e"; done; unset IFS; "$@" )
    }
    if [ $chain = 1 ]; then
      run timeout -k 10 150 python tools/chain_probe.py > "$OUT/$tag.chain.txt" 2>&1 || exit 1
      line="$line chain_us $(tail -1 "$OUT/$tag.chain.txt" | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["us_per_segment"])')"
    fi
    if [ $shard = 1 ]; then
      run timeout -k 10 240 python tools/shard_breakdown.py 8 1 > "$OUT/$tag.shard.txt" 2>&1 || exit 1
      line="$line shard8/1_ms $(sed -n 3p "$OUT/$tag.shard.txt" | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["wall_ms"])')"
    fi
    if [ $bench = 1 ]; then
      run timeout -k 10 400 python bench.py --no-cpu --steps 3 --warmup 1 $opts > "$OUT/$tag.json" 2> "$OUT/$tag.err" || exit 1
      line="$line $(python3 -c "import json;j=json.load(open('$OUT/$tag.json'));k=j['kernel_ms_profile_pass'];print(j['value'], 'ext', k['ms_extend'], 'shade', k['ms_shade'], 'conn', k['ms_connect'], 'tail', k['ms_tail'], k['tail_paths'], 'it', j['iterations_per_render'])")"
    fi
    echo "$line"
  done
done
