# Drain timeline of the C3 bench (diagnostics): per-replay in-flight counts and tail stages on stderr.
mkdir -p gpurun_out/drain
SURF_DEBUG_DRAIN=1 SURF_DEBUG_TAIL=1 timeout -k 10 200 python bench.py --no-cpu --profile-pass 0 $1 > gpurun_out/drain/bench$2.json 2> gpurun_out/drain/err$2.txt
