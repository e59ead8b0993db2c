# kernel timeline of the late fork (SURF_FORK=1) vs default
mkdir -p gpurun_out/r4/tl
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SURF_FORK=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4/tl/f1 -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu --profile-pass 0 > gpurun_out/r4/tl/f1.json 2> gpurun_out/r4/tl/f1.err || exit 1
echo ok
