set -o pipefail
mkdir -p gpurun_out/r4_adv
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_adv/gpu_tests_lag.log 2>&1 && \
N=4096 WINDOWS=0 timeout -k 10 200 python -u tools/dropin_loop.py > gpurun_out/r4_adv/dropin_lag_4096.jsonl 2>&1 && \
N=1024 WINDOWS=0 timeout -k 10 200 python -u tools/dropin_loop.py > gpurun_out/r4_adv/dropin_lag_1024.jsonl 2>&1 && \
SURF_LOOP_LAG=0 N=4096 WINDOWS=0 timeout -k 10 200 python -u tools/dropin_loop.py > gpurun_out/r4_adv/dropin_nolag_4096.jsonl 2>&1
