set -o pipefail
mkdir -p gpurun_out/r4_adv
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r4_adv/gpu_tests.log 2>&1 && \
timeout -k 10 240 python -u tools/dropin_loop.py > gpurun_out/r4_adv/dropin_loop.jsonl 2>&1
