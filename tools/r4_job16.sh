set -o pipefail
mkdir -p gpurun_out/r4_adv
N=4096 WINDOWS=256,1024,4096 timeout -k 10 400 python -u tools/dropin_loop.py > gpurun_out/r4_adv/dropin_loop_4096.jsonl 2>&1
