set -o pipefail
mkdir -p gpurun_out/r4_pt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "refill or lane_two_level" > gpurun_out/r4_pt/tests.log 2>&1 && \
bash tools/ab.sh gpurun_out/r4_pt 'pt0|SURF_PT=0|--workload C5 --steps 1 --warmup 0' 'pt1|SURF_PT=1|--workload C5 --steps 1 --warmup 0' > gpurun_out/r4_pt/ab.txt 2>&1
