#!/bin/bash
# Round-4 final check, part A: the -m gpu suite, smoke(), and the rocprofv3 summaries of C3/C2/C4
# (the k_connect LDS staging changed the wavefront phase; C5 does not use it).  usage: tools/r4_final_a.sh
set -o pipefail
mkdir -p gpurun_out/r4_final
timeout -k 10 500 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r4_final/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/r4_final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r4_final/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_final/smoke.log 2>&1 || { tail -5 gpurun_out/r4_final/smoke.log; exit 1; }
tail -1 gpurun_out/r4_final/smoke.log
bash tools/r4_profiles.sh gpurun_out/r4_final/prof C3 C2 C4
