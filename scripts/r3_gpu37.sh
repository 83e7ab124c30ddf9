#!/bin/bash
# final tree: GPU suite + smoke
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r3_last_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r3_last_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r3_last_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_last_smoke.log 2>&1 || { tail -20 gpurun_out/r3_last_smoke.log; exit 1; }
tail -1 gpurun_out/r3_last_smoke.log
