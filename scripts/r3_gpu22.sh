#!/bin/bash
# NaN hunt, step 6: native convolutions inside captured graphs
set -o pipefail
cd "$(dirname "$0")/.."
H=scripts/r3_nan_hunt.sh
echo "== unprofiled, overlap on"
P2PFL_CHECK_FINITE=1 P2PFL_LOCKCHECK=0 timeout -k 10 300 python -u -m p2pfl_amd.examples.fault_tolerance --rounds 3 2>&1 | grep -E "non_finite|round_ms|Error" | cut -c1-400
bash $H resnet18 --rounds 3 --model resnet18 || exit $?
bash $H fix2 --rounds 6 || exit $?
rm -rf gpurun_out/nan/prof_resnet18
export P2PFL_LOCKCHECK=0
timeout -k 10 300 python bench.py --model resnet18 --steps 3 --warmup 1 > gpurun_out/r3_bench_resnet18.log 2>&1 || { tail -30 gpurun_out/r3_bench_resnet18.log; exit 1; }
tail -1 gpurun_out/r3_bench_resnet18.log | cut -c1-200
