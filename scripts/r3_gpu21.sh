#!/bin/bash
# NaN hunt, step 5: the 8-peer ResNet-50 scenario still goes non-finite under rocprofv3
# after the 1x1 fix.  Which ingredient is needed: per-node streams, step graphs, MIOpen, the profiler?
set -o pipefail
cd "$(dirname "$0")/.."
H=scripts/r3_nan_hunt.sh
bash $H streams_off --rounds 2 --overlap off || exit $?
bash $H no_graphs --rounds 2 --no-step-graphs || exit $?
P2PFL_NATIVE_CONV=1 bash $H native_conv --rounds 2 || exit $?
bash $H resnet18 --rounds 2 --model resnet18 || exit $?
echo "== unprofiled, overlap on"
P2PFL_CHECK_FINITE=1 P2PFL_LOCKCHECK=0 timeout -k 10 300 python -u -m p2pfl_amd.examples.fault_tolerance --rounds 2 2>&1 | grep -E "non_finite|round_ms|Error" | cut -c1-300
exit 0
