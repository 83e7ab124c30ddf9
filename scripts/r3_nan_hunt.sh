#!/bin/bash
# verdict r2 #4: the 8-peer ResNet-50 scenario under rocprofv3 --kernel-trace,
# with every received / aggregated / trained arena checked for NaN/Inf
# (P2PFL_CHECK_FINITE=1) to name the first non-finite tensor.
#   bash scripts/r3_nan_hunt.sh TAG [example args...]
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
mkdir -p "$ROOT/gpurun_out/nan"
export TMPDIR=/tmp P2PFL_CHECK_FINITE=1 P2PFL_LOCKCHECK=0 PYTHONPATH="$ROOT"
TAG=$1; shift
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/nan/prof_$TAG" -o run -- \
  python3 -u -m p2pfl_amd.examples.fault_tolerance "$@" 2>&1 | grep --line-buffered -v "duplicate kernel symbol" \
  | tee "$ROOT/gpurun_out/nan/run_$TAG.log" | grep --line-buffered -E "non_finite|non-finite|fault_tolerance|round_ms|Error" 
st=("${PIPESTATUS[@]}")
echo "[$TAG] profiler exit ${st[0]}"
# keep a kernel-time summary, drop the raw trace (whole-run traces exceed gpurun's copy-back limit)
cd "$ROOT" && python3 tools/prof_summary.py "gpurun_out/nan/prof_$TAG" --top 25 > /dev/null 2>&1
rm -rf "gpurun_out/nan/prof_$TAG"
case "${st[0]}" in 124|137|134|139) exit "${st[0]}";; esac
exit 0
