#!/bin/bash
# rocprofv3 kernel table of the ResNet-18 step (config 3) on this tree: native convolutions in the step graphs
set -o pipefail
cd "$(dirname "$0")/.."
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp P2PFL_LOCKCHECK=0 PYTHONPATH="$ROOT"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/r3_resnet18_prof" -o run -- python3 "$ROOT/bench.py" --model resnet18 --steps 3 --warmup 1 > "$ROOT/gpurun_out/r3_resnet18_prof.log" 2>&1
rc=$?
cd "$ROOT"
tail -1 gpurun_out/r3_resnet18_prof.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py gpurun_out/r3_resnet18_prof --window-ms 150 --top 20 > /dev/null
rm -rf gpurun_out/r3_resnet18_prof
head -40 gpurun_out/r3_resnet18_prof.md
