#!/bin/bash
# rocprofv3 kernel tables of the ViT-B/16 (config 4) and ResNet-50 (config 5 model) rounds on this tree
set -o pipefail
cd "$(dirname "$0")/.."
ROOT=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp P2PFL_LOCKCHECK=0 PYTHONPATH="$ROOT"
for m in vit_b16 resnet50; do
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/r3_${m}_prof" -o run -- python3 "$ROOT/bench.py" --model $m --steps 3 --warmup 1 > "$ROOT/gpurun_out/r3_${m}_prof.log" 2>&1
  rc=$?
  cd "$ROOT"
  tail -1 gpurun_out/r3_${m}_prof.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
  python3 tools/prof_summary.py gpurun_out/r3_${m}_prof --window-ms 400 --top 25 > /dev/null
  rm -rf gpurun_out/r3_${m}_prof
  head -45 gpurun_out/r3_${m}_prof.md | cut -c1-200
done
