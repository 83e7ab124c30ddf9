#!/bin/bash
# BN statistics passes with 4 rows in flight: numerics, ResNet rounds, per-kernel medians of the ResNet-18 step
set -o pipefail
cd "$(dirname "$0")/.."
ROOT=$(pwd)
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_batchnorm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_bn4_pytest.log 2>&1 || { tail -40 gpurun_out/r3_bn4_pytest.log; exit 1; }
tail -1 gpurun_out/r3_bn4_pytest.log
for m in resnet18 resnet50; do
  timeout -k 10 300 python bench.py --model $m --steps 3 --warmup 1 > gpurun_out/r3_bn4_$m.log 2>&1 || { tail -30 gpurun_out/r3_bn4_$m.log; exit 1; }
  echo "$m $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3_bn4_$m.log)"
done
export TMPDIR=/tmp PYTHONPATH="$ROOT"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/r3_bn4_prof" -o run -- python3 "$ROOT/bench.py" --model resnet18 --steps 3 --warmup 1 > "$ROOT/gpurun_out/r3_bn4_prof.log" 2>&1
rc=$?
cd "$ROOT"
[ $rc -eq 0 ] || { tail -20 gpurun_out/r3_bn4_prof.log; exit $rc; }
python3 tools/prof_summary.py gpurun_out/r3_bn4_prof --window-ms 150 --top 40 > /dev/null
rm -rf gpurun_out/r3_bn4_prof
grep "p2bn::" gpurun_out/r3_bn4_prof.md | cut -c1-200 | head -30
