#!/bin/bash
# BN statistics + finalize in one launch: numerics, ResNet-18 / ResNet-50 rounds with and without it, kernel profile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export P2PFL_LOCKCHECK=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_batchnorm.py tests/test_gpu_graph_memory.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3_bn_pytest.log 2>&1 || { tail -40 gpurun_out/r3_bn_pytest.log; exit 1; }
tail -1 gpurun_out/r3_bn_pytest.log
for f in 1 0 1 0; do
  P2PFL_BN_FUSED_STATS=$f timeout -k 10 300 python bench.py --model resnet18 --steps 3 --warmup 1 > gpurun_out/r3_bn_r18_$f.log 2>&1 || { tail -30 gpurun_out/r3_bn_r18_$f.log; exit 1; }
  echo "fused=$f $(tail -1 gpurun_out/r3_bn_r18_$f.log | cut -c1-160)"
done
for f in 1 0; do
  P2PFL_BN_FUSED_STATS=$f timeout -k 10 300 python bench.py --model resnet50 --steps 3 --warmup 1 > gpurun_out/r3_bn_r50_$f.log 2>&1 || { tail -30 gpurun_out/r3_bn_r50_$f.log; exit 1; }
  echo "fused=$f $(tail -1 gpurun_out/r3_bn_r50_$f.log | cut -c1-160)"
done
ROOT=$(pwd)
export TMPDIR=/tmp PYTHONPATH="$ROOT"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/gpurun_out/r3_bn_prof" -o run -- python3 "$ROOT/bench.py" --model resnet18 --steps 3 --warmup 1 > "$ROOT/gpurun_out/r3_bn_prof.log" 2>&1
rc=$?
cd "$ROOT"
tail -1 gpurun_out/r3_bn_prof.log | cut -c1-200
[ $rc -eq 0 ] || exit $rc
python3 tools/prof_summary.py gpurun_out/r3_bn_prof --window-ms 150 --top 30 > /dev/null
rm -rf gpurun_out/r3_bn_prof
head -50 gpurun_out/r3_bn_prof.md | cut -c1-200
