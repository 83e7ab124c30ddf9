set -e
cd "${GRAFT_REPO_ROOT:-.}"
for m in gemm conv legacy; do
  P2PFL_CONV1X1_MODE=$m timeout -k 10 300 python -u bench.py --model resnet50 --steps 8 --warmup 1 > gpurun_out/r50_$m.log 2>&1
  echo "r50 $m: $(grep -h '^{"metric"' gpurun_out/r50_$m.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
for m in gemm conv; do
  P2PFL_CONV1X1_MODE=$m timeout -k 10 300 python -u bench.py --model resnet18 --steps 8 --warmup 1 > gpurun_out/r18_$m.log 2>&1
  echo "r18 $m: $(grep -h '^{"metric"' gpurun_out/r18_$m.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
done
