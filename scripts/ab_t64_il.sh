set -e
# A/B of the 64x64 conv tiles' in-launch split-K candidates, same box, alternating runs
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for il in 1 0; do
    for m in resnet18 resnet50; do
      P2PFL_CONV_T64_IL=$il timeout -k 10 300 python -u bench.py --model $m --steps 8 --warmup 1 > gpurun_out/ab_${m}_il${il}_$rep.log 2>&1
      echo "$m il=$il rep=$rep: $(grep -h '^{"metric"' gpurun_out/ab_${m}_il${il}_$rep.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
    done
  done
done
