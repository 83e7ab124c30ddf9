set -e
# Same-box A/B of BatchNorm statistics + finalize in one launch (P2PFL_BN_FUSED_STATS)
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for f in 0 1; do
    P2PFL_BN_FUSED_STATS=$f timeout -k 10 300 python -u bench.py --model resnet18 --steps 8 --warmup 1 > gpurun_out/abbn_r18_f${f}_$rep.log 2>&1
    echo "resnet18 fused=$f rep=$rep: $(grep -h '^{"metric"' gpurun_out/abbn_r18_f${f}_$rep.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
