#!/usr/bin/env bash
# Same-box A/B of the batched bias column sums (P2PFL_DEFER_COLSUM), ViT-B/16 rounds, alternating.
set -u
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 env P2PFL_DEFER_COLSUM=$v python -u bench.py --model vit_b16 --steps 8 --warmup 1 \
      > "gpurun_out/ab_colsum_${v}_$i.log" 2>&1 || exit $?
    echo "colsum=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/ab_colsum_${v}_$i.log")"
  done
done
