#!/usr/bin/env bash
# Same-box A/B of the 16-B vector path of the ResNet head kernels (P2PFL_HEAD_VEC), alternating.
set -u
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in ${AB_MODELS:-resnet50 resnet18}; do
  for i in 1 2; do
    for v in 1 0; do
      timeout -k 10 300 env P2PFL_HEAD_VEC=$v python -u bench.py --model $m --steps 8 --warmup 1 \
        > "gpurun_out/ab_head_${m}_${v}_$i.log" 2>&1 || exit $?
      echo "$m head_vec=$v run $i: $(grep -o '"ms_per_step": [0-9.]*' "gpurun_out/ab_head_${m}_${v}_$i.log")"
    done
  done
done
