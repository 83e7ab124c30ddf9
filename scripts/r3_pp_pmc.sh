#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) of the ping-pong GEMM vs
# hipBLASLt at 8192^3 and on the ViT QKV forward: where does the ping-pong kernel lose?
set -o pipefail
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
ROOT=$(pwd)
OUT=gpurun_out/pppmc
rm -rf $OUT; mkdir -p $OUT
i=0
for pass in "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS" \
            "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum" \
            "FETCH_SIZE"; do
  i=$((i+1))
  for cfg in "8192 2048" "8192 0 lib"; do
    tag=$(echo "$cfg" | tr ' ' '_')_p$i
    timeout -s KILL 60 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/$tag -o run -- python3 $ROOT/scripts/gemm_one.py $cfg > $OUT/$tag.log 2>&1 || { echo "pass $tag failed rc=$?"; tail -5 $OUT/$tag.log; exit 1; }
  done
done
python3 scripts/pmc_summary.py $OUT/8192_2048_p* --md > $OUT/pp.md 2>&1 || true
python3 scripts/pmc_summary.py $OUT/8192_0_lib_p* --md > $OUT/lib.md 2>&1 || true
cat $OUT/pp.md $OUT/lib.md
find $OUT -type f -size +256k -delete
