set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/cpmc1 -o run -- python scripts/conv_one.py fwd > gpurun_out/cpmc1.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_INSTS_LDS --output-format csv -d gpurun_out/cpmc2 -o run -- python scripts/conv_one.py fwd > gpurun_out/cpmc2.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d gpurun_out/cpmc3 -o run -- python scripts/conv_one.py fwd > gpurun_out/cpmc3.log 2>&1 || true
