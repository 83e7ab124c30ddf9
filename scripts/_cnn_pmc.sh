# PMC passes over the fused-CNN step kernels (scripts/kbench.py, isolated
# launches).  One counter group per pass; each pass under its own kill timer.
set -e
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
K="python3 scripts/kbench.py --no-graph --reps 20"
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- $K > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- $K > gpurun_out/pmc_write.log 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq -o run -- $K > gpurun_out/pmc_sq.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_sq --md > gpurun_out/pmc_cnn.md
