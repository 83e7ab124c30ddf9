cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for lr in 0.01 0.01 0.05; do
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovl -o run -- python -m p2pfl_amd.examples.fault_tolerance --peers 8 --rounds 4 --overlap off --lr $lr > gpurun_out/ovl_$lr.log 2>&1
  rc=$?
  rm -f gpurun_out/ovl/run_kernel_trace.csv
  echo "lr $lr rc $rc: $(grep -E 'max.diff|survivors_equal' gpurun_out/ovl_$lr.log | tr '\n' ' ' | cut -c1-160)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2_cnn_merged_adam -o run -- python bench.py --steps 10 --warmup 3 > gpurun_out/r2_cnn_merged_adam.log 2>&1 && python tools/prof_summary.py gpurun_out/r2_cnn_merged_adam --window-ms 50 > /dev/null
echo "cnn prof rc $?"
