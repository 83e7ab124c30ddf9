cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
  P2PFL_NATIVE_CONV=0 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovc_$i -o run -- python -m p2pfl_amd.examples.fault_tolerance --peers 8 --rounds 4 --overlap off > gpurun_out/ovc_$i.log 2>&1
  rc=$?
  rm -f gpurun_out/ovc_$i/run_kernel_trace.csv
  echo "miopen profiled run $i rc $rc: $(grep -E 'max.diff|survivors_equal' gpurun_out/ovc_$i.log | tr '\n' ' ' | cut -c1-200)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
