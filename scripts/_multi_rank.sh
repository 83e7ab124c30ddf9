cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --steps 5 --warmup 2 > gpurun_out/mr_$n.log 2>&1
  rc=$?
  echo "N=$n rc $rc: $(grep -h '"metric"' gpurun_out/mr_$n.log | cut -c1-250)"
  grep -h "bench rank\|fallback\|Error\|error" gpurun_out/mr_$n.log | head -8
  if [ $rc -ge 124 ]; then exit $rc; fi
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2_vit_prof2 -o run -- python bench.py --model vit_b16 --steps 2 --warmup 1 --watchdog 380 > gpurun_out/r2_vit_prof2.log 2>&1 && python tools/prof_summary.py gpurun_out/r2_vit_prof2 --window-ms 300 --top 30 > /dev/null
echo "vit prof rc $?"
