#!/usr/bin/env bash
# One GPU-box session: GPU test-suite, then benches / profiles named on the
# command line.  Every GPU step has its own time limit; a crash-class exit
# (abort 134, segfault 139, timeout 124/137) ends the session at once.
#   tools/gpu_check.sh tests bench_cnn prof_r18 ...
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp

fatal() { case "$1" in 124|134|137|139) return 0;; esac; return 1; }

run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name exit $rc" | tee -a gpurun_out/session.log
  tail -3 "gpurun_out/$name.log"
  # summarise the steady-state tail of the kernel trace, then keep only the
  # summaries (the traces exceed gpurun's 64 MiB copy-back)
  if [ -d "gpurun_out/$name" ]; then
    tr=$(find "gpurun_out/$name" -name '*kernel_trace.csv' | head -1)
    if [ -n "$tr" ]; then python tools/prof_summary.py "$tr" 30 --tail-ms "${TAIL_MS:-200}" > "gpurun_out/$name/tail_stats.md" 2>&1; fi
    find "gpurun_out/$name" -type f ! -name '*stats*' -delete
  fi
  if fatal $rc; then echo "crash-class exit: stopping" | tee -a gpurun_out/session.log; exit $rc; fi
  return 0
}

for step in "$@"; do
  case "$step" in
    tests) run gpu_tests 700 python -u -m pytest tests -m gpu -v --maxfail=8 --timeout 150 --timeout-method thread -p no:cacheprovider ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench_cnn) run bench_cnn 240 python bench.py --steps 10 --warmup 2 ;;
    bench_r18) run bench_r18 300 python bench.py --model resnet18 --impl torch --steps 3 --warmup 1 ;;
    bench_r50) run bench_r50 400 python bench.py --model resnet50 --impl torch --steps 3 --warmup 1 ;;
    bench_vit) run bench_vit 400 python bench.py --model vit_b16 --impl torch --steps 3 --warmup 1 ;;
    bench_node) run bench_node 400 python bench_node.py ;;
    prof_cnn) TAIL_MS=30 run prof_cnn 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cnn -o run -- python bench.py --steps 5 --warmup 1 ;;
    prof_r18) TAIL_MS=120 run prof_r18 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r18 -o run -- python bench.py --model resnet18 --impl torch --steps 3 --warmup 1 ;;
    prof_r50) TAIL_MS=250 run prof_r50 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r50 -o run -- python bench.py --model resnet50 --impl torch --steps 2 --warmup 1 ;;
    prof_vit) TAIL_MS=700 run prof_vit 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_vit -o run -- python bench.py --model vit_b16 --impl torch --steps 2 --warmup 1 ;;
    t:*) f=${step#t:}; run "test_$(basename "$f" .py)" 400 python -u -m pytest "$f" -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
