#!/usr/bin/env bash
# One parameterised GPU runner (replaces the round-3 one-off scripts/r3_*.sh).
#
# Every step runs under its own time limit, output goes to gpurun_out/<tag>.log,
# and the lock checker stays ON (the driver's configuration, tests/conftest.py).
# A timeout, abort, segfault or kill ends the script at once so nothing more
# touches a possibly-wedged GPU; an ordinary failure ends it too (exit 1).
#
#   scripts/gpu.sh suite                    pytest -m gpu (whole GPU suite) + smoke()
#   scripts/gpu.sh tests <pytest args...>   selected tests, e.g. tests/test_gpu_conv.py -k bn
#   scripts/gpu.sh smoke                    __graft_entry__.smoke()
#   scripts/gpu.sh bench [bench args...]    bench.py (N=1 headline unless args say otherwise)
#   scripts/gpu.sh models [steps]           configs 3-5: resnet18, resnet50, vit_b16 rounds
#   scripts/gpu.sh rehearsal [N...]         split-hosts multi-rank rehearsal on the one GPU (default 2 4 8)
#   scripts/gpu.sh prof <tag> <cmd...>      rocprofv3 --kernel-trace --stats of <cmd> -> gpurun_out/prof_<tag>
#                                           (PROF_GAPS=1: also the GPU idle-gap table, tools/gap_summary.py)
#   scripts/gpu.sh overlap [on|off] [rounds] 8 virtual ResNet-50 peers (fault-tolerance scenario) under a
#                                           kernel trace + cross-stream overlap summary of training / FedAvg
#   scripts/gpu.sh rccl_overlap [N]         N split-host ranks (default 2) under a kernel trace: RCCL transfers /
#                                           FedAvg fold beside training, per rank (tools/overlap_summary.py)
#   scripts/gpu.sh pmc <tag> <cmd...>       rocprofv3 --kernel-trace --pmc passes of <cmd> (one counter group
#                                           per pass, each under its own kill timer; groups from $PMC_PASSES,
#                                           ";"-separated) + scripts/pmc_summary.py table -> gpurun_out/pmc_<tag>.md
#   scripts/gpu.sh py <secs> <tag> <cmd...> any python command, own limit
#
# Several modes can be chained with "+", e.g.
#   scripts/gpu.sh suite + bench + models
set -u
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"

step() {  # step <secs> <tag> <cmd...>
  local secs=$1 tag=$2; shift 2
  echo "=== [$tag] $* (limit ${secs}s, env: P2PFL_LOCKCHECK=${P2PFL_LOCKCHECK:-default(1 under pytest)})"
  # heartbeat on stdout while the step runs (a fresh box's first torch import and the
  # long tests print nothing for minutes; gpurun takes 3 silent minutes for a hang)
  ( while sleep 50; do echo "[gpu.sh] $tag still running $(date +%T): $(tail -c 120 "gpurun_out/$tag.log" | tr '\n' ' ')"; done ) &
  local hb=$!
  timeout -k 10 "$secs" "$@" > "gpurun_out/$tag.log" 2>&1
  local rc=$?
  kill "$hb" 2>/dev/null; wait "$hb" 2>/dev/null
  echo "=== [$tag] exit $rc"
  tail -n 25 "gpurun_out/$tag.log" | cut -c1-400
  if [ $rc -ne 0 ]; then echo "=== stopping after [$tag] (exit $rc)"; exit $rc; fi
}

run_mode() {
  local mode=$1; shift
  case $mode in
    suite)
      step 900 pytest_gpu python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rs
      step 300 smoke python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests)
      step 600 pytest_sel python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" ;;
    smoke)
      step 300 smoke python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)
      step 300 bench python -u bench.py "$@" ;;
    models)
      local k=${1:-3}
      for m in resnet18 resnet50 vit_b16; do
        step 300 "bench_$m" python -u bench.py --model $m --steps "$k" --warmup 1
      done ;;
    rehearsal)
      for n in ${@:-2 4 8}; do
        step 300 "rehearsal_n$n" env P2PFL_RCCL_SPLIT_HOSTS=1 P2PFL_BENCH_SPANS=1 python -u bench.py --gpus "$n" --steps 6 --warmup 2 --watchdog 240
      done ;;
    prof)
      local tag=$1; shift
      rm -rf "gpurun_out/prof_$tag"
      step 400 "prof_$tag" rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof_$tag" -o run -- "$@"
      step 120 "prof_${tag}_summary" python tools/prof_summary.py "gpurun_out/prof_$tag" --window-ms "${PROF_WINDOW_MS:-150}" --top 40 \
        ${PROF_GAPS:+--keep-trace}
      if [ -n "${PROF_GAPS:-}" ]; then  # idle-gap table of the trace, then drop it (too big to copy back)
        step 120 "prof_${tag}_gaps" python tools/gap_summary.py "gpurun_out/prof_$tag/run_kernel_trace.csv" \
          --window-ms "${PROF_WINDOW_MS:-150}" --out "gpurun_out/prof_${tag}_gaps.md"
        if [ -n "${PROF_OVERLAP:-}" ]; then  # "A_REGEX;B_REGEX": cross-stream overlap of two kernel classes
          step 120 "prof_${tag}_overlap" python tools/overlap_summary.py "gpurun_out/prof_$tag/run_kernel_trace.csv" \
            --a "${PROF_OVERLAP%%;*}" --b "${PROF_OVERLAP#*;}" --out "gpurun_out/prof_${tag}_overlap.md"
        fi
        rm -f "gpurun_out/prof_$tag/run_kernel_trace.csv"
      fi ;;
    overlap)
      local mode=${1:-on} rounds=${2:-5} d=gpurun_out/prof_overlap_${1:-on}
      rm -rf "$d"
      step 600 "overlap_$mode" rocprofv3 --kernel-trace --output-format csv -d "$d" -o run -- \
        python -u -m p2pfl_amd.examples.fault_tolerance --peers 8 --rounds "$rounds" --overlap "$mode"
      local csv
      csv=$(ls "$d"/*kernel_trace.csv "$d"/*/*kernel_trace.csv 2>/dev/null | head -1)
      step 120 "overlap_${mode}_train" python tools/overlap_summary.py "$csv" --a 'conv_kernel|p2bn|sgd_mt|p2head' \
        --b 'conv_kernel|p2bn|sgd_mt|p2head' --out "$d/overlap_train.md"
      step 120 "overlap_${mode}_fedavg" python tools/overlap_summary.py "$csv" --a 'wsum|weighted' \
        --b 'conv_kernel|p2bn|sgd_mt|p2head' --out "$d/overlap_fedavg.md"
      rm -f "$csv" ;;
    rccl_overlap)
      # 2 split-host ranks (a real 2-rank RCCL communicator over RCCL's socket transport,
      # time-sharing the one GPU -- not xGMI) under a kernel trace, one trace per rank:
      # how much of the RCCL transfer kernels and of the FedAvg fold ran beside training
      local n=${1:-2} d=gpurun_out/prof_rccl
      rm -rf "$d"
      step 600 rccl_overlap env P2PFL_RCCL_SPLIT_HOSTS=1 P2PFL_BENCH_SPANS=1 rocprofv3 --kernel-trace --output-format csv \
        -d "$d" -o %pid%_run -- python -u bench.py --gpus "$n" --steps 6 --warmup 2 --watchdog 240
      local csv k=0
      for csv in $(ls "$d"/*kernel_trace.csv "$d"/*/*kernel_trace.csv 2>/dev/null); do
        k=$((k + 1))
        step 120 "rccl_overlap_r${k}_nccl" python tools/overlap_summary.py "$csv" --a 'nccl|rccl' \
          --b 'p2cnn::' --out "$d/overlap_nccl_$k.md"
        step 120 "rccl_overlap_r${k}_wsum" python tools/overlap_summary.py "$csv" --a 'wsum' \
          --b 'p2cnn::' --out "$d/overlap_wsum_$k.md"
        step 120 "rccl_overlap_r${k}_timeline" python tools/rccl_timeline.py "$csv" --out "$d/timeline_$k.md"
        rm -f "$csv"
      done ;;
    pmc)
      # per-pass limits of the hardware (MI355X_MICROARCH.md): <= 8 SQ, 4 TCC (FETCH_SIZE 3, WRITE_SIZE 2), 2 GRBM
      local tag=$1; shift
      local passes=${PMC_PASSES:-"FETCH_SIZE;WRITE_SIZE;SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"}
      local dirs=() n=0 group
      IFS=';' read -ra groups <<< "$passes"
      for group in "${groups[@]}"; do
        n=$((n + 1)); rm -rf "gpurun_out/pmc_${tag}_$n"
        # shellcheck disable=SC2086
        step 120 "pmc_${tag}_$n" timeout -s KILL 100 rocprofv3 --kernel-trace --pmc $group --output-format csv \
          -d "gpurun_out/pmc_${tag}_$n" -o run -- "$@"
        dirs+=("gpurun_out/pmc_${tag}_$n")
      done
      step 120 "pmc_${tag}_summary" sh -c "python scripts/pmc_summary.py ${dirs[*]} --md > gpurun_out/pmc_$tag.md" ;;
    py)
      local secs=$1 tag=$2; shift 2
      step "$secs" "$tag" "$@" ;;
    *) echo "unknown mode $mode"; exit 2 ;;
  esac
}

args=("$@")
i=0
while [ $i -lt ${#args[@]} ]; do
  mode=${args[$i]}; i=$((i + 1)); sub=()
  while [ $i -lt ${#args[@]} ] && [ "${args[$i]}" != "+" ]; do sub+=("${args[$i]}"); i=$((i + 1)); done
  i=$((i + 1))
  run_mode "$mode" "${sub[@]+"${sub[@]}"}"
done
