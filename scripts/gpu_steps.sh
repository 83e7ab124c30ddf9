#!/usr/bin/env bash
# Run GPU steps in order; each step has its own time limit.  An ordinary
# failure (exit 1/2) is recorded and the next step runs; a timeout, abort,
# segfault or kill (124/134/137/139 or signal) ends the script immediately so
# nothing more touches a possibly-wedged GPU.
#   usage: scripts/gpu_steps.sh "<secs>|<name>|<command>" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $cmd (limit ${secs}s)"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] exit $rc"; tail -n 5 "gpurun_out/$name.log"
  case $rc in
    0) ;;
    1|2|3|4|5) status=1 ;;
    *) echo "=== fatal exit $rc in [$name]; stopping"; exit $rc ;;
  esac
done
exit $status
