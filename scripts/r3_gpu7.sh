#!/bin/bash
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/nan
export P2PFL_LOCKCHECK=0
echo "== poison, graphs"; timeout -k 10 170 python -u scripts/graph_poison.py --poison 2>&1 | grep -v "^W2026" | tail -6
echo "== poison, eager"; timeout -k 10 170 python -u scripts/graph_poison.py --poison --no-graphs 2>&1 | grep -v "^W2026" | tail -6
echo "== profiled, graphs, no poison"
cd /tmp; export TMPDIR=/tmp
timeout -k 10 170 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/nan/prof_poison" -o run -- python3 -u "$GRAFT_REPO_ROOT/scripts/graph_poison.py" 2>&1 | grep -v "^W2026" | tail -6
exit 0
