#!/bin/bash
cd "$(dirname "$0")/.."
echo "== A: 8 peers, eager steps (no HIP graphs), profiled"
bash scripts/r3_nan_hunt.sh eager8 --peers 8 --rounds 3 --overlap off --no-step-graphs || exit $?
echo "== B: 2 peers, HIP graphs, profiled"
bash scripts/r3_nan_hunt.sh graph2 --peers 2 --rounds 3 --overlap off || exit $?
