cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 400 "$@" > gpurun_out/mb_$name.log 2>&1; rc=$?; echo "$name rc $rc: $(grep -h '"metric"' gpurun_out/mb_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>/dev/null) $(grep -h 'kernel choice' gpurun_out/mb_$name.log)"; [ $rc -lt 124 ]; }
run vit_auto python bench.py --model vit_b16 --steps 3 --warmup 1 --watchdog 380 || exit 1
run r50_auto python bench.py --model resnet50 --steps 3 --warmup 1 --watchdog 380 || exit 1
run r18_auto python bench.py --model resnet18 --steps 5 --warmup 1 --watchdog 380 || exit 1
