# A/B of MIOpen's solver choice on the ResNet-18 config: the default find
# result vs the same with the ASM implicit-GEMM NHWC backward solvers disabled
# (their output pre-zeroing shows up as SubTensorOpWithScalar1d, ~7 % of the
# step in profiles/r2_resnet18_miopen_conv_steady_state.md).
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { name=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab_$name.log 2>&1; rc=$?; echo "$name rc $rc: $(grep -h '"metric"' gpurun_out/ab_$name.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])' 2>/dev/null)"; [ $rc -lt 124 ]; }
run r18_default python bench.py --model resnet18 --steps 5 --warmup 2 --watchdog 280 || exit 1
run r18_noasm env MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 python bench.py --model resnet18 --steps 5 --warmup 2 --watchdog 280 || exit 1
run r18_noasm_bwd env MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 python bench.py --model resnet18 --steps 5 --warmup 2 --watchdog 280 || exit 1
