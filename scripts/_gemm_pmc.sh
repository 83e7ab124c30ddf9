#!/bin/bash
# Counter passes for the square GEMM (one rocprofv3 --pmc pass each, kernel-trace only).
export TMPDIR=/tmp
cd /root/repo
mkdir -p gpurun_out/gpmc
timeout -k 10 200 python scripts/gemm_probe.py > gpurun_out/gpmc/probe.md 2>&1 || exit 1
for cfg in "8192 64"; do
  tag=$(echo $cfg | tr ' ' '_')
  for pass in "TCC_HIT_sum TCC_MISS_sum" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    ptag=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 60 rocprofv3 --pmc $pass --kernel-trace --stats --output-format csv -d gpurun_out/gpmc/${tag}_${ptag} -o run -- python scripts/gemm_one.py $cfg > gpurun_out/gpmc/${tag}_${ptag}.log 2>&1 || { echo "pass $tag $ptag failed rc=$?"; exit 1; }
  done
done
find gpurun_out/gpmc -type f | head -30; du -sh gpurun_out/gpmc
python - <<'PY'
import csv, glob, os
for d in sorted(glob.glob("gpurun_out/gpmc/*_*/")):
    f = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not f:
        print(d, "no counter csv"); continue
    rows = list(csv.DictReader(open(f[0])))
    agg = {}
    for r in rows:
        k = (r.get("Kernel_Name", "")[:60], r["Counter_Name"])
        agg.setdefault(k, []).append(float(r["Counter_Value"]))
    for (kn, cn), vals in sorted(agg.items()):
        if "gemm" in kn.lower() or "Cijk" in kn:
            print(os.path.basename(d.rstrip("/")), kn, cn, "median", sorted(vals)[len(vals)//2])
PY
find gpurun_out/gpmc -type f -size +512k -delete
du -sh gpurun_out/gpmc
