"""Summarise gfx950 ISA per kernel: loads, MFMAs, LDS ops and vmcnt waits.

usage: python scripts/isa_summary.py csrc/cnn_bwd.hip [kernel-substring]
Compiles device-only assembly with the same flags as setup.py.
"""
import collections
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
out = "/tmp/_isa.s"
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-std=c++17", "-ffp-contract=fast",
                       "-munsafe-fp-atomics", "-Icsrc", "--cuda-device-only", "-S", src, "-o", out])
cur, body = None, collections.defaultdict(list)
for line in open(out):
    m = re.match(r"^(_Z\w+):", line)
    if m:
        cur = m.group(1)
        continue
    if cur and line.strip().startswith("s_endpgm"):
        cur = None
    if cur:
        body[cur].append(line)
for k, lines in body.items():
    if filt not in k:
        continue
    txt = "".join(lines)
    waits = collections.Counter(re.findall(r"s_waitcnt vmcnt\((\d+)\)", txt))
    print(f"{k[:90]}\n  lines={len(lines)} gload={txt.count('global_load')} gstore={txt.count('global_store')} "
          f"mfma={txt.count('v_mfma')} ds_read={txt.count('ds_read')} ds_write={txt.count('ds_write')} "
          f"vmcnt waits={dict(sorted(waits.items(), key=lambda kv: int(kv[0])))}")
