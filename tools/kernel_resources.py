#!/usr/bin/env python3
"""VGPRs / spills / occupancy of every kernel of a .hip file (hipcc
-Rpass-analysis=kernel-resource-usage), one line per kernel.

    python tools/kernel_resources.py firedancer_amd/csrc/fd_ed25519_kernels.hip [extra hipcc flags]
"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, {}
for line in err.splitlines():
    m = re.search(r"remark: +(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, r in rows.items():
    short = re.sub(r"^_Z\d+", "", name).split("26fd_")[0].split("P")[0]
    print(f"{short:40s} VGPR {r.get('VGPRs', '?'):>4}  AGPR {r.get('AGPRs', '?'):>4}  spill {r.get('VGPRs Spill', '?'):>4}  "
          f"scratch {r.get('ScratchSize [bytes/lane]', '?'):>4}  occ {r.get('Occupancy [waves/SIMD]', '?')}")
