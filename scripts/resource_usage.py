#!/usr/bin/env python3
"""Per-kernel register use of one HIP source (tuning aid): compiles it for
gfx950 with -Rpass-analysis=kernel-resource-usage and prints one line per
kernel: VGPRs, AGPRs, SGPRs, spills, scratch, occupancy.

    python scripts/resource_usage.py hummingbird_amd/csrc/odd.hip [name-regex]
"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, f"-I{ROOT}/include",
       f"-I{ROOT}/hummingbird_amd/csrc", "-Rpass-analysis=kernel-resource-usage", "-o", "/dev/null",
       *[f"-D{d}" for d in sys.argv[3:]]]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark: (.*) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    print(f'{r["name"][:70]:70s} V={r.get("VGPRs")} A={r.get("AGPRs")} S={r.get("TotalSGPRs")} '
          f'Sspill={r.get("SGPRs Spill")} Vspill={r.get("VGPRs Spill")} scratch={r.get("ScratchSize [bytes/lane]")} '
          f'occ={r.get("Occupancy [waves/SIMD]")}')
