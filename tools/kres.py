#!/usr/bin/env python3
"""Per-kernel resource usage of one HIP source (hipcc -Rpass-analysis=kernel-resource-usage), as a
table: VGPRs, AGPRs, spills, LDS, occupancy.  CPU only (cross-compiles for gfx950).

  python tools/kres.py csrc/gpu/cg_carry_ar.hip [--filter carry_ar]
"""
import argparse
import re
import subprocess
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-Icsrc/include", "-Wno-unused-function",
           "--offload-arch=gfx950", "-munsafe-fp-atomics", "-c", a.src, "-o", "/dev/null",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line) or re.search(r"Name: (\S+) \[", line)
        if m and "Function Name" in line or (m and cur is None):
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\S+) \[", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
    if "error" in out and not rows:
        print(out[-3000:])
        return 1
    for r in rows:
        if a.filter not in r["name"]:
            continue
        dm = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
        dm = re.sub(r"mcg::kern::\(anonymous namespace\)::", "", dm)
        dm = dm.split("(")[0]
        print(f"{r.get('VGPRs', '?'):>4} v {r.get('AGPRs', '?'):>3} a  spill v{r.get('VGPRs Spill', '?')} "
              f"s{r.get('SGPRs Spill', '?')}  occ {r.get('Occupancy [waves/SIMD]', '?')}  lds {r.get('LDS Size [bytes/block]', '?'):>6}  {dm}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
