#!/usr/bin/env python3
"""Per-dispatch counter totals from rocprofv3 CSV output (--output-format csv), for kernels whose
name contains a substring; DRAM_32B counters are converted to GB, and with GRBM_GUI_ACTIVE the
dispatch's bytes / time (GRBM_GUI_ACTIVE counts each of the 8 XCDs' busy cycles: divided by 8 at
the `--mhz` clock, default 2400, it matches the kernel-trace duration).

  python bench/pmc_csv.py gpurun_out/<dir> k_tiles [--mhz 2400]
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel")
    ap.add_argument("--mhz", type=float, default=2400.0)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    agg = collections.OrderedDict()
    names = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if a.kernel not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            cn, v = r["Counter_Name"], float(r["Counter_Value"])
            slot = agg.setdefault(d, collections.defaultdict(float))
            # GRBM_GUI_ACTIVE is reported per XCD (the same cycles 8 times): keep the largest
            slot[cn] = max(slot[cn], v) if cn.startswith("GRBM") else slot[cn] + v
            nm = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            names[d] = nm.split("(")[0].replace("void mcg::kern::", "")
    for d, cs in sorted(agg.items()):
        parts = []
        rd = cs.get("TCC_EA0_RDREQ_DRAM_32B_sum")
        wr = cs.get("TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")
        if rd is not None:
            parts.append(f"DRAM read {rd * 32e-9:8.2f} GB")
        if wr is not None:
            parts.append(f"write {wr * 32e-9:7.2f} GB")
        h, m = cs.get("TCC_HIT_sum"), cs.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            parts.append(f"L2 hit {100 * h / (h + m):5.1f} % ({h:.3e} hits, {m:.3e} misses)")
        g = cs.get("GRBM_GUI_ACTIVE")
        if g:
            ms = g / 8 / (a.mhz * 1e3)
            parts.append(f"{ms:8.2f} ms")
            if rd is not None:
                parts.append(f"{(rd + (wr or 0)) * 32 / (ms * 1e-3) / 1e12:5.2f} TB/s")
        print(f"{d:5d} {names[d][:60]:60s} " + "  ".join(parts))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
