#!/usr/bin/env python3
"""Inter-kernel gaps of the CG pass kernels from a rocprofv3 kernel trace (csv).

  python bench/gap_summary.py gpurun_out/gap2/run_kernel_trace.csv
Takes the last N pass kernels (k_cg_f1*) and the reduce kernels between them, and reports the
mean wall time per iteration, the mean busy time and the mean idle gap between kernels."""
import csv
import sys


def main(path, last=120):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in rows if "k_cg_" in r["Kernel_Name"]]
    ks = ks[-2 * last:]
    t0, t1 = int(ks[0]["Start_Timestamp"]), int(ks[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks)
    iters = sum(1 for r in ks if "reduce" in r["Kernel_Name"])
    gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(ks, ks[1:])]
    print(f"{path}: {iters} iterations, wall {(t1 - t0) / iters / 1e3:.1f} us/iter, "
          f"busy {busy / iters / 1e3:.1f} us/iter, mean gap {sum(gaps) / len(gaps) / 1e3:.2f} us, "
          f"max gap {max(gaps) / 1e3:.1f} us")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
