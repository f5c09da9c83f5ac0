#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output (kernel stats + optional PMC runs) into markdown.

  python bench/prof_summary.py --stats gpurun_out/prof/run_kernel_stats.csv \
      --pmc gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/xxx.md
"""
import argparse
import collections
import csv
import glob
import os
import re


def short(name: str) -> str:
    m = re.search(r"(k_\w+(<[^>]*>)?)", name)
    return m.group(1) if m else name[:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stats")
    ap.add_argument("--pmc", nargs="*", default=[])
    ap.add_argument("--title", default="rocprofv3 summary")
    a = ap.parse_args()
    print(f"# {a.title}\n")
    if a.stats and os.path.isdir(a.stats):  # a rocprofv3 output directory: its kernel-stats CSV
        found = glob.glob(os.path.join(a.stats, "**", "*kernel_stats.csv"), recursive=True)
        a.stats = found[0] if found else None
    if a.stats:
        rows = list(csv.DictReader(open(a.stats)))
        print("| kernel | calls | avg µs | total ms | % |")
        print("|---|---|---|---|---|")
        for r in rows:
            print(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
                  f"{float(r['TotalDurationNs'])/1e6:.2f} | {float(r['Percentage']):.1f} |")
        print()
    if a.pmc:
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        dur = collections.defaultdict(list)
        for d in a.pmc:
            for r in csv.DictReader(open(d + "/run_counter_collection.csv")):
                k = short(r["Kernel_Name"])
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        print("| kernel | median µs | FETCH_SIZE GB | WRITE_SIZE GB | TCC hit % | L2->fabric read GB | fabric write GB |")
        print("|---|---|---|---|---|---|---|")
        for k, v in agg.items():
            if not k.startswith("k_cg") and not k.startswith("k_dot"):
                continue
            f = v.get("FETCH_SIZE")
            w = v.get("WRITE_SIZE")
            h = v.get("TCC_HIT_sum")
            m = v.get("TCC_MISS_sum")
            fs = f"{sum(f)/len(f)/1e6:.3f}" if f else "-"
            ws = f"{sum(w)/len(w)/1e6:.3f}" if w else "-"
            hr = f"{100*sum(h)/(sum(h)+sum(m)):.1f}" if h and m else "-"
            rd = v.get("TCC_EA0_RDREQ_DRAM_32B_sum")
            wd = v.get("TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")
            rds = f"{32*sum(rd)/len(rd)/1e9:.2f}" if rd else "-"
            wds = f"{32*sum(wd)/len(wd)/1e9:.2f}" if wd else "-"
            ds = sorted(dur[k])
            print(f"| `{k}` | {ds[len(ds)//2]:.1f} | {fs} | {ws} | {hr} | {rds} | {wds} |")
        print("\nFETCH_SIZE/WRITE_SIZE are reported in KB by rocprofv3 (shown here as GB). On gfx950 FETCH_SIZE"
              " reads ~1/2 of the bytes of 16-B/lane streaming loads (MI355X_MICROARCH.md §HBM); compare ratios."
              " L2->fabric columns: TCC_EA0_{RDREQ,WRREQ_WRITE}_DRAM_32B x 32 B (calibrated exact on a copy kernel;"
              " includes Infinity-Cache hits), averaged over the profiled passes.")


if __name__ == "__main__":
    main()
