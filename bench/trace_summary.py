#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite ``*_results.db`` or ``kernel_trace.csv``).

Prints per-kernel totals, and for the steady-state iteration window (the last ``--iters``
dispatches of the main pass kernel, matched by ``--pass``) the kernels launched per iteration
and the inter-kernel gaps (start of one dispatch - end of the previous one, same queue order).

  python bench/trace_summary.py gpurun_out/prof4096fc/run_results.db --pass k_cg_f1 --iters 48
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import sqlite3
import statistics
import sys


def load(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        rows = c.execute("select name, start, end from kernels order by start").fetchall()
        return [(n, int(s), int(e)) for n, s, e in rows]
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(out, key=lambda t: t[1])


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "").replace("mcg::kern::", "")[:80]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--pass", dest="pat", default="k_cg_f1", help="substring of the per-iteration pass kernel")
    ap.add_argument("--iters", type=int, default=48, help="steady-state iterations to analyse (from the end)")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    ks = load(a.trace)
    tot = collections.defaultdict(lambda: [0, 0])
    for n, s, e in ks:
        t = tot[short(n)]
        t[0] += 1
        t[1] += e - s
    idx = [i for i, (n, _, _) in enumerate(ks) if a.pat in n]
    if len(idx) < 2:
        print("pass kernel not found", file=sys.stderr)
        return 1
    idx = idx[-(a.iters + 1):]
    lo, hi = idx[0], idx[-1]
    window = ks[lo:hi]
    per_iter = (hi - lo) / (len(idx) - 1)
    names = collections.Counter(short(n) for n, _, _ in window)
    gaps = [window[i + 1][1] - window[i][2] for i in range(len(window) - 1)]
    pass_us = [(e - s) / 1e3 for n, s, e in window if a.pat in n]
    res = {
        "iterations": len(idx) - 1,
        "kernels_per_iteration": round(per_iter, 3),
        "kernels_in_window": dict(names),
        "gap_us_mean": round(statistics.mean(gaps) / 1e3, 3) if gaps else None,
        "gap_us_median": round(statistics.median(gaps) / 1e3, 3) if gaps else None,
        "gap_us_max": round(max(gaps) / 1e3, 3) if gaps else None,
        "pass_us_mean": round(statistics.mean(pass_us), 2),
        "iteration_us_mean": round((ks[hi][1] - ks[lo][1]) / 1e3 / (len(idx) - 1), 2),
    }
    if a.json:
        print(json.dumps(res))
    else:
        print("per-kernel totals (calls, total us, mean us):")
        for k, (c, d) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:15]:
            print(f"  {c:7d} {d / 1e3:12.1f} {d / 1e3 / c:9.2f}  {k}")
        for k, v in res.items():
            print(f"{k}: {v}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
