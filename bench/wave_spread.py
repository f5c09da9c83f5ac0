#!/usr/bin/env python3
"""Per-wave timing of one carry pass (the -DMCG_CARRY_DIAG build, cg_carry_ar.hip): how long the pass's
fill, drain and reduction tail take, and whether the slow waves are the youngest workgroups on their CU.

  python bench/wave_spread.py gpurun_out/diag4096.1500 [...]

Input lines: block wave t_in t_work t_out hw_id xcc_id (wall clock, 100 MHz ticks).
"""
from __future__ import annotations

import json
import sys
from collections import defaultdict

TICK_US = 0.01  # s_memrealtime: 100 MHz


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * (len(xs) - 1) + 0.5))]


def summarise(path: str) -> dict:
    rows = []
    for line in open(path):
        f = line.split()
        if len(f) < 7:
            continue
        b, w, ti, tw, to, hw, xcc = (int(x) for x in f[:7])
        if ti == 0 or to == 0:
            continue
        rows.append((b, w, ti, tw, to, hw, xcc))
    t0 = min(r[2] for r in rows)
    t_end = max(r[4] for r in rows)
    t_work_max = max(r[3] for r in rows)
    start = [(r[2] - t0) * TICK_US for r in rows]
    work = [(r[3] - r[2]) * TICK_US for r in rows]
    fin = [(r[3] - t0) * TICK_US for r in rows]
    # age rank of a workgroup on its CU: order of its entry among the CU's workgroups
    per_cu = defaultdict(dict)
    for b, w, ti, tw, to, hw, xcc in rows:
        cu = (xcc, (hw >> 8) & 0xFF)
        per_cu[cu][b] = min(ti, per_cu[cu].get(b, ti))
    rank = {}
    for cu, blocks in per_cu.items():
        for i, (b, _) in enumerate(sorted(blocks.items(), key=lambda kv: (kv[1], kv[0]))):
            rank[b] = i
    by_rank = defaultdict(list)
    for r, wk in zip(rows, work):
        by_rank[rank[r[0]]].append(wk)
    return {
        "file": path,
        "waves": len(rows),
        "cus": len(per_cu),
        "pass_us": round((t_end - t0) * TICK_US, 2),
        "entry_spread_us": {"p50": round(pct(start, 0.5), 2), "p99": round(pct(start, 0.99), 2), "max": round(max(start), 2)},
        "work_us": {"min": round(min(work), 2), "p50": round(pct(work, 0.5), 2), "p90": round(pct(work, 0.9), 2),
                    "max": round(max(work), 2)},
        "finish_us": {"p10": round(pct(fin, 0.1), 2), "p50": round(pct(fin, 0.5), 2), "p90": round(pct(fin, 0.9), 2),
                      "p99": round(pct(fin, 0.99), 2), "max": round(max(fin), 2)},
        "reduction_tail_us": round((t_end - t_work_max) * TICK_US, 2),
        "work_us_by_age_on_cu": {str(k): round(sum(v) / len(v), 2) for k, v in sorted(by_rank.items())},
    }


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(json.dumps(summarise(p)))
