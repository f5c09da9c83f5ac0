#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench/corun_probe.py: for every probe dispatch (RCCL
send/recv, the spin controls, the torch add) its queue id, and how long after its previous
co-queued pass dispatch started it began (start delay) vs how long it ran.

  python bench/corun_trace.py gpurun_out/<dir>/..._kernel_trace.csv
"""
from __future__ import annotations

import csv
import sys


def main(path: str) -> int:
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    passes = [r for r in rows if "carry" in r["Kernel_Name"] or "fused1" in r["Kernel_Name"]]
    probes = [r for r in rows if any(k in r["Kernel_Name"] for k in ("rccl", "Rccl", "k_spin", "add", "Add"))]
    qids = sorted({r.get("Queue_Id", "?") for r in rows})
    print(f"queues seen: {qids}; pass dispatches {len(passes)}, probe dispatches {len(probes)}")
    print("kernel | queue | start after a pass was running (us) | ran (us) | pass running at start")
    for r in probes:
        t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        running = [p for p in passes if int(p["Start_Timestamp"]) <= t0 < int(p["End_Timestamp"])]
        prev_end = max([int(p["End_Timestamp"]) for p in passes if int(p["End_Timestamp"]) <= t0], default=None)
        name = r["Kernel_Name"].split("(")[0][:48]
        gap = (t0 - prev_end) / 1e3 if prev_end else float("nan")
        print(f"{name:48s} | {r.get('Queue_Id', '?'):>3s} | after prev pass end {gap:9.1f} | {(t1 - t0) / 1e3:8.1f} | "
              f"{'yes' if running else 'no'}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
