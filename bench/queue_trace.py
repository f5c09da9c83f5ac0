#!/usr/bin/env python3
"""Per-hardware-queue view of a rocprofv3 kernel trace (csv): for every kernel kind, which queues it
ran on and how long it took there.  Written for the DelayComm overlap anomaly:
`bench/pipe_latency.py --overlaps 1 --delays 10,20` under `rocprofv3 --kernel-trace --output-format
csv`; the run holds two solver instances (D = 10 us, then D = 20 us), split at the largest gap
between passes.

    python bench/queue_trace.py gpurun_out/anom/run_kernel_trace.csv
"""
import collections
import csv
import json
import statistics
import sys


def kind(name: str) -> str:
    if "k_spin" in name:
        return "spin"
    if "k_cg_carry_ar" in name:
        return "pass"
    return "other"


def main(path: str) -> None:
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind(r["Kernel_Name"]), r["Queue_Id"]) for r in rows]
    passes = [i for i, e in enumerate(ev) if e[2] == "pass"]
    gaps = [(ev[passes[j + 1]][0] - ev[passes[j]][1], j) for j in range(len(passes) - 1)]
    cut = passes[max(gaps)[1] + 1]  # the second solver instance starts after the longest gap
    for label, sub in (("first instance", ev[:cut]), ("second instance", ev[cut:])):
        ps = [e for e in sub if e[2] == "pass"]
        it = [(ps[i + 1][0] - ps[i][0]) / 1e3 for i in range(len(ps) - 1)]
        per_q = collections.defaultdict(list)
        for s, e, k, q in sub:
            if k == "spin":
                per_q[q].append((e - s) / 1e3)
        print(json.dumps({
            "instance": label, "passes": len(ps), "pass_queues": sorted({e[3] for e in ps}),
            "median_us_between_pass_starts": round(statistics.median(it), 2) if it else None,
            "spins_by_queue": {q: {"n": len(v), "median_us": round(statistics.median(v), 2),
                                   "over_30us": sum(1 for x in v if x > 30)} for q, v in sorted(per_q.items())},
        }))


if __name__ == "__main__":
    main(sys.argv[1])
