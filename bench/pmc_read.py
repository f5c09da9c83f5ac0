#!/usr/bin/env python3
"""Print per-dispatch PMC values of the CG pass kernels from rocprofv3 SQLite output dirs.

  python bench/pmc_read.py gpurun_out/pmc_c1_a gpurun_out/pmc_c1_b
"""
import collections
import re
import sqlite3
import sys

for d in sys.argv[1:]:
    db = sqlite3.connect(f"{d}/run_results.db")
    cur = db.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(counters_collection)")]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in cur.execute("select * from counters_collection"):
        row = dict(zip(cols, r))
        name = str(row["kernel_name"])
        if "k_cg_f1" not in name and "k_cg_carry_ar" not in name:  # (k_cg_carry_ar3 included)
            continue
        k = re.search(r"(k_cg_(?:f1|carry_ar)\w*<[^>]*>)", name).group(1)
        agg[k][row["counter_name"]].append(row["value"])
    for k, v in agg.items():
        for cn, vals in sorted(v.items()):
            scale = 32e-9 if "DRAM_32B" in cn else 1.0
            print(d.split("/")[-1], k, cn, " ".join("%.4g" % (x * scale) for x in vals))
