#!/usr/bin/env python3
"""Does a wave of ~270 VGPRs start on CUs that a CU-masked resident grid leaves free?  (one MI355X)

profiles/r3_corun_root_cause.md shows that RCCL's kernels (261-280 VGPRs per wave) and a fat
control kernel without RCCL both wait for the resident CG pass, while a thin kernel starts at once.
The round-2 review asked about the one row that does not fit that explanation: with 16 CUs withheld
from the pass through a CU-masked queue (r2_corun_probe.md) the send/recv still waited.  That run
sized the pass's grid for all 256 CUs, so its blocks overflowed onto a second round and the pass
took 1.6x as long; whether the withheld CUs were really free was never observed.

This probe removes the solver from the question.  A hog grid (k_spin<kHogRegs>, ~120 VGPRs, 4
blocks of 256 threads per CU: the carry pass's footprint) spins for `--hog-us` on a CU-masked
stream, sized to 4 blocks per CU the mask enables; each block records __smid().  Then, on a
high-priority unmasked side stream: the fat spin (20 us, records where it ran), the thin spin, and
a 1-rank RCCL grouped send/recv to itself.  For each mask: how long the side kernel took with the
hog resident, how many distinct CUs the hog used, and whether the fat wave landed outside them.

  python bench/cumask_probe.py [--hog-us 2000] [--withhold 0,8,16,32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def masks(ncu: int, withhold: int, how: str) -> list[int]:
    """ncu bits, `withhold` of them cleared: the top ones ("top") or spread evenly ("spread")."""
    bits = [1] * ncu
    if withhold > 0:
        if how == "top":
            for i in range(ncu - withhold, ncu):
                bits[i] = 0
        else:
            step = ncu // withhold
            for j in range(withhold):
                bits[j * step + step - 1] = 0
    words = []
    for w in range((ncu + 31) // 32):
        v = 0
        for b in range(32):
            i = w * 32 + b
            if i < ncu and bits[i]:
                v |= 1 << b
        words.append(v)
    return words


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--hog-us", type=float, default=2000.0)
    ap.add_argument("--withhold", default="0,8,16,32")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rccl", type=int, default=1)
    a = ap.parse_args()

    import torch

    import cuda_mpi_parallel_amd as mcg

    torch.cuda.set_device(0)
    C = mcg.native()
    K = C.kernels
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    side = torch.cuda.Stream(priority=-1)
    out = torch.zeros(8192, dtype=torch.float64, device="cuda")
    hog_where = torch.full((8192,), -1, dtype=torch.int32, device="cuda")
    fat_where = torch.full((8,), -1, dtype=torch.int32, device="cuda")
    comm = C.Comm(0, 1, C.unique_id(), C.unique_id()) if a.rccl else None
    msg = 3 * 16384
    src = torch.rand(msg, dtype=torch.float64, device="cuda")
    dst = torch.zeros_like(src)

    def side_op(kind):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(side)
        if kind == "spin_fat":
            K.spin(out.data_ptr(), 20.0, True, 1, side.cuda_stream, fat_where.data_ptr())
        elif kind == "spin_thin":
            K.spin(out.data_ptr(), 20.0, False, 1, side.cuda_stream)
        else:
            comm.sendrecv_ptr(src.data_ptr(), 0, dst.data_ptr(), 0, msg, side.cuda_stream)
        e1.record(side)
        return e0, e1

    rows = []
    all_used: set = set()
    for how in ("top", "spread"):
        for w in [int(x) for x in a.withhold.split(",")]:
            if how == "spread" and w == 0:
                continue
            words = masks(ncu, w, how)
            st = K.cu_mask_stream(words)
            ms = torch.cuda.ExternalStream(st)
            blocks = 4 * (ncu - w)
            row = {"mask": how, "withheld": w, "hog_blocks": blocks}
            # the hog alone: one round of blocks takes hog_us if the mask enables ncu - w CUs
            h0, h1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            h0.record(ms)
            K.hog(out.data_ptr(), a.hog_us, blocks, st, hog_where.data_ptr())
            h1.record(ms)
            torch.cuda.synchronize()
            row["hog_alone_us"] = round(h0.elapsed_time(h1) * 1e3, 1)
            used = set(hog_where[:blocks].tolist())
            row["hog_distinct_cus"] = len(used)
            if w == 0:
                all_used = used
                row["smids"] = sorted(used)  # __smid = xcc | se | cu (amd_device_functions.h)
            else:
                row["smids_missing"] = sorted(all_used - used)
            kinds = ["spin_fat", "spin_thin"] + (["rccl"] if comm is not None else [])
            for kind in kinds:
                vals, landed_free = [], []
                for _ in range(a.reps):
                    torch.cuda.synchronize()
                    fat_where.fill_(-1)
                    torch.cuda.synchronize()
                    K.hog(out.data_ptr(), a.hog_us, blocks, st, 0)
                    time.sleep(0.0003)  # let the hog's blocks land
                    e0, e1 = side_op(kind)
                    torch.cuda.synchronize()
                    vals.append(round(e0.elapsed_time(e1) * 1e3, 1))
                    if kind == "spin_fat":
                        landed_free.append(int(fat_where[0].item()) not in used)
                row[kind + "_with_hog_us"] = vals
                if kind == "spin_fat":
                    row["fat_on_cu_hog_did_not_use"] = landed_free
            torch.cuda.synchronize()
            K.stream_destroy(st)
            rows.append(row)
            print(json.dumps(row), flush=True)
    if comm is not None:
        comm.check_async()
    print(json.dumps({"ncu": ncu, "hog_us": a.hog_us, "rows": len(rows)}), flush=True)
    torch.cuda.synchronize()
    sys.stdout.flush()
    os._exit(0)


if __name__ == "__main__":
    sys.exit(main())
