#!/usr/bin/env python3
"""Kernel-variant / launch-geometry sweep on one GPU (one process, configs interleaved
over rounds so clock drift hits every config alike).

A config is  fmt:vV:pP:bB:uU  (format csr|sell|sell16|sellc8, SpMV engine V, batch/lanes P,
blocks per CU B, residual-update unroll U; also nN non-temporal, xX XCD map, sS slices/wave,
rR recurrence, iI interleaved r/Ap pairs, wW LDS-window pass, BN update blocks per CU, cC line-carry pass,
kK line-carry blocks per CU, dD line-carry prefetch depth, T1 line-carry non-temporal operand loads), e.g.

  python bench/sweep.py --n 16384 --steps 30 --cfg csr:v1:p6:b8:u2 csr:v0:p6:b6:u2 sell:v1:p6:b8:u2
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cuda_mpi_parallel_amd as mcg  # noqa: E402


def parse_cfg(s):
    parts = s.split(":")
    d = {"format": parts[0], "v": -1, "p": 0, "b": 0, "u": 1, "g": 1, "n": 0, "x": -1, "s": 1, "r": 0, "i": -1, "w": -1, "P": -1, "S": -1, "c": 0, "k": 4, "d": 0, "T": 0}
    for q in parts[1:]:
        d[q[0]] = int(q[1:])
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--problem", default="poisson2d")
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--band", type=int, default=4096)
    ap.add_argument("--density", type=float, default=0.16)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--cfg", nargs="+", default=["csr:v1:p6:b8:u2"])
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    C = mcg.native()
    if args.problem == "randspd":
        spec = mcg.make_problem("randspd", rows=args.rows, band=args.band, density=args.density)
    else:
        spec = mcg.make_problem(args.problem, n=args.n)
    results = {}
    ref_rnorm = None
    for rnd in range(args.rounds):
        for cs in args.cfg:
            c = parse_cfg(cs)
            o = C.CgOptions(maxit=1 << 30, tol=-1.0, check_every=1 << 30, use_graph=bool(c["g"]), format=c["format"],
                            blocks_per_cu=c["b"], spmv_variant=c["v"], recurrence=c["r"])
            # fields of earlier experiments (strip, carry_depth, carry_nt, ...) were removed in r3
            for key, field in (("B", "update_blocks_per_cu"), ("i", "interleave"), ("w", "window"), ("P", "pipeline"),
                               ("c", "carry")):
                if key in c and hasattr(o, field):
                    setattr(o, field, c[key])
            s = C.Solver(spec.native(), o, 0, 1, None)
            s.setup()
            s.reset()
            s.run_iterations(args.warmup)
            s.synchronize()
            t0 = time.perf_counter()
            s.run_iterations(args.steps)
            s.synchronize()
            dt = time.perf_counter() - t0
            r = s.result()
            if ref_rnorm is None:
                ref_rnorm = r["rnorm"]
            agree = abs(r["rnorm"] - ref_rnorm) <= 1e-6 * abs(ref_rnorm)
            results.setdefault(cs, []).append(args.steps / dt)
            info = s.info
            print(json.dumps({"round": rnd, "cfg": cs, "it_per_s": round(args.steps / dt, 2),
                              "tb_s": round(info["bytes_per_iter_model"] * args.steps / dt / 1e12, 3),
                              "rnorm_agrees": agree, "variant": info["spmv_variant"], "param": info["spmv_param"],
                              "grid_a": info["grid_a"]}), flush=True)
            del s
    best = {k: round(max(v), 2) for k, v in results.items()}
    print(json.dumps({"best": dict(sorted(best.items(), key=lambda kv: -kv[1]))}))


if __name__ == "__main__":
    main()
