#!/usr/bin/env python3
"""One recipe runner for every GPU-box command of this repo (replaces the per-experiment shell
launchers).  Run on the box:

  gpurun -- 'python bench/gpu_run.py check'            # GPU tests + smoke + headline bench
  gpurun -- 'python bench/gpu_run.py prof --grid 4096' # rocprofv3 kernel trace + summary
  python bench/gpu_run.py --list                       # recipes and their steps

Every step runs under its own ``timeout -k 10 <s>``, writes stdout/stderr to
``gpurun_out/<recipe>_<step>.{out,err}``, and the recipe stops at the first failing step (a GPU
fault, an abort or a time limit ends the call: no step runs after it).  Counter passes hold at
most one PMC group per rocprofv3 run (the limits of MI355X_MICROARCH.md: 8 SQ, 4 TCC).
"""
from __future__ import annotations

import argparse
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PY = sys.executable
PYTEST = f"{PY} -u -m pytest -x -q --timeout 300 --timeout-method thread"
PROF = "rocprofv3"
# BASELINE config 5, genuinely irregular: a P = 8 rank's share (12.5 M rows, 8.33 G nnz, ~101 GB) of the
# scrambled random SPD (P^T A P), alone on one GPU with collectives that move nothing
C5SCR = "--problem randspd --rows 100000000 --band 410 --density 1.0 --scramble 1 --sim-world 8 --sim-rank 3"


def bench(extra: str = "") -> str:
    return f"{PY} bench.py {extra}".strip()


def prof(tag: str, cmd: str, pmc: str = "") -> str:
    """rocprofv3 around `cmd` (the program itself right after --, never a wrapper)."""
    what = f"--pmc {pmc}" if pmc else "--kernel-trace --stats"
    return f"{PROF} {what} -d {OUT}/{tag} -o run -- {cmd}"


def recipes(a) -> dict:
    g = a.grid
    return {
        # round-end style check: what the driver runs, in one call
        "check": [
            ("pytest_gpu", 900, f"{PYTEST} tests -m gpu"),
            ("smoke", 300, f"{PY} -c 'import __graft_entry__ as g; g.smoke()'"),
            ("bench", 200, bench()),
            ("bench_spawn", 200, bench("--gpus 1 --spawn")),
            ("bench_3d", 200, bench("--problem poisson3d --grid 512")),
        ],
        "tests": [("pytest_gpu", 900, f"{PYTEST} tests -m gpu")],
        "bench": [
            ("smoke", 300, f"{PY} -c 'import __graft_entry__ as g; g.smoke()'"),
            ("bench", 200, bench()),
            ("bench_spawn", 200, bench("--gpus 1 --spawn")),
            ("bench_3d", 200, bench("--problem poisson3d --grid 512")),
            ("bench_4096", 200, bench("--grid 4096 --steps 2000 --warmup 100")),
        ],
        # BASELINE.json configs on one GPU (config 5 at its per-GPU share: 12.5 M rows, ~150 GB)
        "configs": [
            ("c1_cpu_1024", 900, f"bin/mcg-cg --device cpu --problem poisson2d --n 1024 --fixed-iters 200 "
                                 f"--report json"),
            ("c2_4096", 200, bench("--grid 4096 --steps 2000 --warmup 100")),
            ("c3_16384", 200, bench()),
            ("c4_512", 200, bench("--problem poisson3d --grid 512")),
            ("c5_randspd", 600, bench("--problem randspd --rows 12500000 --band 650 --density 1.0 "
                                      "--spread 12500000 --steps 10 --warmup 2 --phases 3")),
        ],
        # variants of the current tree on the same box: every number of the README table
        "variants": [
            ("generic_c8", 200, bench("--set carry=0")),
            ("sell16", 200, bench("--format sell16")),
            ("csr_two", 200, bench("--format csr --recurrence 0")),
            ("csr_single", 200, bench("--format csr --recurrence 1")),
            ("no_fused_reduce", 200, bench("--set fused_reduce=0")),
            ("force_comm", 200, bench("--force-comm")),
        ],
        # kernel trace + per-iteration kernel count / gaps of one grid
        "prof": [
            ("trace", 300, prof(f"prof{g}", f"{PY} {ROOT}/bench.py --grid {g} --steps 64 --warmup 8 --phases 0 "
                                            f"--force-comm")),
            ("summary", 60, f"{PY} bench/trace_summary.py {OUT}/prof{g}/run_results.db --pass k_cg_carry_ar --iters 48"),
        ],
        # counter passes (one group per run) of the headline pass
        "pmc": [
            ("bytes", 90, prof("pmc_bytes", f"{PY} {ROOT}/bench.py --grid {g} --steps 4 --warmup 2 --phases 0 "
                                             f"--no-verify", "TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum "
                                                             "GRBM_GUI_ACTIVE")),
            ("waves", 90, prof("pmc_waves", f"{PY} {ROOT}/bench.py --grid {g} --steps 4 --warmup 2 --phases 0 "
                                             f"--no-verify", "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY "
                                                             "SQ_ACTIVE_INST_ANY SQ_WAVES")),
        ],
        # irregular-sparsity path (config 5): split pass, wide matrix, user matrices
        "irregular": [
            ("pytest", 900, f"{PYTEST} -v tests/test_gpu_irregular.py tests/test_gpu_user_matrix.py "
                            f"tests/test_gpu_rccl.py tests/test_gpu_fused_reduce.py"),
            ("rand200", 600, bench("--problem randspd --rows 12500000 --band 650 --density 1.0 --spread 12500000 "
                                   "--steps 10 --warmup 2 --phases 3")),
            ("rand30", 300, bench("--problem randspd --rows 12500000 --band 100 --density 1.0 --spread 12500000 "
                                  "--steps 20 --warmup 2")),
            ("rand30_fused", 300, bench("--problem randspd --rows 12500000 --band 100 --density 1.0 "
                                        "--spread 12500000 --steps 20 --warmup 2 --set pmat=0")),
            ("prof_rand30", 400, prof("prof_rand30", f"{PY} {ROOT}/bench.py --problem randspd --rows 12500000 "
                                                     f"--band 100 --density 1.0 --spread 12500000 --steps 10 "
                                                     f"--warmup 2 --phases 0")),
        ],
        # config 5 at ~200 GB per GPU: bench, XCD-ordered slices, kernel stats, L2->fabric bytes
        "config5": [
            ("bench", 900, bench("--problem randspd --rows 12500000 --band 820 --density 1.0 --spread 12500000 "
                                 "--steps 6 --warmup 1 --phases 2")),
            ("bench1640", 900, bench("--problem randspd --rows 12500000 --band 1640 --density 1.0 "
                                     "--spread 12500000 --steps 4 --warmup 1 --phases 2")),
            ("plain820", 900, bench("--problem randspd --rows 12500000 --band 820 --density 1.0 --spread 12500000 "
                                    "--steps 6 --warmup 1 --phases 2 --set sell_aligned=0")),
            ("xcd100", 300, bench("--problem randspd --rows 12500000 --band 100 --density 1.0 --spread 12500000 "
                                  "--steps 20 --warmup 2 --set xcd_map=1")),
            ("xcd650", 600, bench("--problem randspd --rows 12500000 --band 650 --density 1.0 --spread 12500000 "
                                  "--steps 6 --warmup 1 --set xcd_map=1")),
            ("stats", 900, prof("c5_stats", f"{PY} {ROOT}/bench.py --problem randspd --rows 12500000 --band 820 "
                                            f"--density 1.0 --spread 12500000 --steps 4 --warmup 1 --phases 0")),
            ("bytes", 900, prof("c5_bytes", f"{PY} {ROOT}/bench.py --problem randspd --rows 12500000 --band 820 "
                                            f"--density 1.0 --spread 12500000 --steps 2 --warmup 1 --phases 0 "
                                            f"--no-verify", "TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum "
                                                            "GRBM_GUI_ACTIVE")),
        ],
        # one rank's share of a P-rank run, alone on this GPU (NullComm: collectives move nothing):
        # the per-rank work the scaling runs will see, without the communication latency
        "simrank": [
            (f"p{P}_r{r}", 200, bench(f"--sim-world {P} --sim-rank {r} --steps 400 --warmup 40 --phases 10"))
            for P, r in ((2, 0), (4, 1), (8, 0), (8, 3), (8, 7))
        ] + [
            (f"p{P}_r{r}_3d", 200, bench(f"--problem poisson3d --grid 512 --sim-world {P} --sim-rank {r} "
                                         f"--steps 400 --warmup 40 --phases 10"))
            for P, r in ((8, 3),)
        ],
        # config 5 at a P = 8 rank's share (1e8 rows spread over all rows, 12.5 M per rank): the
        # all-gather overlap halves (own-block slots || all-gather, then the rest) vs one pass
        "agoverlap": [
            ("pytest", 600, f"{PYTEST} -v tests/test_gpu_irregular.py -k 'all_gather or aligned'"),
        ] + [
            (f"sim8_ag{ag}", 900, bench(f"--problem randspd --rows 100000000 --band 820 --density 1.0 "
                                        f"--spread 100000000 --sim-world 8 --sim-rank 3 --steps 6 --warmup 1 "
                                        f"--phases 2 --set ag_overlap={ag}"))
            for ag in (1, 0)
        ],
        # does a halo collective find CUs while the (fully resident) carry pass runs?
        "corun": [
            ("graph", 180, f"{PY} bench/corun_probe.py"),
            ("eager", 180, f"{PY} bench/corun_probe.py --graph 0"),
            ("b3", 180, f"{PY} bench/corun_probe.py --set carry_blocks_per_cu=3"),
            ("generic", 180, f"{PY} bench/corun_probe.py --set carry=0"),
        ],
        # CUs withheld from the compute stream (CU-masked queue) so the collective finds room; the
        # pass time with the mask (full grid and a P = 8 rank's share) is the price
        # Ap recomputed by the line-carry pass instead of stored as {r, Ap} pairs
        "apr": [
            ("pytest", 900, f"{PYTEST} tests -m gpu"),
        ] + [
            (f"b{i}_ar{ar}", 200, bench(f"--set ap_recompute={ar}")) for i, ar in enumerate((-1, 0, -1, 0))
        ] + [
            ("b4096_ar", 200, bench("--grid 4096 --steps 2000 --warmup 100")),
            ("b4096_st", 200, bench("--grid 4096 --steps 2000 --warmup 100 --set ap_recompute=0")),
            ("sim8_ar", 200, bench("--sim-world 8 --sim-rank 3 --steps 400 --warmup 40 --phases 10")),
            ("sim8_st", 200, bench("--sim-world 8 --sim-rank 3 --steps 400 --warmup 40 --phases 10 "
                                   "--set ap_recompute=0")),
        ],
        # quick A/B of the Ap-recomputing carry (numerics tests + 16384^2 / 4096^2 / P = 8 share)
        "arquick": [
            ("pytest", 300, f"{PYTEST} tests/test_gpu_solver.py tests/test_gpu_multirank.py -k 'ap_recompute or halo_ahead'"),
        ] + [
            (f"{nm}_{g}", 200, bench(f"{'--grid 4096 --steps 2000 --warmup 100 ' if g == 4096 else ''}--phases 0 "
                                     f"{arg}"))
            for g in (16384, 4096)
            for nm, arg in (("ar_d2", "--set carry_depth=2"), ("ar_d3", "--set carry_depth=3"),
                            ("st", "--set ap_recompute=0"), ("ar_d3b", "--set carry_depth=3"))
        ],
        # Ap-recomputing carry: prefetch depth x blocks per CU (16384^2 and 4096^2)
        "arsweep": [
            (f"d{d}_b{b}_{g}", 200, bench(f"{'--grid 4096 --steps 2000 --warmup 100 ' if g == 4096 else ''}"
                                        f"--phases 0 --no-verify --set carry_depth={d} --set carry_blocks_per_cu={b}"))
            for g in (16384, 4096) for d in (2, 3, 4, 5) for b in (4, 3)
        ],
        # issue-side counters of the Ap-recomputing vs the storing carry pass (16384^2)
        "arpmc": [
            (f"{tag}_{nm}", 120, prof(f"arpmc_{tag}_{nm}", f"{PY} {ROOT}/bench.py --steps 8 --warmup 2 --phases 0 "
                                                         f"--no-verify --set ap_recompute={ar}", cnt))
            for tag, ar in (("ar", -1), ("st", 0))
            for nm, cnt in (("valu", "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU "
                                     "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS"),
                            ("mem", "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS "
                                    "SQ_INSTS_SALU SQ_WAIT_ANY GRBM_GUI_ACTIVE"))
        ],
        # halo exchanged ahead (next to the all-reduce, one full pass) vs interior || halo + boundary
        "haloahead": [
            ("pytest", 600, f"{PYTEST} -v tests/test_gpu_multirank.py -k 'halo_ahead'"),
        ] + [
            (f"sim{P}_{pr}_ha{ha}", 200, bench(f"{'--problem poisson3d --grid 512 ' if pr == '3d' else ''}"
                                              f"--sim-world {P} --sim-rank {r} --steps 400 --warmup 40 --phases 10 "
                                              f"--set halo_ahead={ha}"))
            for P, r, pr in ((8, 3, "2d"), (4, 1, "2d"), (8, 3, "3d")) for ha in (1, 0)
        ],
        # does the pass leave room for RCCL's kernels?  (CU-masked compute queue: negative result,
        # profiles/r2_corun_probe.md)
        "corun2": [
            ("graph", 180, f"{PY} bench/corun_probe.py"),
            ("eager", 180, f"{PY} bench/corun_probe.py --graph 0"),
            ("generic", 180, f"{PY} bench/corun_probe.py --set carry=0"),
            ("m16", 180, f"{PY} bench/corun_probe.py --set comm_cus=16"),
        ],
        # line-carry geometry at a P = 8 rank's share (2046 interior lines of 16384^2)
        "carrysweep": [
            (f"b{b}_d{d}", 200, bench(f"--sim-world 8 --sim-rank 3 --steps 400 --warmup 40 --phases 0 --no-verify "
                                      f"--set carry_blocks_per_cu={b} --set carry_depth={d}"))
            for b in (2, 3, 4, 6, 8) for d in (2, 3)
        ] + [
            (f"full_b{b}", 200, bench(f"--steps 100 --warmup 10 --phases 0 --no-verify --set carry_blocks_per_cu={b}"))
            for b in (2, 4, 8)
        ],
        # the distributed path at headline sizes as P in-process ranks on one GPU
        "dia": [
            ("pytest", 600, f"{PY} -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py "
                            f"tests/test_gpu_multirank.py tests/test_gpu_fused_reduce.py -m gpu"),
            ("b_dia", 200, f"{PY} bench.py"),
            ("b_c4", 200, f"{PY} bench.py --set carry_dia=0"),
            ("b_dia2", 200, f"{PY} bench.py"),
            ("b_c4_2", 200, f"{PY} bench.py --set carry_dia=0"),
            ("b4096_dia", 200, f"{PY} bench.py --grid 4096 --steps 2000 --warmup 100"),
            ("b4096_c4", 200, f"{PY} bench.py --grid 4096 --steps 2000 --warmup 100 --set carry_dia=0"),
            ("sim8_dia", 200, f"{PY} bench.py --sim-world 8 --sim-rank 3 --steps 400 --warmup 40"),
            ("sim8_c4", 200, f"{PY} bench.py --sim-world 8 --sim-rank 3 --steps 400 --warmup 40 --set carry_dia=0"),
        ],
        # counters of the dia4 pass (VALU issue, wave cycles) and its HBM bytes, one group per run
        "diapmc": [
            ("valu", 120, prof("diapmc_valu", f"{PY} {ROOT}/bench.py --steps 8 --warmup 2 --phases 0 --no-verify",
                               "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU "
                               "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS")),
            ("bytes", 120, prof("diapmc_bytes", f"{PY} {ROOT}/bench.py --steps 8 --warmup 2 --phases 0 --no-verify",
                                "TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE")),
            ("trace", 200, prof("diatrace", f"{PY} {ROOT}/bench.py --steps 64 --warmup 8 --phases 0")),
        ],
        # 3-D Ap-recomputing plane carry (dia4, +-N rows through LDS): tests, kw sweep, store form, P = 8 share
        "ar3": [
            ("pytest", 600, f"{PY} -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py "
                            f"tests/test_gpu_multirank.py -m gpu -k 'ap_recompute or halo_ahead or carry'"),
            ("kw8", 200, bench("--problem poisson3d --grid 512")),
            ("kw4", 200, bench("--problem poisson3d --grid 512 --set carry3_kw=4")),
            ("kw16", 200, bench("--problem poisson3d --grid 512 --set carry3_kw=16")),
            ("store", 200, bench("--problem poisson3d --grid 512 --set ap_recompute=0")),
            ("kw8_b", 200, bench("--problem poisson3d --grid 512")),
            ("sim8", 200, bench("--problem poisson3d --grid 512 --sim-world 8 --sim-rank 3 --steps 400 --warmup 40")),
            ("sim8_store", 200, bench("--problem poisson3d --grid 512 --sim-world 8 --sim-rank 3 --steps 400 "
                                      "--warmup 40 --set ap_recompute=0")),
        ],
        "ar3pmc": [
            ("valu", 120, prof("ar3pmc_valu", f"{PY} {ROOT}/bench.py --problem poisson3d --grid 512 --steps 8 --warmup 2 "
                                              f"--phases 0 --no-verify",
                               "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU "
                               "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS")),
            ("bytes", 120, prof("ar3pmc_bytes", f"{PY} {ROOT}/bench.py --problem poisson3d --grid 512 --steps 8 "
                                                f"--warmup 2 --phases 0 --no-verify",
                                "TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE")),
            ("trace", 200, prof("ar3trace", f"{PY} {ROOT}/bench.py --problem poisson3d --grid 512 --steps 64 "
                                            f"--warmup 8 --phases 0")),
            ("sim8", 200, bench("--problem poisson3d --grid 512 --sim-world 8 --sim-rank 3 --steps 400 --warmup 40")),
            ("qd3", 200, bench("--problem poisson3d --grid 512 --set carry_depth=3")),
        ],
        # knobs of the dia4 line carry on the headline grid
        "diaknobs": [
            ("nt", 200, bench("--set carry_nt=1")),
            ("d2", 200, bench("--set carry_depth=2")),
            ("d4", 200, bench("--set carry_depth=4")),
            ("d5", 200, bench("--set carry_depth=5")),
            ("base", 200, bench()),
            ("nt3d", 200, bench("--problem poisson3d --grid 512 --set carry_nt=1")),
        ],
        # r4: variable-coefficient stencils on the line carry (SELL-64/diav)
        "vc": [
            ("pytest", 600, f"{PY} -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_varcoef.py"),
            ("b16384", 300, bench("--coef 1 --steps 100 --warmup 10 --phases 0")),
            ("b16384_generic", 300, bench("--coef 1 --steps 50 --warmup 5 --phases 0 --set carry_vc=0")),
            ("b4096", 300, bench("--coef 1 --grid 4096 --steps 1000 --warmup 100 --phases 0")),
        ],
        # r4: tile pacing mechanism (counter polls vs step flags, lag) at the scrambled config-5 P = 8 share
        "c5pace": [
            (f"{tag}", 400, bench(f"{C5SCR} --steps 6 --warmup 2 --phases 0 --no-verify " +
                                  " ".join(f"--set {kv}" for kv in sets)))
            for tag, sets in (("p2", ["tile_pace=2"]), ("p4", ["tile_pace=4"]), ("p3", ["tile_pace=3"]),
                              ("p4_s18_lag1", ["tile_pace=4", "tile_seg_log2=18", "tile_pace_lag=1"]),
                              ("p4_s18", ["tile_pace=4", "tile_seg_log2=18"]),
                              ("p2_again", ["tile_pace=2"]))
        ],
        # r4: can a copy-engine (hipMemcpyDeviceToDeviceNoCU) halo run beside the resident pass?
        "copyprobe": [
            ("p2d", 240, f"{PY} bench/corun_probe.py --reps 4 --kinds rccl,spin_thin --copy-kib 128 --copy-kib 2048"),
            ("p3d", 240, f"{PY} bench/corun_probe.py --reps 4 --problem poisson3d --grid 512 --kinds rccl "
                         f"--copy-kib 2048"),
        ],
        "rehearse": [
            ("r16384", 600, f"{PY} bench/rehearse_ranks.py --n 16384 --iters 20 --world 1 2 4 8 --phases 10"),
            ("r512", 600, f"{PY} bench/rehearse_ranks.py --problem poisson3d --n 512 --iters 20 --world 1 2 4 8 "
                          f"--phases 10"),
            ("rwide", 600, f"{PY} bench/rehearse_ranks.py --problem randspd --iters 20 --world 1 2 4 8 --phases 10"),
        ],
    }


def run(name: str, steps, dry: bool) -> int:
    os.makedirs(OUT, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp", HSA_ENABLE_IPC_MODE_LEGACY="0")
    for step, limit, cmd in steps:
        full = f"timeout -k 10 {limit} {cmd}"
        print(f"[gpu_run] {name}/{step}: {full}", flush=True)
        if dry:
            continue
        t0 = time.time()
        base = os.path.join(OUT, f"{name}_{step}")
        with open(base + ".out", "w") as fo, open(base + ".err", "w") as fe:
            proc = subprocess.Popen(shlex.split(full), cwd=ROOT, env=env, stdout=fo, stderr=fe)
            beat = time.time()
            while proc.poll() is None:  # heartbeat: a silent step must not look hung to the pool
                time.sleep(1.0)
                if time.time() - beat >= 60:
                    beat = time.time()
                    print(f"[gpu_run] {name}/{step}: running {beat - t0:.0f}s", flush=True)
            rc = proc.returncode
        print(f"[gpu_run] {name}/{step}: rc={rc} {time.time() - t0:.1f}s", flush=True)
        if rc != 0:
            with open(base + ".err") as fe:
                sys.stdout.write(fe.read()[-3000:])
            with open(base + ".out") as fo:
                sys.stdout.write(fo.read()[-3000:])
            return rc
        with open(base + ".out") as fo:
            tail = fo.read().strip().splitlines()[-3:]
        for line in tail:
            print("   " + line[:400])
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("recipe", nargs="*", help="recipe names (in order)")
    ap.add_argument("--grid", type=int, default=4096, help="grid edge for prof / pmc")
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    R = recipes(a)
    if a.list or not a.recipe:
        for k, steps in R.items():
            print(k + ": " + ", ".join(s for s, _, _ in steps))
        return 0
    for name in a.recipe:
        name, _, only = name.partition("/")  # "recipe/step" runs one step of a recipe
        if name not in R:
            print(f"unknown recipe {name!r}", file=sys.stderr)
            return 2
        steps = [s for s in R[name] if not only or s[0] == only]
        if not steps:
            print(f"unknown step {only!r} of {name!r}", file=sys.stderr)
            return 2
        rc = run(name, steps, a.dry_run)
        if rc != 0:
            return rc
    return 0


if __name__ == "__main__":
    sys.exit(main())
