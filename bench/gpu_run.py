#!/usr/bin/env python3
"""One recipe runner for every GPU-box command of this repo (the round-3 per-experiment shell
launchers bench/r3_*.sh are folded in here as recipes).  Run on the box:

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


def prof(tag: str, cmd: str, pmc: str = "", fmt: str = "csv") -> str:
    """rocprofv3 around `cmd` (the program itself right after --, never a wrapper); csv output for
    prof_summary.py / pmc_csv.py, fmt "" = the rocpd database (trace_summary.py)."""
    what = f"--pmc {pmc}" if pmc else "--kernel-trace --stats"
    of = f" --output-format {fmt}" if fmt else ""
    return f"{PROF} {what} -d {OUT}/{tag} -o run{of} -- {cmd}"


def recipes(a) -> dict:
    g = a.grid
    c5 = f"{C5SCR} --phases 0 --no-verify"
    dram = "TCC_EA0_RDREQ_DRAM_32B_sum TCC_EA0_WRREQ_WRITE_DRAM_32B_sum GRBM_GUI_ACTIVE"
    WAVES = ("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY "
             "SQ_WAIT_INST_ANY SQ_INSTS_LDS")
    S8 = "--sim-world 8 --sim-rank 3 --set halo_pull=1"

    def stats(tag, args):  # kernel trace + stats of one bench run, summarised to markdown
        return [(tag, 300, prof(tag, f"{PY} {ROOT}/bench.py --phases 0 {args}")),
                (tag + "_md", 60, f"{PY} bench/prof_summary.py --stats {OUT}/{tag} --title '{tag}: bench.py {args}'")]

    def counters(tag, kernel, args, pmc=dram):  # one counter pass (one group per rocprofv3 run)
        return [(tag, 300, prof(tag, f"{PY} {ROOT}/bench.py --phases 0 --no-verify {args}", pmc)),
                (tag + "_txt", 60, f"{PY} bench/pmc_csv.py {OUT}/{tag} {kernel}")]

    def sets(kvs):
        return " ".join(f"--set {kv}" for kv in kvs)

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
        "fix3d": [("pytest", 300, f"{PYTEST} -v tests/test_gpu_solver.py -k 'ap_recompute_3d'")],
        # the whole GPU suite without stopping at the first failure (every failure in one call)
        "suite": [("pytest_gpu", 1000, f"{PY} -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu")],
        "headline": [
            ("b16384", 200, bench("--phases 0")),
            ("b512", 200, bench("--problem poisson3d --grid 512 --phases 0")),
            ("b4096", 200, bench("--grid 4096 --steps 2000 --warmup 100 --phases 0")),
        ],
        # BASELINE.json configs on one GPU (config 5 at a P = 8 rank's share of the scrambled family)
        "configs": [
            ("c1_cpu_1024", 900, f"bin/mcg-cg --device cpu --problem poisson2d --n 1024 --fixed-iters 200 "
                                 f"--report json"),
            ("c2_4096", 200, bench("--grid 4096 --steps 2000 --warmup 100")),
            ("c3_16384", 200, bench()),
            ("c4_512", 200, bench("--problem poisson3d --grid 512")),
            ("c5_scrambled", 600, bench(f"{C5SCR} --steps 10 --warmup 3 --phases 5")),
        ],
        # every README row of the current tree on one box (r3_readme_table.sh)
        "variants": [
            (tag, 200, bench(args)) for tag, args in (
                ("p2d_default", ""), ("p2d_generic3", "--set dia_uniform=0"), ("p2d_two_term", "--set p3=0"),
                ("p2d_c8", "--set carry_dia=0"), ("p2d_store", "--set ap_recompute=0"),
                ("p2d_generic", "--set carry=0"), ("p2d_pipelined", "--recurrence 2 --steps 100 --warmup 10"),
                ("p2d_sell16", "--format sell16 --steps 100 --warmup 10"),
                ("p2d_csr_two", "--format csr --recurrence 0 --steps 60 --warmup 5"),
                ("p2d_csr_single", "--format csr --recurrence 1 --steps 60 --warmup 5"),
                ("p2d_force_comm", "--force-comm"),
                ("p2d_varcoef", "--coef 1"), ("p2d_varcoef_d16", "--coef 1 --set carry_vc=0 --steps 60 --warmup 5"),
                ("p3d_default", "--problem poisson3d --grid 512"),
                ("p3d_generic3", "--problem poisson3d --grid 512 --set dia_uniform=0"),
                ("p3d_two_term", "--problem poisson3d --grid 512 --set p3=0"),
                ("p3d_store", "--problem poisson3d --grid 512 --set ap_recompute=0"),
                ("p4096", "--grid 4096 --steps 2000 --warmup 100"))
        ],
        # rocprofv3 kernel stats of the default paths (r3_final_profiles.sh / r3_lean_profiles.sh)
        "stats": stats("stats_16384", "--steps 64 --warmup 8") + stats("stats_512", "--problem poisson3d --grid 512 "
                                                                       "--steps 64 --warmup 8")
                 + stats("stats_4096", "--grid 4096 --steps 640 --warmup 64")
                 + stats("stats_pipe_4096_p8", "--grid 4096 --recurrence 2 --sim-world 8 --sim-rank 3 --steps 256 "
                                               "--warmup 32"),
        # DRAM bytes per pass (one counter group per run)
        "dram": counters("dram_16384", "k_cg_carry_ar", "--steps 8 --warmup 2")
                + counters("dram_512", "k_cg_carry_ar3", "--problem poisson3d --grid 512 --steps 8 --warmup 2")
                + counters("dram_4096", "k_cg_carry_ar", "--grid 4096 --steps 64 --warmup 8"),
        # issue-side counters of one grid's pass (--grid)
        "waves": counters(f"waves_{g}", "k_cg_carry_ar", f"--grid {g} --steps 8 --warmup 2", WAVES),
        # kernel trace + per-iteration kernel count / gaps of one grid (--grid)
        "trace": [
            ("trace", 300, prof(f"prof{g}", f"{PY} {ROOT}/bench.py --grid {g} --steps 64 --warmup 8 --phases 0 "
                                            f"--force-comm", fmt="")),
            ("summary", 60, f"{PY} bench/trace_summary.py {OUT}/prof{g}/run_results.db --pass k_cg_carry_ar --iters 48"),
        ],
        # BASELINE config 5, scrambled (r3_pmc_tiles.sh / r3_gpu_round.sh): tiles vs CSR, DRAM + L2 counters
        "config5": [
            ("tiles", 400, bench(f"{C5SCR} --steps 10 --warmup 3")),
            ("csr", 600, bench(f"{c5} --steps 5 --warmup 2 --format csr --set tiles=0")),
        ] + counters("c5_dram", "k_tiles", f"{C5SCR} --steps 2 --warmup 1")
          + counters("c5_l2", "k_tiles", f"{C5SCR} --steps 2 --warmup 1", "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"),
        # tile segment size (r3_tiles_sweep.sh; the pacing variants were pruned in r5)
        "c5sweep": [
            (tag, 400, bench(f"{c5} --steps 6 --warmup 2 {sets(kv)}"))
            for tag, kv in (("s18", ["tile_seg_log2=18"]), ("s17", ["tile_seg_log2=17"]),
                            ("s19", ["tile_seg_log2=19"]), ("s18_again", ["tile_seg_log2=18"]))
        ],
        # r4: the pacing beside other kernels (fat = RCCL's register footprint) and the collision test
        "useraligned": [
            ("pytest", 600, f"{PYTEST} -v tests/test_gpu_user_matrix.py -k 'aligned'"),
        ],
        "pacecorun": [
            ("probe", 400, f"{PY} -u bench/pace_corun.py --set tile_seg_log2=18"),
            ("pytest", 300, f"{PYTEST} -v tests/test_gpu_irregular.py -k 'colliding or tiles'"),
        ],
        # r4: next-segment L2 prefetch during the pacing wait
        "c5ag": [
            ("ag_thin", 400, bench(f"{c5} --steps 6 --warmup 2 --delay-comm 10,2330")),
            ("noag_thin", 400, bench(f"{c5} --steps 6 --warmup 2 --delay-comm 10,2330 --set ag_overlap=0")),
            ("ag_fat", 400, bench(f"{c5} --steps 6 --warmup 2 --delay-comm 10,2330,fat")),
            ("ag_null", 400, bench(f"{c5} --steps 6 --warmup 2")),
            ("ag_thin_eager", 400, bench(f"{c5} --steps 6 --warmup 2 --delay-comm 10,2330 --no-graph")),
            ("noag_thin_eager", 400, bench(f"{c5} --steps 6 --warmup 2 --delay-comm 10,2330 --no-graph "
                                           f"--set ag_overlap=0")),
            ("ag_copy", 400, bench(f"{c5} --steps 6 --warmup 2 --delay-comm 10,0,copy")),
            ("noag_copy", 400, bench(f"{c5} --steps 6 --warmup 2 --delay-comm 10,0,copy --set ag_overlap=0")),
        ],
        "c5v32big": [
            ("share200", 900, bench(f"{C5SCR.replace('--band 410', '--band 820')} --steps 4 --warmup 1 --phases 2")),
        ],
        # config 5 at ~200 GB per GPU and with the all-gather priced (DelayComm)
        "c5big": [
            ("share200", 900, bench(f"{C5SCR.replace('--band 410', '--band 820')} --steps 4 --warmup 1 --phases 2")),
            ("share101_priced", 600, bench(f"{c5} --steps 6 --warmup 2 --delay-comm 10,2330")),
        ],
        # config 5's other family: the wide multi-diagonal random SPD (SELL-64/aligned, all-gather overlap)
        "config5_wide": [
            ("band820", 900, bench("--problem randspd --rows 12500000 --band 820 --density 1.0 --spread 12500000 "
                                   "--steps 6 --warmup 1 --phases 2")),
            ("sim8_ag", 900, bench("--problem randspd --rows 100000000 --band 820 --density 1.0 --spread 100000000 "
                                   "--sim-world 8 --sim-rank 3 --steps 6 --warmup 1 --phases 2")),
        ],
        # one rank's share of a P-rank run alone on this GPU (NullComm: collectives move nothing)
        "simrank": [
            (f"p{P}_r{r}", 200, bench(f"--sim-world {P} --sim-rank {r} --steps 400 --warmup 40 --phases 10"))
            for P, r in ((2, 0), (4, 1), (8, 0), (8, 3), (8, 7))
        ] + [("p8_r3_3d", 200, bench("--problem poisson3d --grid 512 --sim-world 8 --sim-rank 3 --steps 400 "
                                     "--warmup 40 --phases 10"))],
        # the same shares priced with collective latency (r3_priced_shares.sh, r3_overlap_ab.sh)
        "priced": [
            (f"{prob}_{w}", 200, f"{PY} bench/pipe_latency.py {args} --world {w} --rank {3 if w > 2 else 1} "
                                 f"--recurrences 1 --graphs 1 --overlaps 1,0 --delays 0,10,20 --halo-us 10 --iters 320")
            for prob, args in (("16384", "--grid 16384"), ("4096", "--grid 4096"),
                               ("512", "--problem poisson3d --grid 512"))
            for w in (2, 4, 8)
        ],
        # can a collective / copy run beside the resident pass? (r3_probe_corun.sh + the r4 copy engine)
        "corun": [
            ("p2d", 240, f"{PY} bench/corun_probe.py --reps 4 --kinds rccl,rccl_graph,spin_fat,spin_thin "
                         f"--copy-kib 128 --copy-kib 2048"),
            ("p3d", 240, f"{PY} bench/corun_probe.py --reps 4 --problem poisson3d --grid 512 --kinds rccl "
                         f"--copy-kib 2048"),
            ("trace", 300, prof("corun_trace", f"{PY} {ROOT}/bench/corun_probe.py --reps 2")),
        ],
        # CU-masked compute stream (r3_cumask.sh)
        "cumask": [
            ("probe", 300, f"{PY} -u bench/cumask_probe.py"),
        ] + [
            (f"full_rc{rc}", 300, bench(f"--steps 64 --warmup 8 --set reserve_cus={rc}")) for rc in (0, 32)
        ] + [
            (f"split_{gg}", 300, f"{PY} -u bench/pipe_latency.py --grid {gg} --world 8 --rank 3 --recurrences 1 "
                                 f"--graphs 1 --overlaps 1 --fat 1 --delays 10 --halo-us 30 --iters 640 "
                                 f"--reserve-cus 0,32 --halo-ahead 0,1") for gg in (16384, 4096)
        ],
        # r4: the 3-D plane carry's runs per job column (kern::carry3_runs) with CUs withheld, and a
        # non-power-of-two grid whose jobs do not fill the blocks
        "runs3": [
            (f"p{g}_rc{rc}", 300, bench(f"--problem poisson3d --grid {g} --steps 64 --warmup 8 --phases 0 "
                                        f"--set reserve_cus={rc}"))
            for g in (512, 384) for rc in (0, 32)
        ],
        # the distributed path at headline sizes as P in-process ranks on one GPU (r3_rehearse_lean.sh)
        "rehearse": [
            ("r16384", 600, f"{PY} bench/rehearse_ranks.py --n 16384 --iters 40 --world 1 2 4 8 --no-overlap"),
            ("r512", 600, f"{PY} bench/rehearse_ranks.py --problem poisson3d --n 512 --iters 40 --world 1 2 4 8 "
                          f"--no-overlap"),
            ("rwide", 600, f"{PY} bench/rehearse_ranks.py --problem randspd --iters 20 --world 1 2 4 8 --phases 10"),
        ],
        # box-to-box spread: repeated runs in one call (r3_repeat.sh)
        "repeat": [
            (f"{tag}_{rep}", 200, bench(args)) for rep in (1, 2, 3)
            for tag, args in (("g4096", "--grid 4096 --steps 2000 --warmup 100"),
                              ("sim8", "--sim-world 8 --sim-rank 3 --steps 400 --warmup 40"))
        ],
        # 3-D block height (r3_kw_ab.sh) and setup placement probe depth (r3_placement_tries.sh)
        "placement": [(f"t{t}_{rep}", 150, bench(f"--phases 0 --set placement_tries={t}"))
                      for rep in (1, 2) for t in (1, 3, 6)],
        # r4: 4096^2 (BASELINE config 2) lean-pass geometry: prefetch depth x blocks per CU
        "mix": [
            ("pytest", 300, f"{PYTEST} -v tests/test_gpu_solver.py -k 'lean_mix'"),
        ] + [
            (f"{tag}_{rep}", 200, bench(f"--grid 4096 --steps 2000 --warmup 100 --phases 0 {kv}"))
            for rep in (1, 2, 3) for tag, kv in (("mix", ""), ("r3", "--set lean_packed=0"))
        ] + [("g16384", 200, bench("--phases 0"))],
        # a P = 8 rank's share of 16384^2 (2048 lines, 8 blocks per CU: the driver's N = 8 scaling
        # point) and of 4096^2 (512 lines) with the packed-edge geometry
        "lsplit": [
            ("pytest", 300, f"{PYTEST} -v tests/test_gpu_user_matrix.py -k 'lean'"),
        ],
        "lsplit_ab": [
            ("pytest", 300, f"{PYTEST} -v tests/test_gpu_user_matrix.py -k 'lean'"),
            ("ab4096", 200, f"{PY} -u bench/lean_split_ab.py --n 4096 --steps 2000 --warmup 100"),
            ("ab8192", 300, f"{PY} -u bench/lean_split_ab.py --n 8192 --steps 800 --warmup 50"),
            ("ab16384", 900, f"{PY} -u bench/lean_split_ab.py --n 16384 --steps 300 --warmup 20 --reps 2"),
        ],
        # r6: split ranks on three p buffers -- the bitwise tests, then the A/B (side = three buffers, two = r5)
        "lsplit3": [
            ("pytest", 600, f"{PYTEST} -v tests/test_gpu_user_matrix.py -k 'lean_split'"),
            ("ab16384", 900, f"{PY} -u bench/lean_split_ab.py --n 16384 --steps 300 --warmup 20 --reps 3 "
                             "--arms uniform,side,two,sideplain"),
            ("ab4096", 300, f"{PY} -u bench/lean_split_ab.py --n 4096 --steps 2000 --warmup 100 --reps 2 "
                            "--arms uniform,generic,side,two"),
        ],
        # ... a P = 8 rank's share (rank 5 holds two of the three changed rows), NullComm, in-kernel halo
        "lsplit3s8": [
            ("pytest", 600, f"{PYTEST} -v tests/test_gpu_user_matrix.py -k 'lean_split'"),
            ("s8", 900, f"{PY} -u bench/lean_split_ab.py --n 16384 --steps 2000 --warmup 200 --reps 2 "
                        "--arms uniform,side,serial,stream,two --sim-world 8 --sim-rank 5"),
            ("ab16384", 900, f"{PY} -u bench/lean_split_ab.py --n 16384 --steps 300 --warmup 20 --reps 2 "
                             "--arms uniform,side,stream,two"),
            ("b16384", 200, bench("--phases 0")),
            ("b4096", 200, bench("--grid 4096 --steps 2000 --warmup 200 --phases 0")),
        ],
        "lsplit3b": [
            ("ab16384", 900, f"{PY} -u bench/lean_split_ab.py --n 16384 --steps 300 --warmup 20 --reps 3 --arms side,two"),
            ("t3", 600, prof("lsplit_t3", f"{PY} {ROOT}/bench/lean_split_ab.py --n 16384 --steps 100 --warmup 10 "
                                          "--arms side")),
            ("t3_md", 60, f"{PY} bench/prof_summary.py --stats {OUT}/lsplit_t3 --title 'lean_split, three p buffers, 16384^2'"),
            ("two", 600, prof("lsplit_two", f"{PY} {ROOT}/bench/lean_split_ab.py --n 16384 --steps 100 --warmup 10 "
                                            "--arms two")),
            ("two_md", 60, f"{PY} bench/prof_summary.py --stats {OUT}/lsplit_two --title 'lean_split, two p buffers, 16384^2'"),
        ],
        # r6: config-5 tiles in two 8-wave workgroups per CU (tile_waves 8) against four 4-wave ones, interleaved
        "c5w8": [("pytest", 300, f"{PYTEST} -v tests/test_gpu_irregular.py -k wide_workgroups")] + [
            (f"w{ww}_{rep}", 400, bench(f"{C5SCR} --phases 0 --steps 10 --warmup 3 --set tile_waves={ww}"))
            for rep in ("a", "b") for ww in (4, 8)
        ],
        # r6: plain (MALL-allocating) stores for the vectors a pass writes, against non-temporal ones, by size
        # (var/tstore: -DMCG_NT_STORES=0, built like var/colx)
        "tstore": [
            (f"{tag}_{g}_{rep}", 200, f"{PY} {script} --grid {g} --phases 0 "
                                      + ("--steps 2000 --warmup 200" if g <= 4096 else "--steps 300 --warmup 30"))
            for rep in ("a", "b") for g in (4096, 8192, 16384)
            for tag, script in (("nt", "bench.py"), ("plain", "var/tstore/run_bench.py"))
        ],
        # r6: the reduction's CgState snapshot loaded in the group winners (f1_common.hpp book_snap) against
        # the tree before it (var/old: the previous commit's package and extension, built like var/colx)
        "bsnap": [("pytest", 600, f"{PYTEST} tests/test_gpu_fused_reduce.py tests/test_gpu_solver.py")] + [
            (f"{tag}_{g}_{rep}", 200, f"{PY} {script} --grid {g} --phases 0 "
                                      + ("--steps 2000 --warmup 200" if g <= 4096 else "--steps 300 --warmup 30"))
            for rep in ("a", "b", "c") for g in (4096, 8192, 16384)
            for tag, script in (("snap", "bench.py"), ("old", "var/old/run_bench.py"))
        ] + [(f"{tag}_512_{rep}", 200, f"{PY} {script} --problem poisson3d --grid 512 --phases 0")
             for rep in ("a", "b") for tag, script in (("snap", "bench.py"), ("old", "var/old/run_bench.py"))],
        # r6: the combined split on short runs (4096^2 / 8192^2: 64-line runs, where the auto rule kept the
        # generic kernels), forced against the generic fallback and the uniform matrix
        "lsplit3short": [("pytest", 600, f"{PYTEST} -v tests/test_gpu_user_matrix.py -k 'lean_split'")] + [
            (f"ab{n}", 600, f"{PY} -u bench/lean_split_ab.py --n {n} --steps {st} --warmup {st // 10} --reps 2 "
                            "--arms uniform,generic,side")
            for n, st in ((4096, 2000), (8192, 800))
        ],
        # kernel trace of the split share with the generic launch ahead on one stream (per-call durations)
        "lsplit3tr": [
            ("tr", 600, prof("lsplit_ser", f"{PY} {ROOT}/bench/lean_split_ab.py --n 16384 --steps 300 --warmup 20 "
                                          "--arms serial --sim-world 8 --sim-rank 5")),
        ],
        # kernel trace of the split pass at 16384^2 (lean + generic launches per pass) and of the generic one
        "lsplit_prof": [
            ("side", 600, prof("lsplit_side", f"{PY} {ROOT}/bench/lean_split_ab.py --n 16384 --steps 100 --warmup 10 "
                                              "--arms side")),
            ("side_md", 60, f"{PY} bench/prof_summary.py --stats {OUT}/lsplit_side --title 'lean_split side, 16384^2'"),
            ("generic", 600, prof("lsplit_gen", f"{PY} {ROOT}/bench/lean_split_ab.py --n 16384 --steps 100 --warmup 10 "
                                                "--arms generic")),
            ("generic_md", 60, f"{PY} bench/prof_summary.py --stats {OUT}/lsplit_gen --title 'lean_split=0, 16384^2'"),
        ],
        "streamop": [
            ("probe", 240, f"{PY} -c 'import torch, json, cuda_mpi_parallel_amd as m; torch.cuda.init(); "
                          f"print(json.dumps(dict(m.native().kernels.streamop_probe())))'"),
        ],
        # r4: the copy-engine halo across processes (PeerHaloComm, IPC-mapped buffers), P ranks on one GPU
        "peer": [
            ("check2", 180, f"{PY} -u bench/peer_halo_check.py --world 2"),
            ("check4", 180, f"{PY} -u bench/peer_halo_check.py --world 4 --n 512 --rounds 6"),
            ("check4_ag", 180, f"{PY} -u bench/peer_halo_check.py --world 4 --problem scrambled --rounds 4"),
        ] + [
            (f"bench{w}_{t}", 300, f"{PY} -m torch.distributed.run --nnodes=1 --nproc-per-node {w} "
                                   f"--master-addr 127.0.0.1 --master-port {29600 + w} bench.py --gpus {w} "
                                   f"--rehearse-ranks --steps 200 --warmup 20 --phases 0 --halo-transport {t}")
            for w in (2, 4) for t in ("rccl", "sdma")
        ],
        # r5: a P = 8 rank's share of 16384^2 and 512^3 (the in-kernel halo's pass, NullComm):
        # kernel trace, DRAM bytes and issue counters of the pass
        "share8": stats("share8_2d", f"{S8} --steps 256 --warmup 32")
                  + stats("share8_3d", f"--problem poisson3d --grid 512 {S8} --steps 256 --warmup 32")
                  + counters("share8_2d_dram", "k_cg_carry_ar", f"{S8} --steps 32 --warmup 4")
                  + counters("share8_3d_dram", "k_cg_carry_ar3", f"--problem poisson3d --grid 512 {S8} --steps 32 --warmup 4")
                  + counters("share8_2d_waves", "k_cg_carry_ar", f"{S8} --steps 32 --warmup 4", WAVES)
                  + counters("p1_2d_waves", "k_cg_carry_ar", "--steps 8 --warmup 2", WAVES)
                  + counters("p1_2d_dram", "k_cg_carry_ar", "--steps 8 --warmup 2"),
        # r5: three p buffers (the lean 2-D carry without compact edge arrays) against two, kernel stats + DRAM
        "p3buf": stats("p3_16384", "--steps 64 --warmup 8") + stats("p2_16384", "--steps 64 --warmup 8 --set p3buf=0")
                 + stats("p3_4096", "--grid 4096 --steps 640 --warmup 64")
                 + stats("p2_4096", "--grid 4096 --steps 640 --warmup 64 --set p3buf=0")
                 + counters("p3_16384_dram", "k_cg_carry_ar", "--steps 8 --warmup 2")
                 + counters("p3_4096_dram", "k_cg_carry_ar", "--grid 4096 --steps 64 --warmup 8")
                 + counters("p2_4096_dram", "k_cg_carry_ar", "--grid 4096 --steps 64 --warmup 8 --set p3buf=0"),
        # r5: the 3-D lean plane carry on three p buffers against two: A/B, kernel stats, DRAM, priced shares
        "p3buf3d": [(f"{t}{i}", 300, bench(f"--problem poisson3d --grid 512 --phases 0{a}"))
                    for i in (1, 2) for t, a in (("ab3", ""), ("ab2", " --set p3buf=0"))]
                   + stats("p3_512", "--problem poisson3d --grid 512 --steps 64 --warmup 8")
                   + counters("p3_512_dram", "k_cg_carry_ar3", "--problem poisson3d --grid 512 --steps 8 --warmup 2")
                   + counters("p2_512_dram", "k_cg_carry_ar3", "--problem poisson3d --grid 512 --steps 8 --warmup 2 --set p3buf=0")
                   + [(f"priced512_{w}", 200, f"{PY} bench/pipe_latency.py --problem poisson3d --grid 512 --world {w} "
                                              f"--rank {3 if w > 2 else 1} --recurrences 1 --graphs 1 --overlaps 1,0 "
                                              f"--delays 0,10,20 --halo-us 10 --iters 320") for w in (2, 4, 8)],
        # the 3-D P = 8 share on three p buffers: kernel stats and DRAM counters
        "share3d": stats("s3d", f"--problem poisson3d --grid 512 {S8} --steps 256 --warmup 32")
                   + counters("s3d_dram", "k_cg_carry_ar3", f"--problem poisson3d --grid 512 {S8} --steps 32 --warmup 4")
                   + counters("s3d_waves", "k_cg_carry_ar3", f"--problem poisson3d --grid 512 {S8} --steps 32 --warmup 4", WAVES)
                   + counters("p1_3d_waves", "k_cg_carry_ar3", "--problem poisson3d --grid 512 --steps 8 --warmup 2", WAVES),
        # the headline's priced P-rank shares on the final r5 tree
        "priced16k": [(f"p16k_{w}", 200, f"{PY} bench/pipe_latency.py --grid 16384 --world {w} --rank {3 if w > 2 else 1} "
                                         f"--recurrences 1 --graphs 1 --overlaps 1,0 --delays 0,10,20 --halo-us 10 --iters 320")
                      for w in (2, 4, 8)] + [("p16k_1", 200, bench("--phases 0"))],
        # variable coefficients on three p buffers: DRAM counters (2-D and 3-D diav lean carries)
        "vcp3": counters("vc2_dram", "k_cg_carry_ar", "--coef 1 --steps 8 --warmup 2")
                + counters("vc3_dram", "k_cg_carry_ar3", "--problem poisson3d --grid 512 --coef 1 --steps 8 --warmup 2"),
        # config 5 tiles on the final r5 tree (straggler priority, 10 per lane): L2 and DRAM counters
        "c5final": counters("c5f_l2", "k_tiles", f"{C5SCR} --steps 2 --warmup 1", "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE")
                   + counters("c5f_dram", "k_tiles", f"{C5SCR} --steps 2 --warmup 1")
                   + counters("c5f_req", "k_tiles", f"{C5SCR} --steps 2 --warmup 1", "TCC_REQ_sum TCC_READ_sum GRBM_GUI_ACTIVE"),
        # the final r5 tree: kernel stats and DRAM counters of the headline, 4096^2 and 512^3 passes
        "final": stats("f_16384", "--steps 64 --warmup 8") + stats("f_4096", "--grid 4096 --steps 640 --warmup 64")
                 + stats("f_512c", "--problem poisson3d --grid 512 --steps 64 --warmup 8")
                 + counters("f_16384_dram", "k_cg_carry_ar", "--steps 8 --warmup 2")
                 + counters("f_4096_dram", "k_cg_carry_ar", "--grid 4096 --steps 64 --warmup 8")
                 + counters("f_512c_dram", "k_cg_carry_ar3", "--problem poisson3d --grid 512 --steps 8 --warmup 2"),
        # r6: the 2-D carries read one 128-B line per slice and pass above the byte model -- the slice-edge
        # rows of neighbouring columns held by other workgroups?  A/B against the diagnostic build whose
        # workgroups' waves take columns SS / 4 apart (every edge between workgroups): var/colx, built with
        # cp -r cuda_mpi_parallel_amd var/colx/ (minus _C*.so); make BUILD=var/colx/build
        # EXTRA_HIPFLAGS=-DMCG_COLMAP_SPREAD PYMOD=var/colx/cuda_mpi_parallel_amd/_C<ext> <that PYMOD>, and a
        # var/colx/run_bench.py that puts var/colx first on sys.path and runs bench.py (profiles/r6/colmap)
        "colmap": [
            ("base", 300, bench("--phases 0 --steps 200 --warmup 20")),
            ("spread", 300, f"{PY} var/colx/run_bench.py --phases 0 --steps 200 --warmup 20"),
        ] + counters("base_dram", "k_cg_carry_ar", "--steps 8 --warmup 2") + [
            ("spread_dram", 300, prof("spread_dram", f"{PY} {ROOT}/var/colx/run_bench.py --phases 0 --no-verify --steps 8 "
                                                     f"--warmup 2", dram)),
            ("spread_dram_txt", 60, f"{PY} bench/pmc_csv.py {OUT}/spread_dram k_cg_carry_ar"),
        ] + counters("base4k_dram", "k_cg_carry_ar", "--grid 4096 --steps 64 --warmup 8"),
        # r6: wider workgroups for the packed-edge three-buffer kernels (PassForm::lean_waves), bitwise test
        # then interleaved A/B at 16384^2 / 8192^2 / 4096^2 and the DRAM counters of the widest
        "leanww": [
            ("pytest", 600, f"{PYTEST} -v tests/test_gpu_solver.py -k 'lean_waves or p3buf_bitwise'"),
        ] + [
            (f"w{ww}_{g}_{rep}", 200, bench(f"--grid {g} --phases 0 --set lean_waves={ww} "
                                            + ("--steps 2000 --warmup 200" if g == 4096 else "--steps 300 --warmup 30")))
            for rep in ("a", "b") for g in (16384, 8192, 4096) for ww in (4, 8, 16)
        ] + counters("w16_dram", "k_cg_carry_ar", "--steps 8 --warmup 2 --set lean_waves=16")
          + counters("w8_dram", "k_cg_carry_ar", "--steps 8 --warmup 2 --set lean_waves=8"),
        # r6: per-wave timing of one even and one odd 2-D pass (var/diag: the build with -DMCG_CARRY_DIAG,
        # made like var/colx above), eager; bench/wave_spread.py summarises
        "wavediag": [
            (f"d{g}", 300, f"env MCG_CARRY_DIAG_FILE={OUT}/diag{g} MCG_CARRY_DIAG_AT={at} {PY} var/diag/run_bench.py "
                           f"--grid {g} --no-graph --phases 0 --steps {st} --warmup 20")
            for g, at, st in ((4096, 1500, 2000), (16384, 300, 400))
        ],
        # r6: issue priority by a workgroup's arrival rank on its CU (var/ageprio: -DMCG_CARRY_AGEPRIO from
        # profiles/r6/waves/ageprio_and_diag.patch, reverted), A/B interleaved, and the per-wave timings with
        # it (var/agediag) next to the default's (var/diag: -DMCG_CARRY_DIAG, in the tree)
        "ageprio": [
            (f"{tag}_{g}_{rep}", 200, f"{PY} {script} --grid {g} --phases 0 "
                                      + ("--steps 2000 --warmup 200" if g == 4096 else "--steps 300 --warmup 30"))
            for rep in ("a", "b") for g in (16384, 8192, 4096)
            for tag, script in (("base", "bench.py"), ("prio", "var/ageprio/run_bench.py"))
        ] + [
            (f"{tag}{g}", 300, f"env MCG_CARRY_DIAG_FILE={OUT}/{tag}{g} MCG_CARRY_DIAG_AT={at} {PY} var/{tag}/run_bench.py "
                               f"--grid {g} --no-graph --phases 0 --steps {st} --warmup 20")
            for tag in ("diag", "agediag") for g, at, st in ((4096, 1500, 2000), (16384, 300, 400))
        ],
        # r4: variable-coefficient stencils on the line carry (SELL-64/diav)
        "vc": [
            ("pytest", 600, f"{PY} -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_varcoef.py"),
        ],
        # how far rounding alone moves CG residual histories apart (CPU oracle, GPU two-reduction CSR,
        # generic single-reduction d16, diav carry), constant vs variable coefficients
        "vcdiv": [
            ("coef1", 300, f"{PY} -u bench/vc_divergence.py --coef 1"),
            ("coef0", 300, f"{PY} -u bench/vc_divergence.py --coef 0"),
        ],
        "vcb": [
            ("b16384", 300, bench("--coef 1 --steps 100 --warmup 10 --phases 0")),
            ("b16384_generic", 300, bench("--coef 1 --steps 50 --warmup 5 --phases 0 --set carry_vc=0")),
            ("b4096", 300, bench("--coef 1 --grid 4096 --steps 1000 --warmup 100 --phases 0")),
            ("b512", 300, bench("--coef 1 --problem poisson3d --grid 512 --steps 60 --warmup 6 --phases 0")),
            ("b512_generic", 300, bench("--coef 1 --problem poisson3d --grid 512 --steps 30 --warmup 3 --phases 0 "
                                        "--set carry_vc=0")),
        ] + counters("vc_dram", "k_cg_carry_ar", "--coef 1 --steps 8 --warmup 2")
          + counters("vc3_dram", "k_cg_carry_ar3", "--coef 1 --problem poisson3d --grid 512 --steps 8 --warmup 2"),
        # r4: 3-D lean plane carry across sizes: below / past 2^29 rows (BIG: bases moved along the run)
        "sizes3": [
            (f"n{n}", 400, bench(f"--problem poisson3d --grid {n} --steps {st} --warmup 4 --phases 0 --no-verify"))
            for n, st in ((512, 60), (640, 40), (768, 30), (800, 30), (832, 20), (1024, 12))
        ],
        # r4: ranks past 2^29 rows on the lean carries (BIG kernels)
        "large": [
            ("pytest", 900, f"{PY} -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_large.py"),
            ("b32768", 600, bench("--grid 32768 --steps 40 --warmup 4 --phases 0")),
            ("b1024", 600, bench("--problem poisson3d --grid 1024 --steps 40 --warmup 4 --phases 0")),
        ],
        # the round-end set the driver runs (r5's tools/steps/r5final.txt): smoke, the three stencil
        # headlines, config 5's share, the whole GPU suite
        "roundend": [
            ("smoke", 300, f"{PY} -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"),
            ("bench", 300, bench()),
            ("bench3", 300, bench("--problem poisson3d --grid 512")),
            ("bench4k", 300, bench("--grid 4096 --steps 2000 --warmup 200")),
            ("c5", 400, bench(f"{C5SCR} --phases 0 --steps 10 --warmup 3")),
            ("suite", 1100, f"{PY} -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread"),
        ],
        # r6: the transport probe and both CLIs' P > 1 path, rehearsed on one GPU
        "transport": [
            ("pytest", 900, f"{PYTEST} -v tests/test_gpu_transport.py tests/test_gpu_peer.py"),
            ("multirank", 900, f"{PYTEST} tests/test_gpu_multirank.py tests/test_gpu_user_matrix.py "
                               f"-k 'in_kernel_halo or p3buf or lean_split'"),
        ],
        # r6: the system-scope release after a wave publishes a rank-end line, A/B on the P = 8 shares
        # (the variant without it: make BUILD=exp_x/nofence/build EXTRA_HIPFLAGS=-DMCG_PULL_FENCE=0
        # PYMOD=exp_x/nofence/cuda_mpi_parallel_amd/_C<ext> next to a copy of the package, run through
        # exp_x/nofence/run_bench.py)
        "fence_ab": [
            (f"{tag}{pr}_{rep}", 200, f"{PY} -u {script} {args} {S8} --steps 2000 --warmup 200 --phases 0")
            for rep in ("a", "b") for pr, args in (("2d", ""), ("3d", "--problem poisson3d --grid 512"))
            for tag, script in (("fence", "bench.py"), ("nofence", "exp_x/nofence/run_bench.py"))
        ],
        # r6: the pulled ghost lines served from pinned host memory (PCIe, a slow
        # remote) on the P = 8 shares, next to the local stand-in; NullComm and a 10 us all-reduce
        "pull_proxy": [
            (f"{src}{pr}{tag}", 200, bench(f"{args} {S8} --set pull_proxy={px} {dc} --steps 2000 --warmup 200 "
                                           f"--phases 0"))
            for pr, args in (("2d", ""), ("3d", "--problem poisson3d --grid 512"))
            for src, px in (("host", 1), ("local", 0)) for tag, dc in (("", ""), ("_d10", "--delay-comm 10,0"))
        ],
        # r6: a grid barrier between resident passes against the kernel boundary
        "persist": [("probe", 240, "build/persist_probe")],  # (make builds it)
        # r6: the priced shares with the in-kernel halo forced on, and the kernel trace
        # of the DelayComm overlap=1 anomaly (D = 10 us slower than 20 us)
        "priced_pull": [(f"p16k_{w}", 300, f"{PY} bench/pipe_latency.py --grid 16384 --world {w} --rank {3 if w > 2 else 1} "
                                           f"--recurrences 1 --graphs 1 --overlaps 0 --delays 0,10,20 --halo-pull 1 "
                                           f"--iters 320") for w in (2, 4, 8)],
        "anomaly": [("trace", 400, prof("anom", f"{PY} {ROOT}/bench/pipe_latency.py --grid 16384 --world 8 --rank 3 "
                                                f"--delays 10,20 --recurrences 1 --graphs 1 --overlaps 1 --halo-us 10 "
                                                f"--iters 320", fmt=""))],
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
