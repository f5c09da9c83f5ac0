// Solver options / results shared by the CPU reference path and the GPU solver,
// plus the CPU reference path itself.
//
// Defaults reproduce the reference exactly: maxit = 2000, tol = 1e-7 on the
// ABSOLUTE residual norm ||r||_2 (CUDACG.cu:244-245,333 — the "relative
// residual" comment at :238 is not what the code does), x0 = 0, r0 = p0 = b,
// and no abort on non-positive curvature (the demo matrix is indefinite).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "mcg/partition.hpp"
#include "mcg/problem.hpp"

namespace mcg {

// Pass-form overrides.  Every field's default is the dispatcher's automatic choice (the measured
// fastest form for the matrix, rank layout and recurrence); setting one forces a form on or off for
// tests, sweeps and A/B measurements.  None changes the arithmetic of CG, only how a pass is built.
struct PassForm {
  int interleave = -1;       // single-reduction + SELL: {r, Ap} stored as 16-B pairs (one gather load); -1 = auto
  int pipeline = -1;         // single-reduction SELL d16/c8 + interleave, rows <= 8 nonzeros: software-pipelined
                             // pass (next slice's codes + own-row operands issued ahead); -1 = when applicable.
                             // With the XCD-aware 3-D sweep it is the faster pass (419 vs 383 it/s at 512^3,
                             // profiles/sweep_xcd_3d.log; in natural order it was slower, sweep_pipeline.log)
  int carry = -1;            // single-reduction SELL d16/c8 + interleave on a structured grid (whole 64-row slices
                             // per grid line / plane): line-carry pass — a wave walks down a column of slices and
                             // keeps the +-one-line and +-1 neighbours' p_k in registers.  -1 = auto: when every
                             // stored offset is carried (2-D stencils, c8); 1 = on (also with the slow path); 0 = off
  int window = -1;           // single-reduction + SELL: p_k staged once per 1024-row chunk in an LDS window
                             // (long banded rows); -1 = auto (windows fit and mean row length >= 32)
  int pmat = -1;             // single-reduction form: materialized-p split pass (update kernel + SpMV gathering the
                             // stored p only; cg_split.hip) — the irregular-sparsity path; -1 = auto (long rows
                             // without an LDS window, or the all-gather layout), 0 = off, 1 = on
  int sell_sigma = -1;       // SELL-C-sigma for user matrices: rows sorted by length inside windows of this many
                             // rows (multiple of 64) so slices pad less; -1 = auto (4096-row windows when that cuts
                             // the padded SELL slots by >= 10 %), 0 = off
  int sell_aligned = -1;     // wide random SPD: SELL-64/aligned (one column offset per slot shared by the slice's
                             // rows, values only; contiguous gathers); -1 = auto (expected fill <= 1.6), 0 = off
  int ag_overlap = -1;       // SELL-64/aligned or tiles on an all-gather ghost layout: sum the own-block column slots
                             // (tiles: the column segments inside the own block) while the
                             // all-gather of p is in flight, the rest after it (two SpMV halves); -1 = auto (on
                             // when the halo overlap is on), 0 = off
  int tiles = -1;            // irregular sparsity: the split pass's SpMV on L2-segment COO tiles (cg_tiles.hip: rows
                             // in blocks of 1024 owned by one wave, columns in segments of 2^tile_seg_log2, every
                             // wave sweeping the segments together so the gathers of p hit the L2); -1 = auto (the
                             // scrambled random SPD, or a non-stencil user matrix on the all-gather layout), 0 = off
  int tile_seg_log2 = 18;    // tiles: column segment = 2^k doubles (18: 2 MiB of p, half an XCD's L2; at a P = 8
                             // rank's share of the scrambled config 5 with step-flag pacing: 17 / 18 / 19 -> 18.5 /
                             // 19.3-19.5 / 17.5 it/s, profiles/r4/c5; r3's counter pacing peaked at 19: 14.0)
                             // (r5 pruned the tile variants that measured slower: 960-row blocks, 12 entries per
                             // lane, fp32 values, prefetch, the other pacing modes -- cg_tiles.hip header)
  int tile_waves = -1;       // tiles: waves per workgroup, 4 (four workgroups per CU) or 16 (one per CU, so the
                             // pacing barrier holds waves of one age); -1 = auto (4)
  int fused_reduce = -1;     // single-reduction form: sum the pass's block partials inside the pass (last-arriver
                             // fan-in, kernels.hpp RedCtl) instead of a separate single-block reduce launch, so an
                             // iteration is one kernel (+ the all-reduce); -1 = auto (on), 0 = off
  int ap_recompute = -1;     // 2-D line-carry pass: recompute Ap_{k-1} = A p_{k-1} from the p it reads instead of
                             // storing {r, Ap} pairs (r and p read once, written once: ~16 B/row less;
                             // cg_carry_ar.hip); -1 = auto (when the specialised 2-D carry covers every row
                             // in one launch), 0 = off, 1 = required
  int carry_dia = -1;        // Ap-recomputing 2-D carry: SELL-64/dia4 storage (slot u = the u-th canonical offset
                             // -line, -1, 0, +1, +line; 4-bit value indices), so the pass neither decodes offsets
                             // nor selects operands per entry; -1 = auto (when every entry's offset is canonical
                             // and in ascending order, <= 16 distinct values), 0 = off (c4 codes), 1 = required
  int p3 = -1;               // Ap-recomputing 2-D dia4 carry, three-term form: r_{k-1} = p_{k-1} - beta_{k-2} p_{k-2}
                             // recovered from the two p buffers the pass reads anyway, so r is stored only at the
                             // slices' edge rows and the runs' outer lines (24 instead of 32 B/row for r and p,
                             // and the paired x update needs no extra p read); rounding differs from the
                             // two-term form (not bitwise); -1 = auto (on with dia4), 0 = off, 1 = required
  int carry_vc = -1;         // variable-coefficient 2-D 5-point stencils (no c8 dictionary): the Ap-recomputing line
                             // carry on SELL-64/diav, streaming each row's d, e, s (a symmetric matrix's west / north
                             // values are its partners' east / south); -1 = auto, 0 = off (generic d16 pass), 1 = required
  int dia_uniform = -1;      // dia4 carry: slices whose 64 rows share one value-index pattern take a lean loop with the
                             // values in scalar registers and no codes streamed (the 2-D three-term pass over runs
                             // of such lines; bitwise the same sums); -1 = auto (on), 0 = off
  int lean_split = -1;       // 2-D three-term dia4 carry when some runs' slice patterns are not uniform (a user matrix
                             // with a few odd rows): the lean kernels over the runs that qualify, the generic ones
                             // over the rest, in two launches; -1 = auto (when most runs qualify), 0 = off (every run
                             // on the generic kernels), 1 = on; the generic launch runs on a side stream, concurrent with
                             // the lean one (r4: 548-557 vs 523-525 it/s after it, profiles/r4/lsplit)
  int halo_pull = -1;        // multi-rank lean carries (2-D line, 3-D plane): the in-kernel halo -- the waves that
                             // read a ghost line load it straight from the neighbour's rows (peer-mapped: IPC or
                             // another thread's pointers) and every pass stores its first / last line write-through,
                             // so an iteration is the pass + the all-reduce, with no halo step (from iteration 2 on;
                             // the first two exchange as before).  -1 = auto (when the communicator maps its peers:
                             // Communicator::maps_peers), 0 = off, 1 = on (with a rehearsal communicator that moves no
                             // data, the rank's own first / last line stands in for the neighbours': timing only)
  int p3buf = -1;            // 2-D lean three-term dia4 carry (every run lean, every line's slices one value
                             // pattern): three p buffers -- p_k written to one this pass does not read, so r is
                             // recovered from p_{k-1} / p_{k-2} everywhere and the neighbouring slices' edge rows
                             // recomputed: no compact edge arrays, no stored r (bitwise the same sums); -1 = auto, 0 = off
  int halo_ahead = -1;       // multi-rank stencils, single-reduction pass: exchange the halo iteration k+1 reads
                             // right after pass k wrote it (side stream, next to the all-reduce) and run one
                             // full pass per iteration instead of interior || halo then boundary.  RCCL's
                             // kernels cannot start next to a resident pass (profiles/r2_corun_probe.md), so
                             // the split never overlapped; -1 = auto (on when the halo overlap is on), 0 = off
};

// Test and fault-injection hooks (never set in production runs).
struct TestHooks {
  int fail_graph_launch_at = -1;  // test hook: report the graph launch at this iteration as failed (nothing enqueued)
  int force_idx64 = 0;       // test hook: int64 row pointers even when int32 would do
  int inject_nan_at = -1;    // fault-injection hook: poison r at this iteration (breakdown detection test)
  int pull_proxy = 0;        // rehearsal (a communicator that moves no data) with halo_pull 1: the pulled ghost lines
                             // read 0 = this rank's own first / last line (local HBM), 1 = pinned host memory over
                             // PCIe (a slow remote: an upper bound on what the pull costs over the fabric)
  int probe_pick_halo = -1;  // test hook: the transport probe runs every arm but keeps the pulled (1) / exchanged (0)
                             // halo whatever the times (a pulled run that did not match the exchanged one still loses)
  int probe_pick_ar = -1;    // test hook: ... keeps the alternative (1) / the first (0) all-reduce (a failed one loses)
  int lean_packed = -1;      // test hook: 0 = the packed-edge geometry (solver_setup.cpp auto_mix_: even passes on 5,
                             // odd ones on 4 blocks per CU) with the default lean kernels instead of the packed-edge
                             // ones -- the bit-for-bit reference of those kernels
  int split_serial = -1;     // a split rank on three p buffers: -1 = one combined launch (generic ranges' workgroups
                             // first), 0 = the generic launch beside the lean one on the side stream, 1 = ahead of
                             // it on one stream
  int gen_piece_lines = -1;  // test hook: a split rank's generic ranges on three p buffers cut into pieces of at
                             // most this many lines (TileRanges::gen_list; -1 = 32)
};

// Pass forms pruned in r5 (measured slower and kept opt-in until then): lean_depth 4 / 6 (fewer waves
// per SIMD, deeper prefetch), lean_bpc / lean_bpc_odd / lean_depth_odd (now only the setup's rules:
// the 4096^2-class grids still take the packed-edge kernels, solver_setup.cpp auto_mix_), lean_split_side
// 0, carry3_kw 4 / 8 on dia4 and 4 on diav (16 / 8 kept), carry3_runs (auto only) and halo_hide (the
// copy-engine halo split around the pass; superseded by halo_pull).  Their measurements stay in profiles/.

struct CgOptions {
  int maxit = 2000;          // CUDACG.cu:244
  double tol = 1e-7;         // CUDACG.cu:245 (absolute ||r||_2)
  double rtol = 0.0;         // > 0: stop on ||r||_2 < rtol * ||b||_2 instead (the "relative" of the comment at :238)
  int check_every = 32;      // host polls the device convergence latch every k iterations
  bool overlap = true;       // halo on a side stream, overlapped with the interior SpMV
  bool use_graph = true;     // capture iteration pairs into a hipGraph
  bool force_comm = false;   // run RCCL collectives even with one rank
  int format = 0;            // 0 = CSR, 1 = SELL-64
  int blocks_per_cu = 0;     // SpMV grid (blocks per CU); 0 = auto (SELL 48, CSR 8: measured sweeps; the line
                             // carries 16 / 8 / 4 by their run lengths, solver_setup.cpp)
  int spmv_variant = -1;     // CSR engine: 0 LDS-staged tiles, 1 direct, 2 CSR-vector, 4 row-length adaptive per
                             // tile (direct or 16 lanes per row); -1 = auto (1 when every row has <= 16 entries, else 4)
  int recurrence = 0;        // 0 = two-pass / two-reduction (reference order), 1 = single-reduction fused pass,
                             // 2 = pipelined CG (Ghysels-Vanroose: the all-reduce overlaps the SpMV; cg_pipe.hip)
  int pipe_rr = 0;           // pipelined CG: every |k| iterations recompute w = A r, s = A p, z = A s (their
                             // recurrences drift); k < 0 also replaces r = b - A x (true residual); 0 = off
  int halo_mode = -1;        // ghosts: 0 = column-window ranges (p2p send/recv), 1 = all-gather of equal row blocks
                             // (unstructured sparsity), -1 = auto (partition_rows)
  int checkpoint_every = 0;  // > 0: solve() writes a checkpoint every ~k iterations (at poll points)
  std::string checkpoint_path;  // per-rank file prefix ("<path>.rank<r>")
  double watchdog_seconds = 0.0;  // > 0: solve() fails (and aborts the communicator) if one poll interval
                                  // makes no progress for this long (bounded host wait)
  int graph_iters = 32;      // iterations per graph launch (even, >= 2); the last < graph_iters run as pairs
                             // (32 vs 2: 4096^2 4700 -> 5025 it/s, profiles/r1_graph_iters.log)
  int placement_tries = 6;   // single-reduction form: time the pass on this many physical placements of the vector
                             // set at setup and keep the fastest (1 = off; profiles/r1_placement_probe.md)
  int placement_leads = 16;  // ... times this many start offsets of the vectors inside their allocations
                             // (16384^2: 3 x 8 -> 503-517 it/s, 6 x 8 -> 516-525, 6 x 16 -> 524-525;
                             // profiles/r3_placement_depth.txt)
  int transport_probe = -1;  // P > 1, at the first reset: the transport probe (GpuCgSolver::probe_transport_) runs the
                             // same iterations from the same start with the ghost lines pulled (halo_pull auto) and
                             // exchanged, then with the alternative all-reduce (a PeerHaloComm whose IPC mailboxes are
                             // mapped but not selected) against the first, and keeps the fastest correct arm: the
                             // pulled run must reproduce the exchanged one bit for bit, the IPC sums the RCCL ones to
                             // rounding.  -1 = auto (on when there is a choice), 0 = off (the configured transport)
  int reserve_cus = 0;       // CUs withheld from the compute stream (a CU-masked queue, the mask's top bits; 32 = one
                             // per shader engine) so a collective's ~270-VGPR kernels find a free CU beside the
                             // resident pass (profiles/r3_cumask_probe.md); the pass grids are sized for the CUs
                             // left.  0 = off
  PassForm form;             // pass-form overrides (auto by default)
  TestHooks hooks;           // test / fault-injection hooks
};

struct CgResult {
  int iterations = 0;        // number of SpMVs performed (= reference loop trips)
  bool converged = false;
  bool breakdown = false;    // NaN/Inf in a reduction
  double rnorm = 0.0;        // final ||r||_2 (recurrence residual)
  int beta_clamps = 0;       // single-reduction form: passes whose expanded ||r_k||^2 estimate was clamped at 0
  double rr0_local = 0.0;    // b.b over this rank's rows (||r_0||^2 summed over ranks)
  double setup_seconds = 0.0;
  double solve_seconds = 0.0;
  double iters_per_second() const { return solve_seconds > 0 ? iterations / solve_seconds : 0.0; }
};

// Host CSR with int64 row pointers, int32 (ext-local) columns, fp64 values.
struct HostCsr {
  int64_t n_rows = 0;
  std::vector<int64_t> rowptr;
  std::vector<int32_t> cols;
  std::vector<double> vals;
  int64_t nnz() const { return rowptr.empty() ? 0 : rowptr.back(); }
};

// Owned rows of `L`, columns mapped to L.ext_index().  Multithreaded.
HostCsr build_local_csr(const ProblemSpec& s, const LocalLayout& L, int threads = 0);
std::vector<double> build_rhs(const ProblemSpec& s, int64_t r0, int64_t r1);
// y[i] = sum_j A[i,j] x_ext[j]  (x in ext coordinates)
void csr_spmv(const HostCsr& A, const double* x_ext, double* y);

// Single-process CPU reference CG: the reference recurrence op-for-op
// (copy, nrm2, SpMV, dot, axpy, axpy, nrm2, scal, axpy — CUDACG.cu:248-351).
CgResult cpu_cg(const ProblemSpec& s, const CgOptions& opt, std::vector<double>* x_out,
                std::vector<double>* rnorm_history = nullptr);

// Same recurrence with P virtual ranks in one process: each rank owns a
// LocalLayout, builds its local CSR, exchanges halos per the plan (memcpy from
// the peer's owned block into its ghosts) and reduces dot products in rank
// order.  Validates the partition + halo plan used by the GPU solver.
CgResult cpu_cg_partitioned(const ProblemSpec& s, int world, const CgOptions& opt,
                            std::vector<double>* x_out,
                            std::vector<double>* rnorm_history = nullptr);

}  // namespace mcg
