// Distributed GPU CG solver (one rank = one GPU).
//
// Per rank: the owned rows of A (CSR int32/int64 row pointers, or SELL-64),
// generated on device; ext-layout r and p (double-buffered) vectors with ghost
// regions; owned x / Ap / b; a device-resident CgState.  The iteration is a
// fixed sequence of stream operations with zero host synchronisation:
//
//  compute stream S0                              comm stream S1
//  ─────────────────                              ──────────────
//  record E_r (r_k, p_{k-1} final) ─────────────► wait E_r; RCCL group{send/recv
//  K_A interior rows (no ghosts needed)            r and p_{k-1} boundary rows};
//  wait E_h ◄──────────────────────────────────── record E_h
//  K_A boundary rows
//  cg_reduce(A) ; ncclAllReduce(pAp)  (8 B)
//  K_B (r -= alpha Ap, partial r.r)
//  cg_reduce(B) ; ncclAllReduce(rr_new) (8 B)
//
// The host enqueues iterations (pairs are captured once into a hipGraph and
// replayed), and polls the device convergence latch every `check_every`
// iterations through a pinned buffer; iterations enqueued after the latch
// fires are no-ops, so the iteration count is exactly the reference's.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>
#include <memory>
#include <vector>

#include "mcg/cg.hpp"
#include "mcg/comm.hpp"
#include "mcg/device.hpp"
#include "mcg/kernels.hpp"
#include "mcg/partition.hpp"

namespace mcg {

struct SolverInfo {
  int64_t n_global = 0, n_local = 0, nnz_local = 0;
  int64_t ext_len = 0, halo_in = 0, halo_out = 0;
  int64_t interior_rows = 0;
  bool idx64 = false;
  int format = 0;
  size_t device_bytes = 0;
  double bytes_per_iter_model = 0;  // modelled HBM bytes per iteration (this rank)
  int grid_a = 0, grid_b = 0;
  int grid_odd = 0;  // 2-D lean-only odd passes on a grid of their own (CgOptions::form.lean_bpc_odd), else 0
  bool lean_mix = false;  // ... chosen by the setup: packed edges, even passes 5 waves / SIMD, odd depth 4
  double lean_split = 0.0;  // > 0: lean and generic launches split by run (the fraction of runs on the lean one)
  int64_t max_row_len = 0;
  int spmv_variant = 0, spmv_param = 0;
  int recurrence = 0;
  int pipe_rr = 0;  // pipelined CG: residual-replacement period (0 = none)
  bool pipe_ar_first = false;  // pipelined CG: the all-reduce branch is enqueued before S (it took longer)
  double pipe_spmv_us = 0.0, pipe_allreduce_us = 0.0;  // the two branch times measured at setup
  bool interleave = false;
  int window = 0;  // LDS window width (doubles) of the windowed pass; 0 = off
  bool pipeline = false;
  bool carry = false;  // line-carry pass (single GPU: every pass; multi-rank: the interior launch)
  bool fused_reduce = false;  // the pass reduces its own block partials (one kernel per iteration)
  bool pmat = false;          // materialized-p split pass (irregular-sparsity path)
  bool tiles = false;         // ... its SpMV on L2-segment COO tiles (CgOptions::tiles)
  int tiles_tu = 0;           // ... entries per lane in flight (kern::tiles_tu; 0 = no tiles)
  int tile_segments = 0;      // column segments of the tiles (G)
  int sigma = 0;              // SELL-C-sigma window (rows) of a user matrix; 0 = slices in row order
  double sell_fill = 1.0;     // stored SELL slots / nonzeros (padding overhead)
  bool allgather = false;     // ghosts refreshed by all-gather (unstructured sparsity)
  bool ag_overlap = false;    // the own-block SpMV half runs while the all-gather is in flight
  bool ap_recompute = false;  // line-carry pass recomputes Ap instead of storing it (CgOptions::ap_recompute)
  bool halo_ahead = false;    // multi-rank stencil halo exchanged right after the pass that produced it, next to
                              // the all-reduce; one full pass per iteration (CgOptions::halo_ahead)
  double ag_local_frac = 0.0; // own-block slots / all slots (the part of the SpMV that hides the all-gather)
  int graph_fallbacks = 0;    // graph captures / launches that fell back to eager iterations
  bool graphs = false;        // iterations replayed as hipGraphs (false: eager launches)
  bool xcd_map = false;  // XCD-aware contiguous slice regions (auto for the 3-D stencil's generic pass)
  bool dia4 = false;     // SELL-64/dia4 storage for the Ap-recomputing line-carry pass (CgOptions::carry_dia)
  bool halo_pull = false;  // PassForm::halo_pull: the in-kernel halo (ghost lines read from the peers' rows)
  bool p3buf = false;      // PassForm::p3buf: three p buffers, no compact edge arrays (cg_carry_ar.hip T3)
  bool diav = false;
  double aligned_fill = 0.0;  // user matrices: SELL-64/aligned slots per nonzero of the per-slice offset unions     // SELL-64/diav: the line carry streams per-row coefficients (variable-coefficient stencils)
  bool p3 = false;       // ... in its three-term form (CgOptions::p3)
  double dia_uniform = 0.0;  // dia4 slices whose 64 rows share one value pattern (no codes streamed; PassForm::dia_uniform)
  bool lean_only = false;    // every run of the three-term carry takes the lean step (lean-only kernels)
  int ar3_kw = 0;        // 3-D Ap-recomputing plane carry: waves (grid lines) per block; 0 = not in use
  int ar3_runs = 0;      // ... runs of planes per job column (kern::carry3_runs)
  bool carry_xchg = false;  // 3-D plane carry: the +-N rows of a block's inner waves exchanged through LDS
  int placement_sets = 1;       // vector placements timed at setup (CgOptions::placement_tries)
  double placement_gain = 1.0;  // slowest / fastest of the timed placements (the fastest is kept)
  double placement_best_ms = 0.0, placement_worst_ms = 0.0;  // two even/odd pass pairs
  int placement_lead_trial = 0;  // start-offset trial kept (0 = allocation starts)
  size_t placement_peak_bytes = 0;  // extra device bytes held while the probe compared vector sets
  // the transport probe (GpuCgSolver::probe_transport_; P > 1, the first reset): microseconds per iteration,
  // the mean over the ranks, of each arm it ran (0: not run) -- pulled / exchanged ghost lines with the first
  // all-reduce, the alternative (IPC) all-reduce with the halo chosen -- and what it found
  bool probe_ran = false;
  double probe_pull_us = 0.0, probe_xchg_us = 0.0, probe_alt_us = 0.0;
  int probe_iters = 0;             // timed iterations per arm (after 2 + as many untimed)
  bool probe_pull_bitwise = false; // the pulled run reproduced the exchanged one bit for bit on every rank
  bool probe_alt_close = false;    // the alternative all-reduce's run matched the first's to 1e-6, no time-out
  bool probe_alt_timeout = false;  // ... its bounded wait gave up on some rank
  bool alt_allreduce = false;      // the all-reduce runs on the alternative transport (IPC mailboxes)
};

class GpuCgSolver {
 public:
  // `comm` may be null for a single rank; it is not owned.
  GpuCgSolver(const ProblemSpec& spec, const CgOptions& opt, int rank = 0, int world = 1,
              Communicator* comm = nullptr);
  ~GpuCgSolver();
  GpuCgSolver(const GpuCgSolver&) = delete;
  GpuCgSolver& operator=(const GpuCgSolver&) = delete;

  void setup();                     // generate matrix + RHS on device (timed as setup)
  void reset();                     // x = 0, r = b, p = 0, scalars; iteration counter = 0
  CgResult solve(bool resume = false);  // [reset +] iterate to tol/maxit with polling + finalise
  // checkpoint / resume of the full iteration state (x, r, p, Ap, device scalars,
  // iteration counter) of this rank; the file is "<prefix>.rank<r>"
  void save_checkpoint(const std::string& prefix);
  void load_checkpoint(const std::string& prefix);
  void run_iterations(int k);       // enqueue k more iterations (benchmark mode), no sync
  void finalize();                  // enqueue the deferred last x update (if not latched)
  void synchronize();
  CgResult result();                // read the device state (syncs)
  std::vector<double> x_local();    // owned part of x (syncs)
  double true_residual_norm();      // ||b - A x||_2 over all ranks (syncs)
  // Diagnostic: run `iters` more single-reduction iterations eagerly with hipEvents at every
  // phase boundary (halo on the side stream, interior / boundary passes, reduce, all-reduce) and
  // return the mean microseconds per phase (the first iteration is an untimed warm-up when iters > 1).
  // Advances the solver like run_iterations().
  std::vector<std::pair<std::string, double>> phase_profile(int iters);

  const SolverInfo& info() const { return info_; }
  const LocalLayout& layout() const { return L_; }
  hipStream_t stream() const { return s0_.get(); }
  int iterations_enqueued() const { return k_; }

 private:
  template <typename IdxT> void build_csr_(DeviceBuffer<int64_t>& rp64, const HostCsr* user);
  void enqueue_iteration_(int k);
  void enqueue_spmv_(int k, int which, int final_mode);  // which: 0 all, 1 interior, 2 boundary
  // single-reduction fused pass; `fused_red`: this launch takes part in the in-kernel reduction
  void enqueue_f1_(int k, int which, int final_mode, bool fused_red = false);
  void enqueue_halo_f1_(int k, hipStream_t s);            // ghosts iteration k of the single-reduction form reads
  void wait_bounded_(hipEvent_t ev);                       // poll wait with the optional watchdog
  void enqueue_iteration_f1_(int k);
  int enqueue_pass_(int k, bool fused_red);  // the pass over every owned row (lean_split: two launches)
  void enqueue_iteration_split_(int k);                   // materialized-p split pass (pmat_)
  void enqueue_iteration_pipe_(int k);                    // pipelined CG (recurrence 2)
  void pick_pipe_order_();                                // pipelined CG: which fork branch goes first
  void spmv_plain_(const double* x_ext, double* y, hipStream_t s);  // y = A x, the format's plain SpMV
  void enqueue_split_spmv_(int k, int which, bool fused_red, int part = 0);  // part: cg_split_spmv
  void capture_pair_(int kind, int phase);
  void join_halo_();            // s0_ waits for a halo in flight on s1_
  void ensure_ghosts_(int k);   // ghosts of iteration k in place on s0_ (joins a prefetch or exchanges now)
  void inject_fault_(int k);
  std::vector<DeviceBuffer<double>*> vectors_();  // the per-pass vector streams (x, r / Ap / pairs, p)
  void allocate_vectors_();
  void probe_placement_();
  bool all_ranks_agree_(bool mine);  // setup-time agreement across ranks (one all-reduce)  // keep the fastest of several placements of the vectors (CgOptions::placement_*)
  static constexpr size_t kLeadCap = (4u << 20) / sizeof(double);  // room for vector start offsets (4 MiB)

  ProblemSpec spec_;
  CgOptions opt_;
  int rank_, world_;
  Communicator* comm_;
  LocalLayout L_;
  SolverInfo info_;
  bool use_comm_ = false, use_halo_ = false;
  bool setup_done_ = false;
  int k_ = 0;  // host-side iteration counter (parity of the p double buffer)
  bool finalized_ = false;
  bool prefetch_halo_ = false;  // single-reduction form: next iteration's halo right after the boundary pass
  int halo_ready_for_ = -1;     // iteration whose halo is already enqueued on s1_ (ev_h_)
  bool halo_ahead_ = false;     // CgOptions::halo_ahead in effect
  bool pull_ = false;           // PassForm::halo_pull in effect (in-kernel halo)
  int pull_from_ = 2;           // ... first iteration that pulls (reset / resume + 2: the earlier ones exchange)
  bool pull_mapped_ = false;    // ... pull_p_ / pull_ap_ resolved (map_pull_)
  bool pull_checked_ = false;   // ... verify_pull_ ran (the first reset)
  const double* pull_p_[3][2] = {{nullptr, nullptr}, {nullptr, nullptr}, {nullptr, nullptr}};  // [p buffer][lo, hi side]
  const double* pull_ap_[2][2] = {{nullptr, nullptr}, {nullptr, nullptr}};  // [apx buffer][lo, hi side]
  std::vector<double*> halo_reg_;  // the buffers registered with the communicator (its peer_view order)
  double* pull_host_ = nullptr;    // TestHooks::pull_proxy 1: the stand-in ghost lines in pinned host memory
  bool map_pull_();     // false: a peer's buffers are not mapped here (not attached), or their layout differs
  void verify_pull_();  // the first reset: every rank reads a pattern through the pull pointers, or pull_ goes off
  void first_reset_checks_();  // verify_pull_ + probe_transport_, once (the first reset or checkpoint load)
  void probe_transport_();     // P > 1: time (and check) the halo / all-reduce transports, keep the best
  void reset_state_();         // reset()'s state: x = 0, r = b, p = 0, scalars, k = 0
  void allreduce_host_(double* v, int n);  // setup-time sum of n host doubles over the ranks
  bool probed_ = false;
  bool lean_split_ = false;     // 2-D three-term dia4 carry: the lean kernels over the runs that qualify, then the
                                // generic kernels over the rest (same grid; the second launch finishes the reduction)
  bool combo_ = false;           // ... and one combined launch (TileRanges::gen_blocks)
  double split_t3_lean_ = -1.0;  // ... with three p buffers (runs whose neighbouring columns match too): the lean
                                 // share of the runs, -1 = not applicable
  bool ar_ = false;             // CgOptions::ap_recompute in effect
  bool ar3_ = false;            // ... the 3-D plane carry (cg_carry_ar3)
  bool p3_ = false;             // ... the 2-D carry's three-term form (CgOptions::p3)
  bool lean_only_ = false;      // ... every run lean (carry_lean_failures == 0)
  bool probing_ = false;        // placement probe running: passes take k's kernels, never first / check
  bool split_ = false;          // interior / boundary launches around an overlapped halo
  int ghosts_for_ = -1;         // halo_ahead: iteration whose ghosts are in place or in flight on s1_
  bool halo_pending_ = false;   // ... in flight: s0_ must wait for ev_h_ before reading them

  Stream s0_, s1_, s2_;
  int ncu_ = 0;  // CUs of the device
  Event ev_r_, ev_h_, ev_t0_, ev_t1_, ev_poll_[2], ev_sync_[2], ev_ls_[2];
  // matrix
  DeviceBuffer<int32_t> rp32_;
  DeviceBuffer<int64_t> rp64_;
  DeviceBuffer<int32_t> cols_;
  DeviceBuffer<double> vals_;
  DeviceBuffer<int64_t> slice_ptr_;
  DeviceBuffer<int16_t> dcols_;  // SELL-64/d16 column offsets
  bool d16_ = false;
  DeviceBuffer<uint8_t> codes_;  // SELL-64/c8 dictionary codes
  DeviceBuffer<double2> dict_;
  DeviceBuffer<uint8_t> dia4_;    // SELL-64/dia4 copy (Ap-recomputing carry; 160 B per slice)
  DeviceBuffer<double> cv_;       // SELL-64/diav: cvd | cve | cvs, (n + line) doubles each (kernels.hpp SellDev)
  int64_t cv_len_ = 0;            // ... 3-D (diav3_): | cvt, (n + plane) doubles each
  bool diav_ = false;
  bool diav3_ = false;
  DeviceBuffer<double> dvals_;    // ... its value table (16 doubles)
  DeviceBuffer<uint64_t> dpat_;   // ... its uniform-slice patterns and run lengths (SellDev::dpat)
  DeviceBuffer<int32_t> gen_list_;  // a split rank on three p buffers: its generic runs (TileRanges::gen_list)
  DeviceBuffer<int32_t> perm_;    // SELL-C-sigma slot -> local row (user matrices)
  DeviceBuffer<int32_t> soffs_;   // SELL-64/aligned per-slot column offsets
  bool aligned_ = false;
  bool user_aligned_ = false;  // SELL-64/aligned from a user matrix's per-slice offset unions (host-built)
  DeviceBuffer<int32_t> lslots_;  // SELL-64/aligned + all-gather: per slice the own-block slot run {a, b}
  bool ag_overlap_ = false;
  int ndict_ = 0;
  bool c8_ = false;
  // L2-segment COO tiles (cg_tiles.hip): tile pointers, packed (row, column) indices, values, pacing
  bool tiles_ = false;
  int tile_ww_ = 4;  // PassForm::tile_waves in effect
  kern::TilesGeometry tgeo_;
  DeviceBuffer<int64_t> tptr_;
  DeviceBuffer<uint32_t> tidx_;
  DeviceBuffer<double> tvals_;
  DeviceBuffer<unsigned> tpace_;
  int tg_lo_ = 0, tg_hi_ = 0;  // the tile segments inside the own block of p (all-gather overlap)
  kern::TilesDev tiles_view() const {
    kern::TilesDev t;
    t.tptr = tptr_.get();
    t.idx = tidx_.get();
    t.vals = tvals_.get();
    t.n_rows = L_.n_local();
    t.nblocks = tgeo_.nblocks;
    t.G = tgeo_.G;
    t.seg_shift = tgeo_.seg_shift;
    t.tb = tgeo_.tb;
    t.pace = tpace_.get();
    t.ext_len = L_.ext_len;
    t.g_lo = tg_lo_;
    t.g_hi = tg_hi_;
    const double ntiles = (double)tgeo_.nblocks * (double)tgeo_.G;
    t.tu = kern::tiles_tu(ntiles > 0 ? (double)tidx_.size() / ntiles : 0.0);
    t.ww = tile_ww_;
    if (const char* e = std::getenv("MCG_TILES_TU")) t.tu = std::atoi(e) == 8 ? 8 : 10;  // test override
    return t;
  }
  DeviceBuffer<int32_t> win_;  // per-chunk [lo, hi) ext-column windows (windowed pass)
  int win_doubles_ = 0;         // 0 = windowed pass off
  bool pipe_ = false;           // software-pipelined stencil pass
  bool carry_all_ = false, carry_int_ = false;  // line-carry pass for the all-rows / interior launch
  bool carry_general_ = true;                   // line-carry pass with the memory-gather slow path
  int32_t carry_lo2_ = 0;                       // line-carry pass: second carried offset (3-D: N)
  std::vector<int64_t> dict_offsets_;           // SELL-64/c8: the distinct column offsets
  SellDev sell_view() const {
    SellDev s{slice_ptr_.get(), cols_.get(), vals_.get(), L_.n_local()};
    s.dcols = dcols_.get();
    s.own_off = L_.own_off;
    s.codes = codes_.get();
    s.dict = dict_.get();
    s.ndict = ndict_;
    s.perm = perm_.get();
    s.soffs = soffs_.get();
    s.ext_len = L_.ext_len;
    s.local_slots = lslots_.get();
    s.smeta = smeta_.get();
    s.dia4 = dia4_.get();
    s.dvals = dvals_.get();
    s.dpat = dpat_.get();
    if (cv_.get() != nullptr) {
      s.cvd = cv_.get();
      s.cve = cv_.get() + cv_len_;
      s.cvs = cv_.get() + 2 * cv_len_;
      if (diav3_) s.cvt = cv_.get() + 3 * cv_len_;
    }
    return s;
  }
  // vectors
  DeviceBuffer<double> x_, r_, p_[3], Ap_, b_, partials_;  // p_[2]: the third p buffer (p3buf_)
  bool p3buf_ = false;  // PassForm::p3buf: p_j in p_[j mod 3] (else p_[j & 1])
  int pidx_(int j) const { return p3buf_ ? ((j % 3) + 3) % 3 : (j & 1); }
  double* pbuf_(int j) { return p_[pidx_(j)].get(); }
  DeviceBuffer<double> r1_, Ap1_;  // second parity buffers of the single-reduction recurrence
  bool pipe_ar_first_ = false;
  DeviceBuffer<double> w_, z_, q_, xe_;  // pipelined CG: w = A r (ext), z = A s, q = A w, x in the ext layout
  DeviceBuffer<double> xt_;  // x in the ext layout for true_residual_norm, registered with a peer-mapping
                             // communicator (its halo can only move registered buffers)
  DeviceBuffer<double> ra_[2];     // interleaved {r, Ap} pairs by parity (2 * ext_len doubles each)
  DeviceBuffer<uint32_t> smeta_;  // Ap-recomputing carry: per-slice (first slot / 64 | width << 28)
  DeviceBuffer<double> ape_[2];    // Ap-recomputing carry: Ap of the slices' edge rows, by parity
  DeviceBuffer<double> apx_[2];    // ... multi-rank: Ap of the first / last line + ghost lines (ext layout)
  int pstride_ = 0;                // partial-array stride (4 arrays in the single-reduction form)
  int bnd_base_ = 0;               // first partial slot of the boundary launch (a multiple of kRedGroup)
  bool fused_red_ = false;         // in-kernel reduction of the fused pass (CgOptions::fused_reduce)
  bool pmat_ = false;              // materialized-p split pass (CgOptions::pmat)
  int red_groups_all_ = 0, red_groups_split_ = 0, red_groups_b_ = 0, red_l2s_ = 0, red_groups_odd_ = 0;
  DeviceBuffer<unsigned> red_cnt_;  // group counters + top counter (zeroed at setup, reset by the kernels)
  DeviceBuffer<double> red_l2_;     // [4][red_l2s_] group sums
  DeviceBuffer<CgState> st_;
  PinnedBuffer<CgState> host_st_;
  // launch geometry
  TileRanges tr_all_, tr_int_, tr_bnd_;
  int g_all_ = 1, g_int_ = 1, g_bnd_ = 1, g_b_ = 1;
  int g_odd_ = 0;  // 2-D lean-only odd passes: their own grid (0 = g_all_)
  int32_t alt_chunk_even_ = 0, alt_chunk_odd_ = 0;  // ... run lengths (lines) of the even / odd decompositions
  int lean_depth_even_ = 0, lean_depth_odd_ = 0;       // 2-D lean prefetch depth per parity (0 = 3; 13 / 14 packed edges)
  bool auto_mix_ = false;                              // ... chosen by the setup (4-blocks-per-CU grids)
  // graph of two iterations (even, odd)
  // [0]: one iteration pair, [1]: graph_iters iterations (when > 2)
  // [kind][phase]: with three p buffers (p3buf_) a captured run of iterations depends on k mod 3 too
  hipGraph_t graph_[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
  hipGraphExec_t graph_exec_[2][3] = {{nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr}};
  void drop_graphs_();
  double setup_seconds_ = 0.0;
  uint64_t fingerprint_ = 0;  // problem_fingerprint(spec_), recorded in checkpoints (computed on first use:
  bool fingerprint_done_ = false;  // O(nnz) on the host for a user matrix, so never at setup)
  uint64_t fingerprint() {
    if (!fingerprint_done_) {
      fingerprint_ = problem_fingerprint(spec_);
      fingerprint_done_ = true;
    }
    return fingerprint_;
  }
};

}  // namespace mcg
