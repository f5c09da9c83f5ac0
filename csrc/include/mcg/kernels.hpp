// Hand-written gfx950 kernels (launchers).  Device code lives in
// csrc/gpu/*.hip; nothing here calls rocBLAS/rocSPARSE — the reference's
// cuBLAS/cuSPARSE calls are replaced by:
//
//   cg_spmv_fused   K6+K8+K9(x)+K12+K13 : p_k = r + beta p_{k-1} (on the fly),
//                   Ap = A p_k (CSR, LDS-staged row tiles), x += alpha_{k-1} p_{k-1},
//                   block partials of p_k . Ap
//   cg_update_r     K10+K11 : r -= alpha Ap, block partials of r . r
//   cg_reduce       fixed-order sum of block partials + device-side scalar
//                   bookkeeping (alpha/beta/rho never visit the host; K3/K8/K11's
//                   blocking D2H reads are gone)
//   gen_*           on-device generation of each rank's owned rows + RHS
//   spmv_csr / dot / axpy / xpby   unfused building blocks (ops API, tests)
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <vector>

#include "mcg/problem.hpp"

namespace mcg {

// Device-resident CG scalars.  All fields are written only by the single-block
// cg_reduce kernel (or by RCCL in-place all-reduces of rr_new / pAp), and read
// by the streaming kernels, so no intra-launch hand-off is ever needed.
struct alignas(64) CgState {
  double rr_new;  // r_k . r_k (global) — the newest residual norm^2 (all-reduce slot)
  double rho;     // r_{k-1} . r_{k-1} after rotation (the reference's `rho`)
  double pAp;     // p . Ap of the last SpMV (global after all-reduce; all-reduce slot)
  double rr0;     // b . b
  double rr_final;  // rr_new captured when the latch fires (later no-op all-reduces may clobber rr_new)
  double a_prev;    // single-reduction form: alpha of the pass before the last (paired x updates)
  double b_prev;    // ... and the beta that pass used (p_{k-1} = r_{k-1} + b_prev p_{k-2}: the three-term carry
                    // recovers r_{k-1} from the two stored p's, cg_carry_ar.hip)
  double pad0_[1];
  // single-reduction recurrence: {p.Ap, r.Ap, Ap.Ap, r.r} of the last fused pass
  // (one contiguous 32-B all-reduce slot)
  double red[4];
  int iter;      // completed iterations (SpMVs whose residual update ran)
  int done;       // latch: 1 = converged in-loop, 2 = maxit finalised, 3 = breakdown
  int conv_iter;  // iteration count at the latch
  int converged;  // ||r|| < tol at the end
  int breakdown;  // NaN/Inf seen
  int clamps;     // single-reduction form: passes whose expanded ||r - a Ap||^2 was <= 0 (beta clamped to 0)
  int pad_[2];
};

enum ReduceMode : int { kReduceInit = 0, kReduceA = 1, kReduceB = 2, kReduceFinal = 3, kReduceScalar = 4 };

// Rows of a launch = up to two local row ranges [b0,e0) ∪ [b1,e1), cut in
// tiles of kTileRows consecutive rows.
constexpr int kTileRows = 256;
struct TileRanges {
  int64_t b0 = 0, e0 = 0, b1 = 0, e1 = 0;
  int64_t nt0 = 0, ntiles = 0;
  int32_t xcd = 0;  // > 1: XCD-aware contiguous tile regions (see spmv_engines.hpp tile_cursor)
  // > 0 (single range, nt0 % strip == 0): units are visited in "vertical strips" — unit
  // index u = col * L + line maps to b0 + line * strip + col (L = nt0 / strip), and every wave
  // takes a contiguous run of u.  With strip = slices per grid line, a wave walks one column of
  // slices down the grid, so a row's +-N (next/previous line) neighbours are the wave's own
  // previous/next slices: cache hits instead of a second/third HBM read of the same vector rows.
  int32_t strip = 0;
  // 3-D plane carry: runs of planes per job column (> 0: chosen at setup by carry3_runs, so the
  // jobs fill whole rounds of the launch's blocks); 0 = blocks / jobs-per-run (at least 1)
  int32_t runs3 = 0;
  // 2-D lean three-term carry with the odd passes on a grid of their own (lean_bpc_odd): the other
  // parity's run length in lines.  The next pass reads r_{k-1} on the line before / after each of ITS
  // runs, which this pass stores only on its own runs' first / last lines, so it also stores r on the
  // first / last line of every run of the other decomposition; 0 = both parities share the runs
  int32_t alt_chunk = 0;
  // 2-D three-term dia4 carry split by run eligibility (a matrix whose slice patterns are uniform only
  // in places): 1 = this launch (the lean kernels) takes only the runs that qualify for the lean loop,
  // 2 = this launch (the generic kernels, same grid) only the others; 0 = every run
  int32_t lean_split = 0;
  // a split rank on three p buffers (T3): a T3 run needs nothing stored by its neighbours, so it splits at
  // any line.  sub_ranges != 0: the lean launch (lean_split 1) takes every lean stretch of its runs
  // (next_lean_range) and the generic launch (lean_split 2) only the ranges listed in gen_list (ngen
  // triples: slice column, first line, end line; ascending, pieces of at most 32 lines) -- a small grid,
  // one wave a range, where whole generic runs on single waves had been the split pass's critical path
  int32_t sub_ranges = 0;
  int32_t ngen = 0;
  const int32_t* gen_list = nullptr;
  // lean_split 1 with sub_ranges: > 0 = one combined launch -- its first gen_blocks workgroups (a multiple of 8)
  // run the generic step over gen_list, the rest the lean stretches (no second launch, no side stream)
  int32_t gen_blocks = 0;
};
// `tile` = rows per tile (kTileRows for CSR row tiles, 1 for SELL slice units)
TileRanges make_tiles(int64_t b0, int64_t e0, int64_t b1 = 0, int64_t e1 = 0, int64_t tile = kTileRows);

template <typename IdxT>
struct CsrDev {
  const IdxT* rowptr;
  const int32_t* cols;
  const double* vals;
  int64_t n_rows;
};

// SELL-C-sigma (C = 64 = one wave, sigma = 1 i.e. no sorting) view: slice s
// holds rows [64s, 64s+64), width w_s; entry j of row 64s+l is at
// slice_ptr[s] + 64 j + l (column-major inside the slice -> every lane's load
// of entry j is one coalesced 512-B wave access).  Padding entries have
// val 0 and col = the row's own diagonal column.
struct SellDev {
  const int64_t* slice_ptr;  // n_slices + 1
  const int32_t* cols;
  const double* vals;
  int64_t n_rows;
  // SELL-64/d16: 16-bit column offsets relative to the row's own ext column
  // (col = own_off + row + dcols[k]); used when the matrix bandwidth fits int16.
  // Index bytes per entry 4 -> 2.
  const int16_t* dcols = nullptr;
  int64_t own_off = 0;
  // SELL-64/c8 (csrc/gpu/dict.hip): one byte per entry indexing `dict`, pairs
  // {value, int64 column offset bits}; used when the matrix has <= 256 distinct
  // (value, offset) combinations.  Index + value bytes per entry 10 -> 1.
  const uint8_t* codes = nullptr;
  const double2* dict = nullptr;
  int32_t ndict = 0;
  // SELL-C-sigma (user matrices): slot i of the slices holds local row perm[i] (rows sorted by
  // length inside windows, so a slice pads less); nullptr = identity.  int32 columns only.
  const int32_t* perm = nullptr;
  // Ap-recomputing line carry: per slice (first slot / 64) | (width << 28) (slice_meta)
  const uint32_t* smeta = nullptr;
  // SELL-64/dia4 (Ap-recomputing 2-D line carry, sell_to_dia4): every slice has 5 slots, slot u
  // of a row holding its entry at the u-th canonical column offset (-line, -1, 0, +1, +line) as a
  // 4-bit index into `dvals` (an absent entry indexes +0.0).  Slice s, slot u: 32 bytes at
  // (5 s + u) * 32, lanes 2i / 2i+1 in one byte.  Diagonal-slot storage (DIA inside SELL): the
  // column offset is the slot's, so the pass needs no per-entry offset decode or operand select.
  const uint8_t* dia4 = nullptr;
  const double* dvals = nullptr;
  // SELL-64/dia4 slice patterns (dia_patterns): per slice, bit 31 set when all 64 rows hold the
  // same value index in every slot (the indices packed 4 bits per slot in bits 0..27; bit 28 / 29:
  // except lane 0's -1 / lane 63's +1 entry, absent: a slice at the start / end of a grid line),
  // and in the high word the number of consecutive lines, from this slice's line down the same slice column,
  // whose slices carry that same uniform pattern.  The line carry streams no codes over such runs
  // (the values sit in scalar registers); nullptr = every slice through the codes.
  const uint64_t* dpat = nullptr;
  // SELL-64/diav (variable-coefficient 2-D 5-point stencils, sell_to_diav): the row's own values in
  // three arrays of local rows shifted by one grid line (index line + i): cvd = a_ii, cve = a_{i,i+1},
  // cvs = a_{i,i+line}; the extra line in front holds zeros and, in cvs, the rank's line 0 north
  // coefficients (a_{i,i-line} of its first line).  A symmetric matrix's other two coefficients of
  // row i are its partners': west a_{i,i-1} = cve[i - 1], north a_{i,i-line} = cvs[i - line] (checked
  // bitwise at setup).  24 B per row streamed instead of one shared value table.
  // 3-D 7-point (sell_to_diav with plane > 0): four arrays shifted by one PLANE (index plane + i),
  // cvt = a_{i,i+plane} as well, the front plane of cvt holding the rank's plane 0 down coefficients
  // (a_{i,i-plane}); south a_{i,i-N} = cvs[i - N], down a_{i,i-plane} = cvt[i - plane].  32 B per row.
  const double* cvd = nullptr;
  const double* cve = nullptr;
  const double* cvs = nullptr;
  const double* cvt = nullptr;
  // SELL-64/aligned (long rows whose slices share their column offsets, e.g. the wide random-SPD
  // family): entry j of EVERY lane of slice s is the row's own column + soffs[slice_ptr[s] / 64 + j]
  // (one wave-uniform offset per slot, clamped to [0, ext_len); absent entries hold 0.0), so a
  // slot's 64 gathers are one contiguous 512-B run and no per-entry column index is stored.
  const int32_t* soffs = nullptr;
  int64_t ext_len = 0;
  // SELL-64/aligned with an all-gather ghost layout: per slice {a, b}, the run of slots whose 64
  // columns all lie in the rank's own block (aligned_local_slots); the split pass sums them while
  // the all-gather of p is in flight
  const int32_t* local_slots = nullptr;
};

namespace kern {

int num_cus();  // of the current device (cached)

// ---- generation (csrc/gpu/gen.hip) ----
void gen_rowlen(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t* rowptr, hipStream_t st);
void scan_inclusive_i64(int64_t* a, int64_t n, int64_t* tmp, hipStream_t st);  // tmp >= n/4096+1
int64_t scan_tmp_elems(int64_t n);
template <typename IdxT>
void gen_fill(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t col_lo, int64_t pad,
              const int64_t* rowptr64, IdxT* rowptr_out, int32_t* cols, double* vals, hipStream_t st);
void gen_rhs(const ProblemSpec& s, int64_t row_begin, int64_t n, double* b, hipStream_t st);
// max over a[0..n) (synchronous; setup only)
int64_t max_i64(const int64_t* a, int64_t n, hipStream_t st);
// CSR -> SELL-64 (slice_ptr must be precomputed on the host/device from row lengths)
void sell_slice_widths(const int64_t* rowptr64, int64_t n, int64_t* slice_ptr /* ns+1 */, hipStream_t st);
template <typename IdxT>
void csr_to_sell(const IdxT* rowptr, const int32_t* cols, const double* vals, int64_t n,
                 int64_t own_off, const int64_t* slice_ptr, int32_t* scols, double* svals,
                 hipStream_t st, int16_t* dcols = nullptr /* write 16-bit deltas instead of scols */);

// direct SELL-64(/d16) generation — no CSR intermediate (peak memory = the SELL arrays):
// rowptr64 = inclusive-scanned row lengths, slice_ptr from sell_slice_widths + scan;
// exactly one of scols (int32 ext columns) / dcols (int16 offsets from the row's own column)
void gen_fill_sell(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t col_lo, int64_t pad, int64_t own_off,
                   const int64_t* rowptr64, const int64_t* slice_ptr, int32_t* scols, int16_t* dcols, double* svals,
                   hipStream_t st);
// SELL-64/aligned for the wide random-SPD family: per 64-row slice, the candidate offsets that
// reach a column of the matrix for some row of the slice (sorted: the lower candidates descending,
// 0, the upper ascending); slice_ptr[s+1] = 64 * that count (then scan), and the fill writes the
// per-slot offsets (soffs[slice_ptr[s] / 64 + j]) and every lane's value (0 when absent)
void randspd_aligned_widths(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t* slice_ptr,
                            hipStream_t st);
void randspd_fill_aligned(const ProblemSpec& s, int64_t row_begin, int64_t n, const int64_t* rowptr64,
                          const int64_t* slice_ptr, int32_t* soffs, double* svals, hipStream_t st);
// per slice of an aligned matrix (S.slice_ptr, S.soffs, S.own_off, S.n_rows): out[2s..2s+1] = the
// slot run [a, b) whose columns own_off + 64 s + lane + offset lie in [own_off, own_off + n_rows)
// for all 64 lanes
void aligned_local_slots(const SellDev& S, int32_t* out, hipStream_t st);
// SELL-64/c8 dictionary (csrc/gpu/dict.hip) from a generated SELL-64(/d16) matrix: false if
// it has too many distinct values / offsets.  dict[vi * nd + di] = {value_vi, bits(offset_di)}.
bool sell_dict_build(const SellDev& S, std::vector<double2>& dict, int& nv, int& nd, hipStream_t st);
void sell_to_c8(const SellDev& S, const double2* dict, int nv, int nd, uint8_t* codes, hipStream_t st);

// ---- CG kernels (csrc/gpu/cg_kernels.hip) ----
// variant: 0 = LDS-staged tiles, 1 = direct thread-per-row, 2 = CSR-vector (G lanes/row),
//          3 = direct with non-temporal matrix loads;
// param: batch size U in {4,6,8} (variants 0/1) or G in {4,8,16} (variant 2)
template <typename IdxT>
void cg_spmv_fused(const CsrDev<IdxT>& A, const double* r_ext, const double* pold_ext,
                   double* pnew_ext, double* x, double* Ap, int64_t own_off, const TileRanges& tr,
                   double* partials, int grid, const CgState* st, double tol, int first,
                   int final_mode, int variant, int param, hipStream_t stream);
int spmv_param_for(int variant, int64_t max_row_len);
// `slices`: TileRanges in units of 64-row slices
void cg_spmv_fused_sell(const SellDev& A, const double* r_ext, const double* pold_ext,
                        double* pnew_ext, double* x, double* Ap, int64_t own_off,
                        const TileRanges& slices, double* partials, int grid,
                        const CgState* st, double tol, int first, int final_mode, int param,
                        int flags /* bit0: non-temporal matrix loads, bit1: two slices per wave,
                                     bit2: d16 column offsets, bit3: c8 dictionary codes */,
                        hipStream_t stream);
void cg_update_r(double* r_own, const double* Ap, int64_t n, double* partials, int grid,
                 const CgState* st, int unroll, hipStream_t stream);
void cg_reduce(const double* partials, int np, CgState* st, int mode, int first, double tol,
               hipStream_t stream);
void dot_partials(const double* a, const double* b, int64_t n, double* partials, int grid,
                  hipStream_t stream);
// scalar[0] = fixed-order sum of partials
void sum_partials(const double* partials, int np, double* out, hipStream_t stream);

// ---- single-reduction fused CG iteration (csrc/gpu/cg_fused1.hip) ----
// One streaming pass per iteration k:
//   r_k = r_{k-1} - a_{k-1} Ap_{k-1};  p_k = r_k + b_{k-1} p_{k-1};  x += a_{k-1} p_{k-1};
//   Ap_k = A p_k;  partials of {p_k.Ap_k, r_k.Ap_k, Ap_k.Ap_k, r_k.r_k}
// then ONE reduction (+ one 32-B all-reduce).  a_k = rr_k / pAp_k (exact norms);
// b_k = rr_{k+1} / rr_k with rr_{k+1} = rr_k - 2 a_k (r_k.Ap_k) + a_k^2 (Ap_k.Ap_k)
// (an exact expansion of ||r_k - a_k Ap_k||^2 over the actual vectors; convergence is
// tested on the exact rr_k of the stored residual, as in the reference).
// `fmt`: 0 CSR direct (param U), 1 SELL-64 (U), 2 SELL-64 two slices/wave (U), 3 SELL-64/d16,
// 4 SELL-64/c8.
struct F1Vectors {
  const double *r_old, *ap_old, *p_old;  // ext layout, iteration k-1
  double *r_new, *ap_new, *p_new;        // ext layout, iteration k
  double* x;                             // owned
  // interleaved layout: {r, Ap} pairs in one 16-B element per row, so a neighbour
  // gather is one 16-B load (+ the 8-B p load) instead of three 8-B loads
  const double2* ra_old = nullptr;
  double2* ra_new = nullptr;
  // x is updated in pairs: pass k odd applies a_{k-2} p_{k-2} (read from p_new before it is
  // overwritten) and a_{k-1} p_{k-1}; even passes leave x alone (-4 B/row/iteration).  p_fix =
  // the parity-1 p buffer, for the one-term catch-up when convergence latches after an even pass.
  const double* p_fix = nullptr;
  int64_t ext_len = 0;  // ext-layout length of r / Ap / p (bounds of the line-carry pass's edge loads)
  // Ap-recomputing carry (cg_carry_ar.hip): Ap of each slice's two edge rows (lanes 0 / 63),
  // 2 doubles per owned slice, iteration k-1 / k; r_old/new, p_old/new as above, ap_old/new the
  // ext-layout Ap of the rank's first / last line and of its ghost lines (multi-rank, else null).
  // The three-buffer lean passes (p_m2 below) neither read nor write the compact arrays (only pass 0,
  // the two-term kernel, still writes them)
  const double* ape_old = nullptr;
  double* ape_new = nullptr;
  // ... its three-term form: r of the same edge rows, same compact layout (2 doubles per slice), so
  // the neighbouring waves read 16 contiguous bytes per slice instead of two scattered sectors
  const double* re_old = nullptr;
  double* re_new = nullptr;
  // In-kernel halo (multi-rank lean carries; solver pull_): [0] the lo, [1] the hi ghost line / plane
  // read straight from the neighbour's rows instead of this rank's ghost rows.  pull_p[s][e] for an
  // ext index e of that ghost line is the owner's p_{k-1} of the same global row (a pointer into the
  // neighbour's mapped buffer, shifted by the two layouts' offsets), pull_ap likewise its Ap_{k-1};
  // nullptr: that side reads the local ghost rows a halo exchange filled.  The pass also copies the
  // pulled p_{k-1} into its own ghost rows of p_old (the p_{k-2} the next pass recovers r from).
  const double* pull_p[2] = {nullptr, nullptr};
  const double* pull_ap[2] = {nullptr, nullptr};
  // store the rank's first / last line's p_k and Ap_k write-through at system scope: the neighbours'
  // next pass reads them over the fabric, ordered after this pass by the all-reduce between
  int pull_pub = 0;
  // Three p buffers (solver p3buf_, the 2-D lean three-term carry, cg_carry_ar.hip T3): p_new is a buffer
  // this pass does not read, p_m2 = p_{k-2} (read-only); nullptr: two buffers, p_new holds p_{k-2} on
  // entry and is overwritten in place.  p_fix3[j % 3] = p_j's buffer (final mode's catch-up of a latched
  // even m reads p_{m-1}, m known on the device only)
  const double* p_m2 = nullptr;
  const double* p_fix3[3] = {nullptr, nullptr, nullptr};
};
// In-kernel reduction of a fused pass's block partials (replaces the cg_reduce_f1 launch, so
// one iteration is ONE kernel + the 32-B all-reduce).  Two-level last-arriver fan-in: each block
// stores its 4 partials write-through (sc1) and adds to its group's counter (kRedGroup blocks
// per group); the group's last arriver sums the group's partials in block order into lvl2 and
// adds to the top counter; the last group sums lvl2 in group order and updates the CgState
// exactly as cg_reduce_f1 mode 0 does.  Every sum has a fixed order (bitwise reproducible, and
// the same value however the blocks are scheduled).  Counters are zeroed at setup and reset by
// their last arriver.  The launches of one iteration (interior + boundary) share the groups:
// `base` = the launch's first partial slot, a multiple of kRedGroup.
constexpr int kRedGroup = 64;
struct RedCtl {
  unsigned* cnt = nullptr;  // [top] group counters, cnt[top] = the top counter
  double* lvl2 = nullptr;   // [4][l2s] group sums
  int l2s = 0, top = 0;
  int base = 0;
  int ngroups = 0;          // groups over every launch of the iteration; 0 = off
  int check = 0, first = 0; // as cg_reduce_f1 mode 0
};
// `k`: pass index (its parity selects the paired x update; final mode: m = k)
template <typename IdxT>
void cg_fused1(int fmt, int param, const CsrDev<IdxT>& A, const SellDev& S, const F1Vectors& v, int64_t own_off,
               const TileRanges& tr, double* partials, int pstride, int grid, CgState* st, double tol,
               int first, int check, int final_mode, int k, hipStream_t stream,
               bool pipe = false /* software-pipelined stencil pass: SELL d16/c8 + interleaved, every slice
                                    width <= param */,
               const RedCtl& rc = RedCtl());
// Line-carry variant for structured-grid stencils (SELL d16/c8 + interleaved {r, Ap}, every
// slice width <= param): `slices.strip` = S slices per grid line (the carried column offset is
// one line, 64 S rows), the launch one range of whole lines; a wave walks down one column of
// slices and keeps the previous / current / next line's p_k in registers.
// The plane carry's block exchange applies: lo2 whole slices, kWaves | grid lines per plane, 7-8 entries
bool carry_block_exchange_ok(int param, int32_t lo2, int64_t strip);
// Line-carry pass that recomputes Ap_{k-1} = A p_{k-1} instead of storing Ap (cg_carry_ar.hip):
// 2-D stencils (offsets 0, +-1, +-one line), SELL-64/c8 (cm 2) or /c4 (cm 3), <= 5 entries per
// row, one launch over the rank's whole lines.  final_mode: finalize()'s r_m / x_m pass.
void slice_meta(const int64_t* slice_ptr, int64_t n_slices, uint32_t* meta, hipStream_t stream);
// SELL-64/c8 (S.codes, S.dict with nd distinct offsets) -> SELL-64/dia4 (`dia4`: 160 B per slice,
// `dvals`: <= 16 doubles).  False (nothing usable written) when a nonzero entry's offset is not
// one of 0, +-1, +-line, a row's nonzero offsets are not strictly increasing in slot order (the
// dia4 sum must add the same products in the same order as the slot-order sum), or there are more
// than 16 distinct values.
// ln = 0: the 2-D offsets (-line, -1, 0, +1, +line), 160 B per slice; ln > 0: the 3-D offsets
// (-line, -ln, -1, 0, +1, +ln, +line), 224 B per slice
bool sell_to_dia4(const SellDev& S, int nd, int64_t line, int64_t ln, uint8_t* dia4, double* dvals,
                  hipStream_t stream);
// SELL-64 (d16 / int32 columns / c8) of a 2-D 5-point stencil (line = grid line, every local row
// in whole lines) -> SELL-64/diav: cv = 3 * (n + line) doubles (cvd | cve | cvs, SellDev).  False
// when an entry sits at another offset, a row's offsets are not strictly increasing, or the matrix
// is not bitwise symmetric inside the rank (west / north entries = their partners' east / south).
// plane > 0: a 3-D 7-point stencil (line = N, plane = N^2, every local row in whole planes): cv =
// 4 * (n + plane) doubles (cvd | cve | cvs | cvt)
bool sell_to_diav(const SellDev& S, int64_t line, double* cv, hipStream_t stream, int64_t plane = 0);
// SellDev::dpat from a dia4 copy (and its value table) of ns = ss * lines slices (ss slices per line,
// nslot 5 or 7); returns the number of uniform slices (synchronises the stream)
int64_t dia_patterns(const uint8_t* dia4, const double* dvals, int64_t ns, int64_t ss, int nslot, uint64_t* dpat,
                     hipStream_t stream);
// 3-D (7-pt) Ap-recomputing plane carry (SELL-64/dia4 with ln = N): blocks of kw = 16 waves on
// kw consecutive grid lines of one x slice; v.ap_old / ap_new = ext-layout Ap (outer lines, slice
// edge rows, and with gfull the first / last plane for the ghosts); grid = blocks (any count).
// With S.cvt set (SELL-64/diav 3-D, variable coefficients) the per-row values are streamed instead
// (kw = 8, 2 waves per SIMD: the lean loop's coefficient chain needs up to 256 VGPRs)
void cg_carry_ar3(int depth, int kw, const SellDev& S, const F1Vectors& v, int64_t own_off, const TileRanges& tr,
                  int32_t ln, bool gfull, double* partials, int pstride, int grid, CgState* st, double tol,
                  int first, int check, int k, int final_mode, hipStream_t stream, const RedCtl& rc = RedCtl(),
                  bool p3 = false, bool lean = false);
// True when every line's uniform slices share one value pattern (the pattern words of dia_patterns equal
// up to the line-start / line-end flags, bits 28 / 29): the three-buffer lean carry recomputes a slice's
// neighbours' edge rows with its own values (cg_carry_ar.hip T3)
bool dia_lines_uniform(const uint64_t* dpat, int64_t ss, int64_t nl, hipStream_t stream);
// Runs of a line (kw = 0, 2-D) / plane (kw = waves per block, 3-D, ln = N) carry launch of `grid`
// blocks over ss * nl slices that do not qualify for the lean step (SellDev::dpat); 0 lets the
// three-term passes launch their lean-only kernels (`lean`).  Synchronises the stream.
// The 3-D plane carry's run count (TileRanges::runs3) for `nb` blocks, `jpr` jobs per run and nl
// planes: the R whose job rounds x (planes per run + the 3-plane prologue) is least (ties: fewer runs);
// max_chunk > 0: only runs of at most that many planes (past 2^29 rows a lean run keeps its planes
// within 4 GiB of its base)
int32_t carry3_runs(int64_t nb, int64_t jpr, int64_t nl, int64_t max_chunk = 0);
// the 2-D carry's job decomposition of a launch of nw waves over nl lines of ss slices (every line in
// one launch): runs per slice column and lines per run
void carry_jobs_host(int64_t nw, int64_t ss, int64_t nl, int64_t& runs, int64_t& chunk);
// the in-kernel halo's setup check: out[i] = base[i] for i < n, loaded like the pass loads a pulled
// ghost line (system scope)
void pull_probe(const double* base, int64_t n, double* out, hipStream_t stream);
// a split rank on three p buffers: the ranges (slice column, first line, end line; at most maxlen lines, in a
// fixed order) the lean stretches of the lean launch's runs leave to the generic launch; false on overflow
bool split_generic_ranges(const uint64_t* dpat, int64_t ss, int64_t nl, int64_t ext_len, int grid, int maxlen,
                          std::vector<int32_t>& ranges, hipStream_t stream);
int64_t carry_lean_failures(const uint64_t* dpat, int64_t ss, int64_t nl, int64_t ext_len, int grid, int kw,
                            int32_t ln, hipStream_t stream, int runs3 = 0,
                            bool nbr = false,  // nbr: lean_eligible's neighbour check (split ranks, three p buffers)
                            std::vector<int32_t>* failed = nullptr);  // 2-D: the failing jobs, ascending
// cm: 2 SELL-64/c8, 3 SELL-64/c4, 4 SELL-64/dia4 (S.dia4 / S.dvals), 5 SELL-64/diav (S.cvd / cve / cvs,
// variable coefficients; lean runs stream them: every run of >= 3 lines).  p3 (dia4): three-term form --
// r_{k-1} = p_{k-1} - b_prev p_{k-2} from the two p buffers, r stored only at the slices' edge rows
// and the runs' first / last lines (v.r_old / r_new hold just those rows; pass 0 reads r_{-1} = b)
void cg_carry_ar(int cm,int param, int depth, const SellDev& S, const F1Vectors& v, int64_t own_off,
                 const TileRanges& slices, double* partials, int pstride, int grid, CgState* st, double tol,
                 int first, int check, int k, int final_mode, hipStream_t stream, const RedCtl& rc = RedCtl(),
                 bool p3 = false, int unroll = 1, bool lean = false);  // lean: the lean-only kernels
void cg_fused1_carry(int cm /* 1 SELL-64/d16, 2 SELL-64/c8, 3 SELL-64/c4 */, int param, int depth /* operand prefetch, lines */,
                     bool general /* false: every dictionary offset is 0, +-1, +-one line or +-lo2 (no slow path) */,
                     int32_t lo2 /* > 0: a second carried offset, gathered one line ahead (3-D: N); 0 = none */,
                     bool block_exchange /* lo2 rows of a block's inner waves through LDS (carry_block_exchange_ok) */,
                     const SellDev& S, const F1Vectors& v, int64_t own_off, const TileRanges& slices,
                     double* partials, int pstride, int grid, CgState* st, double tol, int first, int check,
                     int k, hipStream_t stream, const RedCtl& rc = RedCtl());
// Windowed variant for long banded rows: 1024-row chunks (16 slices) stage p_k for their
// column window [win[2c], win[2c+1]) in LDS once, the SpMV gathers from LDS.
constexpr int kWinRows = 1024;
constexpr size_t kWinMaxLds = 150 * 1024;  // dynamic LDS budget per block (gfx950: 160 KB per CU)
void chunk_windows(const SellDev& S, int32_t* win /* 2 per chunk */, hipStream_t stream);
int64_t win_chunks(const TileRanges& slices);  // chunks touched by a launch (grid sizing)
void cg_fused1_win_prepare(int win_doubles);     // setup: dynamic-LDS limit of the windowed kernels
void cg_fused1_win(int cm /* 0 SELL-64, 1 SELL-64/d16 */, int param, const SellDev& S, const F1Vectors& v,
                   int64_t own_off, const TileRanges& slices, const int32_t* win, int win_doubles, double* partials,
                   int pstride, int grid, CgState* st, double tol, int first, int check, int k,
                   hipStream_t stream, const RedCtl& rc = RedCtl());
// ---- materialized-p single-reduction iteration (csrc/gpu/cg_split.hip) ----
// The irregular-sparsity path: U (elementwise x / r / p_k update of the owned rows, same scalars
// as cg_fused1) then S (SpMV gathering the stored p_k only + the 4 partials, in-kernel reduction).
// final_mode U: r_m and x_m only + the r.r partials (then cg_reduce_f1 modes 1 / 2).
void cg_split_update(double* x, double* r, const double* Ap, double* p_own, int64_t n, CgState* st, double tol,
                     int first, int check, int final_mode, double* partials, int pstride, int grid,
                     hipStream_t stream);
// fmt: 0 CSR thread-per-row (param U), 5 CSR-vector (param G lanes per row), 1 SELL-64, 3 SELL-64/d16,
// 4 SELL-64/c8, 6 SELL-64/aligned.  part (fmt 6 with S.local_slots): 0 every slot; 1 the local-column
// slots only, Ap := that partial sum (no partials, no reduction); 2 the other slots, Ap += them, then
// the epilogue / partials / reduction of part 0
template <typename IdxT>
void cg_split_spmv(int fmt, int param, const CsrDev<IdxT>& A, const SellDev& S, const double* p_ext, const double* r,
                   double* Ap, int64_t own_off, const TileRanges& tr, double* partials, int pstride, int grid,
                   CgState* st, double tol, int first, int check, hipStream_t stream, const RedCtl& rc = RedCtl(),
                   int part = 0);
// ---- L2-segment COO tiles (csrc/gpu/cg_tiles.hip): the irregular-sparsity SpMV ----
// Row blocks of kTileB rows x column segments of 2^seg_shift doubles; tile (b, g) holds the block's
// nonzeros in segment g as (row in block << 22 | column in segment) + value.  Every wave owns one
// block at a time (sums in LDS) and all waves sweep the segments together (paced per segment), so
// the gathers of p hit the L2.
constexpr int kTileB = 1024;
constexpr int kTileMaxSegments = 8192;  // LDS counters of the build kernels (32 KiB)
constexpr int kTilePaceCnt = 8 * 64;     // pacing arrival counters: 8 groups, 256 B apart
constexpr int kTilePaceWords = kTilePaceCnt + 8 * 8 * 64;  // + per group 8 replicas of its step flag, 256 B apart
struct TilesGeometry {
  int tb = kTileB;  // rows per block (kTileB or kTileB5)
  int64_t nblocks = 0;
  int G = 0;
  int seg_shift = 18;
};
struct TilesDev {
  const int64_t* tptr = nullptr;  // nblocks * G + 1
  const uint32_t* idx = nullptr;
  const double* vals = nullptr;
  int64_t n_rows = 0, nblocks = 0;
  int G = 0, seg_shift = 18;
  int tb = kTileB;           // rows per block
  unsigned* pace = nullptr;  // kTilePaceWords, zeroed by the launchers; nullptr = unpaced
  int64_t ext_len = 0;       // length of p (the last segment may be short)
  int g_lo = 0, g_hi = 0;    // the segments inside this rank's own block of p (all-gather overlap, part 1 / 2)
  int tu = 10;               // entries per lane in flight, 8 or 10 (tiles_tu)
  int ww = 4;                // waves per workgroup: 4 (four workgroups per CU) or 16 (one per CU; PassForm::tile_waves)
};
// entries per lane in flight for tiles of mean size m: 8 or 10, whichever fills the batches of 64 x TU
// entries better (config 5's ~1790-entry tiles: 3 batches of 640 rather than 4 of 512; the 201 GB
// share's ~3580: 7 of 512 rather than 6 of 640)
inline int tiles_tu(double m) {
  auto fill = [m](int tu) {
    const double b = 64.0 * tu;
    return m <= 0.0 ? 1.0 : m / (std::ceil(m / b) * b);
  };
  return fill(10) > fill(8) ? 10 : 8;
}
TilesGeometry tiles_geometry(int64_t n_rows, int64_t ext_len, int seg_shift);
int tiles_grid(int ncu, int ww = 4);  // workgroups of the SpMV on ncu CUs: the resident count (pacing waits on every
                                      // workgroup); ww = waves per workgroup (4 or 16)
// count (fill = false: tptr[b * G + g + 1] = tile sizes; scan them, tptr[0] = 0) then fill
struct TilesOut {
  int64_t* tptr = nullptr;
  uint32_t* idx = nullptr;
  double* vals = nullptr;
};
void tiles_build_gen(const ProblemSpec& s, int64_t row_begin, int64_t n, int64_t col_lo, int64_t pad,
                     const int64_t* rp64, const TilesGeometry& geo, const TilesOut& out, bool fill, hipStream_t st);
void tiles_build_csr(const int64_t* rp, const int32_t* cols, const double* cvals, int64_t n, const TilesGeometry& geo,
                     const TilesOut& out, bool fill, hipStream_t st);
// the split pass's SpMV on tiles (same contract as cg_split_spmv part 0)
// part: 0 = every segment; 1 / 2 = the own-block segments [g_lo, g_hi) / the others (all-gather overlap)
void cg_split_spmv_tiles(const TilesDev& T, const double* p_ext, const double* r, double* Ap, int64_t own_off,
                         double* partials, int pstride, int grid, CgState* st, double tol, int first, int check,
                         hipStream_t stream, const RedCtl& rc = RedCtl(), int part = 0);
void spmv_tiles(const TilesDev& T, const double* x_ext, double* y, int grid, hipStream_t stream);

// ---- pipelined CG (csrc/gpu/cg_pipe.hip), recurrence = 2 ----
// owned-row pointers: x, z, q owned vectors; r, w, p, s the owned parts of ext-layout vectors
struct PipeVectors {
  double *x, *r, *w, *p, *s, *z;
  const double* q;
};
// U_i: the vector recurrences with alpha_i / beta_i from CgState (red = the all-reduced {gamma_i, delta_i}),
// the latch on gamma_i (rc.check), and {gamma_{i+1}, delta_{i+1}} reduced in the kernel (rc over `grid`)
void cg_pipe_update(const PipeVectors& v, int64_t n, double* partials, int pstride, int grid, CgState* st, double tol,
                    hipStream_t stream, const RedCtl& rc);
// local {r.r, w.r} -> CgState::red (mode 0: the initial state, mode 1: after a residual replacement)
void cg_pipe_dots(const double* r, const double* w, int64_t n, double* partials, int pstride, int grid, CgState* st,
                  int mode, hipStream_t stream);
void cg_pipe_final(CgState* st, double tol, hipStream_t stream);  // latch after the last update
void sub_vec(const double* b, const double* y, double* out, int64_t n, hipStream_t stream);  // out = b - y

// out[i] = {a[i], 0} (seeds the interleaved {r, Ap} layout)
void pack_pairs(const double* a, double2* out, int64_t n, hipStream_t stream);
// modes: 0 = after a fused pass (conv check on the previous rr, sum 4 partials),
//        1 = after the final pass (sum rr only), 2 = latch after the final all-reduce
// `first`: after pass 0 (a_prev := 0)
void cg_reduce_f1(const double* partials, int pstride, int np, CgState* st, int mode, int check, int first,
                  double tol, hipStream_t stream);

// ---- unfused ops (ops API / tests) ----
template <typename IdxT>
void spmv_csr(const CsrDev<IdxT>& A, const double* x, double* y, hipStream_t stream, int variant = 0);
void spmv_sell(const SellDev& A, const double* x, double* y, hipStream_t stream);
void axpy(double alpha, const double* x, double* y, int64_t n, hipStream_t stream);  // y += a x
void xpby(const double* x, double beta, double* y, int64_t n, hipStream_t stream);   // y = x + b y

int grid_for(int64_t work_items, int block, int blocks_per_cu);

// ---- IPC all-reduce (csrc/gpu/ipc_allreduce.hip): the CG scalars through peer-mapped mailboxes ----
constexpr int kIpcArMax = 8;      // doubles per all-reduce
constexpr int kIpcMaxRanks = 16;
struct IpcMailboxes {
  double* slots[kIpcMaxRanks] = {};               // rank q's mailbox as mapped here: [2 parities][world][kIpcArMax]
  unsigned long long* flags[kIpcMaxRanks] = {};   // rank q's arrival flags [world], + its call counter [world]
  unsigned long long* err = nullptr;              // host-mapped: 1 when a peer did not arrive within the budget
  int rank = 0, world = 1;
};
// in-place sum of `count` doubles over the ranks, in rank order (the same bits everywhere); one wave
void ipc_allreduce(double* buf, int count, const IpcMailboxes& mb, double budget_seconds, hipStream_t stream);

// ---- probes (csrc/gpu/probe_kernels.hip) ----
// `blocks` workgroups of 256 threads spinning for `microseconds` on the realtime clock; fat: ~270
// VGPRs per wave live (RCCL's kernels' footprint), else a handful.  out: one double per block or null
void spin(double* out, double microseconds, bool fat, int blocks, hipStream_t stream, int* where = nullptr);
// the same with ~120 VGPRs per wave (4 blocks of 256 per CU fill a CU's register file)
void hog(double* out, double microseconds, int blocks, hipStream_t stream, int* where = nullptr);

}  // namespace kern
}  // namespace mcg
