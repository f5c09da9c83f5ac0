// Persistent-pass probe: would keeping the CG pass's blocks resident across
// iterations -- a device-wide barrier between passes instead of a kernel boundary -- shorten a short
// pass (4096^2 on one GPU, a P = 8 rank's share of 512^3)?
//
// Stand-in pass: a streaming sweep out = in + c * in_shifted over n doubles (16-B lanes, each block a
// contiguous chunk, the shifted read crossing into the NEXT block's chunk, so a pass reads what
// another workgroup wrote in the pass before -- as the carries' run ends and slice edges do), 32 B
// moved per row like the lean three-term carry's p stream.  Two forms over the same passes:
//   graph:      one kernel per pass, the passes captured in one hipGraph and replayed (the solver's
//               form: a kernel boundary between passes);
//   persistent: ONE launch of the same grid (every block resident: the grid is clamped to the
//               occupancy query) looping over the passes with an XCD-hierarchical grid barrier
//               (MI355X_MICROARCH.md "barrier-xcd": per-XCC counter, the XCC's last arriver adds to a
//               top counter, the top's last arriver bumps every XCC's generation; agent release before
//               arriving, acquire after) between them.  Blocks register their XCC (s_getreg XCC_ID)
//               at the start behind a one-counter barrier, so no dispatch-placement assumption is made.
// Every wait is bounded by the wall clock (1 s): a barrier that never completes sets an error word and
// every block leaves the loop, so the grid always drains.
//
// Prints one JSON line per (rows, grid): us per pass for both forms, the persistent form's barrier
// alone (passes of zero rows), and the graph form's kernel boundary alone (empty passes).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 bench/persist_probe.hip -o build/persist_probe
//   build/persist_probe [rows ...]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));       \
      std::exit(1);                                                                                \
    }                                                                                              \
  } while (0)

namespace {

constexpr int kBS = 256;
constexpr int kXcc = 8;
constexpr int kPad = 32;  // unsigned words per cache line (128 B): one counter per line

struct Bar {
  unsigned reg_cnt[kPad];        // start-up: blocks registered (one-counter barrier)
  unsigned members[kXcc * kPad]; // blocks per XCC
  unsigned cnt[kXcc * kPad];     // arrivals per XCC (reset by its last arriver)
  unsigned top[kPad];            // XCCs arrived (reset by the last)
  unsigned gen[kXcc * kPad];     // per-XCC generation (bumped by the top's last arriver)
  unsigned err[kPad];            // a wait that timed out
};

typedef __attribute__((address_space(1))) unsigned g_u32;

__device__ __forceinline__ unsigned ld_sc1(const unsigned* p) {
  return __hip_atomic_load((g_u32*)const_cast<unsigned*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(unsigned* p, unsigned v) {
  __hip_atomic_store((g_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned add_agent(unsigned* p, unsigned v) {
  return __hip_atomic_fetch_add((g_u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int xcc_id() {
  return (int)(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (2 << 11)) & 7);  // HW_REG_XCC_ID, bits [2:0]
}

// poll *p until it differs from `old` (or the budget runs out: error word, false)
__device__ bool wait_change(Bar* b, const unsigned* p, unsigned old, long long budget) {
  const long long t0 = wall_clock64();
  while (ld_sc1(p) == old) {
    if (ld_sc1(b->err) != 0u) return false;
    if (wall_clock64() - t0 > budget) {
      st_sc1(b->err, 1u);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

// one-counter barrier over the grid at start-up (registers each block's XCC)
__device__ bool register_xcc(Bar* b, int& xcc, long long budget) {
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    xcc = xcc_id();
    add_agent(&b->members[xcc * kPad], 1u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // counted before this block counts as arrived
    const unsigned a = add_agent(b->reg_cnt, 1u);
    bool ok = true;
    if (a + 1 < gridDim.x) {
      const long long t0 = wall_clock64();
      while (ld_sc1(b->reg_cnt) < gridDim.x) {
        if (ld_sc1(b->err) != 0u || wall_clock64() - t0 > budget) {
          st_sc1(b->err, 1u);
          ok = false;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    s_ok = ok;
  }
  __syncthreads();
  xcc = __shfl(xcc, 0, 64);
  return s_ok != 0;
}

// XCD-hierarchical barrier (MI355X_MICROARCH.md barrier-xcd)
__device__ bool grid_barrier(Bar* b, int xcc, long long budget) {
  __shared__ int s_ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this block's pass stores before its arrival
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned* gx = &b->gen[xcc * kPad];
    const unsigned g = ld_sc1(gx);
    const unsigned m = ld_sc1(&b->members[xcc * kPad]);
    bool ok = true;
    if (add_agent(&b->cnt[xcc * kPad], 1u) + 1 == m) {  // the XCC's last arriver
      st_sc1(&b->cnt[xcc * kPad], 0u);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // reset before this XCC counts as arrived
      int nx = 0;
      for (int x = 0; x < kXcc; ++x) nx += ld_sc1(&b->members[x * kPad]) > 0u ? 1 : 0;
      if ((int)add_agent(b->top, 1u) + 1 == nx) {  // the last XCC: release everyone
        st_sc1(b->top, 0u);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (int x = 0; x < kXcc; ++x) st_sc1(&b->gen[x * kPad], g + 1u);
      } else {
        ok = wait_change(b, gx, g, budget);
      }
    } else {
      ok = wait_change(b, gx, g, budget);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the other blocks' pass stores visible here
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// one pass over this block's chunk: out[i] = in[i] + c * in[i + shift] (shift: half a chunk, so the
// second half of every chunk reads the next block's chunk)
__device__ __forceinline__ void pass(const double2* __restrict__ in, double2* __restrict__ out, long n2, long chunk,
                                     long shift, double c) {
  const long b0 = (long)blockIdx.x * chunk, b1 = b0 + chunk < n2 ? b0 + chunk : n2;
  for (long i = b0 + threadIdx.x; i < b1; i += kBS) {
    long j = i + shift;
    if (j >= n2) j -= n2;
    const double2 a = in[i], s = in[j];
    out[i] = make_double2(fma(c, s.x, a.x), fma(c, s.y, a.y));
  }
}

__global__ __launch_bounds__(kBS) void k_pass(const double2* in, double2* out, long n2, long chunk, long shift) {
  pass(in, out, n2, chunk, shift, 0.5);
}

__global__ __launch_bounds__(kBS) void k_persist(double2* a, double2* b, long n2, long chunk, long shift, int passes,
                                                 Bar* bar, long long budget) {
  int xcc = 0;
  if (!register_xcc(bar, xcc, budget)) return;
  for (int k = 0; k < passes; ++k) {
    pass((k & 1) ? b : a, (k & 1) ? a : b, n2, chunk, shift, 0.5);
    if (!grid_barrier(bar, xcc, budget)) return;
  }
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<long> rows_list;
  for (int i = 1; i < argc; ++i) rows_list.push_back(std::atol(argv[i]));
  if (rows_list.empty()) rows_list = {0, 1L << 22, 16777216L, 33554432L};  // 0: the barrier / boundary alone
  int dev = 0, ncu = 0, khz = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
  int occ = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_persist, kBS, 0));
  const long long budget = (long long)khz * 1000;  // 1 s of wall clock
  const long max_rows = 33554432L;
  double2 *a = nullptr, *b = nullptr;
  CK(hipMalloc(&a, max_rows * 16));
  CK(hipMalloc(&b, max_rows * 16));
  CK(hipMemset(a, 0, max_rows * 16));
  CK(hipMemset(b, 0, max_rows * 16));
  Bar* bar = nullptr;
  CK(hipMalloc(&bar, sizeof(Bar)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int passes = 64;
  for (int bpc : {1, 2, 4, 6}) {
    if (bpc > occ) continue;
    const int grid = ncu * bpc;
    for (long rows : rows_list) {
      // rows doubles of each vector; 16-B lanes: n2 pairs
      const long n2 = rows > 0 ? rows / 2 : 0;
      const long chunk = n2 > 0 ? (n2 + grid - 1) / grid : 0;
      const long shift = chunk / 2;
      // graph form
      hipGraph_t g;
      hipGraphExec_t ge;
      CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int k = 0; k < passes; ++k)
        hipLaunchKernelGGL(k_pass, dim3(grid), dim3(kBS), 0, s, (k & 1) ? b : a, (k & 1) ? a : b, n2, chunk, shift);
      CK(hipStreamEndCapture(s, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipGraphLaunch(ge, s));  // warm
      CK(hipEventRecord(e0, s));
      for (int r = 0; r < 4; ++r) CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms_g = 0.f;
      CK(hipEventElapsedTime(&ms_g, e0, e1));
      CK(hipGraphExecDestroy(ge));
      CK(hipGraphDestroy(g));
      // persistent form (fresh barrier state per launch)
      float ms_p = 0.f;
      unsigned err = 0;
      for (int r = 0; r < 5; ++r) {
        CK(hipMemsetAsync(bar, 0, sizeof(Bar), s));
        CK(hipEventRecord(e0, s));
        hipLaunchKernelGGL(k_persist, dim3(grid), dim3(kBS), 0, s, a, b, n2, chunk, shift, passes, bar, budget);
        CK(hipGetLastError());
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned e = 0;
        CK(hipMemcpy(&e, bar->err, sizeof(unsigned), hipMemcpyDeviceToHost));
        err |= e;
        if (r > 0) ms_p += ms;  // the first launch warms
      }
      const double us_g = 1e3 * ms_g / (4.0 * passes), us_p = 1e3 * ms_p / (4.0 * passes);
      const double gbytes = 16.0 * (double)rows / 1e9;  // per row 8 B read + 8 B written (the shifted re-read aside)
      std::printf("{\"rows\": %ld, \"grid\": %d, \"blocks_per_cu\": %d, \"occupancy\": %d, \"us_per_pass_graph\": %.3f, "
                  "\"us_per_pass_persistent\": %.3f, \"persistent_minus_graph_us\": %.3f, \"graph_tb_s\": %.3f, "
                  "\"barrier_error\": %u}\n",
                  rows, grid, bpc, occ, us_g, us_p, us_p - us_g, us_g > 0 ? gbytes * 1e3 / us_g : 0.0,
                  err);
      std::fflush(stdout);
      if (err) return 2;  // a barrier that timed out: stop here
    }
  }
  return 0;
}
