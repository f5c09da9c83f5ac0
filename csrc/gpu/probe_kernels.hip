// Device-side delay / register-pressure probes.
//
//  * k_spin<NREGS>: a workgroup that spins for a given time on the 100 MHz realtime clock.  The
//    fat form keeps ~270 VGPRs per wave live (like RCCL's p2p / collective kernels, 261-280 VGPRs,
//    profiles/r2_corun_probe.md), the thin form a handful: launched next to the resident CG pass
//    they separate "an RCCL kernel cannot start because the register file is full" from
//    "it cannot start for another reason" (bench/corun_probe.py --control).  The hog form (~120
//    VGPRs, 4 blocks per CU) stands in for the resident pass on a CU-masked stream
//    (bench/cumask_probe.py): does a fat wave start on the CUs the mask leaves free?
//  * DelayComm (comm.hpp) enqueues the thin spin as its "collective": a communicator whose
//    all-reduce and halo cost a fixed device-side latency and move nothing (latency-tolerance tests).
// The clock is read with s_memrealtime (a scalar READ of the realtime counter; nothing is written
// through the scalar cache).
#include <hip/hip_runtime.h>

#include "mcg/check.hpp"
#include "mcg/kernels.hpp"

namespace mcg {
namespace kern {
namespace {

constexpr int kFatRegs = 134;  // doubles per lane kept live -> ~270 VGPRs (RCCL: 261-280)
constexpr int kHogRegs = 56;   // -> ~120 VGPRs: 4 waves per SIMD fill the file, like the carry pass

// NREGS doubles per lane live while spinning (0: thin); `where` (nullable) gets each block's
// __smid() (XCC / SE / CU of the workgroup), so a probe can see which CUs a grid landed on
template <int NREGS>
__global__ __launch_bounds__(256) void k_spin(double* __restrict__ out, int* __restrict__ where, long long ticks) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  double acc = 0.0;
  if constexpr (NREGS > 0) {
    double v[NREGS];
#pragma unroll
    for (int i = 0; i < NREGS; ++i) v[i] = (double)(threadIdx.x + i);
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
#pragma unroll
      for (int i = 0; i < NREGS; ++i) v[i] = fma(v[i], 1.0000000001, 1e-12);
    }
#pragma unroll
    for (int i = 0; i < NREGS; ++i) acc += v[i];
  } else {
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) acc = fma(acc, 0.5, 1.0);
  }
  if (out != nullptr && threadIdx.x == 0) out[blockIdx.x] = acc;
  if (where != nullptr && threadIdx.x == 0) where[blockIdx.x] = (int)__smid();
}

}  // namespace

void spin(double* out, double microseconds, bool fat, int blocks, hipStream_t stream, int* where) {
  const long long ticks = (long long)(microseconds * 100.0);  // 100 MHz realtime clock
  if (fat) hipLaunchKernelGGL(k_spin<kFatRegs>, dim3(blocks), dim3(256), 0, stream, out, where, ticks);
  else hipLaunchKernelGGL(k_spin<0>, dim3(blocks), dim3(256), 0, stream, out, where, ticks);
  MCG_HIP(hipGetLastError(), "kernel launch failed(spin)");
}

void hog(double* out, double microseconds, int blocks, hipStream_t stream, int* where) {
  const long long ticks = (long long)(microseconds * 100.0);
  hipLaunchKernelGGL(k_spin<kHogRegs>, dim3(blocks), dim3(256), 0, stream, out, where, ticks);
  MCG_HIP(hipGetLastError(), "kernel launch failed(hog)");
}

}  // namespace kern
}  // namespace mcg
