// Repro: stream memory operations (hipStreamWaitValue64 / hipStreamWriteValue64) and copy-engine copies
// (hipMemcpyDeviceToDeviceNoCU) eager vs captured in a hipGraph -- the ordering PeerHaloComm's
// copy-engine halo relies on (csrc/gpu/peer_halo.cpp).  VERDICT r4 item 6 / weak 6.
//
// A producer stream fills `src` with the round's value v after a ~200 us spin and then writes v into
// `flag`; the consumer waits for flag == v, copies src -> dst on a copy engine, counts the entries of
// dst that are not v and writes v into `done`, which the producer waits for before the next fill (the
// ready / done pair of peer_halo.cpp).  Modes:
//   eager    the consumer's operations enqueued per round
//   graph    the consumer's four operations of each round captured (one graph per round value)
//   fork     graph, the consumer's copy on a branch forked / joined by events (CopyFan's capture form;
//            r4 saw a SIGSEGV there: a SIGSEGV handler prints the host backtrace)
//   g_wait / g_copy / g_check / g_write / g_copy_check   only those operations captured, the rest eager
//            (which node kind breaks the ordering)
// Prints one JSON line per mode: rounds, mismatching entries, whether the consumer ever ran ahead.
//   make build/streamop_capture && build/streamop_capture [ROUNDS [MODE]]
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("{\"error\": \"%s\", \"at\": \"%s:%d\"}\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(2);                                                                    \
    }                                                                                  \
  } while (0)

__global__ void k_fill(double* src, int n, double v, long long spin) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(8);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) src[i] = v;
}
__global__ void k_check(const double* dst, int n, double v, unsigned long long* bad) {
  unsigned long long b = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) b += dst[i] != v;
  if (b) atomicAdd(bad, b);
}

static const char* g_mode = "";
static void on_alarm(int) {
  std::printf("{\"mode\": \"%s\", \"hung\": true}\n", g_mode);
  std::fflush(stdout);
  std::_Exit(3);
}

static void on_segv(int sig) {
  void* bt[64];
  const int n = backtrace(bt, 64);
  std::fprintf(stderr, "signal %d: host backtrace\n", sig);
  backtrace_symbols_fd(bt, n, 2);
  std::_Exit(128 + sig);
}

int main(int argc, char** argv) {
  signal(SIGSEGV, on_segv);
  signal(SIGALRM, on_alarm);
  const int n = 16384, rounds = argc > 1 ? std::atoi(argv[1]) : 20;
  int rate = 0;
  CK(hipDeviceGetAttribute(&rate, hipDeviceAttributeWallClockRate, 0));
  const long long spin = (long long)rate * 200 / 1000;  // ~200 us in wall-clock ticks (rate in kHz)
  double *src, *dst;
  uint64_t *flag, *done;
  unsigned long long* bad;
  CK(hipMalloc(&src, n * sizeof(double)));
  CK(hipMalloc(&dst, n * sizeof(double)));
  CK(hipMalloc(&flag, sizeof(uint64_t)));
  CK(hipMalloc(&done, sizeof(uint64_t)));
  CK(hipMalloc(&bad, sizeof(unsigned long long)));
  hipStream_t A, B, C;
  CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&C, hipStreamNonBlocking));
  hipEvent_t fork, join;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));

  // the consumer's four operations for round value v; `ops` selects which (bit 0 wait, 1 copy, 2 check,
  // 3 done write)
  auto consumer = [&](hipStream_t s, uint64_t v, unsigned ops, bool forked) {
    if (ops & 1) CK(hipStreamWaitValue64(s, flag, v, hipStreamWaitValueEq, ~0ull));
    if (ops & 2) {
      if (forked) {
        CK(hipEventRecord(fork, s));
        CK(hipStreamWaitEvent(C, fork, 0));
        CK(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDeviceNoCU, C));
        CK(hipEventRecord(join, C));
        CK(hipStreamWaitEvent(s, join, 0));
      } else {
        CK(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDeviceNoCU, s));
      }
    }
    if (ops & 4) hipLaunchKernelGGL(k_check, dim3(64), dim3(256), 0, s, dst, n, (double)v, bad);
    if (ops & 8) CK(hipStreamWriteValue64(s, done, v, 0));  // the producer may overwrite src now
  };
  // mode -> the operations captured (one graph per round value; the others stay eager, in order)
  struct Mode { const char* name; unsigned cap; bool forked; };
  const Mode modes[] = {{"eager", 0, false}, {"graph", 15, false}, {"fork", 15, true}, {"g_wait", 1, false},
                        {"g_copy", 2, false}, {"g_check", 4, false}, {"g_write", 8, false},
                        {"g_copy_check", 6, false}};
  const std::string only = argc > 2 ? argv[2] : "";
  for (const Mode& md : modes) {
    const std::string m = md.name;
    if (!only.empty() && m != only) continue;
    g_mode = md.name;
    alarm(20);  // a mode that hangs ends the program with a line saying so
    CK(hipMemset(flag, 0, sizeof(uint64_t)));
    CK(hipMemset(done, 0, sizeof(uint64_t)));
    CK(hipMemset(bad, 0, sizeof(unsigned long long)));
    CK(hipMemset(src, 0, n * sizeof(double)));
    CK(hipDeviceSynchronize());
    hipGraphExec_t gx[3] = {nullptr, nullptr, nullptr};
    if (md.cap) {
      for (uint64_t v = 1; v <= 2; ++v) {
        hipGraph_t g = nullptr;
        CK(hipStreamBeginCapture(B, hipStreamCaptureModeThreadLocal));
        consumer(B, v, md.cap, md.forked);
        CK(hipStreamEndCapture(B, &g));
        CK(hipGraphInstantiate(&gx[v], g, nullptr, nullptr, 0));
      }
    }
    const unsigned low = md.cap & (~md.cap + 1);  // first captured op
    const unsigned pre = md.cap ? low - 1 : 15, post = md.cap ? (15 & ~(pre | md.cap)) : 0;
    double launch_us = 0.0;
    for (int r = 0; r < rounds; r += 2) {
      // the producer's pair first (its second fill waits on the device for the consumer's done = 1), so
      // a consumer launch that blocked the host until its waits are met could not deadlock
      for (uint64_t v = 1; v <= 2; ++v) {
        if (v == 2) CK(hipStreamWaitValue64(A, done, 1, hipStreamWaitValueEq, ~0ull));
        hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, A, src, n, (double)v, spin);
        CK(hipStreamWriteValue64(A, flag, v, 0));
      }
      const auto t0 = std::chrono::steady_clock::now();
      for (uint64_t v = 1; v <= 2; ++v) {
        consumer(B, v, pre, false);
        if (md.cap) CK(hipGraphLaunch(gx[v], B));
        consumer(B, v, post, false);
      }
      launch_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      CK(hipStreamSynchronize(A));
      CK(hipStreamSynchronize(B));
      // reset the flags for the next pair (the waits are for equality)
      CK(hipMemset(flag, 0, sizeof(uint64_t)));
      CK(hipMemset(done, 0, sizeof(uint64_t)));
      CK(hipDeviceSynchronize());
    }
    alarm(0);
    unsigned long long h = 0;
    CK(hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost));
    std::printf("{\"mode\": \"%s\", \"captured_ops\": %u, \"rounds\": %d, \"mismatches\": %llu, \"ordered\": %s, \"host_launch_us\": %.1f}\n",
                md.name, md.cap, rounds, h, h == 0 ? "true" : "false", launch_us / (rounds / 2));
    std::fflush(stdout);
    for (hipGraphExec_t e : gx)
      if (e) CK(hipGraphExecDestroy(e));
  }
  return 0;
}
