// Repro: stream memory operations (hipStreamWaitValue64 / hipStreamWriteValue64) and copy-engine copies
// (hipMemcpyDeviceToDeviceNoCU) eager vs captured in a hipGraph -- the ordering PeerHaloComm's
// copy-engine halo relies on (csrc/gpu/peer_halo.cpp).  VERDICT r4 item 6 / weak 6.
//
// A producer stream fills `src` with the round's value v after a ~200 us spin and then writes v into
// `flag`; the consumer waits for flag == v, copies src -> dst on a copy engine, counts the entries of
// dst that are not v and writes v into `done`, which the producer waits for before the next fill (the
// ready / done pair of peer_halo.cpp).  Modes:
//   eager    the consumer's operations enqueued per round
//   graph    the consumer's two rounds (v = 1, 2) captured once into a graph and replayed per pair
//   graphw   as graph, the producer's flag write captured too (its own graph)
//   fork     graph, the consumer's copy on a branch forked / joined by events (CopyFan's capture form;
//            r4 saw a SIGSEGV there: a SIGSEGV handler prints the host backtrace)
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

  auto consumer = [&](hipStream_t s, uint64_t v, bool forked) {
    CK(hipStreamWaitValue64(s, flag, v, hipStreamWaitValueEq, ~0ull));
    if (forked) {
      CK(hipEventRecord(fork, s));
      CK(hipStreamWaitEvent(C, fork, 0));
      CK(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDeviceNoCU, C));
      CK(hipEventRecord(join, C));
      CK(hipStreamWaitEvent(s, join, 0));
    } else {
      CK(hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDeviceNoCU, s));
    }
    hipLaunchKernelGGL(k_check, dim3(64), dim3(256), 0, s, dst, n, (double)v, bad);
    CK(hipStreamWriteValue64(s, done, v, 0));  // the producer may overwrite src now
  };
  const char* modes[] = {"eager", "graph", "graphw", "fork"};
  const std::string only = argc > 2 ? argv[2] : "";
  for (const char* mode : modes) {
    const std::string m = mode;
    if (!only.empty() && m != only) continue;
    g_mode = mode;
    alarm(20);  // a mode that hangs ends the program with a line saying so
    CK(hipMemset(flag, 0, sizeof(uint64_t)));
    CK(hipMemset(done, 0, sizeof(uint64_t)));
    CK(hipMemset(bad, 0, sizeof(unsigned long long)));
    CK(hipMemset(src, 0, n * sizeof(double)));
    CK(hipDeviceSynchronize());
    hipGraphExec_t gb = nullptr, gw = nullptr;
    hipGraph_t g = nullptr;
    if (m != "eager") {  // the consumer's pair (v = 1, 2)
      CK(hipStreamBeginCapture(B, hipStreamCaptureModeThreadLocal));
      consumer(B, 1, m == "fork");
      consumer(B, 2, m == "fork");
      CK(hipStreamEndCapture(B, &g));
      CK(hipGraphInstantiate(&gb, g, nullptr, nullptr, 0));
    }
    if (m == "graphw") {  // the producer's flag writes captured too (the kernels stay eager)
      hipGraph_t g2 = nullptr;
      CK(hipStreamBeginCapture(A, hipStreamCaptureModeThreadLocal));
      CK(hipStreamWriteValue64(A, flag, 1, 0));
      CK(hipStreamEndCapture(A, &g2));
      CK(hipGraphInstantiate(&gw, g2, nullptr, nullptr, 0));
    }
    double launch_us = 0.0;
    for (int r = 0; r < rounds; r += 2) {
      // the producer's pair first (its second fill waits on the device for the consumer's done = 1), so
      // a consumer launch that blocked the host until its waits are met could not deadlock
      for (uint64_t v = 1; v <= 2; ++v) {
        if (v == 2) CK(hipStreamWaitValue64(A, done, 1, hipStreamWaitValueEq, ~0ull));
        hipLaunchKernelGGL(k_fill, dim3(64), dim3(256), 0, A, src, n, (double)v, spin);
        if (m == "graphw" && v == 1) CK(hipGraphLaunch(gw, A));
        else CK(hipStreamWriteValue64(A, flag, v, 0));
      }
      const auto t0 = std::chrono::steady_clock::now();
      if (m == "eager") {
        consumer(B, 1, false);
        consumer(B, 2, false);
      } else {
        CK(hipGraphLaunch(gb, B));
      }
      launch_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      CK(hipStreamSynchronize(A));
      CK(hipStreamSynchronize(B));
      // reset the flags for the next pair (the waits are for equality)
      CK(hipMemset(flag, 0, sizeof(uint64_t)));
      CK(hipMemset(done, 0, sizeof(uint64_t)));
      CK(hipDeviceSynchronize());
    }
    unsigned long long h = 0;
    CK(hipMemcpy(&h, bad, sizeof(h), hipMemcpyDeviceToHost));
    std::printf("{\"mode\": \"%s\", \"rounds\": %d, \"mismatches\": %llu, \"ordered\": %s, \"host_launch_us\": %.1f}\n",
                mode, rounds, h, h == 0 ? "true" : "false", launch_us / (rounds / 2));
    std::fflush(stdout);
    if (gb) CK(hipGraphExecDestroy(gb));
    if (gw) CK(hipGraphExecDestroy(gw));
  }
  return 0;
}
