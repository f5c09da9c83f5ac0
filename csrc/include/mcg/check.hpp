// Error handling for the mcg runtime.
//
// The reference routes every failed CUDA/cuBLAS/cuSPARSE call through one
// CLEANUP(msg) macro that prints a short message to stdout, frees everything and
// exits 1 (reference CUDACG.cu:10-33, 31 call sites, messages listed in SURVEY.md
// §5.3).  Here a failure throws mcg::Error carrying the same short "what" text
// (e.g. "device malloc failed(x)") plus a detail string (the HIP/RCCL error);
// RAII destructors do the cleanup and the CLI prints what() to stdout and exits 1.
#pragma once

#include <stdexcept>
#include <string>

namespace mcg {

class Error : public std::runtime_error {
 public:
  Error(const std::string& msg, const std::string& detail = std::string())
      : std::runtime_error(msg), detail_(detail) {}
  const std::string& detail() const { return detail_; }

 private:
  std::string detail_;
};

[[noreturn]] inline void fail(const std::string& msg, const std::string& detail = std::string()) {
  throw Error(msg, detail);
}

}  // namespace mcg

// MCG_HIP(expr, "message"): throw mcg::Error("message", hipGetErrorString) on failure.
#define MCG_HIP(expr, msg)                                                           \
  do {                                                                               \
    hipError_t mcg_e_ = (expr);                                                      \
    if (mcg_e_ != hipSuccess)                                                        \
      ::mcg::fail((msg), std::string(#expr) + ": " + hipGetErrorString(mcg_e_) +     \
                             " (" __FILE__ ":" + std::to_string(__LINE__) + ")");    \
  } while (0)

#define MCG_RCCL(expr, msg)                                                          \
  do {                                                                               \
    ncclResult_t mcg_r_ = (expr);                                                    \
    if (mcg_r_ != ncclSuccess)                                                       \
      ::mcg::fail((msg), std::string(#expr) + ": " + ncclGetErrorString(mcg_r_) +    \
                             " (" __FILE__ ":" + std::to_string(__LINE__) + ")");    \
  } while (0)

#define MCG_CHECK(cond, msg)                                                         \
  do {                                                                               \
    if (!(cond)) ::mcg::fail((msg), std::string("check failed: " #cond " (") +       \
                                        __FILE__ ":" + std::to_string(__LINE__) + ")"); \
  } while (0)
