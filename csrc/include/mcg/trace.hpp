// Tracing: roctx ranges around the solver phases (setup, reset, each enqueued
// iteration, halo, all-reduce, solve), visible in `rocprofv3 --marker-trace`
// timelines.  The reference has only a dead gettimeofday helper
// (cpuSecond, CUDACG.cu:35-39).  roctx is loaded with dlopen on first use when
// MCG_TRACE=1 (or MCG_TRACE=roctx), so the runtime has no hard dependency on it
// and ranges cost one branch when tracing is off.
#pragma once

namespace mcg {
namespace trace {

bool enabled();
void push(const char* name);
void pop();
void mark(const char* name);

class Range {
 public:
  explicit Range(const char* name) : on_(enabled()) {
    if (on_) push(name);
  }
  ~Range() {
    if (on_) pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_;
};

}  // namespace trace
}  // namespace mcg
