#include "mcg/trace.hpp"

#include <dlfcn.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

namespace mcg {
namespace trace {

namespace {
using PushFn = int (*)(const char*);
using PopFn = int (*)();
using MarkFn = void (*)(const char*);

struct Roctx {
  bool on = false;
  PushFn push = nullptr;
  PopFn pop = nullptr;
  MarkFn mark = nullptr;
};

const Roctx& roctx() {
  static Roctx r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* e = std::getenv("MCG_TRACE");
    if (!e || !(std::strcmp(e, "1") == 0 || std::strcmp(e, "roctx") == 0)) return;
    // rocprofiler-sdk's roctx (what rocprofv3 --marker-trace intercepts), then legacy roctracer roctx
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    r.push = reinterpret_cast<PushFn>(dlsym(h, "roctxRangePushA"));
    r.pop = reinterpret_cast<PopFn>(dlsym(h, "roctxRangePop"));
    r.mark = reinterpret_cast<MarkFn>(dlsym(h, "roctxMarkA"));
    r.on = r.push && r.pop;
  });
  return r;
}
}  // namespace

bool enabled() { return roctx().on; }
void push(const char* name) {
  if (roctx().on) roctx().push(name);
}
void pop() {
  if (roctx().on) roctx().pop();
}
void mark(const char* name) {
  if (roctx().on && roctx().mark) roctx().mark(name);
}

}  // namespace trace
}  // namespace mcg
