// SPDX-License-Identifier: MIT
// roctx ranges around the scheduler's phases, resolved at run time so the
// libraries carry no link dependency: set GS_ROCTX=1 and run under
// `rocprofv3 --marker-trace` (or any roctx consumer) to see exchange / fused / step / bc
// ranges on the timeline.  Off (one predictable branch per phase) otherwise.
#pragma once

#include <dlfcn.h>
#include <stdlib.h>

namespace gs {

struct Roctx {
  typedef int (*push_fn)(const char*);
  typedef int (*pop_fn)();
  push_fn push = nullptr;
  pop_fn pop = nullptr;

  static Roctx& get() {
    static Roctx r = load();
    return r;
  }

 private:
  static Roctx load() {
    Roctx r;
    const char* e = getenv("GS_ROCTX");
    if (!e || atoi(e) == 0) return r;
    void* h = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return r;
    r.push = (push_fn)dlsym(h, "roctxRangePushA");
    r.pop = (pop_fn)dlsym(h, "roctxRangePop");
    if (!r.push || !r.pop) r.push = nullptr, r.pop = nullptr;
    return r;
  }
};

// RAII range: `TraceRange tr("exchange");`
class TraceRange {
 public:
  explicit TraceRange(const char* name) {
    const Roctx& r = Roctx::get();
    on_ = r.push != nullptr;
    if (on_) r.push(name);
  }
  ~TraceRange() {
    if (on_) Roctx::get().pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_ = false;
};

}  // namespace gs
