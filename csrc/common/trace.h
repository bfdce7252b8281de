// Optional roctx ranges for the native runtime (SURVEY.md §5.1 tracing).
//
// Enabled with BLENDTORCH_ROCTX=1; libroctx64 is dlopen'ed on first use, so
// nothing links against it and the ranges cost one branch when disabled.
// Ranges show up in `rocprofv3 --marker-trace` timelines next to the HIP
// kernels and copies they explain (recv -> assemble -> H2D + decode).
#pragma once

#include <dlfcn.h>

#include <cstdlib>

namespace btn {
namespace trace {

struct Roctx {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  bool on = false;
  Roctx() {
    const char* e = std::getenv("BLENDTORCH_ROCTX");
    if (!e || e[0] != '1') return;
    // prefer the roctx the process already loaded (torch links its own copy,
    // and that is the one rocprofv3 hooks); else load one
    push = reinterpret_cast<int (*)(const char*)>(dlsym(RTLD_DEFAULT, "roctxRangePushA"));
    pop = reinterpret_cast<int (*)()>(dlsym(RTLD_DEFAULT, "roctxRangePop"));
    if (!push || !pop) {
      void* h = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
      if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
      if (!h) return;
      push = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      pop = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
    }
    on = push && pop;
  }
  static Roctx& get() {
    static Roctx r;
    return r;
  }
};

// RAII range: `trace::Range r("btn.launch");`
struct Range {
  bool on;
  explicit Range(const char* name) : on(Roctx::get().on) {
    if (on) Roctx::get().push(name);
  }
  ~Range() {
    if (on) Roctx::get().pop();
  }
};

}  // namespace trace
}  // namespace btn
