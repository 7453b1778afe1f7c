// roctx ranges from C++ (visible on rocprofv3 --marker-trace / sys-trace timelines), enabled with FAN_ROCTX=1.
//
// The library is opened at run time (the rocprofiler-sdk roctx first, the legacy roctracer one as fallback), so the
// extension has no link-time dependency and a disabled range costs one branch. Reference: the NIC's per-state cycle
// counters and the host's DETAILED_PROFILE phase timers (hw/all_reduce.sv:892-1085; sw/mlp_mpi_example_f32.cpp:32-33,
// 702-814) — here every request phase (pack, all-to-all, reduce, all-gather, ring round, epilogue) is a named range.
#pragma once
#include <dlfcn.h>

#include <cstdlib>
#include <cstring>

namespace fan {

class Roctx {
 public:
  static Roctx& get() {
    static Roctx r;
    return r;
  }
  bool on() const { return push_ != nullptr; }
  void push(const char* name) const {
    if (push_) push_(name);
  }
  void pop() const {
    if (pop_) pop_();
  }

 private:
  Roctx() {
    const char* e = std::getenv("FAN_ROCTX");
    if (!e || std::strcmp(e, "1") != 0) return;
    for (const char* lib : {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                            "libroctx64.so"}) {
      void* h = dlopen(lib, RTLD_NOW | RTLD_GLOBAL);
      if (!h) continue;
      auto p = reinterpret_cast<int (*)(const char*)>(dlsym(h, "roctxRangePushA"));
      auto q = reinterpret_cast<int (*)()>(dlsym(h, "roctxRangePop"));
      if (p && q) {
        push_ = p;
        pop_ = q;
        return;
      }
    }
  }
  int (*push_)(const char*) = nullptr;
  int (*pop_)() = nullptr;
};

// Scoped range: RoctxRange r("mesh/all_to_all");
class RoctxRange {
 public:
  explicit RoctxRange(const char* name) : on_(Roctx::get().on()) {
    if (on_) Roctx::get().push(name);
  }
  ~RoctxRange() {
    if (on_) Roctx::get().pop();
  }
  RoctxRange(const RoctxRange&) = delete;
  RoctxRange& operator=(const RoctxRange&) = delete;

 private:
  bool on_;
};

}  // namespace fan
