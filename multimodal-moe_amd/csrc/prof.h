// RAII launch profiler scope (see capi.hip): while profiling is enabled
// (moe_profile_enable), records a hipEvent pair on `stream` around the kernel
// launched inside the scope, plus the launch's algorithmic work
// work_fixed + work_per_row * (*dev_rows) (dev_rows: a device int such as
// offsets[G], copied back stream-ordered after the kernel).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace moe {

enum ProfKind { PROF_GEMM = 0, PROF_ROWMOVE = 1, PROF_ROUTER = 2, PROF_SCAN = 3, PROF_TOKEN_BWD = 4, PROF_MSDA = 5 };

class ProfScope {
 public:
  ProfScope(hipStream_t s, int kind, double work_fixed, const int32_t* dev_rows = nullptr,
            double work_per_row = 0.0);
  ~ProfScope();
  ProfScope(const ProfScope&) = delete;
  ProfScope& operator=(const ProfScope&) = delete;

 private:
  hipStream_t stream_;
  bool active_;
  int idx_;
  const int32_t* dev_rows_ = nullptr;
};

}  // namespace moe
