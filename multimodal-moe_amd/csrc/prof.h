// RAII launch profiler scope (see capi.hip).  While profiling is enabled
// (moe_profile_enable) the kernel launched through MOE_LAUNCH inside the scope
// gets a start/stop hipEvent pair stamped by its own dispatch packet
// (hipExtLaunchKernel: kernel execution time, no host gaps), and the scope
// records the launch's algorithmic HBM bytes bytes_fixed + bytes_per_row * R and
// flops flops_per_row * R (per_row = false: bytes_fixed and flops_per_row are
// the launch's totals), where R (the routed row count, known only on the
// device) is written by the kernel itself into rows_slot() -- a device int of
// the profiler -- so profiling adds no copies or launches.  Events come from a
// pool created when profiling is enabled.  Disabled: MOE_LAUNCH is a plain
// hipLaunchKernelGGL and rows_slot() is nullptr.
#pragma once

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace moe {

enum ProfKind {
  PROF_GEMM = 0,
  PROF_ROWMOVE = 1,
  PROF_ROUTER = 2,
  PROF_SCAN = 3,
  PROF_TOKEN_BWD = 4,
  PROF_MSDA = 5,
  PROF_QUANT = 6,
  PROF_CONV_EPI = 7,
  PROF_OPTIM = 8,
  PROF_MATCH = 9,
  PROF_GEMM_FP8 = 10,  // grouped GEMM on the fp8 (MXFP8 e4m3) MFMA: priced against the fp8 peak
  PROF_LINEAR = 11,    // dense linear weight + bias gradients (rtdetr_linear_wgrad)
  PROF_ATTN = 12,      // multi-head self-attention (rtdetr_attn_fwd / _bwd)
  PROF_CONV = 13,      // implicit-GEMM convolutions (rtdetr_conv_*)
  PROF_ROUTER_WGRAD = 14  // router weight / context-bias gradients (moe_router_wgrad)
};

class ProfScope {
 public:
  ProfScope(hipStream_t s, int kind, double bytes_fixed, bool per_row = false, double bytes_per_row = 0.0,
            double flops_per_row = 0.0);
  ~ProfScope() = default;
  bool active() const { return active_ && idx_ >= 0; }
  hipEvent_t start_event() const;
  hipEvent_t stop_event() const;
  int32_t* rows_slot() const;  // device int the kernel sets to its row count, or nullptr
  ProfScope(const ProfScope&) = delete;
  ProfScope& operator=(const ProfScope&) = delete;

 private:
  bool active_;
  int idx_;
};

}  // namespace moe

#define MOE_LAUNCH(prof, kern, grid, block, shmem, stream, ...)                                          \
  do {                                                                                                    \
    if ((prof).active())                                                                                  \
      hipExtLaunchKernelGGL(kern, grid, block, shmem, stream, (prof).start_event(), (prof).stop_event(), 0, \
                            __VA_ARGS__);                                                                 \
    else                                                                                                  \
      hipLaunchKernelGGL(kern, grid, block, shmem, stream, __VA_ARGS__);                                  \
  } while (0)
