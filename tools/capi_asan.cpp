// Host-side argument checks of libmoe_hip.so under AddressSanitizer (SURVEY.md
// 5, "race detection / sanitizers"): every call below hands the C-ABI an
// invalid argument (NULL operand, bad shape, unknown option) and must come
// back with a non-zero code and a moe_last_error() message -- before any
// launch, so it needs no GPU.  Built and run by tests/test_capi_asan.py with
// the library and this driver compiled `-Xarch_host -fsanitize=address`
// (build_ext.py --asan); any out-of-bounds host access, use-after-free or leak
// in the checking / error paths fails the run.
#include <cstdio>
#include <cstring>

#include "../include/moe_hip.h"

static int g_fail = 0, g_n = 0;

static void expect_error(const char* what, int rc) {
  ++g_n;
  const char* msg = moe_last_error();
  if (rc == 0 || msg == nullptr || std::strlen(msg) == 0) {
    std::printf("FAIL %s: rc=%d msg=%s\n", what, rc, msg ? msg : "(null)");
    ++g_fail;
  } else {
    std::printf("ok   %-28s rc=%d  %s\n", what, rc, msg);
  }
}

int main() {
  // plausible-looking (never dereferenced) device pointers for the non-NULL arguments
  char buf[4096] __attribute__((aligned(256)));
  void* p = buf;
  auto* i32 = reinterpret_cast<int32_t*>(buf);
  auto* f32 = reinterpret_cast<float*>(buf);
  hipStream_t s = nullptr;
  expect_error("router_topk_fwd E=0", moe_router_topk_fwd(p, f32, nullptr, nullptr, 0, 16, 16, 256, 0, 1, 1, i32, f32,
                                                          f32, f32, i32, i32, f32, s));
  expect_error("router_topk_fwd d=100", moe_router_topk_fwd(p, f32, nullptr, nullptr, 0, 16, 16, 100, 8, 2, 1, i32,
                                                            f32, f32, f32, i32, i32, f32, s));
  expect_error("route_scan k=0", moe_route_scan(i32, 1, 0, 8, 0, i32, i32, i32, s));
  expect_error("permute_fwd d=7", moe_permute_fwd(p, i32, i32, i32, i32, 16, 7, 8, 2, 0, p, i32, s));
  expect_error("combine_fwd k=0", moe_combine_fwd(p, i32, f32, 16, 256, 0, p, s));
  expect_error("token_bwd d=100", moe_token_bwd(p, i32, f32, i32, f32, f32, f32, nullptr, nullptr, f32, 16, 100, 8,
                                                2, 1, p, f32, s));
  expect_error("token_bwd dw=NULL", moe_token_bwd(p, i32, f32, i32, f32, nullptr, f32, nullptr, nullptr, f32, 16, 256,
                                                  8, 2, 1, p, f32, s));
  expect_error("grouped_gemm N=100", moe_grouped_gemm(0, p, p, p, i32, 8, 64, 100, 256, 1, 0, nullptr, nullptr,
                                                      nullptr, s));
  expect_error("grouped_gemm bias epi, no bias", moe_grouped_gemm(0, p, p, p, i32, 8, 64, 1024, 256, 1, 1, nullptr,
                                                                  nullptr, nullptr, s));
  expect_error("grouped_gemm_gather G=0", moe_grouped_gemm_gather(0, p, i32, p, p, i32, 0, 64, 1024, 256, 1, 0,
                                                                  nullptr, nullptr, s));
  expect_error("wgrad_rows M=63", moe_grouped_gemm_wgrad_rows(0, p, p, p, nullptr, i32, 8, 63, 128, 0, 0, s));
  expect_error("bwd_pair epilogue=9", moe_grouped_gemm_bwd_pair(p, nullptr, nullptr, p, p, i32, 8, 64, 1024, 256, 9,
                                                                nullptr, p, nullptr, nullptr, p, nullptr, p, p,
                                                                1024, 256, 1, s));
  expect_error("expert_ffn_fwd d=128", moe_expert_ffn_fwd(0, p, nullptr, p, p, p, p, i32, 8, 64, 1024, 128, p, p,
                                                          nullptr, 0, s));
  expect_error("expert_ffn_fwd w1=NULL", moe_expert_ffn_fwd(0, p, nullptr, nullptr, p, p, p, i32, 8, 64, 1024, 256,
                                                            p, p, nullptr, 0, s));
  expect_error("expert_ffn_fwd fp8 dtype", moe_expert_ffn_fwd(1, p, nullptr, p, p, p, p, i32, 8, 64, 1024, 256, p,
                                                              p, nullptr, 0, s));
  expect_error("ep_compaction W=0", moe_ep_compaction(i32, i32, 0, 2, 16, 64, i32, i32, i32, s));
  expect_error("ep_compaction gather=NULL", moe_ep_compaction(i32, i32, 8, 2, 16, 64, nullptr, i32, i32, s));
  expect_error("quantize_mx K=31", moe_quantize_mx(p, 16, 31, p, p, s));
  expect_error("router_wgrad E=0", moe_router_wgrad(f32, p, nullptr, 1, 16, 0, 256, 0, f32, f32, nullptr, s));
  expect_error("aux_loss_fwd E=0", moe_aux_loss_fwd(f32, 1, 0, i32, 16, 2, 0.01f, 0.001f, f32, f32, s));
  expect_error("set_tuning unknown key", moe_set_tuning("no_such_knob", 1));
  expect_error("set_tuning bad value", moe_set_tuning("ksplit", 99));
  const float lr = 1e-4f;
  expect_error("adamw_step 0 groups", train_adamw_step(p, i32, 1, f32, f32, f32, f32, i32, &lr, 0, 0.f, 0.9f,
                                                       0.999f, 1e-8f, s));
  std::printf("%d checks, %d failed\n", g_n, g_fail);
  return g_fail == 0 ? 0 : 1;
}
