"""ctypes binding of libmoe_hip.so (C-ABI declared in include/moe_hip.h).

This is the only place Python touches the HIP kernels.  Every wrapper takes
torch tensors that must already live on the GPU, passes raw device pointers
plus torch's current HIP stream, and raises ``MoEKernelError`` on a non-zero
return code.  There is no fallback: if the library is missing or fails to
load, ``lib()`` raises ``MoELibraryMissing`` (the GPU path fails loudly).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch

_PKG = Path(__file__).resolve().parents[2]  # multimodal-moe_amd/
LIB_PATH = Path(os.environ.get("MOE_HIP_LIB", _PKG / "lib" / "libmoe_hip.so"))

MOE_BF16 = 0
MOE_FP8_E4M3 = 1
MOE_BIAS_BF16 = 0x100  # OR into the grouped-GEMM dtype: bf16 bias
MOE_DENSE_LAYER = 0x200  # OR into the grouped-GEMM dtype: a dense layer (profiled with the dense linears)
EPI_NONE, EPI_BIAS, EPI_BIAS_RELU, EPI_RELU_MASK, EPI_RELU_MASK_MX = 0, 1, 2, 3, 4
MX_BLOCK = 32  # MXFP8: one E8M0 exponent byte per 32 e4m3 elements of a row

# name -> (restype, argtypes); mirrors include/moe_hip.h
_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float
_LL = ctypes.c_longlong
SIGNATURES = {
    "moe_router_num_blocks": (_I, [_I]),
    "moe_router_topk_fwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "moe_route_scan": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "moe_permute_fwd": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "moe_combine_fwd": (_I, [_P, _P, _P, _I, _I, _I, _P, _P]),
    "moe_combine_bwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P, _P]),
    "moe_token_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "moe_grouped_gemm": (_I, [_I, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "moe_grouped_gemm_wgrad": (_I, [_I, _P, _P, _P, _P, _P, _I, _I, _I, _P]),
    "moe_grouped_gemm_wgrad_rows": (_I, [_I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "rtdetr_linear_wgrad": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "rtdetr_linear_wgrad_batch": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "rtdetr_linear_wgrad_narrow_parts": (_I, [_I, _I, _I]),
    "rtdetr_linear_wgrad_narrow": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _P]),
    "rtdetr_linear_wgrad_narrow_batch_parts": (ctypes.c_longlong, [_I, _P, _P, _P]),
    "rtdetr_linear_wgrad_narrow_batch": (_I, [_I, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, ctypes.c_longlong, _I,
                                              _P]),
    "rtdetr_topk_rows": (_I, [_P, _I, _I, _I, _P, _P, _P]),
    "rtdetr_conv3x3_direct_fwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "rtdetr_linear_narrow_supported": (_I, [_I, _I]),
    "rtdetr_linear_narrow_fwd": (_I, [_P, _P, _P, _I, _P, _LL, _I, _I, _I, _P]),
    "rtdetr_linear_narrow_dgrad": (_I, [_P, _P, _P, _P, _LL, _I, _I, _P]),
    "moe_route_index": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "moe_route_dispatch": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _F, _F, _P, _P, _P, _P, _P, _P, _P, _P]),
    "moe_grouped_gemm_gather": (_I, [_I, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "moe_grouped_gemm_scatter": (_I, [_I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "moe_expert_ffn_supported": (_I, [_I, _I, _I]),
    "moe_expert_ffn_fwd": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _I, _P]),
    "moe_ep_compaction": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P]),
    "moe_grouped_gemm_bwd_pair_scatter": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P,
                                               _P, _P, _P, _I, _I, _I, _P]),
    "moe_grouped_gemm_wgrad_gather": (_I, [_I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P]),
    "moe_grouped_gemm_bwd_pair": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P,
                                       _I, _I, _I, _P]),
    "moe_token_bwd_dw": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "moe_token_bwd_res": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P,
                               _P]),
    "moe_combine_res_fwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _P, _P]),
    "moe_quantize_mx": (_I, [_P, ctypes.c_longlong, _I, _P, _P, _P]),
    "moe_permute_fwd_mx": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "moe_grouped_gemm_mx": (_I, [_P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P]),
    "moe_grouped_gemm_wgrad_mx": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _P]),
    "rtdetr_bias_act_nhwc": (_I, [_P, _P, ctypes.c_longlong, _I, _I, _P, _P]),
    "rtdetr_add_bias_relu_nhwc": (_I, [_P, _P, _P, ctypes.c_longlong, _I, _P, _P]),
    "rtdetr_relu_grad2_nhwc": (_I, [_P, _P, _P, ctypes.c_longlong, _I, _P, _P]),
    "rtdetr_fold_scale_multi": (_I, [_P, _P, _I, _P]),
    "rtdetr_fold_scale_batch": (_I, [_I, _P, _P, _P, _P, _P, _P]),
    "rtdetr_bn_act_workspace": (ctypes.c_size_t, [ctypes.c_longlong, _I, _I]),
    "rtdetr_bn_act_fwd": (_I, [_P, _P, _P, _P, _P, _I, ctypes.c_longlong, _I, _I, _F, _F, _P, _P, _P, _P]),
    "rtdetr_bn_act_eval": (_I, [_P, _P, _P, _P, _P, _I, ctypes.c_longlong, _I, _I, _F, _P, _P, _P]),
    "rtdetr_bn_act_bwd": (_I, [_P, _P, _P, _I, ctypes.c_longlong, _I, _I, _P, _P, _P, _P, _P, _P]),
    "rtdetr_avgpool2x2_nhwc_fwd": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "rtdetr_avgpool2x2_nhwc_bwd": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "rtdetr_avgpool2x2_nhwc_bwd_add": (_I, [_P, _P, _I, _I, _I, _I, _P, _P]),
    "rtdetr_maxpool3x3s2_nhwc_fwd": (_I, [_P, _I, _I, _I, _I, _P, _P]),
    "rtdetr_upcat_nhwc_fwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "rtdetr_upcat_nhwc_bwd": (_I, [_P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rtdetr_bias_grad_parts": (_I, [ctypes.c_longlong, _I]),
    "rtdetr_bias_grad": (_I, [_P, ctypes.c_longlong, _I, _P, _I, _P, _I, _P]),
    "rtdetr_add_layer_norm_parts": (_I, [ctypes.c_longlong]),
    "rtdetr_add_layer_norm_fwd": (_I, [_P, _P, _P, _P, _I, ctypes.c_longlong, _I, _F, _P, _P, _P, _P]),
    "rtdetr_add_layer_norm_bwd": (_I, [_P, _P, _P, _P, _I, _P, _P, ctypes.c_longlong, _I, _P, _P, _I, _P, _P]),
    "rtdetr_add_layer_norm_pos_fwd": (_I, [_P, _P, _P, _P, _I, ctypes.c_longlong, _I, _F, _P, _P, _P, _P, _P, _P]),
    "rtdetr_add_layer_norm_bwd2": (_I, [_P, _P, _P, _P, _P, _I, _P, _P, ctypes.c_longlong, _I, _P, _P, _I, _P, _P]),
    "rtdetr_add_layer_norm_final_batch": (_I, [_I, _P, _P, _P, _P, _P, _P]),
    "rtdetr_box_refine_fwd": (_I, [_P, _I, _P, ctypes.c_longlong, _F, _P, _P]),
    "rtdetr_box_refine_bwd": (_I, [_P, _P, _P, _P, ctypes.c_longlong, _F, _P, _I, _P, _P]),
    "rtdetr_msda_fwd": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "rtdetr_msda_bwd": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "rtdetr_msda_bwd_bf16": (_I, [_P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "rtdetr_msda_fused_fwd": (_I, [_P, _P, _P, _P, _P, _P, _F, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "rtdetr_msda_fused_bwd": (_I, [_P, _P, _P, _P, _P, _P, _F, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "rtdetr_msda_vgrad_workspace": (_LL, [_I, _I, _I, _I, _I]),
    "rtdetr_msda_fused_bwd_det": (_I, [_P, _LL, _P, _P, _P, _P, _P, _P, _F, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P,
                                       _P, _LL, _P]),
    "rtdetr_msda_fused_fwd_ld": (_I, [_P, ctypes.c_longlong, _P, _P, _P, _P, _P, _F, _I, _I, _I, _I, _I, _I, _I,
                                      _P, _P]),
    "rtdetr_msda_fused_bwd_ld": (_I, [_P, ctypes.c_longlong, _P, _P, _P, _P, _P, _F, _P, _I, _I, _I, _I, _I, _I, _I,
                                      _P, _I, _P, _P, _P]),
    "moe_set_tuning": (_I, [ctypes.c_char_p, _I]),
    "moe_set_splitk_workspace": (_I, [_P, ctypes.c_size_t, _P, _I]),
    "moe_router_wgrad_workspace": (_LL, [_I, _I, _I, _I]),
    "moe_router_wgrad": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "rtdetr_hungarian_match": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "rtdetr_set_criterion_match": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rtdetr_set_criterion_loss": (_I, [_P, _P, _P, _P, _P, _P, _P, _F, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P]),
    "rtdetr_set_criterion_loss_bwd": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "moe_aux_loss_fwd": (_I, [_P, _I, _I, _P, _I, _I, _F, _F, _P, _P, _P]),
    "rtdetr_attn_fwd": (_I, [_P, _LL, _P, _LL, _P, _LL, _P, _LL, _P, _I, _I, _I, _I, _F, _P]),
    "rtdetr_attn_bwd": (_I, [_P, _LL, _P, _LL, _P, _LL, _P, _LL, _P, _LL, _P, _P, _P, _LL, _P, _LL, _P, _LL,
                             _I, _I, _I, _I, _F, _P]),
    "rtdetr_conv_fwd": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _I, _P]),
    "rtdetr_conv_fwd_act": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _I, _I, _LL, _LL, _P]),
    "rtdetr_conv_fwd_stats_rows": (_I, [_I, _I, _I, _I, _I, _I, _I]),
    "rtdetr_conv_fwd_stats": (_I, [_P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P]),
    "rtdetr_bn_act_fwd_part": (_I, [_P, _P, _P, _P, _P, _I, ctypes.c_longlong, _I, _I, _F, _F, _P, _I, _P, _P, _P]),
    "rtdetr_bn_act_fwd_rows": (_I, [_P, _P, _P, _P, _P, _I, ctypes.c_longlong, _I, _I, _F, _F, _P, _I, _P, _P, _P,
                                    _P, ctypes.c_longlong, ctypes.c_longlong, _P]),
    "rtdetr_bn_act_bwd_rows": (_I, [_P, ctypes.c_longlong, ctypes.c_longlong, _P, _P, _I, ctypes.c_longlong, _I, _I,
                                    _P, _P, _P, _P, _P, _P]),
    "rtdetr_conv_dgrad_workspace": (_LL, [_I, _I, _I, _I, _I, _I]),
    "rtdetr_conv_dgrad": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rtdetr_conv_dgrad_preflipped": (_I, [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "rtdetr_conv_weight_flip_multi": (_I, [_P, _I, _I, _P]),
    "rtdetr_conv_wgrad_splits": (_I, [_I, _I, _I, _I, _I, _I]),
    "rtdetr_conv_set_tuning": (_I, [ctypes.c_char_p, _I]),
    "rtdetr_conv_wgrad": (_I, [_P, _P, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "rtdetr_conv_wgrad_part": (_I, [_P, _P, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P]),
    "rtdetr_conv_wgrad_reduce_batch": (_I, [_I, _P, _P, _P, _P, _I, _P]),
    "train_grad_pack": (_I, [_P, _P, _I, _P, _P]),
    "train_grad_sqnorm": (_I, [_P, _P, _I, _P, _P]),
    "train_grad_norm_finalize": (_I, [_P, _I, _F, _F, _P, _P, _I, _P, _P]),
    "train_adamw_step": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, _P, _I, _F, _F, _F, _F, _P]),
    "moe_profile_enable": (_I, [_I]),
    "moe_profile_count": (_I, []),
    "moe_profile_get": (_I, [_I, _P, _P, _P, _P]),
    "moe_profile_clear": (_I, []),
    "moe_expert_ffn_bwd": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P]),
    "moe_launch_counts": (_I, [_P, _I]),
    "moe_launch_counts_reset": (_I, []),
    "moe_last_error": (ctypes.c_char_p, []),
    "moe_version": (ctypes.c_char_p, []),
}


class MoELibraryMissing(RuntimeError):
    pass


class MoEKernelError(RuntimeError):
    pass


_LIB = None


def load_library(path: Path | str | None = None) -> ctypes.CDLL:
    """Load the shared library and bind every exported symbol (no GPU needed)."""
    p = Path(path) if path is not None else LIB_PATH
    if not p.exists():
        raise MoELibraryMissing(
            f"{p} not found: build it with `python multimodal-moe_amd/build_ext.py` "
            "(or __graft_entry__.build()); the GPU MoE path has no fallback."
        )
    try:
        cdll = ctypes.CDLL(str(p), mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover - depends on the box
        raise MoELibraryMissing(f"failed to load {p}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(cdll, name)  # AttributeError if a symbol is missing
        fn.restype = res
        fn.argtypes = args
    return cdll


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is None:
        _LIB = load_library()
    return _LIB


PROF_KINDS = {0: "grouped_gemm", 1: "dispatch", 2: "router", 3: "route_scan", 4: "token_bwd", 5: "msda",
              6: "mx_quant", 7: "conv_epilogue", 8: "optimizer", 9: "matcher", 10: "grouped_gemm_fp8",
              11: "linear_wgrad", 12: "attention", 13: "conv", 14: "router_wgrad"}
PEAK_BF16_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_FP8_TFLOPS = 5000.0   # MI355X dense fp8 / MXFP8 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E
# dense MFMA peak each profiled kind's flops are priced against
PEAK_TFLOPS_OF = {"grouped_gemm_fp8": PEAK_FP8_TFLOPS}


class KernelProfiler:
    """Per-launch kernel timing by the library's own profiler (moe_profile_*).

    While enabled, libmoe_hip stamps each launch with a hipEvent pair from its
    own dispatch packet (hipExtLaunchKernel: kernel execution only) and records
    its algorithmic HBM bytes and flops (include/moe_hip.h).  ``harvest()``
    adds the completed records to running totals per kind, including the
    roofline time sum(max(flops / peak_flops, bytes / peak_bw)) of each launch.
    Not usable inside hipGraph capture.
    """

    def __init__(self):
        self.enabled = False
        self.acc = {}

    def start(self):
        _check(lib().moe_profile_enable(1), "moe_profile_enable")
        self.acc = {}
        self.enabled = True

    def stop(self):
        lib().moe_profile_enable(0)
        self.enabled = False

    def reset_totals(self):
        self.acc = {}

    def harvest(self):
        """Consume the library's records into the totals (waits for them)."""
        if not self.enabled:
            return
        for kind, ms, flops, byts in profile_records():
            name = PROF_KINDS.get(kind, str(kind))
            d = self.acc.setdefault(name, {"launches": 0, "total_ms": 0.0, "flops": 0.0, "bytes": 0.0,
                                           "t_mfma_ms": 0.0, "t_hbm_ms": 0.0, "t_roof_ms": 0.0})
            t_f = flops / (PEAK_TFLOPS_OF.get(name, PEAK_BF16_TFLOPS) * 1e9)  # ms
            t_b = byts / (PEAK_HBM_GBS * 1e6)       # ms
            d["launches"] += 1
            d["total_ms"] += ms
            d["flops"] += flops
            d["bytes"] += byts
            d["t_mfma_ms"] += t_f
            d["t_hbm_ms"] += t_b
            d["t_roof_ms"] += max(t_f, t_b)

    def summary(self):
        """{kind: dict(launches, total_ms, avg_us, flops, bytes, t_*_ms)} of the harvested launches."""
        out = {k: dict(v) for k, v in self.acc.items()}
        for d in out.values():
            d["avg_us"] = 1e3 * d["total_ms"] / max(d["launches"], 1)
        return out


TIMER = KernelProfiler()


def profile_records(clear=True):
    """[(kind, kernel ms, flops, bytes)] of the launches recorded since the
    profiler was enabled or last cleared (waits for them)."""
    kind, ms, flops, byts = ctypes.c_int(), ctypes.c_float(), ctypes.c_double(), ctypes.c_double()
    out = []
    for i in range(lib().moe_profile_count()):
        _check(lib().moe_profile_get(i, ctypes.byref(kind), ctypes.byref(ms), ctypes.byref(flops),
                                     ctypes.byref(byts)), "moe_profile_get")
        out.append((kind.value, ms.value, flops.value, byts.value))
    if clear:
        lib().moe_profile_clear()
    return out


def launch_counts(reset=False) -> dict:
    """{kind name: launches} the library has issued since the last reset
    (host-side counts, graph capture included: moe_launch_counts)."""
    n = max(PROF_KINDS) + 1
    buf = (ctypes.c_longlong * n)()
    _check(lib().moe_launch_counts(ctypes.cast(buf, ctypes.c_void_p), n), "moe_launch_counts")
    if reset:
        lib().moe_launch_counts_reset()
    return {PROF_KINDS[i]: int(buf[i]) for i in range(n) if buf[i]}


def _ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().moe_last_error()
        raise MoEKernelError(f"{what} failed (rc={rc}): {msg.decode() if msg else ''}")


def _need(t: torch.Tensor, dtype: torch.dtype, name: str) -> None:
    if not t.is_cuda:
        raise MoEKernelError(f"{name} must be a GPU tensor (HIP path has no CPU fallback)")
    if t.dtype != dtype:
        raise MoEKernelError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise MoEKernelError(f"{name} must be contiguous")


# ---------------------------------------------------------------------------
# thin typed wrappers (tensors in, tensors out; shapes checked on the host)
# ---------------------------------------------------------------------------
def set_tuning(key: str, value: int) -> None:
    """A libmoe_hip tuning override: conv_* keys go to rtdetr_conv_set_tuning
    (the convolutions), the rest to moe_set_tuning (the grouped GEMMs)."""
    if key.startswith("conv_"):
        _check(lib().rtdetr_conv_set_tuning(key.encode(), int(value)), f"rtdetr_conv_set_tuning({key}={value})")
        return
    _check(lib().moe_set_tuning(key.encode(), int(value)), f"moe_set_tuning({key}={value})")


# Split-K workspace of the grouped GEMMs (moe_set_splitk_workspace), one per
# device, registered on first use outside graph capture and kept alive for the
# process (captured graphs bake its address in).  64 MiB of fp32 slices covers
# every C2-C5 split launch; a launch whose slices do not fit runs unsplit.
SPLITK_WS_BYTES = 64 << 20
SPLITK_COUNTERS = 1 << 16
_SPLIT_WS: dict[int, tuple[torch.Tensor, torch.Tensor]] = {}


def ensure_splitk_workspace(device: torch.device) -> None:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx in _SPLIT_WS or torch.cuda.is_current_stream_capturing():
        return
    with torch.cuda.device(idx):
        ws = torch.empty(SPLITK_WS_BYTES // 4, dtype=torch.float32, device=f"cuda:{idx}")
        cnt = torch.zeros(SPLITK_COUNTERS, dtype=torch.int32, device=f"cuda:{idx}")
        torch.cuda.current_stream().synchronize()  # counters are zero before any launch reads them
        _check(lib().moe_set_splitk_workspace(_ptr(ws), SPLITK_WS_BYTES, _ptr(cnt), SPLITK_COUNTERS),
               "moe_set_splitk_workspace")
    _SPLIT_WS[idx] = (ws, cnt)


ROUTER_BLOCK_TOKENS = 16  # kRouterBlockTokens (csrc/moe_common.h); moe_router_num_blocks agrees (test_capi)


def router_num_blocks(T: int) -> int:
    return (T + ROUTER_BLOCK_TOKENS - 1) // ROUTER_BLOCK_TOKENS


def router_topk_fwd(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize):
    """Returns (topk_idx, topk_w, probs, lse, local_rank, block_counts, aux_partials)."""
    T, d = x.shape
    E = wg.shape[0]
    _need(x, torch.bfloat16, "x")
    _need(wg, torch.float32, "wg")
    if wg.shape[1] != d:
        raise MoEKernelError(f"wg shape {tuple(wg.shape)} does not match d={d}")
    if ctx_bias is not None:
        _need(ctx_bias, torch.float32, "ctx_bias")
        if ctx_bias.shape[1] != E:
            raise MoEKernelError("ctx_bias must be [C, E]")
        _need(ctx_img, torch.int32, "ctx_img")
        if tokens_per_image <= 0 or ctx_img.numel() * tokens_per_image < T:
            raise MoEKernelError("ctx_img does not cover every token")
    dev = x.device
    nblk = router_num_blocks(T)
    topk_idx = torch.empty((T, k), dtype=torch.int32, device=dev)
    topk_w = torch.empty((T, k), dtype=torch.float32, device=dev)
    probs = torch.empty((T, E), dtype=torch.float32, device=dev)
    lse = torch.empty((T,), dtype=torch.float32, device=dev)
    local_rank = torch.empty((T, k), dtype=torch.int32, device=dev)
    block_counts = torch.empty((nblk, k, E), dtype=torch.int32, device=dev)
    aux_partials = torch.empty((nblk, E + 1), dtype=torch.float32, device=dev)
    rc = lib().moe_router_topk_fwd(
        _ptr(x), _ptr(wg), _ptr(ctx_bias), _ptr(ctx_img) if ctx_bias is not None else None,
        int(ctx_bias.shape[0]) if ctx_bias is not None else 0, int(tokens_per_image), T, d, E, k, int(normalize),
        _ptr(topk_idx), _ptr(topk_w), _ptr(probs), _ptr(lse), _ptr(local_rank),
        _ptr(block_counts), _ptr(aux_partials), _stream())
    _check(rc, "moe_router_topk_fwd")
    return topk_idx, topk_w, probs, lse, local_rank, block_counts, aux_partials


def route_scan(block_counts, cap):
    nblk, k, E = block_counts.shape
    _need(block_counts, torch.int32, "block_counts")
    dev = block_counts.device
    rank_base = torch.empty_like(block_counts)
    hist = torch.empty((E,), dtype=torch.int32, device=dev)
    offsets = torch.empty((E + 1,), dtype=torch.int32, device=dev)
    rc = lib().moe_route_scan(_ptr(block_counts), nblk, k, E, int(cap), _ptr(rank_base),
                              _ptr(hist), _ptr(offsets), _stream())
    _check(rc, "moe_route_scan")
    return rank_base, hist, offsets


def permute_fwd(x, topk_idx, local_rank, rank_base, offsets, E, cap, rows_alloc):
    T, d = x.shape
    k = topk_idx.shape[1]
    _need(x, torch.bfloat16, "x")
    xp = torch.empty((max(rows_alloc, 1), d), dtype=torch.bfloat16, device=x.device)
    pos = torch.empty((T, k), dtype=torch.int32, device=x.device)
    rc = lib().moe_permute_fwd(
        _ptr(x), _ptr(topk_idx), _ptr(local_rank), _ptr(rank_base), _ptr(offsets), T, d, E, k, int(cap),
        _ptr(xp), _ptr(pos), _stream())
    _check(rc, "moe_permute_fwd")
    return xp, pos


def combine_fwd(yp, pos, topk_w, T, resid=None):
    """y = sum_j topk_w[t,j] yp[pos[t,j]] (+ resid[t] when given: the layer's residual, one rounding)."""
    d = yp.shape[1]
    k = pos.shape[1]
    _need(yp, torch.bfloat16, "yp")
    y = torch.empty((T, d), dtype=torch.bfloat16, device=yp.device)
    if resid is not None:
        _need(resid, torch.bfloat16, "resid")
        if tuple(resid.shape) != (T, d):
            raise MoEKernelError(f"combine_fwd: resid shape {tuple(resid.shape)} != {(T, d)}")
        rc = lib().moe_combine_res_fwd(
            _ptr(yp), _ptr(pos), _ptr(topk_w), _ptr(resid), T, d, k, _ptr(y), _stream())
    else:
        rc = lib().moe_combine_fwd(
            _ptr(yp), _ptr(pos), _ptr(topk_w), T, d, k, _ptr(y), _stream())
    _check(rc, "moe_combine_fwd")
    return y


def combine_bwd(dy, yp, pos, topk_w):
    T, d = dy.shape
    k = pos.shape[1]
    _need(dy, torch.bfloat16, "dy")
    _need(yp, torch.bfloat16, "yp")
    dyp = torch.empty_like(yp)
    dw = torch.empty((T, k), dtype=torch.float32, device=dy.device)
    rc = lib().moe_combine_bwd(
        _ptr(dy), _ptr(yp), _ptr(pos), _ptr(topk_w), T, d, k, _ptr(dyp), _ptr(dw), _stream())
    _check(rc, "moe_combine_bwd")
    return dyp, dw


def token_bwd(dxp, pos, probs, topk_idx, topk_w, dw, lse, dprob_bias, zc, wg, normalize):
    T, k = pos.shape
    E, d = wg.shape
    dx = torch.empty((T, d), dtype=torch.bfloat16, device=wg.device)
    dlogits = torch.empty((T, E), dtype=torch.float32, device=wg.device)
    rc = lib().moe_token_bwd(_ptr(dxp), _ptr(pos), _ptr(probs), _ptr(topk_idx), _ptr(topk_w),
                             _ptr(dw), _ptr(lse), _ptr(dprob_bias), _ptr(zc), _ptr(wg),
                             T, d, E, k, int(normalize), _ptr(dx), _ptr(dlogits), _stream())
    _check(rc, "moe_token_bwd")
    return dx, dlogits


def grouped_gemm(a, b, offsets, G, max_rows, N, K, trans_b, epilogue, bias=None, aux=None,
                 out=None, dense=False):
    _need(a, torch.bfloat16, "a")
    _need(b, torch.bfloat16, "b")
    if aux is not None:
        _need(aux, torch.uint8 if epilogue == EPI_RELU_MASK_MX else torch.bfloat16, "aux")
    if b.numel() != G * N * K:
        raise MoEKernelError(f"grouped_gemm: b has {b.numel()} elements, want {G}*{N}*{K}")
    if a.shape[1] != K or a.shape[0] < max_rows:
        raise MoEKernelError("grouped_gemm: a must be [>=max_rows, K]")
    c = out if out is not None else torch.empty((a.shape[0], N), dtype=torch.bfloat16, device=a.device)
    ensure_splitk_workspace(a.device)
    rc = lib().moe_grouped_gemm(
        _gemm_dtype(bias, G, N) | (MOE_DENSE_LAYER if dense else 0), _ptr(a), _ptr(b), _ptr(c), _ptr(offsets), G,
        int(max_rows), N, K, int(trans_b),
        int(epilogue), _ptr(bias), _ptr(aux), None, _stream())
    _check(rc, "moe_grouped_gemm")
    return c


def _gemm_dtype(bias, G, N):
    """MOE_BF16, | MOE_BIAS_BF16 when the bias is a bf16 tensor (read as is)."""
    if bias is None:
        return MOE_BF16
    if bias.dtype not in (torch.float32, torch.bfloat16) or not bias.is_contiguous() or bias.numel() != G * N:
        raise MoEKernelError(f"grouped_gemm: bias must be a contiguous fp32 / bf16 [G, N] tensor ({G} x {N})")
    return MOE_BF16 | (MOE_BIAS_BF16 if bias.dtype == torch.bfloat16 else 0)


def route_index(topk_idx, local_rank, rank_base, offsets, E, cap, rows_alloc):
    """-> (pos int32 [T, k], src_tok int32 [max(rows_alloc, 1)]): the dispatch's
    index half; the GEMMs gather token rows through src_tok (moe_route_index)."""
    T, k = topk_idx.shape
    dev = topk_idx.device
    pos = torch.empty((T, k), dtype=torch.int32, device=dev)
    tok = torch.empty((max(rows_alloc, 1),), dtype=torch.int32, device=dev)
    _check(lib().moe_route_index(_ptr(topk_idx), _ptr(local_rank), _ptr(rank_base), _ptr(offsets), T, E, k,
                                 int(cap), _ptr(pos), _ptr(tok), _stream()), "moe_route_index")
    return pos, tok


def route_dispatch(block_counts, topk_idx, local_rank, topk_w, aux_partials, T, E, cap, rows, lb_coef=None,
                   z_coef=None, row_gate=False):
    """Scan + index (+ aux losses) in one launch (moe_route_dispatch).
    -> (pos, src_tok, hist, offsets, row_gate or None, aux_out3 or None, wcoef or None)."""
    nblk, k, E_ = block_counts.shape
    dev = block_counts.device
    pos = torch.empty((T, k), dtype=torch.int32, device=dev)
    tok = torch.empty((max(rows, 1),), dtype=torch.int32, device=dev)
    hist = torch.empty((E,), dtype=torch.int32, device=dev)
    offsets = torch.empty((E + 1,), dtype=torch.int32, device=dev)
    gate = torch.empty((max(rows, 1),), dtype=torch.float32, device=dev) if row_gate else None
    aux = lb_coef is not None
    out3 = torch.empty(3, dtype=torch.float32, device=dev) if aux else None
    wcoef = torch.empty(E + 1, dtype=torch.float32, device=dev) if aux else None
    _check(lib().moe_route_dispatch(_ptr(block_counts), nblk, T, k, E, int(cap), _ptr(topk_idx), _ptr(local_rank),
                                    _ptr(topk_w), _ptr(aux_partials) if aux else None,
                                    float(lb_coef or 0.0), float(z_coef or 0.0), _ptr(hist), _ptr(offsets),
                                    _ptr(pos), _ptr(tok), _ptr(gate), _ptr(out3), _ptr(wcoef), _stream()),
           "moe_route_dispatch")
    return pos, tok, hist, offsets, gate, out3, wcoef


def grouped_gemm_gather(x, src_tok, b, offsets, G, max_rows, N, K, trans_b, epilogue, bias=None, aux=None):
    """grouped_gemm with routed row r of A = x[src_tok[r]] (x: bf16 token rows [T, K])."""
    _need(x, torch.bfloat16, "x")
    _need(b, torch.bfloat16, "b")
    _need(src_tok, torch.int32, "src_tok")
    if b.numel() != G * N * K or x.shape[1] != K or src_tok.numel() < max_rows:
        raise MoEKernelError("grouped_gemm_gather: shapes")
    c = torch.empty((max(max_rows, 1), N), dtype=torch.bfloat16, device=x.device)
    ensure_splitk_workspace(x.device)
    _check(lib().moe_grouped_gemm_gather(_gemm_dtype(bias, G, N), _ptr(x), _ptr(src_tok), _ptr(b), _ptr(c),
                                         _ptr(offsets), G,
                                         int(max_rows), N, K, int(trans_b), int(epilogue), _ptr(bias), _ptr(aux),
                                         _stream()), "moe_grouped_gemm_gather")
    return c


def expert_ffn_supported(G, F, d):
    return bool(lib().moe_expert_ffn_supported(int(G), int(F), int(d)))


def grouped_gemm_scatter(a, b, offsets, G, max_rows, N, K, trans_b, epilogue, c_rows, out, bias=None, aux=None):
    """grouped_gemm whose output row r goes to row c_rows[r] of out (bf16
    [>= max c_rows + 1, N]; rows no r maps to are left as they are)."""
    _need(a, torch.bfloat16, "a")
    _need(b, torch.bfloat16, "b")
    _need(c_rows, torch.int32, "c_rows")
    _need(out, torch.bfloat16, "out")
    if b.numel() != G * N * K or a.shape[1] != K or a.shape[0] < max_rows or c_rows.numel() < max_rows:
        raise MoEKernelError("grouped_gemm_scatter: shapes")
    if out.dim() != 2 or out.shape[1] != N or not out.is_contiguous():
        raise MoEKernelError("grouped_gemm_scatter: out must be a contiguous [rows, N] tensor")
    ensure_splitk_workspace(a.device)
    _check(lib().moe_grouped_gemm_scatter(_gemm_dtype(bias, G, N), _ptr(a), None, _ptr(b), _ptr(out), _ptr(c_rows),
                                          _ptr(offsets), G, int(max_rows), N, K, int(trans_b), int(epilogue),
                                          _ptr(bias), _ptr(aux), _stream()), "moe_grouped_gemm_scatter")
    return out


def expert_ffn_fwd(x, src_tok, w1, b1, w2, b2, offsets, G, max_rows, yp_rows=None, yp_n=0):
    """One launch (moe_expert_ffn_fwd): h = relu(x[src_tok[r]] W1_g^T + b1_g),
    yp = h W2_g^T + b2_g for every routed row r (src_tok None: x holds the
    routed rows).  w1 bf16 [G, F, d], w2 bf16 [G, d, F]; b1 / b2 fp32 or bf16
    (both the same).  yp_rows (int32): routed row r is stored at row
    yp_rows[r] of a yp_n-row yp (the EP received layout; unmapped rows are
    left uninitialised).  -> (h bf16 [rows, F], yp bf16 [rows or yp_n, d])."""
    _need(x, torch.bfloat16, "x")
    _need(w1, torch.bfloat16, "w1")
    _need(w2, torch.bfloat16, "w2")
    if src_tok is not None:
        _need(src_tok, torch.int32, "src_tok")
    Gw, F, d = w1.shape
    if Gw != G or tuple(w2.shape) != (G, d, F) or x.shape[1] != d or b1.numel() != G * F or b2.numel() != G * d:
        raise MoEKernelError("expert_ffn_fwd: shapes")
    if b1.dtype != b2.dtype or b1.dtype not in (torch.float32, torch.bfloat16):
        raise MoEKernelError("expert_ffn_fwd: b1 / b2 must both be fp32 or both bf16")
    if src_tok is not None and src_tok.numel() < max_rows:
        raise MoEKernelError("expert_ffn_fwd: src_tok shorter than max_rows")
    if yp_rows is not None:
        _need(yp_rows, torch.int32, "yp_rows")
        if yp_rows.numel() < max_rows:
            raise MoEKernelError("expert_ffn_fwd: yp_rows shorter than max_rows")
    h = torch.empty((max(max_rows, 1), F), dtype=torch.bfloat16, device=x.device)
    n_out = int(yp_n) if yp_rows is not None else max(max_rows, 1)
    yp = torch.empty((max(n_out, 1), d), dtype=torch.bfloat16, device=x.device)
    dt = MOE_BF16 | (MOE_BIAS_BF16 if b1.dtype == torch.bfloat16 else 0)
    _check(lib().moe_expert_ffn_fwd(dt, _ptr(x), _ptr(src_tok), _ptr(w1), _ptr(b1.contiguous()),
                                    _ptr(w2), _ptr(b2.contiguous()), _ptr(offsets), G, int(max_rows), F, d,
                                    _ptr(h), _ptr(yp), _ptr(yp_rows), n_out, _stream()), "moe_expert_ffn_fwd")
    return h, yp


def ep_compaction(recv_cnt, hist, S):
    """recv_cnt int32 [W, El] (rows received per source and local expert,
    capped at S), hist int32 [E] (this rank's send histogram) -> (gather
    int32 [W El S], offsets int32 [El + 1], overflow int32 [1]) in one launch
    (moe_ep_compaction)."""
    _need(recv_cnt, torch.int32, "recv_cnt")
    _need(hist, torch.int32, "hist")
    W, El = recv_cnt.shape
    gather = torch.empty(W * El * S, dtype=torch.int32, device=recv_cnt.device)  # (all entries written)
    offsets = torch.empty(El + 1, dtype=torch.int32, device=recv_cnt.device)
    overflow = torch.empty(1, dtype=torch.int32, device=recv_cnt.device)
    _check(lib().moe_ep_compaction(_ptr(recv_cnt), _ptr(hist), W, El, hist.numel(), int(S), _ptr(gather),
                                   _ptr(offsets), _ptr(overflow), _stream()), "moe_ep_compaction")
    return gather, offsets, overflow


def expert_ffn_bwd(dy, tok, gate, x, h, w1, w2, offsets, G, max_rows, out_dtype=torch.bfloat16):
    """The expert FFN backward in two launches (moe_expert_ffn_bwd): dy, x bf16
    [T, d] token rows, tok / gate [>= max_rows] row -> token map and gate, h
    bf16 [max_rows, F] the forward's H, w1 bf16 [G, F, d], w2 bf16 [G, d, F].
    -> (dh [max_rows, F], dxp [max_rows, d], dW1, db1, dW2, db2)."""
    for t, n in ((dy, "dy"), (x, "x"), (h, "h"), (w1, "w1"), (w2, "w2")):
        _need(t, torch.bfloat16, n)
    _need(tok, torch.int32, "tok")
    _need(gate, torch.float32, "gate")
    Gw, F, d = w1.shape
    if Gw != G or tuple(w2.shape) != (G, d, F) or dy.shape[1] != d or x.shape[1] != d or h.shape[1] != F:
        raise MoEKernelError("expert_ffn_bwd: shapes")
    if tok.numel() < max_rows or gate.numel() < max_rows or h.shape[0] < max_rows:
        raise MoEKernelError("expert_ffn_bwd: tok / gate / h shorter than max_rows")
    dev = dy.device
    rows = max(int(max_rows), 1)
    dh = torch.empty((rows, F), dtype=torch.bfloat16, device=dev)
    dxp = torch.empty((rows, d), dtype=torch.bfloat16, device=dev)
    dw1 = torch.empty((G, F, d), dtype=out_dtype, device=dev)
    db1 = torch.empty((G, F), dtype=out_dtype, device=dev)
    dw2 = torch.empty((G, d, F), dtype=out_dtype, device=dev)
    db2 = torch.empty((G, d), dtype=out_dtype, device=dev)
    ensure_splitk_workspace(dev)
    _check(lib().moe_expert_ffn_bwd(_ptr(dy), _ptr(tok), _ptr(gate), _ptr(x), _ptr(h), _ptr(w1), _ptr(w2),
                                    _ptr(offsets), G, int(max_rows), F, d, _ptr(dh), _ptr(dxp), _ptr(dw1), _ptr(db1),
                                    _ptr(dw2), _ptr(db2), int(out_dtype == torch.bfloat16), _stream()),
           "moe_expert_ffn_bwd")
    return dh, dxp, dw1, db1, dw2, db2


def grouped_gemm_bwd_pair(a, b, offsets, G, max_rows, N, K, epilogue, aux, wx, wy, wy_gather=None,
                          out_dtype=torch.bfloat16, a_gather=None, row_scale=None, wx_gather=None, wx_scale=None,
                          c_rows=None, c_n=0):
    """One launch: C = epi(s_r A(r) . B_g) (dgrad, B stored [K][N] per group;
    A(r) = a[a_gather[r]] when given, s_r = row_scale[r]) and the weight
    gradient WC_g = WX_g^T WY_g with colsum (WX(r) = bf16(wx_scale[r] *
    wx[wx_gather[r]]), WY(r) = wy[wy_gather[r]] when given).
    -> (C bf16 [rows, N], WC [G, M2, N2], colsum [G, M2])."""
    _need(a, torch.bfloat16, "a")
    _need(b, torch.bfloat16, "b")
    _need(wx, torch.bfloat16, "wx")
    _need(wy, torch.bfloat16, "wy")
    for t, n in ((a_gather, "a_gather"), (wx_gather, "wx_gather"), (wy_gather, "wy_gather")):
        if t is not None:
            _need(t, torch.int32, n)
    for t, n in ((row_scale, "row_scale"), (wx_scale, "wx_scale")):
        if t is not None:
            _need(t, torch.float32, n)
    if aux is not None:
        _need(aux, torch.uint8 if epilogue == EPI_RELU_MASK_MX else torch.bfloat16, "aux")
    if b.numel() != G * N * K or a.shape[1] != K or (a_gather is None and a.shape[0] < max_rows):
        raise MoEKernelError("grouped_gemm_bwd_pair: dgrad shapes")
    M2, N2 = wx.shape[1], wy.shape[1]
    if (wy_gather is None and wy.shape[0] < max_rows) or (wx_gather is None and wx.shape[0] < max_rows):
        raise MoEKernelError("grouped_gemm_bwd_pair: wgrad shapes")
    rows_out = max(max_rows, 1) if a_gather is not None else a.shape[0]
    if c_rows is not None:  # dgrad row r lands at C row c_rows[r] of a c_n-row C (the rest uninitialised)
        _need(c_rows, torch.int32, "c_rows")
        if c_rows.numel() < max_rows:
            raise MoEKernelError("grouped_gemm_bwd_pair: c_rows shorter than max_rows")
        rows_out = max(int(c_n), 1)
    c = torch.empty((rows_out, N), dtype=torch.bfloat16, device=a.device)
    wc = torch.empty((G, M2, N2), dtype=out_dtype, device=a.device)
    cs = torch.empty((G, M2), dtype=out_dtype, device=a.device)
    ensure_splitk_workspace(a.device)
    _check(lib().moe_grouped_gemm_bwd_pair_scatter(_ptr(a), _ptr(a_gather), _ptr(row_scale), _ptr(b), _ptr(c),
                                                   _ptr(c_rows), _ptr(offsets), G, int(max_rows), N, K,
                                                   int(epilogue), _ptr(aux), _ptr(wx), _ptr(wx_gather),
                                                   _ptr(wx_scale), _ptr(wy), _ptr(wy_gather), _ptr(wc), _ptr(cs), M2,
                                                   N2, int(out_dtype == torch.bfloat16), _stream()),
           "moe_grouped_gemm_bwd_pair")
    return c, wc, cs


def token_bwd_dw(dxp, pos, probs, topk_idx, topk_w, dy, yp, lse, dprob_bias, zc, wg, normalize, want_dw=False,
                 dres=None):
    """token_bwd forming dw = <dy[t], yp[pos]> itself (no combine_bwd): -> (dx, dlogits, dw or None).
    dres (bf16 [T, d]): a residual gradient added into dx (moe_token_bwd_res)."""
    T, k = pos.shape
    E, d = wg.shape
    _need(dy, torch.bfloat16, "dy")
    _need(yp, torch.bfloat16, "yp")
    dx = torch.empty((T, d), dtype=torch.bfloat16, device=wg.device)
    dlogits = torch.empty((T, E), dtype=torch.float32, device=wg.device)
    dw = torch.empty((T, k), dtype=torch.float32, device=wg.device) if want_dw else None
    if dres is not None:
        _need(dres, torch.bfloat16, "dres")
        if tuple(dres.shape) != (T, d):
            raise MoEKernelError(f"token_bwd: dres shape {tuple(dres.shape)} != {(T, d)}")
        _check(lib().moe_token_bwd_res(_ptr(dxp), _ptr(pos), _ptr(probs), _ptr(topk_idx), _ptr(topk_w), None,
                                       _ptr(dy), _ptr(yp), _ptr(dw), _ptr(dres), _ptr(lse), _ptr(dprob_bias),
                                       _ptr(zc), _ptr(wg), T, d, E, k, int(normalize), _ptr(dx), _ptr(dlogits),
                                       _stream()), "moe_token_bwd_res")
        return dx, dlogits, dw
    _check(lib().moe_token_bwd_dw(_ptr(dxp), _ptr(pos), _ptr(probs), _ptr(topk_idx), _ptr(topk_w), None, _ptr(dy),
                                  _ptr(yp), _ptr(dw), _ptr(lse), _ptr(dprob_bias), _ptr(zc), _ptr(wg), T, d, E, k,
                                  int(normalize), _ptr(dx), _ptr(dlogits), _stream()), "moe_token_bwd_dw")
    return dx, dlogits, dw


def router_wgrad(dlogits, x, ctx_img, tokens_per_image, n_ctx):
    """(dwg fp32 [E, d], dcb fp32 [n_ctx, E] or None): the router weight and
    context-bias gradients from token_bwd's dlogits (moe_router_wgrad)."""
    _need(dlogits, torch.float32, "dlogits")
    _need(x, torch.bfloat16, "x")
    T, E = dlogits.shape
    d = x.shape[1]
    has_ctx = ctx_img is not None and n_ctx > 0
    # the image split shapes the token chunks (the same with or without dcb, so
    # dWg does not depend on it); without a context bias any tokens_per_image
    # works: one "image" of all T tokens when it does not divide T
    tpi = int(tokens_per_image) if tokens_per_image else 0
    if has_ctx and (tpi <= 0 or T % tpi):
        raise MoEKernelError(f"router_wgrad: T = {T} is not a multiple of tokens_per_image = {tpi}")
    if tpi <= 0 or T % tpi:
        tpi = max(T, 1)
    B = T // tpi
    dwg = torch.empty((E, d), dtype=torch.float32, device=x.device)
    dcb = None
    if has_ctx:
        _need(ctx_img, torch.int32, "ctx_img")
        dcb = torch.empty((n_ctx, E), dtype=torch.float32, device=x.device)
    _check(lib().moe_router_wgrad(_ptr(dlogits), _ptr(x), _ptr(ctx_img) if dcb is not None else None, B, tpi, E, d,
                                  int(n_ctx) if dcb is not None else 0, None, _ptr(dwg), _ptr(dcb), _stream()),
           "moe_router_wgrad")
    return dwg, dcb


def aux_loss_fwd(auxp, hist, T, k, lb_coef, z_coef):
    """-> (out fp32 [3] = (lb, z, lb_coef lb + z_coef z), wcoef fp32 [E+1])."""
    _need(auxp, torch.float32, "aux_partials")
    _need(hist, torch.int32, "hist")
    nblk, E1 = auxp.shape
    out = torch.empty(3, dtype=torch.float32, device=auxp.device)
    wcoef = torch.empty(E1, dtype=torch.float32, device=auxp.device)
    _check(lib().moe_aux_loss_fwd(_ptr(auxp), nblk, E1 - 1, _ptr(hist), int(T), int(k), float(lb_coef),
                                  float(z_coef), _ptr(out), _ptr(wcoef), _stream()), "moe_aux_loss_fwd")
    return out, wcoef


def hungarian_match(cost, n_valid, status=None):
    """cost fp32 [S, B, Q, M] (queries x padded targets), n_valid int32 [B] ->
    assign int32 [S, B, M]: the query scipy's linear_sum_assignment matches to
    each real target, -1 for padding.  ``status`` (int32 [1], zeroed by the
    caller) records failures without a host sync."""
    _need(cost, torch.float32, "cost")
    _need(n_valid, torch.int32, "n_valid")
    S, B, Q, M = cost.shape
    assign = torch.empty((S, B, M), dtype=torch.int32, device=cost.device)
    if status is None:
        status = torch.zeros(1, dtype=torch.int32, device=cost.device)
    rc = lib().rtdetr_hungarian_match(_ptr(cost), _ptr(n_valid), S, B, Q, M, _ptr(assign), _ptr(status), _stream())
    _check(rc, "rtdetr_hungarian_match")
    return assign


def grouped_gemm_wgrad(x, y, offsets, G, want_colsum=True, out_dtype=torch.float32):
    """(C [G, M, N], colsum [G, M]) in out_dtype (float32 or bfloat16)."""
    _need(x, torch.bfloat16, "x")
    _need(y, torch.bfloat16, "y")
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise MoEKernelError("grouped_gemm_wgrad: out_dtype must be float32 or bfloat16")
    M, N = x.shape[1], y.shape[1]
    c = torch.empty((G, M, N), dtype=out_dtype, device=x.device)
    cs = torch.empty((G, M), dtype=out_dtype, device=x.device) if want_colsum else None
    ensure_splitk_workspace(x.device)
    rc = lib().moe_grouped_gemm_wgrad_rows(
        MOE_BF16, _ptr(x), _ptr(y), _ptr(c), _ptr(cs), _ptr(offsets), G, M, N, int(x.shape[0]),
        int(out_dtype == torch.bfloat16), _stream())
    _check(rc, "moe_grouped_gemm_wgrad_rows")
    return c, cs


_DENSE_OFFSETS = {}


def linear_wgrad(gy, x, out_dtype):
    """A dense linear layer's weight and bias gradients in one launch: the
    grouped wgrad kernel with G = 1 (rows split over up to 8 workgroup slices),
    dW = gy^T x [M, N] and db = colsum(gy) [M], both in out_dtype.  gy bf16
    [K, M], x bf16 [K, N]; M % 64 == 0 and N % 128 == 0."""
    K = int(gy.shape[0])
    key = (K, gy.device)
    off = _DENSE_OFFSETS.get(key)
    if off is None:  # built on the device (capture-safe: no host copy)
        off = torch.arange(2, dtype=torch.int32, device=gy.device) * K
        _DENSE_OFFSETS[key] = off
    _need(gy, torch.bfloat16, "gy")
    _need(x, torch.bfloat16, "x")
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise MoEKernelError("linear_wgrad: out_dtype must be float32 or bfloat16")
    M, N = int(gy.shape[1]), int(x.shape[1])
    dw = torch.empty((M, N), dtype=out_dtype, device=gy.device)
    db = torch.empty((M,), dtype=out_dtype, device=gy.device)
    ensure_splitk_workspace(gy.device)
    rc = lib().rtdetr_linear_wgrad(_ptr(gy), _ptr(x), _ptr(dw), _ptr(db), _ptr(off), K, M, N,
                                   int(out_dtype == torch.bfloat16), _stream())
    _check(rc, "rtdetr_linear_wgrad")
    return dw, db


def linear_wgrad_narrow(gy, x, out_dtype):
    """Weight and bias gradients of a narrow dense linear (out_features M <=
    128 with N even: class heads, box-head last layers, attention weights; or
    in_features N <= 128 with M even: the query position head's first layer):
    dW = gy^T x [M, N], db = colsum(gy) [M] in out_dtype, deterministic.  gy
    bf16 [K, M], x bf16 [K, N], both contiguous."""
    _need(gy, torch.bfloat16, "gy")
    _need(x, torch.bfloat16, "x")
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise MoEKernelError("linear_wgrad_narrow: out_dtype must be float32 or bfloat16")
    K, M, N = int(gy.shape[0]), int(gy.shape[1]), int(x.shape[1])
    if x.shape[0] != K:
        raise MoEKernelError("linear_wgrad_narrow: gy and x row counts differ")
    part = torch.empty((int(lib().rtdetr_linear_wgrad_narrow_parts(K, M, N)),), dtype=torch.float32, device=gy.device)
    dw = torch.empty((M, N), dtype=out_dtype, device=gy.device)
    db = torch.empty((M,), dtype=out_dtype, device=gy.device)
    _check(lib().rtdetr_linear_wgrad_narrow(_ptr(gy), _ptr(x), _ptr(dw), _ptr(db), _ptr(part), K, M, N,
                                            int(out_dtype == torch.bfloat16), _stream()),
           "rtdetr_linear_wgrad_narrow")
    return dw, db


TOPK_MAX_N, TOPK_MAX_K = 32768, 1024


def topk_rows(x, k, values=False):
    """Top-k of each row of fp32 x [rows, n] (rtdetr_topk_rows: radix select +
    bitonic sort in LDS, n <= 32768, k <= 1024) -> int64 indices [rows, k],
    sorted by value descending (equal values: lower index first; and the
    lowest indices among equal values at the cut), plus the values when asked."""
    if not x.is_cuda or x.dtype != torch.float32 or x.dim() != 2:
        raise MoEKernelError("topk_rows: x must be an fp32 [rows, n] GPU tensor (no CPU fallback)")
    x = x.contiguous()
    rows, n = x.shape
    idx = torch.empty((rows, k), dtype=torch.int64, device=x.device)
    val = torch.empty((rows, k), dtype=torch.float32, device=x.device) if values else None
    _check(lib().rtdetr_topk_rows(_ptr(x), rows, n, int(k), _ptr(idx), _ptr(val), _stream()), "rtdetr_topk_rows")
    return (idx, val) if values else idx


def conv3x3_direct_fwd(x, w, bias, stride=1, relu=True):
    """relu(conv3x3(x, w, pad 1) + bias) for the stem's 3 -> 32 layer
    (rtdetr_conv3x3_direct_fwd): x bf16 [B, 3, H, W] channels_last, w bf16
    [32, 3, 3, 3] (any strides), bias fp32 [32] or None -> bf16 channels_last."""
    for t, name in ((x, "x"), (w, "w")):
        if not t.is_cuda or t.dtype != torch.bfloat16:
            raise MoEKernelError(f"conv3x3_direct_fwd: {name} must be a bf16 GPU tensor (no CPU fallback)")
    B, C, H, W = x.shape
    N = w.shape[0]
    if not x.is_contiguous(memory_format=torch.channels_last) or tuple(w.shape[1:]) != (C, 3, 3):
        raise MoEKernelError("conv3x3_direct_fwd: x channels_last [B, C, H, W], w [N, C, 3, 3]")
    if bias is not None:
        _need(bias, torch.float32, "bias")
        if bias.numel() != N or not bias.is_contiguous():
            raise MoEKernelError("conv3x3_direct_fwd: bias fp32 [N]")
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    wf = w.permute(2, 3, 1, 0).reshape(9 * C, N).float().contiguous()  # [(ky 3 + kx) C + c][n]
    y = torch.empty((B, N, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    _check(lib().rtdetr_conv3x3_direct_fwd(_ptr(x), _ptr(wf), _ptr(bias), _ptr(y), B, H, W, C, N, int(stride),
                                           int(bool(relu)), _stream()), "rtdetr_conv3x3_direct_fwd")
    return y


def linear_narrow_ok(K, N):
    """Shapes rtdetr_linear_narrow_fwd takes (N <= 8 with K % 8 == 0, or K <= 8 with N % 8 == 0)."""
    return (1 <= N <= 8 and K >= 8 and K % 8 == 0) or (1 <= K <= 8 and N >= 8 and N % 8 == 0)


def linear_narrow_fwd(x, w, b, relu=False):
    """y = act(x w^T + b) for a narrow layer (rtdetr_linear_narrow_fwd): x bf16
    [M, K] contiguous, w bf16 [N, K], b bf16 / fp32 [N] or None -> bf16 [M, N]."""
    _need(x, torch.bfloat16, "x")
    _need(w, torch.bfloat16, "w")
    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K or not x.is_contiguous() or not w.is_contiguous():
        raise MoEKernelError("linear_narrow_fwd: x [M, K] and w [N, K] contiguous")
    if b is not None and (b.dtype not in (torch.bfloat16, torch.float32) or b.numel() != N or not b.is_contiguous()):
        raise MoEKernelError("linear_narrow_fwd: b must be a contiguous bf16 / fp32 [N] tensor")
    y = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    _check(lib().rtdetr_linear_narrow_fwd(_ptr(x), _ptr(w), _ptr(b), int(b is not None and b.dtype == torch.bfloat16),
                                          _ptr(y), M, K, N, int(bool(relu)), _stream()), "rtdetr_linear_narrow_fwd")
    return y


def linear_narrow_dgrad(g, w, mask=None):
    """gx = (g w) * [mask > 0] through a narrow layer (rtdetr_linear_narrow_dgrad):
    g bf16 [M, N <= 8] contiguous, w bf16 [N, K], mask bf16 [M, K] or None."""
    _need(g, torch.bfloat16, "g")
    _need(w, torch.bfloat16, "w")
    M, N = g.shape
    K = w.shape[1]
    if w.shape[0] != N or not g.is_contiguous() or not w.is_contiguous():
        raise MoEKernelError("linear_narrow_dgrad: g [M, N] and w [N, K] contiguous")
    if mask is not None:
        _need(mask, torch.bfloat16, "mask")
        if tuple(mask.shape) != (M, K) or not mask.is_contiguous():
            raise MoEKernelError("linear_narrow_dgrad: mask must be a contiguous [M, K] tensor")
    gx = torch.empty((M, K), dtype=torch.bfloat16, device=g.device)
    _check(lib().rtdetr_linear_narrow_dgrad(_ptr(g), _ptr(w), _ptr(mask), _ptr(gx), M, K, N, _stream()),
           "rtdetr_linear_narrow_dgrad")
    return gx


LINEAR_WGRAD_BATCH = 24  # problems per rtdetr_linear_wgrad_batch launch


LN_FINAL_BATCH = 48  # problems per rtdetr_add_layer_norm_final_batch launch


def add_layer_norm_final_batch(jobs):
    """[(partials fp32 [P, 2d], out [2, d] bf16 / fp32 contiguous)]: the
    LayerNorms' [dgamma; dbeta] from their row-pass partials, batched."""
    for i in range(0, len(jobs), LN_FINAL_BATCH):
        part = jobs[i:i + LN_FINAL_BATCH]
        n = len(part)
        ps, outs = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)()
        Ps, Ns, bf = (ctypes.c_int * n)(), (ctypes.c_int * n)(), (ctypes.c_int * n)()
        for q, (pt, out) in enumerate(part):
            _need(pt, torch.float32, "partials")
            if out.dtype not in (torch.float32, torch.bfloat16) or not out.is_contiguous() or pt.dim() != 2 \
                    or out.numel() != pt.shape[1] or not pt.is_contiguous():
                raise MoEKernelError("add_layer_norm_final_batch: partials [P, 2d] and out [2, d] contiguous")
            ps[q], outs[q] = pt.data_ptr(), out.data_ptr()
            Ps[q], Ns[q], bf[q] = int(pt.shape[0]), int(pt.shape[1]), int(out.dtype == torch.bfloat16)
        c = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
        _check(lib().rtdetr_add_layer_norm_final_batch(n, c(ps), c(Ps), c(Ns), c(outs), c(bf), _stream()),
               "rtdetr_add_layer_norm_final_batch")


NARROW_BATCH = 32  # problems per rtdetr_linear_wgrad_narrow_batch launch pair


def linear_wgrad_narrow_batch(groups, out_dtype):
    """Narrow dense weight + bias gradients, batched: groups = [([(gy bf16
    [K, M], x bf16 [K, N]), ...], dw [M, N], db [M])] -- each group's outputs
    the sum over its problems (contiguous out_dtype tensors)."""
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise MoEKernelError("linear_wgrad_narrow_batch: out_dtype must be float32 or bfloat16")
    chunk, n = [], 0
    for grp in groups + [None]:
        if grp is None or n + len(grp[0]) > NARROW_BATCH:
            if chunk:
                _narrow_batch_launch(chunk, out_dtype)
            chunk, n = [], 0
            if grp is None:
                break
        if len(grp[0]) > NARROW_BATCH:
            raise MoEKernelError("linear_wgrad_narrow_batch: a group of more than 32 problems")
        chunk.append(grp)
        n += len(grp[0])


def _narrow_batch_launch(groups, out_dtype):
    probs = [pr for g in groups for pr in g[0]]
    n, ng = len(probs), len(groups)
    gys, xs = (ctypes.c_void_p * n)(), (ctypes.c_void_p * n)()
    Ks, Ms, Ns = (ctypes.c_int * n)(), (ctypes.c_int * n)(), (ctypes.c_int * n)()
    for q, (gy, x) in enumerate(probs):
        _need(gy, torch.bfloat16, "gy")
        _need(x, torch.bfloat16, "x")
        if gy.dim() != 2 or x.dim() != 2 or gy.shape[0] != x.shape[0] or not (gy.is_contiguous() and x.is_contiguous()):
            raise MoEKernelError("linear_wgrad_narrow_batch: gy [K, M] and x [K, N] contiguous")
        gys[q], xs[q] = gy.data_ptr(), x.data_ptr()
        Ks[q], Ms[q], Ns[q] = int(gy.shape[0]), int(gy.shape[1]), int(x.shape[1])
    cnt = (ctypes.c_int * ng)(*[len(g[0]) for g in groups])
    dws, dbs = (ctypes.c_void_p * ng)(), (ctypes.c_void_p * ng)()
    for g, (_, dw, db) in enumerate(groups):
        if dw.dtype != out_dtype or db.dtype != out_dtype or not (dw.is_contiguous() and db.is_contiguous()):
            raise MoEKernelError("linear_wgrad_narrow_batch: dw / db must be contiguous out_dtype tensors")
        dws[g], dbs[g] = dw.data_ptr(), db.data_ptr()
    floats = int(lib().rtdetr_linear_wgrad_narrow_batch_parts(n, ctypes.cast(Ks, ctypes.c_void_p),
                                                               ctypes.cast(Ms, ctypes.c_void_p),
                                                               ctypes.cast(Ns, ctypes.c_void_p)))
    if floats < 0:
        raise MoEKernelError("linear_wgrad_narrow_batch: a problem outside the narrow shapes")
    part = torch.empty(max(floats, 2), dtype=torch.float32, device=probs[0][0].device)
    c = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
    _check(lib().rtdetr_linear_wgrad_narrow_batch(n, c(gys), c(xs), c(Ks), c(Ms), c(Ns), ng, c(cnt), c(dws), c(dbs),
                                                  part.data_ptr(), floats, int(out_dtype == torch.bfloat16),
                                                  _stream()), "rtdetr_linear_wgrad_narrow_batch")


def linear_wgrad_batch(jobs, out_dtype):
    """Several dense weight + bias gradients in ceil(n / 24) launches:
    jobs = [(gy bf16 [K, M], x bf16 [K, N], dw [M, N], db [M])] with dw / db
    contiguous out_dtype outputs (views into larger buffers allowed); dw =
    gy^T x, db = colsum(gy).  M % 64 == 0, N % 128 == 0."""
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise MoEKernelError("linear_wgrad_batch: out_dtype must be float32 or bfloat16")
    ensure_splitk_workspace(jobs[0][0].device)
    for i in range(0, len(jobs), LINEAR_WGRAD_BATCH):
        part = jobs[i:i + LINEAR_WGRAD_BATCH]
        n = len(part)
        ptrs = [(ctypes.c_void_p * n)() for _ in range(4)]
        dims = [(ctypes.c_int * n)() for _ in range(3)]
        for q, (gy, x, dw, db) in enumerate(part):
            _need(gy, torch.bfloat16, "gy")
            _need(x, torch.bfloat16, "x")
            if dw.dtype != out_dtype or db.dtype != out_dtype or not (dw.is_contiguous() and db.is_contiguous()):
                raise MoEKernelError("linear_wgrad_batch: dw / db must be contiguous out_dtype tensors")
            K, M, N = int(gy.shape[0]), int(gy.shape[1]), int(x.shape[1])
            if x.shape[0] != K or dw.shape != (M, N) or db.shape != (M,):
                raise MoEKernelError("linear_wgrad_batch: shape mismatch")
            for arr, t in zip(ptrs, (gy, x, dw, db)):
                arr[q] = t.data_ptr()
            dims[0][q], dims[1][q], dims[2][q] = K, M, N
        args = [ctypes.cast(a, ctypes.c_void_p) for a in (*ptrs, *dims)]
        rc = lib().rtdetr_linear_wgrad_batch(n, *args, int(out_dtype == torch.bfloat16), _stream())
        _check(rc, "rtdetr_linear_wgrad_batch")


# ---------------------------------------------------------------------------
# MXFP8 (config C5): e4m3 data as torch.uint8, E8M0 exponents as torch.uint8
# ---------------------------------------------------------------------------
def quantize_mx(x):
    """x bf16 [..., K] -> (q uint8 [..., K] e4m3, s uint8 [..., K/32] E8M0)."""
    _need(x, torch.bfloat16, "x")
    K = x.shape[-1]
    R = x.numel() // max(K, 1)
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    sc = torch.empty((*x.shape[:-1], K // MX_BLOCK), dtype=torch.uint8, device=x.device)
    _check(lib().moe_quantize_mx(_ptr(x), R, K, _ptr(q), _ptr(sc), _stream()), "moe_quantize_mx")
    return q, sc


def permute_fwd_mx(x, topk_idx, local_rank, rank_base, offsets, E, cap, rows_alloc):
    T, d = x.shape
    k = topk_idx.shape[1]
    _need(x, torch.bfloat16, "x")
    n = max(rows_alloc, 1)
    xq = torch.empty((n, d), dtype=torch.uint8, device=x.device)
    xs = torch.empty((n, d // MX_BLOCK), dtype=torch.uint8, device=x.device)
    pos = torch.empty((T, k), dtype=torch.int32, device=x.device)
    rc = lib().moe_permute_fwd_mx(
        _ptr(x), _ptr(topk_idx), _ptr(local_rank), _ptr(rank_base), _ptr(offsets), T, d, E, k, int(cap),
        _ptr(xq), _ptr(xs), _ptr(pos), _stream())
    _check(rc, "moe_permute_fwd_mx")
    return xq, xs, pos


def grouped_gemm_mx(aq, as_, bq, bs, offsets, G, max_rows, N, K, epilogue, bias=None, out_mx=False):
    """MXFP8 rows-grouped GEMM, B stored [G, N, K].  Returns bf16 C [rows, N], or
    (e4m3 C uint8 [rows, N], exponents uint8 [rows, N/32]) when out_mx."""
    for t, n in ((aq, "a"), (as_, "a_scales"), (bq, "b"), (bs, "b_scales")):
        _need(t, torch.uint8, n)
    if bq.numel() != G * N * K or bs.numel() != G * N * K // MX_BLOCK:
        raise MoEKernelError(f"grouped_gemm_mx: b must be [{G}, {N}, {K}] with [{G}, {N}, {K // MX_BLOCK}] scales")
    if aq.shape[1] != K or aq.shape[0] < max_rows or as_.shape != (aq.shape[0], K // MX_BLOCK):
        raise MoEKernelError("grouped_gemm_mx: a must be [>=max_rows, K] with [rows, K/32] scales")
    rows = aq.shape[0]
    if out_mx:
        c = torch.empty((rows, N), dtype=torch.uint8, device=aq.device)
        cs = torch.empty((rows, N // MX_BLOCK), dtype=torch.uint8, device=aq.device)
    else:
        c = torch.empty((rows, N), dtype=torch.bfloat16, device=aq.device)
        cs = None
    rc = lib().moe_grouped_gemm_mx(
        _ptr(aq), _ptr(as_), _ptr(bq), _ptr(bs), _ptr(c), _ptr(cs), _ptr(offsets), G, int(max_rows), N, K,
        int(epilogue), _ptr(bias), _stream())
    _check(rc, "moe_grouped_gemm_mx")
    return (c, cs) if out_mx else c


def grouped_gemm_wgrad_mx(x, yq, ys, offsets, G, want_colsum=True):
    """C_g = X_g^T deq(Y_g): x bf16 [rows, M], yq/ys MXFP8 [rows, N] -> fp32 [G, M, N] (+ colsum of x)."""
    _need(x, torch.bfloat16, "x")
    _need(yq, torch.uint8, "y")
    _need(ys, torch.uint8, "y_scales")
    M, N = x.shape[1], yq.shape[1]
    c = torch.empty((G, M, N), dtype=torch.float32, device=x.device)
    cs = torch.empty((G, M), dtype=torch.float32, device=x.device) if want_colsum else None
    rc = lib().moe_grouped_gemm_wgrad_mx(
        _ptr(x), _ptr(yq), _ptr(ys), _ptr(c), _ptr(cs), _ptr(offsets), G, M, N, _stream())
    _check(rc, "moe_grouped_gemm_wgrad_mx")
    return c, cs


def _nhwc_rows(t, name):
    """[B, C, H, W] channels_last (or [M, C] contiguous) bf16 -> (M, C)."""
    _need_dtype_dev(t, torch.bfloat16, name)
    if t.dim() == 4:
        if not t.is_contiguous(memory_format=torch.channels_last):
            raise MoEKernelError(f"{name} must be channels_last")
        B, C, H, W = t.shape
        return B * H * W, C
    if not t.is_contiguous():
        raise MoEKernelError(f"{name} must be contiguous")
    return t.shape[0], t.shape[1]


def _need_dtype_dev(t, dtype, name):
    if not t.is_cuda:
        raise MoEKernelError(f"{name} must be a GPU tensor (HIP path has no CPU fallback)")
    if t.dtype != dtype:
        raise MoEKernelError(f"{name}: expected {dtype}, got {t.dtype}")


def bias_act_nhwc(x, bias, relu, out=None):
    """y = act(x + bias[c]) over a channels_last bf16 activation (out may be x)."""
    M, C = _nhwc_rows(x, "x")
    _need(bias, torch.float32, "bias")
    y = out if out is not None else torch.empty_like(x)
    _check(lib().rtdetr_bias_act_nhwc(_ptr(x), _ptr(bias), M, C, 1 if relu else 0, _ptr(y), _stream()),
           "rtdetr_bias_act_nhwc")
    return y


def add_bias_relu_nhwc(a, b, bias):
    """y = relu(a + b + bias[c]) over channels_last bf16 activations (bias may be None)."""
    M, C = _nhwc_rows(a, "a")
    if _nhwc_rows(b, "b") != (M, C):
        raise MoEKernelError("add_bias_relu: a and b differ in shape")
    if bias is not None:
        _need(bias, torch.float32, "bias")
    y = torch.empty_like(a)
    _check(lib().rtdetr_add_bias_relu_nhwc(_ptr(a), _ptr(b), _ptr(bias), M, C, _ptr(y), _stream()),
           "rtdetr_add_bias_relu_nhwc")
    return y


def relu_grad2_nhwc(g1, g2, y):
    """(g1 + g2) * (y > 0) over channels_last bf16 tensors (g2 may be None)."""
    M, C = _nhwc_rows(y, "y")
    if _nhwc_rows(g1, "g1") != (M, C) or (g2 is not None and _nhwc_rows(g2, "g2") != (M, C)):
        raise MoEKernelError("relu_grad2: shapes differ")
    out = torch.empty_like(y)
    _check(lib().rtdetr_relu_grad2_nhwc(_ptr(g1), _ptr(g2), _ptr(y), M, C, _ptr(out), _stream()),
           "rtdetr_relu_grad2_nhwc")
    return out


def _ptrs(ts):
    arr = (ctypes.c_void_p * len(ts))(*[_ptr(t) for t in ts])
    return ctypes.cast(arr, ctypes.c_void_p), arr  # keep arr alive with the call


def _bn_ws(M, C, nb, dev):
    n = int(lib().rtdetr_bn_act_workspace(M, C, nb)) // 4
    return torch.empty(n, dtype=torch.float32, device=dev)


def bn_act_fwd(xs, gammas, betas, run_means, run_vars, act, eps, momentum, resid=None):
    """Training BatchNorm of 1-2 channels_last bf16 branches, summed, act
    (0 none / 1 silu) [+ resid, bf16 like x] -> (y, saved fp32 [nb, 4, C])."""
    if resid is not None:
        return _bn_act_fwd_resid(xs, gammas, betas, run_means, run_vars, act, eps, momentum, None, resid)
    M, C = _nhwc_rows(xs[0], "x0")
    nb = len(xs)
    for i, x in enumerate(xs[1:], 1):
        if _nhwc_rows(x, f"x{i}") != (M, C):
            raise MoEKernelError("bn_act: branches differ in shape")
    for t in list(gammas) + list(betas) + [r for r in run_means + run_vars if r is not None]:
        _need(t, torch.float32, "bn affine/statistics")
    y = torch.empty_like(xs[0])
    saved = torch.empty((nb, 4, C), dtype=torch.float32, device=y.device)
    ws = _bn_ws(M, C, nb, y.device)
    px, kx = _ptrs(xs)
    pg, kg = _ptrs(gammas)
    pb, kb = _ptrs(betas)
    has_run = all(r is not None for r in run_means + run_vars)
    pm, km = _ptrs(run_means) if has_run else (None, None)
    pv, kv = _ptrs(run_vars) if has_run else (None, None)
    _check(lib().rtdetr_bn_act_fwd(px, pg, pb, pm, pv, nb, M, C, int(act), float(eps), float(momentum),
                                   _ptr(saved), _ptr(ws), _ptr(y), _stream()), "rtdetr_bn_act_fwd")
    return y, saved


def bn_act_eval(xs, gammas, betas, run_means, run_vars, act, eps, resid=None):
    """Inference-mode BatchNorm (running statistics) of 1-2 channels_last bf16
    branches, summed, act (0 none / 1 silu) [+ resid after the act], one pass
    (rtdetr_bn_act_eval) -> y."""
    M, C = _nhwc_rows(xs[0], "x0")
    nb = len(xs)
    for i, x in enumerate(xs[1:], 1):
        if _nhwc_rows(x, f"x{i}") != (M, C):
            raise MoEKernelError("bn_act_eval: branches differ in shape")
    if resid is not None and (_nhwc_rows(resid, "resid") != (M, C) or resid.data_ptr() % 16):
        raise MoEKernelError("bn_act_eval: resid must be a 16-B aligned channels_last bf16 tensor like x")
    for t in list(gammas) + list(betas) + list(run_means) + list(run_vars):
        _need(t, torch.float32, "bn affine/statistics")
    y = torch.empty_like(xs[0])
    px, kx = _ptrs(xs)
    pg, kg = _ptrs(gammas)
    pb, kb = _ptrs(betas)
    pm, km = _ptrs(run_means)
    pv, kv = _ptrs(run_vars)
    _check(lib().rtdetr_bn_act_eval(px, pg, pb, pm, pv, nb, M, C, int(act), float(eps), _ptr(resid), _ptr(y),
                                    _stream()), "rtdetr_bn_act_eval")
    return y


def _bn_act_fwd_resid(xs, gammas, betas, run_means, run_vars, act, eps, momentum, part, resid):
    """bn_act_fwd / bn_act_fwd_part with y = act(z) + resid
    (rtdetr_bn_act_fwd_rows, contiguous rows)."""
    M, C = _nhwc_rows(xs[0], "x0")
    nb = len(xs)
    for i, x in enumerate(xs[1:], 1):
        if _nhwc_rows(x, f"x{i}") != (M, C):
            raise MoEKernelError("bn_act: branches differ in shape")
    if _nhwc_rows(resid, "resid") != (M, C) or resid.data_ptr() % 16:
        raise MoEKernelError("bn_act: resid must be a 16-B aligned channels_last bf16 tensor like x")
    if part is not None:
        _need(part, torch.float32, "part")
        if part.dim() != 4 or part.shape[0] != nb or part.shape[2] != 2 or part.shape[3] != C:
            raise MoEKernelError(f"bn_act_fwd_part: part must be [{nb}, nblk, 2, {C}], got {tuple(part.shape)}")
    for t in list(gammas) + list(betas) + [r for r in run_means + run_vars if r is not None]:
        _need(t, torch.float32, "bn affine/statistics")
    y = torch.empty_like(xs[0])
    saved = torch.empty((nb, 4, C), dtype=torch.float32, device=y.device)
    ws = None if part is not None else _bn_ws(M, C, nb, y.device)
    px, kx = _ptrs(xs)
    pg, kg = _ptrs(gammas)
    pb, kb = _ptrs(betas)
    has_run = all(r is not None for r in run_means + run_vars)
    pm, km = _ptrs(run_means) if has_run else (None, None)
    pv, kv = _ptrs(run_vars) if has_run else (None, None)
    _check(lib().rtdetr_bn_act_fwd_rows(px, pg, pb, pm, pv, nb, M, C, int(act), float(eps), float(momentum),
                                        _ptr(part), int(part.shape[1]) if part is not None else 0, _ptr(ws),
                                        _ptr(saved), _ptr(resid), _ptr(y), 0, 0, _stream()), "rtdetr_bn_act_fwd_rows")
    return y, saved


def bn_act_fwd_part(xs, gammas, betas, run_means, run_vars, act, eps, momentum, part, resid=None):
    """bn_act_fwd with the statistics partials of rtdetr_conv_fwd_stats:
    part fp32 [nb, nblk, 2, C]."""
    if resid is not None:
        return _bn_act_fwd_resid(xs, gammas, betas, run_means, run_vars, act, eps, momentum, part, resid)
    M, C = _nhwc_rows(xs[0], "x0")
    nb = len(xs)
    for i, x in enumerate(xs[1:], 1):
        if _nhwc_rows(x, f"x{i}") != (M, C):
            raise MoEKernelError("bn_act: branches differ in shape")
    _need(part, torch.float32, "part")
    if part.dim() != 4 or part.shape[0] != nb or part.shape[2] != 2 or part.shape[3] != C:
        raise MoEKernelError(f"bn_act_fwd_part: part must be [{nb}, nblk, 2, {C}], got {tuple(part.shape)}")
    for t in list(gammas) + list(betas) + [r for r in run_means + run_vars if r is not None]:
        _need(t, torch.float32, "bn affine/statistics")
    y = torch.empty_like(xs[0])
    saved = torch.empty((nb, 4, C), dtype=torch.float32, device=y.device)
    px, kx = _ptrs(xs)
    pg, kg = _ptrs(gammas)
    pb, kb = _ptrs(betas)
    has_run = all(r is not None for r in run_means + run_vars)
    pm, km = _ptrs(run_means) if has_run else (None, None)
    pv, kv = _ptrs(run_vars) if has_run else (None, None)
    _check(lib().rtdetr_bn_act_fwd_part(px, pg, pb, pm, pv, nb, M, C, int(act), float(eps), float(momentum),
                                        _ptr(part), int(part.shape[1]), _ptr(saved), _ptr(y), _stream()),
           "rtdetr_bn_act_fwd_part")
    return y, saved


def bn_act_bwd(dy, xs, gammas, saved, act):
    """-> ([dx_i bf16], dgb fp32 [nb, 2, C] = dgamma, dbeta)."""
    M, C = _nhwc_rows(xs[0], "x0")
    if _nhwc_rows(dy, "dy") != (M, C):
        raise MoEKernelError("bn_act_bwd: dy shape")
    nb = len(xs)
    dxs = [torch.empty_like(x) for x in xs]
    coef = torch.empty((nb, 3, C), dtype=torch.float32, device=dy.device)
    dgb = torch.empty((nb, 2, C), dtype=torch.float32, device=dy.device)
    ws = _bn_ws(M, C, nb, dy.device)
    px, kx = _ptrs(xs)
    pg, kg = _ptrs(gammas)
    pd, kd = _ptrs(dxs)
    _check(lib().rtdetr_bn_act_bwd(_ptr(dy), px, pg, nb, M, C, int(act), _ptr(saved), _ptr(ws), _ptr(coef), pd,
                                   _ptr(dgb), _stream()), "rtdetr_bn_act_bwd")
    return dxs, dgb


def bn_act_fwd_rows(x, gamma, beta, run_mean, run_var, act, eps, momentum, part, y, row0, hw, bstride):
    """One-branch bn_act_fwd whose output goes to rows of a wider tensor: y
    bf16 [B', S, C] contiguous, x's row r (image r // hw, pixel r % hw) to y's
    flat row (r // hw) * bstride + row0 + r % hw.  part: conv-epilogue
    statistics fp32 [1, nblk, 2, C] or None (a statistics pass).  -> saved."""
    M, C = _nhwc_rows(x, "x")
    _need(y, torch.bfloat16, "y")
    if not y.is_contiguous() or y.shape[-1] != C or M % hw or (M // hw - 1) * bstride + row0 + hw > y.numel() // C:
        raise MoEKernelError("bn_act_fwd_rows: y layout")
    for t in [gamma, beta] + [r for r in (run_mean, run_var) if r is not None]:
        _need(t, torch.float32, "bn affine/statistics")
    saved = torch.empty((1, 4, C), dtype=torch.float32, device=x.device)
    ws = None if part is not None else _bn_ws(M, C, 1, x.device)
    if part is not None:
        _need(part, torch.float32, "part")
        if part.dim() != 4 or part.shape[0] != 1 or part.shape[2] != 2 or part.shape[3] != C:
            raise MoEKernelError("bn_act_fwd_rows: part must be [1, nblk, 2, C]")
    px, kx = _ptrs([x])
    pg, kg = _ptrs([gamma])
    pb, kb = _ptrs([beta])
    has_run = run_mean is not None and run_var is not None
    pm, km = _ptrs([run_mean]) if has_run else (None, None)
    pv, kv = _ptrs([run_var]) if has_run else (None, None)
    _check(lib().rtdetr_bn_act_fwd_rows(px, pg, pb, pm, pv, 1, M, C, int(act), float(eps), float(momentum),
                                        _ptr(part), int(part.shape[1]) if part is not None else 0, _ptr(ws),
                                        _ptr(saved), None, y.data_ptr() + row0 * C * 2, hw, bstride, _stream()),
           "rtdetr_bn_act_fwd_rows")
    return saved


def bn_act_bwd_rows(dy, row0, hw, bstride, x, gamma, saved, act):
    """One-branch bn_act_bwd reading dy from rows of a wider tensor (the
    layout of bn_act_fwd_rows).  -> (dx bf16 like x, dgb fp32 [1, 2, C])."""
    M, C = _nhwc_rows(x, "x")
    _need(dy, torch.bfloat16, "dy")
    if not dy.is_contiguous() or dy.shape[-1] != C or M % hw or (M // hw - 1) * bstride + row0 + hw > dy.numel() // C:
        raise MoEKernelError("bn_act_bwd_rows: dy layout")
    dx = torch.empty_like(x)
    coef = torch.empty((1, 3, C), dtype=torch.float32, device=x.device)
    dgb = torch.empty((1, 2, C), dtype=torch.float32, device=x.device)
    ws = _bn_ws(M, C, 1, x.device)
    px, kx = _ptrs([x])
    pg, kg = _ptrs([gamma])
    pd, kd = _ptrs([dx])
    _check(lib().rtdetr_bn_act_bwd_rows(dy.data_ptr() + row0 * C * 2, hw, bstride, px, pg, 1, M, C, int(act),
                                        _ptr(saved), _ptr(ws), _ptr(coef), pd, _ptr(dgb), _stream()),
           "rtdetr_bn_act_bwd_rows")
    return dx, dgb


def msda_fwd(value, shapes, starts, loc, attn):
    """value bf16 [B,S,H,D]; shapes/starts int32 on device; loc fp32 [B,Q,H,L,P,2];
    attn fp32 [B,Q,H,L,P] -> bf16 [B,Q,H*D]."""
    B, S, H, D = value.shape
    Q, L, P = loc.shape[1], loc.shape[3], loc.shape[4]
    _need(value, torch.bfloat16, "value")
    _need(loc, torch.float32, "loc")
    _need(attn, torch.float32, "attn")
    out = torch.empty((B, Q, H * D), dtype=torch.bfloat16, device=value.device)
    rc = lib().rtdetr_msda_fwd(
        _ptr(value), _ptr(shapes), _ptr(starts), _ptr(loc), _ptr(attn), B, S, Q, H, D, L, P, _ptr(out), _stream())
    _check(rc, "rtdetr_msda_fwd")
    return out


def msda_fused_fwd(value, shapes, starts, off, ref, logits, offset_scale, L, P):
    """value bf16 [B,S,H,D]; off bf16 [B,Q,H*L*P*2]; ref fp32 [B,Q,4]; logits bf16 [B,Q,H*L*P] -> bf16 [B,Q,H*D]."""
    B, S, H, D = value.shape
    Q = off.shape[1]
    for t, n, dt in ((value, "value", torch.bfloat16), (off, "off", torch.bfloat16), (ref, "ref", torch.float32),
                     (logits, "logits", torch.bfloat16)):
        _need(t, dt, n)
    if off.numel() != B * Q * H * L * P * 2 or logits.numel() != B * Q * H * L * P or ref.numel() != B * Q * 4:
        raise MoEKernelError("msda_fused: shape mismatch")
    out = torch.empty((B, Q, H * D), dtype=torch.bfloat16, device=value.device)
    _check(lib().rtdetr_msda_fused_fwd(_ptr(value), _ptr(shapes), _ptr(starts), _ptr(off), _ptr(ref), _ptr(logits),
                                       float(offset_scale), B, S, Q, H, D, L, P, _ptr(out), _stream()),
           "rtdetr_msda_fused_fwd")
    return out


def msda_fused_bwd(value, shapes, starts, off, ref, logits, offset_scale, L, P, grad_out):
    """-> (grad_value bf16 [B,S,H,D], grad_off bf16 like off, grad_logits bf16 like logits)."""
    B, S, H, D = value.shape
    Q = off.shape[1]
    _need(grad_out, torch.bfloat16, "grad_out")
    gv = torch.empty_like(value)
    go = torch.empty_like(off)
    gl = torch.empty_like(logits)
    _check(lib().rtdetr_msda_fused_bwd(_ptr(value), _ptr(shapes), _ptr(starts), _ptr(off), _ptr(ref), _ptr(logits),
                                       float(offset_scale), _ptr(grad_out), B, S, Q, H, D, L, P, _ptr(gv), _ptr(go),
                                       _ptr(gl), _stream()), "rtdetr_msda_fused_bwd")
    return gv, go, gl


def msda_fused_fwd_slice(value_all, col0, H, D, shapes, starts, off, ref, logits, offset_scale, L, P):
    """MSDA on the column slice [col0, col0 + H*D) of value_all bf16 [B, S, C]
    (rtdetr_msda_fused_fwd_ld: row stride C) -> bf16 [B, Q, H*D]."""
    B, S, C = value_all.shape
    Q = off.shape[1]
    _need(value_all, torch.bfloat16, "value_all")
    if col0 < 0 or col0 + H * D > C or off.numel() != B * Q * H * L * P * 2 or logits.numel() != B * Q * H * L * P:
        raise MoEKernelError("msda_fused_slice: shape mismatch")
    out = torch.empty((B, Q, H * D), dtype=torch.bfloat16, device=value_all.device)
    base = value_all.data_ptr() + 2 * col0
    _check(lib().rtdetr_msda_fused_fwd_ld(base, C, _ptr(shapes), _ptr(starts), _ptr(off), _ptr(ref), _ptr(logits),
                                          float(offset_scale), B, S, Q, H, D, L, P, _ptr(out), _stream()),
           "rtdetr_msda_fused_fwd_ld")
    return out


def msda_fused_bwd_slice(value_all, grad_all, col0, H, D, shapes, starts, off, ref, logits, offset_scale, L, P,
                         grad_out):
    """Backward of msda_fused_fwd_slice: the value gradient is ACCUMULATED into
    the same column slice of grad_all (bf16 [B, S, C], zeroed by the caller);
    -> (grad_off, grad_logits)."""
    B, S, C = value_all.shape
    Q = off.shape[1]
    _need(grad_out, torch.bfloat16, "grad_out")
    _need(grad_all, torch.bfloat16, "grad_all")
    if grad_all.shape != value_all.shape:
        raise MoEKernelError("msda_fused_slice: grad_all must match value_all")
    go = torch.empty_like(off)
    gl = torch.empty_like(logits)
    _check(lib().rtdetr_msda_fused_bwd_ld(value_all.data_ptr() + 2 * col0, C, _ptr(shapes), _ptr(starts), _ptr(off),
                                          _ptr(ref), _ptr(logits), float(offset_scale), _ptr(grad_out), B, S, Q, H, D,
                                          L, P, grad_all.data_ptr() + 2 * col0, 0, _ptr(go), _ptr(gl), _stream()),
           "rtdetr_msda_fused_bwd_ld")
    return go, gl


def msda_det_ok(L, P, D):
    """Shapes the deterministic MSDA backward takes (the RT-DETR decoder's)."""
    return L == 3 and P == 4 and D in (32, 64)


def msda_fused_bwd_slice_det(value_all, grad_all, col0, H, D, shapes, starts, hw, off, ref, logits, offset_scale, L,
                             P, grad_out):
    """Deterministic backward of msda_fused_fwd_slice (rtdetr_msda_fused_bwd_det):
    the value gradient of the column slice is WRITTEN (every element; fp32
    sums in a fixed order, one bf16 rounding) -- grad_all needs no zeroing.
    hw: the L level sizes h_l w_l (host ints).  -> (grad_off, grad_logits)."""
    B, S, C = value_all.shape
    Q = off.shape[1]
    _need(grad_out, torch.bfloat16, "grad_out")
    _need(grad_all, torch.bfloat16, "grad_all")
    if grad_all.shape != value_all.shape or len(hw) != L:
        raise MoEKernelError("msda_fused_bwd_slice_det: shapes")
    go = torch.empty_like(off)
    gl = torch.empty_like(logits)
    nbytes = int(lib().rtdetr_msda_vgrad_workspace(B, Q, H, L, P))
    work = torch.empty(nbytes, dtype=torch.uint8, device=value_all.device)
    hw_c = (ctypes.c_int32 * L)(*[int(v) for v in hw])
    _check(lib().rtdetr_msda_fused_bwd_det(value_all.data_ptr() + 2 * col0, C, _ptr(shapes), _ptr(starts), hw_c,
                                           _ptr(off), _ptr(ref), _ptr(logits), float(offset_scale), _ptr(grad_out),
                                           B, S, Q, H, D, L, P, grad_all.data_ptr() + 2 * col0, _ptr(go), _ptr(gl),
                                           _ptr(work), nbytes, _stream()), "rtdetr_msda_fused_bwd_det")
    return go, gl


def msda_bwd(value, shapes, starts, loc, attn, grad_out, bf16_grad_value=False):
    """grad_value fp32 (fp32 atomics) or, with bf16_grad_value, bf16 (packed bf16 atomics)."""
    B, S, H, D = value.shape
    Q, L, P = loc.shape[1], loc.shape[3], loc.shape[4]
    _need(grad_out, torch.bfloat16, "grad_out")
    gv = torch.empty((B, S, H, D), dtype=torch.bfloat16 if bf16_grad_value else torch.float32, device=value.device)
    gl = torch.empty_like(loc)
    ga = torch.empty_like(attn)
    fn = lib().rtdetr_msda_bwd_bf16 if bf16_grad_value else lib().rtdetr_msda_bwd
    rc = fn(_ptr(value), _ptr(shapes), _ptr(starts), _ptr(loc), _ptr(attn), _ptr(grad_out), B, S, Q, H, D, L, P,
            _ptr(gv), _ptr(gl), _ptr(ga), _stream())
    _check(rc, "rtdetr_msda_bwd")
    return gv, gl, ga
