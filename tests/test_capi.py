"""The C-ABI library builds, loads and exports every symbol include/moe_hip.h
declares (no GPU needed; no compute calls)."""
from __future__ import annotations

import ctypes
import re
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "moe_hip.h"


def declared_symbols():
    text = HEADER.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b((?:moe|rtdetr|train)_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_expected_entry_points():
    syms = declared_symbols()
    for s in ["moe_router_topk_fwd", "moe_route_scan", "moe_permute_fwd", "moe_combine_fwd", "moe_combine_bwd",
              "moe_token_bwd", "moe_grouped_gemm", "moe_grouped_gemm_wgrad", "moe_last_error",
              "moe_quantize_mx", "moe_permute_fwd_mx", "moe_grouped_gemm_mx", "moe_grouped_gemm_wgrad_mx",
              "moe_set_splitk_workspace", "train_grad_pack", "rtdetr_attn_fwd", "rtdetr_attn_bwd", "rtdetr_conv_fwd", "rtdetr_conv_dgrad", "rtdetr_conv_dgrad_workspace", "rtdetr_conv_wgrad_splits", "rtdetr_conv_set_tuning", "rtdetr_conv_wgrad", "train_grad_sqnorm", "train_grad_norm_finalize", "train_adamw_step",
              "moe_router_wgrad", "moe_router_wgrad_workspace",
              "rtdetr_linear_wgrad_narrow", "rtdetr_linear_wgrad_narrow_parts",
              "rtdetr_maxpool3x3s2_nhwc_fwd", "rtdetr_upcat_nhwc_fwd", "rtdetr_upcat_nhwc_bwd"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    import sys

    sys.path.insert(0, str(ROOT / "multimodal-moe_amd"))
    import build_ext

    lib_path = build_ext.build()
    cdll = ctypes.CDLL(str(lib_path))
    for s in declared_symbols():
        assert hasattr(cdll, s), f"{s} missing from {lib_path}"
    from src.moe import _lib

    assert set(_lib.SIGNATURES) == set(declared_symbols())
    lib = _lib.load_library(lib_path)
    assert lib.moe_version().decode().startswith("moe_hip")
    assert lib.moe_router_num_blocks(130) == 9 == _lib.router_num_blocks(130)  # 16-token router blocks


def test_gpu_path_refuses_cpu_tensors():
    import pytest
    import torch
    from src.moe import _lib

    with pytest.raises(_lib.MoEKernelError, match="GPU tensor"):
        _lib._need(torch.zeros(2), torch.float32, "x")
