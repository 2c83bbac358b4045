"""Summarise one gpu_round.sh session into profiles/<round>/.

Reads (under gpurun_out/<tag>/):
  prof/run_kernel_stats.csv           rocprofv3 --kernel-trace --stats of `python bench.py`
  pmc_fetch/p_counter_collection.csv  rocprofv3 --pmc FETCH_SIZE   (MoE/MSDA kernels only)
  pmc_write/p_counter_collection.csv  rocprofv3 --pmc WRITE_SIZE
and writes profiles/<round>/kernel_summary.json: per kernel group (the same
groups bench.py's library profiler reports) the rocprof launch count and
average duration, and the HBM bytes per launch from the PMC passes with the
MI355X_MICROARCH.md gfx950 corrections (FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE counts half the bytes of a wide streaming read, so it is doubled).

    python tools/profile_summary.py gpurun_out/r01b profiles/r01 [c2]
(with a workload name it also writes profiles/pmc_traffic_<workload>.json,
which bench.py reports as roofline.traffic)
"""
from __future__ import annotations

import csv
import json
import re
import sys
from pathlib import Path

GROUPS = [
    # the detector's MLP heads on the grouped GEMM (MOE_DENSE_LAYER: FL_DENSE = 16 in the template) are
    # not expert GEMMs -- matched first, kept out of the roofline group
    ("dense_gemm", re.compile(r"gemm_v\d_kernel<[^>]*, 16>")),
    ("grouped_gemm", re.compile(r"gemm_v\d_kernel|gemm_pair_kernel|gemm_triple_kernel|expert_ffn_fwd_kernel")),
    ("linear_wgrad", re.compile(r"linear_wgrad_kernel")),
    ("dispatch", re.compile(r"permute_fwd(_mx)?_kernel|combine_fwd_kernel|combine_bwd_kernel")),
    ("router", re.compile(r"router_topk_fwd_kernel")),
    ("route_scan", re.compile(r"route_scan_kernel|route_dispatch_kernel|route_index_kernel")),
    ("quantize_mx", re.compile(r"quantize_mx_kernel")),
    ("token_bwd", re.compile(r"token_bwd_kernel")),
    ("router_wgrad", re.compile(r"router_wgrad_kernel")),
    ("msda", re.compile(r"msda_(fused_)?(fwd|bwd)(_lp)?_kernel|msda_vgrad_(sort|tile)_kernel")),
]


def group_of(name: str):
    for g, rx in GROUPS:
        if rx.search(name):
            return g
    return None


def kernel_stats(path: Path):
    out, total_ns = {}, 0.0
    with open(path) as f:
        for row in csv.DictReader(f):
            total_ns += float(row["TotalDurationNs"])
            g = group_of(row["Name"])
            if g is None:
                continue
            d = out.setdefault(g, {"launches": 0, "total_ns": 0.0})
            d["launches"] += int(row["Calls"])
            d["total_ns"] += float(row["TotalDurationNs"])
    for d in out.values():
        d["avg_us"] = round(d["total_ns"] / d["launches"] / 1e3, 3)
    return out, total_ns


def pmc(path: Path, counter: str):
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            g = group_of(row["Kernel_Name"])
            if g is None:
                continue
            d = out.setdefault(g, {"launches": 0, "kib": 0.0})
            d["launches"] += 1
            d["kib"] += float(row["Counter_Value"])
    return out


def pmc_multi(path: Path, counters):
    """{group: {counter: summed value, "launches": n}} over the listed counters."""
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            c = row["Counter_Name"]
            if c not in counters:
                continue
            g = group_of(row["Kernel_Name"])
            if g is None:
                continue
            d = out.setdefault(g, {"dispatches": set()})
            d[c] = d.get(c, 0.0) + float(row["Counter_Value"])
            d["dispatches"].add(row.get("Dispatch_Id", row.get("Correlation_Id", len(d["dispatches"]))))
    for d in out.values():
        d["launches"] = len(d.pop("dispatches"))
    return out


# MI355X: 256 CUs x 4 SIMDs; rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs
# (MI355X_MICROARCH.md, DVFS note), so the kernel's active cycles are GRBM / 8
N_CU, N_SIMD, N_XCD = 256, 4, 8
FLOP_PER_MFMA = 2 * 16 * 16 * 32  # v_mfma_f32_16x16x32_bf16, the grouped GEMM's instruction


def mfma_summary(path: Path):
    cs = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_MFMA", "SQ_INSTS_VALU_MFMA_MOPS_BF16",
          "GRBM_GUI_ACTIVE")
    out = {}
    for g, d in pmc_multi(path, cs).items():
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in d or "GRBM_GUI_ACTIVE" not in d:
            continue
        n = d["launches"]
        active = d["GRBM_GUI_ACTIVE"] / N_XCD
        e = {"pmc_launches": n,
             "mfma_busy_cycles_per_launch": round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / n),
             "gui_active_cycles_per_launch": round(active / n),
             # fraction of all SIMD-cycles of the kernel's lifetime the matrix cores were busy
             "mfma_counter_frac": round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / (active * N_CU * N_SIMD), 4)}
        if "SQ_INSTS_MFMA" in d:
            e["mfma_insts_per_launch"] = round(d["SQ_INSTS_MFMA"] / n)
            e["mfma_busy_cycles_per_inst"] = round(d["SQ_VALU_MFMA_BUSY_CYCLES"] / max(d["SQ_INSTS_MFMA"], 1), 2)
            e["mfma_inst_flops_per_launch"] = round(d["SQ_INSTS_MFMA"] * FLOP_PER_MFMA / n)
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in d:  # rocprofv3's MfmaFlopsBF16 = MOPS x 512
            e["mfma_bf16_flops_per_launch"] = round(d["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / n)
        if "SQ_BUSY_CYCLES" in d:
            e["sq_busy_cycles_per_launch"] = round(d["SQ_BUSY_CYCLES"] / n)
        out[g] = e
    return out


def main(src: str, dst: str):
    src_p, dst_p = Path(src), Path(dst)
    dst_p.mkdir(parents=True, exist_ok=True)
    stats, total_ns = kernel_stats(src_p / "prof" / "run_kernel_stats.csv")
    fetch = pmc(src_p / "pmc_fetch" / "p_counter_collection.csv", "FETCH_SIZE")
    write = pmc(src_p / "pmc_write" / "p_counter_collection.csv", "WRITE_SIZE")
    mp = src_p / "pmc_mfma" / "p_counter_collection.csv"
    mfma = mfma_summary(mp) if mp.exists() else {}
    res = {"source": str(src_p), "all_kernels_total_ms": round(total_ns / 1e6, 3), "groups": {}}
    # the profiled bench line: its build id and configuration let bench.py tell
    # whether this summary belongs to the build it runs (bench.rocprof_headline)
    bj = src_p / "prof" / "bench.json"
    if bj.exists():
        lines = [ln for ln in bj.read_text().splitlines() if ln.startswith("{")]
        if lines:
            b = json.loads(lines[-1])
            res["bench"] = {"libmoe_hip_sha16": b.get("build", {}).get("libmoe_hip_sha16"),
                            "precision": b.get("build", {}).get("precision"),
                            "graphs": b.get("build", {}).get("graphs"),
                            "workload": b.get("config", {}).get("workload"),
                            "batch": b.get("config", {}).get("batch"),
                            "steps": b.get("steps"), "warmup": b.get("warmup"), "value": b.get("value")}
    for g, _ in GROUPS:
        e = dict(stats.get(g, {}))
        if g in fetch and g in write:
            rd = 2.0 * fetch[g]["kib"] * 1024 / fetch[g]["launches"]
            wr = write[g]["kib"] * 1024 / write[g]["launches"]
            e.update({"hbm_read_bytes_per_launch": round(rd), "hbm_write_bytes_per_launch": round(wr),
                      "hbm_bytes_per_launch": round(rd + wr), "pmc_launches": fetch[g]["launches"]})
        if g in mfma:
            e.update(mfma[g])
        if e:
            e.pop("total_ns", None)
            res["groups"][g] = e
    out = dst_p / "kernel_summary.json"
    out.write_text(json.dumps(res, indent=1) + "\n")
    if len(sys.argv) > 3:  # also publish as the PMC traffic bench.py reads for this workload
        res["source"] = str(out)
        (dst_p.parent / f"pmc_traffic_{sys.argv[3]}.json").write_text(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:3])
