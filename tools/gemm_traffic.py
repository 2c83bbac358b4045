"""Per-launch HBM traffic of the expert GEMMs against their algorithmic bytes
(which launch carries the excess of the grouped-GEMM
group's PMC traffic over its algorithmic bytes).

Inputs, from one eager (--no-graphs) bench command run three times on the box
(tools/gpu_gemm_traffic.sh):
  records.json          bench.py --dump-prof-records: the timed step's library
                        records in launch order (kind, ms, flops, algorithmic bytes)
  fetch/…counter_collection.csv, write/…counter_collection.csv
                        rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over the
                        same command (gfx950 corrections as tools/profile_summary.py:
                        KiB; FETCH_SIZE doubled)
The expert-GEMM dispatches of the timed step are the LAST n rows of each PMC
pass whose kernel is an expert GEMM (n = the records of kind grouped_gemm);
they are joined by position.

    python tools/gemm_traffic.py <dir> [out.json]
"""
from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

EXPERT = re.compile(r"gemm_v\d_kernel|gemm_pair_kernel|gemm_triple_kernel|expert_ffn_fwd_kernel")
DENSE = re.compile(r"gemm_v\d_kernel<[^>]*, 16>")


def short(name: str) -> str:
    n = re.sub(r"\(.*", "", name).replace("void ", "")
    if "gemm_triple" in n:
        return "gemm_triple"
    if "gemm_pair" in n:
        return "gemm_pair"
    if "expert_ffn_fwd" in n:
        return "expert_ffn_fwd"
    m = re.search(r"gemm_v2_kernel<(.*)>", n)
    return "gemm_v2<" + (m.group(1) if m else "?") + ">"


def pmc_rows(path: Path, counter: str):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            n = r["Kernel_Name"]
            if EXPERT.search(n) and not DENSE.search(n):
                rows.append((int(r["Dispatch_Id"]), n, int(r["Grid_Size"]), float(r["Counter_Value"])))
    rows.sort()
    return rows


def main():
    d = Path(sys.argv[1])
    rec = json.loads((d / "records.json").read_text())
    gem = [r for r in rec["records"] if r[0] == "grouped_gemm"]
    fetch = pmc_rows(next((d / "fetch").glob("*counter_collection.csv")), "FETCH_SIZE")
    write = pmc_rows(next((d / "write").glob("*counter_collection.csv")), "WRITE_SIZE")
    n = len(gem)
    if len(fetch) < n or len(write) < n:
        raise SystemExit(f"fewer PMC rows ({len(fetch)}, {len(write)}) than records ({n})")
    fetch, write = fetch[-n:], write[-n:]
    per = []
    agg = defaultdict(lambda: {"launches": 0, "alg": 0.0, "read": 0.0, "write": 0.0, "ms": 0.0, "flops": 0.0})
    for (kind, ms, fl, by), (_, name, grid, fk), (_, name2, _, wk) in zip(gem, fetch, write):
        if short(name) != short(name2):
            raise SystemExit(f"FETCH and WRITE passes disagree: {name} vs {name2}")
        rd, wr = 2.0 * fk * 1024, wk * 1024
        key = f"{short(name)} grid {grid // 256}"
        per.append({"kernel": key, "alg_bytes": by, "pmc_read": rd, "pmc_write": wr, "ratio": (rd + wr) / max(by, 1)})
        a = agg[key]
        a["launches"] += 1
        a["alg"] += by
        a["read"] += rd
        a["write"] += wr
        a["ms"] += ms
        a["flops"] += fl
    tot_alg = sum(a["alg"] for a in agg.values())
    tot_pmc = sum(a["read"] + a["write"] for a in agg.values())
    print(f"{n} expert-GEMM launches: algorithmic {tot_alg / 1e6:.1f} MB, PMC {tot_pmc / 1e6:.1f} MB "
          f"({tot_pmc / tot_alg:.3f}x)")
    print(f"{'kernel':58s} {'n':>3s} {'alg MB':>8s} {'read MB':>8s} {'write MB':>8s} {'ratio':>6s} "
          f"{'excess MB':>9s} {'avg us':>7s}")
    rows = []
    for k, a in sorted(agg.items(), key=lambda kv: -(kv[1]["read"] + kv[1]["write"] - kv[1]["alg"])):
        L = a["launches"]
        ex = (a["read"] + a["write"] - a["alg"]) / 1e6
        print(f"{k:58s} {L:3d} {a['alg'] / L / 1e6:8.2f} {a['read'] / L / 1e6:8.2f} {a['write'] / L / 1e6:8.2f} "
              f"{(a['read'] + a['write']) / a['alg']:6.2f} {ex:9.2f} {1e3 * a['ms'] / L:7.1f}")
        rows.append({"kernel": k, "launches": L, "alg_bytes_per_launch": a["alg"] / L,
                     "pmc_read_per_launch": a["read"] / L, "pmc_write_per_launch": a["write"] / L,
                     "ratio": (a["read"] + a["write"]) / a["alg"], "excess_mb_total": ex,
                     "avg_us_eager_events": 1e3 * a["ms"] / L})
    if len(sys.argv) > 2:
        Path(sys.argv[2]).write_text(json.dumps({"source": str(d), "launches": n, "alg_bytes": tot_alg,
                                                 "pmc_bytes": tot_pmc, "ratio": tot_pmc / tot_alg,
                                                 "kernels": rows, "per_launch": per}, indent=1))


if __name__ == "__main__":
    main()
