"""Per-kernel time of one training step from a rocprofv3 kernel trace of
bench.py (``--kernel-trace --output-format csv``).  Steps are delimited by the
AdamW launch (one per step); the graph-replay steps are the windows with the
fewest launches (the eager warm-up and the dispatch-timing steps launch ~4x
more).  The last ``--steps`` such windows are summarised.

    python tools/step_breakdown.py <run_kernel_trace.csv> [--steps 10] [--top 40] > step_breakdown.txt
"""
from __future__ import annotations

import argparse
import csv
import re
from collections import defaultdict


def short(name: str) -> str:
    n = name.split("(")[0]
    n = re.sub(r"<.*", "", n)
    n = n.replace("void ", "").strip()
    if "Cijk_" in name:
        return "hipBLASLt GEMM"
    if n.startswith("__amd_rocclr"):
        return "memcpy"
    if "at::native" in n or n.startswith("at::"):
        m = re.search(r"(\w+_kernel\w*|CUDAFunctor_\w+|\w+Functor\w*)", name)
        return "torch:" + (m.group(1) if m else n.split("::")[-1])
    return "moe:" + n.split("::")[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if "adamw_step_kernel" in r[2]]
    wins = [(ends[j] + 1, ends[j + 1] + 1) for j in range(len(ends) - 1)]
    if not wins:
        raise SystemExit("no AdamW-delimited steps in the trace")
    counts = [b - e for e, b in wins]
    lo = min(counts)
    graph = [w for w, c in zip(wins, counts) if c <= lo * 1.1]
    sel = graph[-a.steps:]
    per = defaultdict(lambda: [0.0, 0])
    busy = 0.0
    for s, e in sel:
        for t0, t1, n in rows[s:e]:
            k = short(n)
            per[k][0] += (t1 - t0) * 1e-6
            per[k][1] += 1
            busy += (t1 - t0) * 1e-6
    n = len(sel)
    wall = (rows[sel[-1][1] - 1][1] - rows[sel[0][0] - 1][1]) * 1e-6 / n
    launches = sum(v[1] for v in per.values()) / n
    print(f"steps {n}: wall {wall:.2f} ms/step, kernel busy {busy / n:.2f} ms/step, {launches:.0f} launches/step")
    for k, (ms, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:a.top]:
        print(f"{ms / n:8.3f} ms {100 * ms / busy:5.1f}% {c / n:8.1f}/step  {k}")


if __name__ == "__main__":
    main()
