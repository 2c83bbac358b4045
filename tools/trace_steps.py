"""Per-step kernel-time breakdown of the timed region from a rocprofv3
kernel trace (csv): the last `--steps` steps are found as the window between
the last `--steps`+1 launches of the step-marker kernel (the fused AdamW
update), and kernels are grouped into categories.

  python tools/trace_steps.py gpurun_out/<tag>/prof/run_kernel_trace.csv --steps 10
"""
import argparse
import csv
import re
from collections import defaultdict


def category(n):
    if "moe::" in n:
        return "moe:" + n.split("moe::")[1].split("<")[0].split("(")[0]
    if n.startswith("igemm") or "conv" in n.lower() or "MIOpen" in n:
        return "conv/bn (MIOpen, CK)"
    if n.startswith("Cijk"):
        return "hipBLASLt GEMM"
    if "attn_fwd" in n or "bwd_kernel_d" in n or "bwd_preprocess" in n:
        return "attention (aotriton)"
    if "ck::" in n:
        return "CK other"
    if "rocclr_fill" in n:
        return "memset"
    if "rocclr_copy" in n:
        return "memcpy"
    if "at::native" in n:
        m = re.search(r"at::native::(?:\(anonymous namespace\)::)?(?:[a-z_]+_kernel[^<(]*<[^,>]*, )?(?:at::native::)?"
                      r"(?:\(anonymous namespace\)::)?([A-Za-z_0-9]+)", n)
        return "torch:" + (m.group(1) if m else n[:40])
    return n[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default="adamw_step_kernel", help="kernel launched once per step (torch fused AdamW: FusedAdamMathFunctor)")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--skip", type=int, default=0,
                    help="ignore the last N steps (bench.py's eager kernel-timing steps follow the timed graph replays)")
    ap.add_argument("--full", default=None, help="regex over categories: list those kernels by full name + grid")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    # last marker launch of each step: markers come in bursts (one per param group)
    ends = [marks[j] for j in range(len(marks)) if j + 1 == len(marks) or
            int(rows[marks[j + 1]]["Start_Timestamp"]) - int(rows[marks[j]]["End_Timestamp"]) > 1_000_000]
    if a.skip:
        ends = ends[: -a.skip]
    lo, hi = ends[-a.steps - 1] + 1, ends[-1] + 1
    win = rows[lo:hi]
    span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e6 / a.steps
    busy = defaultdict(float)
    cnt = defaultdict(int)
    for r in win:
        c = category(r["Kernel_Name"])
        busy[c] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / a.steps
        cnt[c] += 1
    tot = sum(busy.values())
    print(f"steps {a.steps}: wall {span:.2f} ms/step, kernel busy {tot:.2f} ms/step, "
          f"{len(win) / a.steps:.0f} launches/step")
    for c, v in sorted(busy.items(), key=lambda x: -x[1])[: a.top]:
        print(f"{v:7.3f} ms {100 * v / tot:5.1f}%  {cnt[c] / a.steps:6.1f}/step  {c}")
    if a.full:
        gcol = next((k for k in ("Grid_Size", "Grid_Size_X", "Grid_X") if k in win[0]), None)
        fb, fc = defaultdict(float), defaultdict(int)
        for r in win:
            if not re.search(a.full, category(r["Kernel_Name"])):
                continue
            key = (r["Kernel_Name"][:140], r.get(gcol, "?") if gcol else "?")
            fb[key] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 / a.steps
            fc[key] += 1
        print(f"# kernels of categories /{a.full}/ by full name and grid ({gcol})")
        for (n, gsz), v in sorted(fb.items(), key=lambda x: -x[1])[:80]:
            k = fc[(n, gsz)] / a.steps
            print(f"{v:7.3f} ms {k:6.1f}/step {1e3 * v / max(k, 1e-9):8.1f} us  grid {gsz:>9}  {n}")


if __name__ == "__main__":
    main()
