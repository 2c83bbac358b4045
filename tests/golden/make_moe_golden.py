"""Generate the MoE-layer golden fixtures from the CPU oracle (build container).

SURVEY.md 7.1: golden vectors for every BASELINE config, made by the build's
own float64 oracle (oracle/moe_oracle.py; the reference has no MoE code, so a2-a7
parity is "unpinned" -- these fixtures pin the GPU path and the oracle against
the same numbers over time).  Inputs are NOT stored: tests/moe_cases.py
regenerates them from each case's seed.  Per case, tests/golden/moe_<name>.npz
holds the oracle's outputs for loss = <dy, y> + 0.7 lb + 0.3 z (bf16-expert
cases with the single-GPU layer's fused-dgrad rounding points,
moe_oracle.moe_backward(fused_dgrad=True); MXFP8 cases without):

  idx int8 [T,k], pos int32 [T,k] (-1 = dropped), hist int32 [E], offsets int32 [E+1]
  margin fp32 [T]          top-(k+1) logit gap per token (routing tie distance)
  lb, z                    aux losses
  y, dx uint16 [T/s,d]     bf16 bit patterns of tokens t % s == 0, s = tok_stride (the
                           oracle emulates the GPU's bf16 stores); y_sum, dx_sum over all tokens
  dwg [E,d], dctx_bias [6,E], db1 [E,F], db2 [E,d]   fp32
  dw1_rows [E,4,d], dw2_rows [E,4,F]                4 output rows per expert, fp32
  dw1_sum/_sumsq, dw2_sum/_sumsq                    full-tensor checksums (float64)

Usage:  python tests/golden/make_moe_golden.py [name ...]
"""
from __future__ import annotations

import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]
for p in (str(ROOT), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import moe_cases as MC  # noqa: E402


def main(names):
    for name in names or list(MC.GOLDEN):
        c = MC.GOLDEN[name]
        t0 = time.perf_counter()
        st, gr = MC.run_oracle(c, MC.make_inputs(c), fused_dgrad=not c.mx)
        out = HERE / f"moe_{name}.npz"
        np.savez_compressed(out, **MC.summarize(c, st, gr))
        print(f"{out.name}: {out.stat().st_size / 1e6:.2f} MB, {time.perf_counter() - t0:.1f} s")


if __name__ == "__main__":
    main(sys.argv[1:])
