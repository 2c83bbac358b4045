"""Margin report of the element-wise bf16 comparisons (tolerance tuning):
with BF16_CLOSE_REPORT=<file> every call appends one JSON line with the
largest error beyond one bf16 ulp of the reference, in units of the
reference's RMS, and the fraction of elements beyond one ulp."""
import json
import os

import numpy as np


def report(what, got, ref):
    path = os.environ.get("BF16_CLOSE_REPORT")
    if not path:
        return
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(got - ref)
    rms = max(float(np.sqrt((ref ** 2).mean())), 1e-12)
    excess = np.maximum(err - 2.0 ** -8 * np.abs(ref), 0.0) / rms
    with open(path, "a") as f:
        f.write(json.dumps({"what": what, "n": int(ref.size), "max_excess_over_rms": float(excess.max()),
                            "p999_excess_over_rms": float(np.quantile(excess, 0.999)),
                            "p99_excess_over_rms": float(np.quantile(excess, 0.99)),
                            "frac_beyond_1ulp": float((err > 2.0 ** -8 * np.abs(ref)).mean()),
                            "max_over_maxref": float(err.max() / max(float(np.abs(ref).max()), 1e-12)),
                            "rms_over_maxref": rms / max(float(np.abs(ref).max()), 1e-12)}) + "\n")
