"""float32 ulp distance, the parity unit of the float32 parameter state (src/multicalib.cpp:426,
495-501 keep x in CV_32F)."""
import numpy as np


def _ordered(a):
    i = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    return np.where(i < 0, -(i & 0x7FFFFFFF), i)   # monotonic in the float value, +0 == -0


def f32_ulp_diff(a, b):
    """|a - b| in float32 ulps, elementwise (0 = bitwise equal up to the sign of zero)."""
    return np.abs(_ordered(a) - _ordered(b))


def state_resolution_diff(a, b):
    """max |a - b| per parameter class in units of the float32 spacing of that class's largest
    magnitude: rotation components (6k .. 6k+2) and translation components (6k+3 .. 6k+5) of the
    [rvec, tvec] blocks buildParas lays out (src/multicalib.cpp:422-440).  1 means the
    difference is one ulp of the largest rotation / translation the state holds."""
    a = np.asarray(a, np.float32).reshape(-1, 6)
    b = np.asarray(b, np.float32).reshape(-1, 6)
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    out = 0.0
    for cols in (slice(0, 3), slice(3, 6)):
        res = float(np.spacing(np.float32(np.abs(b[:, cols]).max())))
        out = max(out, float(d[:, cols].max()) / res)
    return out


def report(case, x, x_ref, **extra):
    """MCC_PARITY_REPORT=<dir>: one JSON record per final-iterate comparison (tools/ulp_report.py --final
    collects them): how many float32 parameters differ from the oracle's, by how many ulps, and the
    state-resolution distance the full-size bar uses."""
    import json
    import os
    d = os.environ.get("MCC_PARITY_REPORT")
    if not d:
        return
    ulp = f32_ulp_diff(x, x_ref)
    hist = {"0": int((ulp == 0).sum()), "1": int((ulp == 1).sum()), "2-4": int(((ulp >= 2) & (ulp <= 4)).sum()),
            "5-16": int(((ulp >= 5) & (ulp <= 16)).sum()), "17-256": int(((ulp >= 17) & (ulp <= 256)).sum()),
            ">256": int((ulp > 256).sum())}
    rec = dict(case=case, params=int(ulp.size), differ=int((ulp > 0).sum()), max_ulp=int(ulp.max()),
               ulp_histogram=hist, state_resolution_diff=float(state_resolution_diff(x, x_ref)), **extra)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"{case}.json"), "w") as f:
        json.dump(rec, f, indent=1)
