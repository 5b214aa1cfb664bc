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
