"""float32 ulp distance, the parity unit of the float32 parameter state (src/multicalib.cpp:426,
495-501 keep x in CV_32F)."""
import numpy as np


def _ordered(a):
    i = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    return np.where(i < 0, -(i & 0x7FFFFFFF), i)   # monotonic in the float value, +0 == -0


def f32_ulp_diff(a, b):
    """|a - b| in float32 ulps, elementwise (0 = bitwise equal up to the sign of zero)."""
    return np.abs(_ordered(a) - _ordered(b))
