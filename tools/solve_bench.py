"""k_solve's dense elimination alone (mcc_debug_solve): device microseconds per solve and the
per-phase stamp deltas (s_memtime ticks of thread 0) for a few m.  Usage: python tools/solve_bench.py [m ...]"""
import sys

import numpy as np

sys.path.insert(0, ".")
from multi_camera_calibration_amd import api  # noqa: E402
from tests.test_dense_solve import spd  # noqa: E402

ms = [int(a) for a in sys.argv[1:]] or [48, 90, 126]
for m in ms:
    S, r = spd(m, 1e4, seed=m, camera_scaling=True)
    x, us, st = api.debug_solve(S, r, reps=200, stamps=True)
    ok = np.allclose(S @ x, r, rtol=0, atol=1e-9 * np.abs(r).max())
    nb = (m + 15) // 16
    t0 = st[0]
    print(f"m={m}: {us:.2f} us/solve (200 launches), residual ok={ok}; stamps (ticks from slot 0):")
    row = []
    for kb in range(nb):
        a, b, c = st[1 + 3 * kb] - t0, st[2 + 3 * kb] - t0, st[3 + 3 * kb] - t0
        extra = ""
        if kb + 1 < nb and st[40 + kb]:
            extra = (f"  [w0 item done {st[40 + kb] - t0}, inverse done {st[48 + kb] - t0}; "
                     f"w1 items done {st[56 + kb] - t0}]")
        row.append(f"kb{kb}: start {a} scaled {b} elim {c}{extra}")
    print("   " + "\n   ".join(row))
    print(f"   end {st[63] - t0}")
