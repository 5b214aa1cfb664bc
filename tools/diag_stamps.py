#!/usr/bin/env python3
"""Per-phase cycle shares of k_linearize from the diagnostic build (libmcc_diag.so, s_memtime
stamps at phase boundaries; cdna guide section 7 'In-kernel stamps').  Never quote this build's
run time: read its shares.

    MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so python tools/diag_stamps.py [config] [views]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_camera_calibration_amd import api, rig  # noqa: E402

PHASES = ["pending-update", "prologue", "sweep(wave0)", "reduce+barrier", "chain+H", "photo-chol", "Y/out"]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
    views = int(sys.argv[2]) if len(sys.argv) > 2 else None
    p = rig.make_config(cfg, n_views=views)
    ba = api.BundleAdjuster(p)
    ba.set_params(p.x0)
    ba.step(20)
    ba.synchronize()
    ba.stamps()          # arm
    ba.step(3)
    ba.synchronize()
    s = ba.stamps().astype(np.float64)
    t0 = s[:, 0]
    ok = t0 > 0
    s = s[ok]
    # stamp 3 is taken per sweep round by wave 0, 4 after each chain round: use the last values
    d = np.diff(s[:, :8], axis=1)
    print(f"{cfg}: {ok.sum()} workgroups stamped")
    for k, name in enumerate(PHASES):
        col = d[:, k]
        print(f"  {name:16s} median {np.median(col):9.0f}  p90 {np.percentile(col, 90):9.0f}  (s_memtime ticks)")
    tot = s[:, 7] - s[:, 0]
    print(f"  {'total':16s} median {np.median(tot):9.0f}  p90 {np.percentile(tot, 90):9.0f}")
    span = s[:, 7].max() - s[:, 0].min()
    print(f"  kernel span (first start -> last end): {span:.0f} ticks; start spread {s[:, 0].max() - s[:, 0].min():.0f}")


if __name__ == "__main__":
    main()
