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
    raw = ba.stamps().reshape(-1)
    nv = max(p.n_photos, 1)
    lin = raw[:16 * nv].reshape(nv, 16).astype(np.float64)
    sch = raw[16 * nv:].reshape(-1, 8).astype(np.float64)
    s = lin
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
    ok = sch[:, 0] > 0
    it = sch[ok]
    print(f"k_schur: {ok.sum()} workgroups; item compute median {np.median(it[:, 1] - it[:, 0]):.0f}, "
          f"ticket median {np.median(it[:, 2] - it[:, 1]):.0f} (non-last rows have 0 in slot 2)")
    last = sch[sch[:, 3] > 0]
    if len(last):
        L = last[0]
        names = ["start", "items", "acquire", "assembly", "stoptest", "crout", "trisolve", "end"]
        print("  last arriver: " + ", ".join(f"{names[k]}->{names[k+1]} {L[k+1]-L[k]:.0f}" for k in range(7)))
        print(f"  kernel span {sch[ok, 0].min():.0f} -> {L[7]:.0f}: {L[7] - sch[ok, 0].min():.0f} ticks; "
              f"last item start {sch[ok, 0].max() - sch[ok, 0].min():.0f} after the first")


if __name__ == "__main__":
    main()
