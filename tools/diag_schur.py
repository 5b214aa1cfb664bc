#!/usr/bin/env python3
"""The m <= 30 split step's tail on the diagnostic build (libmcc_diag.so): when the last k_group
workgroup ends, when k_schur's item workgroups start and finish, and the final workgroup's phases
(ticks from the first k_group start, s_memtime).  Never quote this build's run time.

    MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so python tools/diag_schur.py [config] [views]

With a -DMCC_DIAG_RT build (the chip-wide 100 MHz s_memrealtime; s_memtime is per XCD, so its
cross-workgroup differences are meaningless) set MCC_DIAG_RT=1: times are then printed in us.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_camera_calibration_amd import api, rig  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config4"
views = int(sys.argv[2]) if len(sys.argv) > 2 else None
p = rig.make_config(cfg, n_views=views)
ba = api.BundleAdjuster(p)
ba.set_params(p.x0)
ba.step(20)
ba.synchronize()
ba.stamps()
RT = os.environ.get("MCC_DIAG_RT") == "1"
SC = 0.01 if RT else 1.0   # 100 MHz ticks -> us


def q(v):
    return f"{v * SC:.2f}" if RT else f"{v:.0f}"


for rep in range(3):
    ba.step(1)
    ba.synchronize()
    raw = ba.stamps().reshape(-1)
    nv = max(p.n_photos, 1)
    ph = raw[:32 * nv].reshape(nv, 32)
    sch = raw[32 * nv:-16].reshape(-1, 16)
    sch = sch[(sch != 0).any(axis=1)]
    g0 = ph[:, 0][ph[:, 0] > 0]
    t0 = g0.min()
    gend = ph[:, 10][ph[:, 10] > 0]
    print(f"rep {rep}: k_group {len(g0)} groups: start spread {q(g0.max() - t0)}, end median {q(np.median(gend) - t0)}, last {q(gend.max() - t0)}"
          + (" (us)" if RT else " (ticks)"))
    ok = (ph[:, 0] > 0) & (ph[:, 10] > 0)
    if ok.any():   # k_group's phases (slots 1..10 from the group's own start), median over groups
        rel = ph[ok][:, 1:11] - ph[ok][:, :1]
        print("  k_group phases (median from group start): " + " ".join(
            f"{k}:{q(np.median(rel[:, k - 1]))}" for k in range(1, 11) if (rel[:, k - 1] > 0).any()))
    if ok.any():   # per wave: the edge rounds done (slots 16 + wave), median over groups
        w = ph[ok][:, 16:24] - ph[ok][:, :1]
        print("  k_group rounds done per wave (median from group start): " + " ".join(
            f"w{k}:{q(np.median(w[:, k]))}" for k in range(8) if (w[:, k] > 0).all()))
    fin = sch[sch[:, 7] > t0]   # (rows of earlier launches: stale final stamps, skipped)
    items = sch[sch[:, 7] == 0]
    if len(items):
        lv1 = items[:, 2][items[:, 2] > 0]
        print(f"  k_schur items: {len(items)}, start min {q(items[:, 0].min() - t0)} max {q(items[:, 0].max() - t0)}, "
              f"items summed max {q(items[:, 1].max() - t0)}, level-1 max {q(lv1.max() - t0) if len(lv1) else '-'}")
    for f in fin:
        names = ["solve entry", "GJ start (w1)", "GJ end (w1)", "final: before packed loads", "stop-test barrier", "-",
                 "camera update", "end", "one level: batch landed", "sums placed", "fold: final start"]
        print("  final WG: " + ", ".join(f"{n} {q(v - t0)}" for n, v in zip(names, f) if v))
ba.close()
