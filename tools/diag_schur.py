#!/usr/bin/env python3
"""The m <= 30 split step's tail on the diagnostic build (libmcc_diag.so): when the last k_group
workgroup ends, when k_schur's item workgroups start and finish, and the final workgroup's phases
(ticks from the first k_group start, s_memtime).  Never quote this build's run time.

    MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so python tools/diag_schur.py [config] [views]
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
for rep in range(3):
    ba.step(1)
    ba.synchronize()
    raw = ba.stamps().reshape(-1)
    nv = max(p.n_photos, 1)
    ph = raw[:32 * nv].reshape(nv, 32)
    sch = raw[32 * nv:].reshape(-1, 8)
    sch = sch[(sch != 0).any(axis=1)]
    g0 = ph[:, 0][ph[:, 0] > 0]
    t0 = g0.min()
    gend = ph[:, 10][ph[:, 10] > 0]
    print(f"rep {rep}: k_group {len(g0)} groups: start spread {g0.max() - t0}, end median {np.median(gend) - t0:.0f}, last {gend.max() - t0}")
    fin = sch[sch[:, 7] > 0]
    items = sch[sch[:, 7] == 0]
    if len(items):
        print(f"  k_schur items: {len(items)}, start min {items[:, 0].min() - t0}, items summed max {items[:, 1].max() - t0}, level-1 max {items[:, 2].max() - t0}")
    for f in fin:
        names = ["solve entry", "GJ start (w1)", "GJ end (w1)", "final: before packed loads", "stop-test barrier", "-", "camera update", "end"]
        print("  final WG: " + ", ".join(f"{n} {v - t0}" for n, v in zip(names, f) if v))
ba.close()
