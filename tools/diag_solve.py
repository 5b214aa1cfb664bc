#!/usr/bin/env python3
"""Per-phase shader-clock stamps of k_solve's m > 30 warm solve (MCC_DIAG build: make diag ->
libmcc_diag.so, run with MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so).  Median over
repetitions of the last step's k_solve row:
  0 entry | 4 state + packed loads + epochs checked (barrier) | 8 [S | r] staged in LDS (epoch
  published here when there is no inverse to use) | 9 S_t^-1 loaded into LDS, rows of S gathered
  (epoch published) | 10 refined | 11 after the direct elimination, if any | 5 after the solve |
  6 camera update written
    python tools/diag_solve.py [config3] [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multi_camera_calibration_amd import api, rig  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "config3"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
p = rig.make_config(name)
ba = api.BundleAdjuster(p)
ba.set_params(p.x0)
ba.step(30)
ba.synchronize()
ba.stamps()   # arm
rows = []
for r in range(reps):
    ba.step(5)
    ba.synchronize()
    st = ba.stamps()
    rows.append(st)
ba.close()
# k_solve's row is the last 16-slot row of the device buffer (after k_linearize's 32-slot rows per
# photo and k_schur's 16-slot rows; mcc_debug_stamps' layout): the row of the last nonzero stamp
nv = max(p.n_photos, 1)
last = int(np.nonzero(rows[-1])[0].max())
base = 32 * nv + 16 * ((last - 32 * nv) // 16)
labels = {0: "entry", 4: "loads+epochs", 8: "staged", 9: "Sinv in LDS", 10: "refined", 11: "after GJ",
          5: "solved", 6: "update"}
order = [0, 4, 8, 9, 10, 11, 5, 6]
vals = np.array([[r[base + k] for k in order] for r in rows], dtype=np.int64)
d = np.diff(vals, axis=1)
med = np.median(d, axis=0)
for (a, b), v in zip(zip(order, order[1:]), med):
    print(f"{labels[a]:>20s} -> {labels[b]:<20s} {v:9.0f} cycles")
print(f"{'total':>20s}    {np.median(vals[:, -1] - vals[:, 0]):9.0f} cycles")
