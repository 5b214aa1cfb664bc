#!/usr/bin/env python3
"""The m > 30 split step's tail on the realtime-stamped diagnostic build (make -C
multi_camera_calibration_amd diagrt -> libmcc_diagrt.so): when the linearisation's last group ends,
k_schur's items start and finish, its two hand-off levels, and k_solve's phases (entry, the helper's
solution in, the camera update), in us from the first group's start (chip-wide 100 MHz clock).
Never quote this build's run time.

    MCC_LIB=multi_camera_calibration_amd/libmcc_diagrt.so python tools/diag_tail.py config3 [shard N] [reps]
With a shard N the problem is rank 0's photo shard of config3 split N ways (bench.py shard_line).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multi_camera_calibration_amd import api, rig  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
shard = int(sys.argv[2]) if len(sys.argv) > 2 else 1
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
full = rig.make_config(cfg)
if shard > 1:
    owner = api.partition_photos(full, shard)
    p = rig.subset_photos(full, np.nonzero(owner == 0)[0])
else:
    p = full
ba = api.BundleAdjuster(p)
print(f"{cfg} shard 1/{shard}: {p.n_photos} views, {p.n_edges} edges, path {ba.step_kernels()}, "
      f"{ba.photo_groups()} groups", flush=True)
ba.set_params(p.x0)
ba.step(40)
ba.synchronize()
steps_per_rep = int(os.environ.get("TAIL_STEPS", "1"))   # > 1: the last of a batch (a resident helper's steady state)
ba.stamps()   # arm
nv = max(p.n_photos, 1)
out = []
for r in range(reps):
    ba.step(steps_per_rep)
    ba.synchronize()
    raw = ba.stamps().reshape(-1).astype(np.int64)
    # the helper's [4 systems][16] at the buffer's end (-1 until written; slot 15 never is)
    hb = int(np.nonzero(raw == -1)[0].max()) - 63
    hst = raw[hb:hb + 64].reshape(4, 16).copy()
    raw[hb:] = 0
    ph = raw[:32 * nv].reshape(nv, 32)
    g0 = ph[:, 0][ph[:, 0] > 0]
    ge = ph[:, 10][ph[:, 10] > 0]
    if not len(g0):
        continue
    t0 = g0.min()
    last = int(np.nonzero(raw)[0].max())
    base = 32 * nv + 16 * ((last - 32 * nv) // 16)   # k_solve's row: the row of the last stamp
    sch = raw[32 * nv:base].reshape(-1, 16)
    sch = sch[(sch[:, 0] >= t0)]
    ks = raw[base:base + 16]
    us = lambda v: (v - t0) * 0.01   # noqa: E731
    row = {"groups_started_by": us(g0.max()), "group_end_median": us(np.median(ge)), "last_group_end": us(ge.max()),
           "schur_first_start": us(sch[:, 0].min()), "schur_items_done": us(sch[:, 1].max()),
           "level1_done": us(sch[:, 2][sch[:, 2] > 0].max()) if (sch[:, 2] > 0).any() else float("nan"),
           "level2_reached": us(sch[:, 4][sch[:, 4] > 0].max()) if (sch[:, 4] > 0).any() else float("nan"),
           "solve_entry": us(ks[0]), "solve_loads": us(ks[4]) if ks[4] else float("nan"),
           "solve_x_in": us(ks[11]) if ks[11] else float("nan"), "solve_done": us(ks[5]) if ks[5] else float("nan"),
           "camera_update": us(ks[6]) if ks[6] else float("nan")}
    # the helper: this step's system (the largest epoch) seen, staged, refined, x published; the
    # previous system's inversion end
    cur = int(np.argmax(hst[:, 7]))
    e = int(hst[cur, 7])
    prv = [i for i in range(4) if hst[i, 7] == e - 1]
    for k, name in enumerate(("helper_seen", "helper_staged", "helper_gathered", "helper_refined", "helper_x_published")):
        row[name] = us(hst[cur, k]) if hst[cur, k] > 0 else float("nan")
    row["helper_prev_inverted"] = us(hst[prv[0], 5]) if prv and hst[prv[0], 5] > 0 else float("nan")
    row["helper_inverted"] = us(hst[cur, 5]) if hst[cur, 5] > 0 else float("nan")
    row["helper_corrections"] = float(hst[cur, 6])
    out.append(row)
ba.close()
keys = list(out[0])
print("median over", len(out), "steps (us from the first group's start):")
for k in keys:
    v = np.array([o[k] for o in out])
    print(f"  {k:>20s} {np.nanmedian(v):8.2f}   (min {np.nanmin(v):7.2f}, max {np.nanmax(v):7.2f})")
print(f"  tail after the last group: {np.nanmedian([o['camera_update'] - o['last_group_end'] for o in out]):.2f} us")
