#!/usr/bin/env python3
"""Per-phase s_memtime shares of the split step's kernels (k_prep, k_edge, k_photo) from the
diagnostic build (libmcc_diag.so).  Never quote this build's run time: read its shares.

    MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so python tools/diag_split.py [config] [views]

k_group (the split step's group kernel) group g -> row g slots 0..10 (start, loads, photo update and
Rodrigues, round 0's prologue, sweep, chain, the later rounds, Hpp sums, Cholesky, U / Y', pairs).
Otherwise rows of the stamp buffer (32 slots each): k_photo photo p -> row p slots 0..5 (start, staged,
Cholesky, U / Y', pairs stored; slot 2 unused); k_prep workgroup w -> row w slots 8..11 (start, update,
photo Rodrigues, edges stored); k_edge workgroup w -> row w / 2 slots 16 + 8 (w & 1) + 0..4
(start, corners staged, sweep, butterfly, H stored).
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_camera_calibration_amd import api, rig  # noqa: E402


def med(v):
    v = v[v > 0]
    return f"median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}  (n={len(v)})" if len(v) else "n/a"


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
    views = int(sys.argv[2]) if len(sys.argv) > 2 else None
    p = rig.make_config(cfg, n_views=views)
    os.environ.setdefault("MCC_FUSED", "0")
    ba = api.BundleAdjuster(p)
    ba.set_params(p.x0)
    ba.step(20)
    ba.synchronize()
    ba.stamps()          # arm
    ba.step(1)
    ba.synchronize()
    raw = ba.stamps().reshape(-1)
    nv = max(p.n_photos, 1)
    s = raw[:32 * nv].reshape(nv, 32).astype(np.float64)

    def phases(cols, names, title):
        blk = s[:, cols]
        ok = (blk > 0).all(axis=1)
        d = np.diff(blk[ok], axis=1)
        print(f"{title}: {ok.sum()} workgroups")
        for k, n in enumerate(names):
            print(f"  {n:22s} {med(d[:, k])}")
        print(f"  {'total':22s} {med(blk[ok][:, -1] - blk[ok][:, 0])}")

    if ba.step_kernels() == "k_group":
        ng = int(np.count_nonzero(s[:, 0]))
        phases(list(range(11)), ["loads (round trip 1)", "photo update+Rodrigues", "edge prologue (r0)", "sweep (r0)",
                                 "butterfly+chain (r0)", "later rounds", "photo Hpp sums", "Cholesky", "U, Y'",
                                 "pairs+store"], f"k_group ({ng} groups)")
        return
    phases([0, 1, 3, 4, 5], ["load+stage+sums", "Cholesky, Li", "U, Y'", "pairs+store"], "k_photo")
    phases([8, 9, 10, 11], ["photo update", "photo Rodrigues", "edge prologues"], "k_prep")
    for h in (0, 1):
        base = 16 + 8 * h
        phases([base, base + 1, base + 2, base + 3, base + 4], ["stage corners", "sweep", "butterfly", "chain+store"],
               f"k_edge (half {h})")


if __name__ == "__main__":
    main()
