#!/usr/bin/env python3
"""Per-step warm-solve statistics of the m > 30 path (one step at a time), for the helper-refine and
k_solve-refine forms:  python3 tools/warm_trace.py [config3] [views] [n_cams] [steps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_camera_calibration_amd import api, rig  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "config3"
views = int(sys.argv[2]) if len(sys.argv) > 2 else 40
cams = int(sys.argv[3]) if len(sys.argv) > 3 else 9
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 12
p = rig.make_config(cfg, n_cams=cams, n_views=views)
for hr in ("0", "1"):
    os.environ["MCC_HELPER_REFINE"] = hr
    ba = api.BundleAdjuster(p)
    ba.set_params(p.x0)
    prev = ba.solve_stats()
    seq = []
    for s in range(steps):
        ba.step(1)
        ba.synchronize()
        st = ba.solve_stats()
        seq.append("".join(k[0] for k in ("warm", "direct", "fallbacks", "waited") if st[k] != prev[k]) or "-")
        prev = st
    print("MCC_HELPER_REFINE", hr, " ".join(seq), prev)
    x, m, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
    print("  optimize it", it, ba.solve_stats())
    ba.close()
