"""How many float32 residuals of the GPU path differ from the oracle's, per config.

    python tools/ulp_report.py [--out profiles/r05_ulp_report.json] [config ...]

For each BASELINE config at full size (and the small fixtures' shapes), mcc_debug_residuals (the
linearisation kernels' own sweep: k_linearize / k_group / k_edge) against the oracle's per-edge
restatement (ora_edge_linearize) at x0: the number of corners' residual components that differ, and
the largest difference in float32 ulps.  The device's matrix -> vector Rodrigues of the composed pose
skips the polar re-orthonormalisation OpenCV applies (mcc_device.hpp rodrigues_m2v vs
oracle/mcc_oracle.c polar3); the differences this report counts are where that, or a 1-ulp tie of an FP64
transcendental, moves the float32 composed pose or pixel by one ulp."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_camera_calibration_amd import api, rig  # noqa: E402
from oracle import oracle_py as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("configs", nargs="*", default=["config1", "config2", "config3", "config4", "config5"])
ap.add_argument("--out", default=None)
ap.add_argument("--final", default=None, metavar="DIR",
                help="collect the final-iterate records the GPU parity tests wrote with MCC_PARITY_REPORT=DIR "
                     "(tests/test_full_size.py::test_full_size_optimize, tests/test_peer_transport.py::"
                     "test_peer_ranks_one_device) into --out instead")
args = ap.parse_args()
if args.final:
    recs = {}
    for fn in sorted(os.listdir(args.final)):
        if fn.endswith(".json"):
            r = json.load(open(os.path.join(args.final, fn)))
            recs[r["case"]] = r
            print(r["case"], {k: r[k] for k in ("differ", "params", "max_ulp", "state_resolution_diff",
                                                  "iters_gpu", "iters_oracle", "mean_abs_diff_px")}, flush=True)
    res = {"what": "final optimizeExtrinsics iterates (COUNT+EPS, 200, eps 1e-7, from x0) of the GPU path against the "
                   "oracle's on the whole problem: float32 parameters that differ, the largest difference in ulps, "
                   "an ulp histogram, and state_resolution_diff (tests/ulp.py: the difference in units of the "
                   "float32 spacing of the largest rotation / translation the state holds; the full-size bar is "
                   "<= 2); *_x1 from tests/test_full_size.py, *_xN from tests/test_peer_transport.py (N ranks as "
                   "processes on one device, peer transport)",
           "cases": recs}
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)
    sys.exit(0)
rows = {}
for cfg in args.configs:
    t0 = time.time()
    p = rig.make_config(cfg)
    ba = api.BundleAdjuster(p)
    try:
        r = ba.residuals(p.x0)
        kern = ba.step_kernels()
    finally:
        ba.close()
    o = O.Oracle(p)
    ref = np.concatenate([o.edge_linearize(p.x0, e)[2] for e in range(p.n_edges)]).astype(np.float32)
    diff = r != ref
    ulp = np.abs(r.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))[diff]
    rows[cfg] = {"kernels": kern, "corners": int(p.n_corners), "residual_components": int(r.size),
                 "differ": int(diff.sum()), "differ_fraction": float(diff.mean()),
                 "max_ulp": int(ulp.max()) if ulp.size else 0,
                 "edges_with_a_difference": int(len({int(e) for e in np.repeat(np.arange(p.n_edges), 2 * p.edge_n)[diff]})),
                 "seconds": round(time.time() - t0, 1)}
    print(cfg, rows[cfg], flush=True)
res = {"what": "float32 residual components of the GPU sweep (mcc_debug_residuals) that differ from the oracle "
               "(ora_edge_linearize) at x0, full BASELINE sizes", "configs": rows}
if args.out:
    json.dump(res, open(args.out, "w"), indent=1)
