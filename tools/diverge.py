"""Where the GPU's optimizeExtrinsics iterate first leaves the oracle's (a config at full size): for
k = 1 .. K, both run exactly k Gauss-Newton updates from x0 (crit COUNT, src/multicalib.cpp:475-477) and
the float32 states are compared; plus the first linearisation's solved step Delta and JTE.

    python tools/diverge.py config5 [--steps 6] [--out gpurun_out/diverge_config5.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from multi_camera_calibration_amd import api, rig  # noqa: E402
from oracle import oracle_py as O  # noqa: E402
from ulp import f32_ulp_diff, state_resolution_diff  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("config")
ap.add_argument("--steps", type=int, default=6)
ap.add_argument("--views", type=int, default=None)
ap.add_argument("--out", default=None)
args = ap.parse_args()
p = rig.make_config(args.config, n_views=args.views) if args.views else rig.make_config(args.config)
o = O.Oracle(p)
g = api.BundleAdjuster(p)
out = {"config": args.config, "views": p.n_photos, "path": g.step_kernels(), "steps": []}
try:
    d_ref, j_ref = o.linearize_solve(p.x0, "schur")
    d, j = g.compute_jacobian_extrinsic(p.x0)
    m = p.global_dim
    out["delta_rel"] = float(np.abs(d - d_ref).max() / np.abs(d_ref).max())
    out["delta_global_rel"] = float(np.abs(d[:m] - d_ref[:m]).max() / np.abs(d_ref[:m]).max())
    out["jte_rel"] = float(np.abs(j - j_ref).max() / np.abs(j_ref).max())
    print({k: out[k] for k in ("delta_rel", "delta_global_rel", "jte_rel")}, flush=True)
    # at the first common iterate x1 (one update; bitwise equal on every config so far): residuals,
    # JTE and the solved step, to tell a linearisation difference from a solve difference
    x1, _, _, _ = o.optimize(p.x0, crit_type=1, max_count=1)
    r = g.residuals(x1)
    ref = np.concatenate([o.edge_linearize(x1, e)[2] for e in range(p.n_edges)]).astype(np.float32)
    diff = r != ref
    out["x1_residuals_differ"] = int(diff.sum())
    if diff.any():
        out["x1_residual_max_ulp"] = int(np.abs(r[diff].view(np.int32).astype(np.int64) - ref[diff].view(np.int32)).max())
        e_of = np.repeat(np.arange(p.n_edges), 2 * p.edge_n)[diff]
        out["x1_differing_edges"] = [int(e) for e in sorted(set(e_of.tolist()))[:20]]
        side = getattr(p, "edge_side", None)
        if side is not None:
            out["x1_differing_edge_sides"] = [int(side[e]) for e in out["x1_differing_edges"]]
    d1r, j1r = o.linearize_solve(x1, "schur")
    d1, j1 = g.compute_jacobian_extrinsic(x1)
    out["x1_delta_rel"] = float(np.abs(d1 - d1r).max() / np.abs(d1r).max())
    out["x1_delta_global_rel"] = float(np.abs(d1[:m] - d1r[:m]).max() / np.abs(d1r[:m]).max())
    out["x1_jte_rel"] = float(np.abs(j1 - j1r).max() / np.abs(j1r).max())
    out["x1_delta_global"] = {"gpu": [float(v) for v in d1[:m]], "oracle": [float(v) for v in d1r[:m]]}
    print({k: v for k, v in out.items() if k.startswith("x1_")}, flush=True)
    for k in range(1, args.steps + 1):
        xr, mr, itr, _ = o.optimize(p.x0, crit_type=1, max_count=k)
        x, mg, it, _ = g.optimize_extrinsics(p.x0, crit_type=1, max_count=k)
        u = f32_ulp_diff(x, xr)
        row = {"k": k, "differ": int((u > 0).sum()), "differ_global": int((u[:m] > 0).sum()), "max_ulp": int(u.max()),
               "max_ulp_global": int(u[:m].max()), "state_resolution_diff": float(state_resolution_diff(x, xr)),
               "first_differing": [int(i) for i in np.nonzero(u)[0][:8]]}
        if row["differ"]:
            i = int(np.argmax(u))
            row["worst"] = {"index": i, "gpu": float(x[i]), "oracle": float(xr[i])}
        out["steps"].append(row)
        print(row, flush=True)
finally:
    g.close()
if args.out:
    json.dump(out, open(args.out, "w"), indent=1)
