#!/usr/bin/env python3
"""One Gauss-Newton iteration of the reference's own algorithm on config2 (SURVEY.md 8(d)(1)
'ref-faithful'): the zero-filled dense J (2 sum N x P = 345 488 x 3 018 doubles, 8.3 GB), JTJ = J^T J
and JTE = J^T E as dense products, Jacobi-CG solved twice (src/mymulticalib.cpp:680-805,
src/multicalib.cpp:565-592), single-threaded -- the oracle's restatement (test infrastructure,
oracle/mcc_oracle.c ora_normal_dense_j + ora_cg) timed once, offline, on this container's host core.
BASELINE.md's protocol asks for it beside the bench line; it takes tens of minutes, so bench.py cites
the committed result (profiles/ref_faithful_config2.json) instead of re-running it.

    python tools/ref_faithful_config2.py [out.json]
"""
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("OMP_NUM_THREADS", "1")

from multi_camera_calibration_amd import rig  # noqa: E402
from oracle import oracle_py as O  # noqa: E402


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "ref_faithful_config2.json")
    p = rig.make_config("config2")
    o = O.Oracle(p)
    rows = 2 * int(np.asarray(p.edge_n).sum())
    t0 = time.perf_counter()
    d, j = o.linearize_solve(p.x0, "dense_j")
    dt = time.perf_counter() - t0
    ds, js = o.linearize_solve(p.x0, "schur")
    res = {
        "config": "config2", "views": p.n_photos, "cameras": p.n_cams, "corners": p.n_corners, "params": p.n_params,
        "dense_J_shape": [rows, p.n_params], "dense_J_bytes": rows * p.n_params * 8,
        "seconds_per_iteration": dt, "corner_evals_per_s": p.n_corners / dt, "threads": 1,
        "kind": "port (the oracle's dense-J + Jacobi-CG restatement of the reference algorithm)",
        "host": platform.processor() or platform.machine(), "cpu_count_visible": os.cpu_count(),
        "delta_vs_schur_max_rel": float(np.abs(d - ds).max() / np.abs(ds).max()),
        "note": "offline, this build container's host core (not the GPU box's); one linearisation + "
                "the two CG solves = one optimizeExtrinsics iteration",
    }
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
