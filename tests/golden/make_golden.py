"""Generates the golden fixtures tests/golden/*.npz (SURVEY.md 8(c) pin v).

Run from the repo root:  python tests/golden/make_golden.py

Each fixture is self-contained data: the full problem inputs (rig.problem_to_arrays, float32 as
the reference stores them) and the CPU oracle's outputs on them:
  resid ............. float32 residuals fl32(obs - proj) of every corner at x0, reference order
  jc_s / jp_s / es .. the 2N x 6 global/photo Jacobian blocks of a spread sample of edges es
  delta / jte ....... step-0 deltaX and JTE of the exact Schur solve (computeJacobianExtrinsic)
  delta_cg .......... step-0 deltaX of the faithful dense J^T J + Eigen-CG x2 path
  pe_edge / pe_mean . computeProjectError at x0 (per-edge mean error, the reference's mean)
  x_opt, mean_opt, iters_opt, change_opt .. optimizeExtrinsics with the sample's TermCriteria
                      (COUNT+EPS, 200, 1e-7; DoubleSide 1e-8: mymulticalib.hpp:96, doubleSide.hpp:105)

The oracle is the reference restated (parity against OpenCV itself is unpinned, see
tests/test_oracle_math.py); these vectors freeze it so the GPU path and any later oracle change
are checked against the same numbers.  numpy's PCG64 streams are stable, so rig.make_config
regenerates the inputs bit-exactly (tests/test_golden.py checks that too).
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from multi_camera_calibration_amd import rig  # noqa: E402
from oracle import oracle_py as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))

CASES = {
    "config1": lambda: rig.make_config("config1"),
    "config2_v24": lambda: rig.make_config("config2", n_views=24),
    "config3_v12": lambda: rig.make_config("config3", n_views=12),
    "config4_v10": lambda: rig.make_config("config4", n_views=10),
    "config5_v8": lambda: rig.make_config("config5", n_views=8),
    "pinhole_back_v8": lambda: rig.make_config("config5", n_views=8, model=rig.PINHOLE, double_sided=True),
}


def generate(name, p):
    o = O.Oracle(p)
    out = rig.problem_to_arrays(p)
    out["resid"] = np.concatenate([o.edge_linearize(p.x0, e)[2] for e in range(p.n_edges)]).astype(np.float32)
    es = np.unique(np.linspace(0, p.n_edges - 1, 8).astype(np.int64))
    blocks = [o.edge_linearize(p.x0, int(e)) for e in es]
    out["es"] = es
    out["jc_s"] = np.concatenate([b[0] for b in blocks])
    out["jp_s"] = np.concatenate([b[1] for b in blocks])
    d, j = o.linearize_solve(p.x0, "schur")
    out["delta"], out["jte"] = d, j
    out["delta_cg"] = o.linearize_solve(p.x0, "cg")[0]
    out["pe_edge"], pe_mean = o.project_error(p.x0)
    out["pe_mean"] = np.float64(pe_mean)
    eps = 1e-8 if p.model == rig.DOUBLESIDE else 1e-7
    x, mean, iters, change = o.optimize(p.x0, 3, 200, eps)
    out["crit"] = np.array([3, 200], np.int64)
    out["crit_eps"] = np.float64(eps)
    out["x_opt"], out["mean_opt"] = x, np.float64(mean)
    out["iters_opt"], out["change_opt"] = np.int64(iters), np.float64(change)
    return out


def main():
    for name, mk in CASES.items():
        p = mk()
        out = generate(name, p)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **out)
        print(f"{name}: E={p.n_edges} corners={p.n_corners} P={p.n_params} iters={int(out['iters_opt'])} "
              f"mean={float(out['mean_opt']):.6f} -> {os.path.getsize(path) // 1024} KiB")


if __name__ == "__main__":
    main()
