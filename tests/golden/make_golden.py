"""Generates the golden fixtures tests/golden/*.npz (SURVEY.md 8(c) pin v).

Run from the repo root:  python tests/golden/make_golden.py [name ...]

Each fixture is self-contained data: the full problem inputs (rig.problem_to_arrays, float32 as
the reference stores them) and the CPU oracle's outputs on them:
  resid ............. float32 residuals fl32(obs - proj) of every corner at x0, reference order
  jc_s / jp_s / es .. the 2N x 6 global/photo Jacobian blocks of a spread sample of edges es
  delta / jte ....... step-0 deltaX and JTE of the exact Schur solve (computeJacobianExtrinsic)
  delta_cg .......... step-0 deltaX of the faithful dense J^T J + Eigen-CG x2 path
  pe_edge / pe_mean . computeProjectError at x0 (per-edge mean error, the reference's mean)
  x_opt, mean_opt, iters_opt, change_opt .. optimizeExtrinsics with the sample's TermCriteria
                      (COUNT+EPS, 200, 1e-7; DoubleSide 1e-8: mymulticalib.hpp:96, doubleSide.hpp:105)
  x_opt_cg, mean_opt_cg, iters_opt_cg, change_opt_cg .. the same loop with the reference's own
                      solver in every step (dense J^T J + Jacobi-CG solved twice,
                      src/multicalib.cpp:565-592): the final iterate of the reference's algorithm

Cases: reduced synthetic rigs of every BASELINE config shape (seeds of SURVEY 8(d)), the MyMulti
back-side chain, the DoubleSide rig at C = 2 (the only camera count the reference's DoubleSide
runs at: src/doubleSide.cpp:44-50, 643), and `tutorial_stereo_v20`: REAL corners -- the first 20
views of the reference's tutorials/data/omni_stereocalib_data.xml (2 omnidirectional cameras,
8x6 board, 80 mm squares, 704x576), built the way the base class builds its problem
(MultiCameraCalibration::loadImages / initialize, src/multicalib.cpp:182-321, 380-420): per camera
cv::omnidir::calibrate (the oracle's restatement, TermCriteria(COUNT+EPS, 300, 1e-7)), one edge per
calibrated view with the view pose as its transform, photo vertices by timestamp, the BFS pose
chain from camera 0, then buildParas; optimised with the base class default TermCriteria
(COUNT, 20, 1e-7) (multicalib.hpp:140).  The fixture carries the raw 20-view corner arrays too,
so no GPU test reads /root/reference.

The oracle is the reference restated (parity against OpenCV itself is unpinned, see
tests/test_oracle_math.py); these vectors freeze it so the GPU path and any later oracle change
are checked against the same numbers.  numpy's PCG64 streams are stable, so rig.make_config
regenerates the inputs bit-exactly (tests/test_golden.py checks that too).
"""
import os
import sys
import xml.etree.ElementTree as ET

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from multi_camera_calibration_amd import rig  # noqa: E402
from oracle import oracle_py as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
STEREO_XML = "/root/reference/tutorials/data/omni_stereocalib_data.xml"


# ---------------------------------------------------------------- the real-corner case
def read_stereo_xml(path=STEREO_XML):
    """omni_stereocalib_data.xml -> (img1 [V,48,2], img2 [V,48,2], obj [V,48,3], (w, h)), float64."""
    root = ET.parse(path).getroot()

    def mats(tag):
        out = []
        for m in root.find(tag):
            rows, cols = int(m.find("rows").text), int(m.find("cols").text)
            ch = int(m.find("dt").text.strip().strip('"')[0])
            out.append(np.array(m.find("data").text.split(), np.float64).reshape(rows * cols, ch))
        return np.array(out)
    size = tuple(int(v) for v in root.find("imageSize1").text.split())
    return mats("imagePoints1"), mats("imagePoints2"), mats("objectPoints"), size


def _rod(r):
    R, _ = O.rodrigues_v2m(np.asarray(r, np.float64))
    return R


def _rod_inv(R):
    r, _ = O.rodrigues_m2v(np.asarray(R, np.float64))
    return r


def base_class_problem(imgs, obj, size, name, crit=(3, 300, 1e-7)):
    """MultiCameraCalibration::loadImages + initialize + buildParas on pre-detected corners
    (src/multicalib.cpp:182-321, 323-346, 361-420, 422-440) with the oracle's omnidir calibrate.
    imgs: per camera [V, N, 2]; obj [V, N, 3].  The finder hands the loader CV_32F points, which
    calibrate converts to CV_64F (src/omnidir.cpp:1083-1094): points are rounded to float32."""
    C = len(imgs)
    W, H = size
    n_vertex = C                      # camera vertices 0..C-1, photo vertices appended by timestamp
    vtx_ts = [-1] * C
    edges = []                        # (camera, photo vertex, R float32, t float32, img, obj)
    K = np.zeros((C, 3, 3), np.float32)
    D = np.zeros((C, 4), np.float32)
    xi = np.zeros(C, np.float32)
    intr = []
    for c in range(C):
        V = imgs[c].shape[0]
        n = imgs[c].shape[1]
        fi = imgs[c].astype(np.float32)
        fo = obj.astype(np.float32)
        off = np.arange(V + 1, dtype=np.int32) * n
        ov = O.OmniViews(off, fo.reshape(-1, 3).astype(np.float64), fi.reshape(-1, 2).astype(np.float64))
        rms, Kc, xic, Dc, om, t, idx, it = O.omni_calibrate(ov, W, H, 0, *crit)
        K[c], D[c], xi[c] = Kc.astype(np.float32), Dc.astype(np.float32), np.float32(xic)
        intr.append((rms, Kc, xic, Dc, it))
        for i in range(len(om)):
            ts = int(idx[i])                            # timestampAvailable[camera][idx[i]]
            if ts in vtx_ts:
                pv = vtx_ts.index(ts)
            else:
                vtx_ts.append(ts)
                pv = n_vertex
                n_vertex += 1
            r32 = om[i].astype(np.float32)
            t32 = t[i].astype(np.float32)
            R32 = _rod(r32.astype(np.float64)).astype(np.float32)
            edges.append((c, pv, R32, t32, fi[ts], fo[ts]))
    # initialize(): buildGraph (later edge of a pair wins), BFS from camera 0 with neighbours in
    # increasing vertex order, pose chaining in float32 (4x4 CV_32F Mats)
    adj = [dict() for _ in range(n_vertex)]
    for e, (c, pv, *_rest) in enumerate(edges):
        adj[c][pv] = e
        adj[pv][c] = e
    order, pre = [0], {0: -1}
    q = [0]
    for v in q:
        for nb in sorted(adj[v]):
            if nb not in pre:
                pre[nb] = v
                q.append(nb)
                order.append(nb)
    pose = [np.eye(4, dtype=np.float32) for _ in range(n_vertex)]
    for v in order[1:]:
        e = adj[v][pre[v]]
        T = np.eye(4, dtype=np.float32)
        T[:3, :3], T[:3, 3] = edges[e][2], edges[e][3]
        prev_inv = np.linalg.inv(pose[pre[v]].astype(np.float64))
        if v < C:
            pose[v] = (T.astype(np.float64) @ prev_inv).astype(np.float32)
        else:
            pose[v] = (prev_inv @ T.astype(np.float64)).astype(np.float32)
    # buildParas: vertices 1.. -> Rodrigues(float32 R), t
    x0 = []
    for v in range(1, n_vertex):
        x0.append(_rod_inv(pose[v][:3, :3].astype(np.float64)).astype(np.float32))
        x0.append(pose[v][:3, 3].astype(np.float32))
    x0 = np.concatenate(x0).astype(np.float32)
    E = len(edges)
    edge_n = np.array([len(e[4]) for e in edges], np.int32)
    edge_off = np.zeros(E, np.int32)
    edge_off[1:] = np.cumsum(edge_n)[:-1]
    p = rig.Problem(model=rig.OMNI, n_cams=C, n_photos=n_vertex - C,
                    edge_cam=np.array([e[0] for e in edges], np.int32),
                    edge_photo=np.array([e[1] - C for e in edges], np.int32),
                    edge_side=np.zeros(E, np.int32), edge_off=edge_off, edge_n=edge_n,
                    obj=np.concatenate([e[5] for e in edges]).astype(np.float32),
                    img=np.concatenate([e[4] for e in edges]).astype(np.float32),
                    K=K, D=D, xi=xi, ds_pose=None, cam_pose=None, x0=x0, x_true=x0.copy(),
                    timestamps=np.array(vtx_ts[C:], np.int64), image_size=(W, H), name=name)
    return p, intr


def tutorial_stereo(n_views=20):
    i1, i2, ob, size = read_stereo_xml()
    p, intr = base_class_problem([i1[:n_views], i2[:n_views]], ob[:n_views], size, f"tutorial_stereo_v{n_views}")
    extra = {"raw_img1": i1[:n_views], "raw_img2": i2[:n_views], "raw_obj": ob[:n_views],
             "calib_rms": np.array([v[0] for v in intr]), "calib_iters": np.array([v[4] for v in intr], np.int64),
             "calib_K": np.array([v[1] for v in intr]), "calib_xi": np.array([v[2] for v in intr]),
             "calib_D": np.array([v[3] for v in intr])}
    return p, extra


CASES = {
    "config1": lambda: rig.make_config("config1"),
    "config2_v24": lambda: rig.make_config("config2", n_views=24),
    "config3_v12": lambda: rig.make_config("config3", n_views=12),
    "config4_v10": lambda: rig.make_config("config4", n_views=10),
    "config5_v8": lambda: rig.make_config("config5", n_views=8),
    "config5_c2": lambda: rig.make_config("config5", n_cams=2, n_views=20),
    "pinhole_back_v8": lambda: rig.make_config("config5", n_views=8, model=rig.PINHOLE, double_sided=True),
    "tutorial_stereo_v20": lambda: tutorial_stereo(20),
}
# TermCriteria of the loop per case: the sample's MyMulti (COUNT+EPS, 200, 1e-7), DoubleSide's
# (COUNT+EPS, 200, 1e-8), the base class default (COUNT, 20, 1e-7) for the tutorial flow
CRIT = {"tutorial_stereo_v20": (1, 20, 1e-7)}


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
    crit = CRIT.get(name, (3, 200, 1e-8 if p.model == rig.DOUBLESIDE else 1e-7))
    out["crit"] = np.array(crit[:2], np.int64)
    out["crit_eps"] = np.float64(crit[2])
    x, mean, iters, change = o.optimize(p.x0, *crit)
    out["x_opt"], out["mean_opt"] = x, np.float64(mean)
    out["iters_opt"], out["change_opt"] = np.int64(iters), np.float64(change)
    x, mean, iters, change = o.optimize(p.x0, *crit, solver="cg")
    out["x_opt_cg"], out["mean_opt_cg"] = x, np.float64(mean)
    out["iters_opt_cg"], out["change_opt_cg"] = np.int64(iters), np.float64(change)
    return out


def make(name):
    r = CASES[name]()
    p, extra = r if isinstance(r, tuple) else (r, {})
    out = generate(name, p)
    out.update(extra)
    return p, out


def main():
    names = sys.argv[1:] or list(CASES)
    for name in names:
        p, out = make(name)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **out)
        print(f"{name}: E={p.n_edges} corners={p.n_corners} P={p.n_params} iters={int(out['iters_opt'])} "
              f"(cg {int(out['iters_opt_cg'])}) mean={float(out['mean_opt']):.9f} (cg {float(out['mean_opt_cg']):.9f}) "
              f"x bitwise equal: {np.array_equal(out['x_opt'], out['x_opt_cg'])} -> {os.path.getsize(path) // 1024} KiB")


if __name__ == "__main__":
    main()
