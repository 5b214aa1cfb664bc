"""Independent float64 numpy restatement of the reference's per-edge model (test infrastructure).

A second derivation, written from the formulas only, that the C oracle is checked against
(SURVEY.md 8(c) pins (i)/(ii)): values here, derivatives by central finite differences of these
functions.  Nothing is rounded to float32 except where a test asks for it explicitly.

  rodrigues / log_so3 ...... cv::Rodrigues
  compose .................. compose_motion values, src/multicalib.cpp:1030-1051 (R3 = R2 R1,
                             T3 = R2 T1 + T2)
  project_pinhole .......... cv::projectPoints (k1,k2,p1,p2,k3,k4,k5,k6,s1..s4; Appendix A.3)
  project_omni ............. cv::omnidir::projectPoints, src/omnidir.cpp:141-162
  edge_pose / edge_pixels .. the pose chain of computePhotoCameraJacobian:
                             front (photo o camera), src/mymulticalib.cpp:498-500;
                             back ((photo o camera) o ds), src/mymulticalib.cpp:503-505;
                             DoubleSide with fixed cameras and ds as the global block,
                             src/doubleSide.cpp:312-328.
"""
from __future__ import annotations

import numpy as np

PINHOLE, OMNI, DOUBLESIDE = 0, 1, 2
BACK = 1


def skew(w):
    return np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])


def rodrigues(w):
    w = np.asarray(w, np.float64)
    th = np.linalg.norm(w)
    if th < 1e-300:
        return np.eye(3)
    k = w / th
    K = skew(k)
    return np.eye(3) + np.sin(th) * K + (1.0 - np.cos(th)) * (K @ K)


def log_so3(R):
    """Matrix -> vector by the trace/skew formula (no orthonormalisation), theta in (0, pi)."""
    R = np.asarray(R, np.float64)
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    s = 0.5 * np.linalg.norm(v)
    c = np.clip(0.5 * (np.trace(R) - 1.0), -1.0, 1.0)
    th = np.arctan2(s, c)
    if s < 1e-12:
        return np.zeros(3)
    return v * (th / (2.0 * s))


def log_formula(Rflat):
    """OpenCV's matrix -> vector formula as a function of all 9 entries (for its 9x3 Jacobian)."""
    R = np.asarray(Rflat, np.float64).reshape(3, 3)
    v = np.array([R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]])
    s = np.sqrt((v @ v) * 0.25)
    c = np.clip((np.trace(R) - 1.0) * 0.5, -1.0, 1.0)
    return v * (np.arccos(c) / (2.0 * s))


def compose(om1, T1, om2, T2):
    R1, R2 = rodrigues(om1), rodrigues(om2)
    return log_so3(R2 @ R1), R2 @ np.asarray(T1, np.float64) + np.asarray(T2, np.float64)


def project_pinhole(X, om, T, K, D):
    X = np.asarray(X, np.float64).reshape(-1, 3)
    K = np.asarray(K, np.float64).reshape(3, 3)
    k = np.zeros(12)
    D = np.asarray(D, np.float64).ravel()
    k[:min(D.size, 12)] = D[:12]
    k1, k2, p1, p2, k3, k4, k5, k6, s1, s2, s3, s4 = k
    Xc = X @ rodrigues(om).T + np.asarray(T, np.float64)
    z = np.where(Xc[:, 2] != 0, 1.0 / Xc[:, 2], 1.0)
    x, y = Xc[:, 0] * z, Xc[:, 1] * z
    r2 = x * x + y * y
    r4, r6 = r2 * r2, r2 * r2 * r2
    cdist = 1 + k1 * r2 + k2 * r4 + k3 * r6
    icd = 1.0 / (1 + k4 * r2 + k5 * r4 + k6 * r6)
    a1, a2, a3 = 2 * x * y, r2 + 2 * x * x, r2 + 2 * y * y
    xd = x * cdist * icd + p1 * a1 + p2 * a2 + s1 * r2 + s2 * r4
    yd = y * cdist * icd + p1 * a3 + p2 * a1 + s3 * r2 + s4 * r4
    if D.size == 14 and (D[12] != 0 or D[13] != 0):
        # the tilted image sensor, from the model's definition (OpenCV camera model docs): the
        # distorted point on the plane z = 1, rotated by R(tau) = Ry(tau_y) Rx(tau_x), then projected
        # along the rotated optical axis back onto that plane: [[R33, 0, -R13], [0, R33, -R23], [0, 0, 1]]
        tx, ty = D[12], D[13]
        Rx = np.array([[1, 0, 0], [0, np.cos(tx), np.sin(tx)], [0, -np.sin(tx), np.cos(tx)]])
        Ry = np.array([[np.cos(ty), 0, -np.sin(ty)], [0, 1, 0], [np.sin(ty), 0, np.cos(ty)]])
        Rt = Ry @ Rx
        w = np.stack([xd, yd, np.ones_like(xd)], 1) @ Rt.T
        xd = Rt[2, 2] * w[:, 0] / w[:, 2] - Rt[0, 2]
        yd = Rt[2, 2] * w[:, 1] / w[:, 2] - Rt[1, 2]
    return np.stack([K[0, 0] * xd + K[0, 2], K[1, 1] * yd + K[1, 2]], 1)


def project_omni(X, om, T, K, xi, D):
    X = np.asarray(X, np.float64).reshape(-1, 3)
    K = np.asarray(K, np.float64).reshape(3, 3)
    k1, k2, p1, p2 = np.asarray(D, np.float64).ravel()[:4]
    Xc = X @ rodrigues(om).T + np.asarray(T, np.float64)
    Xs = Xc / np.linalg.norm(Xc, axis=1, keepdims=True)
    xu, yu = Xs[:, 0] / (Xs[:, 2] + xi), Xs[:, 1] / (Xs[:, 2] + xi)
    r2 = xu * xu + yu * yu
    r4 = r2 * r2
    xd = xu * (1 + k1 * r2 + k2 * r4) + 2 * p1 * xu * yu + p2 * (r2 + 2 * xu * xu)
    yd = yu * (1 + k1 * r2 + k2 * r4) + p1 * (r2 + 2 * yu * yu) + 2 * p2 * xu * yu
    return np.stack([K[0, 0] * xd + K[0, 1] * yd + K[0, 2], K[1, 1] * yd + K[1, 2]], 1)


def _pose(x, col):
    return np.asarray(x[col:col + 3], np.float64), np.asarray(x[col + 3:col + 6], np.float64)


def ds_rt(prob):
    """(rvec, tvec) of the MyMulti doubleSideTransform (CV_64F 4x4)."""
    M = np.asarray(prob.ds_pose, np.float64).reshape(4, 4)
    return log_so3(M[:3, :3]), M[:3, 3].copy()


def edge_pose(prob, x, e):
    """Composed (om, T) an edge projects with, float64, from the float64 parameter vector x."""
    x = np.asarray(x, np.float64)
    c, v = int(prob.edge_cam[e]), int(prob.edge_photo[e])
    side = int(prob.edge_side[e]) if prob.edge_side is not None else 0
    omp, Tp = _pose(x, prob.photo_col(v))
    if prob.model == DOUBLESIDE:
        M = np.asarray(prob.cam_pose, np.float64).reshape(-1, 4, 4)[c]
        omc, Tc = log_so3(M[:3, :3]), M[:3, 3]
        omd, Td = _pose(x, 0)
    else:
        if c == 0:
            omc, Tc = np.zeros(3), np.zeros(3)
        else:
            omc, Tc = _pose(x, 6 * (c - 1))
        if side == BACK:
            omd, Td = ds_rt(prob)
    om, T = compose(omp, Tp, omc, Tc)
    if side == BACK:
        om, T = compose(omd, Td, om, T)
    return om, T


def edge_pixels(prob, x, e, om=None, T=None):
    """Projected pixels [u0, v0, u1, v1, ...] of edge e (float64 throughout)."""
    if om is None:
        om, T = edge_pose(prob, x, e)
    c, o, n = int(prob.edge_cam[e]), int(prob.edge_off[e]), int(prob.edge_n[e])
    X = np.asarray(prob.obj, np.float64).reshape(-1, 3)[o:o + n]
    K = np.asarray(prob.K, np.float64).reshape(-1, 9)[c]
    D = np.asarray(prob.D, np.float64).reshape(-1, prob.nd)[c]
    if prob.model == OMNI:
        px = project_omni(X, om, T, K, float(np.float32(prob.xi[c])), D)
    else:
        px = project_pinhole(X, om, T, K, D)
    return px.reshape(-1)


def fd_jacobian(f, x0, cols, h=1e-6):
    """Central differences of f at x0 w.r.t. x0[cols] (relative step for large entries)."""
    x0 = np.asarray(x0, np.float64)
    out = []
    for c in cols:
        hc = h * max(1.0, abs(x0[c]))
        xp, xm = x0.copy(), x0.copy()
        xp[c] += hc
        xm[c] -= hc
        out.append((f(xp) - f(xm)) / (2 * hc))
    return np.stack(out, 1)
