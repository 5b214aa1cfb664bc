"""Synthetic multi-camera rigs in the reference's problem layout.

The reference builds its BA problem from per-camera corner files
(MyMultiCameraCalibration::loadImages, src/mymulticalib.cpp:348-405).  This module produces the
same structure directly:

* camera vertices 0..C-1 (camera 0 = identity, not optimised), photo vertices C..C+V-1 created in
  first-appearance order of a camera-major sweep (getPhotoVertex, src/multicalib.cpp:323-346);
* edges in camera-major, timestamp-sorted order (loadOneSerial's cv::glob order,
  src/mymulticalib.cpp:268-301, 354-402);
* a view enters only if at least two cameras see it (identifyMultiCameraTimestamps,
  src/mymulticalib.cpp:314-347); for the double-sided board it must be seen from both sides
  (DoubleSideCalibration::findTimStamp, src/doubleSide.cpp:100-112);
* float32 object/image points (storeReadedImp, src/mymulticalib.cpp:229-230);
* the parameter vector laid out as buildParas does (src/multicalib.cpp:422-440,
  src/doubleSide.cpp:233-261), float32.

Geometry honours the reference's runtime asserts: 300 < |t| < 3000 for every edge and photo
(src/mymulticalib.cpp:210, 706, 714) and projected corners inside 1920x1080 for pinhole
(src/multicalib.cpp:704-715); composed rotation angles stay in [0.3, 2.8] rad.
"""
from __future__ import annotations

import dataclasses
from typing import Optional

import numpy as np

PINHOLE, OMNI, DOUBLESIDE = 0, 1, 2
FRONT, BACK = 0, 1


@dataclasses.dataclass
class Problem:
    model: int
    n_cams: int
    n_photos: int
    edge_cam: np.ndarray      # int32 [E]
    edge_photo: np.ndarray    # int32 [E] photo index (vertex - C)
    edge_side: np.ndarray     # int32 [E]
    edge_off: np.ndarray      # int32 [E]
    edge_n: np.ndarray        # int32 [E]
    obj: np.ndarray           # float32 [corners, 3]
    img: np.ndarray           # float32 [corners, 2]
    K: np.ndarray             # float32 [C, 3, 3]
    D: np.ndarray             # float32 [C, nd]
    xi: np.ndarray            # float32 [C]
    ds_pose: Optional[np.ndarray]   # float64 [4, 4] (MyMulti doubleSideTransform)
    cam_pose: Optional[np.ndarray]  # float32 [C, 4, 4] (DoubleSide fixed cameras)
    x0: np.ndarray            # float32 [P] initial parameters
    x_true: np.ndarray        # float32 [P] ground truth (information only)
    timestamps: np.ndarray    # int64 [V] photo vertex timestamps
    image_size: tuple
    name: str = ""

    @property
    def n_edges(self) -> int:
        return int(self.edge_cam.shape[0])

    @property
    def n_corners(self) -> int:
        return int(self.obj.shape[0])

    @property
    def nd(self) -> int:
        return int(self.D.shape[1])

    @property
    def n_params(self) -> int:
        if self.model == DOUBLESIDE:
            return 6 * (1 + self.n_photos)
        return 6 * (self.n_cams - 1 + self.n_photos)

    @property
    def global_dim(self) -> int:
        return 6 if self.model == DOUBLESIDE else 6 * (self.n_cams - 1)

    def photo_col(self, photo):
        if self.model == DOUBLESIDE:
            return 6 * (1 + np.asarray(photo))
        return 6 * (self.n_cams - 1 + np.asarray(photo))


# ----------------------------------------------------------------------------- SO(3) helpers

def rodrigues(r):
    """Rotation vector(s) [..., 3] -> matrices [..., 3, 3] (float64)."""
    r = np.asarray(r, dtype=np.float64)
    th = np.linalg.norm(r, axis=-1, keepdims=True)
    k = np.where(th > 1e-300, r / np.maximum(th, 1e-300), 0.0)
    kx, ky, kz = k[..., 0], k[..., 1], k[..., 2]
    z = np.zeros_like(kx)
    Kx = np.stack([np.stack([z, -kz, ky], -1), np.stack([kz, z, -kx], -1),
                   np.stack([-ky, kx, z], -1)], -2)
    th = th[..., None]
    eye = np.broadcast_to(np.eye(3), Kx.shape)
    return eye + np.sin(th) * Kx + (1 - np.cos(th)) * (Kx @ Kx)


def log_so3(R):
    R = np.asarray(R, dtype=np.float64)
    c = np.clip((np.trace(R, axis1=-2, axis2=-1) - 1) * 0.5, -1, 1)
    th = np.arccos(c)
    v = np.stack([R[..., 2, 1] - R[..., 1, 2], R[..., 0, 2] - R[..., 2, 0],
                  R[..., 1, 0] - R[..., 0, 1]], -1)
    s = np.sin(th)
    f = np.where(s > 1e-12, th / (2 * np.maximum(s, 1e-300)), 0.5)
    return v * f[..., None]


def rot_angle(R):
    return np.arccos(np.clip((np.trace(R, axis1=-2, axis2=-1) - 1) * 0.5, -1, 1))


def look_at(pos, target, up=(0.0, -1.0, 0.0)):
    """World->camera rotation for a camera at pos looking at target (x right, y down)."""
    z = np.asarray(target, float) - np.asarray(pos, float)
    z /= np.linalg.norm(z)
    x = np.cross(np.asarray(up, float), z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    Rwc = np.stack([x, y, z], 1)           # camera->world columns
    return Rwc.T


# ----------------------------------------------------------------------------- camera models

def project_pinhole(Xc, K, D):
    """Brown-Conrady (k1,k2,p1,p2,k3) pinhole, float64.  Xc [..., 3]."""
    x = Xc[..., 0] / Xc[..., 2]
    y = Xc[..., 1] / Xc[..., 2]
    k1, k2, p1, p2 = D[0], D[1], D[2], D[3]
    k3 = D[4] if len(D) > 4 else 0.0
    r2 = x * x + y * y
    cd = 1 + k1 * r2 + k2 * r2 * r2 + k3 * r2 ** 3
    xd = x * cd + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * cd + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([K[0, 0] * xd + K[0, 2], K[1, 1] * yd + K[1, 2]], -1)


def project_omni(Xc, K, xi, D):
    """Mei unified model (src/omnidir.cpp:141-166), float64."""
    Xs = Xc / np.linalg.norm(Xc, axis=-1, keepdims=True)
    den = Xs[..., 2] + xi
    x = Xs[..., 0] / den
    y = Xs[..., 1] / den
    k1, k2, p1, p2 = D
    r2 = x * x + y * y
    cd = 1 + k1 * r2 + k2 * r2 * r2
    xd = x * cd + 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
    yd = y * cd + p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
    return np.stack([K[0, 0] * xd + K[0, 1] * yd + K[0, 2], K[1, 1] * yd + K[1, 2]], -1)


def board_points(cols, rows, square):
    """Row-major inner-corner grid on Z = 0 (cv::Size(width=cols, height=rows))."""
    yy, xx = np.meshgrid(np.arange(rows), np.arange(cols), indexing="ij")
    pts = np.stack([xx.ravel() * square, yy.ravel() * square, np.zeros(rows * cols)], -1)
    return pts.astype(np.float64)


# ----------------------------------------------------------------------------- configs

CONFIGS = {
    # BASELINE.json configs (SURVEY.md section 8(d) seeds).  config1 stands in for the 20 real
    # 9x6 views (no real pinhole corner data ships with the reference).
    "config1": dict(model=PINHOLE, n_cams=2, n_views=20, board=(9, 6), seed=1),
    "config2": dict(model=PINHOLE, n_cams=4, n_views=500, board=(11, 8), seed=2),
    "config3": dict(model=PINHOLE, n_cams=16, n_views=5000, board=(11, 8), seed=3, visibility=0.5),
    "config4": dict(model=OMNI, n_cams=4, n_views=1000, board=(11, 8), seed=4),
    "config5": dict(model=DOUBLESIDE, n_cams=8, n_views=2000, board=(8, 11), back=(7, 10), seed=5),
}


def make_config(name: str, n_views: Optional[int] = None, **over) -> Problem:
    cfg = dict(CONFIGS[name])
    if n_views is not None:
        cfg["n_views"] = n_views
    cfg.update(over)
    p = make_rig(**cfg)
    p.name = name
    return p


def _perturb(rng, r, t, rot_deg=0.5, trans_mm=3.0):
    """truth (+) (rotation of rot_deg about a random axis, translation of trans_mm)."""
    a = rng.normal(size=3)
    a *= np.deg2rad(rot_deg) / np.linalg.norm(a)
    R = rodrigues(a) @ rodrigues(r)
    d = rng.normal(size=3)
    d *= trans_mm / np.linalg.norm(d)
    return log_so3(R), t + d


def make_rig(model=PINHOLE, n_cams=4, n_views=500, board=(11, 8), back=(7, 10), square=40.0,
             seed=2, visibility=1.0, noise_px=0.2, rot_deg=0.5, trans_mm=3.0,
             double_sided=False) -> Problem:
    """double_sided: ring rig around a two-sided board (config 5 geometry); with model=PINHOLE this
    gives MyMulti BACK edges (fixed doubleSideTransform, src/mymulticalib.cpp:503-518)."""
    rng = np.random.default_rng(seed)
    C = n_cams
    ring = model == DOUBLESIDE or double_sided
    omni = model == OMNI
    W, H = (1280, 960) if omni else (1920, 1080)
    margin = 40.0

    # ---- intrinsics
    K = np.zeros((C, 3, 3))
    if omni:
        D = np.zeros((C, 4))
        xi = rng.uniform(0.8, 1.2, C)
        for c in range(C):
            f = 350.0 * rng.uniform(0.97, 1.03)
            K[c] = [[f, 0, 640 + rng.uniform(-10, 10)], [0, f * rng.uniform(0.99, 1.01),
                                                         480 + rng.uniform(-10, 10)], [0, 0, 1]]
            D[c] = [rng.uniform(-0.1, 0.0), rng.uniform(0.0, 0.05),
                    rng.uniform(-5e-4, 5e-4), rng.uniform(-5e-4, 5e-4)]
    else:
        D = np.zeros((C, 5))
        xi = np.zeros(C)
        for c in range(C):
            K[c] = [[rng.uniform(1000, 1400), 0, 960 + rng.uniform(-20, 20)],
                    [0, rng.uniform(1000, 1400), 540 + rng.uniform(-20, 20)], [0, 0, 1]]
            D[c] = [rng.uniform(-0.15, -0.05), rng.uniform(0.0, 0.1),
                    rng.uniform(-5e-4, 5e-4), rng.uniform(-5e-4, 5e-4), 0.0]
    K = K.astype(np.float32).astype(np.float64)
    D = D.astype(np.float32).astype(np.float64)
    xi = xi.astype(np.float32).astype(np.float64)

    # ---- extrinsics: camera vertex pose maps cam0 (world) coordinates to camera coordinates
    Rc = np.zeros((C, 3, 3))
    tc = np.zeros((C, 3))
    center = np.zeros((C, 3))
    depth0 = 1400.0
    if ring:
        n_front = (C + 1) // 2
        for c in range(C):
            if c < n_front:
                yaw = 0.0 if c == 0 else np.deg2rad(-30 + 60 * c / max(1, n_front - 1))
                pos = np.array([400 * np.sin(yaw), 60.0 * ((c % 2) * 2 - 1) * (c > 0), 400 * (1 - np.cos(yaw))])
                target = np.array([0.0, 0.0, depth0])
            else:
                j = c - n_front
                nb = C - n_front
                yaw = np.deg2rad(-30 + 60 * j / max(1, nb - 1))
                pos = np.array([400 * np.sin(yaw), 60.0 * ((j % 2) * 2 - 1), 2 * depth0 - 400 * (1 - np.cos(yaw))])
                target = np.array([0.0, 0.0, depth0])
            R = np.eye(3) if c == 0 else look_at(pos, target)
            Rc[c], center[c] = R, pos
            tc[c] = -R @ pos
    else:
        for c in range(C):
            if c == 0:
                Rc[c] = np.eye(3)
                continue
            frac = (c - 1) / max(1, C - 2)
            yaw = np.deg2rad(-40 + 80 * frac) if C > 2 else np.deg2rad(25.0)
            if abs(yaw) < np.deg2rad(3):
                yaw = np.deg2rad(5.0)
            pitch_off = 80.0 * (((c % 3) - 1)) if C > 4 else 30.0 * (c % 2)
            pos = np.array([400 * np.sin(yaw), pitch_off, 400 * (1 - np.cos(yaw))])
            target = np.array([0.0, 0.0, depth0]) + rng.normal(0, 30, 3)
            R = look_at(pos, target)
            Rc[c], center[c] = R, pos
            tc[c] = -R @ pos
    # round trip through float32 params (the reference keeps poses in float32)
    rc_vec = log_so3(Rc).astype(np.float32).astype(np.float64)
    tc = tc.astype(np.float32).astype(np.float64)
    Rc = rodrigues(rc_vec)
    rc_vec[0] = 0.0
    tc[0] = 0.0
    Rc[0] = np.eye(3)

    front_pts = board_points(board[0], board[1], square)
    back_pts = board_points(back[0], back[1], square) if ring else None
    ctr_b = front_pts.mean(0)
    # double side: back pattern -> front pattern coordinates (doubleSideTransform)
    R_ds = rodrigues(np.array([0.0, np.pi - 0.02, 0.0]))
    t_ds = np.array([(board[0] - 1) * square * 0.5 + (back[0] - 1) * square * 0.5 + 5.0,
                     ((board[1] - 1) - (back[1] - 1)) * square * 0.5, 25.0])
    r_ds = log_so3(R_ds).astype(np.float32).astype(np.float64)
    t_ds = t_ds.astype(np.float32).astype(np.float64)
    R_ds = rodrigues(r_ds)

    def project(c, Xc):
        if omni:
            return project_omni(Xc, K[c], xi[c], D[c])
        return project_pinhole(Xc, K[c], D[c])

    views = []   # list of (r_p, t_p, [(cam, side, pixels, objpts)])
    attempts = 0
    while len(views) < n_views:
        attempts += 1
        if attempts > 200 * n_views + 10000:
            raise RuntimeError("rig generator could not place enough views")
        # board pose: pattern -> cam0 (world)
        dirn = rng.normal(size=3) * np.array([0.12, 0.09, 0.0]) + np.array([0, 0, 1.0])
        dirn /= np.linalg.norm(dirn)
        dist = rng.uniform(950, 1850) if not ring else rng.uniform(1100, 1700)
        ctr_w = dirn * dist
        if ring:
            ctr_w[2] = depth0 + rng.uniform(-150, 150)
        roll = rng.uniform(0.35, 0.7) * rng.choice([-1, 1])
        tilt_ax = rng.normal(size=3) * np.array([1, 1, 0])
        tilt_ax /= np.linalg.norm(tilt_ax)
        tilt = rng.uniform(0.05, 0.45)
        Rp = rodrigues(tilt_ax * tilt) @ rodrigues(np.array([0, 0, roll]))
        rp = log_so3(Rp).astype(np.float32).astype(np.float64)
        Rp = rodrigues(rp)
        tp = (ctr_w - Rp @ ctr_b).astype(np.float32).astype(np.float64)
        if not (350 < np.linalg.norm(tp) < 2900):
            continue
        obs = []
        for c in range(C):
            if visibility < 1.0 and rng.uniform() > visibility:
                continue
            sides = [FRONT] if not ring else [FRONT, BACK]
            for side in sides:
                if side == FRONT:
                    Rt, tt, pts = Rc[c] @ Rp, Rc[c] @ tp + tc[c], front_pts
                else:
                    Rb = Rp @ R_ds
                    tb = Rp @ t_ds + tp
                    Rt, tt, pts = Rc[c] @ Rb, Rc[c] @ tb + tc[c], back_pts
                ang = rot_angle(Rt)
                if not (0.3 <= ang <= 2.8):
                    continue
                if not (350 < np.linalg.norm(tt) < 2900):
                    continue
                Xc = pts @ Rt.T + tt
                if np.any(Xc[:, 2] < 200):
                    continue
                # facing: pattern z axis points away from the camera
                nz = Rt[:, 2]
                ctr_c = Xc.mean(0)
                cosang = nz @ ctr_c / np.linalg.norm(ctr_c)
                if cosang < np.cos(np.deg2rad(65)):
                    continue
                uv = project(c, Xc)
                if np.any(uv[:, 0] < margin) or np.any(uv[:, 0] > W - margin) or \
                   np.any(uv[:, 1] < margin) or np.any(uv[:, 1] > H - margin):
                    continue
                obs.append((c, side, uv, pts))
        cams_seen = {o[0] for o in obs}
        if model == DOUBLESIDE:
            sides_seen = {o[1] for o in obs}
            if sides_seen != {FRONT, BACK}:
                continue
        elif len(cams_seen) < 2:
            continue
        views.append((rp, tp, obs))

    # ---- reference ordering: camera-major, timestamp-sorted; photo vertices by first appearance
    V = len(views)
    ts = 100000 + np.arange(V)          # fixed-width timestamps: glob order == numeric order
    photo_of_view = -np.ones(V, dtype=np.int64)
    photo_views = []
    edges = []
    for c in range(C):
        for v in range(V):
            for (cc, side, uv, pts) in views[v][2]:
                if cc != c:
                    continue
                if photo_of_view[v] < 0:
                    photo_of_view[v] = len(photo_views)
                    photo_views.append(v)
                edges.append((c, int(photo_of_view[v]), side, uv, pts))
    n_photos = len(photo_views)
    E = len(edges)
    edge_cam = np.array([e[0] for e in edges], np.int32)
    edge_photo = np.array([e[1] for e in edges], np.int32)
    edge_side = np.array([e[2] for e in edges], np.int32)
    edge_n = np.array([len(e[4]) for e in edges], np.int32)
    edge_off = np.zeros(E, np.int32)
    edge_off[1:] = np.cumsum(edge_n)[:-1]
    obj = np.concatenate([e[4] for e in edges]).astype(np.float32)
    uv = np.concatenate([e[3] for e in edges])
    img = (uv + rng.normal(0, noise_px, uv.shape)).astype(np.float32)

    # ---- parameters (buildParas layout)
    def pack(rvecs_cam, tvecs_cam, rvecs_ph, tvecs_ph, ds_rt=None):
        out = []
        if model == DOUBLESIDE:
            out.append(np.concatenate(ds_rt))
        else:
            for c in range(1, C):
                out.append(np.concatenate([rvecs_cam[c], tvecs_cam[c]]))
        for p in range(n_photos):
            out.append(np.concatenate([rvecs_ph[p], tvecs_ph[p]]))
        return np.concatenate(out).astype(np.float32)

    r_ph = [views[v][0] for v in photo_views]
    t_ph = [views[v][1] for v in photo_views]
    x_true = pack(rc_vec, tc, r_ph, t_ph, (r_ds, t_ds))
    r_c0, t_c0 = [None] * C, [None] * C
    for c in range(C):
        r_c0[c], t_c0[c] = _perturb(rng, rc_vec[c], tc[c], rot_deg, trans_mm) if c else (rc_vec[0], tc[0])
    r_p0, t_p0 = [], []
    for p in range(n_photos):
        r, t = _perturb(rng, r_ph[p], t_ph[p], rot_deg, trans_mm)
        r_p0.append(r)
        t_p0.append(t)
    ds0 = _perturb(rng, r_ds, t_ds, rot_deg, trans_mm)
    x0 = pack(r_c0, t_c0, r_p0, t_p0, ds0)

    ds_pose = np.eye(4)
    ds_pose[:3, :3] = R_ds
    ds_pose[:3, 3] = t_ds
    cam_pose = None
    if model == DOUBLESIDE:
        cam_pose = np.zeros((C, 4, 4), np.float32)
        for c in range(C):
            cam_pose[c, :3, :3] = Rc[c]
            cam_pose[c, :3, 3] = tc[c]
            cam_pose[c, 3, 3] = 1
    return Problem(model=model, n_cams=C, n_photos=n_photos, edge_cam=edge_cam,
                   edge_photo=edge_photo, edge_side=edge_side, edge_off=edge_off, edge_n=edge_n,
                   obj=obj, img=img, K=K.astype(np.float32), D=D.astype(np.float32),
                   xi=xi.astype(np.float32), ds_pose=ds_pose,
                   cam_pose=cam_pose, x0=x0, x_true=x_true,
                   timestamps=ts[np.array(photo_views)], image_size=(W, H))


def subset_photos(p: Problem, photos) -> Problem:
    """Sub-problem restricted to the given photo indices (keeps cameras, reindexes photos and
    edges in reference order).  Used for per-rank shards and small parity cases."""
    photos = np.asarray(photos, dtype=np.int64)
    remap = -np.ones(p.n_photos, np.int64)
    remap[photos] = np.arange(len(photos))
    keep = np.nonzero(remap[p.edge_photo] >= 0)[0]
    edge_n = p.edge_n[keep]
    edge_off = np.zeros(len(keep), np.int32)
    edge_off[1:] = np.cumsum(edge_n)[:-1]
    idx = np.concatenate([np.arange(p.edge_off[e], p.edge_off[e] + p.edge_n[e]) for e in keep])
    g = p.global_dim
    cols = np.concatenate([np.arange(g)] + [p.photo_col(ph) + np.arange(6) for ph in photos])
    return Problem(model=p.model, n_cams=p.n_cams, n_photos=len(photos),
                   edge_cam=p.edge_cam[keep].copy(), edge_photo=remap[p.edge_photo[keep]].astype(np.int32),
                   edge_side=p.edge_side[keep].copy(), edge_off=edge_off, edge_n=edge_n.copy(),
                   obj=p.obj[idx].copy(), img=p.img[idx].copy(), K=p.K, D=p.D, xi=p.xi,
                   ds_pose=p.ds_pose, cam_pose=p.cam_pose, x0=p.x0[cols].copy(),
                   x_true=p.x_true[cols].copy(), timestamps=p.timestamps[photos],
                   image_size=p.image_size, name=p.name + "[subset]")


# ----------------------------------------------------------------------------- (de)serialisation
_ARRAY_FIELDS = ("edge_cam", "edge_photo", "edge_side", "edge_off", "edge_n", "obj", "img", "K", "D",
                 "xi", "ds_pose", "cam_pose", "x0", "x_true", "timestamps")


def problem_to_arrays(p: Problem, prefix: str = "") -> dict:
    """Flat dict of numpy arrays (npz-ready, no pickles) holding every input of a Problem."""
    out = {prefix + "meta": np.array([p.model, p.n_cams, p.n_photos, p.image_size[0], p.image_size[1]],
                                     np.int64)}
    for f in _ARRAY_FIELDS:
        v = getattr(p, f)
        if v is not None:
            out[prefix + f] = np.asarray(v)
    return out


def problem_from_arrays(a, prefix: str = "", name: str = "") -> Problem:
    meta = [int(v) for v in a[prefix + "meta"]]
    kw = {f: (np.array(a[prefix + f]) if (prefix + f) in a else None) for f in _ARRAY_FIELDS}
    return Problem(model=meta[0], n_cams=meta[1], n_photos=meta[2], image_size=(meta[3], meta[4]),
                   name=name, **kw)


# ----------------------------------------------------------------------------- omni intrinsic views
@dataclasses.dataclass
class OmniCalibViews:
    """One omnidirectional camera's per-view chessboard corners, as cv::omnidir::calibrate takes
    them (src/omnidir.cpp:1067-1090; CV_64F after its convertTo): view i holds corners
    off[i]..off[i+1] of obj (x, y, 0) and img (u, v)."""
    off: np.ndarray           # int32 [n+1]
    obj: np.ndarray           # float64 [corners, 3]
    img: np.ndarray           # float64 [corners, 2]
    image_size: tuple         # (width, height)
    K: np.ndarray             # truth (information only)
    xi: float
    D: np.ndarray
    om: np.ndarray            # [n, 3]
    t: np.ndarray             # [n, 3]

    @property
    def n_views(self) -> int:
        return len(self.off) - 1


def make_omni_views(n_views=1000, board=(11, 8), square=40.0, seed=4, noise_px=0.2,
                    size=(1280, 960), K=None, xi=None, D=None) -> OmniCalibViews:
    """Mei-model camera (config 4's intrinsics: f ~ 350, xi ~ U(0.8, 1.2), 1280x960, D = 4; or the
    given K / xi / D) and n_views board poses 350-1300 mm away, up to 55 deg off axis, tilted up to
    45 deg, every corner inside the image with a 20 px margin; 0.2 px Gaussian corner noise."""
    rng = np.random.default_rng(seed)
    W, H = size
    f = 350.0 * rng.uniform(0.97, 1.03)
    K0 = np.array([[f, 0.0, W / 2 + rng.uniform(-10, 10)], [0, f * rng.uniform(0.99, 1.01), H / 2 + rng.uniform(-10, 10)],
                   [0, 0, 1]])
    xi0 = float(rng.uniform(0.8, 1.2))
    D0 = np.array([rng.uniform(-0.1, 0.0), rng.uniform(0.0, 0.05), rng.uniform(-5e-4, 5e-4), rng.uniform(-5e-4, 5e-4)])
    K = K0 if K is None else np.asarray(K, np.float64)
    xi = xi0 if xi is None else float(xi)
    D = D0 if D is None else np.asarray(D, np.float64)
    pts = board_points(board[0], board[1], square)
    ctr = pts.mean(0)
    oms, ts, imgs = [], [], []
    margin = 20.0
    while len(oms) < n_views:
        dist = rng.uniform(350.0, 1300.0)
        off_ang = np.deg2rad(rng.uniform(0, 55))
        az = rng.uniform(-np.pi, np.pi)
        dirv = np.array([np.sin(off_ang) * np.cos(az), np.sin(off_ang) * np.sin(az), np.cos(off_ang)])
        center = dist * dirv
        # board normal roughly facing the camera, tilted up to 45 deg, random in-plane spin
        R0 = look_at(np.zeros(3), center)   # camera looking at the board centre
        tilt = rng.normal(size=3)
        tilt *= np.deg2rad(rng.uniform(0, 45)) / np.linalg.norm(tilt)
        spin = rodrigues(np.array([0.0, 0.0, rng.uniform(-np.pi, np.pi)]))
        Rb = R0.T @ rodrigues(tilt) @ spin            # board -> camera rotation
        tb = center - Rb @ ctr
        Xc = pts @ Rb.T + tb
        if np.any(Xc[:, 2] < 50.0):
            continue
        uv = project_omni(Xc, K, xi, D)
        if np.any(uv[:, 0] < margin) or np.any(uv[:, 0] > W - margin) or np.any(uv[:, 1] < margin) \
                or np.any(uv[:, 1] > H - margin):
            continue
        oms.append(log_so3(Rb))
        ts.append(tb)
        imgs.append(uv + rng.normal(scale=noise_px, size=uv.shape))
    n = len(oms)
    off = np.arange(n + 1, dtype=np.int32) * len(pts)
    return OmniCalibViews(off, np.tile(pts, (n, 1)), np.concatenate(imgs), (W, H), K, xi, D,
                          np.array(oms), np.array(ts))
