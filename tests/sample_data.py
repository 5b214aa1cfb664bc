"""Synthetic datasets in the reference sample's on-disk layout, and the sample's problem dump.

Layout read by MyMultiCameraCalibration (src/mymulticalib.cpp:118-131, 182-301):
    <config>/<serial>.xml          Intrinsics (3x3), Distortion (1 x nd), depth_scale, height,
                                   CameraMatrix (rewritten by writeParameters2config)
    <data>/<serial>/<ts>.yaml      corners (N x 2), objects (N x 3): one view of the board
written here from a rig.Problem (the reference's own data files are not in its repository; these
stand in, with the formats its readers imply).
"""
import os

import numpy as np

from multi_camera_calibration_amd import rig

MAGIC = 0x4D434331


def _mat_yaml(name, a, dt="d"):
    a = np.asarray(a, np.float64)
    vals = ", ".join(repr(float(v)) for v in a.ravel())
    return f"{name}: !!opencv-matrix\n   rows: {a.shape[0]}\n   cols: {a.shape[1]}\n   dt: {dt}\n   data: [ {vals} ]\n"


def _mat_xml(name, a, dt="d"):
    a = np.asarray(a, np.float64)
    vals = " ".join(repr(float(v)) for v in a.ravel())
    return (f'<{name} type_id="opencv-matrix">\n  <rows>{a.shape[0]}</rows>\n  <cols>{a.shape[1]}</cols>\n'
            f"  <dt>{dt}</dt>\n  <data>\n    {vals}</data></{name}>\n")


def outlier_noise(e: int, n: int, px: float) -> np.ndarray:
    """The per-corner error of a bad detection (seeded by the edge): a pose cannot absorb it, so
    only the corrupted view's mean error exceeds removeOutlier's 0.5 px."""
    return np.random.default_rng(1000 + e).normal(size=(n, 2)) * px


def write_dataset(p: "rig.Problem", root: str, outlier_edges=(), outlier_px=2.0, back_views=0, ts0=100000,
                  serials=None, ds_config=None):
    """Writes p's views as corner files (one per edge) and camera configs under root.
    outlier_edges: edge indices whose corners get outlier_noise(e, n, outlier_px) (outliers for
    pass 1);
    back_views: extra 70-corner files per camera (back-pattern views the loader must drop).
    serials: camera serial names (default cam00, cam01, ...); ds_config: also write the rig's
    double-side transform there (key "transform", src/mymulticalib.cpp:99-103).
    Returns (serials, data dir, config dir, {file: edge}, timestamps of the rig's photos)."""
    serials = list(serials) if serials is not None else [f"cam{c:02d}" for c in range(p.n_cams)]
    if ds_config is not None:
        with open(ds_config, "w") as f:
            f.write("%YAML:1.0\n---\n" + _mat_yaml("transform", p.ds_pose))
    data, config = os.path.join(root, "data"), os.path.join(root, "config")
    os.makedirs(config, exist_ok=True)
    for c, s in enumerate(serials):
        os.makedirs(os.path.join(data, s), exist_ok=True)
        with open(os.path.join(config, s + ".xml"), "w") as f:
            f.write('<?xml version="1.0"?>\n<opencv_storage>\n<depth_scale>1.0000000474974513e-03</depth_scale>\n'
                    "<height>480.</height>\n")
            f.write(_mat_xml("CameraMatrix", p.cam_pose[c] if p.cam_pose is not None else np.eye(4)))
            f.write(_mat_xml("Intrinsics", p.K[c]))
            f.write(_mat_xml("Distortion", p.D[c][None, :]))
            f.write("</opencv_storage>\n")
    stamps = ts0 + np.arange(p.n_photos)
    files = {}
    out = set(int(e) for e in outlier_edges)
    for e in range(p.n_edges):
        c, ph = int(p.edge_cam[e]), int(p.edge_photo[e])
        o, n = int(p.edge_off[e]), int(p.edge_n[e])
        img = np.asarray(p.img[o:o + n], np.float64)
        if e in out:
            img = img + outlier_noise(e, n, outlier_px)
        fn = os.path.join(data, serials[c], f"{stamps[ph]}.yaml")
        with open(fn, "w") as f:
            f.write("%YAML:1.0\n---\n")
            f.write(_mat_yaml("corners", img))
            f.write(_mat_yaml("objects", np.asarray(p.obj[o:o + n], np.float64)))
        files[fn] = e
    for c, s in enumerate(serials):   # back-pattern views (70 corners): MyMulti's storeReaded drops them
        for k in range(back_views):
            e = int(np.nonzero(p.edge_cam == c)[0][k])
            o = int(p.edge_off[e])
            fn = os.path.join(data, s, f"{ts0 + p.n_photos + 1000 + k}.yaml")
            with open(fn, "w") as f:
                f.write("%YAML:1.0\n---\n")
                f.write(_mat_yaml("corners", np.asarray(p.img[o:o + 70], np.float64)))
                f.write(_mat_yaml("objects", np.asarray(p.obj[o:o + 70], np.float64)))
    return serials, data, config, files, stamps


def read_dump(path):
    """The sample's --dump-problem blob -> (rig.Problem with x0 = the sample's buildParas(),
    photo timestamps)."""
    b = open(path, "rb").read()
    pos = 0

    def take(dt, n):
        nonlocal pos
        a = np.frombuffer(b, dt, n, pos)
        pos += a.nbytes
        return a.copy()

    h = take(np.int32, 11)
    assert h[0] == MAGIC
    model, C, V, E, nd, corners, has_ds, has_cp = (int(v) for v in h[1:9])
    take(np.float64, 1)
    ecam, ephoto, eside, eoff, en = (take(np.int32, E) for _ in range(5))
    obj = take(np.float32, 3 * corners).reshape(-1, 3)
    img = take(np.float32, 2 * corners).reshape(-1, 2)
    K = take(np.float32, 9 * C).reshape(C, 3, 3)
    D = take(np.float32, nd * C).reshape(C, nd)
    xi = take(np.float32, C)
    ds = take(np.float64, 16).reshape(4, 4) if has_ds else None
    cp = take(np.float32, 16 * C).reshape(C, 4, 4) if has_cp else None
    P = (6 if model == rig.DOUBLESIDE else 6 * (C - 1)) + 6 * V
    x0 = take(np.float32, P)
    ts = take(np.int32, V)
    assert pos == len(b)
    prob = rig.Problem(model=model, n_cams=C, n_photos=V, edge_cam=ecam, edge_photo=ephoto, edge_side=eside,
                       edge_off=eoff, edge_n=en, obj=obj, img=img, K=K, D=D, xi=xi, ds_pose=ds, cam_pose=cp,
                       x0=x0, x_true=x0.copy(), timestamps=ts.astype(np.int64), image_size=(1920, 1080),
                       name="sample-dump")
    return prob, ts


def read_result(path):
    out = {"outliers": []}
    for line in open(path):
        t = line.split()
        if not t:
            continue
        if t[0] == "x":
            out["x"] = np.array([float(v) for v in t[1:]], np.float32)
        elif t[0] == "outlier":
            out["outliers"].append(line.split(" ", 1)[1].strip())
        elif t[0] == "iterations":
            out["iterations"] = int(t[1])
        elif t[0] == "error_exact":
            out["error"] = float(t[1])
    return out


def write_omni_list(p: "rig.Problem", root: str, ts0: int = 500, few_points=(), extra_views=0):
    """An omnidirectional rig as the base MultiCameraCalibration reads it on this build
    (include/mcc_multicalib.hpp loadImages): an imagelist_creator list `images.yaml` whose first
    entry is the pattern and whose others are per-view corner files `cameraIdx-timestamp.yaml`
    (imagePoints N x 1 2-channel, objectPoints N x 1 3-channel, imageSize), in the reference's
    file naming (tutorials/multi_camera_tutorial.markdown).  few_points: edges written with only
    15 points (dropped by nMiniMatches = 20).  extra_views: per camera, that many single-camera
    views of wide-angle board poses (rig.make_omni_views with the camera's intrinsics) under
    timestamps of their own -- what the per-camera intrinsic calibration needs beyond the rig's
    distant shared views; they become one-edge photo vertices (the reference keeps those:
    simplifyPhotoVertexs is commented out, src/multicalib.cpp:351).
    Returns (list path, {file: edge (-1 - k for extra view k)}, photo timestamps)."""
    os.makedirs(root, exist_ok=True)
    stamps = ts0 + np.arange(p.n_photos)
    files, names = {}, ["pattern.png"]
    few = set(int(e) for e in few_points)
    W, H = p.image_size
    for e in range(p.n_edges):
        c, ph = int(p.edge_cam[e]), int(p.edge_photo[e])
        o, n = int(p.edge_off[e]), int(p.edge_n[e])
        if e in few:
            n = 15
        name = f"{c}-{stamps[ph]}.yaml"
        img = np.asarray(p.img[o:o + n], np.float64)
        obj = np.asarray(p.obj[o:o + n], np.float64)
        with open(os.path.join(root, name), "w") as f:
            f.write("%YAML:1.0\n---\n")
            f.write(f"imagePoints: !!opencv-matrix\n   rows: {n}\n   cols: 1\n   dt: \"2f\"\n   data: [ "
                    + ", ".join(repr(float(v)) for v in img.ravel()) + " ]\n")
            f.write(f"objectPoints: !!opencv-matrix\n   rows: {n}\n   cols: 1\n   dt: \"3f\"\n   data: [ "
                    + ", ".join(repr(float(v)) for v in obj.ravel()) + " ]\n")
            f.write(f"imageSize: [ {int(W)}, {int(H)} ]\n")
        files[os.path.join(root, name)] = e
        names.append(name)
    k = 0
    for c in range(p.n_cams):
        if not extra_views:
            break
        v = rig.make_omni_views(extra_views, seed=100 + c, K=p.K[c], xi=float(p.xi[c]), D=p.D[c])
        for i in range(v.n_views):
            sl = slice(v.off[i], v.off[i + 1])
            n = int(v.off[i + 1] - v.off[i])
            name = f"{c}-{ts0 + p.n_photos + 1000 + k}.yaml"
            with open(os.path.join(root, name), "w") as f:
                f.write("%YAML:1.0\n---\n")
                f.write(f"imagePoints: !!opencv-matrix\n   rows: {n}\n   cols: 1\n   dt: \"2f\"\n   data: [ "
                        + ", ".join(repr(float(x)) for x in v.img[sl].ravel()) + " ]\n")
                f.write(f"objectPoints: !!opencv-matrix\n   rows: {n}\n   cols: 1\n   dt: \"3f\"\n   data: [ "
                        + ", ".join(repr(float(x)) for x in v.obj[sl].ravel()) + " ]\n")
                f.write(f"imageSize: [ {int(W)}, {int(H)} ]\n")
            files[os.path.join(root, name)] = -1 - k
            names.append(name)
            k += 1
    lst = os.path.join(root, "images.yaml")
    with open(lst, "w") as f:
        f.write("%YAML:1.0\n---\nimages:\n" + "".join(f"   - {nm}\n" for nm in names))
    return lst, files, stamps
