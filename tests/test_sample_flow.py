"""The reference sample's flow on this build: MyMultiCameraCalibration
over corner files -> loadImages (solvePnP init, multi-camera filter) -> initialize (graph BFS) ->
optimizeExtrinsics (GPU) -> removeOutlier -> reset -> loadImages(outliers) -> initialize ->
optimizeExtrinsics -> writeParameters (samples/multi_cameras_calibration.cpp:46-83).

Driven through multi_camera_calibration_amd/build/multi_cameras_calibration on a synthetic rig
written in the reference's on-disk layout (tests/sample_data.py; the reference's own corner data
is not in its repository).

CPU: the loaded problem (edges in camera-major file order, photo vertices in first-appearance
order, points, the 88-corner front filter) equals the rig's; the solvePnP + BFS initial poses are
close to the truth; the FileStorage reader parses the reference's tutorial XML.
GPU: outliers found are exactly the corrupted files; the pass-2 optimisation equals the oracle
run on the sample's own problem and initial vector; the written XML results and rewritten camera
configs carry the optimised poses.
"""
import os
import subprocess
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from multi_camera_calibration_amd import api, rig
from oracle import oracle_py as O

import sample_data as SD

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUTORIAL = "/root/reference/tutorials/data"


@pytest.fixture(scope="module")
def sample():
    api.build()
    return api.SAMPLE_PATH


def _rig():
    return rig.make_rig(n_cams=3, n_views=40, seed=11, visibility=0.7)


def _run(sample, args, timeout=300):
    r = subprocess.run([sample] + args, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _rot(rv):
    rv = np.asarray(rv, np.float64)
    th = np.linalg.norm(rv)
    if th < 1e-300:
        return np.eye(3)
    k = rv / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def test_storage_reads_reference_tutorial_data(tmp_path):
    if not os.path.isdir(TUTORIAL):
        pytest.skip("reference tutorial data not present")
    api.build()
    exe = str(tmp_path / "t")
    libdir = os.path.dirname(api.LIB_PATH)
    subprocess.run(["g++", "-std=c++17", "-O2", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "test_multicalib.cpp"), "-L", libdir, "-lmcc_host", "-lmcc",
                    f"-Wl,-rpath,{libdir}", "-o", exe], check=True)
    out = subprocess.run([exe, "storage", os.path.join(TUTORIAL, "omni_calib_data.xml")], capture_output=True,
                         text=True, check=True).stdout.split("\n")
    assert "objectPoints seq 15 mat" in out and "imagePoints seq 15 mat" in out and "imageSize seq 2 scalar" in out
    out = subprocess.run([exe, "storage", os.path.join(TUTORIAL, "omni_stereocalib_data.xml")], capture_output=True,
                         text=True, check=True).stdout.split("\n")
    assert "objectPoints seq 39 mat" in out and "imagePoints2 seq 39 mat" in out


def _expected_order(p, stamps, skip_edges=()):
    """Edges as loadImages builds them: per camera, its views in file (timestamp) order; photo
    vertices in order of first appearance (getPhotoVertex)."""
    skip = set(int(e) for e in skip_edges)
    edges = []
    for c in range(p.n_cams):
        es = [int(e) for e in np.nonzero(p.edge_cam == c)[0] if int(e) not in skip]
        es.sort(key=lambda e: stamps[int(p.edge_photo[e])])
        edges += es
    # the multi-camera filter: timestamps seen by >= 2 cameras among the kept views
    cnt = {}
    for e in edges:
        cnt[int(p.edge_photo[e])] = cnt.get(int(p.edge_photo[e]), 0) + 1
    edges = [e for e in edges if cnt[int(p.edge_photo[e])] >= 2]
    photos = []
    for e in edges:
        ph = int(p.edge_photo[e])
        if ph not in photos:
            photos.append(ph)
    return edges, photos


def test_sample_load_initialize_cpu(sample, tmp_path):
    p = _rig()
    outl = [3, 17, 40]
    serials, data, config, files, stamps = SD.write_dataset(p, str(tmp_path), outlier_edges=outl, back_views=2)
    dump = str(tmp_path / "problem.bin")
    _run(sample, ["--serials", ",".join(serials), "--data", data, "--config", config, "--init-only",
                  "--dump-problem", dump])
    q, ts = SD.read_dump(dump)
    edges, photos = _expected_order(p, stamps)
    assert q.n_edges == len(edges) and q.n_photos == len(photos)   # back views (70 corners) dropped
    assert list(ts) == [int(stamps[ph]) for ph in photos]
    for k, e in enumerate(edges):
        assert int(q.edge_cam[k]) == int(p.edge_cam[e])
        assert photos[int(q.edge_photo[k])] == int(p.edge_photo[e])
        o, n = int(p.edge_off[e]), int(p.edge_n[e])
        qo = int(q.edge_off[k])
        assert np.array_equal(q.obj[qo:qo + n], p.obj[o:o + n])
        shift = SD.outlier_noise(e, n, 2.0) if e in outl else 0.0
        assert np.array_equal(q.img[qo:qo + n], (p.img[o:o + n].astype(np.float64) + shift).astype(np.float32))
    # solvePnP + BFS chaining: initial poses near the truth (0.2 px noise, outliers 2 px, errors
    # accumulate along the chain; solvePnP itself is pinned on exact data by the C++ selftest)
    m = 6 * (p.n_cams - 1)
    for c in range(1, p.n_cams):
        xq, xt = q.x0[6 * (c - 1):6 * c], p.x_true[6 * (c - 1):6 * c]
        assert np.abs(_rot(xq[:3]) - _rot(xt[:3])).max() < 1e-2
        assert np.abs(xq[3:] - xt[3:]).max() < 20.0
    for k, ph in enumerate(photos):
        xq, xt = q.x0[m + 6 * k:m + 6 * k + 6], p.x_true[p.photo_col(ph):p.photo_col(ph) + 6]
        assert np.abs(_rot(xq[:3]) - _rot(xt[:3])).max() < 1e-2
        assert np.abs(xq[3:] - xt[3:]).max() < 20.0


def test_strict_reference_invalid_pose(sample, tmp_path):
    """A view whose solvePnP pose fails isValidPose (300 < |t| < 3000 mm): the default loader drops
    it with the reference's message (src/mymulticalib.cpp:292-299); strict-reference mode
    (MCC_STRICT_REFERENCE=1) aborts as the reference's assert does (src/mymulticalib.cpp:210,
    calcPatternPose).  Host only: the loader runs before any device work."""
    p = _rig()
    serials, data, config, files, stamps = SD.write_dataset(p, str(tmp_path))
    far = sorted(files)[0]   # objects x 4 with the same corners: the same view seen 4x farther away
    txt = open(far).read()
    head, objs = txt.split("objects:")
    e = files[far]
    o, n = int(p.edge_off[e]), int(p.edge_n[e])
    with open(far, "w") as f:
        f.write(head + SD._mat_yaml("objects", 4.0 * np.asarray(p.obj[o:o + n], np.float64)))
    args = ["--serials", ",".join(serials), "--data", data, "--config", config, "--init-only"]
    out = _run(sample, args)
    assert "invalid pattern" in out and far in out
    r = subprocess.run([sample] + args, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MCC_STRICT_REFERENCE="1"))
    assert r.returncode in (-6, 134), (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "isValidPose(tvec)" in r.stderr and "src/mymulticalib.cpp:210" in r.stderr


def _xml_mat(root, key):
    e = root.find(key)
    rows, cols = int(e.find("rows").text), int(e.find("cols").text)
    return np.array([float(v) for v in e.find("data").text.split()]).reshape(rows, cols)


@pytest.mark.gpu
def test_sample_two_pass_flow(sample, tmp_path):
    p = _rig()
    outl = [3, 17, 40]
    serials, data, config, files, stamps = SD.write_dataset(p, str(tmp_path), outlier_edges=outl, back_views=2)
    dump, res, out = str(tmp_path / "problem.bin"), str(tmp_path / "result.txt"), str(tmp_path / "results.xml")
    _run(sample, ["--serials", ",".join(serials), "--data", data, "--config", config, "--out", out,
                  "--dump-problem", dump, "--dump-result", res])
    r = SD.read_result(res)
    # pass 1 finds exactly the corrupted views (per-edge mean error > 0.5 px)
    assert sorted(r["outliers"]) == sorted(fn for fn, e in files.items() if e in outl)
    # pass 2: the sample's own problem and initial vector through the oracle
    q, ts = SD.read_dump(dump)
    edges, photos = _expected_order(p, stamps, skip_edges=outl)
    assert q.n_edges == len(edges)
    crit = (3, 200, 1e-7)
    x_ref, m_ref, it_ref, _ = O.Oracle(q).optimize(q.x0, *crit)
    assert r["iterations"] == it_ref
    assert abs(r["error"] - m_ref) <= 1e-6
    xo = r["x"].astype(np.float64).reshape(-1, 6)
    xr = np.asarray(x_ref, np.float64).reshape(-1, 6)
    for a, b in zip(xo, xr):   # as poses (buildParas' matrix -> vector step may flip near pi)
        assert np.abs(_rot(a[:3]) - _rot(b[:3])).max() <= 1e-3
    assert np.abs(xo[:, 3:] - xr[:, 3:]).max() <= 1e-4 * np.abs(xr[:, 3:]).max()
    # writeParameters: the reference's keys and the optimised poses
    root = ET.parse(out).getroot()
    assert int(root.find("nCameras").text) == 3
    assert abs(float(root.find("meanReprojectError").text) - r["error"]) <= 1e-12 * max(1.0, r["error"])
    assert np.allclose(_xml_mat(root, "camera_pose_0"), np.eye(4))
    for c in range(1, 3):
        P = _xml_mat(root, f"camera_pose_{c}")
        assert np.abs(P[:3, :3] - _rot(xo[c - 1, :3])).max() <= 1e-5   # float Rodrigues round trips
        assert np.abs(P[:3, 3] - xo[c - 1, 3:]).max() <= 1e-3
        assert np.allclose(_xml_mat(root, f"camera_matrix_{c}"), p.K[c], rtol=1e-6)
    assert sum(1 for e in root if e.tag.startswith("pose_timestamp_")) == q.n_photos
    # writeParameters2config: each camera config rewritten with CameraMatrix = its pose
    for c, s in enumerate(serials):
        croot = ET.parse(os.path.join(config, s + ".xml")).getroot()
        assert np.allclose(_xml_mat(croot, "CameraMatrix"), _xml_mat(root, f"camera_pose_{c}"))
        assert np.allclose(_xml_mat(croot, "Intrinsics"), p.K[c], rtol=1e-6)
        assert croot.find("depth_scale") is not None and croot.find("height") is not None


# ---------------------------------------------------------------- DoubleSideCalibration
def _ds_rig():
    return rig.make_config("config5", n_views=16)


def _expected_order_ds(p, stamps, skip_edges=()):
    """DoubleSide loadImages: every view is stored; a view enters when another camera saw the
    other side at the same timestamp (findTimStamp, src/doubleSide.cpp:100-112)."""
    skip = set(int(e) for e in skip_edges)
    edges = []
    for c in range(p.n_cams):
        es = [int(e) for e in np.nonzero(p.edge_cam == c)[0] if int(e) not in skip]
        es.sort(key=lambda e: stamps[int(p.edge_photo[e])])
        edges += es
    sides = {}
    for e in edges:
        sides.setdefault(int(p.edge_photo[e]), set()).add(int(p.edge_n[e]))
    edges = [e for e in edges if len(sides[int(p.edge_photo[e])]) >= 2]
    photos = []
    for e in edges:
        if int(p.edge_photo[e]) not in photos:
            photos.append(int(p.edge_photo[e]))
    return edges, photos


def _pose(x6):
    P = np.eye(4)
    P[:3, :3] = _rot(x6[:3])
    P[:3, 3] = x6[3:]
    return P


def test_doubleside_load_initialize_cpu(sample, tmp_path):
    p = _ds_rig()
    serials, data, config, files, stamps = SD.write_dataset(p, str(tmp_path))
    dump = str(tmp_path / "problem.bin")
    _run(sample, ["--double-side", "--serials", ",".join(serials), "--data", data, "--config", config,
                  "--init-only", "--dump-problem", dump])
    q, ts = SD.read_dump(dump)
    assert q.model == rig.DOUBLESIDE
    edges, photos = _expected_order_ds(p, stamps)
    assert q.n_edges == len(edges) and list(ts) == [int(stamps[ph]) for ph in photos]
    assert np.array_equal(q.cam_pose, p.cam_pose)
    for k, e in enumerate(edges):
        assert int(q.edge_cam[k]) == int(p.edge_cam[e]) and int(q.edge_side[k]) == int(p.edge_side[e])
        o, n, qo = int(p.edge_off[e]), int(p.edge_n[e]), int(q.edge_off[k])
        assert np.array_equal(q.obj[qo:qo + n], p.obj[o:o + n]) and np.array_equal(q.img[qo:qo + n], p.img[o:o + n])
    # the double-side transform from the first photo seen on both sides, then the photos
    assert np.abs(_pose(q.x0[:6]) - _pose(p.x_true[:6]))[:3, :3].max() < 1e-2
    assert np.abs(_pose(q.x0[:6]) - _pose(p.x_true[:6]))[:3, 3].max() < 20.0
    for k, ph in enumerate(photos):
        xq, xt = q.x0[6 + 6 * k:12 + 6 * k], p.x_true[p.photo_col(ph):p.photo_col(ph) + 6]
        assert np.abs(_rot(xq[:3]) - _rot(xt[:3])).max() < 1e-2
        assert np.abs(xq[3:] - xt[3:]).max() < 20.0


@pytest.mark.gpu
def test_doubleside_two_pass_flow(sample, tmp_path):
    p = _ds_rig()
    outl = [5, 30]
    serials, data, config, files, stamps = SD.write_dataset(p, str(tmp_path), outlier_edges=outl)
    dump, res = str(tmp_path / "problem.bin"), str(tmp_path / "result.txt")
    r0 = subprocess.run([sample, "--double-side", "--serials", ",".join(serials), "--data", data, "--config", config,
                         "--dump-problem", dump, "--dump-result", res], capture_output=True, text=True,
                        timeout=300, cwd=str(tmp_path))
    assert r0.returncode == 0, r0.stdout[-3000:] + r0.stderr[-3000:]
    r = SD.read_result(res)
    assert sorted(r["outliers"]) == sorted(fn for fn, e in files.items() if e in outl)
    q, ts = SD.read_dump(dump)
    edges, photos = _expected_order_ds(p, stamps, skip_edges=outl)
    assert q.n_edges == len(edges)
    x_ref, m_ref, it_ref, _ = O.Oracle(q).optimize(q.x0, 3, 200, 1e-8)   # DoubleSide's TermCriteria
    assert r["iterations"] == it_ref
    assert abs(r["error"] - m_ref) <= 1e-6
    xo = r["x"].astype(np.float64).reshape(-1, 6)
    xr = np.asarray(x_ref, np.float64).reshape(-1, 6)
    for a, b in zip(xo, xr):
        assert np.abs(_rot(a[:3]) - _rot(b[:3])).max() <= 1e-3
    assert np.abs(xo[:, 3:] - xr[:, 3:]).max() <= 1e-4 * np.abs(xr[:, 3:]).max()
    # writeParameters: doublesideTransform.yaml in the working directory, key "transform"
    txt = open(tmp_path / "doublesideTransform.yaml").read()
    vals = [float(v) for v in txt.split("data:")[1].replace("[", " ").replace("]", " ").replace(",", " ").split()]
    T = np.array(vals).reshape(4, 4)
    assert np.abs(T - _pose(xo[0])).max() <= 1e-3 * max(1.0, np.abs(T).max())
    assert np.abs(T[:3, 3] - p.x_true[3:6]).max() < 5.0   # near the synthetic truth


# ---------------------------------------------------------------- base class, omnidirectional
def _omni_rig():
    return rig.make_config("config4", n_views=40, seed=21)


EXTRA = 40


def _camera_views(p, cam, few=()):
    """One camera's views in the order the loader reads them (list order: the rig's edges, then
    the extra single-camera views), minus the views with too few points; points as float32 (the
    files hold the rig's float32 values)."""
    few = set(int(e) for e in few)
    es = [e for e in range(p.n_edges) if int(p.edge_cam[e]) == cam and e not in few]
    objs = [p.obj[p.edge_off[e]:p.edge_off[e] + p.edge_n[e]] for e in es]
    imgs = [p.img[p.edge_off[e]:p.edge_off[e] + p.edge_n[e]] for e in es]
    v = rig.make_omni_views(EXTRA, seed=100 + cam, K=p.K[cam], xi=float(p.xi[cam]), D=p.D[cam])
    for i in range(v.n_views):
        objs.append(v.obj[v.off[i]:v.off[i + 1]])
        imgs.append(v.img[v.off[i]:v.off[i + 1]])
    offs = np.cumsum([0] + [len(o) for o in objs]).astype(np.int32)
    obj = np.concatenate(objs).astype(np.float32).astype(np.float64)
    img = np.concatenate(imgs).astype(np.float32).astype(np.float64)
    return O.OmniViews(offs, obj, img), es


def test_omni_list_reader_without_gpu(sample, tmp_path):
    """The list / corner-file reader runs up to the first device call (the per-camera omnidir
    calibration), which must fail loudly without a GPU."""
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("checks the no-GPU failure mode")
    except Exception:
        pass
    p = _omni_rig()
    lst, _, _ = SD.write_omni_list(p, str(tmp_path / "omni"))
    r = subprocess.run([sample, "--list", lst, "--omni", "--cameras", str(p.n_cams), "--init-only"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "error" in r.stderr


@pytest.mark.gpu
def test_omni_base_class_flow(sample, tmp_path):
    """MultiCameraCalibration(OMNIDIRECTIONAL, ...) over a corner-file list: per camera the GPU
    omnidir calibration equals the oracle's on that camera's views; the problem loadImages +
    initialize build has the rig's edges (views with <= nMiniMatches points dropped); the GPU
    optimizeExtrinsics from the sample's own x0 equals the oracle run from it; the results file
    carries xi_i."""
    p = _omni_rig()
    few = [3, 17]
    lst, files, stamps = SD.write_omni_list(p, str(tmp_path / "omni"), few_points=few, extra_views=EXTRA)
    dump, res, out = str(tmp_path / "p.bin"), str(tmp_path / "r.txt"), str(tmp_path / "res.xml")
    _run(sample, ["--list", lst, "--omni", "--cameras", str(p.n_cams), "--min-matches", "20",
                  "--dump-problem", dump, "--dump-result", res, "--out", out])
    q, ts = SD.read_dump(dump)
    assert q.model == rig.OMNI and q.n_cams == p.n_cams
    assert q.n_edges <= p.n_edges - len(few) + EXTRA * p.n_cams
    # intrinsics: exactly mcc_omnidir_calibrate of each camera's kept views in list order with the
    # loader's TermCriteria(COUNT + EPS, 300, 1e-7) (its parity with the oracle restatement is
    # tests/test_omnidir_calib.py's; the dense oracle would take minutes at ~70 views x 300 steps)
    for c in range(p.n_cams):
        v, _ = _camera_views(p, c, few)
        rms, K, xi, D, om, t, idx, it = api.omnidir_calibrate(v.off, v.obj, v.img, p.image_size, 0, 3, 300, 1e-7)
        assert rms < 0.5   # converged to the corner noise (0.2 px per axis)
        np.testing.assert_array_equal(q.K[c], K.astype(np.float32))
        assert q.xi[c] == np.float32(xi)
        np.testing.assert_array_equal(q.D[c], D.astype(np.float32))
    # the extrinsic optimisation from the sample's own x0 (TermCriteria(COUNT, 20, 1e-7))
    r = SD.read_result(res)
    xo, mo, ito, _ = O.Oracle(q).optimize(q.x0, crit_type=1, max_count=20, eps=1e-7)
    assert r["iterations"] == ito == 20
    assert abs(r["error"] - mo) <= 1e-6
    # the dumped x is buildParas() after paras2vertex (pose -> Rodrigues): a rotation whose angle
    # the update pushed past pi comes back as its equivalent (2 pi - angle about -axis), so the
    # rotations are compared as matrices (near pi the float32 log round trip is good to ~1e-5:
    # its axis error scales with 1 / sin(angle))
    xg, xo6 = r["x"].reshape(-1, 6).astype(np.float64), xo.reshape(-1, 6).astype(np.float64)
    for a, b in zip(xg, xo6):
        assert np.abs(_rot(a[:3]) - _rot(b[:3])).max() <= 1e-4
    assert np.abs(xg[:, 3:] - xo6[:, 3:]).max() <= 1e-5 * max(1.0, np.abs(xo6[:, 3:]).max())
    root = ET.parse(out).getroot()
    assert root.find("xi_0") is not None and root.find("nCameras").text.strip() == str(p.n_cams)


STEREO_FIXTURE = os.path.join(ROOT, "tests", "golden", "tutorial_stereo_v20.npz")


def _write_corner_file(path, img, obj, size):
    n = len(img)
    with open(path, "w") as f:
        f.write("%YAML:1.0\n---\n")
        f.write(f"imagePoints: !!opencv-matrix\n   rows: {n}\n   cols: 1\n   dt: \"2f\"\n   data: [ "
                + ", ".join(repr(float(v)) for v in np.asarray(img, np.float32).ravel()) + " ]\n")
        f.write(f"objectPoints: !!opencv-matrix\n   rows: {n}\n   cols: 1\n   dt: \"3f\"\n   data: [ "
                + ", ".join(repr(float(v)) for v in np.asarray(obj, np.float32).ravel()) + " ]\n")
        f.write(f"imageSize: [ {int(size[0])}, {int(size[1])} ]\n")


@pytest.mark.gpu
def test_tutorial_stereo_real_corners(sample, tmp_path):
    """REAL corners through the base-class flow on the GPU: the first 20 views of the reference's
    tutorials/data/omni_stereocalib_data.xml (2 omnidirectional cameras; the corner arrays travel
    in the committed fixture tests/golden/tutorial_stereo_v20.npz) as "camera-timestamp" corner
    files -> MultiCameraCalibration(OMNIDIRECTIONAL, 2, list) loadImages (GPU omnidir calibrate
    per camera) -> initialize -> optimizeExtrinsics (GPU, TermCriteria(COUNT, 20, 1e-7)).
    Against the fixture, which the CPU oracle made along the same flow: the same edges and photo
    vertices, intrinsics and initial poses to the oracle calibration's rounding, and the GPU
    optimisation equal to the oracle's from the sample's own initial vector."""
    g = dict(np.load(STEREO_FIXTURE))
    size = tuple(int(v) for v in g["meta"][3:5])
    root = tmp_path / "stereo"
    os.makedirs(root)
    names = ["pattern.png"]
    for c, key in enumerate(("raw_img1", "raw_img2")):
        for i in range(g[key].shape[0]):
            name = f"{c}-{i}.yaml"
            _write_corner_file(root / name, g[key][i], g["raw_obj"][i], size)
            names.append(name)
    lst = root / "images.yaml"
    lst.write_text("%YAML:1.0\n---\nimages:\n" + "".join(f"   - {nm}\n" for nm in names))
    dump, res, out = str(tmp_path / "p.bin"), str(tmp_path / "r.txt"), str(tmp_path / "res.xml")
    _run(sample, ["--list", str(lst), "--omni", "--cameras", "2", "--min-matches", "20",
                  "--dump-problem", dump, "--dump-result", res, "--out", out])
    q, ts = SD.read_dump(dump)
    p = rig.problem_from_arrays(g)
    # the problem loadImages + initialize built: same kept views, edges, photo vertices, points
    for f in ("edge_cam", "edge_photo", "edge_off", "edge_n"):
        assert np.array_equal(getattr(q, f), getattr(p, f)), f
    assert list(ts) == list(p.timestamps)
    assert np.array_equal(q.obj, p.obj) and np.array_equal(q.img, p.img)
    # intrinsics: GPU calibrate vs the oracle restatement (300 iterations each, float32 stored)
    for c in range(2):
        assert np.allclose(q.K[c], p.K[c], rtol=1e-4, atol=1e-3), (c, q.K[c], p.K[c])
        assert abs(float(q.xi[c]) - float(p.xi[c])) <= 1e-4 * abs(float(p.xi[c])), c
        assert np.allclose(q.D[c], p.D[c], rtol=1e-3, atol=1e-6), (c, q.D[c], p.D[c])
    x0q = q.x0.reshape(-1, 6).astype(np.float64)
    x0p = p.x0.reshape(-1, 6).astype(np.float64)
    for a, b in zip(x0q, x0p):
        assert np.abs(_rot(a[:3]) - _rot(b[:3])).max() <= 1e-3
    assert np.abs(x0q[:, 3:] - x0p[:, 3:]).max() <= 1e-3 * np.abs(x0p[:, 3:]).max()
    # the GPU optimisation from the sample's own problem equals the oracle's (both solvers)
    r = SD.read_result(res)
    o = O.Oracle(q)
    for solver in ("schur", "cg"):
        xo, mo, ito, _ = o.optimize(q.x0, crit_type=1, max_count=20, eps=1e-7, solver=solver)
        assert r["iterations"] == ito == 20
        assert abs(r["error"] - mo) <= 1e-6, (solver, r["error"], mo)
    assert abs(r["error"] - float(g["mean_opt"])) <= 1e-3   # same data, seeds from two calibrations
    root_xml = ET.parse(out).getroot()
    assert root_xml.find("xi_1") is not None and root_xml.find("nCameras").text.strip() == "2"
