"""The drop-in boundary at source level: the reference's own sample,
/root/reference/samples/multi_cameras_calibration.cpp, compiled IN PLACE and unchanged against this
build's source-compatible headers (include/opencv2/ccalib/{multicalib,mymulticalib,doubleSide}.hpp:
cv::multicalib::MyMultiCameraCalibration / DoubleSideCalibration, cv::Size, cv::TermCriteria) and
linked with libmcc_host.so + libmcc.so.  The source file is never copied into this repository:
the CPU test compiles it where it lies (skipped where the reference tree is absent), and the
prebuilt binary (multi_camera_calibration_amd/build/ref_multi_cameras_calibration, made by
api.build() next to the reference) is what the GPU box runs.

The sample hard-codes its serials ("839112060578", "839512061262", "f0220380"), its data folder,
camera-config folder and double-side config (samples/multi_cameras_calibration.cpp:50-53); the
tests write a synthetic 3-camera dataset in the reference's on-disk layout under those serials and
point the hard-coded paths at it with MCC_PATH_MAP (mcc_storage.hpp resolve_path).

CPU: it compiles; it loads and initialises the problem and then fails loudly at the first device
call (no CPU fallback).  GPU: its two-pass run writes the same multi-camera-results.xml, and
rewrites the same camera configs, as this build's own sample on the same data.
"""
import os
import shutil
import subprocess
import xml.etree.ElementTree as ET

import numpy as np
import pytest

from multi_camera_calibration_amd import api, rig

import sample_data as SD

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SERIALS = ["839112060578", "839512061262", "f0220380"]          # samples/multi_cameras_calibration.cpp:53
DATA = "/2t/data/recordedSamples/board/12.14opsite/color"        # :50
CONFIGS = "/home/dd/working/pypose/configs"                      # :51-52 (warmup1hour/, doublesideTransform.yaml)


def _dataset(root):
    p = rig.make_rig(n_cams=3, n_views=40, seed=11, visibility=0.7)   # 11x8 = 88 corners = cv::Size(8,11)
    os.makedirs(os.path.join(root, "configs"), exist_ok=True)
    serials, data, config, files, stamps = SD.write_dataset(
        p, root, outlier_edges=[3, 17, 40], back_views=2, serials=SERIALS,
        ds_config=os.path.join(root, "configs", "doublesideTransform.yaml"))
    shutil.move(config, os.path.join(root, "configs", "warmup1hour"))
    return p, data, os.path.join(root, "configs", "warmup1hour"), files


def _env(root):
    return dict(os.environ, MCC_PATH_MAP=f"{DATA}={root}/data;{CONFIGS}={root}/configs")


def test_reference_sample_compiles_unchanged(tmp_path):
    if not os.path.exists(api.REF_SAMPLE_SRC):
        pytest.skip("the reference tree is not on this machine")
    api.build()
    libdir = os.path.dirname(api.LIB_PATH)
    exe = str(tmp_path / "ref_sample")
    r = subprocess.run(["g++", "-std=c++17", "-I", os.path.join(ROOT, "include", "opencv2", "ccalib"),
                        "-I", os.path.join(ROOT, "include"), api.REF_SAMPLE_SRC, "-L", libdir, "-lmcc_host", "-lmcc",
                        f"-Wl,-rpath,{libdir}", "-o", exe], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert os.path.exists(exe)


def _have_binary():
    if not os.path.exists(api.REF_SAMPLE_PATH):
        pytest.skip("the reference sample binary was not built (no reference tree where build() ran)")


def test_reference_sample_fails_loudly_without_gpu(tmp_path):
    """Unchanged sample, no GPU: the constructor (camera configs, double-side transform),
    loadImages (corner files, solvePnP) and initialize run on the host; optimizeExtrinsics' first
    device call throws (the sample does not catch, so it terminates, as an uncaught cv::Exception
    would) -- never a silent CPU result."""
    _have_binary()
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("checks the no-GPU failure mode")
    except Exception:
        pass
    _dataset(str(tmp_path))
    r = subprocess.run([api.REF_SAMPLE_PATH], cwd=str(tmp_path), env=_env(str(tmp_path)), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0
    assert "mcc:" in r.stderr
    assert not os.path.exists(tmp_path / "multi-camera-results.xml")


def _xml(path):
    out = {}
    for e in ET.parse(path).getroot():
        if e.find("data") is not None:
            out[e.tag] = np.array([float(v) for v in e.find("data").text.split()])
        else:
            out[e.tag] = (e.text or "").strip()
    return out


@pytest.mark.gpu
def test_reference_sample_runs_unchanged(tmp_path):
    _have_binary()
    a, b = tmp_path / "ref", tmp_path / "own"
    os.makedirs(a)
    os.makedirs(b)
    _, _, cfg_a, files_a = _dataset(str(a))
    _, data_b, cfg_b, files_b = _dataset(str(b))
    r = subprocess.run([api.REF_SAMPLE_PATH], cwd=str(a), env=_env(str(a)), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "number of outliers: 3" in r.stdout
    out_b = str(b / "multi-camera-results.xml")
    api.build()
    rb = subprocess.run([api.SAMPLE_PATH, "--serials", ",".join(SERIALS), "--data", data_b, "--config", cfg_b,
                         "--doubleside", str(b / "configs" / "doublesideTransform.yaml"), "--out", out_b],
                        capture_output=True, text=True, timeout=300)
    assert rb.returncode == 0, rb.stdout[-3000:] + rb.stderr[-3000:]
    ra, rb_ = _xml(str(a / "multi-camera-results.xml")), _xml(out_b)
    assert sorted(ra) == sorted(rb_)
    for k in ra:
        if isinstance(ra[k], np.ndarray):
            assert np.array_equal(ra[k], rb_[k]), k
        else:
            assert ra[k] == rb_[k], k
    assert int(ra["nCameras"]) == 3 and float(ra["meanReprojectError"]) < 0.3
    for s in SERIALS:   # writeParameters2config rewrote each camera config alike
        ca, cb = _xml(os.path.join(cfg_a, s + ".xml")), _xml(os.path.join(cfg_b, s + ".xml"))
        assert np.array_equal(ca["CameraMatrix"], cb["CameraMatrix"]), s
