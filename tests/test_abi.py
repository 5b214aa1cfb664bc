"""C-ABI boundary checks that need no GPU (libmcc.so loads on a CPU host: it links the HIP and
RCCL runtimes but makes no device call until mcc_create).

* every function include/mcc.h declares is exported by libmcc.so (and nothing mcc_* undeclared);
* argument validation returns MCC_EINVAL with a message, before any device work;
* the photo partitioner (host-only) is deterministic, complete and balanced;
* without a GPU, creating a problem fails loudly (MCC_EHIP) -- the product has no CPU fallback.
"""
import ctypes
import dataclasses
import os
import re
import subprocess

import numpy as np
import pytest

from multi_camera_calibration_amd import api, rig

MCC_EINVAL, MCC_EHIP = -1, -2


@pytest.fixture(scope="module")
def L():
    api.build()
    return api.lib()


def test_header_symbols_exported(L):
    decl = api.declared_symbols()
    assert len(decl) >= 20
    for s in decl:
        assert hasattr(L, s), f"libmcc.so does not export {s}"
    # and the library exports no undeclared mcc_* entry point
    nm = subprocess.run(["nm", "-D", "--defined-only", api.LIB_PATH], capture_output=True, text=True,
                        check=True).stdout
    exported = sorted(set(re.findall(r"\bT (mcc_[a-z_]+)$", nm, re.M)))
    assert exported == decl


def test_header_constants_match_python():
    txt = open(api.HEADER).read()
    consts = dict((k, int(v)) for k, v in re.findall(r"#define (MCC_[A-Z_0-9]+) \(?(-?\d+)\)?", txt))
    assert consts["MCC_MODEL_PINHOLE"] == rig.PINHOLE
    assert consts["MCC_MODEL_OMNI"] == rig.OMNI
    assert consts["MCC_MODEL_DOUBLESIDE"] == rig.DOUBLESIDE
    assert consts["MCC_FRONT"] == rig.FRONT and consts["MCC_BACK"] == rig.BACK
    assert consts["MCC_EINVAL"] == MCC_EINVAL and consts["MCC_EHIP"] == MCC_EHIP
    assert consts["MCC_UNIQUE_ID_BYTES"] == 128


def test_null_arguments_rejected(L):
    assert L.mcc_create(None, None) == MCC_EINVAL
    assert b"null" in L.mcc_last_error()
    out = ctypes.c_void_p()
    assert L.mcc_create(ctypes.byref(out), None) == MCC_EINVAL
    assert L.mcc_partition_photos(3, 0, None, None, 0, None) == MCC_EINVAL


@pytest.mark.parametrize("bad", ["model", "nd", "edge_range", "omni_back", "too_many_corners", "empty"])
def test_invalid_problem_rejected_before_device_work(bad):
    p = rig.make_config("config1")
    kw = {}
    if bad == "empty":   # no photos / edges: the reference's mean error would be 0/0
        p = dataclasses.replace(p, n_photos=0, edge_cam=p.edge_cam[:0], edge_photo=p.edge_photo[:0],
                                edge_side=p.edge_side[:0], edge_off=p.edge_off[:0], edge_n=p.edge_n[:0],
                                obj=p.obj[:0], img=p.img[:0], x0=p.x0[:6 * (p.n_cams - 1)],
                                x_true=p.x_true[:6 * (p.n_cams - 1)], timestamps=p.timestamps[:0])
    elif bad == "model":
        kw["model"] = 7
    elif bad == "nd":
        p.D = np.zeros((p.n_cams, 6), np.float32)
    elif bad == "edge_range":
        p.edge_cam = p.edge_cam.copy(); p.edge_cam[3] = p.n_cams
    elif bad == "omni_back":
        p = rig.make_config("config4", n_views=4)
        p.edge_side = p.edge_side.copy(); p.edge_side[0] = rig.BACK
    elif bad == "too_many_corners":
        p.edge_n = p.edge_n.copy(); p.edge_n[0] = 2000
    if "model" in kw:
        p.model = kw["model"]
    with pytest.raises(api.MccError) as ei:
        api.BundleAdjuster(p)
    assert "(-1)" in str(ei.value)


# (no torch here: its bundled HIP runtime shares SONAMEs with /opt/rocm's and would shadow it)
@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="checks the no-GPU behaviour")
def test_no_gpu_fails_loudly():
    p = rig.make_config("config1")
    with pytest.raises(api.MccError) as ei:
        api.BundleAdjuster(p)
    assert "(-2)" in str(ei.value)


def test_partition_balanced_and_deterministic():
    p = rig.make_config("config3", n_views=200)
    for n in (1, 2, 3, 8):
        a = api.partition_photos(p, n)
        b = api.partition_photos(p, n)
        assert np.array_equal(a, b)
        assert a.min() >= 0 and a.max() < n and len(np.unique(a)) == n
        w = np.bincount(p.edge_photo, weights=p.edge_n, minlength=p.n_photos)
        load = np.bincount(a, weights=w, minlength=n)
        # greedy longest-first: every rank within one photo's weight of the mean
        assert load.max() - load.min() <= w.max()


def test_partition_shards_cover_problem():
    p = rig.make_config("config2", n_views=40)
    owner = api.partition_photos(p, 3)
    parts = [rig.subset_photos(p, np.nonzero(owner == r)[0]) for r in range(3)]
    assert sum(q.n_edges for q in parts) == p.n_edges
    assert sum(q.n_corners for q in parts) == p.n_corners
    g = p.global_dim
    for q in parts:
        assert np.array_equal(q.x0[:g], p.x0[:g])
