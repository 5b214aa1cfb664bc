"""The reference's own known-answer tests on the HIP path (VERDICT r4 "missing" item 3).

camodocal/PinholeCamera_test.cc:10-85 is the only known-answer test the reference holds for this
path's arithmetic.  tests/test_oracle_math.py checks it against the oracle; here the same camera
(k1 = -0.473, k2 = 0.273, p1 = -0.001, p2 = 0.001, fx = 712.557492, fy = 714.825860,
cx = 370.075592, cy = 244.759309; :12-14) goes through the GPU's residual sweep (mcc_debug_residuals,
the k_linearize / k_group / k_edge projection the optimiser uses):

  * P = (0, 0, 1) at the identity pose lands on (cx, cy) exactly at float32 (spaceToPlane, :16-43; the
    reference stores K as CV_32F, src/mymulticalib.cpp:118-132, so float32 cx, cy is the answer);
  * P = (1, -1, 4) projects to the oracle's pixel bitwise (the consistency test's forward half,
    :65-85; its lift-back half is checked on the oracle, whose projection this pins the device to).

The residual is fl32(obs - proj) (src/mymulticalib.cpp:566-571); with obs = (0, 0) it is -proj
exactly.  Camera 0 is fixed at the identity (buildParas, src/multicalib.cpp:422-440) and the photo's
pose is set to rvec = tvec = 0, so the composed edge pose is the identity and camera-frame points are
the object points (the theta = 0 Rodrigues branch on both sides).  Every path runs it: the fused step,
the split step's k_group and the three-kernel split step.
"""
import numpy as np
import pytest

from multi_camera_calibration_amd import api, rig
from oracle import oracle_py as O

pytestmark = pytest.mark.gpu

CAMO_D = np.array([-0.473, 0.273, -0.001, 0.001], np.float32)
CAMO_K = np.array([[712.557492, 0, 370.075592], [0, 714.825860, 244.759309], [0, 0, 1]], np.float32)
KAT = [(0.0, 0.0, 1.0), (1.0, -1.0, 4.0)]


def _kat_problem():
    p = rig.make_rig(rig.PINHOLE, n_cams=2, n_views=6, board=(9, 6), seed=1)
    p.D = np.concatenate([CAMO_D[None, :], p.D[1:2, :4]], 0).astype(np.float32)   # nd = 4 (k1 k2 p1 p2)
    p.K = p.K.astype(np.float32).copy()
    p.K[0] = CAMO_K
    e0 = int(np.flatnonzero(p.edge_cam == 0)[0])
    ph = int(p.edge_photo[e0])
    x = p.x0.copy()
    c = int(p.photo_col(ph))
    x[c:c + 6] = 0.0
    # every corner of the photo's edges in front of both cameras (z >= 1); the KAT points first
    obj = p.obj.copy()
    img = p.img.copy()
    for e in np.flatnonzero(p.edge_photo == ph):
        o, n = int(p.edge_off[e]), int(p.edge_n[e])
        k = np.arange(n, dtype=np.float64)
        obj[o:o + n] = np.stack([0.05 * k - 1.0, 0.5 - 0.03 * k, 1.0 + 0.1 * k], 1).astype(np.float32)
    o0 = int(p.edge_off[e0])
    obj[o0:o0 + 2] = np.array(KAT, np.float32)
    img[o0:o0 + 2] = 0.0
    p.obj, p.img, p.x0 = obj, img, x
    return p, o0


@pytest.mark.parametrize("env", [{}, {"MCC_FUSED": "0"}, {"MCC_FUSED": "0", "MCC_GROUP": "0"}],
                         ids=["fused", "k_group", "three_kernel"])
def test_camodocal_known_answers_on_gpu(env, monkeypatch):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    p, o0 = _kat_problem()
    ba = api.BundleAdjuster(p)
    try:
        kern = ba.step_kernels()
        r = ba.residuals(p.x0)
    finally:
        ba.close()
    assert kern == {"fused": "k_linearize", "k_group": "k_group", "three_kernel": "k_prep+k_edge+k_photo"}[
        {(): "fused", ("MCC_FUSED",): "k_group", ("MCC_FUSED", "MCC_GROUP"): "three_kernel"}[tuple(env)]]
    proj = -r[2 * o0:2 * o0 + 4].reshape(2, 2)
    # spaceToPlane (:16-43): the optical axis lands on the principal point, float32-exact
    assert proj[0, 0] == np.float32(370.075592) and proj[0, 1] == np.float32(244.759309), proj[0]
    # consistency (:65-85): (1, -1, 4) is the oracle's pixel, bitwise
    ref, _ = O.project_pinhole(np.array([KAT[1]], np.float32), np.zeros(3), np.zeros(3), CAMO_K, CAMO_D, jac=False)
    ref = ref[0].astype(np.float32)
    assert np.array_equal(proj[1].view(np.int32), ref.view(np.int32)), (proj[1], ref)
    # and the whole problem's residuals against the oracle's (test_gpu_parity's bar)
    o = O.Oracle(p)
    full = np.concatenate([o.edge_linearize(p.x0, e)[2] for e in range(p.n_edges)]).astype(np.float32)
    diff = r != full
    assert diff.sum() <= 1 + 1e-5 * r.size, int(diff.sum())
    if diff.any():
        assert np.abs(r[diff].view(np.int32) - full[diff].view(np.int32)).max() <= 1
