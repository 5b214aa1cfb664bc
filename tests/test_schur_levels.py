"""k_schur's hand-off for m <= 30: one level -- every item and norm chunk
writes its partial, ONE ticket, the last arriver sums each camera-pair block's items in item order and
solves from the sums -- in place of round 3's two levels (blocks, then the blocks and norms).  The
per-entry sums are the same additions in the same order, so the result is bitwise the two-level one
(MCC_SCHUR_ONE_LEVEL=0): the optimize loop (COUNT and EPS), the free-running steps, the linearisation
(deltaX, JTE), single GPU and at world 2 over the peer transport.  The reduction it implements is
the reference's normal equations (src/multicalib.cpp:565-579) reduced onto the cameras; the oracle
comparison of the same paths is tests/test_gpu_parity.py / test_full_size.py."""
import os

import numpy as np
import pytest

from multi_camera_calibration_amd import api, rig

pytestmark = pytest.mark.gpu


def _run(p, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ba = api.BundleAdjuster(p)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        d, j = ba.compute_jacobian_extrinsic(p.x0)
        x, m, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        ba.set_params(p.x0)
        ba.step(24)
        ba.check()
        xs = ba.get_params()
        path = ba.step_kernels()
    finally:
        ba.close()
    return d, j, x, it, xs, path


@pytest.mark.parametrize("cfg,env,want", [
    ("config4", {}, "k_group"),                                          # the headline: k_group -> k_schur
    ("config2", {"MCC_FUSED": "0"}, "k_group"),                           # pinhole m = 18 on the split step
    ("config5", {}, "k_prep+k_edge+k_photo"),                             # DoubleSide m = 6, three kernels
])
def test_one_level_is_bitwise_two_level(cfg, env, want):
    p = rig.make_config(cfg)
    # (the m <= 30 warm solve needs the one-level form: off in both runs, so both eliminate)
    a = _run(p, dict(env, MCC_SCHUR_ONE_LEVEL="1", MCC_SMALL_WARM="0"))
    b = _run(p, dict(env, MCC_SCHUR_ONE_LEVEL="0", MCC_SMALL_WARM="0"))
    assert a[5] == want
    assert a[3] == b[3]
    for u, v in zip(a[:5], b[:5]):
        assert np.array_equal(np.asarray(u), np.asarray(v))
