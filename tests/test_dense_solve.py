"""The reduced camera system's dense solve for m > 30 (k_solve's elimination, through
mcc_debug_solve) against numpy.  It replaces the reference's sparse CG on the whole normal
equations (/root/reference/src/multicalib.cpp:565-592); the step-level parity tests cover it end
to end (config3_small, cams22_m126), this pins the solve alone on harder systems: sizes 36..126
(every padding of the 16-wide blocks), conditioning up to 1e8, the camera-block scaling the
reduced system has (rotation rows in radians next to translation rows in mm), and a matrix that is
not positive definite."""
import numpy as np
import pytest

from multi_camera_calibration_amd import api

pytestmark = pytest.mark.gpu


def spd(m, cond, seed, camera_scaling=False):
    rng = np.random.default_rng(seed)
    q, _ = np.linalg.qr(rng.standard_normal((m, m)))
    ev = np.geomspace(1.0, cond, m)
    S = (q * ev) @ q.T
    if camera_scaling:   # 6-blocks: 3 rotation rows (~1) and 3 translation rows (~1e3)
        d = np.tile([1.0, 1.0, 1.0, 1e3, 1e3, 1e3], m // 6 + 1)[:m]
        S = S * np.outer(d, d)
    return 0.5 * (S + S.T), rng.standard_normal(m)


@pytest.mark.parametrize("m", [36, 42, 48, 60, 90, 96, 120, 126])
@pytest.mark.parametrize("cond,scaled", [(1e2, False), (1e6, True), (1e8, False)])
def test_dense_solve_backward_error(m, cond, scaled):
    S, r = spd(m, cond, seed=m, camera_scaling=scaled)
    x, _, _ = api.debug_solve(S, r)
    x_ref = np.linalg.solve(S, r)
    # normwise backward error of a stable SPD elimination: ||S x - r|| <= c m eps ||S|| ||x||
    res = np.linalg.norm(S @ x - r) / (np.linalg.norm(S, 2) * np.linalg.norm(x) + np.linalg.norm(r))
    assert res < 64 * m * np.finfo(np.float64).eps, res
    # forward error within the conditioning bound
    fe = np.linalg.norm(x - x_ref) / np.linalg.norm(x_ref)
    assert fe < 64 * m * np.finfo(np.float64).eps * np.linalg.cond(S), fe


def test_dense_solve_not_pd():
    S, r = spd(90, 1e3, seed=7)
    S[40, 40] = -1.0
    with pytest.raises(api.MccError):
        api.debug_solve(S, r)


def test_dense_solve_timing_and_stamps():
    S, r = spd(90, 1e4, seed=3, camera_scaling=True)
    x, us, st = api.debug_solve(S, r, reps=50, stamps=True)
    assert us is not None and 0.0 < us < 1000.0
    assert st[0] > 0 and st[63] >= st[0]
