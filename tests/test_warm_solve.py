"""The warm solve of the m > 30 reduced camera system: k_solve refines with
the previous step's inverse, which the resident helper kernel computes while the next step
linearises, and falls back to the direct elimination (the blocked Gauss-Jordan the oracle's
Schur / Cholesky restatement is pinned against) when the refinement does not converge.  The solve
it replaces is the reference's sparse CG on the whole normal equations
(/root/reference/src/multicalib.cpp:565-592) inside optimizeExtrinsics (:462-514).

  * warm on vs off (MCC_WARM=0): the same iteration count and final float32 parameters within 1 ulp,
    both against the oracle's optimize at the single-GPU bars; the solve statistics show the warm
    path ran (every update step after the first refines);
  * the result does not depend on timing: a helper that holds each inverse back (MCC_WARM_DELAY_US)
    gives bitwise the undelayed result (k_solve waits; it never switches algorithms), a helper that
    does not deliver within MCC_WARM_TIMEOUT_MS fails the step with MCC_ETIMEOUT, and an
    optimisation does not depend on the problem's earlier ones (each starts without an inverse);
  * a NaN inverse (MCC_WARM_POISON=1) makes every warm solve fall back, and the fallback is the
    direct elimination: bitwise the MCC_WARM=0 result;
  * m = 126 (beyond the staged warm path's M <= 96) runs the direct elimination only;
  * the helper's look-ahead inversion (round 6) is bitwise the round-5 schedule's.
"""
import os
import sys

import numpy as np
import pytest

from multi_camera_calibration_amd import api, rig
from oracle import oracle_py as O

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ulp import f32_ulp_diff  # noqa: E402

pytestmark = pytest.mark.gpu

CASES = {
    "config3_small": lambda: rig.make_config("config3", n_views=48),                # m = 90
    "m48": lambda: rig.make_config("config3", n_cams=9, n_views=40),                 # m = 48
    "m126": lambda: rig.make_config("config3", n_cams=22, n_views=120),              # m = 126: direct only
}


def make(p, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return api.BundleAdjuster(p)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def run(p, env):
    ba = make(p, env)
    try:
        x, m, it, ch = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        stats = ba.solve_stats()
    finally:
        ba.close()
    return x, m, it, stats


@pytest.mark.parametrize("name", ["config3_small", "m48"])
def test_warm_matches_direct_and_oracle(name):
    p = CASES[name]()
    x_ref, m_ref, it_ref, _ = O.Oracle(p).optimize(p.x0, crit_type=3, max_count=200, eps=1e-7)
    xw, mw, itw, sw = run(p, {"MCC_WARM": "1"})
    xd, md, itd, sd = run(p, {"MCC_WARM": "0"})
    assert itw == itd == it_ref, (itw, itd, it_ref)
    for x, m in ((xw, mw), (xd, md)):
        assert abs(m - m_ref) <= 1e-6
        assert f32_ulp_diff(x, x_ref).max() <= 1
    assert f32_ulp_diff(xw, xd).max() <= 1
    # every update step but the run's first tried the helper's inverse; from a rough start the
    # systems move too far between the first steps for the previous inverse (those fall back after a
    # correction or two), so only the bench's steady state is required to refine
    # (test_warm_steady_state)
    assert sw["direct"] == 1, sw
    assert sw["warm"] + sw["direct"] >= itw, sw
    assert sw["corrections"] <= 4 * sw["warm"], sw
    assert sd == dict(warm=0, corrections=0, fallbacks=0, direct=0, waited=0)


def test_warm_fallback_is_the_direct_elimination():
    p = CASES["config3_small"]()
    xp, mp, itp, sp = run(p, {"MCC_WARM": "1", "MCC_WARM_POISON": "1"})
    xd, md, itd, _ = run(p, {"MCC_WARM": "0"})
    assert sp["warm"] > 0 and sp["fallbacks"] == sp["warm"], sp
    assert itp == itd and mp == md
    assert np.array_equal(xp, xd)


def test_m126_direct_only():
    p = CASES["m126"]()
    x, m, it, s = run(p, {})
    assert s == dict(warm=0, corrections=0, fallbacks=0, direct=0, waited=0)


def test_warm_steady_state():
    """Free-running steps near convergence (the bench's loop): every solve after the first refines
    with at most two corrections and none falls back."""
    p = CASES["config3_small"]()
    ba = api.BundleAdjuster(p)
    try:
        ba.set_params(p.x0)
        ba.step(40)
        ba.synchronize()
        s0 = ba.solve_stats()
        ba.step(64)
        ba.synchronize()
        ba.check()
        s1 = ba.solve_stats()
    finally:
        ba.close()
    warm = s1["warm"] - s0["warm"]
    assert warm == 64, (s0, s1)
    assert s1["fallbacks"] == s0["fallbacks"], (s0, s1)
    assert s1["corrections"] - s0["corrections"] <= 2 * warm, (s0, s1)


def test_delayed_helper_is_bitwise_the_undelayed_run():
    """A helper that holds every inverse back by 2 ms (4x the round-3 wait bound, after which
    k_solve used to switch to the direct elimination): every k_solve waits, takes the same branch
    and gives the same bits -- the optimize and the free-running steps are bitwise the undelayed
    ones."""
    p = CASES["config3_small"]()
    out = []
    for env in ({}, {"MCC_WARM_DELAY_US": "2000"}, {"MCC_WARM_DELAY_US": "2000", "MCC_HELPER_POLL": "1"}):
        ba = make(p, env)
        try:
            x, m, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
            ba.set_params(p.x0)
            ba.step(24)
            ba.check()
            xs = ba.get_params()
            st = ba.solve_stats()
        finally:
            ba.close()
        out.append((x, it, xs, st))
    (x0, it0, xs0, st0) = out[0]
    for (x1, it1, xs1, st1) in out[1:]:
        assert it0 == it1
        assert np.array_equal(x0, x1) and np.array_equal(xs0, xs1)
        assert st1["waited"] >= st1["warm"] > 0, st1
        for k in ("warm", "corrections", "fallbacks", "direct"):
            assert st0[k] == st1[k], (st0, st1)


@pytest.mark.parametrize("name", ["config3_small", "m48"])
@pytest.mark.parametrize("poll", ["0", "1"])
def test_helper_refinement_is_bitwise_k_solves(name, poll):
    """Single GPU: the helper refines with the inverse it holds in LDS and k_solve only waits for its
    solution (default; MCC_HELPER_REFINE=0: k_solve loads the inverse and refines itself).  The same
    warm_refine on the same system and the same inverse: the optimize, the free-running steps and
    the solve statistics are bitwise / exactly those of the k_solve form.  poll = 1: k_schur publishes
    the system when it starts and the helper stages prev2's words as the blocks land (each word its own
    flag, emptied by the next step's k_schur: the three-kernel step's default); 0: published at
    k_schur's end (k_group's default)."""
    p = CASES[name]()
    out = []
    for env in ({"MCC_HELPER_REFINE": "0"}, {"MCC_HELPER_POLL": poll}):
        ba = make(p, env)
        try:
            x, m, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
            ba.set_params(p.x0)
            ba.step(24)
            ba.check()
            xs = ba.get_params()
            st = ba.solve_stats()
        finally:
            ba.close()
        out.append((x, it, xs, st))
    (x0, it0, xs0, st0), (x1, it1, xs1, st1) = out
    assert it0 == it1
    assert np.array_equal(x0, x1) and np.array_equal(xs0, xs1)
    for k in ("warm", "corrections", "fallbacks", "direct"):
        assert st0[k] == st1[k], (st0, st1)
    assert st1["warm"] > 0


@pytest.mark.parametrize("name", ["config3_small", "m48"])
@pytest.mark.parametrize("refine", ["0", "1"])
def test_lookahead_inverse_is_bitwise_the_round5_schedule(name, refine):
    """The helper's inverse with the look-ahead schedule (gj_inverse_blocked<true>, the k_group path's
    default) is bitwise the round-5 schedule's (MCC_INV_LA=0): the same products in the same order.
    Checked through everything the inverse feeds -- the optimize, the free-running steps and the solve
    statistics -- with the helper refining (refine = 1) and with k_solve refining from the inverse the
    helper stores (0)."""
    p = CASES[name]()
    out = []
    for la in ("0", "1"):
        ba = make(p, {"MCC_INV_LA": la, "MCC_HELPER_REFINE": refine})
        try:
            x, m, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
            ba.set_params(p.x0)
            ba.step(24)
            ba.check()
            xs = ba.get_params()
            st = ba.solve_stats()
        finally:
            ba.close()
        out.append((x, it, xs, st))
    (x0, it0, xs0, st0), (x1, it1, xs1, st1) = out
    assert it0 == it1
    assert np.array_equal(x0, x1) and np.array_equal(xs0, xs1)
    for k in ("warm", "corrections", "fallbacks", "direct"):
        assert st0[k] == st1[k], (st0, st1)
    assert st1["warm"] > 0


def _recovers_on_the_same_handle(ba, p, fresh_env):
    """after a failed optimisation: the delays off, the same handle optimises again and gives bitwise
    a fresh problem's result (nothing the failed launch left behind is read)"""
    ba.debug_delays(spare_delay_us=0, warm_delay_us=0, warm_timeout_ms=10000)
    x, m, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
    xf, mf, itf, _ = run(p, fresh_env)
    assert it == itf and m == mf, (it, itf, m, mf)
    assert np.array_equal(x, xf)


def test_helper_timeout_fails_the_step():
    """A helper slower than MCC_WARM_TIMEOUT_MS: the step fails with MCC_ETIMEOUT (-6) instead of
    switching algorithms, and the problem recovers on the next optimisation of the same handle."""
    p = CASES["config3_small"]()
    ba = make(p, {"MCC_WARM_DELAY_US": "30000", "MCC_WARM_TIMEOUT_MS": "3"})
    try:
        with pytest.raises(api.MccError, match=r"\(-6\)"):
            ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        _recovers_on_the_same_handle(ba, p, {})
    finally:
        ba.close()


@pytest.mark.parametrize("poll", ["0", "1"])
def test_optimize_independent_of_history(poll):
    """Two optimisations on one problem: the second starts without the first's inverse (its first
    solve is the direct elimination), so both give the same bits as a fresh problem.  With the polled
    staging the first optimisation's last system may stay in prev2 unconsumed (the loop stops in k_solve,
    after k_schur wrote it): set_state empties prev2."""
    p = CASES["config3_small"]()
    ba = make(p, {"MCC_HELPER_POLL": poll})
    try:
        a = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        ba.set_params(p.x0)
        ba.step(30)
        ba.synchronize()
        b = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
    finally:
        ba.close()
    assert a[2] == b[2] and np.array_equal(a[0], b[0])


@pytest.mark.parametrize("cfg,views,env", [
    ("config4", 200, {"MCC_FUSED": "0"}),   # k_group -> k_schur: this step's spare workgroup's inverse
    ("config2", 120, {}),                   # the fused step: the previous launch's (two updates stale)
])
def test_small_m_warm_matches_direct_and_oracle(cfg, views, env):
    """The m <= 30 warm solve (default; MCC_SMALL_WARM=0 turns it off): a spare workgroup inverts the
    previous step's system and the final solve refines with it (S and the inverse in registers), or
    eliminates directly when there is no inverse of the right iteration or the refinement does not
    converge.  Same iterations as the direct path and the oracle, float32 parameters within 1 ulp of
    both."""
    p = rig.make_config(cfg, n_views=views)   # m = 18
    x_ref, m_ref, it_ref, _ = O.Oracle(p).optimize(p.x0, crit_type=3, max_count=200, eps=1e-7)
    xw, mw, itw, _ = run(p, dict(env, MCC_SMALL_WARM="1"))
    xd, md, itd, _ = run(p, dict(env, MCC_SMALL_WARM="0"))
    assert itw == itd == it_ref, (itw, itd, it_ref)
    for x, m in ((xw, mw), (xd, md)):
        assert abs(m - m_ref) <= 1e-6
        assert f32_ulp_diff(x, x_ref).max() <= 1
    assert f32_ulp_diff(xw, xd).max() <= 1


def _fused_runs(p, env):
    """optimize (COUNT + EPS) and 24 free-running steps from x0 on a fresh problem; the solve stats"""
    ba = make(p, env)
    try:
        assert ba.path() == "fused", ba.path()
        x, m, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        s_opt = ba.solve_stats()
        ba.set_params(p.x0)
        ba.step(24)
        ba.check()
        xs = ba.get_params()
        s_all = ba.solve_stats()
    finally:
        ba.close()
    return x, it, xs, s_opt, s_all


@pytest.mark.parametrize("views", [120, 512])
def test_fused_spare_delayed_is_bitwise_the_undelayed_run(views):
    """The fused step's m <= 30 warm solve does not depend on when its spare workgroup runs: the spare
    acknowledges once it holds the previous launch's system, and the final arriver writes neither the
    packed system nor the state before that (small_inverse / spare_wait).  A spare held back by
    MCC_SPARE_DELAY_US = 300 us (ten steps' time: it starts long after the final arriver reached the
    solve) gives bitwise the undelayed optimize and free-running steps, with the same refinement
    statistics; only 'waited' differs.  512 views is the fused path's largest rig (V = 2 x CUs): a grid
    of 513 workgroups, one more than the co-resident slots, so the spare starts only after a photo
    exits.  Both runs repeat bitwise (a second undelayed run), and refine: every update step after
    the first two has an inverse of the right iteration.  The loop is src/multicalib.cpp:462-514."""
    p = rig.make_config("config2", n_views=views)
    st = {"MCC_SOLVE_STATS": "1"}   # the m <= 30 counters (off by default: ~0.5 us per step)
    runs = [_fused_runs(p, dict(st, **env)) for env in ({}, {}, {"MCC_SPARE_DELAY_US": "300"})]
    (x0, it0, xs0, so0, sa0) = runs[0]
    for (x, it, xs, so, sa) in runs[1:]:
        assert it == it0
        assert np.array_equal(x, x0) and np.array_equal(xs, xs0)
        for k in ("warm", "corrections", "fallbacks", "direct"):
            assert so[k] == so0[k] and sa[k] == sa0[k], (so0, so, sa0, sa)
    assert so0["warm"] >= it0 - 3 and so0["warm"] > 0, (it0, so0)
    assert runs[2][4]["waited"] > 0, runs[2][4]
    assert runs[0][4]["waited"] == 0 or views == 512, runs[0][4]
    x_ref, m_ref, it_ref, _ = O.Oracle(p).optimize(p.x0, crit_type=3, max_count=200, eps=1e-7)
    assert it0 == it_ref
    assert f32_ulp_diff(x0, x_ref).max() <= (1 if views <= 120 else 2)


def test_fused_spare_timeout_fails_the_step():
    """A spare slower than the bound (MCC_SPARE_DELAY_US = 30 ms, MCC_WARM_TIMEOUT_MS = 3): the step
    fails with MCC_ETIMEOUT (-6) before writing the system or the state, and a fresh problem recovers."""
    p = rig.make_config("config2", n_views=60)
    ba = make(p, {"MCC_SPARE_DELAY_US": "30000", "MCC_WARM_TIMEOUT_MS": "3"})
    try:
        with pytest.raises(api.MccError, match=r"\(-6\)"):
            ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        _recovers_on_the_same_handle(ba, p, {})
    finally:
        ba.close()
    x, m, it, _ = run(p, {})
    x_ref, m_ref, it_ref, _ = O.Oracle(p).optimize(p.x0, crit_type=3, max_count=200, eps=1e-7)
    assert it == it_ref and abs(m - m_ref) <= 1e-6


@pytest.mark.parametrize("cfg,views,env", [
    ("config4", 200, {"MCC_FUSED": "0"}),                    # k_group -> k_schur (m = 18, spare)
    ("config3", 48, {}),                                      # k_prep -> k_edge -> k_photo (m = 90, helper)
])
def test_timing_probe_keeps_the_trajectory(cfg, views, env):
    """mcc_timing_linearize between free-running steps (bench.py's kernel timing): each probe launch
    re-applies the pending photo update and rewrites Y' and z'; the probe restores them with the
    parameters, so 10 steps + probe + 10 steps is bitwise 20 steps."""
    p = rig.make_config(cfg, n_views=views)
    out = []
    for probe in (False, True):
        ba = make(p, env)
        try:
            assert ba.path() == "split"
            ba.set_params(p.x0)
            ba.step(10)
            if probe:
                assert ba.timing_linearize(16) > 0
            ba.step(10)
            ba.check()
            out.append(ba.get_params())
        finally:
            ba.close()
    assert np.array_equal(out[0], out[1])


@pytest.mark.parametrize("views", [200, 1000])
def test_folded_group_step_is_bitwise_the_two_kernel_step(views):
    """k_group's step with k_schur's reduction and the solve folded into the same launch (the default
    while the items fit: LinArgs::fold) against k_group -> k_schur (MCC_GFOLD=0):
    the same sums in the same order, so the optimize and the free-running steps are bitwise equal.  The
    folded consumers poll the hand-off words themselves (kFoldEmpty until written): with the spare
    workgroup held back 300 us (its status word is what the final workgroup waits for before it writes
    the packed system and the state) the bits do not move.  1 000 views is config4 itself (250 groups on
    256 CUs: the items start only when groups exit).  MCC_FOLD_DYN=1 (the groups take the reduction's
    tasks by ticket as they finish, no trailing workgroups) gives the same bits.  So does the grid laid out
    with the consumers (spare, items, norm chunks, final) at the LOWEST indices
    (MCC_FOLD_CONSUMERS_FIRST=1): progress does not rest on the dispatcher starting the groups first,
    only on the consumers leaving CUs for the producers (mcc_create).  src/multicalib.cpp:462-514."""
    p = rig.make_config("config4", n_views=views)
    runs = []
    for env in ({"MCC_GFOLD": "0"}, {}, {"MCC_SPARE_DELAY_US": "300"}, {"MCC_FOLD_DYN": "1"},
                {"MCC_FOLD_DYN": "1", "MCC_SPARE_DELAY_US": "300"}, {"MCC_FOLD_CONSUMERS_FIRST": "1"},
                {"MCC_FOLD_CONSUMERS_FIRST": "1", "MCC_SPARE_DELAY_US": "300"}):
        ba = make(p, dict(env, MCC_FUSED="0", MCC_SOLVE_STATS="1"))
        try:
            assert ba.step_kernels() == "k_group"
            try:
                x, m, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
            except api.MccError as e:
                raise AssertionError(f"{env}: {e}")
            ba.set_params(p.x0)
            ba.step(24)
            ba.check()
            xs = ba.get_params()
            st = ba.solve_stats()
        finally:
            ba.close()
        runs.append((x, it, xs, st))
    (x0, it0, xs0, st0) = runs[0]
    for (x, it, xs, st) in runs[1:]:
        assert it == it0
        assert np.array_equal(x, x0) and np.array_equal(xs, xs0)
        for k in ("warm", "corrections", "fallbacks", "direct"):
            assert st[k] == st0[k], (st0, st)
    assert st0["warm"] > 0


def test_folded_timeout_then_same_handle_is_a_fresh_run():
    """The folded k_group step (config4 rig, 200 views) with its spare held back 30 ms against a 3 ms
    poll bound: the final workgroup gives up, the step fails with MCC_ETIMEOUT (-6), and the late spare
    still writes its inverse and status, the final's item partials stay unread.  The next optimisation
    on the SAME handle (delays off) starts with every hand-off word empty again (set_state after an
    error) and is bitwise a fresh problem's run; the consumers-first layout recovers the same way."""
    p = rig.make_config("config4", n_views=200)
    for extra in ({}, {"MCC_FOLD_CONSUMERS_FIRST": "1"}):
        env = dict(extra, MCC_FUSED="0")
        ba = make(p, dict(env, MCC_SPARE_DELAY_US="30000", MCC_WARM_TIMEOUT_MS="3"))
        try:
            assert ba.folded()
            with pytest.raises(api.MccError, match=r"\(-6\)"):
                ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
            _recovers_on_the_same_handle(ba, p, env)
        finally:
            ba.close()
