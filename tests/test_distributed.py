"""world_size-2 and -4 gloo runs of the photo-sharded Gauss-Newton loop (CPU).

The ranks each own a share of the photo vertices (mcc_partition_photos), all-reduce the packed
reduced camera system plus the stop-test norms once per step, solve it identically and
back-substitute their own photos (tests/dist_worker.py).  The gathered result is held to the
single-GPU bars against the single-process oracle's optimizeExtrinsics (src/multicalib.cpp:462-514,
COUNT+EPS criterion): the same iteration count, the final meanReProjError within 1e-6 px, every
float32 parameter within 1 ulp, and the stop-test ratio of the last update.
"""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

from oracle import oracle_py as O

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ulp import f32_ulp_diff  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("case,world", [("config2_30", 2), ("config3_40", 4)])
def test_sharded_loop_matches_oracle(case, world):
    import dist_worker
    crit_type, max_count, eps = 3, 200, 1e-7
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=dist_worker.run, args=(case, r, world, port, crit_type, max_count, eps, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0

    p = dist_worker.make_problem(case)
    m = p.global_dim
    o = O.Oracle(p)
    x_ref, m_ref, it_ref, change_ref = o.optimize(p.x0, crit_type, max_count, eps)
    for r in res:
        assert r[3] == it_ref, (case, r[3], it_ref)
        assert r[4] == res[0][4]
    # the replicated global block: identical on every rank
    for r in res[1:]:
        assert np.array_equal(r[2][:m], res[0][2][:m])
    x = np.zeros_like(x_ref)
    x[:m] = res[0][2][:m]
    seen = np.zeros(p.n_photos, bool)
    for rank, mine, xl, _, _ in res:
        for j, ph in enumerate(mine):
            c = int(p.photo_col(ph))
            x[c:c + 6] = xl[m + 6 * j:m + 6 * j + 6]
            seen[ph] = True
    assert seen.all()
    ulp = f32_ulp_diff(x, x_ref)
    assert ulp.max() <= 1, (case, int(ulp.max()), int((ulp > 0).sum()))
    _, mean = o.project_error(x)
    assert abs(mean - m_ref) <= 1e-6, (case, mean, m_ref)
    assert abs(res[0][4] - change_ref) <= 1e-9 * change_ref
