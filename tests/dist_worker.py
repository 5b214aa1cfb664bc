"""Worker for tests/test_distributed.py: one rank of the photo-sharded Gauss-Newton loop on CPU.

It runs the same dataflow as the multi-GPU path (bench.py / mcc_comm_* / mcc_peer_*, SURVEY.md
8(e)) with the oracle standing in for the kernels and gloo for RCCL:
  owner = mcc_partition_photos(...)               (the product's host partitioner)
  local = rig.subset_photos(problem, my photos)   (x_local = [global block, my photos])
  per step k: (S, r) = sum over my photos of the Schur terms, with the stop-test norms of update
            k - 1 appended -> ONE all-reduce (sum) of [S | r | ||G||^2 | ||x||^2]
            stop test on change = ||G|| / ||x|| (src/multicalib.cpp:475-477, 504)
            dg = S^-1 r by Cholesky (identical on every rank), dp = local back-substitution
            G = fl32(0.95^(k+1) delta), x = fl32(x + G)      (src/multicalib.cpp:482-501)
The norms ride in the step's one collective, one step late, as on the device (k_schur / the
fused kernel's last arriver).  Imported only in spawned children: the pytest process never
imports torch.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

CASES = {
    "config2_30": ("config2", 30),
    "config3_40": ("config3", 40),
}


def make_problem(case):
    from multi_camera_calibration_amd import rig
    name, views = CASES[case]
    return rig.make_config(name, n_views=views)


def cholesky_solve(S, r):
    from scipy.linalg import cho_factor, cho_solve
    return cho_solve(cho_factor(S, lower=True), r)


def run(case, rank, world, port, crit_type, max_count, eps, out_q):
    import torch
    import torch.distributed as dist
    from multi_camera_calibration_amd import api
    from oracle import oracle_py as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = make_problem(case)
        owner = api.partition_photos(p, world)
        mine = np.nonzero(owner == rank)[0]
        q = rig_subset(p, mine)
        o = O.Oracle(q)
        m = q.global_dim
        x = q.x0.copy()
        g2 = x2 = 0.0
        change = 1.0
        k = 0
        while True:
            S, r = o.schur_partial(x, 0, q.n_photos)
            buf = torch.from_numpy(np.concatenate([S.ravel(), r, [g2, x2]]))
            dist.all_reduce(buf)                       # the single data-path collective per step
            buf = buf.numpy()
            if k > 0:
                change = float(np.sqrt(buf[-2]) / np.sqrt(buf[-1]))
            stop = ((crit_type == 1 and k >= max_count) or (crit_type == 2 and change <= eps) or
                    (crit_type == 3 and (change <= eps or k >= max_count)))
            if stop:
                break
            S = buf[:m * m].reshape(m, m)
            dg = cholesky_solve(S, buf[m * m:m * m + m])
            dp = o.photo_backsub(x, 0, q.n_photos, dg)
            delta = np.concatenate([dg, dp])
            G = (0.95 ** (k + 1) * delta).astype(np.float32)
            x = (x + G).astype(np.float32)
            # stop-test partials: global block counted once (rank 0), photos by their owner
            Gd, xd = G.astype(np.float64), x.astype(np.float64)
            g2 = float((Gd[m:] ** 2).sum()) + (float((Gd[:m] ** 2).sum()) if rank == 0 else 0.0)
            x2 = float((xd[m:] ** 2).sum()) + (float((xd[:m] ** 2).sum()) if rank == 0 else 0.0)
            k += 1
        out_q.put((rank, mine, x, k, change))
    finally:
        dist.destroy_process_group()


def rig_subset(p, mine):
    from multi_camera_calibration_amd import rig
    return rig.subset_photos(p, mine)
