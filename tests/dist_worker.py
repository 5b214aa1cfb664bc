"""Worker for tests/test_distributed.py: one rank of the photo-sharded Gauss-Newton step on CPU.

It runs the same dataflow as the multi-GPU path (bench.py / mcc_comm_*) with the
oracle standing in for the kernels and gloo for RCCL:
  owner = mcc_partition_photos(...)               (the product's host partitioner)
  local = rig.subset_photos(problem, my photos)   (x_local = [global block, my photos])
  per step: (S, r) = sum over my photos of the Schur terms   -> ONE all-reduce (sum)
            dg = S^-1 r (identical on every rank), dp = local back-substitution
            G = fl32(0.95^(k+1) delta), x = fl32(x + G)      (src/multicalib.cpp:482-501)
Imported only in spawned children: the pytest process never imports torch.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def run(rank, world, port, steps, out_q):
    import torch
    import torch.distributed as dist
    from multi_camera_calibration_amd import api, rig
    from oracle import oracle_py as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        p = rig.make_config("config2", n_views=30)
        owner = api.partition_photos(p, world)
        mine = np.nonzero(owner == rank)[0]
        q = rig.subset_photos(p, mine)
        o = O.Oracle(q)
        m = q.global_dim
        x = q.x0.copy()
        for k in range(steps):
            S, r = o.schur_partial(x, 0, q.n_photos)
            buf = torch.from_numpy(np.concatenate([S.ravel(), r]))
            dist.all_reduce(buf)                       # the single data-path collective per step
            S = buf[:m * m].numpy().reshape(m, m)
            r = buf[m * m:].numpy()
            dg = np.linalg.solve(S, r)
            dp = o.photo_backsub(x, 0, q.n_photos, dg)
            delta = np.concatenate([dg, dp])
            G = (0.95 ** (k + 1) * delta).astype(np.float32)
            x = (x + G).astype(np.float32)
            # stop-test norms: global block counted once (rank 0), photos by their owner
            g2 = float((G[m:].astype(np.float64) ** 2).sum()) + (float((G[:m].astype(np.float64) ** 2).sum()) if rank == 0 else 0.0)
            x2 = float((x[m:].astype(np.float64) ** 2).sum()) + (float((x[:m].astype(np.float64) ** 2).sum()) if rank == 0 else 0.0)
            nb = torch.tensor([g2, x2], dtype=torch.float64)
            dist.all_reduce(nb)
        out_q.put((rank, mine, x, float(np.sqrt(nb[0]) / np.sqrt(nb[1]))))
    finally:
        dist.destroy_process_group()
