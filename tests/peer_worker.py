"""Worker for tests/test_peer_transport.py: one rank of the photo-sharded Gauss-Newton step over the
peer transport (mcc_peer_*), several ranks on ONE device (RCCL refuses that; the peer transport
does not need it).  No torch: the inbox handles travel through files (api.file_allgather).

    python tests/peer_worker.py <case> <rank> <world> <rendezvous dir> <out.npz> [steps] [eps]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from multi_camera_calibration_amd import api, rig  # noqa: E402

CASES = {
    # fused single-kernel step (m = 18): the final arriver exchanges and solves
    "config2_small": lambda: rig.make_config("config2", n_views=40),
    # DoubleSide (m = 6), fused
    "config5_small": lambda: rig.make_config("config5", n_views=24),
    # m = 90: the split step (k_prep, k_edge, k_photo, k_schur), the exchange runs in k_solve
    "config3_small": lambda: rig.make_config("config3", n_views=48),
    # a shard without any observation of one camera (config2, 40 views, camera 3 on rank 0 only)
    "config2_nocam": lambda: rig.make_config("config2", n_views=40),
    # m = 18 on the split step (MCC_FUSED=0: k_group -> k_schur, as each rank of bench.py's config4
    # weak-scaling run takes at 1 000 views per rank): k_schur's final arriver exchanges and solves
    "config4_split": lambda: rig.make_config("config4", n_views=64),
    # BASELINE.json's multi-GPU rigs at full size (bench.py's strong-scaling lines)
    "config3_full": lambda: rig.make_config("config3"),
    "config5_full": lambda: rig.make_config("config5"),
}


def shard(case, world, rank):
    p = CASES[case]()
    owner = api.partition_photos(p, world)
    if case == "config2_nocam":
        # every photo camera 3 observes goes to rank 0: the other ranks' shards have no edge of
        # camera block 2 (their local reduced system is singular, the summed one is not)
        owner[np.unique(p.edge_photo[p.edge_cam == 3])] = 0
    mine = np.nonzero(owner == rank)[0]
    return p, mine, rig.subset_photos(p, mine)


def fault_run(ba, q, eps):
    """A shard whose photo block is reported not positive definite (MCC_FAULT_PHOTO on one rank):
    every rank's optimize must fail with MCC_ENOTPD on the same step, and the replicated camera
    block must stay bit-identical (the flag travels in the exchanged system)."""
    try:
        ba.optimize_extrinsics(q.x0, crit_type=3, max_count=200, eps=eps)
        err = ""
    except api.MccError as e:
        err = str(e)
    return err


def main():
    case, rank, world, rdv, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5]
    steps = int(sys.argv[6]) if len(sys.argv) > 6 else 100
    p, mine, q = shard(case, world, rank)
    if case.endswith("_split"):
        os.environ["MCC_FUSED"] = "0"
    ba = api.BundleAdjuster(q, device=0)
    handles = api.file_allgather(os.path.join(rdv, "handles"), rank, world, ba.peer_handle())
    ba.peer_init(handles, world, rank)
    mx = ba.allreduce_max(rank + 0.5)
    if os.environ.get("MCC_PEER_WORKER_MODE") == "fault":
        err = fault_run(ba, q, float(sys.argv[7]) if len(sys.argv) > 7 else 1e-7)
        x = ba.get_params()
        ba.close()
        np.savez(out, mine=mine, x=x, err=err, mx=mx)
        return
    d, j = ba.compute_jacobian_extrinsic(q.x0)
    eps = float(sys.argv[7]) if len(sys.argv) > 7 else 1e-7   # the TermCriteria eps the test compares at
    x, _, it, ch = ba.optimize_extrinsics(q.x0, crit_type=3, max_count=200, eps=eps)
    # throughput of unconditional steps (the bench's loop) over the transport
    ba.set_params(q.x0)
    ba.step(10)
    ba.synchronize()
    ba.barrier()
    t0 = time.perf_counter()
    ba.step(steps)
    ba.synchronize()
    ba.barrier()
    dt = ba.allreduce_max(time.perf_counter() - t0)
    ba.close()
    np.savez(out, mine=mine, x=x, it=it, ch=ch, d=d, j=j, mx=mx, ms=dt / steps * 1e3)


if __name__ == "__main__":
    main()
