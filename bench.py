#!/usr/bin/env python3
"""Benchmark of the MI355X BA hot path (one Gauss-Newton step of optimizeExtrinsics).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config config2]

One "step" = one pass of the hot path over the whole problem: linearisation of every corner
(residual + Jacobian), normal-equation reduction, Schur solve, float32 update
(MultiCameraCalibration::optimizeExtrinsics loop body, src/multicalib.cpp:481-506).
Workload: BASELINE.json configs[1] (4 pinhole cameras, 500 synthetic 11x8-board views) per
rank; N > 1 ranks (one process per GPU, launched by torch.distributed.run) weak-scale it: the rig
has 500*N views, photo vertices are sharded and each step exchanges the reduced camera system
once: over the peer transport (mcc_peer_*: the final arriving workgroup of each rank writes its
system into every peer's inbox over xGMI and solves, one kernel per step) when the handshake
passes on every rank, else with one RCCL all-reduce (MCC_TRANSPORT=rccl forces it).  Rank 0 prints
one JSON line.

MCC_BENCH_SAME_DEVICE=1 puts every rank on device 0 with the peer transport only (RCCL refuses
two ranks on one device): a rehearsal of the N > 1 code path on a one-GPU box, not a scaling
measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from multi_camera_calibration_amd import api, rig  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
METRIC = "corner residual+Jacobian evals/sec + ms/LM-iter; RMS reproj-err vs ref"


def rendezvous_id(rank: int, world: int) -> bytes:
    """Share the RCCL unique id among the ranks of one node (torchrun's agent is every rank's
    parent, so its pid names the launch)."""
    port = os.environ.get("MASTER_PORT", "0")
    path = f"/tmp/mcc_ncclid_{os.getppid()}_{port}"
    if rank == 0:
        uid = api.unique_id()
        tmp = path + ".tmp"
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.time()
    while True:
        if os.path.exists(path):
            with open(path, "rb") as f:
                uid = f.read()
            if len(uid) == 128:
                return uid
        if time.time() - t0 > 300:
            raise RuntimeError("timed out waiting for the RCCL unique id")
        time.sleep(0.05)


def setup_transport(ba, rank: int, world: int, same_device: bool) -> str:
    """RCCL communicator (distinct devices) plus, unless MCC_TRANSPORT=rccl, the peer transport;
    all ranks agree on the transport over RCCL before it is used."""
    key = f"/tmp/mcc_peer_{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}"
    if not same_device:
        ba.comm_init(rendezvous_id(rank, world), world, rank)
    if os.environ.get("MCC_TRANSPORT", "peer") == "rccl":
        if same_device:
            raise SystemExit("MCC_BENCH_SAME_DEVICE needs the peer transport")
        return "rccl"
    ok = True
    try:
        handles = api.file_allgather(key, rank, world, ba.peer_handle())
        ba.peer_init(handles, world, rank)
    except api.MccError as e:
        if same_device:
            raise
        print(f"rank {rank}: peer transport unavailable, using RCCL: {e}", file=sys.stderr)
        ok = False
    if same_device:
        return "peer"
    if ok:
        ba.peer_enable(False)            # agree over RCCL
    bad = ba.allreduce_max(0.0 if ok else 1.0)
    if ok and bad == 0.0:
        ba.peer_enable(True)
        return "peer"
    return "rccl"


FP64_PEAK_TFS = 78.6   # MI355X FP64 vector peak, AMD spec


def load_profile(prefix: str, config: str, n_views: int):
    """The committed rocprofv3 --pmc result for this workload (profiles/<prefix>_*.json)."""
    best = None
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    for fn in sorted(os.listdir(pdir)):
        if fn.startswith(prefix + "_") and fn.endswith(".json"):
            try:
                d = json.load(open(os.path.join(pdir, fn)))
            except Exception:
                continue
            if d.get("config") == config and d.get("n_views") == n_views:
                best = d
    return best


def load_traffic(config: str, n_views: int):
    """Per-launch HBM bytes of k_linearize from the committed rocprofv3 --pmc pass, if one
    exists for this workload (profiles/traffic_*.json, written by tools/pmc_traffic.py)."""
    best = None
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    for fn in sorted(os.listdir(pdir)):
        if fn.startswith("traffic_") and fn.endswith(".json"):
            try:
                d = json.load(open(os.path.join(pdir, fn)))
            except Exception:
                continue
            if d.get("config") == config and d.get("n_views") == n_views:
                best = d
    return best


def cpu_baseline(prob, target_s: float):
    """The oracle (the C restatement of the reference algorithm, block-sparse Schur variant,
    OpenMP over the host cores) timed on a bounded sample of the same workload."""
    from oracle import oracle_py as O
    o = O.Oracle(prob)
    o.optimize(prob.x0, crit_type=1, max_count=1)          # warm
    n = 1
    t0 = time.perf_counter()
    o.optimize(prob.x0, crit_type=1, max_count=n)
    dt = time.perf_counter() - t0
    n = max(1, int(target_s / max(dt, 1e-6)))
    t0 = time.perf_counter()
    o.optimize(prob.x0, crit_type=1, max_count=n)
    dt = time.perf_counter() - t0
    return dict(value=prob.n_corners * n / dt, unit="corner evals/s", cores=O.num_threads(), kind="port",
                sample=f"{prob.name}: {n} Gauss-Newton steps of the oracle (block-sparse Schur restatement "
                       f"of src/mymulticalib.cpp:668-818 + src/multicalib.cpp:462-514), "
                       f"{O.num_threads()} OpenMP threads, {dt:.2f} s wall",
                ms_per_step=dt / n * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="config2")
    ap.add_argument("--views", type=int, default=None, help="views per rank (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = args.gpus if "WORLD_SIZE" not in os.environ else world

    same_device = os.environ.get("MCC_BENCH_SAME_DEVICE", "0") == "1"
    api.lib()   # load libmcc.so (and its HIP runtime) before anything else
    views_per_rank = args.views or rig.CONFIGS[args.config]["n_views"]
    full = rig.make_config(args.config, n_views=views_per_rank * world)
    if world > 1:
        owner = api.partition_photos(full, world)
        prob = rig.subset_photos(full, np.nonzero(owner == rank)[0])
    else:
        prob = full
    ba = api.BundleAdjuster(prob, device=0 if same_device else local_rank)
    transport = setup_transport(ba, rank, world, same_device) if world > 1 else "none"
    ba.set_params(prob.x0)

    # ---- warmup, then exactly K timed steps between barriers
    ba.step(args.warmup)
    ba.synchronize()
    ba.barrier()
    t0 = time.perf_counter()
    ba.step(args.steps)
    ba.synchronize()
    ba.barrier()
    t1 = time.perf_counter()
    dt = ba.allreduce_max(t1 - t0)

    # ---- dominant kernel (k_linearize) duration with HIP events on the problem's stream
    ba.timing_begin()
    ba.step(min(256, max(8, args.steps // 4)))
    lin_ms, step_ms_ev, nlaunch = ba.timing_end()
    lin_ms = ba.allreduce_max(lin_ms)
    st = ba.stats()
    corners_local = st["corners"]
    corners_total = float(full.n_corners)
    value = corners_total * args.steps / dt
    ms_per_step = dt / args.steps * 1e3

    if rank != 0:
        return
    alg_bytes = st["alg_bytes"]   # this rank's launch (all ranks have equal shards by construction)
    achieved = alg_bytes / (lin_ms * 1e-3) / 1e9
    tr = load_traffic(args.config, views_per_rank) if world == 1 else None
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "corner evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {
            "workload": f"{args.config}: {full.n_cams} pinhole cameras, {views_per_rank} synthetic "
                        f"{'x'.join(map(str, rig.CONFIGS[args.config]['board']))}-board views per rank "
                        f"(BASELINE.json configs[1]), one Gauss-Newton step per 'step'",
            "cameras": full.n_cams, "views": full.n_photos, "edges": full.n_edges,
            "corners_per_step": int(corners_total), "params": full.n_params,
            "parallelism": f"photo-sharded x{world}" + (
                {"peer": " + in-kernel peer exchange of the camera system (LL words over xGMI)",
                 "rccl": " + RCCL all-reduce of the camera system"}[transport] if world > 1 else ""),
            "transport": transport,
            "state_dtype": "f32", "jacobian_dtype": "f64",
        },
        "roofline": {
            "bound": "hbm",
            "kernel": "k_linearize",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": (tr["bytes_per_launch"] if tr else None),
            "alg_bytes_per_launch": alg_bytes,
            "alg_bytes_formula": "20 B/corner (float32 obj xyz + img uv) + 280 B/edge (SURVEY.md 8(d))",
            "kernel_ms_per_launch": lin_ms,
            "kernel_launches_timed": nlaunch,
            "step_ms_events": step_ms_ev,
        },
    }
    fp = load_profile("fp64", args.config, views_per_rank) if world == 1 else None
    if fp and fp.get("fp64_flops_per_launch"):
        tf = fp["fp64_flops_per_launch"] / (lin_ms * 1e-3) / 1e12
        out["fp64_valu"] = {"achieved": tf, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFS,
                            "flops_per_launch": fp["fp64_flops_per_launch"],
                            "flops_per_corner": fp["fp64_flops_per_corner"],
                            "source": "profiles/fp64_*.json (rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes, "
                                      "an upper bound) / the event-timed launch"}
    if not args.no_parity and world == 1:
        from oracle import oracle_py as O
        o = O.Oracle(prob)
        xr, mr, itr, _ = o.optimize(prob.x0, crit_type=3, max_count=200, eps=1e-7)
        ba2 = api.BundleAdjuster(prob, device=local_rank)
        xg, mg, itg, _ = ba2.optimize_extrinsics(prob.x0, crit_type=3, max_count=200, eps=1e-7)
        ba2.close()
        out["parity"] = {"meanReProjError_gpu": mg, "meanReProjError_oracle": mr, "abs_diff_px": abs(mg - mr),
                         "iters_gpu": itg, "iters_oracle": itr,
                         "max_abs_param_diff": float(np.abs(xg - xr).max())}
    if not args.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(prob, args.cpu_seconds)
    ba.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
