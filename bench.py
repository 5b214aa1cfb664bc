#!/usr/bin/env python3
"""Benchmark of the MI355X BA hot path (one Gauss-Newton step of optimizeExtrinsics).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config config4]

One "step" = one pass of the hot path over the whole problem: linearisation of every corner
(residual + Jacobian), normal-equation reduction, Schur solve, float32 update
(MultiCameraCalibration::optimizeExtrinsics loop body, src/multicalib.cpp:481-506).

Headline workload (N = 1): BASELINE.json configs[3] -- 4 omnidirectional cameras, 1 000 synthetic
11x8-board views -- the largest BASELINE config quoted on one MI355X; configs[1] (4 pinhole
cameras, 500 views) is reported at the same level under "configs" (with configs 3 and 5).
N > 1 ranks (one process per GPU, launched by torch.distributed.run) weak-scale the headline
workload: the rig has 1 000*N views, photo vertices are sharded and each step exchanges the reduced
camera system once: over the peer transport (mcc_peer_*: the final arriving workgroup of each rank
writes its system into every peer's inbox over xGMI and solves) when the handshake passes on
every rank, else with one RCCL all-reduce (MCC_TRANSPORT=rccl forces it).

Timing: an untimed clock ramp (>= --ramp-seconds of steps, the same step count on every rank),
W warmup steps, then exactly K steps between barriers (max over ranks); the dominant kernel(s)
are then timed with HIP events over a window of 100 further steps, and the per-step distribution
(median, p10, p90) over 30 event-timed windows of 20 graph-launched steps.

Extra keys (same JSON line):
  * N = 1: "configs" -- the other BASELINE configs (2, 3, 5) at full size on this GPU (ms per
    step, corner evals/s, linearisation time and HBM-roofline fraction, traffic and FP64 from the
    committed rocprofv3 summaries);
  * N > 1: "strong" -- the BASELINE multi-GPU rigs at their fixed size split over the N ranks
    (config3: 16 cameras x 5k views; config5: 8-camera double-sided board x 2k views), the
    strong-scaling curve north_star names, with BOTH transports (peer and RCCL) and each one's
    per-step exchange time;
  * "cpu_baseline" (the OpenMP Schur port on the same workload) and "cpu_baseline_ref_faithful"
    (the reference's own algorithm -- dense J, J^T J, Jacobi-CG x2 -- single-threaded on config1).

MCC_BENCH_SAME_DEVICE=1 puts every rank on device 0 with the peer transport only (RCCL refuses
two ranks on one device): a rehearsal of the N > 1 code path on a one-GPU box, not a scaling
measurement.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from multi_camera_calibration_amd import api, rig  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP64_PEAK_TFS = 78.6    # MI355X FP64 vector peak, AMD spec
METRIC = "corner residual+Jacobian evals/sec + ms/LM-iter; RMS reproj-err vs ref"
DIST_WINDOWS, DIST_STEPS = 30, 20   # the per-step distribution: 30 windows of 20 steps
KERNEL_WINDOW = 100                 # steps of the dominant kernel's event window (queued behind a 5 ms delay)


def _launch_key() -> str:
    return f"{os.getppid()}_{os.environ.get('MASTER_PORT', '0')}"


def rendezvous_id(rank: int, tag: str) -> bytes:
    """Share an RCCL unique id among the ranks of one node (torchrun's agent is every rank's
    parent, so its pid names the launch; tag names the problem)."""
    path = f"/tmp/mcc_ncclid_{_launch_key()}_{tag}"
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


def setup_transport(ba, rank: int, world: int, same_device: bool, tag: str) -> str:
    """RCCL communicator (distinct devices) plus, unless MCC_TRANSPORT=rccl, the peer transport;
    all ranks agree on the transport over RCCL before it is used."""
    key = f"/tmp/mcc_peer_{_launch_key()}_{tag}"
    if not same_device:
        ba.comm_init(rendezvous_id(rank, tag), world, rank)
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


def measure(ba, steps: int, warmup: int, ramp_s: float, window: int):
    """Clock ramp (same step count on every rank: each step may exchange with the peers),
    W warmup steps, K timed steps between barriers (max over ranks), then the HIP-event window
    of the dominant kernel over `window` launches."""
    ba.step(8)
    ba.synchronize()
    t0 = time.perf_counter()
    ba.step(16)
    ba.synchronize()
    per = ba.allreduce_max((time.perf_counter() - t0) / 16)
    n_ramp = int(min(200000, max(64, math.ceil(ramp_s / max(per, 1e-7)))))
    t0 = time.perf_counter()
    ba.step(n_ramp)
    ba.synchronize()
    ramp_wall = time.perf_counter() - t0
    ba.step(warmup)
    ba.synchronize()
    ba.barrier()
    t0 = time.perf_counter()
    ba.step(steps)
    ba.synchronize()
    ba.barrier()
    t1 = time.perf_counter()
    dt = ba.allreduce_max(t1 - t0)
    ba.timing_begin()
    ba.step(window)
    lin_ms, step_ms_ev, nlaunch = ba.timing_end()
    xchg_ms, n_xchg = ba.timing_exchange()
    ba.check()   # a failed step (peer timeout, not PD) stops the later ones: never report that as speed
    lin_ms = ba.allreduce_max(lin_ms)
    step_ms_ev = ba.allreduce_max(step_ms_ev)
    xchg_ms = ba.allreduce_max(xchg_ms)
    # per-step distribution (SURVEY.md 8(d) / BASELINE.md section 3: median, p10, p90): DIST_WINDOWS
    # back-to-back windows of DIST_STEPS graph-launched steps, each timed by HIP events on the step stream
    wins, graph = ba.timing_windows(DIST_WINDOWS, DIST_STEPS)
    ba.check()
    per = wins / DIST_STEPS
    dist = {q: ba.allreduce_max(float(np.percentile(per, v))) for q, v in (("p10", 10), ("median", 50), ("p90", 90))}
    step_ms_ev = ba.allreduce_max(float(np.mean(per)))   # graph-launched steps, like the headline
    if lin_kernels(ba) == "k_linearize" or ba.folded():
        # one kernel per step (the fused kernel, or k_group with the reduction and solve folded in):
        # the kernel's time is the graph-launched step's, as rocprofv3 averages it
        lin_ms = step_ms_ev
    else:
        # the split step's linearisation kernels alone, `window` launches in one captured graph
        # between two HIP events (the eager window above puts an event pair between every kernel)
        lin_ms = ba.allreduce_max(ba.timing_linearize(window))
        ba.check()
    dist.update(unit="ms per step", windows=DIST_WINDOWS, steps_per_window=DIST_STEPS,
                launch="graph" if graph else "eager", timer="HIP events between back-to-back windows (max over ranks)")
    return dict(dt=dt, lin_ms=lin_ms, step_ms_ev=step_ms_ev, nlaunch=nlaunch, xchg_ms=xchg_ms, n_xchg=n_xchg,
                ramp={"steps": n_ramp + 24, "seconds": round(ramp_wall, 3)}, dist=dist)


def lin_kernels(ba) -> str:
    """The kernels of the linearisation window (mcc_timing_*): the fused kernel, the split step's
    group kernel (with the reduction and the m <= 30 solve folded into its launch: the whole step), or
    its three-kernel form (mcc_problem_path says which)."""
    return ba.step_kernels() + (" (folded: the whole step)" if ba.folded() else "")


def roofline(st, lin_ms, tr=None, kernel="k_linearize"):
    achieved = st["alg_bytes"] / (lin_ms * 1e-3) / 1e9
    return {
        "kernel_timing": ("HIP events on the step stream around graph launches: one kernel per step (the fused "
                          "kernel, or k_group with the reduction and solve folded in), a window of graph-launched "
                          "steps; the split step, a captured graph of its linearisation kernels alone, launched "
                          "back to back (mcc_timing_linearize)"),
        "bound": "hbm",
        "kernel": kernel,
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": (tr["bytes_per_launch"] if tr else None),
        "alg_bytes_per_launch": st["alg_bytes"],
        "alg_bytes_formula": "20 B/corner (float32 obj xyz + img uv) + 280 B/edge (SURVEY.md 8(d))",
        "kernel_ms_per_launch": lin_ms,
    }


MODEL_NAMES = {rig.PINHOLE: "pinhole", rig.OMNI: "omnidirectional", rig.DOUBLESIDE: "double-sided-board pinhole"}
CONFIG_INDEX = {"config1": 0, "config2": 1, "config3": 2, "config4": 3, "config5": 4}


def workload_label(name: str, views_per_rank: int, world: int) -> str:
    c = rig.CONFIGS[name]
    board = "x".join(map(str, c["board"]))
    per = " per rank" if world > 1 else ""
    return (f"{name}: {c['n_cams']} {MODEL_NAMES[c['model']]} cameras, {views_per_rank} synthetic {board}-board "
            f"views{per} (BASELINE.json configs[{CONFIG_INDEX[name]}]), one Gauss-Newton step per 'step'")


def config_line(name: str, steps: int = 1000, warmup: int = 10, device: int = 0):
    """One BASELINE config at full size on this GPU (N = 1 extra key), timed like the headline
    (1 000 steps: at 100 the first graph launch's host latency and the final wait were 2-8 % of a
    config2 / config5 window)."""
    t0 = time.time()
    p = rig.make_config(name)
    gen_s = time.time() - t0
    ba = api.BundleAdjuster(p, device=device)
    try:
        ba.set_params(p.x0)
        m = measure(ba, steps, warmup, 0.15, KERNEL_WINDOW)
        st = ba.stats()
        kern = lin_kernels(ba)
        solve = ba.solve_stats()
    finally:
        ba.close()
    ms = m["dt"] / steps * 1e3
    out = {"cameras": p.n_cams, "views": p.n_photos, "edges": p.n_edges, "corners_per_step": p.n_corners,
           "model": {rig.PINHOLE: "pinhole", rig.OMNI: "omnidir", rig.DOUBLESIDE: "doubleside"}[p.model],
           "steps": steps, "ms_per_step": ms, "corner_evals_per_s": p.n_corners / (ms * 1e-3),
           "step_ms_events": m["step_ms_ev"], "launches_timed": m["nlaunch"],
           "roofline": roofline(st, m["lin_ms"], load_profile("traffic", name, p.n_photos), kernel=kern),
           "step_distribution": m["dist"],
           "rig_generation_s": round(gen_s, 2)}
    if solve["warm"] or solve["direct"]:
        # solves by refinement with the previous system's inverse (m > 30: k_sinv_helper on a side
        # stream; m <= 30: the linearisation launch's spare workgroup) over every step of this process
        # (ramp, warmup, timed, window), and how many fell back
        out["warm_solve"] = solve
    fp = load_profile("fp64", name, p.n_photos)
    if fp and fp.get("fp64_flops_per_launch"):
        tf = fp["fp64_flops_per_launch"] / (m["lin_ms"] * 1e-3) / 1e12
        out["fp64_valu"] = {"achieved": tf, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFS,
                            "flops_per_corner": fp["fp64_flops_per_corner"]}
    return out


def optimize_line(name: str, reps: int = 20, device: int = 0):
    """What a caller of optimizeExtrinsics sees (src/multicalib.cpp:462-514, VERDICT r5 missing 2): the
    whole mcc_optimize from x0 under COUNT + EPS, 200 iterations, eps 1e-7 (the reference's
    TermCriteria, include/opencv2/ccalib/mymulticalib.hpp:95) -- parameters in, the device loop to its
    stop test, the pending photo update flushed, parameters out.  The first call (graph capture) is
    reported apart; then the median of `reps` calls: wall ms per call (Python ctypes call), the C
    side's host phases, device ms from the first step launch to the end of the last launched step
    (HIP events) and per iteration.  The solves a call takes (refinements, their corrections,
    fallbacks, direct eliminations) come from one more call on a problem created with MCC_SOLVE_STATS=1
    (the m <= 30 counters cost ~0.5 us per step, so the timed problem runs without them)."""
    p = rig.make_config(name)
    ba = api.BundleAdjuster(p, device=device)
    try:
        t0 = time.perf_counter()
        x, mean, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        first_wall = (time.perf_counter() - t0) * 1e3
        first = ba.optimize_profile()
        rows = []
        for _ in range(reps):
            t0 = time.perf_counter()
            x, mean, it, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
            wall = (time.perf_counter() - t0) * 1e3
            rows.append(dict(ba.optimize_profile(), wall_ms=wall))
        path = ba.step_kernels() + (" (folded)" if ba.folded() else "")
        # the itemisation: device ms of the same call under COUNT with max_count = k (k updates, the
        # stop-test launch, then no-op launches to the end of the 8-step graph), median of 5 calls each;
        # cost(k) - cost(k - 1) is the k-th update step in place of a no-op launch
        by_count = []
        for k in range(0, it + 1):
            dv = []
            for _ in range(5):
                ba.optimize_extrinsics(p.x0, crit_type=1, max_count=k)
                dv.append(ba.optimize_profile()["device_ms"])
            by_count.append(float(np.median(dv)))
    finally:
        ba.close()
    old = os.environ.get("MCC_SOLVE_STATS")
    os.environ["MCC_SOLVE_STATS"] = "1"
    try:
        bs = api.BundleAdjuster(p, device=device)
    finally:
        if old is None:
            del os.environ["MCC_SOLVE_STATS"]
        else:
            os.environ["MCC_SOLVE_STATS"] = old
    try:
        s0 = bs.solve_stats()
        bs.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        s1 = bs.solve_stats()
    finally:
        bs.close()
    med = lambda k: float(np.median([r[k] for r in rows]))   # noqa: E731
    dev = med("device_ms")
    return {"iterations": it, "meanReProjError": mean, "criteria": "COUNT+EPS, 200, 1e-7", "calls": reps,
            "path": path,
            "wall_ms_per_call": med("wall_ms"), "device_ms_per_call": dev, "device_ms_per_iteration": dev / max(it, 1),
            "host_ms": {"setup": med("host_setup_ms"), "steps_and_stop_polls": med("host_steps_ms"),
                        "finish": med("host_finish_ms"), "c_call": med("host_call_ms")},
            "steps_launched": rows[-1]["steps_launched"], "stop_polls": rows[-1]["stop_polls"],
            "first_call": {"wall_ms": first_wall, "host_ms": first["host_call_ms"], "device_ms": first["device_ms"],
                           "note": "graph capture on first use"},
            "solves_per_call": {k: s1[k] - s0[k] for k in ("warm", "corrections", "fallbacks", "direct", "waited")},
            "device_ms_by_count": {"max_count": list(range(0, it + 1)), "device_ms": by_count,
                                   "marginal_ms": [by_count[k] - by_count[k - 1] for k in range(1, it + 1)],
                                   "note": "COUNT criterion, max_count = k: k updates + the stop-test launch + no-op "
                                           "launches to the end of the 8-step graph; marginal = an update step in "
                                           "place of a no-op launch"}}


def strong_line(name: str, rank: int, world: int, local_rank: int, same_device: bool, steps: int = 100):
    """A BASELINE multi-GPU rig at its fixed size, photo vertices split over the ranks; timed with
    the peer transport and with RCCL (the same problem, mcc_peer_enable toggles), each with its
    per-step exchange time (mcc_timing_exchange: in-kernel ticks / HIP events around the
    all-reduce)."""
    full = rig.make_config(name)
    owner = api.partition_photos(full, world)
    prob = rig.subset_photos(full, np.nonzero(owner == rank)[0])
    ba = api.BundleAdjuster(prob, device=0 if same_device else local_rank)
    out = {"views": full.n_photos, "cameras": full.n_cams, "corners_per_step": full.n_corners,
           "unit": "corner evals/s", "n_gpus": world, "scaling": "strong"}
    try:
        first = setup_transport(ba, rank, world, same_device, f"strong_{name}")
        order = [first] + ([t for t in ("peer", "rccl") if t != first and first == "peer"] if not same_device else [])
        for tr in order:
            if not same_device:
                ba.peer_enable(tr == "peer")
            ba.set_params(prob.x0)
            m = measure(ba, steps, 10, 0.15, KERNEL_WINDOW)
            ms = m["dt"] / steps * 1e3
            out[tr] = {"value": full.n_corners / (ms * 1e-3), "ms_per_step": ms,
                       "kernel_ms_per_launch": m["lin_ms"], "step_ms_events": m["step_ms_ev"],
                       "exchange_ms": m["xchg_ms"], "exchanges_timed": m["n_xchg"]}
        out["warm_solve"] = ba.solve_stats()
    finally:
        ba.close()
    best = min((t for t in ("peer", "rccl") if t in out), key=lambda t: out[t]["ms_per_step"])
    out.update(value=out[best]["value"], ms_per_step=out[best]["ms_per_step"], transport=best)
    return out


def shard_line(name: str, world: int, steps: int = 200, device: int = 0):
    """The compute side of the strong-scaling curve, on this one GPU: rank 0's photo shard of a
    BASELINE multi-GPU rig split `world` ways (mcc_partition_photos), timed as a standalone problem --
    its linearisation, reduction, the replicated camera solve and the update; the exchange is what it
    leaves out.  full / shard is the speedup bound of that split before exchange costs."""
    full = rig.make_config(name)
    owner = api.partition_photos(full, world)
    prob = rig.subset_photos(full, np.nonzero(owner == 0)[0])
    ba = api.BundleAdjuster(prob, device=device)
    try:
        ba.set_params(prob.x0)
        m = measure(ba, steps, 10, 0.15, KERNEL_WINDOW)
        kern = lin_kernels(ba)
        solve = ba.solve_stats()
    finally:
        ba.close()
    ms = m["dt"] / steps * 1e3
    out = {"split": world, "views": prob.n_photos, "edges": prob.n_edges, "corners_per_step": prob.n_corners,
           "ms_per_step": ms, "step_distribution": m["dist"], "kernel": kern, "kernel_ms_per_launch": m["lin_ms"],
           "exchange": "excluded (single process: no peers)"}
    if solve["warm"] or solve["direct"]:
        out["warm_solve"] = solve
    return out


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


def cpu_baseline_ref_faithful():
    """The reference's own algorithm on one host core (SURVEY.md 8(d)(1) 'ref-faithful'): per
    Gauss-Newton step a zero-filled dense J (2 sum N x P), JTJ = J^T J and JTE = J^T E as dense
    products, Eigen-style Jacobi CG solved twice (src/mymulticalib.cpp:680-805,
    src/multicalib.cpp:565-592); the whole optimizeExtrinsics run on config1."""
    from oracle import oracle_py as O
    p = rig.make_config("config1")
    o = O.Oracle(p)
    t0 = time.perf_counter()
    _, mean, it, _ = o.optimize(p.x0, crit_type=3, max_count=200, eps=1e-7, solver="dense_j")
    dt = time.perf_counter() - t0
    rows = 2 * p.n_corners
    c2 = rig.CONFIGS["config2"]
    return dict(value=p.n_corners * it / dt, unit="corner evals/s", cores=1, kind="port",
                ms_per_step=dt / it * 1e3, iterations=it, meanReProjError=mean,
                sample=f"config1 (2 cameras, 20 views, 9x6 board): the whole optimizeExtrinsics, {it} steps of dense "
                       f"J ({rows} x {p.n_params}) + J^T J + Jacobi-CG x2, single thread, {dt:.3f} s wall",
                config2=_ref_faithful_config2())


def _ref_faithful_config2():
    """config2's one-iteration ref-faithful timing: 8.3 GB of dense J and ~1.6e12 multiply-adds of
    J^T J per step take tens of minutes on one core, so it is run offline once
    (tools/ref_faithful_config2.py) and the committed result is cited here."""
    f = os.path.join(ROOT, "profiles", "ref_faithful_config2.json")
    if os.path.exists(f):
        d = json.load(open(f))
        d["source"] = "profiles/ref_faithful_config2.json (tools/ref_faithful_config2.py, offline, not this run)"
        return d
    return "not run: tools/ref_faithful_config2.py has not produced profiles/ref_faithful_config2.json"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", default="config4")
    ap.add_argument("--views", type=int, default=None, help="views per rank (default: the config's)")
    ap.add_argument("--ramp-seconds", type=float, default=0.25, help="untimed clock ramp before the warmup")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the per-config / strong-scaling extra keys")
    ap.add_argument("--optimize-only", action="store_true", help="print only the optimize key (N = 1)")
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
    transport = setup_transport(ba, rank, world, same_device, "weak") if world > 1 else "none"
    ba.set_params(prob.x0)

    if args.optimize_only:
        ba.close()
        print(json.dumps({"optimize": {name: optimize_line(name, device=local_rank)
                                       for name in ("config4", "config3", "config2")}}))
        return
    m = measure(ba, args.steps, args.warmup, args.ramp_seconds, KERNEL_WINDOW)
    st = ba.stats()
    kern = lin_kernels(ba)
    solve = ba.solve_stats()
    corners_total = float(full.n_corners)
    value = corners_total * args.steps / m["dt"]
    ms_per_step = m["dt"] / args.steps * 1e3
    ba.close()

    strong = {}
    if world > 1 and not args.no_extra:
        for name in ("config3", "config5"):
            strong[name] = strong_line(name, rank, world, local_rank, same_device)

    if rank != 0:
        return
    tr = load_profile("traffic", args.config, views_per_rank) if world == 1 else None
    model = MODEL_NAMES[rig.CONFIGS[args.config]["model"]]
    rl = roofline(st, m["lin_ms"], tr, kernel=kern)
    rl["kernel_launches_timed"] = m["nlaunch"]
    rl["step_ms_events"] = m["step_ms_ev"]
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
            "workload": workload_label(args.config, views_per_rank, world),
            "model": model,
            "cameras": full.n_cams, "views": full.n_photos, "edges": full.n_edges,
            "corners_per_step": int(corners_total), "params": full.n_params,
            "parallelism": f"photo-sharded x{world}" + (
                {"peer": " + in-kernel peer exchange of the camera system (LL words over xGMI)",
                 "rccl": " + RCCL all-reduce of the camera system"}[transport] if world > 1 else ""),
            "transport": transport,
            "state_dtype": "f32", "jacobian_dtype": "f64",
        },
        "clock_ramp": m["ramp"],
        "step_distribution": m["dist"],
        "exchange_ms": m["xchg_ms"] if world > 1 else None,
        "roofline": rl,
    }
    fp = load_profile("fp64", args.config, views_per_rank) if world == 1 else None
    if fp and fp.get("fp64_flops_per_launch"):
        tf = fp["fp64_flops_per_launch"] / (m["lin_ms"] * 1e-3) / 1e12
        out["fp64_valu"] = {"achieved": tf, "peak": FP64_PEAK_TFS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFS,
                            "flops_per_launch": fp["fp64_flops_per_launch"],
                            "flops_per_corner": fp["fp64_flops_per_corner"],
                            "source": "profiles/fp64_*.json (rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes, "
                                      "an upper bound) / the event-timed launch"}
        sq = load_profile("sq", args.config, views_per_rank)
        ks = [k for k in (sq or {}).get("kernels", {}) if k in kern and "valu_issue_frac" in sq["kernels"][k]]
        if ks:
            # the counter-based frac counts every lane of every FP64 instruction; the SIMDs' VALU issue
            # share (SQ pass) is the utilisation figure
            out["fp64_valu"]["valu_issue_frac"] = {k: round(sq["kernels"][k]["valu_issue_frac"], 4) for k in ks}
            out["fp64_valu"]["valu_issue_source"] = ("profiles/sq_*.json: SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES "
                                                     "x waves per SIMD (tools/pmc_sq.sh)")
    if solve["warm"] or solve["direct"]:
        out["warm_solve"] = solve
    if strong:
        out["strong"] = strong
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
    if world == 1 and not args.no_extra:
        # the ms per iteration of a real optimizeExtrinsics from x0 (the steady-state steps above run at
        # alpha = 0.95^(k+1) ~ 0 after the clock ramp: DESIGN.md section 5)
        out["optimize"] = {name: optimize_line(name, device=local_rank) for name in ("config4", "config3", "config2")}
        out["configs"] = {name: config_line(name, device=local_rank)
                          for name in ("config2", "config3", "config4", "config5") if name != args.config}
        # BASELINE's multi-GPU rigs: rank 0's shard at the rank counts they are quoted on, timed here
        out["shard"] = {}
        for name, w in (("config3", 8), ("config5", 4)):
            sl = shard_line(name, w, device=local_rank)
            full_ms = out["configs"][name]["ms_per_step"] if name in out["configs"] else None
            if full_ms:
                sl["full_ms_per_step"] = full_ms
                sl["compute_speedup_bound"] = full_ms / sl["ms_per_step"]
            out["shard"][f"{name}_x{w}"] = sl
    if not args.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(prob, args.cpu_seconds)
        out["cpu_baseline_ref_faithful"] = cpu_baseline_ref_faithful()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
