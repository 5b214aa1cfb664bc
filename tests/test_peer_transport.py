"""The peer transport (mcc_peer_*): the multi-GPU step's exchange without RCCL, run here as two
ranks (processes) on one device.

Each rank holds a photo shard (mcc_partition_photos); the final arriving workgroup of each rank
writes its packed reduced camera system into the other's inbox (LL words) and sums both in rank
order, so both ranks solve identical bits.  Checked against a single-process run of the whole
problem (tolerances of tests/test_gpu_parity.py; the sums differ only in association order):
  * the global block is bit-identical on both ranks;
  * computeJacobianExtrinsic: deltaX (global and each rank's photos) and the photos' JTE;
  * optimizeExtrinsics: iteration count and parameters;
  * mcc_comm_allreduce_max over the transport.
The fused path (config2, config5 DoubleSide) exchanges in k_linearize, the m > 30 path (config3)
in k_solve.  CPU: host-side argument checks.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from multi_camera_calibration_amd import api, rig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import peer_worker  # noqa: E402


def test_peer_abi_declared():
    decl = api.declared_symbols()
    for s in ("mcc_peer_handle", "mcc_peer_init", "mcc_peer_enable"):
        assert s in decl


def test_file_allgather(tmp_path):
    out = api.file_allgather(str(tmp_path), 0, 1, b"abc")
    assert out == [b"abc"]


def _run_ranks(case, world, tmp_path, steps=100):
    env = dict(os.environ, MCC_PEER_TIMEOUT_MS="20000")
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "peer_worker.py"), case, str(r),
                                       str(world), str(tmp_path / "rdv"), str(tmp_path / f"r{r}.npz"), str(steps)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    logs = []
    for pr in procs:
        try:
            logs.append(pr.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for pp in procs:
                pp.kill()
            raise
    for pr, lg in zip(procs, logs):
        assert pr.returncode == 0, lg
    return [dict(np.load(tmp_path / f"r{r}.npz")) for r in range(world)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["config2_small", "config5_small", "config3_small", "config2_nocam", "config3_full",
                                  "config5_full"])
def test_peer_two_ranks_one_device(case, tmp_path):
    """*_full: BASELINE.json's multi-GPU rigs (config3: 16 cameras x 5k views, m = 90; config5:
    8-camera double-sided board x 2k views) at their fixed size split over two ranks -- the
    strong-scaling split bench.py measures at N > 1."""
    world = 2
    outs = _run_ranks(case, world, tmp_path, steps=20 if case.endswith("_full") else 100)
    p = peer_worker.CASES[case]()
    m = p.global_dim
    ba = api.BundleAdjuster(p)
    try:
        d_ref, j_ref = ba.compute_jacobian_extrinsic(p.x0)
        x_ref, _, it_ref, _ = ba.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
    finally:
        ba.close()
    for o in outs:
        assert float(o["mx"]) == world - 0.5
        assert int(o["it"]) == it_ref, (case, int(o["it"]), it_ref)
    # identical bits of the replicated global block on every rank
    for o in outs[1:]:
        assert np.array_equal(o["x"][:m], outs[0]["x"][:m])
        assert np.array_equal(o["d"][:m], outs[0]["d"][:m])
    # assemble the sharded results in global column order
    x = np.zeros_like(x_ref)
    d = np.zeros_like(d_ref)
    jp = np.zeros_like(j_ref)
    x[:m], d[:m] = outs[0]["x"][:m], outs[0]["d"][:m]
    for o in outs:
        for k, ph in enumerate(o["mine"]):
            c = p.photo_col(int(ph))
            x[c:c + 6] = o["x"][m + 6 * k:m + 6 * k + 6]
            d[c:c + 6] = o["d"][m + 6 * k:m + 6 * k + 6]
            jp[c:c + 6] = o["j"][m + 6 * k:m + 6 * k + 6]
    assert np.abs(d - d_ref).max() <= 1e-6 * np.abs(d_ref).max(), case
    assert np.abs(jp[m:] - j_ref[m:]).max() <= 1e-9 * np.abs(j_ref[m:]).max(), case
    assert np.abs(x - x_ref).max() <= 1e-4 * np.abs(x_ref).max(), case
    print(f"{case}: 2 ranks on one device, {float(outs[0]['ms']):.4f} ms/step")
