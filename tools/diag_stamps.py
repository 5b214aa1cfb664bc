#!/usr/bin/env python3
"""Per-phase cycle shares of k_linearize from the diagnostic build (libmcc_diag.so, s_memtime
stamps at phase boundaries; cdna guide section 7 'In-kernel stamps').  Never quote this build's
run time: read its shares.

    MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so python tools/diag_stamps.py [config] [views]

Slots per workgroup (k_linearize): 0..7 s_memtime at phase boundaries, 8 contribution written, 17 final sum placed,
9 group ticket won, 10 group sum written, 11 final ticket won, 12 system assembled, 13 solved
(fused step); 14 / 15 s_memrealtime (100 MHz, chip-wide) at start / exit; 16, 18, 19 phase-0 detail
(loads, back-solve, photo Rodrigues).  s_memtime is per XCD,
so only differences within one workgroup are meaningful; the cross-workgroup timeline uses 14/15.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_camera_calibration_amd import api, rig  # noqa: E402

PHASES = ["pending-update", "prologue", "sweep(wave0)", "reduce+barrier", "chain+H", "photo-chol", "Y/out"]


def med(v):
    return f"median {np.median(v):8.0f}  p90 {np.percentile(v, 90):8.0f}" if len(v) else "n/a"


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "config2"
    views = int(sys.argv[2]) if len(sys.argv) > 2 else None
    p = rig.make_config(cfg, n_views=views)
    ba = api.BundleAdjuster(p)
    ba.set_params(p.x0)
    ba.step(20)
    ba.synchronize()
    ba.stamps()          # arm
    ba.step(1)
    ba.synchronize()
    raw = ba.stamps().reshape(-1)
    nv = max(p.n_photos, 1)
    s = raw[:32 * nv].reshape(nv, 32).astype(np.float64)
    sch = raw[32 * nv:-16].reshape(-1, 16)[:, :8].astype(np.float64)
    s = s[s[:, 0] > 0]
    d = np.diff(s[:, :8], axis=1)
    print(f"{cfg}: {len(s)} workgroups stamped (s_memtime ticks)")
    for k, name in enumerate(PHASES):
        print(f"  {name:16s} {med(d[:, k])}")
    print(f"  {'linearize total':16s} {med(s[:, 7] - s[:, 0])}")
    print(f"  phase 0: loads+partials {med(s[:, 16] - s[:, 0])}; back-solve/update {med(s[:, 18] - s[:, 16])}; "
          f"photo Rodrigues {med(s[:, 19] - s[:, 18])}; barrier {med(s[:, 1] - s[:, 19])}")
    fused = (s[:, 8] > 0).any()
    if fused:
        print(f"  {'contribution':16s} {med(s[:, 8] - s[:, 7])}")
        g = s[s[:, 9] > 0]
        print(f"  group reducers: {len(g)}; ticket {med(g[:, 9] - g[:, 8])} (drain+barrier {med(g[:, 28] - g[:, 8])}); "
              f"group sum {med(g[:, 10] - g[:, 9])}")
        print(f"  all photos: contribution drain+barrier {med(s[:, 28] - s[:, 8])}")
        f = s[s[:, 11] > 0]
        if len(f):
            F = f[0]
            print(f"  final: ticket {F[11] - F[10]:.0f}, assemble {F[12] - F[11]:.0f}, solve {F[13] - F[12]:.0f}")
            print(f"  assemble: thread 0's sum + placement {F[17] - F[11]:.0f}, then the barrier {F[12] - F[17]:.0f}")
            sv = F[20:27]
            print(f"  solve: stop test (wave 0) {sv[4] - sv[0]:.0f} incl. barrier; GJ (wave 1) {sv[2] - sv[1]:.0f}; "
                  f"after GJ -> update start {sv[5] - sv[4]:.0f}; update {sv[6] - sv[5]:.0f}; tail {F[13] - sv[6]:.0f}")
    r0, r1 = s[:, 14], s[:, 15]
    ok = r1 > 0
    if ok.any():
        t0 = r0.min()
        print(f"  timeline (us, 100 MHz): starts spread {(r0.max() - t0) / 100:.2f}; "
              f"exit median {(np.median(r1[ok]) - t0) / 100:.2f}; last exit {(r1[ok].max() - t0) / 100:.2f}")
        print(f"  workgroup residency (us): {med((r1[ok] - r0[ok]) / 100)}")
        c = s[:, 29]
        if (c > 0).any():
            cc = c[c > 0]
            g = s[s[:, 30] > 0][:, 30]
            f = s[s[:, 31] > 0][:, 31]
            print(f"  contributions written (us): first {(cc.min() - t0) / 100:.2f} median {(np.median(cc) - t0) / 100:.2f} "
                  f"last {(cc.max() - t0) / 100:.2f}; group sums done: last {(g.max() - t0) / 100:.2f}; "
                  f"final ticket won {(f.max() - t0) / 100:.2f}; end {(r1[ok].max() - t0) / 100:.2f}")
    # placement / edge count vs linearisation time (slot 25: xcc << 32 | HW_ID, slot 27: edges)
    hw = s[:, 25].astype(np.int64)
    if (hw != 0).any():
        cu = (hw & 0xFFFFFFFF) >> 8 & 0xF
        sh = (hw & 0xFFFFFFFF) >> 12 & 0x1
        se = (hw & 0xFFFFFFFF) >> 13 & 0x7
        xcc = hw >> 32 & 0xF
        key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
        _, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
        share = cnt[inv]
        lin = s[:, 7] - s[:, 0]
        nes = s[:, 27]
        for n in np.unique(nes):
            sel = nes == n
            print(f"  ne={int(n)}: {sel.sum()} photos, linearize {med(lin[sel])}")
        for k in np.unique(share):
            sel = share == k
            print(f"  {int(k)} workgroup(s) on the CU: {sel.sum()} photos, linearize {med(lin[sel])}")
        print(f"  distinct CUs {len(cnt)}, xcc histogram {np.bincount(xcc.astype(int), minlength=8).tolist()}")
        # co-resident pairs: is wave 0 (the serial phases' wave) of both on the same SIMD?
        simd = (hw & 0xFFFFFFFF) >> 4 & 0x3
        same, diff = [], []
        for k in np.unique(key):
            idx = np.nonzero(key == k)[0]
            if len(idx) == 2:
                (same if simd[idx[0]] == simd[idx[1]] else diff).extend(lin[idx].tolist())
        print(f"  CU pairs with wave 0 on the same SIMD: {len(same) // 2}, linearize {med(np.array(same))}; "
              f"different SIMDs: {len(diff) // 2}, linearize {med(np.array(diff))}")
        print(f"  wave-0 SIMD histogram {np.bincount(simd.astype(int), minlength=4).tolist()}")
    ok = sch[:, 0] > 0
    if ok.any():
        it = sch[ok]
        print(f"k_schur: {ok.sum()} workgroups; item compute {med(it[:, 1] - it[:, 0])}")
        last = sch[sch[:, 3] > 0]
        if len(last):
            L = last[0]
            names = ["start", "items", "acquire", "assembly", "stoptest", "solve", "update", "end"]
            print("  last arriver: " + ", ".join(f"{names[k]}->{names[k+1]} {L[k+1]-L[k]:.0f}" for k in range(7)))


if __name__ == "__main__":
    main()
