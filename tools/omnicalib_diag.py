"""Locates a failing omnidir calibrate run: host initialisation, then the device loop in chunks,
reporting the rms and the worst views after each chunk (diagnostic tool, not a test)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from multi_camera_calibration_amd import api, rig
from oracle import oracle_py as O

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
s = rig.make_omni_views(n, seed=4)
om, t, K, xi, idx = api.omnidir_initialize(s.off, s.obj, s.img, s.image_size)
v = O.OmniViews(s.off, s.obj, s.img).subset(idx)
p = O.omni_encode(om, t, K, xi)
print("kept", len(idx), "K", K[0, 0], flush=True)
oc = api.OmniCalibrator(v.off, v.obj, v.img)
good = p
for chunk in range(12):
    try:
        p2, it, ch = oc.optimize(p, 1, 25 * (chunk + 1), 0.0)
    except api.MccError as e:
        print("fail at <=", 25 * (chunk + 1), e, flush=True)
        # per-view error at the last good params
        errs = []
        for i in range(v.n):
            sl = slice(v.off[i], v.off[i + 1])
            q = good
            proj, _ = O.omni_project_full(v.obj[sl], q[6*i:6*i+3], q[6*i+3:6*i+6],
                                          q[6*v.n:6*v.n+5], q[6*v.n+5], q[6*v.n+6:], jac=False)
            errs.append(np.sqrt(((proj - v.img[sl]) ** 2).sum(1).mean()))
        errs = np.array(errs)
        w = np.argsort(-np.nan_to_num(errs, nan=1e9))[:5]
        print("worst views", w, errs[w], "pose", [good[6*i:6*i+6] for i in w[:2]], flush=True)
        break
    good = p2
    print(25 * (chunk + 1), "rms", oc.rms(p2), "change", ch, "intr", p2[6 * v.n:6 * v.n + 6], flush=True)
