import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from multi_camera_calibration_amd import api, rig
p = rig.make_config("config3", n_cams=9, n_views=40)
for graph in ("1", "0"):
    for hr in ("0", "1"):
        os.environ["MCC_HELPER_REFINE"] = hr
        os.environ["MCC_GRAPH"] = graph
        ba = api.BundleAdjuster(p)
        ba.set_params(p.x0)
        ba.step(12)
        ba.synchronize()
        s1 = ba.solve_stats()
        x1 = ba.get_params()
        ba.close()
        print("graph", graph, "helper_refine", hr, s1, float(abs(x1).sum()))
