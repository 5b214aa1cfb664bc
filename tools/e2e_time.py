"""End-to-end host-visible latency of the C ABI on one problem (what a caller of
optimizeExtrinsics waits for): mcc_create, the first optimize (graph capture included), a second
optimize, project_error and destroy, against the oracle's optimize on the host cores."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multi_camera_calibration_amd import api, rig  # noqa: E402
from oracle import oracle_py as O  # noqa: E402


def main():
    for cfg in sys.argv[1:] or ["config1", "config2", "config3"]:
        p = rig.make_config(cfg)
        t0 = time.perf_counter()
        g = api.BundleAdjuster(p)
        t1 = time.perf_counter()
        x, m, it, _ = g.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        t2 = time.perf_counter()
        x, m, it, _ = g.optimize_extrinsics(p.x0, crit_type=3, max_count=200, eps=1e-7)
        t3 = time.perf_counter()
        e, pm = g.compute_project_error(x)
        t4 = time.perf_counter()
        g.close()
        t5 = time.perf_counter()
        g = api.BundleAdjuster(p)   # a second problem: warm runtime, pooled stream
        t5b = time.perf_counter()
        g.close()
        t5c = time.perf_counter()
        o = O.Oracle(p)
        t6 = time.perf_counter()
        o.optimize(p.x0, crit_type=3, max_count=200, eps=1e-7)
        t7 = time.perf_counter()
        ms = lambda a, b: f"{(b - a) * 1e3:.2f}"  # noqa: E731
        print(f"{cfg}: views {p.n_photos} iters {it} | create {ms(t0, t1)} ms, optimize#1 {ms(t1, t2)} ms, "
              f"optimize#2 {ms(t2, t3)} ms, project_error {ms(t3, t4)} ms, destroy {ms(t4, t5)} ms, "
              f"create+destroy again {ms(t5, t5b)} + {ms(t5b, t5c)} ms | "
              f"oracle optimize {ms(t6, t7)} ms ({O.num_threads() if hasattr(O, 'num_threads') else '?'} threads)",
              flush=True)


if __name__ == "__main__":
    main()
