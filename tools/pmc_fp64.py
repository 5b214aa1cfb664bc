"""FP64 work per launch of the hot kernel from one rocprofv3 --pmc pass (report
the FP64-VALU fraction beside the HBM one).

  rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 \\
            SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 -d <dir> -- python3 bench.py ...
  python tools/pmc_fp64.py --dir <dir> --config config2 --views 500 --corners 172744 \\
         --out profiles/fp64_config2_500.json

SQ_INSTS_VALU_FLOPS_FP64 (+ _TRANS) count FP64 operations of VALU instructions per WAVE
instruction (an FMA counts 2; MFMA excluded): measured, FLOPS_FP64 = 2 FMA_F64 + ADD_F64 + MUL_F64
exactly.  Lane operations are 64 x that (rocprofv3's own derived FLOP expressions multiply by 64),
an upper bound: lanes masked off by EXEC are counted too.  Six SQ counters fit one pass (<= 8).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import read_counters, short  # noqa: E402

COUNTERS = ["SQ_INSTS_VALU_FLOPS_FP64", "SQ_INSTS_VALU_FLOPS_FP64_TRANS", "SQ_INSTS_VALU_FMA_F64",
            "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--config", default="config2")
    ap.add_argument("--views", type=int, default=500)
    ap.add_argument("--corners", type=float, required=True, help="corners per k_linearize launch")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    vals = read_counters(a.dir)
    kernels = {}
    for (name, cn), v in vals.items():
        k = short(name)
        e = kernels.setdefault(k, {"launches": 0})
        e[cn] = sum(v) / len(v)
        e["launches"] = max(e["launches"], len(v))
    for e in kernels.values():
        e["fp64_flops"] = 64.0 * (e.get("SQ_INSTS_VALU_FLOPS_FP64", 0.0) + e.get("SQ_INSTS_VALU_FLOPS_FP64_TRANS", 0.0))
    for e in kernels.values():
        e["fp64_flops_per_corner"] = e["fp64_flops"] / a.corners if a.corners else None
    step_kernels = [k for k in ("k_linearize", "k_group", "k_prep", "k_edge", "k_photo", "k_schur", "k_solve") if k in kernels]
    step = sum(kernels[k]["fp64_flops"] for k in step_kernels)
    lin_k = [k for k in ("k_linearize", "k_group", "k_prep", "k_edge", "k_photo") if k in kernels]
    lin = {"fp64_flops": sum(kernels[k]["fp64_flops"] for k in lin_k)} if lin_k else {}
    out = {"config": a.config, "n_views": a.views, "kernel": "+".join(lin_k),
           "step_kernels": step_kernels, "step_fp64_flops": step,
           "step_fp64_flops_per_corner": step / a.corners if a.corners else None,
           "fp64_flops_per_launch": lin.get("fp64_flops"),
           "fp64_flops_per_corner": (lin.get("fp64_flops", 0.0) / a.corners) if a.corners else None,
           "method": "rocprofv3 --pmc " + " ".join(COUNTERS) + " (one pass); flops = 64 x (FLOPS_FP64 + "
                     "FLOPS_FP64_TRANS) per launch (wave instructions x 64 lanes: an upper bound, EXEC-masked "
                     "lanes included)",
           "kernels": kernels}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("fp64_flops_per_launch", "fp64_flops_per_corner", "step_fp64_flops_per_corner")}))


if __name__ == "__main__":
    main()
