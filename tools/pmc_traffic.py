"""Per-launch memory traffic of the hot kernels from two rocprofv3 --pmc passes.

  python tools/pmc_traffic.py --fetch <dir of the FETCH_SIZE pass> --write <dir of the WRITE_SIZE pass>
         --config config2 --views 500 --out profiles/traffic_config2_500.json

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB from the L2's memory-side request
counters (TCC_EA0_RDREQ / _WRREQ).  Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled here;
WRITE_SIZE is taken as is.  Infinity-Cache hits are counted as memory-side traffic, and this
working set (~4 MB per step) is L2/Infinity-Cache resident, so the figure is memory-side bytes,
not DRAM bytes; our loads are 4 B/lane float SoA streams, a width the guide leaves uncalibrated.
Passes are separate (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def read_counters(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = defaultdict(list)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                cn = row.get("Counter_Name") or row.get("Counter-Name")
                cv = row.get("Counter_Value") or row.get("Counter-Value")
                if cn is None or cv is None:
                    continue
                vals[(name, cn)].append(float(cv))
    return vals


def short(name):
    for k in ("k_linearize", "k_group", "k_schur", "k_solve", "k_backsub", "k_project_error", "k_prep", "k_edge", "k_photo"):
        if k in name:
            return k
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--config", default="config2")
    ap.add_argument("--views", type=int, default=500)
    ap.add_argument("--alg-bytes", type=float, default=None, help="algorithmic bytes per k_linearize launch")
    ap.add_argument("--fetch-correction", type=float, default=2.0,
                    help="FETCH_SIZE multiplier (2 = the guide's 16-B-per-lane figure; tools/fetch_calib.hip measures others)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    fv, wv = read_counters(a.fetch), read_counters(a.write)
    kernels = {}
    for (name, cn), v in list(fv.items()) + list(wv.items()):
        k = short(name)
        e = kernels.setdefault(k, {"launches": 0})
        mean = sum(v) / len(v)
        if cn.startswith("FETCH_SIZE"):
            e["fetch_kib_raw"] = mean
            e["launches"] = max(e["launches"], len(v))
        elif cn.startswith("WRITE_SIZE"):
            e["write_kib"] = mean
    for k, e in kernels.items():
        fb = a.fetch_correction * 1024.0 * e.get("fetch_kib_raw", 0.0)
        wb = 1024.0 * e.get("write_kib", 0.0)
        e["read_bytes_corrected"] = fb
        e["write_bytes"] = wb
        e["bytes_per_launch"] = fb + wb
    step_kernels = [k for k in ("k_linearize", "k_group", "k_prep", "k_edge", "k_photo", "k_schur", "k_solve") if k in kernels]
    step_bytes = sum(kernels[k]["bytes_per_launch"] for k in step_kernels)
    lin_k = [k for k in ("k_linearize", "k_group", "k_prep", "k_edge", "k_photo") if k in kernels]
    lin = {"bytes_per_launch": sum(kernels[k]["bytes_per_launch"] for k in lin_k)} if lin_k else {}
    out = {
        "config": a.config, "n_views": a.views, "kernel": "+".join(lin_k),
        "step_kernels": step_kernels, "step_bytes_per_launch": step_bytes,
        "step_ratio_to_alg": (step_bytes / a.alg_bytes) if a.alg_bytes else None,
        "bytes_per_launch": lin.get("bytes_per_launch"),
        "alg_bytes_per_launch": a.alg_bytes,
        "ratio_to_alg": (lin["bytes_per_launch"] / a.alg_bytes) if (a.alg_bytes and lin) else None,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; "
                  f"bytes = {a.fetch_correction:g} x 1024 x FETCH_SIZE(KiB) [gfx950 correction] + 1024 x WRITE_SIZE(KiB); "
                  "memory-side (L2 -> fabric) bytes incl. Infinity-Cache hits",
        "kernels": kernels,
    }
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
