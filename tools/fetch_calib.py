"""Counter / byte ratios of tools/fetch_calib.hip's kernels (see that file).

  python tools/fetch_calib.py --fetch <FETCH_SIZE pass dir> --write <WRITE_SIZE pass dir>
         --bytes <the JSON line fetch_calib printed> --out profiles/<round>/fetch_calib.json

ratio = counter bytes (KiB x 1024, uncorrected) / bytes the kernel moved; the FETCH correction for
a width is 1 / its read ratio.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import read_counters  # noqa: E402


def per_kernel(vals, prefix):
    out = {}
    for (name, cn), v in vals.items():
        if not cn.startswith(prefix):
            continue
        for k in ("rd_f32_soa", "rd_f64_sc1", "rd_f64", "rd_f128", "wr_f64_sc1", "wr_f64", "wr_f32", "wr_f128"):
            if k in name:
                out[k] = sum(v) / len(v)
                break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--bytes", required=True, help="file holding fetch_calib's JSON line")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    moved = None
    for line in open(a.bytes):
        if line.startswith("{"):
            moved = json.loads(line)
    if moved is None:
        raise SystemExit("no byte line in " + a.bytes)
    fk = per_kernel(read_counters(a.fetch), "FETCH_SIZE")
    wk = per_kernel(read_counters(a.write), "WRITE_SIZE")
    res = {}
    for k, b in moved.items():
        kib = fk.get(k) if k.startswith("rd") else wk.get(k)
        if kib is None:
            continue
        r = kib * 1024.0 / b
        res[k] = {"bytes_moved": b, "counter": "FETCH_SIZE" if k.startswith("rd") else "WRITE_SIZE",
                  "counter_kib": kib, "ratio": r, "correction": (1.0 / r) if r else None}
    out = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of tools/fetch_calib.hip: "
                     "96 MiB per launch (3x aggregate L2), 2048 x 256 threads, grid-stride",
           "kernels": res}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
