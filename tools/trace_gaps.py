"""Per-step timeline of the split step from a rocprofv3 kernel trace: for the last 64 steps, the
median start of each kernel relative to the step's first kernel, its median duration, and (warm
solve) when k_sinv ran against k_schur's start.  Usage: python tools/trace_gaps.py kernel_trace.csv"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ks = []
for r in rows:
    n = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    short = n.split("(")[0].split("<")[0].replace("void ", "").replace("mcc::", "")
    ks.append((s, e, short))
ks.sort()
steps, cur = [], None
for s, e, n in ks:
    if n in ("k_prep", "k_group", "k_linearize"):
        cur = {}
        steps.append(cur)
    if cur is not None:
        cur.setdefault(n, (s, e))
steps = [st for st in steps if "k_solve" in st][-64:]
names = ["k_prep", "k_edge", "k_photo", "k_sinv", "k_schur", "k_solve"]
for n in names:
    v = [(st[n][0] - st["k_prep"][0], st[n][1] - st[n][0]) for st in steps if n in st and "k_prep" in st]
    if v:
        print(f"{n:8s} start {statistics.median(a for a, _ in v) / 1e3:8.2f} us  dur {statistics.median(b for _, b in v) / 1e3:7.2f} us  (n={len(v)})")
per = [st["k_solve"][1] - st["k_prep"][0] for st in steps if "k_prep" in st]
print("step (k_prep start -> k_solve end) median", statistics.median(per) / 1e3 if per else None, "us")
