#!/bin/bash
# SQ counters per kernel (one rocprofv3 --pmc pass, kernel trace only) on a bench configuration:
#   tools/pmc_sq.sh CONFIG OUTDIR [MCC_LIB]
CFG=$1; OUT=$(realpath -m $2); LIB=${3:-}
R=$PWD
mkdir -p "$OUT"
( cd /tmp && export TMPDIR=/tmp && MCC_LIB=${LIB:+$R/$LIB} timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT" -o run \
    --output-format csv -- python3 "$R/bench.py" --config "$CFG" --no-cpu --no-parity --no-extra --steps 20 --warmup 4 \
    > "$OUT/bench.json" 2> "$OUT/bench.err" ) || exit 1
python3 - "$OUT" <<'PY'
import csv, glob, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void mcc::", "").replace("mcc::", "")
    v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in v.items():
    if "rocclr" in k:
        continue
    m = {n: sum(x) / len(x) for n, x in c.items()}
    w = max(m.get("SQ_WAVES", 1), 1)
    print(k, " ".join(f"{n.replace('SQ_', '')}={m[n]:.4g}" for n in sorted(m)),
          f"| VALU/wave={m.get('SQ_INSTS_VALU', 0) / w:.0f} LDS/wave={m.get('SQ_INSTS_LDS', 0) / w:.0f}")
PY
