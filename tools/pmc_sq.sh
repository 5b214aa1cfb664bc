#!/bin/bash
# SQ counters per kernel (one rocprofv3 --pmc pass, kernel trace only) on a bench configuration:
#   tools/pmc_sq.sh CONFIG OUTDIR [MCC_LIB] [JSON VIEWS]
# prints one line per kernel; with JSON (e.g. profiles/sq_config4_1000.json) also writes the per-kernel
# VALU issue figures bench.py reports beside fp64_valu: the VALU-active share of each wave's cycles
# (SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, both quad-cycles) times the waves a SIMD holds at the kernel's
# occupancy (__launch_bounds__: 2 for k_group, k_linearize, k_photo, k_schur) = the SIMD's VALU issue share
CFG=$1; OUT=$(realpath -m $2); LIB=${3:-}; JS=${4:-}; VIEWS=${5:-0}
R=$PWD
mkdir -p "$OUT"
( cd /tmp && export TMPDIR=/tmp && MCC_LIB=${LIB:+$R/$LIB} timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU \
    SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d "$OUT" -o run \
    --output-format csv -- python3 "$R/bench.py" --config "$CFG" --no-cpu --no-parity --no-extra --steps 20 --warmup 4 \
    > "$OUT/bench.json" 2> "$OUT/bench.err" ) || exit 1
python3 - "$OUT" "$CFG" "$JS" "$VIEWS" <<'PY'
import csv, glob, json, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
WPS = {"k_group": 2, "k_linearize": 2, "k_photo": 2, "k_schur": 2}
js = {"config": sys.argv[2], "n_views": int(sys.argv[4]), "source": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU "
      "SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES ... (tools/pmc_sq.sh)", "kernels": {}}
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
    base = k.split("<")[0].strip()
    act = m.get("SQ_ACTIVE_INST_VALU", 0) / max(m.get("SQ_WAVE_CYCLES", 1), 1)
    e = {"valu_insts_per_wave": m.get("SQ_INSTS_VALU", 0) / w, "valu_active_per_wave": act}
    if base in WPS:
        e["waves_per_simd"] = WPS[base]
        e["valu_issue_frac"] = act * WPS[base]
    js["kernels"][base] = e
if sys.argv[3]:
    json.dump(js, open(sys.argv[3], "w"), indent=1)
PY
