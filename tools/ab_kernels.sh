#!/bin/bash
# Per-kernel A/B of libmcc builds on one bench configuration (rocprofv3 kernel stats, interleaved):
#   [ROUNDS=2] [STEPS=200] tools/ab_kernels.sh CONFIG libA.so libB.so ...
CFG=$1; shift
N=${ROUNDS:-2}; K=${STEPS:-200}
R=$PWD
for i in $(seq 1 $N); do
  for L in "$@"; do
    T=$R/gpurun_out/abk_$(basename $L .so)_$i
    ( cd /tmp && export TMPDIR=/tmp && MCC_LIB=$R/$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T -o run \
        --output-format csv -- python3 $R/bench.py --config $CFG --no-cpu --no-parity --no-extra --steps $K --warmup 20 \
        > $T.json 2>$T.err ) || exit 1
    python3 - "$T" "$(basename $L)" <<'PY'
import csv, glob, json, sys
d = json.load(open(sys.argv[1] + ".json"))
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
ks = {r["Name"].split("(")[0].replace("void mcc::", "").replace("mcc::", ""): float(r["AverageNs"]) / 1000 for r in csv.DictReader(open(f))}
print(sys.argv[2], f"{d['ms_per_step'] * 1000:.1f} us/step |", " ".join(f"{k}={v:.1f}" for k, v in sorted(ks.items()) if "rocclr" not in k))
PY
  done
done
