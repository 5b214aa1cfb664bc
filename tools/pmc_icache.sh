#!/bin/bash
# Instruction-cache counters of the config4 step per libmcc build (one rocprofv3 --pmc pass each):
#   tools/pmc_icache.sh <tag> lib1.so [lib2.so ...]   -> gpurun_out/<tag>/icache_<n>.csv
R=$PWD
OUT=$R/gpurun_out/$1; shift
mkdir -p $OUT
n=0
for L in "$@"; do
  n=$((n + 1))
  ( cd /tmp && export TMPDIR=/tmp && MCC_LIB=$R/$L timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_REQ SQ_WAVES \
      -d $OUT/ic_$n -o run --output-format csv -- python3 $R/bench.py --config config4 --no-cpu --no-parity --no-extra \
      --steps 30 --warmup 4 --ramp-seconds 0.05 > $OUT/ic_$n.log 2>&1 ) || exit 1
  f=$(find $OUT/ic_$n -name "*counter_collection.csv" | head -n 1)
  python3 - "$f" "$L" <<'PY'
import csv, sys
from collections import defaultdict
v = defaultdict(list)
for row in csv.DictReader(open(sys.argv[1])):
    if "k_group" in (row.get("Kernel_Name") or ""):
        v[row["Counter_Name"]].append(float(row["Counter_Value"]))
print(sys.argv[2], {k: round(sum(x) / len(x)) for k, x in v.items()})
PY
done
