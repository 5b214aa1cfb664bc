#!/bin/bash
# per-kernel times (rocprofv3 --stats) of one config under environment variants:
#   tools/c3ab.sh config3 "VAR=a" "VAR=b" ...
set -o pipefail
R=$PWD
CFG=$1; shift
mkdir -p gpurun_out/c3ab
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
    i=$((i+1))
    env $v true || exit 2
    ( export $v; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/c3ab/v$i -o run --output-format csv \
        -- python3 $R/bench.py --config $CFG --steps 100 --warmup 10 --no-cpu --no-parity --no-extra > $R/gpurun_out/c3ab/v$i.json 2>&1 ) || exit 3
    f=$(find $R/gpurun_out/c3ab/v$i -name "*kernel_stats.csv" | head -n 1)
    echo "== $v  ms/step $(python3 -c "import json;print(round([json.loads(l) for l in open('$R/gpurun_out/c3ab/v$i.json') if l.startswith('{')][-1]['ms_per_step']*1e3,1))")"
    python3 -c "import csv,sys; [print(r['Name'][:40], round(float(r['AverageNs'])/1e3,1)) for r in csv.DictReader(open('$f')) if 'k_' in r['Name']]"
done
