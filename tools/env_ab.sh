#!/bin/bash
# Interleaved A/B of bench.py ms/step under environment variants (no profiler):
#   tools/env_ab.sh config2 ROUNDS "VAR=a" "VAR=b" ...
set -o pipefail
CFG=$1; N=$2; shift 2
mkdir -p gpurun_out/envab
for r in $(seq 1 $N); do
    for v in "$@"; do
        ( export $v; timeout -k 10 120 python bench.py --config $CFG --no-cpu --no-parity --no-extra > gpurun_out/envab/o.json 2>&1 ) || exit 3
        echo "$CFG round $r $v: $(python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/envab/o.json') if l.startswith('{')][-1];print(round(d['ms_per_step']*1e3,2), 'us/step; window', round(d['roofline']['step_ms_events']*1e3,2))")"
    done
done
