#!/bin/bash
# Interleaved A/B of bench.py at the driver's settings (--steps 20 --warmup 5, no extra keys):
#   tools/driver_ab.sh ROUNDS "VAR=a" "VAR=b" ...
N=$1; shift
mkdir -p gpurun_out/drvab
for r in $(seq 1 $N); do
    for v in "$@"; do
        ( export $v; timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-parity --no-extra > gpurun_out/drvab/o.json 2>&1 ) || exit 3
        echo "round $r $v: $(python3 -c "import json;d=[json.loads(l) for l in open('gpurun_out/drvab/o.json') if l.startswith('{')][-1];print(round(d['ms_per_step']*1e3,2), 'us/step; window', round(d['roofline']['step_ms_events']*1e3,2))")"
    done
done
