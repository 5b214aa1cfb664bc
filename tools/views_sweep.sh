#!/bin/bash
# Step time of config2-shaped rigs against the number of views (one GPU): how the fused step's
# time splits into a per-photo part and a fixed tail.  Usage: tools/views_sweep.sh <tag> [views...]
set -o pipefail
TAG=${1:-vs}; shift
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"
for v in ${*:-64 128 256 384 500 512 640}; do
    timeout -k 10 200 python bench.py --config config2 --views $v --no-cpu --no-parity --no-extra --steps 1000 \
        > "$OUT/v$v.json" 2> "$OUT/v$v.err" || exit 1
    python3 -c "import json; d=json.loads(open('$OUT/v$v.json').read().strip().split('\n')[-1]); print($v, round(d['ms_per_step']*1e3,2), 'us/step', round(d['roofline']['kernel_ms_per_launch']*1e3,2))"
done
