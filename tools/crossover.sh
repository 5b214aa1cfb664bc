#!/bin/bash
# Fused vs split step on config2-shaped rigs (4 pinhole cameras, m = 18) past the fused rule's
# V <= 2 x CUs bound: each view count with MCC_FUSED=1 and =0, 1000 steps, interleaved.
# Usage: tools/crossover.sh <tag> [views...]
set -o pipefail
TAG=${1:-xo}; shift
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"
for v in ${*:-384 512 576 640 768 1024}; do
    for f in 1 0; do
        MCC_FUSED=$f timeout -k 10 200 python bench.py --config config2 --views $v --no-cpu --no-parity --no-extra \
            --steps 1000 > "$OUT/v${v}_f$f.json" 2> "$OUT/v${v}_f$f.err" || exit 1
        python3 -c "import json; d=json.loads(open('$OUT/v${v}_f$f.json').read().strip().split('\n')[-1]); print($v, 'fused' if $f else 'split', round(d['ms_per_step']*1e3,2), 'us/step')"
    done
done
