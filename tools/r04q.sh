#!/bin/bash
# round 4: two independent single-GPU benches at once on one device (no exchange): does the split
# step's same-device N = 2 slowdown come from sharing the GPU between processes?
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r04q; mkdir -p $OUT
for c in config5 config4 config3; do
  timeout -k 10 200 python bench.py --config $c --no-cpu --no-parity --no-extra > $OUT/${c}_solo.json 2>&1 || exit 11
  ( timeout -k 10 300 python bench.py --config $c --no-cpu --no-parity --no-extra > $OUT/${c}_a.json 2>&1 ) &
  PA=$!
  ( timeout -k 10 300 python bench.py --config $c --no-cpu --no-parity --no-extra > $OUT/${c}_b.json 2>&1 ) &
  PB=$!
  wait $PA || exit 12
  wait $PB || exit 13
  python3 -c "
import json
def ms(f): d=[json.loads(l) for l in open(f) if l.startswith('{')][-1]; return round(d['ms_per_step']*1e3,2), round(d['roofline']['kernel_ms_per_launch']*1e3,2)
print('$c solo', ms('$OUT/${c}_solo.json'), 'two at once', ms('$OUT/${c}_a.json'), ms('$OUT/${c}_b.json'))"
done
bash tools/ab_trees.sh config3 2 olfix HEAD || exit 14
