#!/bin/bash
# round 4: the full bench line (driver settings) with its extra keys, and a quick summary
set -o pipefail
OUT=gpurun_out/${1:-r04c}
mkdir -p $OUT
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $OUT/bench_full.json 2> $OUT/bench_full.err || exit 11
python3 -c "
import json; d=json.loads(open('$OUT/bench_full.json').read().strip().split('\n')[-1])
print('headline', round(d['ms_per_step']*1e3,2), 'us', {k:(round(v*1e3,2) if isinstance(v,float) else v) for k,v in d['step_distribution'].items()}, 'kernel', round(d['roofline']['kernel_ms_per_launch']*1e3,2), 'frac', round(d['roofline']['frac'],4))
for k,v in d['configs'].items(): print(k, round(v['ms_per_step']*1e3,2), 'median', round(v['step_distribution']['median']*1e3,2), 'kernel', round(v['roofline']['kernel_ms_per_launch']*1e3,2))
for k,v in d['shard'].items(): print(k, round(v['ms_per_step']*1e3,2), v.get('compute_speedup_bound'))
"
