#!/bin/bash
# Quick GPU pass during kernel work: the -m gpu suite, then a short bench line per config
# (no CPU baseline, no parity leg).  Usage: tools/quick_gpu.sh <tag> [configs...]
set -o pipefail
TAG=${1:-quick}
shift
CFGS=${*:-config2 config3 config4 config5}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -n 5 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
for c in $CFGS; do
    timeout -k 10 300 python bench.py --config $c --no-cpu --no-parity --no-extra > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit 11
    python3 -c "import json,sys; d=json.loads(open('$OUT/bench_$c.json').read().strip().split('\n')[-1]); print('$c', round(d['ms_per_step']*1e3,2), 'us/step', 'kernel', round(d['roofline']['kernel_ms_per_launch']*1e3,2))"
done
exit 0
