#!/bin/bash
# Round-4 focused GPU pass: the named pytest selection, then one short bench line per config.
# Usage: [PYK="<-k expression>"] tools/r04_focus.sh <tag> "<pytest files>" [configs...]
set -o pipefail
TAG=$1; shift
TESTS=$1; shift
CFGS=${*:-}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
if [ -n "$TESTS" ]; then
    KARGS=()
    [ -n "$PYK" ] && KARGS=(-k "$PYK")
    timeout -k 10 900 python -u -m pytest $TESTS "${KARGS[@]}" -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
    rc=$?
    grep -E "PASSED|FAILED|ERROR|passed|failed" "$OUT/pytest.log" | tail -n 40
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
fi
for c in $CFGS; do
    timeout -k 10 300 python bench.py --config $c --no-cpu --no-parity --no-extra > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" || exit 11
    python3 -c "import json; d=json.loads(open('$OUT/bench_$c.json').read().strip().split('\n')[-1]); print('$c', round(d['ms_per_step']*1e3,2), 'us/step', 'kernel', round(d['roofline']['kernel_ms_per_launch']*1e3,2), d.get('warm_solve',''))"
done
exit 0
