#!/bin/bash
# the -m gpu suite, then bench lines for every config (defaults) and config3 with MCC_WARM=0
set -o pipefail
OUT=$PWD/gpurun_out/${1:-s2_check}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -n 8 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
for c in ${CFGS:-config3 config2 config4 config5 config3:0}; do
    cfg=${c%%:*}; w=1; [ "$c" != "$cfg" ] && w=${c##*:}
    MCC_WARM=$w timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-parity --no-extra > "$OUT/bench_${cfg}_w$w.json" 2> "$OUT/bench_${cfg}_w$w.err" || exit 11
    python3 -c "import json; d=json.loads(open('$OUT/bench_${cfg}_w$w.json').read().strip().split('\n')[-1]); print('$cfg warm=$w', round(d['ms_per_step']*1e3,2), 'us/step', d.get('warm_solve'))"
done
exit 0
