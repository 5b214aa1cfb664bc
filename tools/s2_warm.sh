#!/bin/bash
# warm-solve check: the -m gpu suite, then configs 3 and 5 with the warm solve on and off (interleaved)
set -o pipefail
OUT=$PWD/gpurun_out/${1:-s2_warm}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
tail -n 8 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
for r in 1; do
for w in 1 0; do
for c in config3; do
    MCC_WARM=$w timeout -k 10 300 python bench.py --config $c --no-cpu --no-parity --no-extra > "$OUT/bench_${c}_w${w}_$r.json" 2> "$OUT/bench_${c}_w${w}_$r.err" || exit 11
    python3 -c "import json; d=json.loads(open('$OUT/bench_${c}_w${w}_$r.json').read().strip().split('\n')[-1]); print('$c warm=$w', round(d['ms_per_step']*1e3,2), 'us/step', d.get('warm_solve', d['config'].get('warm_solve')))"
done; done; done
bash tools/s2_prof3.sh ${1:-s2_warm}_prof || exit 12
exit 0
