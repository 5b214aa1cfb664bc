#!/bin/bash
# end-of-session GPU pass: the -m gpu suite (full, verbose), bench at the driver's settings and at
# defaults, then the per-config rocprofv3 stats + PMC traffic + FP64 passes (tools/profile_r03.sh)
set -o pipefail
TAG=${1:-r03_final}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc"; tail -n 3 "$OUT/pytest.log"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" || exit 11
timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit 12
python3 -c "
import json
for f in ('bench_driver', 'bench_default'):
    d = json.loads(open('$OUT/' + f + '.json').read().strip().split('\n')[-1])
    print(f, round(d['ms_per_step'] * 1e3, 2), 'us/step', {k: round(v['ms_per_step'] * 1e3, 2) for k, v in d.get('configs', {}).items()})"
bash tools/profile_r03.sh ${TAG}_prof || exit 13
exit 0
