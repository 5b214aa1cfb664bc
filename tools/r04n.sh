#!/bin/bash
# round 4: full GPU suite, smoke, default bench line
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/${1:-r04n}; mkdir -p $OUT
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -20; [ $rc -eq 0 ] || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || exit 11
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 12
tail -c 1500 $OUT/bench.json
