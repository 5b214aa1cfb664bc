#!/bin/bash
# round 4: one-level k_schur -- bitwise tests, poisoned hand-offs, peer config4_split, A/B timing, full bench
set -o pipefail
OUT=gpurun_out/${1:-r04d}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_schur_levels.py tests/test_handoff_poison.py tests/test_peer_transport.py -k "levels or poison or config4_split or config2_small" -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -25; [ $rc -le 1 ] || exit 10
bash tools/env_ab.sh config4 3 MCC_SCHUR_ONE_LEVEL=0 MCC_SCHUR_ONE_LEVEL=1 || exit 12
bash tools/r04c.sh ${1:-r04d} || exit 11
