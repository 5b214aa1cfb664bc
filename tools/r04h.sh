#!/bin/bash
# round 4: one-level k_schur with batched loads: bitwise/parity subset, config4 A/B, tail stamps
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r04h; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_schur_levels.py tests/test_warm_solve.py tests/test_gpu_parity.py tests/test_handoff_poison.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -15; [ $rc -le 1 ] || exit 10
bash tools/ab_trees.sh config4 3 r03 HEAD "HEAD:MCC_SMALL_WARM=0" "HEAD:MCC_SMALL_WARM=0 MCC_SCHUR_ONE_LEVEL=0" || exit 12
bash tools/ab_trees.sh config2 2 r03 HEAD "HEAD:MCC_SCHUR_ONE_LEVEL=0" || exit 13
bash tools/ab_trees.sh config5 2 r03 HEAD "HEAD:MCC_SCHUR_ONE_LEVEL=0" || exit 14
