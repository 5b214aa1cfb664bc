#!/bin/bash
# round 4: one-level k_schur + the m <= 30 warm solve -- parity, poison, peer, A/B timing, full bench
set -o pipefail
OUT=gpurun_out/${1:-r04e}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size.py tests/test_schur_levels.py tests/test_handoff_poison.py tests/test_peer_transport.py tests/test_warm_solve.py -k "not config3_full and not config5_full" -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -25; [ $rc -le 1 ] || exit 10
bash tools/env_ab.sh config4 3 "MCC_SCHUR_ONE_LEVEL=0 MCC_SMALL_WARM=0" "MCC_SMALL_WARM=0" "MCC_SMALL_WARM=1" "MCC_ITEM_SLOTS=64" "MCC_ITEM_SLOTS=128" || exit 12
bash tools/r04c.sh ${1:-r04e} || exit 11
