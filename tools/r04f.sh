#!/bin/bash
# round 4: warm-solve prev2 hand-off + inlined helpers: parity subset, A/B against round 3, k_solve stamps, shard variants
set -o pipefail
OUT=gpurun_out/${1:-r04f}
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_warm_solve.py tests/test_peer_transport.py tests/test_schur_levels.py tests/test_handoff_poison.py tests/test_gpu_parity.py -k "not config3_full and not config5_full" -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -15; [ $rc -le 1 ] || exit 10
bash tools/ab_trees.sh config4 3 r03 HEAD "HEAD:MCC_SMALL_WARM=0" "HEAD:MCC_SMALL_WARM=0 MCC_SCHUR_ONE_LEVEL=0" || exit 12
bash tools/ab_trees.sh config3 2 r03 HEAD || exit 13
MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so timeout -k 10 120 python tools/diag_solve.py config3 20 || exit 14
timeout -k 10 300 python tools/shard_ab.py config3 8 2 - MCC_GROUP=1 || exit 15
