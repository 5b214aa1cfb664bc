#!/bin/bash
# round 4: one-level k_schur with sized batches and stores after the sums: bitwise / parity subset,
# config4 tail timeline, A/B against round 3 and the previous one-level form
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r04l; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_schur_levels.py tests/test_warm_solve.py tests/test_handoff_poison.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -15; [ $rc -eq 0 ] || exit 10
( export MCC_DIAG_RT=1 MCC_LIB=multi_camera_calibration_amd/libmcc_diagrt.so; timeout -k 10 120 python tools/diag_schur.py config4 ) || exit 11
bash tools/ab_trees.sh config4 3 r03 olfix HEAD || exit 12
bash tools/ab_trees.sh config5 2 r03 olfix HEAD || exit 13
