#!/bin/bash
# round 4: register-resident m <= 30 refinement (MCC_SMALL_WARM=1) vs the register Gauss-Jordan
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r04m; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_warm_solve.py -m gpu -x -q --timeout 200 --timeout-method thread -k small > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -5; [ $rc -eq 0 ] || exit 10
bash tools/ab_trees.sh config4 3 HEAD "HEAD:MCC_SMALL_WARM=1" || exit 12
( export MCC_SMALL_WARM=1 MCC_DIAG_RT=1 MCC_LIB=multi_camera_calibration_amd/libmcc_diagrt.so; timeout -k 10 120 python tools/diag_schur.py config4 ) || exit 11
