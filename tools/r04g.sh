#!/bin/bash
# round 4: config4 bisect (round 3 / before the k_schur changes / HEAD / HEAD with both m <= 30 changes
# off), the config4 tail on the realtime-stamped build per variant, k_solve warm stamps at config3
set -o pipefail
export PYTHONUNBUFFERED=1
bash tools/ab_trees.sh config4 3 r03 pre1l HEAD "HEAD:MCC_SMALL_WARM=0" "HEAD:MCC_SMALL_WARM=0 MCC_SCHUR_ONE_LEVEL=0" || exit 12
for v in "MCC_X=0" "MCC_SMALL_WARM=0" "MCC_SMALL_WARM=0 MCC_SCHUR_ONE_LEVEL=0"; do
  echo "== diag_schur config4 $v"
  ( export $v MCC_DIAG_RT=1 MCC_LIB=multi_camera_calibration_amd/libmcc_diagrt.so; timeout -k 10 120 python tools/diag_schur.py config4 ) || exit 13
done
MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so timeout -k 10 120 python tools/diag_solve.py config3 20 || exit 14
