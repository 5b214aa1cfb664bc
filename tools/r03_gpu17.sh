set -o pipefail
export MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so
timeout -k 10 120 python tools/diag_split.py config4 2>&1 | grep -v "^k_schur\|items summed\|level 1\|winner" || exit 1
