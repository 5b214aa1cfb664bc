set -o pipefail
export MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so
timeout -k 10 120 python tools/diag_split.py config4 || exit 1
timeout -k 10 120 python tools/diag_split.py config5 2>&1 | grep -A6 "k_schur" || exit 2
timeout -k 10 120 python tools/diag_split.py config3 2>&1 | grep -A6 "k_schur" || exit 3
