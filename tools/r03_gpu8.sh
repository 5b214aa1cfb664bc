set -o pipefail
export MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so
timeout -k 10 120 python tools/diag_split.py config4 || exit 1
MCC_GROUP=1 timeout -k 10 120 python tools/diag_split.py config5 || exit 2
MCC_GROUP=1 timeout -k 10 120 python tools/diag_split.py config3 || exit 3
