set -o pipefail
export MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so
timeout -k 10 120 python tools/diag_split.py config4 || exit 5
MCC_GROUP_LANES=16 timeout -k 10 120 python tools/diag_split.py config4 || exit 6
