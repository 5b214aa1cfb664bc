set -o pipefail
tools/env_ab.sh config4 3 "MCC_LIB=multi_camera_calibration_amd/libmcc.so" "MCC_LIB=build_ab/pair256/libmcc.so" || exit 2
