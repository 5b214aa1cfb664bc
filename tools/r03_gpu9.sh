set -o pipefail
mkdir -p gpurun_out/r03_gpu9
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gpu9/parity.log 2>&1 || { tail -30 gpurun_out/r03_gpu9/parity.log; exit 1; }
tail -3 gpurun_out/r03_gpu9/parity.log
tools/env_ab.sh config4 2 "MCC_GROUP_LANES=32" "MCC_GROUP_LANES=16" || exit 2
tools/env_ab.sh config5 1 "MCC_GROUP=1" "MCC_GROUP=0" || exit 3
tools/env_ab.sh config3 1 "MCC_GROUP=1" "MCC_GROUP=0" || exit 4
MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so timeout -k 10 120 python tools/diag_split.py config4 || exit 5
