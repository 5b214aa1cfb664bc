set -o pipefail
mkdir -p gpurun_out/r03_gpu13
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gpu13/parity.log 2>&1 || { tail -40 gpurun_out/r03_gpu13/parity.log; exit 1; }
tail -3 gpurun_out/r03_gpu13/parity.log
tools/env_ab.sh config3 2 "MCC_PREP_LANES=4" "MCC_PREP_LANES=1" || exit 2
tools/env_ab.sh config5 2 "MCC_PREP_LANES=4" "MCC_PREP_LANES=1" || exit 3
MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so timeout -k 10 120 python tools/diag_split.py config3 || exit 5
