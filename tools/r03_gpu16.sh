set -o pipefail
mkdir -p gpurun_out/r03_gpu16
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_handoff_poison.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gpu16/parity.log 2>&1 || { tail -40 gpurun_out/r03_gpu16/parity.log; exit 1; }
tail -3 gpurun_out/r03_gpu16/parity.log
tools/env_ab.sh config4 3 "MCC_GROUP_FOLD=1" "MCC_GROUP_FOLD=0" || exit 2
