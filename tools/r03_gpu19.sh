set -o pipefail
mkdir -p gpurun_out/r03_gpu19
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_handoff_poison.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gpu19/parity.log 2>&1 || { tail -40 gpurun_out/r03_gpu19/parity.log; exit 1; }
tail -3 gpurun_out/r03_gpu19/parity.log
tools/env_ab.sh config4 2 "MCC_SCHUR2=1" "MCC_SCHUR2=0" "MCC_SCHUR2_SLOTS=16" "MCC_SCHUR2_SLOTS=64" || exit 2
tools/env_ab.sh config5 2 "MCC_SCHUR2=1" "MCC_SCHUR2=0" || exit 3
