#!/bin/bash
# round 4: k_solve's S^-1 loads ahead of the staging: warm / peer tests, config3 A/B
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r04s; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_warm_solve.py tests/test_peer_transport.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config3 or m48 or m126 or warm or helper or history or delayed or timeout" > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -8; [ $rc -eq 0 ] || exit 10
bash tools/ab_trees.sh config3 3 olfix HEAD || exit 12
