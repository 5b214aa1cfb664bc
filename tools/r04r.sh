#!/bin/bash
# round 4: m <= 30 warm solve on the fused step (config2): tests, A/B
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r04r; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_warm_solve.py tests/test_handoff_poison.py tests/test_gpu_parity.py tests/test_schur_levels.py tests/test_peer_transport.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -8; [ $rc -eq 0 ] || exit 10
bash tools/ab_trees.sh config2 3 r03 olfix HEAD "HEAD:MCC_SMALL_WARM=0" || exit 12
bash tools/ab_trees.sh config4 2 olfix HEAD || exit 13
