#!/bin/bash
# round 4: k_schur norm chunks by wave butterflies: k_schur-path tests, A/B against the previous build
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r04u; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_schur_levels.py tests/test_handoff_poison.py tests/test_gpu_parity.py tests/test_warm_solve.py tests/test_peer_transport.py tests/test_full_size.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -8; [ $rc -eq 0 ] || exit 10
bash tools/ab_trees.sh config4 3 items64 HEAD || exit 12
bash tools/ab_trees.sh config5 2 items64 HEAD || exit 13
bash tools/ab_trees.sh config3 2 items64 HEAD || exit 14
