#!/bin/bash
# round 4: k_group's own hand-off (group tail): parity / poison / peer subset, config4 A/B, tail stamps
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r04i; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_schur_levels.py tests/test_gpu_parity.py tests/test_handoff_poison.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -15; [ $rc -le 1 ] || exit 10; [ $rc -eq 0 ] || exit 11
timeout -k 10 600 python -u -m pytest tests/test_peer_transport.py -m gpu -x -q --timeout 300 --timeout-method thread -k "config4 or config2" > $OUT/peer.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $OUT/peer.log | tail -15; [ $rc -eq 0 ] || exit 12
bash tools/ab_trees.sh config4 3 r03 olfix HEAD "HEAD:MCC_GROUP_TAIL=0" || exit 13
