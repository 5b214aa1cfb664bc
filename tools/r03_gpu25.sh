set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_peer_transport.py -x -v --timeout 300 --timeout-method thread 2>&1 | grep -E "PASS|FAIL|Error|passed|failed" | tail -20 || exit 1
