set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_handoff_poison.py -x -v --timeout 300 --timeout-method thread 2>&1 | tail -15 || exit 1
