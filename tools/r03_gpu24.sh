set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_cpp_host.py -x -q -k "seam_subclass and config5" --timeout 120 --timeout-method thread 2>&1 | grep -v "^ " | tail -25
exit 0
