set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_dense_solve.py -x -q --timeout 120 --timeout-method thread || exit 1
timeout -k 10 120 python tools/solve_bench.py 48 90 126 || exit 2
