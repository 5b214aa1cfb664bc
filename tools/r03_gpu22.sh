set -o pipefail
timeout -k 10 120 python tools/solve_bench.py 90 || exit 2
