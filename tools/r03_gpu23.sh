set -o pipefail
tools/gpu_round.sh r03_full tests bench || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 2
