set -o pipefail
mkdir -p gpurun_out/r03a
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03a/pytest.log | tail -n 30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r03a/bench.json 2> gpurun_out/r03a/bench.err || exit 11
cut -c1-1500 gpurun_out/r03a/bench.json
tools/prof_graph_probe.sh r03a/probe "c4g1 --config config4 --no-extra MCC_GRAPH_SIZES=1" "c4g3 --config config4 --no-extra MCC_GRAPH_SIZES=3" "c4all --config config4 --no-extra"
