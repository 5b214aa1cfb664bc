set -o pipefail
mkdir -p gpurun_out/r03b
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_peer_transport.py -m gpu -v --timeout 300 --timeout-method thread -k "config5_full" > gpurun_out/r03b/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|x resolution" gpurun_out/r03b/pytest.log | tail -n 10
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
tools/prof_graph_probe.sh r03b/probe "c4cap0 --config config4 --no-extra DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "c4kern0 --config config4 --no-extra HIP_FORCE_DEV_KERNARG=0"
