set -o pipefail
O=gpurun_out/r03d
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -n 12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-parity > $O/bench.json 2> $O/bench.err || exit 11
python - <<'PY'
import json; d=json.load(open('gpurun_out/r03d/bench.json'))
print('headline', round(d['ms_per_step']*1e3,1), 'us', d['roofline']['kernel'], round(d['roofline']['kernel_ms_per_launch']*1e3,1))
for k,v in d.get('configs',{}).items(): print(k, round(v['ms_per_step']*1e3,1),'us', v['roofline']['kernel'], round(v['roofline']['kernel_ms_per_launch']*1e3,1))
PY
tools/prof_graph_probe.sh r03d/probe "c4 --config config4 --no-extra" "c4g0cap0 --config config4 --no-extra MCC_GROUP=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "c4g0 --config config4 --no-extra MCC_GROUP=0"
