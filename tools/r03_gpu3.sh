set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -x > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed|x resolution" $O/pytest.log | tail -n 12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-parity > $O/bench.json 2> $O/bench.err || exit 11
python - <<'PY'
import json; d=json.load(open('gpurun_out/r03c/bench.json'))
print('headline', d['config']['workload'][:40], round(d['ms_per_step']*1e3,1), 'us', d['roofline']['kernel'], round(d['roofline']['kernel_ms_per_launch']*1e3,1))
for k,v in d.get('configs',{}).items(): print(k, round(v['ms_per_step']*1e3,1),'us', v['roofline']['kernel'], round(v['roofline']['kernel_ms_per_launch']*1e3,1))
PY
MCC_GROUP=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu --no-parity > $O/bench_g0.json 2> $O/bench_g0.err || exit 12
python - <<'PY'
import json; d=json.load(open('gpurun_out/r03c/bench_g0.json'))
print('G0 headline', round(d['ms_per_step']*1e3,1), 'us', d['roofline']['kernel'], round(d['roofline']['kernel_ms_per_launch']*1e3,1))
for k,v in d.get('configs',{}).items(): print('G0', k, round(v['ms_per_step']*1e3,1),'us', v['roofline']['kernel'], round(v['roofline']['kernel_ms_per_launch']*1e3,1))
PY
tools/prof_graph_probe.sh r03c/probe "c4cap0 --config config4 --no-extra DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "c4kern0 --config config4 --no-extra HIP_FORCE_DEV_KERNARG=0"
