#!/bin/bash
# round 4: packed S^-1 hand-off (helper -> k_solve): warm tests, config3 A/B, k_solve stamps
set -o pipefail
export PYTHONUNBUFFERED=1
OUT=gpurun_out/r04o; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_warm_solve.py tests/test_peer_transport.py -m gpu -x -q --timeout 300 --timeout-method thread -k "not config2 and not config5" > $OUT/pytest.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|Error" $OUT/pytest.log | tail -8; [ $rc -eq 0 ] || exit 10
MCC_LIB=multi_camera_calibration_amd/libmcc_diag.so timeout -k 10 120 python tools/diag_solve.py config3 20 || exit 11
bash tools/ab_trees.sh config3 3 olfix HEAD || exit 12
# bench's N = 2 path as two ranks on ONE device (peer transport): weak config4 line + strong lines
MCC_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r04o/bench_n2.json 2> gpurun_out/r04o/bench_n2.err || exit 13
python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r04o/bench_n2.json') if l.startswith('{')][-1]
print('N=2 same device', round(d['ms_per_step']*1e3,2), 'us/step exchange_ms', d.get('exchange_ms'))
print(json.dumps(d.get('strong'))[:1500])"
for c in config4 config3; do
timeout -k 10 300 python bench.py --config $c --no-cpu --no-parity --no-extra > gpurun_out/r04o/bench_$c.json 2> gpurun_out/r04o/bench_$c.err || exit 14
python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r04o/bench_$c.json') if l.startswith('{')][-1]
r=d['roofline']; print('$c', round(d['ms_per_step']*1e3,2), 'us/step; kernel', r['kernel'], round(r['kernel_ms_per_launch']*1e3,2), 'us frac', round(r['frac'],4), 'step_ms_events', d['roofline'].get('step_ms_events'))"
done
