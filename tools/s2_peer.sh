#!/bin/bash
# peer-transport tests (two / four ranks on one device) and bench.py's N = 2 path rehearsed on one device
set -o pipefail
OUT=$PWD/gpurun_out/${1:-s2_peer}
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_peer_transport.py -m gpu -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?
grep -E "PASS|FAIL|Error" "$OUT/pytest.log" | tail -n 14
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 10
MCC_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 2 --steps 200 --warmup 20 --no-extra > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" || exit 11
python3 -c "import json; d=json.loads(open('$OUT/bench_n2.json').read().strip().split('\n')[-1]); print('N=2 same device', round(d['ms_per_step']*1e3,2), 'us/step', d['config']['transport'], 'exchange_ms', d.get('exchange_ms'))"
exit 0
