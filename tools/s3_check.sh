#!/bin/bash
# Round-3 session-3 GPU pass: the config4 step tail on the realtime-stamped diagnostic build, then
# bench.py's N = 2 path rehearsed as two ranks on one device (peer transport, strong lines included).
set -o pipefail
OUT=$PWD/gpurun_out/s3_check
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
MCC_DIAG_RT=1 MCC_LIB=multi_camera_calibration_amd/libmcc_diagrt.so timeout -k 10 120 \
    python tools/diag_schur.py config4 > "$OUT/schur4rt.txt" 2>&1 || exit 10
cat "$OUT/schur4rt.txt"
MCC_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 \
    > "$OUT/bench_n2.json" 2> "$OUT/bench_n2.err" || exit 11
python3 -c "
import json; d=json.loads(open('$OUT/bench_n2.json').read().strip().split('\n')[-1])
print('N=2 same device', round(d['ms_per_step']*1e3,2), 'us/step', d['config']['transport'], 'exchange_ms', d.get('exchange_ms'))
print({k: (round(v['ms_per_step']*1e3,2), v.get('transport')) for k, v in d.get('strong', {}).items()})"
exit 0
