set -o pipefail
mkdir -p gpurun_out/r03_gpu26
for push in 1 0; do
  MCC_PEER_PUSH=$push MCC_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
     --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 4 --steps 200 --warmup 20 --no-cpu --no-parity \
     > gpurun_out/r03_gpu26/push$push.json 2> gpurun_out/r03_gpu26/push$push.err || { tail -20 gpurun_out/r03_gpu26/push$push.err; exit 1; }
  python3 -c "
import json
d=[json.loads(l) for l in open('gpurun_out/r03_gpu26/push$push.json') if l.startswith('{')][-1]
print('push=$push', 'headline ms', round(d['ms_per_step']*1e3,1), 'us')
for k,v in (d.get('strong') or {}).items(): print('  strong', k, json.dumps(v)[:400])
"
done
