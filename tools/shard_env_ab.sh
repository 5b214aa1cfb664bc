#!/bin/bash
# Interleaved A/B of bench.py's shard line under build / environment variants:
#   [ROUNDS=3] tools/shard_env_ab.sh <config> <ranks> "<lib.so> [VAR=value ...]" ...
CFG=$1; W=$2; shift 2
VARIANTS=("$@")
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in "${VARIANTS[@]}"; do
    read -r L EE <<< "$v"
    env $EE MCC_LIB=$L timeout -k 10 200 python3 tools/shard_run.py $CFG $W > gpurun_out/shab.json 2>gpurun_out/shab.err || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/shab.json').read().strip().splitlines()[-1]); print(sys.argv[1], round(d['ms_per_step']*1e3,2), 'us/step')" "$v"
  done
done
