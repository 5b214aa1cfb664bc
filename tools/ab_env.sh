#!/bin/bash
# Interleaved A/B of one build under environment variants, one config:
#   [ROUNDS=3] [STEPS=2000] tools/ab_env.sh <config> "ENV=1 OTHER=2" "ENV=0" ...   ("-" = no extra env)
CFG=$1; shift
N=${ROUNDS:-3}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for E in "$@"; do
    [ "$E" = "-" ] && EE="" || EE="$E"
    env $EE timeout -k 10 120 python3 bench.py --config $CFG --no-cpu --no-parity --no-extra --steps ${STEPS:-2000} --warmup 100 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[2], sys.argv[1], round(d['ms_per_step']*1000,3), 'us/step', round(d['roofline']['kernel_ms_per_launch']*1000,3))" "$E" $CFG
  done
done
