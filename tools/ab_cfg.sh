#!/bin/bash
# Interleaved A/B of bench step times for several libmcc builds on one box, one config:
#   [ROUNDS=3] [STEPS=2000] tools/ab_cfg.sh <config> libA.so libB.so ...
# prints "<lib dir> <us per step> <kernel us per launch>" per run; stops at the first failure
CFG=$1; shift
N=${ROUNDS:-3}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for L in "$@"; do
    MCC_LIB=$L timeout -k 10 120 python3 bench.py --config $CFG --no-cpu --no-parity --no-extra --steps ${STEPS:-2000} --warmup 100 > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[2], sys.argv[1], round(d['ms_per_step']*1000,3), 'us/step', round(d['roofline']['kernel_ms_per_launch']*1000,3))" $(basename $(dirname $L)) $CFG
  done
done
