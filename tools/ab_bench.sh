#!/bin/bash
# A/B the bench step time of libmcc builds on one box, interleaved:
#   [ROUNDS=3] tools/ab_bench.sh libA.so libB.so [libC.so ...]
N=${ROUNDS:-3}
for i in $(seq 1 $N); do
  for L in "$@"; do
    MCC_LIB=$L timeout -k 10 120 python3 bench.py --no-cpu --no-parity --no-extra --steps 2000 --warmup 100 > gpurun_out/ab.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab.json')); print(sys.argv[1], round(d['ms_per_step']*1000,3), 'us/step', round(d['roofline']['kernel_ms_per_launch']*1000,3))" $(basename $L)
  done
done
