#!/bin/bash
# bench step time plus the warm-solve statistics (MCC_SOLVE_STATS=1) per libmcc build, one config:
#   tools/ab_stats.sh <config> libA.so libB.so ...
CFG=$1; shift
mkdir -p gpurun_out
for L in "$@"; do
  MCC_SOLVE_STATS=1 MCC_LIB=$L timeout -k 10 120 python3 bench.py --config $CFG --no-cpu --no-parity --no-extra --steps ${STEPS:-2000} --warmup 100 > gpurun_out/abs.json 2>gpurun_out/abs.err || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/abs.json')); print(sys.argv[1], round(d['ms_per_step']*1000,3), 'us/step', json.dumps(d.get('warm_solve')))" $(basename $(dirname $L))
done
