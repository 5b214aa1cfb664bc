#!/bin/bash
# A/B the step time of libmcc builds on one bench configuration, interleaved:
#   [ROUNDS=3] [STEPS=200] tools/ab_config.sh CONFIG VIEWS libA.so libB.so ...   (VIEWS 0 = the config's)
CFG=$1; V=$2; shift 2
N=${ROUNDS:-3}; K=${STEPS:-200}
VA=""; [ "$V" != "0" ] && VA="--views $V"
for i in $(seq 1 $N); do
  for L in "$@"; do
    MCC_LIB=$L timeout -k 10 180 python3 bench.py --config $CFG $VA --no-cpu --no-parity --no-extra --steps $K --warmup 20 > gpurun_out/abc.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open('gpurun_out/abc.json')); print(sys.argv[1], sys.argv[2], round(d['ms_per_step']*1000,3), 'us/step')" $CFG $(basename $L)
  done
done
