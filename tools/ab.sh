#!/bin/bash
# Interleaved A/B of bench step times on one box (run from the repo root through gpurun).
#   [ROUNDS=3] [STEPS=2000] [WARMUP=100] [STATS=1] tools/ab.sh <config> <variant> [<variant> ...]
# A variant is a space-separated list of VAR=value settings, "lib=<path to libmcc.so>" among them to
# load another build (MCC_LIB), or "-" for the defaults.  STEPS=20 WARMUP=5 is the driver's own
# setting (its first graph launch's host latency is then part of the step).  STATS=1 adds the
# warm-solve statistics (MCC_SOLVE_STATS=1).  Prints "<variant> <config> <us per step> <kernel us per
# launch> [warm_solve]" per run; stops at the first failure.
CFG=$1; shift
N=${ROUNDS:-3}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for V in "$@"; do
    EE=""
    if [ "$V" != "-" ]; then
      for kv in $V; do
        case $kv in
          lib=*) EE="$EE MCC_LIB=${kv#lib=}" ;;
          *) EE="$EE $kv" ;;
        esac
      done
    fi
    [ -n "$STATS" ] && EE="$EE MCC_SOLVE_STATS=1"
    env $EE timeout -k 10 150 python3 bench.py --config $CFG --no-cpu --no-parity --no-extra \
        --steps ${STEPS:-2000} --warmup ${WARMUP:-100} > gpurun_out/ab.json 2>gpurun_out/ab.err || exit 1
    python3 -c "
import json, sys
d = [json.loads(l) for l in open('gpurun_out/ab.json') if l.startswith('{')][-1]
ws = (' ' + json.dumps(d.get('warm_solve'))) if '$STATS' else ''
print(sys.argv[1], sys.argv[2], round(d['ms_per_step'] * 1e3, 3), 'us/step', round(d['roofline']['kernel_ms_per_launch'] * 1e3, 3) , ws)
" "$V" $CFG
  done
done
