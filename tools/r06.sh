#!/bin/bash
# Round-6 GPU passes (one gpurun call each; every GPU step has its own limit and the script stops at
# the first failure).  Usage: tools/r06.sh <tag> <step> [<step> ...], steps:
#   tests:<pytest args, comma-separated>   e.g. tests:tests/test_warm_solve.py
#   ab:<config>:<steps>                    new build against build_ab/r05head (the round-start library)
#   opt                                    bench.py --optimize-only (the real optimizeExtrinsics key)
#   prof:<config>                          tools/profile_round.sh passes for one config
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
n=0
for s in "$@"; do
  case $s in
    tests:*)
      args=${s#tests:}; args=${args//,/ }
      n=$((n + 1))
      timeout -k 10 1100 python -u -m pytest $args -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest$n.log 2>&1
      rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest$n.log | tail -10; [ $rc -eq 0 ] || exit 10 ;;
    ab:*)
      IFS=: read -r _ cfg st <<< "$s"
      WU=100; [ "$st" -le 50 ] && WU=5
      ROUNDS=${ROUNDS:-3} STEPS=$st WARMUP=$WU tools/ab.sh $cfg "lib=build_ab/r05head/libmcc.so" "-" | tee -a $OUT/ab.txt || exit 11 ;;
    opt)
      timeout -k 10 300 python bench.py --optimize-only > $OUT/opt.json 2> $OUT/opt.err || exit 12
      python3 -c "
import json; d=json.load(open('$OUT/opt.json'))['optimize']
for k,v in d.items(): print(k, v['iterations'], 'iters; wall', round(v['wall_ms_per_call'],3), 'ms; device', round(v['device_ms_per_call'],3), 'ms,', round(v['device_ms_per_iteration']*1e3,1), 'us/iter; host', {a: round(b,3) for a,b in v['host_ms'].items()}, v['solves_per_call'], 'by count', [round(x*1e3,1) for x in v['device_ms_by_count']['device_ms']])
" ;;
    prof:*)
      bash tools/profile_round.sh $TAG ${s#prof:} > $OUT/prof_${s#prof:}.log 2>&1 || { tail -5 $OUT/prof_${s#prof:}.log; exit 13; }
      tail -8 $OUT/prof_${s#prof:}.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
