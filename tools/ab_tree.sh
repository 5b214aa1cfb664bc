#!/bin/bash
# Interleaved A/B of bench.py (ms/step, no profiler) between this tree and an older tree copied under
# build_ab/<name> (its own bench.py, api.py and libmcc.so), plus environment variants of this tree:
#   tools/ab_tree.sh CONFIG ROUNDS OLD_NAME ["VAR=a" ...]
set -o pipefail
CFG=$1; N=$2; OLD=$3; shift 3
mkdir -p gpurun_out/abtree
show() { python3 -c "import json;d=[json.loads(l) for l in open('$1') if l.startswith('{')][-1];print(round(d['ms_per_step']*1e3,2), 'us/step')"; }
for r in $(seq 1 $N); do
    ( cd build_ab/$OLD && timeout -k 10 120 python bench.py --config $CFG --no-cpu --no-parity --no-extra > ../../gpurun_out/abtree/o.json 2>&1 ) || exit 3
    echo "$CFG round $r $OLD: $(show gpurun_out/abtree/o.json)"
    for v in "" "$@"; do
        ( [ -n "$v" ] && export $v; timeout -k 10 120 python bench.py --config $CFG --no-cpu --no-parity --no-extra > gpurun_out/abtree/o.json 2>&1 ) || exit 3
        echo "$CFG round $r HEAD ${v:-default}: $(show gpurun_out/abtree/o.json)"
    done
done
