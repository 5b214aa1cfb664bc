#!/bin/bash
# (interleaved A/B trees: tools/mk_ab_tree.sh NAME COMMIT builds build_ab/NAME from an older commit)
# Interleaved bench.py ms/step over several trees under build_ab/<name> and this tree (HEAD):
#   tools/ab_trees.sh CONFIG ROUNDS NAME... [HEAD] ["HEAD:VAR=a ..."]
set -o pipefail
CFG=$1; N=$2; shift 2
mkdir -p gpurun_out/abtree
show() { python3 -c "import json;d=[json.loads(l) for l in open('$1') if l.startswith('{')][-1];print(round(d['ms_per_step']*1e3,2), 'us/step')"; }
for r in $(seq 1 $N); do
    for t in "$@"; do
        case $t in
        HEAD) ( timeout -k 10 120 python bench.py --config $CFG --no-cpu --no-parity --no-extra > gpurun_out/abtree/o.json 2>&1 ) || exit 3 ;;
        HEAD:*) ( export ${t#HEAD:}; timeout -k 10 120 python bench.py --config $CFG --no-cpu --no-parity --no-extra > gpurun_out/abtree/o.json 2>&1 ) || exit 3 ;;
        *) ( cd build_ab/$t && timeout -k 10 120 python bench.py --config $CFG --no-cpu --no-parity --no-extra > ../../gpurun_out/abtree/o.json 2>&1 ) || exit 3 ;;
        esac
        echo "$CFG round $r $t: $(show gpurun_out/abtree/o.json)"
    done
done
