#!/bin/bash
# rocprofv3 --kernel-trace --stats of bench.py --no-extra under config / env variants, each bounded:
#   tools/repro_prof.sh "config4 MCC_GRAPH=0" "config5 X=1" ...   (prints rc and the first runtime error)
R=$PWD
mkdir -p $R/gpurun_out/repro
cd /tmp && export TMPDIR=/tmp
i=0
for spec in "$@"; do
    i=$((i+1))
    set -- $spec
    cfg=$1; v=$2
    ( export $v; timeout -s KILL 110 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/repro/st$i -o run --output-format csv \
        -- python3 $R/bench.py --config $cfg --steps 20 --warmup 5 --no-cpu --no-parity --no-extra > $R/gpurun_out/repro/b$i.json 2> $R/gpurun_out/repro/b$i.err )
    echo "$spec rc=$?"
    grep -E "aborting|MccError|SIGSEGV" $R/gpurun_out/repro/b$i.err | head -3
done
