#!/bin/bash
# Memory-side traffic (FETCH_SIZE / WRITE_SIZE, separate rocprofv3 passes) and interleaved step
# times of three libmcc builds ab/libmcc_{old,ll,wf2}.so; run from the repo root via gpurun.
set -o pipefail
R=$PWD
ROUNDS=3 bash tools/ab_bench.sh ab/libmcc_old.so ab/libmcc_ll.so ab/libmcc_wf2.so > gpurun_out/ab7.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for L in old ll wf2; do
  MCC_LIB=$R/ab/libmcc_$L.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/tr_$L/f -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 4 --no-cpu --no-parity > $R/gpurun_out/tr_$L.f.log 2>&1 || exit 2
  MCC_LIB=$R/ab/libmcc_$L.so timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/tr_$L/w -o run --output-format csv -- python3 $R/bench.py --steps 40 --warmup 4 --no-cpu --no-parity > $R/gpurun_out/tr_$L.w.log 2>&1 || exit 3
  (cd $R && python3 tools/pmc_traffic.py --fetch gpurun_out/tr_$L/f --write gpurun_out/tr_$L/w --config config2 --views 500 --alg-bytes 4004520 --out gpurun_out/tr_$L.json > gpurun_out/tr_$L.log 2>&1) || exit 4
done
