#!/bin/bash
# One GPU-box measurement pass for a round (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of bench.py      -> per-kernel average durations
#   2. rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE  -> memory-side bytes per launch
#      (separate passes, kernel trace only: no sys/runtime tracing with --pmc)
#   3. tools/pmc_traffic.py                              -> traffic_<config>_<views>.json
#   4. rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 ...       -> fp64_<config>_<views>.json (tools/pmc_fp64.py)
#   5. the default bench.py line (with both files in profiles/ so they are reported)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-r01}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT" "$R/profiles"
cd /tmp && export TMPDIR=/tmp

timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 500 --warmup 50 --no-cpu --no-parity > "$OUT/stats.log" 2>&1 || exit 11
echo "stats pass done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 40 --warmup 4 --no-cpu --no-parity > "$OUT/fetch.log" 2>&1 || exit 12
echo "fetch pass done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 40 --warmup 4 --no-cpu --no-parity > "$OUT/write.log" 2>&1 || exit 13
echo "write pass done"
cd "$R"
ALG=$(python3 -c "import json; print([json.loads(l) for l in open('$OUT/stats.log') if l.startswith('{\"metric')][-1]['roofline']['alg_bytes_per_launch'])") || exit 14
python3 tools/pmc_traffic.py --fetch "$OUT/pmc_fetch" --write "$OUT/pmc_write" --config config2 --views 500 \
    --alg-bytes "$ALG" --out "$OUT/traffic_config2_500.json" > "$OUT/traffic.log" 2>&1 || exit 15
cp "$OUT/traffic_config2_500.json" profiles/ || exit 16
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 -d "$OUT/pmc_fp64" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 40 --warmup 4 --no-cpu --no-parity > "$OUT/fp64.log" 2>&1 || exit 18
echo "fp64 pass done"
cd "$R"
CORNERS=$(python3 -c "import json; print([json.loads(l) for l in open('$OUT/stats.log') if l.startswith('{\"metric')][-1]['config']['corners_per_step'])") || exit 19
python3 tools/pmc_fp64.py --dir "$OUT/pmc_fp64" --config config2 --views 500 --corners "$CORNERS" \
    --out "$OUT/fp64_config2_500.json" > "$OUT/fp64_tool.log" 2>&1 || exit 20
cp "$OUT/fp64_config2_500.json" profiles/ || exit 21
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 17
echo "bench done"
cat "$OUT/bench.json"
