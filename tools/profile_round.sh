#!/bin/bash
# One GPU-box measurement pass for a round (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of bench.py      -> per-kernel average durations
#   2. rocprofv3 --pmc FETCH_SIZE, then --pmc WRITE_SIZE  -> memory-side bytes per launch
#      (separate passes, kernel trace only: no sys/runtime tracing with --pmc)
#   3. tools/pmc_traffic.py                              -> traffic_<config>_<views>.json
#   4. the default bench.py line (with the traffic file in profiles/ so it is reported)
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
timeout -k 10 300 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit 17
echo "bench done"
cat "$OUT/bench.json"
