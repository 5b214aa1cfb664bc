#!/bin/bash
# Round-2 measurement pass (run from the repo root through gpurun; every GPU step has its own limit
# and the script stops at the first failure):
#   calib    FETCH_SIZE / WRITE_SIZE of tools/fetch_calib (known byte counts per access width)
#   <cfg>    for config2 and config3 (bench.py --no-extra): rocprofv3 --kernel-trace --stats,
#            --pmc FETCH_SIZE, --pmc WRITE_SIZE, the FP64 SQ pass -> traffic_/fp64_<cfg>_<views>.json
# Usage: tools/profile_r02.sh <tag> [calib] [config2] [config3]
set -o pipefail
TAG=${1:-r02b}
shift
STEPS=${*:-calib config2 config3}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1

for s in $STEPS; do
    case $s in
    calib)
        [ -x "$R/tools/fetch_calib" ] || { echo "tools/fetch_calib not built"; exit 20; }
        timeout -k 10 60 "$R/tools/fetch_calib" > "$OUT/calib_bytes.json" || exit 21
        ( cd /tmp && export TMPDIR=/tmp &&
          timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/calib_fetch" -o run --output-format csv \
              -- "$R/tools/fetch_calib" > "$OUT/calib_fetch.log" 2>&1 &&
          timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d "$OUT/calib_write" -o run --output-format csv \
              -- "$R/tools/fetch_calib" > "$OUT/calib_write.log" 2>&1 ) || exit 22
        python3 tools/fetch_calib.py --fetch "$OUT/calib_fetch" --write "$OUT/calib_write" --bytes "$OUT/calib_bytes.json" \
            --out "$OUT/fetch_calib.json" > "$OUT/calib.log" 2>&1 || exit 23
        echo "calib done"; cat "$OUT/fetch_calib.json" | grep -E '"(ratio|counter_kib)"|rd_|wr_' | head -40
        ;;
    config2|config3)
        cfg=$s
        if [ $cfg = config2 ]; then ST=500; WU=50; PS=40; VIEWS=500; else ST=100; WU=10; PS=12; VIEWS=5000; fi
        B="$R/bench.py --config $cfg --no-cpu --no-parity --no-extra"
        ( cd /tmp && export TMPDIR=/tmp &&
          timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${cfg}_stats" -o run --output-format csv \
              -- python3 $B --steps $ST --warmup $WU > "$OUT/${cfg}_stats.log" 2>&1 ) || exit 31
        f=$(find "$OUT/${cfg}_stats" -name "*kernel_stats.csv" | head -n 1)
        [ -n "$f" ] && cp "$f" "$OUT/${cfg}_kernel_stats.csv"
        echo "$cfg stats done"; cut -c1-150 "$OUT/${cfg}_kernel_stats.csv"
        ( cd /tmp && export TMPDIR=/tmp &&
          timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/${cfg}_fetch" -o run --output-format csv \
              -- python3 $B --steps $PS --warmup 4 --ramp-seconds 0.05 > "$OUT/${cfg}_fetch.log" 2>&1 &&
          timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/${cfg}_write" -o run --output-format csv \
              -- python3 $B --steps $PS --warmup 4 --ramp-seconds 0.05 > "$OUT/${cfg}_write.log" 2>&1 &&
          timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_FMA_F64 \
              SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 -d "$OUT/${cfg}_fp64" -o run \
              --output-format csv -- python3 $B --steps $PS --warmup 4 --ramp-seconds 0.05 > "$OUT/${cfg}_fp64.log" 2>&1 ) || exit 32
        ALG=$(python3 -c "import json; print([json.loads(l) for l in open('$OUT/${cfg}_stats.log') if l.startswith('{\"metric')][-1]['roofline']['alg_bytes_per_launch'])") || exit 33
        CORNERS=$(python3 -c "import json; print([json.loads(l) for l in open('$OUT/${cfg}_stats.log') if l.startswith('{\"metric')][-1]['config']['corners_per_step'])") || exit 34
        python3 tools/pmc_traffic.py --fetch "$OUT/${cfg}_fetch" --write "$OUT/${cfg}_write" --config $cfg --views $VIEWS \
            --alg-bytes "$ALG" --out "$OUT/traffic_${cfg}_${VIEWS}.json" > "$OUT/${cfg}_traffic.log" 2>&1 || exit 35
        python3 tools/pmc_fp64.py --dir "$OUT/${cfg}_fp64" --config $cfg --views $VIEWS --corners "$CORNERS" \
            --out "$OUT/fp64_${cfg}_${VIEWS}.json" > "$OUT/${cfg}_fp64_tool.log" 2>&1 || exit 36
        echo "$cfg pmc done"; cat "$OUT/${cfg}_fp64_tool.log"
        grep -E '"(bytes_per_launch|ratio_to_alg|step_bytes_per_launch|step_ratio_to_alg)"' "$OUT/traffic_${cfg}_${VIEWS}.json" | head -8
        ;;
    esac
done
exit 0
