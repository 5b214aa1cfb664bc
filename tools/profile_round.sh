#!/bin/bash
# A round's measurement pass at HEAD (run from the repo root through gpurun; every GPU step has its
# own limit and the script stops at the first failure).  "final" first runs the -m gpu suite, smoke()
# and the default bench line (-> <out>/pytest.log, smoke.log, bench.json).  For each config (bench.py --config <cfg>
# --no-extra): rocprofv3 --kernel-trace --stats, --pmc FETCH_SIZE, --pmc WRITE_SIZE and the FP64 SQ
# pass -> <out>/traffic_<cfg>_<views>.json, fp64_<cfg>_<views>.json, <cfg>_kernel_stats.csv, and the
# SQ pass (tools/pmc_sq.sh: VALU / LDS / SALU issue, waits, wave cycles per kernel) -> <out>/<cfg>_sq.txt
# and sq_<cfg>_<views>.json.  Copy the JSON files into profiles/ for bench.py to report them.
# Graph-launched steps throughout, with HIP's graph packet capture off
# (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0): with it on, rocprofv3's kernel-trace interception crashes
# intermittently inside hipGraphLaunch.
# Usage: tools/profile_round.sh <tag> [final] [config2] [config3] [config4] [config5]
set -o pipefail
TAG=${1:-r05}
shift
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
if [ "$1" = "final" ]; then
    shift
    timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
    rc=$?; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -20; [ $rc -eq 0 ] || exit 10
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 11
    tail -1 $OUT/smoke.log
    timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 12
    tail -c 1500 $OUT/bench.json
fi
STEPS=${*:-config4 config2 config3 config5}
export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0

for cfg in $STEPS; do
    case $cfg in
    config2) ST=500; WU=50; PS=40; VIEWS=500 ;;
    config3) ST=100; WU=10; PS=12; VIEWS=5000 ;;
    config4) ST=300; WU=30; PS=30; VIEWS=1000 ;;
    config5) ST=200; WU=20; PS=20; VIEWS=2000 ;;
    *) echo "unknown config $cfg"; exit 30 ;;
    esac
    B="$R/bench.py --config $cfg --no-cpu --no-parity --no-extra"
    ( cd /tmp && export TMPDIR=/tmp &&
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/${cfg}_stats" -o run --output-format csv \
          -- python3 $B --steps $ST --warmup $WU > "$OUT/${cfg}_stats.log" 2>&1 ) || exit 31
    f=$(find "$OUT/${cfg}_stats" -name "*kernel_stats.csv" | head -n 1)
    [ -n "$f" ] && cp "$f" "$OUT/${cfg}_kernel_stats.csv"
    echo "$cfg stats done"; cut -c1-120 "$OUT/${cfg}_kernel_stats.csv" | grep k_
    # the PMC passes serialise the dispatches, so k_solve's warm-solve helper (a second, resident
    # kernel) could only time out: they run with the direct solve (MCC_WARM=0)
    ( cd /tmp && export TMPDIR=/tmp && export MCC_WARM=0 &&
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
    ( export MCC_WARM=0; bash tools/pmc_sq.sh $cfg "$OUT/${cfg}_sq" "" "$OUT/sq_${cfg}_${VIEWS}.json" $VIEWS \
          > "$OUT/${cfg}_sq.txt" 2>&1 ) || exit 37
    echo "$cfg pmc done"
    python3 -c "
import json; t=json.load(open('$OUT/traffic_${cfg}_${VIEWS}.json')); f=json.load(open('$OUT/fp64_${cfg}_${VIEWS}.json'))
print('  traffic lin', t['bytes_per_launch'], 'ratio', t['ratio_to_alg'], 'step', t['step_bytes_per_launch'], 'step ratio', t['step_ratio_to_alg'])
print('  fp64 flop/corner', f.get('fp64_flops_per_corner'))"
done
exit 0
