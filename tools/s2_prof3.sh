#!/bin/bash
# rocprofv3 kernel trace of config3 with the warm solve on / off (graph-launched, packet capture off)
set -o pipefail
R=$PWD
OUT=$R/gpurun_out/${1:-s2_prof3}
mkdir -p "$OUT"
for w in 1 0; do
    ( cd /tmp && export TMPDIR=/tmp && export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && export MCC_WARM=$w && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/w$w" -o run \
        --output-format csv -- python3 "$R/bench.py" --config config3 --steps 20 --warmup 5 --no-cpu --no-parity --no-extra \
        > "$OUT/prof_w$w.json" 2> "$OUT/prof_w$w.err" ) || exit 13
    f=$(find "$OUT/w$w" -name "*kernel_stats.csv" | head -n 1); cp "$f" "$OUT/kernel_stats_w$w.csv"
    t=$(find "$OUT/w$w" -name "*kernel_trace.csv" | head -n 1); cp "$t" "$OUT/kernel_trace_w$w.csv"
    echo "== warm=$w"; cut -d, -f1-4 "$OUT/kernel_stats_w$w.csv" | grep k_
done
python3 tools/trace_gaps.py "$OUT/kernel_trace_w1.csv" || true
exit 0
