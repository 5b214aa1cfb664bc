#!/bin/bash
# One GPU-box pass (run from the repo root through gpurun):
#   1. the -m gpu test suite (every test, failures listed; a crash / timeout stops the script)
#   2. bench.py at the driver's settings (--steps 20 --warmup 5) and at its defaults
#   3. rocprofv3 --kernel-trace --stats of the driver-settings bench, one process per config
# Usage: tools/gpu_round.sh <tag> [tests|bench|prof ...]   (default: all three)
set -o pipefail
TAG=${1:-r03}
shift
STEPS=${*:-tests bench prof}
R=$PWD
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1

ok_rc() {   # test failures (1) are results; anything else (timeout, abort, segfault) stops
    [ "$1" -eq 0 ] || [ "$1" -eq 1 ]
}

for s in $STEPS; do
    case $s in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
            > "$OUT/pytest.log" 2>&1
        rc=$?
        echo "pytest rc=$rc"; tail -n 25 "$OUT/pytest.log"
        ok_rc $rc || exit 10
        ;;
    bench)
        timeout -k 10 400 python bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2> "$OUT/bench_driver.err" || exit 11
        echo "bench (driver settings):"; cut -c1-600 "$OUT/bench_driver.json"
        timeout -k 10 400 python bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || exit 12
        echo "bench (defaults):"; cut -c1-400 "$OUT/bench_default.json"
        ;;
    prof)
        # one process per config (--no-extra), graph-launched, with HIP's graph packet capture off:
        # with it on, rocprofv3's kernel-trace interception crashes intermittently inside
        # hipGraphLaunch; tools/profile_r03.sh adds the PMC passes
        for cfg in config4 config2 config3 config5; do
            ( cd /tmp && export TMPDIR=/tmp && export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/stats_$cfg" -o run \
                --output-format csv -- python3 "$R/bench.py" --config $cfg --steps 20 --warmup 5 --no-cpu --no-parity --no-extra \
                > "$OUT/prof_$cfg.json" 2> "$OUT/prof_$cfg.err" ) || exit 13
            f=$(find "$OUT/stats_$cfg" -name "*kernel_stats.csv" | head -n 1)
            [ -n "$f" ] && cp "$f" "$OUT/kernel_stats_$cfg.csv" && echo "== $cfg" && cut -c1-120 "$OUT/kernel_stats_$cfg.csv" | grep k_
        done
        ;;
    esac
done
exit 0
