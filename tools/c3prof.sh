set -o pipefail
mkdir -p gpurun_out/c3p
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/c3p/st -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config config3 --steps 100 --warmup 10 --no-cpu --no-parity --no-extra > $GRAFT_REPO_ROOT/gpurun_out/c3p/b.json 2>&1 || exit 3
f=$(find $GRAFT_REPO_ROOT/gpurun_out/c3p/st -name "*kernel_stats.csv" | head -n 1); cut -c1-120 $f
