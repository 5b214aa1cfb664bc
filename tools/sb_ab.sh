set -o pipefail
for m in 36 48 90 126; do
  timeout -k 5 30 tools/solve_bench_old $m > gpurun_out/sb_old_$m.log 2>&1 || exit 11
  timeout -k 5 30 tools/solve_bench $m > gpurun_out/sb_new_$m.log 2>&1 || exit 12
done
for m in 36 48 90 126; do echo "== $m"; tail -1 gpurun_out/sb_old_$m.log; tail -1 gpurun_out/sb_new_$m.log; done
head -3 gpurun_out/sb_old_90.log gpurun_out/sb_new_90.log
