set -o pipefail
MCC_LIB=build_ab/pair/libmcc.so timeout -k 10 300 python -u -m pytest tests/test_dense_solve.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3 || exit 1
for L in multi_camera_calibration_amd/libmcc.so build_ab/pair/libmcc.so; do
  echo "== $L"; MCC_LIB=$L timeout -k 10 120 python tools/solve_bench.py 48 90 126 | grep "us/solve" || exit 2
done
