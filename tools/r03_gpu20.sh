set -o pipefail
for L in multi_camera_calibration_amd/libmcc.so build_ab/idle4/libmcc.so build_ab/t256/libmcc.so build_ab/t1024/libmcc.so; do
  echo "== $L"; MCC_LIB=$L timeout -k 10 120 python tools/solve_bench.py 90 126 | grep "us/solve" || exit 2
done
