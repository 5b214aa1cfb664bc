#!/bin/bash
# Build a libmcc.so variant with extra compile definitions for A/B runs on the GPU box:
#   tools/build_variant.sh OUT.so -DNAME=VALUE ...
set -e
OUT=$1; shift
D=$(mktemp -d /tmp/mccv.XXXX)
C=multi_camera_calibration_amd/csrc
F="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wall -Wno-unused-function $*"
/opt/rocm/bin/hipcc $F -c $C/mcc_kernels.hip -o $D/k.o &
/opt/rocm/bin/hipcc $F -x hip -c $C/mcc_api.cpp -o $D/a.o &
wait
/opt/rocm/bin/hipcc $F -shared -o "$OUT" $D/k.o $D/a.o multi_camera_calibration_amd/build/mcc_omnicalib.o \
    multi_camera_calibration_amd/build/mcc_omnicalib_api.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$D"
echo "built $OUT ($*)"
