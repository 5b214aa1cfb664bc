#!/bin/bash
# Build an A/B tree of an older commit under build_ab/NAME (bench.py + its package + libmcc.so):
#   tools/mk_ab_tree.sh NAME COMMIT
set -e
NAME=$1; C=$2; W=/tmp/abw/$NAME
rm -rf $W build_ab/$NAME; mkdir -p $W build_ab/$NAME/multi_camera_calibration_amd
git archive $C | tar -x -C $W
make -s --no-print-directory -C $W/multi_camera_calibration_amd -j8 libmcc.so
cp -r $W/bench.py $W/include $W/oracle $W/profiles build_ab/$NAME/
cp $W/multi_camera_calibration_amd/*.py $W/multi_camera_calibration_amd/libmcc.so build_ab/$NAME/multi_camera_calibration_amd/
rm -rf build_ab/$NAME/profiles/r0*
