#!/bin/bash
# PoseOptimization A/B on one box: the pose/track/native-loop parity tests on the in-tree build,
# then tools/pose_latency.py with ab/liborbmi_a.so (A) and the in-tree build (B), then the
# headline bench alternating A and B (tools/ab_bench.sh).
OUT=gpurun_out/pose_ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_pose_gpu.py tests/test_track_gpu.py tests/test_native_slam_gpu.py \
    -x -q -rf --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
ORBMI_LIB=$PWD/ab/liborbmi_a.so timeout -k 10 120 python tools/pose_latency.py > $OUT/lat_a.log 2>&1 || exit $?
timeout -k 10 120 python tools/pose_latency.py > $OUT/lat_b.log 2>&1 || exit $?
if [ -f ab/liborbmi_c.so ]; then
    ORBMI_LIB=$PWD/ab/liborbmi_c.so timeout -k 10 120 python tools/pose_latency.py > $OUT/lat_c.log 2>&1 || exit $?
fi
grep -E "n_obs|traced" $OUT/lat_*.log
bash tools/ab_bench.sh track 200
