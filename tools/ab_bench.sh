#!/bin/bash
# A/B timing of an alternative liborbmi build: parity tests of the pose/track kernels with the
# variant, then the default bench alternately on the in-tree build (A) and the variant (B).
# Usage (via gpurun): bash tools/ab_bench.sh tools/ab/liborbmi_X.so TAG
V=$1; TAG=${2:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
ORBMI_LIB=$PWD/$V timeout -k 10 300 python -u -m pytest tests/test_pose_gpu.py tests/test_track_gpu.py tests/test_system_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_variant.log 2>&1 || { tail -20 $OUT/pytest_variant.log; exit 1; }
tail -2 $OUT/pytest_variant.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/A$r.log 2>&1 || exit 2
  ORBMI_LIB=$PWD/$V timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/B$r.log 2>&1 || exit 3
  for x in A B; do python -c "import json,sys;d=json.loads(open('$OUT/$x$r.log').read().strip().splitlines()[-1]);print('$x$r',d['value'],d['roofline']['avg_launch_us'],d['track_only_ms_per_frame_back_to_back'])"; done
done
