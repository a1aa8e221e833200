#!/bin/bash
# Parity tests of the tracking chain, then the default bench twice (no CPU baseline).
# Usage (via gpurun): bash tools/gpu_quick_bench.sh TAG [pytest files...]
TAG=${1:-quick}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
T=${@:-tests/test_matcher_gpu.py tests/test_track_gpu.py tests/test_pipeline_gpu.py tests/test_pose_gpu.py tests/test_system_gpu.py}
timeout -k 10 400 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench$r.log 2>&1 || { tail -20 $OUT/bench$r.log; exit 2; }
  python -c "import json;d=json.loads(open('$OUT/bench$r.log').read().strip().splitlines()[-1]);print('bench$r',d['value'],d['roofline']['avg_launch_us'],d['track_only_ms_per_frame_back_to_back'],d['phase_ms_per_frame'])"
done
