#!/bin/bash
# Full GPU parity suite + a short headline bench (no CPU baseline).
OUT=gpurun_out/${1:-check}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest exit $rc"; tail -4 $OUT/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1
echo "bench exit $?"
tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('phase_ms_per_frame'), d.get('track_only_ms_per_frame_back_to_back'), d['roofline']['avg_launch_us'])"
