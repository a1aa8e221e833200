set -o pipefail
mkdir -p gpurun_out/g3
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/pose_latency.py > gpurun_out/g3/pose.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_pose_gpu.py tests/test_track_gpu.py tests/test_lba_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/g3/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/g3/pytest.log
exit $rc
