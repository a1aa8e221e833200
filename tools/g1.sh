set -o pipefail
mkdir -p gpurun_out/g1
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/pose_latency.py > gpurun_out/g1/pose.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/g1/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/g1/pytest.log
exit $rc
