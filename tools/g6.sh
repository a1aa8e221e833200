set -o pipefail
mkdir -p gpurun_out/g6
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_bow_gpu.py -x -q -rf --timeout 180 --timeout-method thread > gpurun_out/g6/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-sample-s 2 > gpurun_out/g6/bench_track.log 2>&1
rc=$?
tail -3 gpurun_out/g6/pytest.log
exit $rc
