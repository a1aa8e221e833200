set -o pipefail
mkdir -p gpurun_out/g5
export TMPDIR=/tmp
timeout -k 5 60 ./tools/solve_trace 20 > gpurun_out/g5/solve.log 2>&1 && \
timeout -k 5 60 ./tools/solve_trace 27 >> gpurun_out/g5/solve.log 2>&1 && \
TPT1=1 timeout -k 5 60 ./tools/solve_trace 20 >> gpurun_out/g5/solve.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_lba_gpu.py tests/test_pose_gpu.py -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/g5/pytest.log 2>&1 && \
timeout -k 10 200 python -u bench.py --mode lba --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g5/bench_lba.log 2>&1
rc=$?
tail -3 gpurun_out/g5/pytest.log
exit $rc
