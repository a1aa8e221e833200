set -o pipefail
mkdir -p gpurun_out/g4
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-sample-s 3 > gpurun_out/g4/bench_track.log 2>&1 && \
timeout -k 10 200 python -u bench.py --mode lba --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/g4/bench_lba.log 2>&1
rc=$?
tail -c 600 gpurun_out/g4/bench_track.log
exit $rc
