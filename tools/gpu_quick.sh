#!/bin/bash
# Quick GPU check: parity tests + short bench runs of every mode.  Stops at the first step that
# crashes or times out (exit status other than 0/1).
OUT=gpurun_out/${1:-quick}
mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name exit $rc" | tee -a $OUT/status.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; tail -30 $OUT/$name.log; exit $rc; fi
    return 0
}
run pytest_gpu 600 python -u -m pytest tests -m gpu -v -rf -x --timeout 120 --timeout-method thread
tail -5 $OUT/pytest_gpu.log
run bench_track 400 python bench.py --steps 60 --warmup 8 --cpu-sample-s 6
tail -2 $OUT/bench_track.log
run bench_lba 300 python bench.py --mode lba --steps 30 --warmup 10 --cpu-sample-s 4
tail -2 $OUT/bench_lba.log
run bench_batch 300 python bench.py --mode batch --steps 30 --warmup 4 --cpu-sample-s 4
tail -2 $OUT/bench_batch.log
