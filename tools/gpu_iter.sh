#!/bin/bash
# One development GPU session: parity tests, then the bench lines named on the command line.
# Usage (via gpurun): bash tools/gpu_iter.sh TAG "pytest-args" [bench-args]...
#   each bench-args string is one `python bench.py ...` invocation.
# Stops at the first step that crashes or times out (exit status other than 0/1).
TAG=${1:-iter}; shift
OUT=gpurun_out/$TAG
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
PT=$1; shift
if [ -n "$PT" ]; then
    run pytest 600 python -u -m pytest $PT -v -rf -s --timeout 120 --timeout-method thread
    grep -E "passed|failed|erase flags|config 5" $OUT/pytest.log | tail -20
fi
i=0
for B in "$@"; do
    i=$((i+1))
    run bench$i 400 python bench.py $B
    tail -1 $OUT/bench$i.log
done
