#!/bin/bash
# A/B on one box: bench mode $1 with ab/liborbmi_a.so (A) and the in-tree build (B), alternating.
MODE=${1:-lba}; STEPS=${2:-50}; OUT=gpurun_out/ab_$MODE
mkdir -p $OUT
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then export ORBMI_LIB=$PWD/ab/liborbmi_a.so; else unset ORBMI_LIB; fi
    timeout -k 10 200 python bench.py --mode $MODE --steps $STEPS --warmup 10 --no-cpu-baseline > $OUT/$v$r.log 2>&1 || exit $?
    echo "$v$r $(tail -1 $OUT/$v$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
