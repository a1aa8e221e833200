#!/bin/bash
# LocalBA iteration: parity tests, kernel stats of the LBA bench, the LBA bench line.
OUT=gpurun_out/${1:-lba}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -2 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o x -- python3 bench.py --mode lba --steps 30 --warmup 5 --no-cpu-baseline > $OUT/prof.log 2>&1
echo "prof exit $?"
python tools/kstats.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) k_ba | head -14
timeout -k 10 300 python bench.py --mode lba --steps 50 --warmup 10 --no-cpu-baseline > $OUT/bench.log 2>&1
echo "bench exit $?"; tail -1 $OUT/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
