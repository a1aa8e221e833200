#!/bin/bash
# One GPU session of round evidence: parity tests, rocprofv3 kernel stats of the default bench,
# two PMC passes (FETCH_SIZE, WRITE_SIZE) for HBM traffic, then the bench lines of every mode.
# Usage (via gpurun): bash tools/gpu_round.sh TAG      -> gpurun_out/TAG/ (summaries under gpurun_out/TAG/profiles/,
# which gpurun merges back; copy them into profiles/TAG/ here)
# Stops at the first step that crashes or times out (exit status other than 0/1).
TAG=${1:-r01}
OUT=gpurun_out/$TAG
P=$OUT/profiles
mkdir -p $OUT $P
export TMPDIR=/tmp
run() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name exit $rc" | tee -a $OUT/status.txt
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; tail -30 $OUT/$name.log; exit $rc; fi
    return 0
}
python -c "import torch; print(torch.cuda.get_device_name(0))" > $OUT/device.txt 2>&1
run pytest_gpu 600 python -u -m pytest tests -m gpu -v -rf --timeout 120 --timeout-method thread
tail -3 $OUT/pytest_gpu.log
cp $OUT/pytest_gpu.log $P/pytest_gpu.log
run prof_stats 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_stats -o stats -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline
run pmc_fetch 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/pmc_fetch -o fetch -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --cpu-sample-s 1
run pmc_write 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/pmc_write -o write -- python3 bench.py --steps 20 --warmup 4 --no-cpu-baseline --cpu-sample-s 1
python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $OUT/traffic.json && cp $OUT/traffic.json $P/traffic.json
find $OUT/prof_stats -name "*kernel_stats.csv" -exec cp {} $P/kernel_stats.csv \;
cp $OUT/prof_stats.log $P/prof_stats_bench.log 2>/dev/null
run bench 400 python bench.py
tail -1 $OUT/bench.log > $P/bench.json; cat $P/bench.json
run bench_lba 300 python bench.py --mode lba --steps 50 --warmup 10
tail -1 $OUT/bench_lba.log > $P/bench_lba.json
run bench_batch 300 python bench.py --mode batch --steps 50 --warmup 4
tail -1 $OUT/bench_batch.log > $P/bench_batch.json
run bench_extract 300 python bench.py --mode extract
tail -1 $OUT/bench_extract.log > $P/bench_extract.json
run bench_system 400 python bench.py --mode system
tail -1 $OUT/bench_system.log > $P/bench_system.json
