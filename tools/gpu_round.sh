#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats, PMC traffic passes.
# Usage (via gpurun): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r1}
OUT=gpurun_out/$TAG
mkdir -p $OUT profiles
export TMPDIR=/tmp
python -c "import torch; print(torch.cuda.get_device_name(0))" > $OUT/device.txt 2>&1
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > $OUT/pytest_gpu.log 2>&1
echo "pytest exit $?" >> $OUT/pytest_gpu.log
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof_stats -o stats -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_prof.log 2>&1 || { echo "rocprof stats failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d $OUT/pmc_fetch -o fetch -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -f csv -d $OUT/pmc_write -o write -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $OUT/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
python tools/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write $OUT/traffic.json && cp $OUT/traffic.json profiles/traffic_latest.json
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
