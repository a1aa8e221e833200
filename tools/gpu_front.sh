#!/bin/bash
# Front-end iteration on the GPU: octree phase trace, extractor/stereo/pipeline parity tests,
# kernel stats of the extraction bench, the extraction and config-5 bench lines.
# Usage (via gpurun): bash tools/gpu_front.sh TAG -> gpurun_out/TAG/
OUT=gpurun_out/${1:-front}
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
python -c "
from orb_slam2_with_comment_amd import synth
L, R, _ = synth.stereo_pair(synth.KITTI, 3)
open('/tmp/kitti.u8','wb').write(L.tobytes())
"
run trace 60 ./tools/octree_trace /tmp/kitti.u8 376 1241
cat $OUT/trace.log
run pytest_front 400 python -u -m pytest tests/test_extract_gpu.py tests/test_stereo_gpu.py tests/test_pipeline_gpu.py -x -q -rf --timeout 120 --timeout-method thread
tail -3 $OUT/pytest_front.log
run prof 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o x -- python3 bench.py --mode extract --steps 100 --warmup 10 --no-cpu-baseline
python tools/kstats.py $(find $OUT/prof -name "*kernel_trace.csv" | head -1) | head -14
run bench_extract 300 python bench.py --mode extract --no-cpu-baseline
tail -1 $OUT/bench_extract.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('stage_ms_per_step'), d['roofline'])"
run bench_batch 300 python bench.py --mode batch --steps 30 --warmup 4 --no-cpu-baseline
tail -1 $OUT/bench_batch.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d.get('stage_ms_per_launch'), d['roofline'])"
