#!/bin/bash
# Front-end A/B on one box: the extractor / config-5 / stereo / pipeline parity tests on the
# in-tree build, then --mode batch and --mode extract alternating ab/liborbmi_a.so (A) and the
# in-tree build (B) (tools/ab_bench.sh).
OUT=gpurun_out/front_ab
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_extract_gpu.py tests/test_config5_gpu.py tests/test_stereo_gpu.py \
    tests/test_pipeline_gpu.py -x -q -rf --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/ab_bench.sh batch 50 || exit $?
bash tools/ab_bench.sh extract 200 || exit $?
for v in A B; do grep -o '"stage_ms_per_[a-z]*": {[^}]*}' gpurun_out/ab_batch/${v}1.log; done
