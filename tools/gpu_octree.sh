#!/bin/bash
# octree phase trace on a KITTI-shaped frame + the extractor/stereo/pipeline parity tests
set -e
python -c "
from orb_slam2_with_comment_amd import synth
L, R, _ = synth.stereo_pair(synth.KITTI, 3)
open('/tmp/kitti.u8','wb').write(L.tobytes())
"
timeout -k 5 60 ./tools/octree_trace /tmp/kitti.u8 376 1241
timeout -k 5 300 python -u -m pytest tests/test_extract_gpu.py tests/test_stereo_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -4
