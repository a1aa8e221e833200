"""k_fast2's one-pass FAST stage (csrc/fast_score.h): the packed arc strength S = max(th, A, B)
decides the segment test at every threshold t >= th (S > t) and equals cornerScore<16> + 1 for a
corner, checked on the CPU against a scalar restatement of OpenCV's FAST_t<16> segment test and
cornerScore<16> (tests/cpp/fast_score_check.cpp, 2e6 patches: uniform, near-centre, ties and
arcs).  The GPU side is pinned by the extraction parity tests (test_extract_gpu.py,
test_config5_gpu.py), which compare every keypoint's response with the oracle."""
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not pathlib.Path(HIPCC).exists(), reason="hipcc not available")
def test_arc_strength_equals_segment_test_and_corner_score(tmp_path):
    exe = tmp_path / "fast_score_check"
    subprocess.run([HIPCC, "-O2", "-std=c++17", str(ROOT / "tests" / "cpp" / "fast_score_check.cpp"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=600)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
    assert int(r.stdout.split("corners ")[1].split()[0]) > 100000  # the corner branch is exercised
