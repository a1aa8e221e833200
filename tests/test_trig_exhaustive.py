"""The rBRIEF rotation's cos/sin (csrc/trig_f64.h, used by k_describe) against the pinned
semantics P6, (float)cos((double)a) / (float)sin((double)a) with glibc, for EVERY float angle in
[0, 2*pi] that IC_Angle can produce (tools/trig_check.c; ~1.1e9 values, a few seconds on 8 cores)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sincos_f64_matches_glibc_on_every_float_angle(tmp_path):
    exe = str(tmp_path / "trig_check")
    subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-I",
                    os.path.join(ROOT, "orb_slam2_with_comment_amd", "csrc"),
                    os.path.join(ROOT, "tools", "trig_check.c"), "-lm", "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout
    assert ": 0 mismatches" in out.stdout, out.stdout
