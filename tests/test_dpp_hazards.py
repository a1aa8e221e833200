"""The MFMA solve's hand-written DPP asm (csrc/lba.hip, csrc/ldl16_steps.inc) is free of the
DPP read-after-write hazard in the code hipcc actually emits (tools/check_dpp_hazards.py), the
LocalBA kernels contain no outlined device-function call, and the generated step file is what
tools/gen_ldl16.py produces.  CPU only: hipcc cross-compiles."""
import importlib.util
import pathlib
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
CSRC = ROOT / "orb_slam2_with_comment_amd" / "csrc"
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_generated_steps_up_to_date(tmp_path, monkeypatch):
    gen = _load("gen_ldl16", ROOT / "tools" / "gen_ldl16.py")
    out = tmp_path / "ldl16_steps.inc"
    monkeypatch.setattr(gen, "OUT", out)
    gen.main()
    assert out.read_text() == (CSRC / "ldl16_steps.inc").read_text(), "run python tools/gen_ldl16.py"


@pytest.mark.skipif(not pathlib.Path(HIPCC).exists(), reason="hipcc not available")
def test_lba_device_code_has_no_dpp_hazard(tmp_path):
    s = tmp_path / "lba.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                    "--cuda-device-only", "-S", str(CSRC / "lba.hip"), "-I", str(ROOT / "include"), "-o", str(s)],
                   check=True, capture_output=True, timeout=600)
    chk = _load("check_dpp_hazards", ROOT / "tools" / "check_dpp_hazards.py")
    text = s.read_text()
    assert "v_fmac_f64_dpp" in text  # the scan sees the hand-written DPP
    assert chk.scan(str(s)) == []
    # no device function outlined into a call (a call frame in k_ba_schur cost it 40 %)
    assert "s_swappc" not in text


def test_checker_flags_unpadded_dpp_source(tmp_path):
    chk = _load("check_dpp_hazards", ROOT / "tools" / "check_dpp_hazards.py")
    bad = tmp_path / "bad.s"
    bad.write_text("k:\n\tv_mov_b64_e32 v[4:5], v[6:7]\n"
                   "\tv_fmac_f64_dpp v[8:9], v[4:5], v[2:3] row_newbcast:1 row_mask:0xf bank_mask:0xf\n")
    good = tmp_path / "good.s"
    good.write_text("k:\n\tv_mov_b64_e32 v[4:5], v[6:7]\n\ts_nop 1\n"
                    "\tv_fmac_f64_dpp v[8:9], v[4:5], v[2:3] row_newbcast:1 row_mask:0xf bank_mask:0xf\n")
    assert len(chk.scan(str(bad))) == 1 and chk.scan(str(good)) == []
