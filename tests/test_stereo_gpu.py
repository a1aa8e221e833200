"""GPU parity: Frame::ComputeStereoMatches on MI355X vs the CPU restatement (bit-exact)."""
import os

import numpy as np
import pytest

from orb_slam2_with_comment_amd import synth

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _pair(orb, p):
    mk = lambda: orb.ORBextractor(p.nfeatures, p.scale_factor, p.nlevels, p.ini_th_fast, p.min_th_fast)
    return mk(), mk()


@pytest.mark.parametrize("frame", [0, 5, 23])
def test_stereo_parity(oracle, frame):
    import orb_slam2_with_comment_amd as orb
    p = oracle.params(2000)
    exL, exR = _pair(orb, p)
    L, R, _ = synth.stereo_pair(synth.KITTI, frame)
    kl, dl = exL(L)
    kr, dr = exR(R)
    u, d = orb.compute_stereo_matches(exL, exR, synth.KITTI.bf, synth.KITTI.fx, len(kl))
    u_ref, d_ref = oracle.stereo(p, L, R, synth.KITTI.bf, synth.KITTI.fx, kl, dl, kr, dr)
    bad = np.nonzero((u != u_ref) | (d != d_ref))[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first {bad[:5]}: gpu {u[bad[:3]]} ref {u_ref[bad[:3]]}"
    assert (d > 0).sum() > 300


def test_stereo_golden(oracle):
    import orb_slam2_with_comment_amd as orb
    g = np.load(os.path.join(GOLD, "kitti_stereo_f0.npz"), allow_pickle=False)
    exL, exR = _pair(orb, oracle.params(2000))
    kl, _ = exL(g["left"])
    exR(g["right"])
    u, d = orb.compute_stereo_matches(exL, exR, float(g["bf"]), float(g["fx"]), len(kl))
    np.testing.assert_array_equal(u, g["u_right"])
    np.testing.assert_array_equal(d, g["depth"])


def test_stereo_no_matches(oracle):
    """Right image unrelated to the left: few/no matches; empty-median case defined."""
    import orb_slam2_with_comment_amd as orb
    p = oracle.params(2000)
    exL, exR = _pair(orb, p)
    L, _, _ = synth.stereo_pair(synth.KITTI, 0)
    R = np.full_like(L, 128)
    R[::7, ::5] = 255
    kl, dl = exL(L)
    kr, dr = exR(R)
    u, d = orb.compute_stereo_matches(exL, exR, synth.KITTI.bf, synth.KITTI.fx, len(kl))
    if dr is None:
        kr, dr = kr[:0], np.zeros((0, 32), np.uint8)
    u_ref, d_ref = oracle.stereo(p, L, R, synth.KITTI.bf, synth.KITTI.fx, kl, dl, kr, dr)
    np.testing.assert_array_equal(u, u_ref)
    np.testing.assert_array_equal(d, d_ref)
