"""The oracle reproduces the committed golden fixtures (tests/golden/make_golden.py)."""
import hashlib
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def test_kitti_extract_golden(oracle):
    g = _load("kitti_stereo_f0.npz")
    p = oracle.params(2000)
    for side in ("left", "right"):
        k, d = oracle.extract(p, g[side])
        np.testing.assert_array_equal(k, g["kps_" + side])
        np.testing.assert_array_equal(d, g["desc_" + side])


def test_kitti_stereo_golden(oracle):
    g = _load("kitti_stereo_f0.npz")
    p = oracle.params(2000)
    u, d = oracle.stereo(p, g["left"], g["right"], float(g["bf"]), float(g["fx"]), g["kps_left"],
                         g["desc_left"], g["kps_right"], g["desc_right"])
    np.testing.assert_array_equal(u, g["u_right"])
    np.testing.assert_array_equal(d, g["depth"])
    assert (d > 0).sum() > 500


def test_crop_levels4_golden(oracle):
    g = _load("crop_283x397_l4.npz")
    k, d = oracle.extract(oracle.params(500, 1.2, 4, 20, 7), g["image"])
    np.testing.assert_array_equal(k, g["kps"])
    np.testing.assert_array_equal(d, g["desc"])


@pytest.mark.slow
def test_euroc5000_digest(oracle):
    g = _load("euroc_f0_digest.npz")
    k, d = oracle.extract(oracle.params(5000), g["image"])
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(k).tobytes())
    h.update(np.ascontiguousarray(d).tobytes())
    assert h.hexdigest() == bytes(g["sha256"]).decode()
    assert len(k) == int(g["n"])


def test_extract_invariants(oracle):
    g = _load("kitti_stereo_f0.npz")
    k = g["kps_left"]
    t = oracle.tables(oracle.params(2000))
    W, H = oracle.level_sizes(oracle.params(2000), 376, 1241)
    assert np.all(np.diff(k["octave"]) >= 0)  # level-major
    for l in range(8):
        kl = k[k["octave"] == l]
        n = t["features_per_level"][l]
        assert n <= len(kl) <= n + 3  # DistributeOctTree stops at >= N, one split adds <= 3
        x = np.rint(kl["x"] / t["scale"][l])
        y = np.rint(kl["y"] / t["scale"][l])
        assert x.min() >= 19 and x.max() < W[l] - 19
        assert y.min() >= 19 and y.max() < H[l] - 19
        assert np.all(kl["size"] == np.float32(int(31 * t["scale"][l])))
    assert np.all((k["angle"] >= 0) & (k["angle"] < 360))
    assert np.all(k["class_id"] == -1)
    assert np.all(k["response"] >= 7)
