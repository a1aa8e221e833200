import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")
    config.addinivalue_line("markers", "slow: longer CPU cases")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle_ctypes as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def kitti_pair():
    from orb_slam2_with_comment_amd import synth
    L, R, _ = synth.stereo_pair(synth.KITTI, 0)
    return L, R


@pytest.fixture(scope="session")
def images():
    """Named parity inputs covering the reference's input space."""
    from orb_slam2_with_comment_amd import synth
    rng = np.random.default_rng(7)
    out = {}
    L, R, _ = synth.stereo_pair(synth.KITTI, 0)
    out["kitti_L0"], out["kitti_R0"] = L, R
    L, R, _ = synth.stereo_pair(synth.KITTI, 11)
    out["kitti_L11"], out["kitti_R11"] = L, R
    out["euroc_0"] = synth.mono(synth.EUROC, 0)
    out["noise_640x480"] = rng.integers(0, 256, (480, 640), dtype=np.uint8)
    grad = np.add.outer(np.arange(300), np.arange(400)).astype(np.float64)
    out["gradient_300x400"] = np.clip(grad * 0.4 + rng.uniform(-3, 3, grad.shape), 0, 255).astype(np.uint8)
    out["flat_240x320"] = np.full((240, 320), 97, np.uint8)
    blocks = rng.integers(0, 256, (24, 33), dtype=np.uint8)
    out["blocks_odd_383x523"] = np.kron(blocks, np.ones((16, 16), np.uint8))[:383, :523].copy()
    return out
