"""Settings files (cv::FileStorage YAML) and the values Tracking derives from them
(src/Tracking.cc:53-143).  CPU only."""
import os

import numpy as np
import pytest

from orb_slam2_with_comment_amd import synth
from orb_slam2_with_comment_amd.settings import load_settings, read_file_storage, write_settings

_TUM_LIKE = """%YAML:1.0

# comment line
Camera.fx: 517.306408
Camera.fy: 516.469215
Camera.cx: 318.643040
Camera.cy: 255.313989

Camera.k1: 0.262383
Camera.k2: -0.953104
Camera.p1: -0.005358
Camera.p2: 0.002628
Camera.k3: 1.163314

Camera.width: 640
Camera.height: 480
Camera.fps: 0.0
Camera.bf: 40.0
Camera.RGB: 1
ThDepth: 40.0
DepthMapFactor: 5000.0
ORBextractor.nFeatures: 1000
ORBextractor.scaleFactor: 1.2
ORBextractor.nLevels: 8
ORBextractor.iniThFAST: 20
ORBextractor.minThFAST: 7
Viewer.PointSize:2
LEFT.D: !!opencv-matrix
   rows: 1
   cols: 5
   dt: d
   data:[-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05, 0.0]
LEFT.K: !!opencv-matrix
   rows: 3
   cols: 3
   dt: d
   data: [458.654, 0.0, 367.215,
          0.0, 457.296, 248.375, 0.0, 0.0, 1.0]
"""


def test_file_storage_parser(tmp_path):
    p = tmp_path / "s.yaml"
    p.write_text(_TUM_LIKE)
    fs = read_file_storage(str(p))
    assert fs["Viewer.PointSize"] == 2                     # `Key:value` without a space
    assert fs["ORBextractor.nFeatures"] == 1000 and isinstance(fs["ORBextractor.nFeatures"], int)
    np.testing.assert_allclose(fs["LEFT.D"], [[-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05, 0.0]])
    assert fs["LEFT.K"].shape == (3, 3) and fs["LEFT.K"][1, 2] == 248.375   # data spanning lines
    with pytest.raises(ValueError):
        bad = tmp_path / "b.yaml"
        bad.write_text("Camera.fx: 1\n")
        read_file_storage(str(bad))


def test_tracking_derived_values(tmp_path):
    p = tmp_path / "s.yaml"
    p.write_text(_TUM_LIKE)
    s = load_settings(str(p))
    assert s.fps == 30 and s.max_frames == 30 and s.min_frames == 0          # fps 0 -> 30 (:79-80)
    assert len(s.dist_coef) == 5 and s.dist_coef[4] == np.float32(1.163314)  # k3 != 0 (:70-74)
    assert s.th_depth == np.float32(np.float32(np.float32(40.0) * np.float32(40.0)) / np.float32(517.306408))
    assert s.depth_map_factor == np.float32(np.float32(1.0) / np.float32(5000.0))  # (:143-147)
    assert s.K[0, 0] == np.float32(517.306408) and s.K[1, 2] == np.float32(255.313989) and s.K[2, 2] == 1
    assert s.rgb and s.n_levels == 8 and s.scale_factor == np.float32(1.2)


def test_missing_keys_read_as_zero(tmp_path):
    p = tmp_path / "m.yaml"
    p.write_text("%YAML:1.0\nCamera.fx: 500\nCamera.fps: 20\n")
    s = load_settings(str(p))
    assert s.bf == 0 and s.th_depth == 0 and len(s.dist_coef) == 4 and s.max_frames == 20
    assert s.depth_map_factor == 1 and s.n_features == 0


def test_write_then_load_kitti_synthetic(tmp_path):
    path = tmp_path / "k.yaml"
    write_settings(str(path), synth.KITTI)
    s = load_settings(str(path))
    for f in ("width", "height", "fx", "fy", "cx", "cy", "bf"):   # float32 like the reference's reads
        assert np.float32(getattr(s.camera, f)) == np.float32(getattr(synth.KITTI, f))
    assert s.max_frames == 10 and s.n_features == 2000
    # KITTI00-02.yaml: mThDepth = 386.1448 * 35 / 718.856 (src/Tracking.cc:136)
    assert abs(float(s.th_depth) - 386.1448 * 35 / 718.856) < 1e-4


@pytest.mark.skipif(not os.path.isdir("/root/reference/Examples"), reason="reference tree not present")
@pytest.mark.parametrize("rel,nfeat,fps", [("Examples/Stereo/KITTI00-02.yaml", 2000, 10),
                                           ("Examples/Stereo/EuRoC.yaml", 1200, 20),
                                           ("Examples/RGB-D/TUM1.yaml", 1000, 30)])
def test_reference_settings_files(rel, nfeat, fps):
    """The reference's own settings files (read as data) parse with the values they state."""
    s = load_settings(os.path.join("/root/reference", rel))
    assert s.n_features == nfeat and s.max_frames == fps and s.n_levels == 8
    assert s.ini_th_fast == 20 and s.min_th_fast == 7
