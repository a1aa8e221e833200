"""GPU parity: ORBextractor on MI355X (liborbmi.so, C ABI) vs the pinned CPU restatement.

Bit-exact on every keypoint field and descriptor byte (BASELINE.json north_star), plus
stage-level parity (pyramid, FAST candidates, octree) so a mismatch is localised."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def orb():
    import orb_slam2_with_comment_amd as m
    return m


def _extractor(orb, p):
    return orb.ORBextractor(p.nfeatures, p.scale_factor, p.nlevels, p.ini_th_fast, p.min_th_fast)


def _stage_report(oracle, p, ex, img):
    """Localise the first diverging stage (pyramid -> FAST -> octree)."""
    import ctypes as C
    from orb_slam2_with_comment_amd import _capi
    msgs = []
    opyr = oracle.pyramid(p, img)
    for l in range(p.nlevels):
        g = ex.pyramid_level(l, padded=True)
        if not np.array_equal(g, opyr[l]):
            bad = np.argwhere(g != opyr[l])
            msgs.append(f"pyramid level {l}: {len(bad)} px differ, first {bad[:3].tolist()}")
            return msgs
    for l in range(p.nlevels):
        ref = oracle.fast_level(p, img, l)
        cap = len(ref) + 4096
        buf = np.zeros((cap, 3), np.int32)
        n = C.c_int()
        _capi.check("dbg", _capi.lib().orbmi_debug_fast_candidates(ex.handle, 0, l, _capi.ptr(buf), cap, C.byref(n)))
        got = buf[:n.value]
        if not np.array_equal(got, ref):
            msgs.append(f"FAST level {l}: gpu {len(got)} vs oracle {len(ref)}")
            return msgs
        ref = oracle.octree_level(p, img, l)
        n = C.c_int()
        _capi.check("dbg", _capi.lib().orbmi_debug_octree_level(ex.handle, 0, l, _capi.ptr(buf), cap, C.byref(n)))
        got = buf[:n.value]
        if not np.array_equal(got, ref):
            msgs.append(f"octree level {l}: gpu {len(got)} vs oracle {len(ref)}; "
                        f"set-equal={set(map(tuple, got.tolist())) == set(map(tuple, ref.tolist()))}")
            return msgs
    msgs.append("stages equal: divergence in orientation/descriptor")
    return msgs


def _assert_same(oracle, p, ex, img, k_gpu, d_gpu):
    k_ref, d_ref = oracle.extract(p, img)
    if len(k_gpu) != len(k_ref) or not np.array_equal(k_gpu, k_ref) or not np.array_equal(d_gpu, d_ref):
        rep = _stage_report(oracle, p, ex, img)
        n = min(len(k_gpu), len(k_ref))
        bad_k = np.nonzero(k_gpu[:n] != k_ref[:n])[0]
        bad_d = np.nonzero((d_gpu[:n] != d_ref[:n]).any(1))[0] if n else []
        pytest.fail(f"n gpu={len(k_gpu)} oracle={len(k_ref)}; kp mismatches {len(bad_k)} (first {bad_k[:5]}), "
                    f"desc mismatches {len(bad_d)} (first {list(bad_d[:5])}); {rep}")


@pytest.mark.parametrize("name", ["kitti_L0", "kitti_R0", "kitti_L11", "euroc_0", "noise_640x480",
                                  "gradient_300x400", "blocks_odd_383x523"])
def test_extract_parity(orb, oracle, images, name):
    p = oracle.params(2000)
    ex = _extractor(orb, p)
    img = images[name]
    k, d = ex(img)
    if d is None:
        d = np.zeros((0, 32), np.uint8)
    _assert_same(oracle, p, ex, img, k, d)


def _low_contrast():
    """A 480x640 texture of +-12 grey levels (FAST corners at 7, rarely at 20: most cells fall back
    to min_th) with a few high-contrast blocks (cells that keep ini_th's corners)."""
    rng = np.random.default_rng(11)
    img = (116 + rng.integers(0, 25, (480, 640))).astype(np.uint8)
    for y, x in [(60, 80), (200, 330), (350, 500), (400, 90)]:
        img[y:y + 24, x:x + 40] = rng.integers(0, 256, (24, 40))
    return img


# FAST at ini_th first and at min_th only for a cell without a survivor (k_fast2): both orders of
# the thresholds, equal ones, and an image where most cells take the fallback
@pytest.mark.parametrize("ini,mn", [(20, 7), (7, 20), (12, 12), (45, 5)])
@pytest.mark.parametrize("name", ["low_contrast", "kitti_L0"])
def test_extract_parity_thresholds(orb, oracle, images, name, ini, mn):
    img = _low_contrast() if name == "low_contrast" else images[name]
    p = oracle.params(2000, 1.2, 8, ini, mn)
    ex = _extractor(orb, p)
    k, d = ex(img)
    if d is None:
        d = np.zeros((0, 32), np.uint8)
    _assert_same(oracle, p, ex, img, k, d)


def test_extract_parity_5000_euroc(orb, oracle, images):
    p = oracle.params(5000)
    ex = _extractor(orb, p)
    k, d = ex(images["euroc_0"])
    _assert_same(oracle, p, ex, images["euroc_0"], k, d)


def test_extract_parity_levels4_crop(orb, oracle):
    g = np.load(os.path.join(GOLD, "crop_283x397_l4.npz"), allow_pickle=False)
    p = oracle.params(500, 1.2, 4, 20, 7)
    ex = _extractor(orb, p)
    k, d = ex(g["image"])
    np.testing.assert_array_equal(k, g["kps"])
    np.testing.assert_array_equal(d, g["desc"])


def test_extract_golden_kitti(orb, oracle):
    g = np.load(os.path.join(GOLD, "kitti_stereo_f0.npz"), allow_pickle=False)
    ex = _extractor(orb, oracle.params(2000))
    for side in ("left", "right"):
        k, d = ex(g[side])
        np.testing.assert_array_equal(k, g["kps_" + side])
        np.testing.assert_array_equal(d, g["desc_" + side])


def test_flat_image_no_keypoints(orb, oracle, images):
    ex = _extractor(orb, oracle.params(2000))
    k, d = ex(images["flat_240x320"])
    assert len(k) == 0 and d is None  # descriptors.release() (src/ORBextractor.cc:1063-1064)


def test_empty_image_returns(orb, oracle):
    ex = _extractor(orb, oracle.params(2000))
    k, d = ex(np.zeros((0, 0), np.uint8))
    assert len(k) == 0 and d is None


def test_too_small_image_unsupported(orb, oracle):
    from orb_slam2_with_comment_amd._capi import OrbmiError, ORBMI_E_UNSUPPORTED
    ex = _extractor(orb, oracle.params(2000))
    with pytest.raises(OrbmiError) as e:
        ex(np.zeros((120, 160), np.uint8))
    assert e.value.code == ORBMI_E_UNSUPPORTED


def test_pyramid_parity(orb, oracle, images):
    p = oracle.params(2000)
    ex = _extractor(orb, p)
    img = images["kitti_L0"]
    ex(img)
    ref = oracle.pyramid(p, img)
    for l in range(8):
        np.testing.assert_array_equal(ex.pyramid_level(l, padded=True), ref[l])
        np.testing.assert_array_equal(ex.pyramid_level(l), ref[l][19:-19, 19:-19])


def test_getters(orb, oracle):
    p = oracle.params(2000)
    ex = _extractor(orb, p)
    t = oracle.tables(p)
    assert ex.GetLevels() == 8
    assert ex.GetScaleFactor() == np.float32(1.2)
    np.testing.assert_array_equal(ex.GetScaleFactors(), t["scale"])
    np.testing.assert_array_equal(ex.GetInverseScaleFactors(), t["inv_scale"])
    np.testing.assert_array_equal(ex.GetScaleSigmaSquares(), t["sigma2"])
    np.testing.assert_array_equal(ex.GetInverseScaleSigmaSquares(), t["inv_sigma2"])
    np.testing.assert_array_equal(ex.features_per_level(), t["features_per_level"])


def test_repeat_and_resize_reuse_handle(orb, oracle, images):
    """One handle across image sizes and repeated calls (geometry re-planning)."""
    p = oracle.params(1000)
    ex = _extractor(orb, p)
    for name in ("kitti_L0", "euroc_0", "kitti_L0"):
        k, d = ex(images[name])
        k2, d2 = oracle.extract(p, images[name])
        np.testing.assert_array_equal(k, k2)
        np.testing.assert_array_equal(d, d2)


def test_batch_device_matches_host_api(orb, oracle, images):
    """orbmi_extract_batch_device over 4 images == per-image results."""
    import ctypes as C
    import torch
    from orb_slam2_with_comment_amd import _capi
    p = oracle.params(2000)
    ex = _extractor(orb, p)
    names = ["kitti_L0", "kitti_R0", "kitti_L11", "kitti_R11"]
    imgs = np.stack([images[n] for n in names])
    d_img = torch.from_numpy(imgs).cuda()
    cap = 2100
    d_k = torch.zeros((4, cap, 7), dtype=torch.int32, device="cuda")
    d_d = torch.zeros((4, cap, 32), dtype=torch.uint8, device="cuda")
    d_n = torch.zeros(4, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _capi.check("batch", _capi.lib().orbmi_extract_batch_device(
        ex.handle, C.c_void_p(d_img.data_ptr()), 4, 376, 1241, 1241, 376 * 1241,
        C.c_void_p(d_k.data_ptr()), C.c_void_p(d_d.data_ptr()), C.c_void_p(d_n.data_ptr()), cap))
    _capi.check("sync", _capi.lib().orbmi_extractor_synchronize(ex.handle))
    counts = d_n.cpu().numpy()
    kk = d_k.cpu().numpy()
    dd = d_d.cpu().numpy()
    for i, n in enumerate(names):
        k_ref, d_ref = oracle.extract(p, images[n])
        assert counts[i] == len(k_ref)
        np.testing.assert_array_equal(kk[i, :counts[i]].view(_capi.KP_DTYPE).reshape(-1), k_ref)
        np.testing.assert_array_equal(dd[i, :counts[i]], d_ref)


@pytest.mark.parametrize("pinned", [True, False])
def test_batch_host_images(orb, oracle, images, pinned):
    """orbmi_extract_batch_host: the images in host memory -- pinned (read in place by the copy
    kernel on the handle's stream) or pageable (staged through the handle's pinned buffers) --
    give the oracle's keypoints and descriptors, call after call on one handle (a pageable
    buffer is reusable as soon as the call returns), and at an odd image size whose bytes are not a
    multiple of 16 (the copy's byte tail)."""
    import ctypes as C
    import torch
    from orb_slam2_with_comment_amd import _capi, _hip
    p = oracle.params(2000)
    ex = _extractor(orb, p)
    cap = 2100
    for names, (r, c) in ((["kitti_L0", "kitti_R0"], (376, 1241)), (["kitti_L11", "kitti_R11"], (376, 1241)),
                          (["kitti_L0", "kitti_R11"], (371, 1237))):
        imgs = np.stack([np.ascontiguousarray(images[n][:r, :c]) for n in names])
        if pinned:
            buf = _hip.PinnedBytes(imgs.nbytes)
            buf.array[:] = imgs.reshape(-1)
            ptr = buf.ptr
        else:
            buf = imgs.copy()
            ptr = buf.ctypes.data
        d_k = torch.zeros((2, cap, 7), dtype=torch.int32, device="cuda")
        d_d = torch.zeros((2, cap, 32), dtype=torch.uint8, device="cuda")
        d_n = torch.zeros(2, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        _capi.check("batch_host", _capi.lib().orbmi_extract_batch_host(
            ex.handle, C.c_void_p(ptr), 2, r, c, r * c, C.c_void_p(d_k.data_ptr()), C.c_void_p(d_d.data_ptr()),
            C.c_void_p(d_n.data_ptr()), cap))
        if not pinned:
            buf[:] = 0  # pageable input: staged during the call, free to reuse at once
        _capi.check("sync", _capi.lib().orbmi_extractor_synchronize(ex.handle))
        counts, kk, dd = d_n.cpu().numpy(), d_k.cpu().numpy(), d_d.cpu().numpy()
        for i in range(2):
            k_ref, d_ref = oracle.extract(p, imgs[i])
            assert counts[i] == len(k_ref)
            np.testing.assert_array_equal(kk[i, :counts[i]].view(_capi.KP_DTYPE).reshape(-1), k_ref)
            np.testing.assert_array_equal(dd[i, :counts[i]], d_ref)
        if pinned:
            buf.close()


def test_batch_levelwise_pyramid_unaligned_rows(orb, oracle, images):
    """Batches > 8 build the pyramid level by level (k_pyr_level0 / k_pyr_resize): 10 frames of an
    odd width on an odd row pitch (rows start at every byte alignment), every padded level of
    several frames and every frame's keypoints / descriptors bit-exact vs the oracle."""
    import ctypes as C
    import torch
    from orb_slam2_with_comment_amd import _capi
    p = oracle.params(1500)
    ex = _extractor(orb, p)
    B, rows, cols, pitch = 10, 353, 647, 653
    base = images["kitti_L0"]
    rng = np.random.default_rng(7)
    imgs = np.zeros((B, rows, pitch), np.uint8)
    for i in range(B):
        y, x = rng.integers(0, base.shape[0] - rows), rng.integers(0, base.shape[1] - cols)
        imgs[i, :, :cols] = base[y:y + rows, x:x + cols]
        imgs[i, :, cols:] = rng.integers(0, 256, (rows, pitch - cols))  # never read
    flat = np.zeros(B * rows * pitch + 5, np.uint8)
    flat[3:3 + imgs.size] = imgs.reshape(-1)  # the batch starts 3 bytes into the allocation
    d_flat = torch.from_numpy(flat).cuda()
    cap = 1600
    d_k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_d = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_n = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _capi.check("batch", _capi.lib().orbmi_extract_batch_device(
        ex.handle, C.c_void_p(d_flat.data_ptr() + 3), B, rows, cols, pitch, rows * pitch,
        C.c_void_p(d_k.data_ptr()), C.c_void_p(d_d.data_ptr()), C.c_void_p(d_n.data_ptr()), cap))
    _capi.check("sync", _capi.lib().orbmi_extractor_synchronize(ex.handle))
    counts, kk, dd = d_n.cpu().numpy(), d_k.cpu().numpy(), d_d.cpu().numpy()
    for i in range(B):
        img = np.ascontiguousarray(imgs[i, :, :cols])
        if i in (0, 5, 9):
            ref = oracle.pyramid(p, img)
            for l in range(p.nlevels):
                np.testing.assert_array_equal(ex.pyramid_level(l, padded=True, item=i), ref[l], err_msg=f"{i} {l}")
        k_ref, d_ref = oracle.extract(p, img)
        assert counts[i] == len(k_ref), i
        np.testing.assert_array_equal(kk[i, :counts[i]].view(_capi.KP_DTYPE).reshape(-1), k_ref, err_msg=str(i))
        np.testing.assert_array_equal(dd[i, :counts[i]], d_ref, err_msg=str(i))
    ex.close()


def _run_batch(orb, imgs, nfeat):
    import ctypes as C
    import torch
    from orb_slam2_with_comment_amd import _capi
    B, rows, cols = imgs.shape
    ex = orb.ORBextractor(nfeat, 1.2, 8, 20, 7)
    cap = nfeat + 64
    d_img = torch.from_numpy(np.ascontiguousarray(imgs)).cuda()
    d_k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_d = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_n = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _capi.check("batch", _capi.lib().orbmi_extract_batch_device(
        ex.handle, C.c_void_p(d_img.data_ptr()), B, rows, cols, cols, rows * cols,
        C.c_void_p(d_k.data_ptr()), C.c_void_p(d_d.data_ptr()), C.c_void_p(d_n.data_ptr()), cap))
    _capi.check("sync", _capi.lib().orbmi_extractor_synchronize(ex.handle))
    return d_n.cpu().numpy(), d_k.cpu().numpy(), d_d.cpu().numpy()


# The A/B alternatives DESIGN.md measures (FAST's separate segment-test and score stages, the
# blur's placements) give the default path's keypoints and descriptors on a 12-frame batch (the
# level-wise pyramid and the side-stream blur); the default is checked against the oracle by
# test_config5_gpu.py and the tests above.
@pytest.mark.parametrize("knob", ["ORBMI_FAST=split", "ORBMI_BLUR=afterfast", "ORBMI_BLUR=perlevel",
                                  "ORBMI_BLUR=serial"])
def test_batch_ab_knobs_equal_default(orb, knob, monkeypatch):
    import config5_frames as C5
    imgs = C5.frames()[:12]
    n0, k0, d0 = _run_batch(orb, imgs, C5.NFEAT)
    var, val = knob.split("=")
    monkeypatch.setenv(var, val)
    n1, k1, d1 = _run_batch(orb, imgs, C5.NFEAT)
    np.testing.assert_array_equal(n1, n0)
    for i in range(len(imgs)):
        np.testing.assert_array_equal(k1[i, :n0[i]], k0[i, :n0[i]])
        np.testing.assert_array_equal(d1[i, :n0[i]], d0[i, :n0[i]])


def test_batch_host_images_levelwise(orb, oracle, images):
    """orbmi_extract_batch_host at a batch of 10 (the level-by-level pyramid of large batches) from
    pageable host memory: every frame equals the oracle."""
    import ctypes as C
    import torch
    from orb_slam2_with_comment_amd import _capi
    p = oracle.params(2000)
    ex = _extractor(orb, p)
    names = ["kitti_L0", "kitti_R0", "kitti_L11", "kitti_R11"]
    imgs = np.stack([images[names[i % 4]] for i in range(10)])
    B, r, c = imgs.shape
    cap = 2100
    d_k = torch.zeros((B, cap, 7), dtype=torch.int32, device="cuda")
    d_d = torch.zeros((B, cap, 32), dtype=torch.uint8, device="cuda")
    d_n = torch.zeros(B, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    _capi.check("batch_host", _capi.lib().orbmi_extract_batch_host(
        ex.handle, C.c_void_p(imgs.ctypes.data), B, r, c, r * c, C.c_void_p(d_k.data_ptr()),
        C.c_void_p(d_d.data_ptr()), C.c_void_p(d_n.data_ptr()), cap))
    _capi.check("sync", _capi.lib().orbmi_extractor_synchronize(ex.handle))
    counts, kk, dd = d_n.cpu().numpy(), d_k.cpu().numpy(), d_d.cpu().numpy()
    for i in range(4):  # the four distinct images (the rest repeat them)
        k_ref, d_ref = oracle.extract(p, imgs[i])
        for j in range(i, B, 4):
            assert counts[j] == len(k_ref)
            np.testing.assert_array_equal(kk[j, :counts[j]].view(_capi.KP_DTYPE).reshape(-1), k_ref)
            np.testing.assert_array_equal(dd[j, :counts[j]], d_ref)
