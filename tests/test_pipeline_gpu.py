"""Device-resident Track pipeline (orb_slam2_with_comment_amd/pipeline.py) and the config-4
cross-stream matcher against the oracle, through the C ABI on the GPU."""
import numpy as np
import pytest

from scenario import frame_data, scale_factors

pytestmark = pytest.mark.gpu


def _lf_view_host(f):
    """Last-frame Frame + points of frame f (host arrays)."""
    from orb_slam2_with_comment_amd import synth, synth_map as SM
    from orb_slam2_with_comment_amd.types import Frame
    kl, dl, u, d, T = frame_data(f)
    rng = np.random.default_rng(100 + f)
    lfp = SM.lastframe_points(kl, dl, d, synth.KITTI, T, rng, outlier_frac=0.05, noobs_frac=0.02)
    return Frame(kl, dl, u, SM.tcw_from_twc(T), synth.KITTI), lfp


def test_tracker_device_resident_matches_oracle(oracle):
    """extract(L,R) -> stereo -> SearchByProjection(CF,LF) -> SearchLocalPoints (the searches
    alone, at the same pose and with empty occupancy; the full chain with PoseOptimization is
    tests/test_track_gpu.py), all enqueued on one stream with device-side keypoint counts,
    equals the oracle on the same frames."""
    import torch
    from orb_slam2_with_comment_amd import synth, synth_map as SM
    from orb_slam2_with_comment_amd.pipeline import StereoTracker
    from orb_slam2_with_comment_amd.types import Frame
    cam = synth.KITTI
    f = 3
    L, R, T = synth.stereo_pair(cam, f)
    tr = StereoTracker(cam, 2000, device=0)
    imgs = torch.from_numpy(np.stack([L, R])).cuda()
    tcw = SM.tcw_from_twc(T + np.pad(np.full((3, 1), 0.01), ((0, 1), (3, 0))))
    lf, lfp = _lf_view_host(f - 1)
    rng = np.random.default_rng(5)
    parts = []
    for g in (f - 1, f - 2):
        kl, dl, u, d, Tg = frame_data(g)
        mp, _ = SM.mappoints_from_frame(kl, dl, d, cam, Tg, scale_factors(), rng, 0.02, 0.0, 0.02)
        parts.append(mp)
    mps = np.concatenate(parts)
    d_lfp = torch.from_numpy(lfp.view(np.uint8).copy()).cuda()
    d_mps = torch.from_numpy(mps.view(np.uint8).copy()).cuda()
    lv = lf.view()  # host arrays: exercises the mixed host/device path too
    tr.extract_stereo(imgs.data_ptr(), cam.height, cam.width)
    tr.search_last_frame(tcw, lv, d_lfp.data_ptr())
    tr.search_local_points(tcw, d_mps.data_ptr(), len(mps))  # tr.occupied is still all zero
    tr.synchronize()
    n = int(tr.counts[0])
    kl, dl, u, d, _ = frame_data(f)
    assert n == len(kl)
    kps = tr.kps[0, :n].cpu().numpy().copy().view(kl.dtype).reshape(-1)
    np.testing.assert_array_equal(kps, kl)
    np.testing.assert_array_equal(tr.desc[0, :n].cpu().numpy(), dl)
    np.testing.assert_array_equal(tr.u_right[0, :n].cpu().numpy(), u)
    cf = Frame(kl, dl, u, tcw, cam)
    occ = np.zeros(n, np.uint8)
    ref_lf, nlf = oracle.search_by_projection_last_frame(cf, occ, lf, lfp, 7.0)
    got_lf = tr.match_lf[:n].cpu().numpy()
    np.testing.assert_array_equal(got_lf, ref_lf)
    assert nlf > 100
    trk = oracle.is_in_frustum(cf, mps, 0.5)
    ref_mp, nmp = oracle.search_by_projection_local(cf, occ, mps, trk, 1.0, 0.8)
    np.testing.assert_array_equal(tr.match_mp[:n].cpu().numpy(), ref_mp)
    assert nmp > 100
    tr.close()


@pytest.mark.parametrize("nseg,cap,skip", [(3, 400, 1), (1, 700, -1), (4, 257, 0)])
def test_cross_stream_matching(oracle, nseg, cap, skip):
    import ctypes as C
    import torch
    from orb_slam2_with_comment_amd.matcher import ORBmatcher
    from orb_slam2_with_comment_amd.pipeline import match_cross_stream
    rng = np.random.default_rng(nseg * 1000 + cap)
    base = rng.integers(0, 256, (600, 32), dtype=np.uint8)
    train = np.zeros((nseg, cap, 32), np.uint8)
    counts = rng.integers(cap // 2, cap + 1, nseg).astype(np.int32)
    for s in range(nseg):
        idx = rng.integers(0, len(base), cap)
        flips = rng.integers(0, 256, (cap, 32), dtype=np.uint8) & rng.integers(0, 2, (cap, 32), dtype=np.uint8)
        train[s] = base[idx] ^ (flips & np.uint8(0x11))
    q = base[rng.integers(0, len(base), 300)].copy()
    q[::7] = rng.integers(0, 256, (len(q[::7]), 32), dtype=np.uint8)  # some unmatched queries
    train[0, :5] = q[:5]  # exact duplicates -> ties across segments
    if nseg > 1:
        train[1, :5] = q[:5]
    ref = oracle.match_descriptors_segments(q, train, counts, skip, 50, 0.6)
    m = ORBmatcher()
    d_q = torch.from_numpy(q).cuda()
    d_t = torch.from_numpy(train).cuda()
    d_c = torch.from_numpy(counts).cuda()
    out = torch.full((len(q),), -7, dtype=torch.int32, device="cuda")
    nm = C.c_int()
    match_cross_stream(m._h, d_q.data_ptr(), len(q), None, d_t, d_c, skip, out, 50, 0.6, nmatches=nm)
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got, ref)
    assert nm.value == int((ref >= 0).sum())
    # device-resident query count: only the first 123 queries are searched
    nq_dev = torch.tensor([123], dtype=torch.int32, device="cuda")
    out.fill_(-7)
    match_cross_stream(m._h, d_q.data_ptr(), len(q), nq_dev.data_ptr(), d_t, d_c, skip, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got[:123], ref[:123])
    assert (got[123:] == -7).all()
    m.close()
