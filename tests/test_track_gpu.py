"""GPU parity of the device-resident Track chain (pipeline.StereoTracker.track):
TrackWithMotionModel + TrackLocalMap (src/Tracking.cc:997-1104) with both PoseOptimizations on
the device and the optimised pose handed to the local-map search through device memory.

Stage by stage, every integer output is compared exactly with the oracle given the GPU's
float inputs of that stage (searches at the GPU's pose, bookkeeping with the GPU's outlier
flags); each pose is compared with the oracle's PoseOptimization within 1e-4 (BASELINE.json
north_star), its outlier flags and inlier count exactly up to an oracle chi2 on the threshold and
its iteration count up to a rounding-decided LM decision (the bars of tests/test_pose_gpu.py).
End to end, the final pose matches the oracle's full chain within 1e-4 and every count and match
array is exact."""
import numpy as np
import pytest

from scenario import frame_data, lastframe, local_map
from test_pose_gpu import check_flags, check_iterations

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-4


def _inv_sigma2(oracle):
    return oracle.tables(oracle.params())["inv_sigma2"]


def _setup(f, lfp_keep=None, dt=(0.03, -0.02, 0.05)):
    import torch
    from orb_slam2_with_comment_amd import synth, synth_map as SM
    from orb_slam2_with_comment_amd.pipeline import StereoTracker
    from orb_slam2_with_comment_amd.types import Frame
    cam = synth.KITTI
    L, R, T = synth.stereo_pair(cam, f)
    Tn = T.copy()
    Tn[:3, 3] += np.array(dt)
    tcw = SM.tcw_from_twc(Tn)
    lf, lfp = lastframe(f - 1, seed=f)
    if lfp_keep is not None:  # keep only the first lfp_keep last-frame map points
        lfp = lfp.copy()
        lfp["flags"][np.nonzero(lfp["flags"] & 1)[0][lfp_keep:]] = 0
    mps = local_map((f - 1, f - 2), seed=f)
    tr = StereoTracker(cam, 2000, device=0)
    d = dict(imgs=torch.from_numpy(np.stack([L, R])).cuda(), lfp=torch.from_numpy(lfp.view(np.uint8).copy()).cuda(),
             mps=torch.from_numpy(mps.view(np.uint8).copy()).cuda())
    kl, dl, u, _, _ = frame_data(f)
    return tr, d, tcw, lf, lfp, mps, Frame(kl, dl, u, tcw, cam)


def _cmp_pose(got_rec, ref, got_out, u_right):
    ref_rec, ref_out, chi2, margins = ref
    assert np.abs(got_rec["tcw"] - ref_rec["tcw"]).max() <= POSE_TOL
    n = int(ref_rec["n_obs"])
    assert int(got_rec["n_obs"]) == n
    nd = check_flags(got_out, ref_out, chi2, np.asarray(u_right) >= 0, tag="PoseOptimization")
    assert abs(int(got_rec["inliers"]) - int(ref_rec["inliers"])) <= nd
    check_iterations(got_rec["iterations"], ref_rec["iterations"], margins, tag="PoseOptimization")


@pytest.mark.parametrize("f", [3, 6])
def test_track_chain_stagewise(oracle, f):
    from orb_slam2_with_comment_amd.types import POSE_FRAME_DTYPE, Frame
    tr, d, tcw, lf, lfp, mps, cf = _setup(f)
    cam, sig = cf.cam, _inv_sigma2(oracle)
    n = len(cf.keys)
    lv = lf.view()
    tr.extract_stereo(d["imgs"].data_ptr(), cam.height, cam.width)
    tr.track_with_motion_model(tcw, lv, d["lfp"].data_ptr())
    tr.synchronize()
    assert int(tr.counts[0]) == n
    g_lf = tr.match_lf[:n].cpu().numpy().copy()
    g_out = tr.outlier[:n].cpu().numpy().copy()
    g_occ = tr.occupied[:n].cpu().numpy().copy()
    g_cnt = tr.tcounts.cpu().numpy().copy()
    rec0 = tr.recs[0].cpu().numpy().copy().view(POSE_FRAME_DTYPE)[0]
    # SearchByProjection(CF, LF, 7): exact
    ref_lf, ref_nm = oracle.search_by_projection_last_frame(cf, np.zeros(n, np.uint8), lf, lfp, 7.0)
    ref_lf = np.ascontiguousarray(ref_lf, np.int32)
    assert g_cnt[0] == ref_nm
    # PoseOptimization: 1e-4
    ref0 = oracle.pose_optimization_frame(cf, sig, ref_lf.copy(), lfp, diag=True)
    _cmp_pose(rec0, ref0, g_out, cf.u_right)
    # discard outliers with the GPU's flags: exact
    upd = ref_lf.copy()
    occ, cnt = oracle.track_update_matches(cf, 0, g_out, upd, lfp)
    np.testing.assert_array_equal(g_lf, upd)
    np.testing.assert_array_equal(g_occ, occ)
    assert list(g_cnt[1:3]) == list(cnt)
    # TrackLocalMap at the GPU's optimised pose
    tr.track_local_map(lv, d["lfp"].data_ptr(), d["mps"].data_ptr(), len(mps))
    tr.synchronize()
    g_mp = tr.match_mp[:n].cpu().numpy().copy()
    g_lf2 = tr.match_lf[:n].cpu().numpy().copy()
    g_out2 = tr.outlier[:n].cpu().numpy().copy()
    g_cnt = tr.tcounts.cpu().numpy().copy()
    rec1 = tr.recs[1].cpu().numpy().copy().view(POSE_FRAME_DTYPE)[0]
    cf2 = Frame(cf.keys, cf.desc, cf.u_right, rec0["tcw"].reshape(4, 4).copy(), cam)
    trk = oracle.is_in_frustum(cf2, mps, 0.5)
    ref_mp, _ = oracle.search_by_projection_local(cf2, g_occ, mps, trk, 1.0, 0.8)
    ref_mp = np.ascontiguousarray(ref_mp, np.int32)
    ref1 = oracle.pose_optimization_frame(cf2, sig, g_lf.copy(), lfp, ref_mp.copy(), mps, diag=True)
    _cmp_pose(rec1, ref1, g_out2, cf.u_right)
    up_lf, up_mp = g_lf.copy(), ref_mp.copy()
    _, cnt = oracle.track_update_matches(cf2, 1, g_out2, up_lf, lfp, up_mp, mps)
    np.testing.assert_array_equal(g_mp, up_mp)
    np.testing.assert_array_equal(g_lf2, up_lf)
    assert list(g_cnt[3:5]) == list(cnt)
    res = tr.results()
    assert res["ok"] and res["inliers"] == cnt[0]
    tr.close()


@pytest.mark.parametrize("f", [4, 7])
def test_track_chain_end_to_end(oracle, f):
    tr, d, tcw, lf, lfp, mps, cf = _setup(f)
    cam = cf.cam
    ref = oracle.track_frame(cf, lf, lfp, mps, _inv_sigma2(oracle))
    tr.track(d["imgs"].data_ptr(), cam.height, cam.width, tcw, lf.view(), d["lfp"].data_ptr(), d["mps"].data_ptr(),
             len(mps))
    res = tr.results()
    assert res["ok"] == ref["ok"] and res["ok"]
    assert np.abs(res["tcw_mm"] - ref["tcw_mm"]).max() <= POSE_TOL
    assert np.abs(res["tcw"] - ref["tcw"]).max() <= POSE_TOL
    n = len(cf.keys)
    st = ref["stats"]
    assert res["search_matches"] == st[0]
    # the local-map search runs at the GPU's pose, 1e-4-close to the oracle's: its matches and
    # both counts are index output and held exact (a map point on a search-window edge at one
    # pose and not the other would show here)
    assert res["nmatches_map"] == st[1] and res["inliers"] == st[2], (res, st)
    np.testing.assert_array_equal(tr.match_mp[:n].cpu().numpy(), ref["match_mp"])
    np.testing.assert_array_equal(tr.match_lf[:n].cpu().numpy(), ref["match_lf"])
    np.testing.assert_array_equal(tr.outlier[:n].cpu().numpy().astype(bool), ref["outlier"])
    tr.close()


def test_track_chain_retry_and_lost(oracle):
    """Few last-frame points: the 2*th retry runs on the device (gate open) and its count
    equals the oracle's; with < 20 after the retry the frame reports tracking lost."""
    for keep, ok in ((40, True), (15, False)):  # 0.3 m off: th=7 finds < 20, th=14 >= 20 with 40 points
        tr, d, tcw, lf, lfp, mps, cf = _setup(5, lfp_keep=keep, dt=(0.3, -0.02, 0.05))
        cam = cf.cam
        ref = oracle.track_frame(cf, lf, lfp, mps, _inv_sigma2(oracle))
        n = len(cf.keys)
        r7, n7 = oracle.search_by_projection_last_frame(cf, np.zeros(n, np.uint8), lf, lfp, 7.0)
        tr.track(d["imgs"].data_ptr(), cam.height, cam.width, tcw, lf.view(), d["lfp"].data_ptr(),
                 d["mps"].data_ptr(), len(mps))
        res = tr.results()
        assert res["search_matches"] == ref["stats"][0]
        assert n7 < 20  # the retry ran and its matches replaced the first search's
        r14, n14 = oracle.search_by_projection_last_frame(cf, np.zeros(n, np.uint8), lf, lfp, 14.0)
        assert res["search_matches"] == n14
        assert res["ok"] == ref["ok"] == ok
        if ok:
            assert np.abs(res["tcw"] - ref["tcw"]).max() <= POSE_TOL
        tr.close()


@pytest.mark.parametrize("f", [4, 7])
def test_track_fused_update_equals_two_launches(f):
    """orbmi_pose_optimization_frame_track (PoseOptimization with Tracking's update pass as its
    tail, the tracker's default) against the two launches it replaces (ORBMI_TRACK_UNFUSED):
    pose records, outlier flags, match arrays, occupancy and counts byte-identical."""
    out = []
    for unfused in (False, True):
        tr, d, tcw, lf, lfp, mps, cf = _setup(f)
        tr.unfused = unfused
        cam = cf.cam
        lv = lf.view()
        tr.extract_stereo(d["imgs"].data_ptr(), cam.height, cam.width)
        tr.track_with_motion_model(tcw, lv, d["lfp"].data_ptr())
        tr.track_local_map(lv, d["lfp"].data_ptr(), d["mps"].data_ptr(), len(mps))
        tr.synchronize()
        n = len(cf.keys)
        out.append({k: getattr(tr, k)[:n].cpu().numpy().copy() for k in ("match_lf", "match_mp", "outlier", "occupied")}
                   | {"tcounts": tr.tcounts.cpu().numpy().copy(), "recs": tr.recs.cpu().numpy().copy()})
        tr.close()
    for k in out[0]:
        np.testing.assert_array_equal(out[0][k], out[1][k], err_msg=k)


@pytest.mark.parametrize("f", [4, 7])
def test_pipelined_grid_ahead_equals_tracking_stream_grid(oracle, f, monkeypatch):
    """The pipelined tracker builds each frame's keypoint grid (Frame::AssignFeaturesToGrid) on
    the extraction stream into the frame slot's grid (orbmi_matcher_build_grid_slot, the default)
    and pins it for the frame's searches; ORBMI_GRID_AHEAD=0 builds it on the tracking stream at
    the first search.  Frame after frame (the slots alternate, each grid reused behind its slot's
    next extraction) the matches, outliers, counts and pose records are byte-identical, and the
    end-to-end results meet the oracle as test_track_chain_end_to_end's."""
    from orb_slam2_with_comment_amd import synth
    from orb_slam2_with_comment_amd.pipeline import StereoTracker
    out = {}
    for ahead in ("1", "0"):
        monkeypatch.setenv("ORBMI_GRID_AHEAD", ahead)
        tr0, d, tcw, lf, lfp, mps, cf = _setup(f)
        tr0.close()
        cam = synth.KITTI
        tr = StereoTracker(cam, 2000, device=0, pipelined=True)
        assert tr.grid_ahead == (ahead == "1")
        lv = lf.view()
        n = len(cf.keys)
        runs = []
        for _ in range(3):
            tr.track(d["imgs"].data_ptr(), cam.height, cam.width, tcw, lv, d["lfp"].data_ptr(), d["mps"].data_ptr(),
                     len(mps))
            res = tr.results()
            runs.append({k: getattr(tr, k)[:n].cpu().numpy().copy() for k in ("match_lf", "match_mp", "outlier")}
                        | {"tcounts": tr.tcounts.cpu().numpy().copy(), "recs": tr.recs.cpu().numpy().copy(),
                           "ok": res["ok"]})
        tr.close()
        out[ahead] = runs
    ref = oracle.track_frame(cf, lf, lfp, mps, _inv_sigma2(oracle))
    for a, b in zip(out["1"], out["0"]):
        for k in a:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
        assert a["ok"] == ref["ok"]
        np.testing.assert_array_equal(a["match_mp"], ref["match_mp"])
        np.testing.assert_array_equal(a["match_lf"], ref["match_lf"])
