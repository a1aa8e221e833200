"""CPU checks of the Tracking restatement (oracle/track_oracle.cpp): TrackWithMotionModel +
TrackLocalMap (src/Tracking.cc:997-1104) on synthetic KITTI-shaped frames with exact ground
truth, PoseOptimization's edge assembly (src/Optimizer.cc:296-375) against the obs-array form,
and the mvpMapPoints bookkeeping against a literal Python restatement of the reference loops."""
import numpy as np
import pytest

from scenario import frame_data, lastframe, local_map, make_frame

from orb_slam2_with_comment_amd import synth, synth_map as SM
from orb_slam2_with_comment_amd.types import MP_HAS_OBS, POSE_OBS_DTYPE


def _inv_sigma2(oracle):
    return oracle.tables(oracle.params())["inv_sigma2"]


def _perturbed(f, dt=(0.03, -0.02, 0.05), yaw=0.003):
    kl, dl, u, d, T = frame_data(f)
    T = T.copy()
    c, s = np.cos(yaw), np.sin(yaw)
    T[:3, :3] = T[:3, :3] @ np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    T[:3, 3] += np.asarray(dt)
    from orb_slam2_with_comment_amd.types import Frame
    return Frame(kl, dl, u, SM.tcw_from_twc(T), synth.KITTI), T


def _center(tcw):
    R, t = tcw[:3, :3].astype(np.float64), tcw[:3, 3].astype(np.float64)
    return -R.T @ t


@pytest.mark.parametrize("f", [3, 6])
def test_track_frame_converges_to_ground_truth(oracle, f):
    cf, T0 = _perturbed(f)
    lf, lfp = lastframe(f - 1, seed=f)
    mps = local_map((f - 1, f - 2), seed=f)
    r = oracle.track_frame(cf, lf, lfp, mps, _inv_sigma2(oracle))
    assert r["ok"], r["stats"]
    gt = frame_data(f)[4][:3, 3]
    e0 = np.linalg.norm(T0[:3, 3] - gt)
    e_mm = np.linalg.norm(_center(r["tcw_mm"]) - gt)
    e = np.linalg.norm(_center(r["tcw"]) - gt)
    assert e_mm < 0.25 * e0 and e < 0.25 * e0, (e0, e_mm, e)
    st = r["stats"]
    assert st[0] >= 20 and st[1] >= 10 and st[2] >= 30 and st[3] > 0
    # final mvpMapPoints: stereo outliers were set to NULL
    has = (r["match_lf"] >= 0) | (r["match_mp"] >= 0)
    assert not (has & r["outlier"]).any()


def test_track_frame_lost_with_few_points(oracle):
    """< 20 matches after the 2*th retry: TrackWithMotionModel returns false."""
    cf, _ = _perturbed(4)
    lf, lfp = lastframe(3, seed=1)
    lfp = lfp.copy()
    lfp["flags"][10:] = 0  # only 10 last-frame points
    r = oracle.track_frame(cf, lf, lfp, local_map((3,)), _inv_sigma2(oracle))
    assert not r["ok"] and r["stats"][0] < 20


def test_pose_frame_equals_obs_form(oracle):
    """Edge assembly in keypoint order (mvpMapPoints -> edges) then the obs-array optimiser."""
    cf, _ = _perturbed(5)
    lf, lfp = lastframe(4, seed=2)
    occ = np.zeros(len(cf.keys), np.uint8)
    m_lf, _ = oracle.search_by_projection_last_frame(cf, occ, lf, lfp, 7.0)
    m_lf = np.ascontiguousarray(m_lf, np.int32)
    sig = _inv_sigma2(oracle)
    rec, out = oracle.pose_optimization_frame(cf, sig, m_lf, lfp)
    idx = np.nonzero(m_lf >= 0)[0]
    ob = np.zeros(len(idx), POSE_OBS_DTYPE)
    ob["Xw"] = lfp["pos"][m_lf[idx]]
    ob["u"], ob["v"] = cf.keys["x"][idx], cf.keys["y"][idx]
    ob["ur"] = cf.u_right[idx]
    ob["inv_sigma2"] = sig[cf.keys["octave"][idx]]
    ob["index"] = idx
    fr = np.zeros(1, rec.dtype)
    fr[0]["tcw"] = cf.tcw.reshape(-1)
    fr[0]["fx"], fr[0]["fy"], fr[0]["cx"], fr[0]["cy"], fr[0]["bf"] = (synth.KITTI.fx, synth.KITTI.fy, synth.KITTI.cx,
                                                                      synth.KITTI.cy, synth.KITTI.bf)
    fr[0]["n_obs"] = len(idx)
    ref_out = oracle.pose_optimization(fr, ob)
    np.testing.assert_array_equal(rec["tcw"], fr[0]["tcw"])
    assert rec["inliers"] == fr[0]["inliers"] and rec["n_obs"] == len(idx)
    np.testing.assert_array_equal(out[idx].astype(bool), ref_out)
    assert not out[m_lf < 0].any()


def _update_ref(stage, outlier, m_lf, lfp, m_mp, mps, stereo):
    """Literal restatement of src/Tracking.cc:1036-1058 (stage 0) and :1085-1104 (stage 1)."""
    m_lf, m_mp = m_lf.copy(), None if m_mp is None else m_mp.copy()
    occ = np.zeros(len(m_lf), np.uint8)
    c = [0, 0]
    for i in range(len(m_lf)):
        if m_mp is not None and m_mp[i] >= 0:
            arr, j, obs = m_mp, m_mp[i], bool(mps[m_mp[i]]["flags"] & MP_HAS_OBS)
        elif m_lf[i] >= 0:
            arr, j, obs = m_lf, m_lf[i], bool(lfp[m_lf[i]]["flags"] & MP_HAS_OBS)
        else:
            continue
        if stage == 0:
            if outlier[i]:
                arr[i] = -1
                c[0] += 1
            elif obs:
                c[1] += 1
                occ[i] = 1
        else:
            if not outlier[i]:
                c[0] += obs
            else:
                c[1] += 1
                if stereo:
                    arr[i] = -1
    return m_lf, m_mp, occ, c


@pytest.mark.parametrize("stage", [0, 1])
def test_track_update_matches_semantics(oracle, stage):
    rng = np.random.default_rng(11 + stage)
    cf = make_frame(2)
    n = len(cf.keys)
    lf, lfp = lastframe(1, seed=3)
    mps = local_map((1,), seed=3)
    m_lf = np.where(rng.random(n) < 0.4, rng.integers(0, len(lfp), n), -1).astype(np.int32)
    m_lf[rng.random(n) < 0.05] = -2  # rotation-rejected entries are NULL too
    m_mp = None
    if stage == 1:
        m_mp = np.where((rng.random(n) < 0.3), rng.integers(0, len(mps), n), -1).astype(np.int32)
    outlier = (rng.random(n) < 0.15).astype(np.uint8)
    ref_lf, ref_mp, ref_occ, ref_c = _update_ref(stage, outlier, m_lf, lfp, m_mp, mps, True)
    got_lf = m_lf.copy()
    got_mp = None if m_mp is None else m_mp.copy()
    occ, cnt = oracle.track_update_matches(cf, stage, outlier, got_lf, lfp, got_mp, mps if stage else None)
    np.testing.assert_array_equal(got_lf, ref_lf)
    if stage == 1:
        np.testing.assert_array_equal(got_mp, ref_mp)
    else:
        np.testing.assert_array_equal(occ, ref_occ)
    assert list(cnt) == ref_c
