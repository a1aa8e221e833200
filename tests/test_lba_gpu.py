"""GPU parity: LocalBundleAdjustment on MI355X (fp64, one persistent workgroup) vs the
sequential g2o restatement.  Tolerance 1e-4 on poses (BASELINE.json north_star)."""
import ctypes as C

import numpy as np
import pytest

from orb_slam2_with_comment_amd import synth_map as SM

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-4
# The erase list (src/Optimizer.cc:758-773) is index output and is held exact, except for an
# edge whose chi2 sits on its threshold (5.991 mono / 7.815 stereo) closer than the rounding
# differences of the two fp64 reduction orders can resolve: the oracle's chi2 for every
# differing flag must lie within this relative distance of the threshold.
ERASE_CHI2_RTOL = 1e-6


@pytest.fixture(scope="module")
def BA():
    from orb_slam2_with_comment_amd.optimizer import LocalBA
    return LocalBA()


def _compare(r, ref, prob, pt_tol=1e-3):
    assert r["aborted"] == ref["aborted"]
    assert r["iterations"] == ref["iterations"], (r["iterations"], ref["iterations"])
    dT = np.abs(r["tcw"] - ref["tcw"]).max()
    assert dT <= POSE_TOL, dT
    dP = np.abs(r["pos"] - ref["pos"]) / np.maximum(1.0, np.abs(ref["pos"]))
    assert dP.max() <= pt_tol, dP.max()
    mism = np.nonzero(r["erase"] != ref["erase"])[0]
    if len(mism):
        th = np.where(prob.edges["ur"][mism] < 0, 5.991, 7.815)
        margin = np.abs(ref["edge_chi2"][mism] - th) / th
        print(f"erase flags differing: {len(mism)} of {len(r['erase'])}, chi2 margins {margin.tolist()}")
        assert (margin <= ERASE_CHI2_RTOL).all(), (mism.tolist(), margin.tolist())
    np.testing.assert_allclose(r["chi2"], ref["chi2"], rtol=1e-6)


@pytest.mark.parametrize("seed,free,fixed,npts", [(3, 6, 2, 300), (42, 20, 4, 3000), (7, 10, 0, 800),
                                                 (11, 21, 3, 1500), (5, 27, 2, 2000)])
def test_lba_parity(oracle, BA, seed, free, fixed, npts):
    prob, _ = SM.local_ba_problem(seed=seed, n_free=free, n_fixed=fixed, n_points=npts)
    ref = oracle.local_ba(prob, edge_chi2=True)
    _compare(BA.run(prob), ref, prob)


@pytest.mark.parametrize("seed,free,fixed,npts", [(42, 20, 4, 3000), (11, 21, 3, 1500)])
def test_lba_parity_valu_solve(oracle, BA, monkeypatch, seed, free, fixed, npts):
    """The VALU pivot-wave solve (ORBMI_BA_SOLVE=pipe), kept for A/B runs, same bars."""
    monkeypatch.setenv("ORBMI_BA_SOLVE", "pipe")
    prob, _ = SM.local_ba_problem(seed=seed, n_free=free, n_fixed=fixed, n_points=npts)
    _compare(BA.run(prob), oracle.local_ba(prob, edge_chi2=True), prob)


@pytest.mark.parametrize("seed,free,fixed,npts", [(3, 6, 2, 300), (42, 20, 4, 3000), (7, 10, 0, 800),
                                                 (11, 21, 3, 1500), (13, 2, 1, 200), (17, 3, 0, 250)])
def test_lba_parity_mfma_solve(oracle, BA, monkeypatch, seed, free, fixed, npts):
    """The reduced system solved by the blocked LDL^T on MFMA (k_ba_solve_mfma<T>, tiles of
    16: 1 to 8 tiles across these sizes, padded last tiles included), same bars."""
    monkeypatch.setenv("ORBMI_BA_SOLVE", "mfma")
    prob, _ = SM.local_ba_problem(seed=seed, n_free=free, n_fixed=fixed, n_points=npts)
    _compare(BA.run(prob), oracle.local_ba(prob, edge_chi2=True), prob)


def test_lba_resume_after_rejections(oracle, BA, monkeypatch):
    """The call is enqueued at once with a few spare trials per optimize(); with none
    (ORBMI_BA_SLACK=0) every rejected trial leaves an optimize() short of trials, the gated
    launches after it do nothing and the host resumes it: results bitwise equal to the default
    schedule's, and parity with the oracle."""
    prob, _ = SM.local_ba_problem(seed=42, n_free=20, n_fixed=4, n_points=3000)
    base = BA.run(prob)
    monkeypatch.setenv("ORBMI_BA_SLACK", "0")
    r = BA.run(prob)
    for k in ("tcw", "pos", "erase"):
        np.testing.assert_array_equal(r[k], base[k])
    assert r["iterations"] == base["iterations"] and list(r["chi2"]) == list(base["chi2"])
    _compare(r, oracle.local_ba(prob, edge_chi2=True), prob)


def test_lba_mono_only(oracle, BA):
    prob, _ = SM.local_ba_problem(seed=11, n_free=8, n_fixed=2, n_points=600, stereo_frac=0.0)
    _compare(BA.run(prob), oracle.local_ba(prob, edge_chi2=True), prob)


def test_lba_bad_points(oracle, BA):
    prob, _ = SM.local_ba_problem(seed=12, n_free=8, n_fixed=2, n_points=600)
    prob.pts["bad"][::17] = 1
    _compare(BA.run(prob), oracle.local_ba(prob, edge_chi2=True), prob)


def test_lba_stop_before_start(oracle, BA):
    prob, _ = SM.local_ba_problem(seed=3, n_free=6, n_fixed=2, n_points=300)
    r = BA.run(prob, stop=C.c_int(1))
    assert r["aborted"] == 1 and r["iterations"] == (0, 0)


def test_lba_from_map_model(oracle, BA):
    """gather_local_ba (src/Optimizer.cc:486-683) over a small map, then parity."""
    from orb_slam2_with_comment_amd import synth
    from orb_slam2_with_comment_amd.optimizer import KeyFrame, MapPoint, gather_local_ba
    from orb_slam2_with_comment_amd.types import KP_DTYPE
    prob, gt = SM.local_ba_problem(seed=21, n_free=5, n_fixed=2, n_points=300)
    inv = np.float32(1.0) / (np.float32(1.2) ** (2 * np.arange(8))).astype(np.float32)
    kfs = []
    for k in range(len(prob.kfs)):
        e = prob.edges[prob.edges["kf"] == k]
        keys = np.zeros(len(e), KP_DTYPE)
        keys["x"], keys["y"] = e["u"], e["v"]
        keys["octave"] = np.rint(np.log(1.0 / e["inv_sigma2"]) / np.log(1.44)).astype(np.int32)
        kfs.append(KeyFrame(int(prob.kfs["id"][k]), prob.kfs["tcw"][k].reshape(4, 4), keys, e["ur"].copy(), inv,
                            synth.KITTI, map_points=[None] * len(e)))
    mps = [MapPoint(int(prob.pts["id"][p]), prob.pts["pos"][p].copy()) for p in range(len(prob.pts))]
    for k, kf in enumerate(kfs):
        idx = np.nonzero(prob.edges["kf"] == k)[0]
        for j, ei in enumerate(idx):
            mp = mps[prob.edges["point"][ei]]
            kf.map_points[j] = mp
            mp.observations[kf] = j
    free = kfs[2:]
    for kf in free:
        kf.covisible = [o for o in free if o is not kf]
    problem, order, _ = gather_local_ba(free[-1])
    assert len(problem.edges) > 0 and problem.kfs["fixed"].sum() >= 1
    _compare(BA.run(problem), oracle.local_ba(problem, edge_chi2=True), problem)


def test_lba_parity_mfma_solve_fused(oracle, BA, monkeypatch):
    """The MFMA solve run by the last block of the Schur kernel (ORBMI_BA_FUSE=1) instead of its
    own launch: the same results as the separate launch, bit for bit, and the oracle's bars."""
    monkeypatch.setenv("ORBMI_BA_SOLVE", "mfma")
    prob, _ = SM.local_ba_problem(seed=42, n_free=20, n_fixed=4, n_points=3000)
    fused = BA.run(prob)
    monkeypatch.setenv("ORBMI_BA_FUSE", "1")
    r = BA.run(prob)
    for k in ("tcw", "pos", "erase"):
        np.testing.assert_array_equal(r[k], fused[k])
    assert r["iterations"] == fused["iterations"]
    _compare(r, oracle.local_ba(prob, edge_chi2=True), prob)
