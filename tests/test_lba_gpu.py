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
    assert (r["stop_check"], r["checks"]) == (ref["stop_check"], ref["checks"]), \
        ((r["stop_check"], r["checks"]), (ref["stop_check"], ref["checks"]))
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
    assert r["aborted"] == 1 and r["iterations"] == (0, 0) and r["stop_check"] == 0


@pytest.mark.parametrize("seed,free,fixed,npts", [(3, 6, 2, 300), (42, 20, 4, 3000), (11, 8, 2, 600)])
def test_lba_interrupted_at_every_check(oracle, BA, seed, free, fixed, npts):
    """pbStopFlag raised mid-run (mbAbortBA, src/LocalMapping.cc:130-135 / InterruptBA), made
    deterministic by orbmi_ba_set_stop_at_check: for every read k of the flag -- #0 at
    src/Optimizer.cc:685, the loop conditions of optimize(5) (sparse_optimizer.cpp:376), the LM
    inner loop after rejected trials (optimization_algorithm_levenberg.cpp:149), bDoMore at :689,
    then optimize(10)'s -- the device stops where the oracle does: the same first raised read,
    iterations, erase list and write-back, poses within 1e-4.  (11, 8, 2, 600) is mono-only."""
    prob, _ = SM.local_ba_problem(seed=seed, n_free=free, n_fixed=fixed, n_points=npts,
                                  stereo_frac=0.0 if seed == 11 else 0.8)
    base = oracle.local_ba(prob)
    n = base["checks"]
    try:
        for k in range(n + 1):
            ref = oracle.local_ba(prob, edge_chi2=True, stop_at_check=k)
            r = BA.run(prob, stop=C.c_int(0), stop_at_check=k)
            assert r["stop_check"] == (k if k < n else -1)
            _compare(r, ref, prob)
    finally:
        BA.set_stop_at_check(-1)


def test_lba_live_flag_replays_by_check(oracle, BA):
    """A flag raised by another thread while the call runs (the concurrent LocalMapping's
    InterruptBA) is first seen at some check s; the call replayed with the hook at s, and the
    oracle stopped at s, give the same results."""
    import threading
    import time
    prob, _ = SM.local_ba_problem(seed=42, n_free=20, n_fixed=4, n_points=3000)
    BA.run(prob)  # warm
    seen = set()
    for delay in (0.0002, 0.0005, 0.001):
        flag = C.c_int(0)
        t = threading.Timer(delay, lambda: setattr(flag, "value", 1))
        t.start()
        live = BA.run(prob, stop=flag)
        t.join()
        s = live["stop_check"]
        seen.add(s)
        if s < 0:
            continue  # finished before the flag went up
        try:
            again = BA.run(prob, stop=C.c_int(0), stop_at_check=s)
        finally:
            BA.set_stop_at_check(-1)
        for k in ("tcw", "pos", "erase"):
            np.testing.assert_array_equal(again[k], live[k])
        assert again["iterations"] == live["iterations"] and again["stop_check"] == s
        _compare(live, oracle.local_ba(prob, edge_chi2=True, stop_at_check=s), prob)
    print("first raised reads seen:", sorted(seen))


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


def test_lba_rejects_duplicate_observation(BA):
    """Two edges for one (point, keyframe) pair cannot come from a map point's observations
    (src/Optimizer.cc:612-680 iterates a std::map per point); the per-keyframe Schur blocks rely
    on it, so such a graph is refused with ORBMI_E_ARG."""
    from orb_slam2_with_comment_amd._capi import ORBMI_E_ARG, OrbmiError
    from orb_slam2_with_comment_amd.types import BAProblem
    prob, _ = SM.local_ba_problem(seed=3, n_free=6, n_fixed=2, n_points=300)
    e = prob.edges
    dup = np.concatenate([e[:1], e])  # edge 0 twice (same point, same keyframe), still grouped by point
    bad = BAProblem(prob.kfs, prob.pts, dup)
    with pytest.raises(OrbmiError) as err:
        BA.run(bad)
    assert err.value.code == ORBMI_E_ARG
