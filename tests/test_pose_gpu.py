"""GPU parity: Optimizer::PoseOptimization on MI355X (fp64, one workgroup per frame) vs the g2o
restatement (oracle/pose_oracle.cpp).  Bars: pose within 1e-4 (BASELINE.json north_star), the
mvbOutlier flags and the returned inlier count identical up to a chi2-on-the-threshold flip
(<= 0.2 % of the edges), LM iteration counts within 2 over the 4 rounds (the stop tests of
converged rounds sit on rounding)."""
import numpy as np
import pytest

from orb_slam2_with_comment_amd import synth_map as SM

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-4


@pytest.fixture(scope="module")
def PO():
    from orb_slam2_with_comment_amd.optimizer import PoseOptimizer
    return PoseOptimizer()


def _compare(fr, out, ref_fr, ref_out):
    for f in range(len(fr)):
        d = np.abs(fr[f]["tcw"] - ref_fr[f]["tcw"]).max()
        assert d <= POSE_TOL, (f, d)
        n = int(fr[f]["n_obs"])
        s = slice(int(fr[f]["obs_begin"]), int(fr[f]["obs_begin"]) + n)
        mism = int((out[s] != ref_out[s]).sum())
        assert mism <= max(1, int(0.002 * n)), (f, mism)
        assert abs(int(fr[f]["inliers"]) - int(ref_fr[f]["inliers"])) <= max(1, int(0.002 * n))
        # the 3-bad-iterations stop compares (iniChi - chi) * 1e3 with iniChi: a chi summed in
        # another order can end a converged round one iteration earlier or later
        assert abs(int(fr[f]["iterations"]) - int(ref_fr[f]["iterations"])) <= 2


@pytest.mark.parametrize("seed,n,stereo,outl,frames", [(1, 600, 0.7, 0.1, 1), (2, 2000, 0.8, 0.1, 1),
                                                        (3, 400, 0.0, 0.1, 2), (4, 500, 1.0, 0.2, 1),
                                                        (5, 300, 0.5, 0.3, 8), (6, 1200, 0.7, 0.05, 4)])
def test_pose_parity(oracle, PO, seed, n, stereo, outl, frames):
    fr, ob, _ = SM.pose_problem(seed=seed, n_obs=n, stereo_frac=stereo, outlier_frac=outl, nframes=frames)
    ref = fr.copy()
    ref_out = oracle.pose_optimization(ref, ob)
    out = PO.run(fr, ob)
    _compare(fr, out, ref, ref_out)


def test_pose_large_initial_error(oracle, PO):
    fr, ob, _ = SM.pose_problem(seed=7, n_obs=800, pose_noise=(0.05, 0.5))
    ref = fr.copy()
    ref_out = oracle.pose_optimization(ref, ob)
    _compare(fr, PO.run(fr, ob), ref, ref_out)


@pytest.mark.parametrize("n", [0, 2, 5, 9])
def test_pose_small(oracle, PO, n):
    """< 3 observations: return 0, pose untouched; < 10: a single round (:468-469)."""
    fr, ob, _ = SM.pose_problem(seed=8 + n, n_obs=max(n, 1), outlier_frac=0.0)
    if n == 0:
        fr["n_obs"] = 0
        ob = ob[:0].copy()
    t0 = fr["tcw"].copy()
    ref = fr.copy()
    ref_out = oracle.pose_optimization(ref, ob)
    out = PO.run(fr, ob)
    _compare(fr, out, ref, ref_out)
    if n < 3:
        np.testing.assert_array_equal(fr["tcw"], t0)
        assert fr[0]["inliers"] == 0
