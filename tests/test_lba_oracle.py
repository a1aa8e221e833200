"""CPU checks of the LocalBundleAdjustment restatement (g2o semantics)."""
import ctypes as C

import numpy as np
import pytest

from orb_slam2_with_comment_amd import synth_map as SM


@pytest.fixture(scope="module")
def small():
    return SM.local_ba_problem(seed=3, n_free=6, n_fixed=2, n_points=300)


def _centers(tcw):
    R = tcw[:, :3, :3]
    t = tcw[:, :3, 3]
    return -np.einsum("kji,kj->ki", R, t)


def test_lba_reduces_pose_error(oracle, small):
    prob, gt = small
    r = oracle.local_ba(prob)
    assert r["iterations"][0] >= 1 and r["iterations"][1] >= 1
    c0 = _centers(prob.kfs["tcw"].reshape(-1, 4, 4).astype(np.float64))
    c1 = _centers(r["tcw"].astype(np.float64))
    e0 = np.linalg.norm(c0 - gt["Twc"][:, :3, 3], axis=1)[2:]
    e1 = np.linalg.norm(c1 - gt["Twc"][:, :3, 3], axis=1)[2:]
    assert e1.mean() < 0.5 * e0.mean()
    # fixed cameras keep their pose (up to the float->quaternion->float round trip)
    np.testing.assert_allclose(r["tcw"][:2], prob.kfs["tcw"][:2].reshape(-1, 4, 4), atol=1e-6)


def test_lba_flags_injected_outliers(oracle):
    prob, gt = SM.local_ba_problem(seed=5, n_free=6, n_fixed=2, n_points=400, outlier_frac=0.1)
    r = oracle.local_ba(prob)
    assert 0.05 < r["erase"].mean() < 0.4


def test_lba_stop_flag_aborts(oracle, small):
    prob, _ = small
    r = oracle.local_ba(prob, stop=True)
    assert r["aborted"] == 1 and r["iterations"] == (0, 0)


def test_lba_deterministic(oracle, small):
    prob, _ = small
    a = oracle.local_ba(prob)
    b = oracle.local_ba(prob)
    np.testing.assert_array_equal(a["tcw"], b["tcw"])
    np.testing.assert_array_equal(a["erase"], b["erase"])


def test_lba_stop_check_numbering(oracle, small):
    """The deterministic pbStopFlag (orbmi_ba_set_stop_at_check's numbering): a run stopped at
    check k is the unstopped run up to that check, so it reports k as the first raised read; #0 is
    src/Optimizer.cc:685 (abort, no write-back), the last read before optimize(10) is :689 (no
    second optimisation), and k past the last read changes nothing."""
    prob, _ = small
    free = oracle.local_ba(prob, stop_at_check=-1)
    n = free["checks"]
    assert free["stop_check"] == -1 and n >= 4
    # 1 (#0) + optimize(5)'s loop reads + inner-loop reads + :689 + optimize(10)'s
    assert n >= 1 + free["iterations"][0] + 1 + free["iterations"][1]
    seen_no_more = False
    for k in range(n + 2):
        r = oracle.local_ba(prob, stop_at_check=k)
        if k < n:
            assert r["stop_check"] == k, (k, r["stop_check"])
        else:
            assert r["stop_check"] == -1
            for key in ("tcw", "pos", "erase"):
                np.testing.assert_array_equal(r[key], free[key])
        if k == 0:
            assert r["aborted"] == 1 and r["iterations"] == (0, 0)
        if k == 1:   # raised before optimize(5)'s first iteration: 0 iterations, no optimize(10)
            assert r["iterations"] == (0, 0) and not r["aborted"]
        if r["iterations"][0] == free["iterations"][0] and r["iterations"][1] == 0 and k < n:
            seen_no_more = True  # the :689 read (or one of optimize(5)'s last) ends the call there
        assert r["iterations"][0] <= free["iterations"][0]
    assert seen_no_more


def test_lba_stop_flag_equals_hook(oracle, small):
    """A flag already raised reads raised at every check: the same as the hook at 0."""
    prob, _ = small
    a = oracle.local_ba(prob, stop=True)
    b = oracle.local_ba(prob, stop_at_check=0)
    assert a["aborted"] == b["aborted"] == 1 and a["stop_check"] == b["stop_check"] == 0
