"""GPU parity: ORBmatcher kernels (candidate search + parallel greedy replay) vs the
sequential CPU restatement, bit-exact on every output index and match count."""
import numpy as np
import pytest

from orb_slam2_with_comment_amd.types import MP_HAS_OBS

from scenario import bow, lastframe, local_map, make_frame

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def M():
    from orb_slam2_with_comment_amd import ORBmatcher
    return ORBmatcher


def test_is_in_frustum_parity(oracle, M):
    F = make_frame(3)
    mps = local_map((0, 1, 2))
    t_ref = oracle.is_in_frustum(F, mps, 0.5)
    t = M().IsInFrustum(F, mps, 0.5)
    assert t_ref["in_view"].sum() > 1000
    np.testing.assert_array_equal(t.view(np.uint8), t_ref.view(np.uint8))


@pytest.mark.parametrize("th,nnratio,dup", [(1.0, 0.8, 1), (3.0, 0.8, 1), (5.0, 0.6, 1), (1.0, 0.8, 3)])
def test_local_search_parity(oracle, M, th, nnratio, dup):
    F = make_frame(3)
    mps = local_map((0, 1, 2), seed=int(th * 10) + dup, dup=dup)
    tr = oracle.is_in_frustum(F, mps, 0.5)
    occ = (np.random.default_rng(5).random(len(F.keys)) < 0.1).astype(np.uint8)
    m_ref, n_ref = oracle.search_by_projection_local(F, occ, mps, tr, th, nnratio)
    m, n = M(nnratio).SearchByProjection(F, occ, mps, tr, th)
    assert n == n_ref and n > 100
    np.testing.assert_array_equal(m, m_ref)


def test_local_search_many_queries(oracle, M):
    """More than 65,536 map-point queries (k_greedy's non-register path, query indices above 16
    bits in its round-tagged claims): the local map tiled 12 times, so later copies compete with
    earlier ones for the same keypoints, index-exact against the sequential replay."""
    F = make_frame(3)
    base = local_map((0, 1, 2), seed=21)
    mps = np.tile(base, 70_000 // len(base) + 1)
    assert len(mps) > 65_536
    tr = oracle.is_in_frustum(F, mps, 0.5)
    occ = np.zeros(len(F.keys), np.uint8)
    m_ref, n_ref = oracle.search_by_projection_local(F, occ, mps, tr, 1.0, 0.8)
    m, n = M(0.8).SearchByProjection(F, occ, mps, tr, 1.0)
    assert n == n_ref and n > 100
    np.testing.assert_array_equal(m, m_ref)


def test_search_local_points_fused(oracle, M):
    F = make_frame(4)
    mps = local_map((1, 2, 3), seed=9)
    occ = np.zeros(len(F.keys), np.uint8)
    tr = oracle.is_in_frustum(F, mps, 0.5)
    m_ref, n_ref = oracle.search_by_projection_local(F, occ, mps, tr, 1.0, 0.8)
    m, n, ntm = M(0.8).SearchLocalPoints(F, occ, mps, 1.0)
    assert ntm == int(tr["in_view"].sum())
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)


@pytest.mark.parametrize("case", ["forward", "backward", "still", "mono", "no_ori", "th14"])
def test_lastframe_parity(oracle, M, case):
    cf = make_frame(3, pose_noise=0.01, seed=1)
    lf, lfp = lastframe(2, seed=4)
    th, mono, ori = 7.0, False, True
    if case == "backward":
        cf = make_frame(2, pose_noise=0.01, seed=2)
        lf, lfp = lastframe(3, seed=5)
    elif case == "still":
        cf = make_frame(3)
        lf, lfp = lastframe(3, seed=6)
    elif case == "mono":
        th, mono = 15.0, True
    elif case == "no_ori":
        ori = False
    elif case == "th14":
        th = 14.0
    occ = (np.random.default_rng(11).random(len(cf.keys)) < 0.05).astype(np.uint8)
    m_ref, n_ref = oracle.search_by_projection_last_frame(cf, occ, lf, lfp, th, mono, ori)
    mt = M(0.9, ori)
    m, n = mt.SearchByProjectionLastFrame(cf, occ, lf, lfp, th, mono)
    assert n == n_ref and n > 50
    np.testing.assert_array_equal(m, m_ref)


@pytest.mark.parametrize("ori", [True, False])
def test_bow_parity(oracle, M, ori):
    kf, ok, kfv, f, fv = bow(2, 3)
    m_ref, n_ref = oracle.search_by_bow(kf, ok, kfv, f, fv, 0.7, ori)
    m, n = M(0.7, ori).SearchByBoW(kf, ok, kfv, f, fv)
    assert n == n_ref and n > 20
    np.testing.assert_array_equal(m, m_ref)


def test_bow_coarse_nodes(oracle, M):
    """Few large nodes (>512 features per node) exercise the non-register exclusion path."""
    from orb_slam2_with_comment_amd.types import FeatureVector
    kf, ok, _, f, _ = bow(2, 3)
    kfv = FeatureVector(np.zeros(len(kf.keys), np.int64))
    fv = FeatureVector(np.zeros(len(f.keys), np.int64))
    m_ref, n_ref = oracle.search_by_bow(kf, ok, kfv, f, fv, 0.7, True)
    m, n = M(0.7, True).SearchByBoW(kf, ok, kfv, f, fv)
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)


def test_empty_inputs(oracle, M):
    F = make_frame(3)
    mps = local_map((2,))[:0]
    tr = oracle.is_in_frustum(F, mps, 0.5)
    m, n = M(0.8).SearchByProjection(F, np.zeros(len(F.keys), np.uint8), mps, tr, 1.0)
    assert n == 0 and (m == -1).all()


def test_device_resident_inputs(oracle, M):
    """Frame arrays already in HBM (torch tensors) are used in place."""
    import torch
    F = make_frame(3)
    mps = local_map((1, 2))
    tr = oracle.is_in_frustum(F, mps, 0.5)
    occ = np.zeros(len(F.keys), np.uint8)
    m_ref, n_ref = oracle.search_by_projection_local(F, occ, mps, tr, 1.0, 0.8)
    d_keys = torch.from_numpy(F.keys.view(np.uint8)).cuda()
    d_desc = torch.from_numpy(F.desc).cuda()
    d_u = torch.from_numpy(F.u_right).cuda()

    class DevFrameProxy:
        keys = F.keys

        def view(self):
            v = F.view()
            v.keys_un, v.desc, v.u_right = d_keys.data_ptr(), d_desc.data_ptr(), d_u.data_ptr()
            self._v = v
            return v

    m, n = M(0.8).SearchByProjection(DevFrameProxy(), occ, mps, tr, 1.0)
    assert n == n_ref
    np.testing.assert_array_equal(m, m_ref)


def test_pinned_grid(oracle, M):
    """orbmi_matcher_assign_features_to_grid (Frame::AssignFeaturesToGrid once per frame): searches
    on the pinned frame skip their grid build and still equal the oracle; a search on another
    frame rebuilds (and unpins), after which the first frame's search rebuilds too; host
    keypoints cannot be pinned."""
    import ctypes as C
    import torch
    from orb_slam2_with_comment_amd._capi import ORBMI_E_ARG, lib

    def dev_proxy(F):
        d = (torch.from_numpy(F.keys.view(np.uint8)).cuda(), torch.from_numpy(F.desc).cuda(),
             torch.from_numpy(F.u_right).cuda())

        class P:
            keys = F.keys
            _keep = d

            def view(self):
                v = F.view()
                v.keys_un, v.desc, v.u_right = d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr()
                self._v = v
                return v
        return P()

    FA, FB = make_frame(3), make_frame(5)
    PA, PB = dev_proxy(FA), dev_proxy(FB)
    mps_a, mps_b = local_map((1, 2)), local_map((3, 4))
    m = M(0.8)

    def ref(F, mps):
        occ = np.zeros(len(F.keys), np.uint8)
        return oracle.search_by_projection_local(F, occ, mps, oracle.is_in_frustum(F, mps, 0.5), 1.0, 0.8)

    def run(P, mps):
        occ = np.zeros(len(P.keys), np.uint8)
        r, n, _ = m.SearchLocalPoints(P, occ, mps, 1.0)
        return r, n

    ra, na = ref(FA, mps_a)
    rb, nb = ref(FB, mps_b)
    va = PA.view()
    assert lib().orbmi_matcher_assign_features_to_grid(m._h, C.addressof(va)) == 0
    for _ in range(2):                        # pinned: no rebuild, same result
        got, n = run(PA, mps_a)
        assert n == na and n > 100
        np.testing.assert_array_equal(got, ra)
    got, n = run(PB, mps_b)                   # another frame: its own grid
    assert n == nb
    np.testing.assert_array_equal(got, rb)
    got, n = run(PA, mps_a)                   # pin gone: frame A's grid is rebuilt
    np.testing.assert_array_equal(got, ra)
    assert lib().orbmi_matcher_release_grid(m._h) == 0
    vh = FA.view()                            # host keypoints: refused
    assert lib().orbmi_matcher_assign_features_to_grid(m._h, C.addressof(vh)) == ORBMI_E_ARG
    m.close()


def test_search_on_cu_masked_stream(oracle, M):
    """orbmi_matcher_reserve_cus: the handle's stream kept off 8 CUs (hipExtStreamCreateWithCUMask)
    gives the same matches; 0 restores an unmasked stream; a negative count is refused."""
    from orb_slam2_with_comment_amd._capi import lib
    F = make_frame(3)
    mps = local_map((0, 1, 2), seed=30)
    tr = oracle.is_in_frustum(F, mps, 0.5)
    occ = np.zeros(len(F.keys), np.uint8)
    m_ref, n_ref = oracle.search_by_projection_local(F, occ, mps, tr, 1.0, 0.8)
    mt = M(0.8)
    for n in (8, 0):
        assert lib().orbmi_matcher_reserve_cus(mt._h, n) == 0
        m, k = mt.SearchByProjection(F, occ, mps, tr, 1.0)
        assert k == n_ref
        np.testing.assert_array_equal(m, m_ref)
    assert lib().orbmi_matcher_reserve_cus(mt._h, -1) != 0
