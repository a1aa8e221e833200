"""GPU parity of MapPoint::ComputeDistinctiveDescriptors (orbmi_compute_distinctive_descriptors)
with the oracle: best rows and descriptors, exact; up to 300 observations per point (rows in
several wave chunks), empty points, device-resident inputs."""
import numpy as np
import pytest

from test_mappoint_oracle import make_obs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("npts,max_obs", [(3000, 12), (200, 70), (16, 300)])
def test_distinctive_matches_oracle(oracle, npts, max_obs):
    from orb_slam2_with_comment_amd.matcher import ORBmatcher
    rng = np.random.default_rng(npts + max_obs)
    d, off = make_obs(rng, npts, max_obs)
    ref_b, ref_d = oracle.compute_distinctive_descriptors(d, off)
    m = ORBmatcher()
    got_b, got_d = m.ComputeDistinctiveDescriptors(d, off)
    np.testing.assert_array_equal(got_b, ref_b)
    np.testing.assert_array_equal(got_d[ref_b >= 0], ref_d[ref_b >= 0])
    m.close()


def test_distinctive_device_resident(oracle):
    import ctypes as C
    import torch
    from orb_slam2_with_comment_amd._capi import lib
    from orb_slam2_with_comment_amd.matcher import ORBmatcher
    rng = np.random.default_rng(9)
    d, off = make_obs(rng, 500, 9)
    ref_b, ref_d = oracle.compute_distinctive_descriptors(d, off)
    m = ORBmatcher()
    dd, doff = torch.from_numpy(d).cuda(), torch.from_numpy(off).cuda()
    best = torch.full((500,), -7, dtype=torch.int32, device="cuda")
    out = torch.zeros((500, 32), dtype=torch.uint8, device="cuda")
    rc = lib().orbmi_compute_distinctive_descriptors(m._h, C.c_void_p(dd.data_ptr()), C.c_void_p(doff.data_ptr()), 500,
                                                     C.c_void_p(best.data_ptr()), C.c_void_p(out.data_ptr()))
    assert rc == 0
    torch.cuda.synchronize()
    np.testing.assert_array_equal(best.cpu().numpy(), ref_b)
    np.testing.assert_array_equal(out.cpu().numpy()[ref_b >= 0], ref_d[ref_b >= 0])
    m.close()
