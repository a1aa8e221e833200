"""GPU parity of the LocalMapping chain the headline bench runs per keyframe
(pipeline.LocalMapper.run_job, src/LocalMapping.cc:47-128): ComputeBoW (DBoW2 transform),
ComputeDistinctiveDescriptors, CreateNewMapPoints (every neighbour's SearchForTriangulation +
triangulation on the device, in the reference's pair order), Fuse in both directions of SearchInNeighbors, LocalBundleAdjustment -- each
output compared with the oracle on the same inputs (bench.setup_local_mapping's job).  Index and
descriptor outputs are exact; LocalBA's iteration counts are identical (its numeric bars are
tests/test_lba_gpu.py's)."""
import argparse
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("prebow", [True, False])  # ComputeBoW ahead on the vocabulary's stream, or in the chain
def test_local_mapping_chain_matches_oracle(oracle, prebow):
    import bench
    from orb_slam2_with_comment_amd import synth_map as SM
    from orb_slam2_with_comment_amd._capi import check, lib
    from orb_slam2_with_comment_amd.pipeline import LocalMapper
    from orb_slam2_with_comment_amd.vocabulary import ORBVocabulary, Vocabulary
    S = bench.setup_track(argparse.Namespace(frames=4, nfeatures=2000), 0, 0)
    vocab = Vocabulary.synthetic(k=10, L=5, seed=7)
    voc = ORBVocabulary(vocab, device=0)
    problem, _ = SM.local_ba_problem(seed=3, n_free=6, n_fixed=2, n_points=300)
    jobs, keep = bench.setup_local_mapping(S, voc, vocab, 0, problem)
    mapper = LocalMapper(0, vocabulary=voc, prebow=prebow)
    try:
        for f in (3, 5):
            job = jobs[f]
            out = mapper.run_job(job)  # synchronous, on this thread
            o, h = mapper._out, job.host
            o["fv"] = o["fv"]()  # the keyframe's FeatureVector, read back from HBM
            # ProcessNewKeyFrame: ComputeBoW -> FeatureVector
            _, _, node, off, feat = oracle.transform(vocab, h["desc"], 4)
            np.testing.assert_array_equal(o["fv"].node_id, node)
            np.testing.assert_array_equal(o["fv"].off, off)
            np.testing.assert_array_equal(o["fv"].feat, feat)
            # ComputeDistinctiveDescriptors
            npts = len(h["obs_off"]) - 1
            best_ref, dsc_ref = oracle.compute_distinctive_descriptors(h["obs_desc"], h["obs_off"])
            np.testing.assert_array_equal(o["best"][:npts].cpu().numpy(), best_ref)
            np.testing.assert_array_equal(o["dsc"][:32 * npts].cpu().numpy().reshape(npts, 32), dsc_ref)
            # CreateNewMapPoints: the reference's loop (the oracle's search with KF1's map points as
            # the earlier pairs left them, the host geometry) -- matches, accepts and positions exact
            n_new = 0
            has1 = h["kf"]["has_mp"].copy()
            tri, tri_ok, x3d_d = o["tri"](), o["tri_ok"](), o["x3d"]()
            for j, nb in enumerate(h["neighbours"]):
                m12, _ = oracle.search_for_triangulation(h["kf"]["frame"], has1, o["fv"], nb["frame"],
                                                         nb["has_mp"], nb["fv"], job.F12[j].reshape(3, 3), False,
                                                         False)
                np.testing.assert_array_equal(tri[j], m12, err_msg=f"keyframe {f} neighbour {j}")
                ok_ref = np.zeros(len(m12), np.uint8)
                idx1 = np.nonzero(m12 >= 0)[0].astype(np.int32)
                if len(idx1):
                    idx2 = np.ascontiguousarray(m12[idx1], np.int32)
                    x3d = np.zeros((len(idx1), 3), np.float32)
                    ok = np.zeros(len(idx1), np.uint8)
                    check("tri", lib().orbmi_triangulate_matches(
                        C.addressof(job.kf.tri), C.addressof(job.neighbours[j].tri), idx1.ctypes.data,
                        idx2.ctypes.data, len(idx1), x3d.ctypes.data, ok.ctypes.data))
                    ok_ref[idx1] = ok
                    sel = ok == 1
                    np.testing.assert_array_equal(x3d_d[j][idx1[sel]].view(np.uint32), x3d[sel].view(np.uint32))
                    has1[idx1[sel]] = 1
                    n_new += int(ok.sum())
                np.testing.assert_array_equal(tri_ok[j], ok_ref, err_msg=f"keyframe {f} neighbour {j} accepted")
            assert out["new_points"] == n_new and n_new > 0
            # SearchInNeighbors: Fuse(target, KF points) per target, then Fuse(KF, targets' points)
            n_kp = len(h["kf_points"])
            bi, bd = o["bi"].cpu().numpy(), o["bd"].cpu().numpy()
            for j, nb in enumerate(h["neighbours"]):
                bi_ref, bd_ref, _ = oracle.fuse_search(nb["frame"], h["kf_points"], None, 3.0)
                np.testing.assert_array_equal(bi[j * n_kp:(j + 1) * n_kp], bi_ref, err_msg=f"fuse target {j}")
                np.testing.assert_array_equal(bd[j * n_kp:(j + 1) * n_kp], bd_ref, err_msg=f"fuse target {j}")
            o0 = len(h["neighbours"]) * n_kp
            bi_ref, bd_ref, _ = oracle.fuse_search(h["kf"]["frame"], h["target_points"], None, 3.0)
            np.testing.assert_array_equal(bi[o0:o0 + len(bi_ref)], bi_ref)
            np.testing.assert_array_equal(bd[o0:o0 + len(bd_ref)], bd_ref)
            assert out["fuse_candidates"] == int((bi[:o0 + len(bi_ref)] >= 0).sum()) > 0
            # LocalBundleAdjustment
            assert tuple(out["local_ba_iterations"]) == tuple(oracle.local_ba(problem)["iterations"])
    finally:
        mapper.close()
        voc.close()
        S["tr"].close()


def test_compute_bow_ahead_on_the_queue(oracle):
    """Two keyframes queued on the LocalMapping thread: the second one's ComputeBoW is issued on the
    vocabulary's stream beside the first one's LocalBA (pipeline.LocalMapper._issue_bow), into the
    other BowVector / FeatureVector set; both FeatureVectors equal the oracle's transform."""
    import bench
    from orb_slam2_with_comment_amd import synth_map as SM
    from orb_slam2_with_comment_amd.pipeline import LocalMapper
    from orb_slam2_with_comment_amd.vocabulary import ORBVocabulary, Vocabulary
    S = bench.setup_track(argparse.Namespace(frames=6, nfeatures=2000), 0, 0)
    vocab = Vocabulary.synthetic(k=10, L=5, seed=7)
    voc = ORBVocabulary(vocab, device=0)
    problem, _ = SM.local_ba_problem(seed=3, n_free=6, n_fixed=2, n_points=300)
    jobs, keep = bench.setup_local_mapping(S, voc, vocab, 0, problem)
    mapper = LocalMapper(0, vocabulary=voc)
    try:
        if not mapper._prebow:
            pytest.skip("ORBMI_LM_PREBOW=0")
        for f in (3, 5, 3):
            mapper.insert_keyframe(jobs[f])
        mapper.wait()
        assert mapper.done == 3 and mapper.bow_ahead >= 1
        for slot, f in ((1, 5), (0, 3)):  # keyframes 2 and 3 took sets 1 and 0
            b = mapper.bows[slot]
            nn = int(b["counts"][1].item())
            _, _, node, off, feat = oracle.transform(vocab, jobs[f].host["desc"], 4)
            np.testing.assert_array_equal(b["node"][:nn].cpu().numpy().view(np.uint32), node)
            np.testing.assert_array_equal(b["off"][:nn + 1].cpu().numpy(), off)
            np.testing.assert_array_equal(b["feat"][:jobs[f].kf.n].cpu().numpy(), feat)
    finally:
        mapper.close()
        voc.close()
        S["tr"].close()
