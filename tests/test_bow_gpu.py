"""GPU parity of TemplatedVocabulary::transform (orbmi_transform, csrc/bow.hip) with the oracle:
word ids, BowVector values (bit-exact: the kernel keeps the reference's summation orders) and
the FeatureVector CSR, on ORB descriptors extracted from the synthetic frames; then
SearchByBoW fed with the GPU FeatureVectors equals the oracle's SearchByBoW fed with its own."""
import numpy as np
import pytest

from scenario import frame_data

pytestmark = pytest.mark.gpu


def _vocab(k, L, seed, **kw):
    from orb_slam2_with_comment_amd.vocabulary import Vocabulary
    return Vocabulary.synthetic(k=k, L=L, seed=seed, **kw)


def _check(got, ref):
    w, val, fv = got
    rw, rval, rnode, roff, rfeat = ref
    np.testing.assert_array_equal(w, rw)
    np.testing.assert_array_equal(val, rval)  # bit-exact
    np.testing.assert_array_equal(fv.node_id, rnode)
    np.testing.assert_array_equal(fv.off, roff)
    np.testing.assert_array_equal(fv.feat, rfeat)


@pytest.mark.parametrize("k,L,levelsup,scoring,weighting,irregular", [
    (10, 4, 4, 0, 0, False),   # ORB-SLAM2 settings: L1 scoring, TF-IDF, levelsup 4 (root node ids here)
    (10, 5, 3, 0, 0, False),
    (8, 4, 2, 1, 1, True),     # L2, TF, irregular tree
    (6, 4, 1, 5, 0, True),     # dot product: 1 / size, no normalisation
    (6, 3, 6, 2, 2, False),    # IDF (addIfNotExist); nid_level < 0
    (20, 3, 1, 0, 0, False),   # fan-out 20 > 16: the thread-per-descriptor kernel
])
def test_transform_matches_oracle(oracle, k, L, levelsup, scoring, weighting, irregular):
    from orb_slam2_with_comment_amd.vocabulary import ORBVocabulary
    v = _vocab(k, L, seed=k * 7 + L, stop_frac=0.05, irregular=irregular, scoring=scoring, weighting=weighting)
    gv = ORBVocabulary(v, device=0)
    for f in (3, 6):
        _, dl, _, _, _ = frame_data(f)
        _check(gv.transform(dl, levelsup), oracle.transform(v, dl, levelsup))
    # repeated descriptors (TF accumulation), the maximum size and the empty input
    rng = np.random.default_rng(k)
    d = frame_data(4)[1]
    big = d[rng.integers(0, len(d), 8192)]
    _check(gv.transform(big, levelsup), oracle.transform(v, big, levelsup))
    _check(gv.transform(big[:1], levelsup), oracle.transform(v, big[:1], levelsup))
    w, val, fv = gv.transform(np.zeros((0, 32), np.uint8), levelsup)
    assert len(w) == 0 and len(fv.node_id) == 0 and list(fv.off) == [0]
    gv.close()


def test_transform_full_depth_device_count(oracle):
    """k = 10, L = 6 (the ORB vocabulary's shape, 1.1 M nodes) with a device-resident count:
    only the first n_dev descriptors are transformed, asynchronously into device buffers."""
    import torch
    from orb_slam2_with_comment_amd.vocabulary import ORBVocabulary
    v = _vocab(10, 6, seed=11)
    gv = ORBVocabulary(v, device=0)
    _, dl, _, _, _ = frame_data(5)
    n = len(dl)
    cap = 4096
    d_desc = torch.zeros((cap, 32), dtype=torch.uint8, device="cuda")
    d_desc[:n] = torch.from_numpy(dl).cuda()
    n_dev = torch.tensor([n - 17], dtype=torch.int32, device="cuda")
    outs = dict(word=torch.zeros(cap, dtype=torch.int32, device="cuda"),
                value=torch.zeros(cap, dtype=torch.float64, device="cuda"),
                node=torch.zeros(cap, dtype=torch.int32, device="cuda"),
                off=torch.zeros(cap + 1, dtype=torch.int32, device="cuda"),
                feat=torch.zeros(cap, dtype=torch.int32, device="cuda"),
                counts=torch.zeros(2, dtype=torch.int32, device="cuda"))
    gv.transform_device(d_desc.data_ptr(), cap, n_dev.data_ptr(), 4, *(outs[k].data_ptr() for k in
                        ("word", "value", "node", "off", "feat", "counts")))
    gv.synchronize()
    rw, rval, rnode, roff, rfeat = oracle.transform(v, dl[:n - 17], 4)
    nw, nn = (int(x) for x in outs["counts"].cpu())
    assert (nw, nn) == (len(rw), len(rnode))
    np.testing.assert_array_equal(outs["word"][:nw].cpu().numpy().astype(np.uint32), rw)
    np.testing.assert_array_equal(outs["value"][:nw].cpu().numpy(), rval)
    np.testing.assert_array_equal(outs["node"][:nn].cpu().numpy().astype(np.uint32), rnode)
    np.testing.assert_array_equal(outs["off"][:nn + 1].cpu().numpy(), roff)
    np.testing.assert_array_equal(outs["feat"][:roff[-1]].cpu().numpy(), rfeat)
    gv.close()


def test_search_by_bow_with_gpu_feature_vectors(oracle):
    """TrackReferenceKeyFrame's chain: ComputeBoW of the keyframe and the frame on the GPU, then
    SearchByBoW (orbmi_search_by_bow) = the oracle's ComputeBoW + SearchByBoW."""
    from orb_slam2_with_comment_amd import synth
    from orb_slam2_with_comment_amd.matcher import ORBmatcher
    from orb_slam2_with_comment_amd.types import FeatureVector, Frame
    from orb_slam2_with_comment_amd.vocabulary import ORBVocabulary
    v = _vocab(10, 5, seed=21)
    gv = ORBVocabulary(v, device=0)
    kk, kd, ku, _, _ = frame_data(3)
    fk, fd, fu, _, _ = frame_data(4)
    KF, F = Frame(kk, kd, ku, None, synth.KITTI), Frame(fk, fd, fu, None, synth.KITTI)
    ok = (np.arange(len(kk)) % 5 != 0).astype(np.uint8)
    for levelsup in (2, 3):  # node ids at levels 3 and 2: both give populated nodes
        _, _, kfv = gv.transform(kd, levelsup)
        _, _, ffv = gv.transform(fd, levelsup)
        r_k = oracle.transform(v, kd, levelsup)
        r_f = oracle.transform(v, fd, levelsup)
        ref, nref = oracle.search_by_bow(KF, ok, FeatureVector.from_csr(*r_k[2:]), F,
                                         FeatureVector.from_csr(*r_f[2:]), 0.7, True)
        m = ORBmatcher(0.7, True)
        got, ngot = m.SearchByBoW(KF, ok, kfv, F, ffv)
        np.testing.assert_array_equal(got, ref)
        assert ngot == nref and nref > 20
        m.close()
    gv.close()


def test_transform_from_two_threads_on_one_handle(oracle):
    """Tracking (TrackReferenceKeyFrame: host descriptors, host outputs, src/Tracking.cc:871-917)
    and LocalMapping (ProcessNewKeyFrame's ComputeBoW with the map lock released: here with device
    outputs, as pipeline.LocalMapper makes them; src/LocalMapping.cc:152-160) transform on one
    vocabulary handle at once -- the reference's const TemplatedVocabulary::transform
    (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1194) is safe from both threads.  Each
    round both threads are released together by a barrier; every result equals the oracle's
    transform of its own descriptors (orbmi_transform serialises calls per handle: its staging
    buffer d_work is shared)."""
    import threading
    import torch
    from orb_slam2_with_comment_amd.vocabulary import ORBVocabulary
    v = _vocab(10, 5, seed=21)
    gv = ORBVocabulary(v, device=0)
    descs = [frame_data(f)[1] for f in range(6)]
    refs = [oracle.transform(v, d, 4) for d in descs]
    rounds = 24
    bar = threading.Barrier(2)
    errors = []

    def tracking():
        try:
            for r in range(rounds):
                i = r % len(descs)
                bar.wait()
                _check(gv.transform(descs[i], 4), refs[i])
        except Exception as e:  # reported by the main thread
            errors.append(("tracking", r, e))
            bar.abort()

    def mapping():
        try:
            torch.cuda.set_device(0)
            cap = max(len(d) for d in descs)
            outs = dict(word=torch.zeros(cap, dtype=torch.int32, device="cuda"),
                        value=torch.zeros(cap, dtype=torch.float64, device="cuda"),
                        node=torch.zeros(cap, dtype=torch.int32, device="cuda"),
                        off=torch.zeros(cap + 1, dtype=torch.int32, device="cuda"),
                        feat=torch.zeros(cap, dtype=torch.int32, device="cuda"),
                        counts=torch.zeros(2, dtype=torch.int32, device="cuda"))
            torch.cuda.synchronize()
            for r in range(rounds):
                i = (r + 3) % len(descs)
                d = np.ascontiguousarray(descs[i])
                bar.wait()
                gv.transform_device(d.ctypes.data, len(d), None, 4, *(outs[k].data_ptr() for k in
                                    ("word", "value", "node", "off", "feat", "counts")))
                gv.synchronize()
                rw, rval, rnode, roff, rfeat = refs[i]
                nw, nn = (int(x) for x in outs["counts"].cpu())
                assert (nw, nn) == (len(rw), len(rnode))
                np.testing.assert_array_equal(outs["word"][:nw].cpu().numpy().astype(np.uint32), rw)
                np.testing.assert_array_equal(outs["value"][:nw].cpu().numpy(), rval)
                np.testing.assert_array_equal(outs["node"][:nn].cpu().numpy().astype(np.uint32), rnode)
                np.testing.assert_array_equal(outs["off"][:nn + 1].cpu().numpy(), roff)
                np.testing.assert_array_equal(outs["feat"][:len(rfeat)].cpu().numpy(), rfeat)
        except Exception as e:
            errors.append(("mapping", r, e))
            bar.abort()

    ts = [threading.Thread(target=tracking), threading.Thread(target=mapping)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    gv.close()
    assert not any(t.is_alive() for t in ts)
    real = [e for e in errors if not isinstance(e[2], threading.BrokenBarrierError)]
    assert not real, real
    assert not errors, errors
