"""DBoW2 TemplatedVocabulary::transform (Frame::ComputeBoW): the C++
oracle against a pure-Python restatement of Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1259
and BowVector.cpp:34-86 on small trees, a hand-built known-answer case, and the text format
round trip (loadFromTextFile / saveToTextFile).  CPU only."""
import numpy as np
import pytest

from orb_slam2_with_comment_amd import vocabulary as VB
from orb_slam2_with_comment_amd.vocabulary import Vocabulary


def py_transform(v: Vocabulary, desc, levelsup):
    """Literal restatement (std::map containers as dicts kept in key order)."""
    must = v.scoring != VB.DOT_PRODUCT
    l2 = v.scoring == VB.L2_NORM
    tf = v.weighting in (VB.TF_IDF, VB.TF)
    bow, fv = {}, {}
    if v.nwords:
        nid_level = v.L - levelsup
        for f, d in enumerate(np.asarray(desc, np.uint8).reshape(-1, 32)):
            node, level, nid = 0, 0, 0
            while True:
                level += 1
                kids = v.children[v.child_off[node]:v.child_off[node + 1]]
                node = int(kids[0])
                best = int(np.unpackbits(d ^ v.desc[node]).sum())
                for c in kids[1:]:
                    dd = int(np.unpackbits(d ^ v.desc[c]).sum())
                    if dd < best:
                        best, node = dd, int(c)
                if level == nid_level:
                    nid = node
                if v.child_off[node] == v.child_off[node + 1]:
                    break
            w = float(v.weight[node])
            word = int(v.word_id[node])
            if w > 0:
                if tf:
                    bow[word] = bow[word] + w if word in bow else w
                elif word not in bow:
                    bow[word] = w
                fv.setdefault(nid, []).append(f)
        if tf and bow and not must:
            nd = float(len(bow))
            bow = {k: x / nd for k, x in bow.items()}
        if must:
            keys = sorted(bow)
            norm = 0.0
            if l2:
                for k in keys:
                    norm += bow[k] * bow[k]
                norm = float(np.sqrt(norm))
            else:
                for k in keys:
                    norm += abs(bow[k])
            if norm > 0:
                bow = {k: bow[k] / norm for k in keys}
    words = np.array(sorted(bow), np.uint32)
    vals = np.array([bow[k] for k in sorted(bow)], np.float64)
    nodes = np.array(sorted(fv), np.uint32)
    off = np.concatenate([[0], np.cumsum([len(fv[k]) for k in sorted(fv)])]).astype(np.int32)
    feat = np.array([f for k in sorted(fv) for f in fv[k]], np.int32)
    return words, vals, nodes, off, feat


def noisy_desc(v, n, rng, flips=0.08):
    leaves = np.nonzero(v.word_id >= 0)[0]
    d = v.desc[rng.choice(leaves, n)].copy()
    bits = np.unpackbits(d, axis=1) ^ (rng.random((n, 256)) < flips).astype(np.uint8)
    return np.packbits(bits, axis=1)


def check_equal(got, ref):
    for g, r in zip(got, ref):
        np.testing.assert_array_equal(np.asarray(g), np.asarray(r))


@pytest.mark.parametrize("k,L,levelsup,scoring,weighting,irregular", [
    (10, 3, 2, VB.L1_NORM, VB.TF_IDF, False),   # the ORB-SLAM2 configuration (L1, TF-IDF)
    (6, 4, 4, VB.L2_NORM, VB.TF, True),         # nid_level = 0: root
    (5, 4, 1, VB.DOT_PRODUCT, VB.TF_IDF, True), # no normalisation: 1 / size
    (4, 3, 2, VB.CHI_SQUARE, VB.IDF, False),    # addIfNotExist, L1
    (4, 3, 5, VB.L1_NORM, VB.BINARY, True),     # nid_level < 0
])
def test_oracle_matches_python(oracle, k, L, levelsup, scoring, weighting, irregular):
    v = Vocabulary.synthetic(k=k, L=L, seed=k * 10 + L, stop_frac=0.1, irregular=irregular, scoring=scoring,
                             weighting=weighting)
    rng = np.random.default_rng(k + L)
    d = noisy_desc(v, 160, rng)
    d[5] = d[3]  # repeated word -> TF accumulation
    check_equal(oracle.transform(v, d, levelsup), py_transform(v, d, levelsup))


def test_known_answer(oracle):
    """k = 2, L = 2 by hand: ties go to the first child, a stopped word is dropped, TF-IDF
    weights accumulate per word and L1-normalise; node ids at level 1."""
    z = np.zeros(32, np.uint8)
    one = z.copy(); one[0] = 0x0F
    two = z.copy(); two[0] = 0xF0
    # nodes: 0 root; 1, 2 level 1; 3, 4 children of 1; 5, 6 children of 2
    desc = np.stack([z, one, two, one, one, two, two ^ np.uint8(1)])
    parent = [-1, 0, 0, 1, 1, 2, 2]
    leaf = [False, False, False, True, True, True, True]
    weight = [0, 0, 0, 2.0, 1.0, 0.0, 3.0]  # word of node 5 is stopped
    v = Vocabulary.from_nodes(2, 2, VB.L1_NORM, VB.TF_IDF, parent, leaf, desc, weight)
    feats = np.stack([one, one, two, two ^ np.uint8(1), z])
    # f0, f1 -> node 1 -> node 3 (tie 3/4: first) word 0, w 2; f2 -> node 2 -> node 5 (stopped);
    # f3 -> node 2 (distance 3 vs 5) -> node 6, word 3, w 3; f4 (zero) -> tie at level 1 ->
    # node 1 -> tie -> node 3, word 0
    w, val, node, off, feat = oracle.transform(v, feats, 1)
    np.testing.assert_array_equal(w, [0, 3])
    np.testing.assert_array_equal(val, np.array([6.0, 3.0]) / 9.0)
    np.testing.assert_array_equal(node, [1, 2])
    np.testing.assert_array_equal(off, [0, 3, 4])
    np.testing.assert_array_equal(feat, [0, 1, 4, 3])


def test_empty_inputs(oracle):
    v = Vocabulary.synthetic(k=3, L=2, seed=3)
    w, val, node, off, feat = oracle.transform(v, np.zeros((0, 32), np.uint8), 1)
    assert len(w) == 0 and len(node) == 0 and list(off) == [0]


def test_text_round_trip(tmp_path):
    v = Vocabulary.synthetic(k=5, L=3, seed=4, stop_frac=0.2, irregular=True)
    p = tmp_path / "voc.txt"
    v.to_text(p)
    with open(p, "a") as f:
        f.write("\n")  # a trailing blank line is skipped
    u = Vocabulary.from_text(p)
    assert (u.k, u.L, u.scoring, u.weighting) == (v.k, v.L, v.scoring, v.weighting)
    for a in ("parent", "child_off", "children", "word_id", "weight"):
        np.testing.assert_array_equal(getattr(u, a), getattr(v, a))
    np.testing.assert_array_equal(u.desc[1:], v.desc[1:])  # the root's descriptor is not stored


def test_text_header_rejected(tmp_path):
    p = tmp_path / "bad.txt"
    p.write_text("30 6  0 0\n")
    with pytest.raises(ValueError):
        Vocabulary.from_text(p)
