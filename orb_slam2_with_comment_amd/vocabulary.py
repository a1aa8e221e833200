"""ORBVocabulary = DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> (include/ORBVocabulary.h)
and Frame::ComputeBoW / KeyFrame::ComputeBoW on the GPU.

Vocabulary            the tree as flat arrays, loaded from / saved to DBoW2's text format
                      (TemplatedVocabulary::loadFromTextFile / saveToTextFile,
                      Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1448), or generated
                      (`synthetic`): the ORB vocabulary itself is not available offline
                      (.MISSING_LARGE_BLOBS:1).
ORBVocabulary         the device handle (orbmi_vocabulary_*); transform() = TemplatedVocabulary::
                      transform(features, BowVector&, FeatureVector&, levelsup), ComputeBoW() the
                      Frame::ComputeBoW call (levelsup = 4, src/Frame.cc:425-432).
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np

from ._capi import check, lib
from .types import FeatureVector, VocabularyDesc

# DBoW2 enums (Thirdparty/DBoW2/DBoW2/BowVector.h:36-53)
TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = 0, 1, 2, 3, 4, 5


@dataclasses.dataclass(eq=False)
class Vocabulary:
    k: int
    L: int
    scoring: int
    weighting: int
    desc: np.ndarray        # nnodes x 32 u8 (node 0 = root)
    parent: np.ndarray      # nnodes int32 (root: -1)
    child_off: np.ndarray   # nnodes + 1 int32
    children: np.ndarray    # int32, children of node i at [child_off[i], child_off[i+1]) in insertion order
    word_id: np.ndarray     # nnodes int32, -1 for inner nodes
    weight: np.ndarray      # nnodes float64

    @property
    def nnodes(self) -> int:
        return len(self.parent)

    @property
    def nwords(self) -> int:
        return int((self.word_id >= 0).sum())

    # ---- construction
    @classmethod
    def from_nodes(cls, k, L, scoring, weighting, parent, is_leaf, desc, weight) -> "Vocabulary":
        """Nodes 1..N-1 in file order (parent, isLeaf, descriptor, weight), node 0 = root; word ids
        are given to leaves in file order, children are kept in insertion order (the
        loadFromTextFile bookkeeping)."""
        n = len(parent)
        parent = np.asarray(parent, np.int32)
        order = np.argsort(parent[1:], kind="stable") + 1      # children grouped by parent, in file order
        child_off = np.zeros(n + 1, np.int32)
        child_off[1:] = np.cumsum(np.bincount(parent[1:], minlength=n))
        children = order.astype(np.int32)
        word_id = np.full(n, -1, np.int32)
        leaves = np.nonzero(np.asarray(is_leaf, bool))[0]
        word_id[leaves] = np.arange(len(leaves), dtype=np.int32)
        return cls(int(k), int(L), int(scoring), int(weighting), np.ascontiguousarray(desc, np.uint8).reshape(n, 32),
                   parent, child_off, children, word_id, np.ascontiguousarray(weight, np.float64))

    @classmethod
    def from_text(cls, path) -> "Vocabulary":
        """TemplatedVocabulary::loadFromTextFile (:1338-1424): header "k L scoring weighting", then
        one line per node "parent isLeaf d0 .. d31 weight".  Blank lines are skipped (the
        reference would parse a trailing blank line as a node with an uninitialised parent)."""
        with open(path) as f:
            head = f.readline().split()
            k, L, n1, n2 = (int(x) for x in head[:4])
            if k < 0 or k > 20 or L < 1 or L > 10 or n1 < 0 or n1 > 5 or n2 < 0 or n2 > 3:
                raise ValueError("Vocabulary loading failure: This is not a correct text file!")
            parent, leaf, desc, weight = [-1], [False], [np.zeros(32, np.uint8)], [0.0]
            for line in f:
                t = line.split()
                if not t:
                    continue
                parent.append(int(t[0]))
                leaf.append(int(t[1]) > 0)
                desc.append(np.array([int(x) & 0xFF for x in t[2:34]], np.uint8))  # FORB::fromString
                weight.append(float(t[34]))
        return cls.from_nodes(k, L, n1, n2, parent, leaf, np.stack(desc), weight)

    def to_text(self, path):
        """TemplatedVocabulary::saveToTextFile (:1429-1448)."""
        with open(path, "w") as f:
            f.write(f"{self.k} {self.L}  {self.scoring} {self.weighting}\n")
            for i in range(1, self.nnodes):
                leaf = 1 if self.child_off[i] == self.child_off[i + 1] else 0
                d = " ".join(str(int(x)) for x in self.desc[i])
                f.write(f"{int(self.parent[i])} {leaf} {d}  {repr(float(self.weight[i]))}\n")

    @classmethod
    def synthetic(cls, k=10, L=6, seed=0, flip=(0.22, 0.12, 0.07, 0.04, 0.025, 0.015), stop_frac=0.0,
                  irregular=False, scoring=L1_NORM, weighting=TF_IDF) -> "Vocabulary":
        """A k-ary tree of depth L grown breadth-first (the order saveToTextFile writes): each child
        descriptor is its parent's with every bit flipped with probability flip[level - 1], so
        the descent groups similar descriptors as a trained tree does.  Leaves carry idf-like
        weights in [0.5, 6]; `stop_frac` of them get weight 0 (stopped words).  irregular=True
        gives nodes 2..k children and lets 10 % of the inner nodes below level 2 end early
        (leaves above level L), as k-means trees over small clusters do."""
        rng = np.random.default_rng(seed)
        parents = [np.array([-1])]
        leaves = [np.array([False])]
        descs = [rng.integers(0, 256, (1, 32), dtype=np.uint8)]
        weights = [np.zeros(1)]
        frontier = np.array([0])           # node ids to expand, breadth-first
        fdesc = descs[0]                   # their descriptors
        nxt_id = 1
        for lv in range(1, L + 1):
            if len(frontier) == 0:
                break
            nk = rng.integers(2, k + 1, len(frontier)) if irregular else np.full(len(frontier), k)
            par = np.repeat(frontier, nk)
            pd = np.repeat(fdesc, nk, axis=0)
            bits = np.unpackbits(pd, axis=1) ^ (rng.random((len(par), 256)) < flip[min(lv - 1, len(flip) - 1)])
            cd = np.packbits(bits.astype(np.uint8), axis=1)
            end = np.full(len(par), lv == L)
            if irregular and lv >= 2 and lv < L:
                end = rng.random(len(par)) < 0.1
            w = np.where(end, rng.uniform(0.5, 6.0, len(par)), 0.0)
            w[end & (rng.random(len(par)) < stop_frac)] = 0.0
            ids = np.arange(nxt_id, nxt_id + len(par))
            nxt_id += len(par)
            parents.append(par)
            leaves.append(end)
            descs.append(cd)
            weights.append(w)
            frontier, fdesc = ids[~end], cd[~end]
        return cls.from_nodes(k, L, scoring, weighting, np.concatenate(parents), np.concatenate(leaves),
                              np.concatenate(descs), np.concatenate(weights))

    def desc_struct(self) -> VocabularyDesc:
        d = VocabularyDesc()
        d.k, d.L, d.scoring, d.weighting, d.nnodes = self.k, self.L, self.scoring, self.weighting, self.nnodes
        self._arrays = [np.ascontiguousarray(a) for a in (self.desc, self.child_off, self.children, self.word_id,
                                                           self.weight)]
        d.desc, d.child_off, d.children, d.word_id, d.weight = (a.ctypes.data for a in self._arrays)
        return d


class ORBVocabulary:
    """Device-resident vocabulary (orbmi_vocabulary_*); transform() / ComputeBoW() mirror
    TemplatedVocabulary::transform and Frame::ComputeBoW."""

    def __init__(self, vocab: Vocabulary, device: int = 0):
        self.vocab = vocab
        self._desc = vocab.desc_struct()
        h = C.c_void_p()
        check("orbmi_vocabulary_create", lib().orbmi_vocabulary_create(device, C.byref(self._desc), C.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().orbmi_vocabulary_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def transform(self, desc: np.ndarray, levelsup: int = 4):
        """-> (bow_word uint32[], bow_value float64[], FeatureVector) for n x 32 host descriptors."""
        desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(desc)
        cap = max(n, 1)
        word = np.zeros(cap, np.uint32)
        value = np.zeros(cap, np.float64)
        node = np.zeros(cap, np.uint32)
        off = np.zeros(cap + 1, np.int32)
        feat = np.zeros(cap, np.int32)
        counts = np.zeros(2, np.int32)
        check("orbmi_transform", lib().orbmi_transform(self._h, desc.ctypes.data, n, None, levelsup, word.ctypes.data,
                                                       value.ctypes.data, node.ctypes.data, off.ctypes.data,
                                                       feat.ctypes.data, counts.ctypes.data))
        nw, nn = int(counts[0]), int(counts[1])
        return word[:nw], value[:nw], FeatureVector.from_csr(node[:nn], off[:nn + 1], feat[:int(off[nn])])

    def transform_device(self, d_desc: int, n: int, n_device, levelsup, d_word, d_value, d_node, d_off, d_feat,
                         d_counts):
        """Asynchronous form on device addresses (outputs stay in HBM; synchronize() before use)."""
        check("orbmi_transform", lib().orbmi_transform(self._h, d_desc, n, n_device, levelsup, d_word, d_value, d_node,
                                                       d_off, d_feat, d_counts))

    def ComputeBoW(self, desc: np.ndarray):
        """Frame::ComputeBoW: transform(mDescriptors, mBowVec, mFeatVec, 4)."""
        return self.transform(desc, 4)

    def synchronize(self):
        check("orbmi_vocabulary_synchronize", lib().orbmi_vocabulary_synchronize(self._h))
