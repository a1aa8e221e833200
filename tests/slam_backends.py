"""Test infrastructure: the oracle (oracle/, CPU restatement) behind the backend interface of
orb_slam2_with_comment_amd/system.py, so that the same Tracking / LocalMapping host logic can run
on the oracle and on the MI355X operators and the two trajectories can be compared.  Never used
by the product path (system.GpuBackend is the only product backend)."""
from __future__ import annotations

import numpy as np

from orb_slam2_with_comment_amd.types import FeatureVector


class OracleBackend:
    def __init__(self, settings, vocabulary=None):
        from oracle import oracle_ctypes as O
        self.O = O
        s = settings
        self.p = O.params(s.n_features, float(s.scale_factor), s.n_levels, s.ini_th_fast, s.min_th_fast)
        t = O.tables(self.p)
        self.scale_factors = np.ascontiguousarray(t["scale"], np.float32)
        self.inv_level_sigma2 = np.ascontiguousarray(t["inv_sigma2"], np.float32)
        self.vocab = vocabulary
        self.calls = {}

    def _count(self, k):
        self.calls[k] = self.calls.get(k, 0) + 1

    def bind_camera(self, cam):
        self.cam = cam

    def extract_stereo(self, imL, imR):
        self._count("extract_stereo")
        O = self.O
        kl, dl = O.extract(self.p, imL)
        kr, dr = O.extract(self.p, imR)
        u, d = O.stereo(self.p, imL, imR, self.cam.bf, self.cam.fx, kl, dl, kr, dr)
        return kl, np.asarray(dl, np.uint8).reshape(-1, 32), u, d

    def compute_bow(self, desc):
        self._count("compute_bow")
        words, _, node, off, feat = self.O.transform(self.vocab, desc, 4)
        fv = FeatureVector.from_csr(node, off, feat)
        fv.n_words = len(words)   # (the BowVector's size, for the per-keyframe state record)
        return fv

    def search_by_bow(self, kf, kf_mp_ok, kf_fv, f, f_fv):
        self._count("search_by_bow")
        return self.O.search_by_bow(kf, kf_mp_ok, kf_fv, f, f_fv, 0.7)

    def search_last_frame(self, cf, occupied, lf, lfp, th):
        self._count("search_last_frame")
        return self.O.search_by_projection_last_frame(cf, occupied, lf, lfp, th)

    def search_local_points(self, cf, occupied, mps, th):
        self._count("search_local_points")
        tr = self.O.is_in_frustum(cf, mps, 0.5)
        if not np.any(tr["in_view"]):
            return np.full(len(cf.keys), -1, np.int32), 0, tr["in_view"].astype(bool)
        m, n = self.O.search_by_projection_local(cf, occupied, mps, tr, th, 0.8)
        return m, n, tr["in_view"].astype(bool)

    def search_for_triangulation(self, kf1, has_mp1, fv1, kf2, has_mp2, fv2, F12):
        self._count("search_for_triangulation")
        return self.O.search_for_triangulation(kf1, has_mp1, fv1, kf2, has_mp2, fv2, F12, False, False)

    def fuse_search(self, kf, mps, in_kf, th=3.0):
        self._count("fuse_search")
        bi, bd, _ = self.O.fuse_search(kf, mps, in_kf, th)
        return bi, bd

    def pose_optimization(self, cf, match_lf=None, lf_points=None, match_mp=None, mps=None):
        self._count("pose_optimization")
        ml = None if match_lf is None else np.ascontiguousarray(match_lf, np.int32)
        mm = None if match_mp is None else np.ascontiguousarray(match_mp, np.int32)
        rec, out = self.O.pose_optimization_frame(cf, self.inv_level_sigma2, ml, lf_points, mm, mps)
        return np.asarray(rec["tcw"], np.float32).reshape(4, 4).copy(), out.copy()

    def distinctive(self, obs_desc, obs_off):
        self._count("distinctive")
        return self.O.compute_distinctive_descriptors(obs_desc, obs_off)[1]

    def local_ba(self, problem, stop=None, stop_at_check=-1):
        self._count("local_ba")
        return self.O.local_ba(problem, stop_at_check=stop_at_check)

    def close(self):
        pass


def sequence_settings(tmpdir, cam=None, **kw):
    """A settings file in the reference's format for the synthetic KITTI-shaped sequence."""
    import os
    from orb_slam2_with_comment_amd import synth
    from orb_slam2_with_comment_amd.settings import load_settings, write_settings
    path = os.path.join(str(tmpdir), "KITTI_synth.yaml")
    write_settings(path, cam or synth.KITTI, **kw)
    return load_settings(path)


def small_vocabulary():
    """A synthetic DBoW2 tree (k=10, L=4); levelsup 4 puts every feature under the root's
    children level 0, so SearchByBoW compares all descriptors -- enough for the one
    TrackReferenceKeyFrame after initialisation."""
    from orb_slam2_with_comment_amd.vocabulary import Vocabulary
    return Vocabulary.synthetic(k=10, L=5, seed=3)


def _render(f):
    from orb_slam2_with_comment_amd import synth
    return synth.stereo_pair(synth.KITTI, f)


def render_sequence(n, workers=None):
    """Frames 0..n-1 of the synthetic KITTI-shaped sequence (synth.stereo_pair), rendered by a
    process pool (the ray caster takes ~0.2-0.3 s per stereo pair on one core)."""
    import multiprocessing as mp
    import os
    workers = workers or max(1, min(16, (os.cpu_count() or 1), n))
    if workers == 1:
        return [_render(f) for f in range(n)]
    with mp.get_context("fork").Pool(workers) as pool:
        return pool.map(_render, range(n))
