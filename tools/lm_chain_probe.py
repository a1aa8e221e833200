"""Per-phase wall time of one LocalMapping chain keyframe (pipeline.LocalMapper.run_job) on an
idle GPU: python tools/lm_chain_probe.py [reps].  Each phase is bracketed by host timers after a
device synchronisation, so the numbers include launch and host costs (run under rocprofv3
--kernel-trace for the kernels' own time)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from orb_slam2_with_comment_amd import pipeline, synth_map as SM  # noqa: E402
from orb_slam2_with_comment_amd.vocabulary import ORBVocabulary, Vocabulary  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    S = bench.setup_track(argparse.Namespace(frames=8, nfeatures=2000), 0, 0)
    vocab = Vocabulary.synthetic(k=10, L=6, seed=7)
    voc = ORBVocabulary(vocab, device=0)
    problem, _ = SM.local_ba_problem(seed=42)
    jobs, keep = bench.setup_local_mapping(S, voc, vocab, 0, problem)
    mapper = pipeline.LocalMapper(0, vocabulary=voc)
    marks = {}
    t_last = [0.0]

    def mark(name):
        torch.cuda.synchronize()
        t = time.perf_counter()
        marks[name] = marks.get(name, 0.0) + (t - t_last[0])
        t_last[0] = t

    # instrument: wrap the library calls the chain makes by name
    from orb_slam2_with_comment_amd import _capi
    L = _capi.lib()
    names = ["orbmi_transform", "orbmi_compute_distinctive_descriptors", "orbmi_search_for_triangulation",
             "orbmi_search_for_triangulation_batch", "orbmi_triangulate_matches", "orbmi_create_new_map_points",
             "orbmi_fuse_search",
             "orbmi_fuse_search_batch", "orbmi_local_bundle_adjustment"]

    class Wrap:
        def __init__(self, lib):
            self._lib = lib

        def __getattr__(self, n):
            f = getattr(self._lib, n)
            if n not in names:
                return f

            def g(*a):
                mark("(host between calls)")
                r = f(*a)
                mark(n)
                return r
            return g
    pipeline.lib = lambda: Wrap(L)

    def wrap_method(obj, attr, name):
        f = getattr(obj, attr)

        def g(*a, **k):
            mark("(host between calls)")
            r = f(*a, **k)
            mark(name)
            return r
        setattr(obj, attr, g)
    wrap_method(mapper.voc, "transform_device", "ComputeBoW (transform)")
    wrap_method(mapper.voc, "synchronize", "ComputeBoW sync")
    wrap_method(mapper.ba, "run", "LocalBundleAdjustment")
    for f in jobs:
        mapper.run_job(jobs[f])  # warm-up
    marks.clear()
    tot = 0.0
    for r in range(reps):
        f = sorted(jobs)[r % len(jobs)]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        t_last[0] = t0
        mapper.run_job(jobs[f])
        mark("(host between calls)")
        tot += time.perf_counter() - t0
    print(f"chain ms per keyframe: {tot / reps * 1e3:.3f}")
    for k, v in sorted(marks.items(), key=lambda kv: -kv[1]):
        print(f"  {k:45s} {v / reps * 1e3:8.3f} ms")
    print("last:", mapper.last_chain)
    mapper.close()


if __name__ == "__main__":
    main()
