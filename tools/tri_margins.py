"""How close CreateNewMapPoints' acceptance tests come to their thresholds over a whole run.

    python tools/tri_margins.py [frames]

Runs the synchronous oracle-driven loop (system.StereoSLAM on tests/slam_backends.OracleBackend,
the sequence of tests/test_native_slam_gpu.py) and, beside every orbmi_triangulate_matches call
the host logic makes, the triangulation oracle (oracle/tri_oracle.cpp) on the same inputs, which
reports per match the smallest relative margin of the decisions it took (|v - th| / max(|v|, |th|)).
The distribution says how large a pose perturbation -- e.g. LocalBA or PoseOptimization results
that agree with the oracle's within tolerance rather than bit for bit -- would be needed to flip a
point's acceptance (the r06zu replay mismatch).  CPU only."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import orb_slam2_with_comment_amd._capi as capi  # noqa: E402
from oracle import oracle_ctypes as O  # noqa: E402
from slam_backends import OracleBackend, render_sequence, sequence_settings, small_vocabulary  # noqa: E402
from orb_slam2_with_comment_amd.system import StereoSLAM  # noqa: E402

MARGINS = []


class _Proxy:
    """The product library with orbmi_triangulate_matches shadowed by the oracle's margins."""

    def __init__(self, real):
        self._real = real

    def __getattr__(self, name):
        fn = getattr(self._real, name)
        if name != "orbmi_triangulate_matches":
            return fn

        def wrapped(p1, p2, idx1, idx2, n, x3d, ok):
            rc = fn(p1, p2, idx1, idx2, n, x3d, ok)
            if n > 0:
                L = O.lib()
                L.orc_triangulate_matches.argtypes = [O.C.c_void_p] * 4 + [O.C.c_int] + [O.C.c_void_p] * 3
                xo = np.zeros((n, 3), np.float32)
                oko = np.zeros(n, np.uint8)
                mg = np.zeros(n, np.float32)
                assert L.orc_triangulate_matches(p1, p2, idx1, idx2, n, xo.ctypes.data, oko.ctypes.data,
                                                 mg.ctypes.data) == 0
                okp = np.ctypeslib.as_array(O.C.cast(ok, O.C.POINTER(O.C.c_uint8)), (n,))
                MARGINS.append((mg.copy(), oko.copy(), int(np.count_nonzero((okp != 0) != (oko != 0)))))
            return rc
        return wrapped


def main():
    nframes = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    real = capi.lib()
    capi.lib = lambda: _Proxy(real)
    frames = render_sequence(nframes)
    s = sequence_settings(__import__("pathlib").Path(tempfile.mkdtemp()))
    slam = StereoSLAM(s, backend=OracleBackend(s, small_vocabulary()))
    for f, (L, R, _) in enumerate(frames):
        slam.TrackStereo(L, R, 0.1 * f)
    mg = np.concatenate([m for m, _, _ in MARGINS]) if MARGINS else np.zeros(0, np.float32)
    acc = np.concatenate([o for _, o, _ in MARGINS]) if MARGINS else np.zeros(0, np.uint8)
    disagree = sum(d for _, _, d in MARGINS)
    print(f"{nframes} frames, {len(MARGINS)} triangulation calls, {len(mg)} matches "
          f"({int(np.count_nonzero(acc))} accepted), product/oracle acceptance disagreements: {disagree}")
    for th in (1e-7, 1e-6, 1e-5, 1e-4, 1e-3):
        print(f"  matches whose closest decision lies within {th:g} (relative) of its threshold: "
              f"{int(np.count_nonzero(mg < th))}")
    if len(mg):
        k = int(np.argmin(mg))
        print(f"  smallest margin {float(mg[k]):.3g} ({'accepted' if acc[k] else 'rejected'})")
    return 0


if __name__ == "__main__":
    sys.exit(main())
