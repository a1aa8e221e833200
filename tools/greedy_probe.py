"""k_greedy statistics over tracked frames (orbmi_debug_greedy_stats): calls, rounds to the
fixpoint, slow-path evaluations, sequential fallbacks.  python tools/greedy_probe.py [frames]"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
from orb_slam2_with_comment_amd import _capi  # noqa: E402


def main():
    nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    S = bench.setup_track(argparse.Namespace(frames=8, nfeatures=2000), 0, 0)
    tr, cam = S["tr"], S["cam"]
    rows, cols = cam.height, cam.width
    L = _capi.lib()
    st = (C.c_ulonglong * 5)()
    for i in range(8):  # warm-up
        f = 2 + i % 8
        tr.track(S["imgs"].data_ptr() + f * 2 * rows * cols, rows, cols, S["tcws"][f], S["lf_views"][f - 1],
                 S["lf_pts"][f - 1].data_ptr(), S["mps"][f].data_ptr(), S["n_mp"][f])
    tr.synchronize()
    L.orbmi_debug_greedy_stats(st, 1)
    cyc = (C.c_ulonglong * 7)()
    L.orbmi_debug_greedy_cycles(cyc, 1)
    for i in range(nfr):
        f = 2 + i % 8
        tr.track(S["imgs"].data_ptr() + f * 2 * rows * cols, rows, cols, S["tcws"][f], S["lf_views"][f - 1],
                 S["lf_pts"][f - 1].data_ptr(), S["mps"][f].data_ptr(), S["n_mp"][f])
    tr.synchronize()
    L.orbmi_debug_greedy_stats(st, 1)
    calls = max(st[0], 1)
    print(f"k_greedy: {st[0]} calls, rounds mean {st[1] / calls:.2f}, max {st[2]}, slow evaluations per call "
          f"{st[3] / calls:.1f}, sequential fallbacks {st[4]}")
    L.orbmi_debug_greedy_cycles(cyc, 0)
    print("k_greedy s_memtime cycles per call: prologue %.0f, rounds %.0f, "
          "outputs %.0f" % tuple(c / calls for c in cyc[:3]))
    print("  rounds (thread 0): claims + barrier %.0f, evaluation %.0f, flag + barrier %.0f"
          % tuple(c / calls for c in cyc[3:6]))
    print("result:", tr.results()["search_matches"], tr.results()["inliers"])
    tr.close()


if __name__ == "__main__":
    main()
