"""How far the GPU LocalBA's poses are from the oracle's, in float ulps (GPU).

    python tools/lba_pose_bits.py

tests/test_lba_gpu.py holds the poses to 1e-4.  This prints, for the same problems, how many
pose entries differ at all and by how many ulps: the perturbation a replay on the oracle inherits
(the r06zu replay mismatch; tools/tri_margins.py has the other half)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle_ctypes as O  # noqa: E402
from orb_slam2_with_comment_amd import synth_map as SM  # noqa: E402
from orb_slam2_with_comment_amd.optimizer import LocalBA  # noqa: E402


def ulps(a, b):
    ia = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    ib = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return np.abs(ia - ib)


def main():
    O.lib()
    ba = LocalBA()
    for seed, free, fixed, npts in [(3, 6, 2, 300), (42, 20, 4, 3000), (7, 10, 0, 800), (11, 21, 3, 1500),
                                    (5, 27, 2, 2000)]:
        prob, _ = SM.local_ba_problem(seed=seed, n_free=free, n_fixed=fixed, n_points=npts)
        ref = O.local_ba(prob)
        r = ba.run(prob)
        u = ulps(r["tcw"], ref["tcw"])
        up = ulps(r["pos"], ref["pos"])
        print(f"seed {seed:2d} ({free} free, {npts} points): pose entries differing {int(np.count_nonzero(u))}"
              f"/{u.size}, max {int(u.max())} ulp, max |d| {float(np.abs(r['tcw'] - ref['tcw']).max()):.3g}; "
              f"point coordinates differing {int(np.count_nonzero(up))}/{up.size}, max {int(up.max())} ulp; "
              f"iterations {r['iterations']} vs {ref['iterations']}", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
