"""Regenerate the golden extraction/stereo fixtures from the oracle (tests/golden/*.npz).

    python tests/golden/make_golden.py

The reference has no tests or golden vectors and cannot be built here
(OpenCV/Eigen absent), so these fixtures are produced by the pinned CPU restatement in
oracle/ and freeze it: tests/test_oracle_golden.py fails if the oracle drifts, and the GPU
parity tests compare the HIP path against the same arrays.  Inputs are stored with the
outputs so the fixtures do not depend on the synthetic renderer's libm.
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle_ctypes as O  # noqa: E402
from orb_slam2_with_comment_amd import synth  # noqa: E402


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def main():
    p = O.params(2000)
    L, R, _ = synth.stereo_pair(synth.KITTI, 0)
    kl, dl = O.extract(p, L)
    kr, dr = O.extract(p, R)
    u, d = O.stereo(p, L, R, synth.KITTI.bf, synth.KITTI.fx, kl, dl, kr, dr)
    np.savez_compressed(os.path.join(HERE, "kitti_stereo_f0.npz"), left=L, right=R,
                        kps_left=kl, desc_left=dl, kps_right=kr, desc_right=dr, u_right=u, depth=d,
                        bf=np.float32(synth.KITTI.bf), fx=np.float32(synth.KITTI.fx))
    # small crop exercising nlevels=4 and odd sizes
    crop = np.ascontiguousarray(L[40:40 + 283, 300:300 + 397])
    p4 = O.params(500, 1.2, 4, 20, 7)
    kc, dc = O.extract(p4, crop)
    np.savez_compressed(os.path.join(HERE, "crop_283x397_l4.npz"), image=crop, kps=kc, desc=dc)
    # digest of a 5000-feature EuRoC-shaped frame (config 5 shape)
    e = synth.mono(synth.EUROC, 0)
    ke, de = O.extract(O.params(5000), e)
    np.savez_compressed(os.path.join(HERE, "euroc_f0_digest.npz"), image=e,
                        sha256=np.frombuffer(digest(ke, de).encode(), np.uint8), n=np.int32(len(ke)))
    print("kitti", len(kl), len(kr), int((d > 0).sum()), "crop", len(kc), "euroc", len(ke))


if __name__ == "__main__":
    main()
