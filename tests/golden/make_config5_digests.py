"""Per-frame digests of config 5 (64 EuRoC-shaped frames, 5000 features) from the oracle.

    python tests/golden/make_config5_digests.py

Stores, per frame, the SHA-256 of the rendered image and of the oracle's keypoints +
descriptors (tests/golden/config5_batch64_digests.npz).  tests/test_config5_gpu.py compares
the GPU batch against the oracle run live on the same images, and against these digests
wherever the image digest matches (the renderer uses numpy's libm, which may differ by host).
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import oracle_ctypes as O  # noqa: E402
import config5_frames as C5  # noqa: E402


def main():
    imgs = C5.frames()
    p = O.params(C5.NFEAT)
    with ThreadPoolExecutor(8) as pool:
        res = list(pool.map(lambda im: O.extract(p, im), imgs))
    img_sha = np.array([np.frombuffer(C5.digest(im).encode(), np.uint8) for im in imgs])
    out_sha = np.array([np.frombuffer(C5.digest(k, d).encode(), np.uint8) for k, d in res])
    n = np.array([len(k) for k, _ in res], np.int32)
    np.savez_compressed(os.path.join(HERE, "config5_batch64_digests.npz"), image_sha256=img_sha,
                        output_sha256=out_sha, n=n)
    print("frames", len(n), "keypoints min/mean/max", n.min(), n.mean(), n.max())


if __name__ == "__main__":
    main()
