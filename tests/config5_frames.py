"""Config 5 inputs: EuRoC-shaped 752x480 mono frames, seed 5000 + frame,
rendered in parallel (numpy releases the GIL in the ray-cast)."""
from concurrent.futures import ThreadPoolExecutor

import numpy as np

BATCH = 64
NFEAT = 5000


def frames(first=0, n=BATCH, threads=8):
    from orb_slam2_with_comment_amd import synth
    with ThreadPoolExecutor(threads) as pool:
        return np.stack(list(pool.map(lambda f: synth.mono(synth.EUROC, f, seed_base=5000), range(first, first + n))))


def digest(*arrays):
    import hashlib
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()
