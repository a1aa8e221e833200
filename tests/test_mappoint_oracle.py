"""MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:247-316):
the oracle against a literal Python restatement (sorted rows, vDists[0.5*(N-1)], strict <) on
random observation sets, incl. ties, single observations and points without observations."""
import numpy as np


def py_distinctive(obs_desc, obs_off):
    best, out = [], []
    for p in range(len(obs_off) - 1):
        D = obs_desc[obs_off[p]:obs_off[p + 1]]
        N = len(D)
        if N == 0:
            best.append(-1)
            out.append(np.zeros(32, np.uint8))
            continue
        bits = np.unpackbits(D, axis=1)
        dist = (bits[:, None, :] != bits[None, :, :]).sum(-1)
        bm, bi = 2 ** 31 - 1, 0
        for i in range(N):
            med = int(np.sort(dist[i])[int(0.5 * (N - 1))])
            if med < bm:
                bm, bi = med, i
        best.append(bi)
        out.append(D[bi])
    return np.array(best, np.int32), np.array(out, np.uint8).reshape(-1, 32)


def make_obs(rng, npts, max_obs=12):
    counts = rng.integers(0, max_obs + 1, npts)
    counts[:3] = [0, 1, 2]
    base = rng.integers(0, 256, (npts, 32), dtype=np.uint8)
    rows = []
    for p, c in enumerate(counts):
        flips = rng.integers(0, 256, (c, 32), dtype=np.uint8) & rng.integers(0, 256, (c, 32), dtype=np.uint8) \
            & rng.integers(0, 256, (c, 32), dtype=np.uint8)
        r = base[p] ^ flips
        if c >= 4:
            r[2] = r[1]  # duplicated observation: equal medians -> first row wins
        rows.append(r)
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    return np.concatenate(rows).reshape(-1, 32), off


def test_oracle_matches_python(oracle):
    rng = np.random.default_rng(3)
    d, off = make_obs(rng, 300)
    best, out = oracle.compute_distinctive_descriptors(d, off)
    rb, ro = py_distinctive(d, off)
    np.testing.assert_array_equal(best, rb)
    np.testing.assert_array_equal(out[best >= 0], ro[rb >= 0])
    assert best[0] == -1 and best[1] == 0
