"""Keypoint / descriptor diff of the device extractor against the oracle on one synthetic frame:
the first differing rows per field and the descriptor bit-difference histogram.
python tools/desc_debug.py   (ORBMI_DESC=wave selects the one-keypoint-per-wave describe)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import orb_slam2_with_comment_amd as orb
    from orb_slam2_with_comment_amd import synth
    from oracle import oracle_ctypes as O
    O.lib()
    img, _, _ = synth.stereo_pair(synth.KITTI, 0)
    p = O.params(2000)
    ex = orb.ORBextractor(p.nfeatures, p.scale_factor, p.nlevels, p.ini_th_fast, p.min_th_fast)
    k, d = ex(img)
    kr, dr = O.extract(p, img)
    print("n", len(k), len(kr))
    n = min(len(k), len(kr))
    k, kr, d, dr = np.asarray(k)[:n], np.asarray(kr)[:n], np.asarray(d)[:n], np.asarray(dr)[:n]
    names = k.dtype.names or [str(i) for i in range(k.shape[1])]
    for i, f in enumerate(names):
        a = k[f] if k.dtype.names else k[:, i]
        b = kr[f] if kr.dtype.names else kr[:, i]
        bad = np.nonzero(a != b)[0]
        print(f"{f}: {len(bad)} differ", [(int(j), a[j], b[j]) for j in bad[:4]])
    bits = np.unpackbits(np.bitwise_xor(d, dr), axis=1).sum(1)
    print("desc rows differing", int((bits > 0).sum()), "bit-diff histogram", np.bincount(bits)[:12])
    j = int(np.argmax(bits > 0)) if (bits > 0).any() else 0
    print("row", j, "gpu", d[j][:8], "ref", dr[j][:8])


if __name__ == "__main__":
    main()
