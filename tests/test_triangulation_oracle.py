"""SearchForTriangulation (src/ORBmatcher.cc:783-975) oracle against a literal Python
restatement on a small subset (CPU; pure-Python loops only for small cases)."""
import numpy as np
import pytest

from tri_scenario import keyframe_pair


def py_search_for_triangulation(kf1, mp1, fv1, kf2, mp2, fv2, F12, only_stereo, check_ori):
    T1, T2 = kf1.tcw.astype(np.float32), kf2.tcw.astype(np.float32)
    f32 = np.float32
    Ow = [-(f32(f32(T1[0, i] * T1[0, 3]) + f32(T1[1, i] * T1[1, 3])) + f32(T1[2, i] * T1[2, 3])) for i in range(3)]
    Ow = [f32(x) for x in Ow]
    C2 = [f32(f32(f32(f32(T2[i, 0] * Ow[0]) + f32(T2[i, 1] * Ow[1])) + f32(T2[i, 2] * Ow[2])) + T2[i, 3]) for i in range(3)]
    invz = f32(f32(1.0) / C2[2])
    cam = kf1.cam
    ex = f32(f32(f32(f32(cam.fx) * C2[0]) * invz) + f32(cam.cx))
    ey = f32(f32(f32(f32(cam.fy) * C2[1]) * invz) + f32(cam.cy))
    sf = kf2.scale_factors.astype(np.float32)
    F = np.asarray(F12, np.float32)
    match = np.full(len(kf1.keys), -1, np.int32)
    hist = [[] for _ in range(30)]
    n = 0
    nodes2 = {int(nid): k for k, nid in enumerate(fv2.node_id)}
    for a, nid in enumerate(fv1.node_id):
        if int(nid) not in nodes2:
            continue
        b = nodes2[int(nid)]
        for i1 in fv1.feat[fv1.off[a]:fv1.off[a + 1]]:
            if mp1[i1]:
                continue
            st1 = kf1.u_right[i1] >= 0
            if only_stereo and not st1:
                continue
            kp1 = kf1.keys[i1]
            best, bidx = 50, -1
            for i2 in fv2.feat[fv2.off[b]:fv2.off[b + 1]]:
                if mp2[i2]:
                    continue
                st2 = kf2.u_right[i2] >= 0
                if only_stereo and not st2:
                    continue
                dist = int(np.unpackbits(kf1.desc[i1] ^ kf2.desc[i2]).sum())
                if dist > 50 or dist > best:
                    continue
                kp2 = kf2.keys[i2]
                if not st1 and not st2:
                    dx, dy = f32(ex - kp2["x"]), f32(ey - kp2["y"])
                    if f32(f32(dx * dx) + f32(dy * dy)) < f32(f32(100) * sf[kp2["octave"]]):
                        continue
                x1, y1 = f32(kp1["x"]), f32(kp1["y"])
                la = f32(f32(f32(x1 * F[0, 0]) + f32(y1 * F[1, 0])) + F[2, 0])
                lb = f32(f32(f32(x1 * F[0, 1]) + f32(y1 * F[1, 1])) + F[2, 1])
                lc = f32(f32(f32(x1 * F[0, 2]) + f32(y1 * F[1, 2])) + F[2, 2])
                num = f32(f32(f32(la * kp2["x"]) + f32(lb * kp2["y"])) + lc)
                den = f32(f32(la * la) + f32(lb * lb))
                if den == 0:
                    continue
                dsqr = f32(f32(num * num) / den)
                if float(dsqr) < 3.84 * float(f32(sf[kp2["octave"]] * sf[kp2["octave"]])):
                    best, bidx = dist, int(i2)
            if bidx >= 0:
                match[i1] = bidx
                n += 1
                if check_ori:
                    rot = f32(kp1["angle"] - kf2.keys[bidx]["angle"])
                    if rot < 0:
                        rot = f32(rot + f32(360))
                    b_ = int(np.floor(float(f32(rot * f32(1.0 / 30))) + 0.5))
                    hist[0 if b_ == 30 else b_].append(int(i1))
    if check_ori:
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i1_ = i2_ = i3_ = -1
        for i, s_ in enumerate(sizes):
            if s_ > m1:
                m3, m2, m1, i3_, i2_, i1_ = m2, m1, s_, i2_, i1_, i
            elif s_ > m2:
                m3, m2, i3_, i2_ = m2, s_, i2_, i
            elif s_ > m3:
                m3, i3_ = s_, i
        if m2 < 0.1 * m1:
            i2_ = i3_ = -1
        elif m3 < 0.1 * m1:
            i3_ = -1
        for i, h in enumerate(hist):
            if i in (i1_, i2_, i3_):
                continue
            for k in h:
                match[k] = -1
                n -= 1
    return match, n


@pytest.mark.parametrize("only_stereo,check_ori,drop", [(False, True, 0.4), (True, True, 0.0), (False, False, 0.6)])
def test_oracle_matches_python(oracle, only_stereo, check_ori, drop):
    (k1, m1, f1), (k2, m2, f2), F12 = keyframe_pair(drop_stereo=drop, seed=int(drop * 10))
    # a small subset of the KF1 nodes keeps the Python loop short
    keep = np.zeros(len(k1.keys), bool)
    for a in range(0, len(f1.node_id), 3):
        keep[f1.feat[f1.off[a]:f1.off[a + 1]]] = True
    m1 = np.where(keep, m1, 1).astype(np.uint8)
    ref, nref = oracle.search_for_triangulation(k1, m1, f1, k2, m2, f2, F12, only_stereo, check_ori)
    got, ngot = py_search_for_triangulation(k1, m1, f1, k2, m2, f2, F12, only_stereo, check_ori)
    np.testing.assert_array_equal(ref, got)
    assert nref == ngot and nref > 5
