"""ORBmatcher::Fuse (src/ORBmatcher.cc:977-1127) search: the oracle against a literal Python
restatement on a subset of map points (CPU)."""
import numpy as np

from scenario import local_map, make_frame
from test_matcher_oracle import _area, _grid


def py_fuse(kf, mps, in_kf, th):
    f32 = np.float32
    cells = _grid(kf)
    T = kf.tcw.astype(np.float32)
    Ow = [f32(-(f32(f32(T[0, c] * T[0, 3]) + f32(T[1, c] * T[1, 3])) + f32(T[2, c] * T[2, 3]))) for c in range(3)]
    sf = kf.scale_factors.astype(np.float32)
    lsf = f32(np.log(f32(sf[1])))
    out_i, out_d = [], []
    cam = kf.cam
    for i, mp in enumerate(mps):
        bi, bd = -1, 256
        ok = not (mp["flags"] & 1) and not in_kf[i]
        if ok:
            p = mp["pos"].astype(np.float32)
            Pc = [f32(f32(f32(f32(T[r, 0] * p[0]) + f32(T[r, 1] * p[1])) + f32(T[r, 2] * p[2])) + T[r, 3]) for r in range(3)]
            ok = not (Pc[2] < 0)
        if ok:
            invz = f32(f32(1) / Pc[2])
            u = f32(f32(f32(cam.fx) * f32(Pc[0] * invz)) + f32(cam.cx))
            v = f32(f32(f32(cam.fy) * f32(Pc[1] * invz)) + f32(cam.cy))
            ok = 0 <= u < cam.width and 0 <= v < cam.height
        if ok:
            ur = f32(u - f32(f32(cam.bf) * invz))
            PO = [f32(p[c] - Ow[c]) for c in range(3)]
            d3 = f32(np.sqrt(float(PO[0]) ** 2 + float(PO[1]) ** 2 + float(PO[2]) ** 2))
            ok = not (d3 < f32(f32(0.8) * mp["min_distance"]) or d3 > f32(f32(1.2) * mp["max_distance"]))
            if ok:
                dot = sum(float(PO[c]) * float(mp["normal"][c]) for c in range(3))
                ok = not (dot < 0.5 * float(d3))
        if ok:
            lvl = int(np.ceil(f32(f32(np.log(float(f32(mp["max_distance"] / d3)))) / lsf)))
            lvl = min(max(lvl, 0), len(sf) - 1)
            idx = _area(kf, cells, u, v, f32(f32(th) * sf[lvl]), -1, -1)
            for j in idx:
                kp = kf.keys[j]
                if kp["octave"] < lvl - 1 or kp["octave"] > lvl:
                    continue
                inv = f32(f32(1) / f32(sf[kp["octave"]] * sf[kp["octave"]]))
                ex, ey = f32(u - kp["x"]), f32(v - kp["y"])
                if kf.u_right is not None and kf.u_right[j] >= 0:
                    er = f32(ur - kf.u_right[j])
                    e2 = f32(f32(f32(ex * ex) + f32(ey * ey)) + f32(er * er))
                    if float(f32(e2 * inv)) > 7.8:
                        continue
                else:
                    e2 = f32(f32(ex * ex) + f32(ey * ey))
                    if float(f32(e2 * inv)) > 5.99:
                        continue
                dist = int(np.unpackbits(mp["desc"] ^ kf.desc[j]).sum())
                if dist < bd:
                    bd, bi = dist, int(j)
        out_i.append(bi if bd <= 50 else -1)
        out_d.append(bd)
    return np.array(out_i, np.int32), np.array(out_d, np.int32)


def test_fuse_oracle_matches_python(oracle):
    kf = make_frame(4)
    mps = local_map((2, 3), seed=4)[::6]  # a subset keeps the Python loop short
    rng = np.random.default_rng(0)
    in_kf = (rng.random(len(mps)) < 0.1).astype(np.uint8)
    bi, bd, n = oracle.fuse_search(kf, mps, in_kf, 3.0)
    ri, rd = py_fuse(kf, mps, in_kf, 3.0)
    np.testing.assert_array_equal(bi, ri)
    np.testing.assert_array_equal(bd, rd)
    assert n == int((ri >= 0).sum()) and n > 20
