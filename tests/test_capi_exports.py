"""The C-ABI library loads and exports every symbol include/orbmi*.h declares (no GPU calls)."""
import ctypes
import os

from orb_slam2_with_comment_amd import _capi
from orb_slam2_with_comment_amd.build import LIB, build


def test_library_builds_and_exports_all_symbols():
    build()
    assert os.path.exists(LIB)
    lib = ctypes.CDLL(LIB)
    names = _capi.declared_symbols()
    assert len(names) >= 15
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    names = set(_capi.declared_symbols())
    assert names <= set(_capi._PROTOS), names - set(_capi._PROTOS)


def test_no_oracle_in_product():
    """The product library never links the oracle restatement."""
    import subprocess
    build()
    out = subprocess.run(["nm", "-D", LIB], capture_output=True, text=True).stdout
    assert "orc_" not in out
    deps = subprocess.run(["ldd", LIB], capture_output=True, text=True).stdout
    assert "oracle" not in deps


def test_lba_schur_block_table_every_size():
    """The k_ba_schur launch's block table (lba.hip ba_block_table / schur_role), host-side, for
    every supported number of free keyframes: pose-pair block ids are a permutation of
    [0, nblk) naming each pair (ra <= rb) exactly once, the keyframe blocks cover each free
    keyframe kSchurKfSplit times, one padding block ends the launch, and every rank a block
    reads is in [0, nf).  A block id no pair takes would read a stale blk_kf entry from the
    staging buffer (the round-4 r04x illegal address)."""
    import numpy as np
    L = ctypes.CDLL(LIB)
    f = L.orbmi_debug_ba_schur_blocks
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    f.restype = ctypes.c_int
    for nf in range(0, 31):
        nblk = nf * (nf + 1) // 2
        n = ctypes.c_int(0)
        t = np.zeros(4 * (nblk + 2 * nf + 1), np.int32)
        assert f(nf, t.ctypes.data, len(t) // 4, ctypes.byref(n)) == 0
        assert n.value == nblk + 2 * nf + 1
        t = t.reshape(-1, 4)
        pairs = t[:nblk]
        assert (pairs[:, 0] == 0).all()
        assert sorted(pairs[:, 3].tolist()) == list(range(nblk))  # ids <-> pairs: a permutation
        ra, rb = pairs[:, 1], pairs[:, 2]
        assert ((0 <= ra) & (ra <= rb) & (rb < max(nf, 1))).all()
        assert (pairs[:, 3] == ra * nf - ra * (ra - 1) // 2 + rb - ra).all()  # the pair it names
        if nf >= 8:  # a row's blocks share an id residue mod 8 (one XCD) unless they spilled
            same = [(pairs[:, 1] == r) for r in range(nf)]
            assert sum(len(set((np.nonzero(m)[0] % 8).tolist())) == 1 for m in same) >= nf // 2
        kfb = t[nblk:nblk + 2 * nf]
        assert (kfb[:, 0] == 1).all()
        assert sorted(kfb[:, 1].tolist()) == sorted(list(range(nf)) * 2)
        assert (kfb[:, 2] >= 0).all() and (kfb[:, 2] < 2).all()
        assert t[-1].tolist() == [2, -1, -1, -1]
    assert f(31, None, 0, ctypes.byref(n)) != 0  # beyond kBaMaxPoses
