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
