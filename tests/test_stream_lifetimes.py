"""CPU regression tests for the round-3 segmentation fault (`gpurun_out/s13/pytest_sel.log`:
exit 139 in test_local_mapping_chain_matches_oracle, at the test's teardown).

Cause: a host word written by a copy on the LocalMapping chain's stream -- a stream liborbmi.so
owns and destroys in LocalMapper.close() -- was a torch pinned tensor.  torch's caching host
allocator records an event on every stream a pinned block was copied on when the tensor is freed;
the tensor outlived the mapper, so the event went to a destroyed stream.  The invariants below
keep that from coming back: no torch pinned memory and no record_stream in the package, every
HIP runtime call from Python through declared prototypes, and LocalMapper.close() settling
everything that refers to its stream before the handles that own the stream are destroyed.
"""
import ctypes as C
import pathlib
import re

import pytest

PKG = pathlib.Path(__file__).resolve().parents[1] / "orb_slam2_with_comment_amd"


def test_no_torch_pinned_memory_on_library_streams():
    for f in sorted(PKG.glob("*.py")):
        text = f.read_text()
        code = "\n".join(l.split("#", 1)[0] for l in text.splitlines())
        assert "pin_memory" not in code, f"{f.name}: torch pinned memory (use _hip.PinnedWords)"
        assert "record_stream" not in code, f"{f.name}: record_stream on a library-owned stream"
        if f.name != "_hip.py":
            assert not re.search(r"CDLL\(\s*['\"]libamdhip64", code), f"{f.name}: HIP runtime outside _hip.py"


def test_hip_runtime_prototypes_declared():
    from orb_slam2_with_comment_amd import _hip
    try:
        rt = _hip.runtime()
    except OSError:
        pytest.skip("libamdhip64 not loadable here")
    for name, (res, args) in _hip.PROTOS.items():
        fn = getattr(rt, name)
        assert fn.restype is res, name
        assert list(fn.argtypes) == list(args), name
    # hipMemcpyAsync(dst, src, bytes, kind, stream): a Python int for a pointer must not be
    # truncated to a C int (the failure mode of undeclared prototypes)
    assert rt.hipMemcpyAsync.argtypes[0] is C.c_void_p and rt.hipMemcpyAsync.argtypes[4] is C.c_void_p


class _Rec:
    def __init__(self, log, name):
        self.log, self.name = log, name

    def __getattr__(self, attr):
        def f(*a, **k):
            self.log.append(f"{self.name}.{attr}")
        return f


def test_local_mapper_close_order(monkeypatch):
    """close(): join the thread, drain the stream, materialise the lazy statistics (their closure
    synchronises the stream), drop the views and buffers, free the pinned words -- and only then
    destroy the LocalBA and matcher handles (the matcher owns the stream)."""
    import queue
    import threading

    from orb_slam2_with_comment_amd import pipeline

    log = []
    m = pipeline.LocalMapper.__new__(pipeline.LocalMapper)
    m.q = queue.Queue()
    m.t = threading.Thread(target=lambda: (m.q.get(), log.append("thread.exit")))
    m.t.start()
    m._ms = _Rec(log, "stream")
    m._counts_hs = [_Rec(log, "pinned")]
    m._vs = None
    m.ba = _Rec(log, "ba")
    m.matcher = _Rec(log, "matcher")
    m.voc = None
    m._one_stream = True
    m._bufs = {"tri": object()}
    m._out = {"tri": lambda: None}
    m.last_chain = pipeline.ChainStats(lambda: (log.append("stats"), {})[1], bow_words=1)
    m.close()
    assert log == ["thread.exit", "stream.synchronize", "stats", "pinned.close", "ba.close", "matcher.close"]
    assert m._bufs == {} and m._out is None
