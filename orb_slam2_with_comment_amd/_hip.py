"""The few HIP runtime calls the Python host code makes itself, with declared prototypes.

Why not torch here: a host word written by a copy on one of liborbmi.so's own streams (e.g. the
LocalMapping chain's search stream) must not be a torch pinned tensor.  torch's caching host
allocator remembers every stream a pinned block was copied on and, when the tensor is freed,
records an event on each of them.  The library destroys its streams when its handle closes, so a
pinned tensor that outlived the handle made torch record an event on a destroyed stream: the
segmentation fault of test_local_mapping_chain_matches_oracle in round 3 (`gpurun_out/s13`), at
the test's teardown, once LocalMapper.close() had destroyed the matcher and its stream.  Host
words written on library streams are therefore plain hipHostMalloc blocks owned by the object
that owns the handle, freed after the stream is drained and before the handle is destroyed.
"""
from __future__ import annotations

import ctypes as C

_vp, _i, _u, _sz = C.c_void_p, C.c_int, C.c_uint, C.c_size_t
HIP_MEMCPY_HOST_TO_DEVICE = 1  # hipMemcpyKind
HIP_MEMCPY_DEVICE_TO_HOST = 2
HIP_EVENT_DISABLE_TIMING = 0x2

PROTOS = {
    "hipHostMalloc": (_i, [C.POINTER(_vp), _sz, _u]),
    "hipHostFree": (_i, [_vp]),
    "hipMemcpyAsync": (_i, [_vp, _vp, _sz, _i, _vp]),
    "hipEventCreateWithFlags": (_i, [C.POINTER(_vp), _u]),
    "hipEventRecord": (_i, [_vp, _vp]),
    "hipEventSynchronize": (_i, [_vp]),
    "hipEventDestroy": (_i, [_vp]),
}

_rt = None


def runtime() -> C.CDLL:
    """libamdhip64 with the prototypes above: the runtime torch and liborbmi.so already use
    (torch bundles libamdhip64.so.7 and loads it first)."""
    global _rt
    if _rt is None:
        try:
            import torch  # noqa: F401  (binds the process to torch's runtime first)
        except ImportError:
            pass
        try:
            L = C.CDLL("libamdhip64.so.7")
        except OSError:
            L = C.CDLL("libamdhip64.so")
        for name, (res, args) in PROTOS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _rt = L
    return _rt


def _ok(what: str, rc: int) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} returned hipError {rc}")


class PinnedWords:
    """n int32 host words in pinned memory, filled by an asynchronous device-to-host copy on a
    caller's stream and read after an event recorded right behind that copy (so the read waits for
    the copy, whichever stream it ran on, and for nothing queued after it)."""

    def __init__(self, n: int):
        self.n = n
        self._rt = runtime()
        self._h = _vp()
        self._ev = _vp()
        _ok("hipHostMalloc", self._rt.hipHostMalloc(C.byref(self._h), 4 * n, 0))
        try:
            _ok("hipEventCreateWithFlags", self._rt.hipEventCreateWithFlags(C.byref(self._ev), HIP_EVENT_DISABLE_TIMING))
        except RuntimeError:
            self._rt.hipHostFree(self._h)
            self._h = _vp()
            raise

    def copy_async(self, src_device_ptr: int, stream_handle: int) -> None:
        _ok("hipMemcpyAsync", self._rt.hipMemcpyAsync(self._h, _vp(src_device_ptr), 4 * self.n,
                                                      HIP_MEMCPY_DEVICE_TO_HOST, _vp(stream_handle)))
        _ok("hipEventRecord", self._rt.hipEventRecord(self._ev, _vp(stream_handle)))

    def read(self) -> tuple:
        _ok("hipEventSynchronize", self._rt.hipEventSynchronize(self._ev))
        return tuple((C.c_int32 * self.n).from_address(self._h.value))

    def close(self) -> None:
        if self._ev:
            self._rt.hipEventSynchronize(self._ev)
            self._rt.hipEventDestroy(self._ev)
            self._ev = _vp()
        if self._h:
            self._rt.hipHostFree(self._h)
            self._h = _vp()


class PinnedBytes:
    """n bytes of pinned host memory (hipHostMalloc) with a numpy view: the source of
    asynchronous host-to-device copies on library streams (a frame's image pair DMA'd to HBM,
    pipeline.StereoTracker.track(host=True)).  The owner keeps it alive until every copy from it
    has completed."""

    def __init__(self, n: int):
        import numpy as np
        self._rt = runtime()
        self._h = _vp()
        _ok("hipHostMalloc", self._rt.hipHostMalloc(C.byref(self._h), max(int(n), 1), 0))
        self.n = int(n)
        self.ptr = self._h.value
        self.array = np.ctypeslib.as_array((C.c_uint8 * max(self.n, 1)).from_address(self.ptr))[:self.n]

    def close(self) -> None:
        if self._h is not None and self._h.value:
            self.array = None
            _ok("hipHostFree", self._rt.hipHostFree(self._h))
            self._h = None


def memcpy_h2d_async(dst_device_ptr: int, src_host_ptr: int, nbytes: int, stream_handle: int) -> None:
    _ok("hipMemcpyAsync", runtime().hipMemcpyAsync(_vp(dst_device_ptr), _vp(src_host_ptr), int(nbytes),
                                                   HIP_MEMCPY_HOST_TO_DEVICE, _vp(stream_handle)))
