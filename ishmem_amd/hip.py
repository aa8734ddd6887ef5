"""Minimal ctypes bindings to the HIP runtime (libamdhip64) for tests and the benchmark.

Device memory moves, streams and events without going through torch, so GPU tests exercise
exactly the native library and HIP.  Every call raises HipError on failure.
"""
from __future__ import annotations

import ctypes
import ctypes.util

import numpy as np

_hip = None
hipMemcpyHostToDevice, hipMemcpyDeviceToHost, hipMemcpyDeviceToDevice, hipMemcpyDefault = 1, 2, 3, 4


class HipError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    global _hip
    if _hip is None:
        for cand in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
            try:
                _hip = ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
                break
            except OSError:
                continue
        if _hip is None:
            raise HipError("libamdhip64.so not found")
        _hip.hipGetErrorString.restype = ctypes.c_char_p
    return _hip


def _check(err: int, what: str) -> None:
    if err != 0:
        msg = lib().hipGetErrorString(err).decode()
        raise HipError(f"{what} failed: {msg} ({err})")


def device_count() -> int:
    n = ctypes.c_int(0)
    err = lib().hipGetDeviceCount(ctypes.byref(n))
    return n.value if err == 0 else 0


def set_device(d: int) -> None:
    _check(lib().hipSetDevice(ctypes.c_int(d)), "hipSetDevice")


def malloc(nbytes: int) -> int:
    p = ctypes.c_void_p()
    _check(lib().hipMalloc(ctypes.byref(p), ctypes.c_size_t(max(nbytes, 1))), "hipMalloc")
    return p.value


def free(ptr: int) -> None:
    _check(lib().hipFree(ctypes.c_void_p(ptr)), "hipFree")


def host_malloc(nbytes: int) -> int:
    p = ctypes.c_void_p()
    _check(lib().hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(max(nbytes, 1)), ctypes.c_uint(0)), "hipHostMalloc")
    return p.value


def host_free(ptr: int) -> None:
    _check(lib().hipHostFree(ctypes.c_void_p(ptr)), "hipHostFree")


def memcpy(dst: int, src: int, nbytes: int, kind: int = hipMemcpyDefault) -> None:
    _check(lib().hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(nbytes),
                           ctypes.c_int(kind)), "hipMemcpy")


def memcpy_async(dst: int, src: int, nbytes: int, stream: int, kind: int = hipMemcpyDefault) -> None:
    _check(lib().hipMemcpyAsync(ctypes.c_void_p(dst), ctypes.c_void_p(src), ctypes.c_size_t(nbytes),
                                ctypes.c_int(kind), ctypes.c_void_p(stream)), "hipMemcpyAsync")


def memset(dst: int, value: int, nbytes: int) -> None:
    _check(lib().hipMemset(ctypes.c_void_p(dst), ctypes.c_int(value), ctypes.c_size_t(nbytes)), "hipMemset")


def upload(dst: int, arr: np.ndarray) -> None:
    a = np.ascontiguousarray(arr)
    memcpy(dst, a.ctypes.data, a.nbytes, hipMemcpyHostToDevice)


def download(src: int, n: int, dtype) -> np.ndarray:
    out = np.empty(n, dtype=dtype)
    if out.nbytes:
        memcpy(out.ctypes.data, src, out.nbytes, hipMemcpyDeviceToHost)
    return out


def synchronize() -> None:
    _check(lib().hipDeviceSynchronize(), "hipDeviceSynchronize")


def mem_get_info() -> tuple[int, int]:
    """(free, total) bytes of the current device (hipMemGetInfo)."""
    free, total = ctypes.c_size_t(0), ctypes.c_size_t(0)
    _check(lib().hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)), "hipMemGetInfo")
    return free.value, total.value


def stream_create() -> int:
    s = ctypes.c_void_p()
    _check(lib().hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1)), "hipStreamCreate")
    return s.value


def stream_destroy(s: int) -> None:
    _check(lib().hipStreamDestroy(ctypes.c_void_p(s)), "hipStreamDestroy")


def stream_query(s: int) -> bool:
    """True when every operation on stream s has completed (hipStreamQuery)."""
    err = lib().hipStreamQuery(ctypes.c_void_p(s))
    if err == 0:
        return True
    if err == 600:  # hipErrorNotReady
        return False
    _check(err, "hipStreamQuery")
    return False


def stream_synchronize(s: int) -> None:
    _check(lib().hipStreamSynchronize(ctypes.c_void_p(s)), "hipStreamSynchronize")


class Event:
    def __init__(self) -> None:
        e = ctypes.c_void_p()
        _check(lib().hipEventCreate(ctypes.byref(e)), "hipEventCreate")
        self.h = e.value

    def record(self, stream: int = 0) -> None:
        _check(lib().hipEventRecord(ctypes.c_void_p(self.h), ctypes.c_void_p(stream)), "hipEventRecord")

    def synchronize(self) -> None:
        _check(lib().hipEventSynchronize(ctypes.c_void_p(self.h)), "hipEventSynchronize")

    def elapsed_ms(self, end: "Event") -> float:
        ms = ctypes.c_float()
        _check(lib().hipEventElapsedTime(ctypes.byref(ms), ctypes.c_void_p(self.h), ctypes.c_void_p(end.h)),
               "hipEventElapsedTime")
        return float(ms.value)

    def __del__(self) -> None:
        try:
            if self.h:
                lib().hipEventDestroy(ctypes.c_void_p(self.h))
        except Exception:
            pass


class Graph:
    """Stream capture into a hipGraph: `with Graph(stream) as g: <enqueue on stream>`, then
    g.launch(stream) replays the captured work."""

    def __init__(self, stream: int) -> None:
        self.stream = stream
        self.graph = None
        self.exec = None

    def __enter__(self) -> "Graph":
        # hipStreamCaptureModeThreadLocal = 1
        _check(lib().hipStreamBeginCapture(ctypes.c_void_p(self.stream), ctypes.c_int(1)), "hipStreamBeginCapture")
        return self

    def __exit__(self, *exc) -> None:
        g = ctypes.c_void_p()
        _check(lib().hipStreamEndCapture(ctypes.c_void_p(self.stream), ctypes.byref(g)), "hipStreamEndCapture")
        self.graph = g.value
        if exc[0] is None:
            ge = ctypes.c_void_p()
            _check(lib().hipGraphInstantiate(ctypes.byref(ge), ctypes.c_void_p(self.graph), None, None,
                                             ctypes.c_size_t(0)), "hipGraphInstantiate")
            self.exec = ge.value

    def launch(self, stream: int | None = None) -> None:
        _check(lib().hipGraphLaunch(ctypes.c_void_p(self.exec), ctypes.c_void_p(self.stream if stream is None else stream)),
               "hipGraphLaunch")

    def __del__(self) -> None:
        try:
            if self.exec:
                lib().hipGraphExecDestroy(ctypes.c_void_p(self.exec))
            if self.graph:
                lib().hipGraphDestroy(ctypes.c_void_p(self.graph))
        except Exception:
            pass
