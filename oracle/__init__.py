"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes + numpy front end of the C restatement in oracle/oracle.c (reference semantics of the
reduction collective, oneapi-src/ishmem v1.5.1).  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module, and only as the checker / the timed CPU
baseline.  The product library (ishmem_amd/libishmem_amd.so) never touches it.

Pinning: see oracle/oracle.h and DESIGN.md §Oracle (reference known-answer generators +
MPICH MPI_Allreduce golden vectors in tests/golden/).
"""
from __future__ import annotations

import ctypes
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "liboracle.so"

OPS = {"and": 0, "or": 1, "xor": 2, "max": 3, "min": 4, "sum": 5, "prod": 6}
DTYPES = {"int8": 0, "int16": 1, "int32": 2, "int64": 3, "uint8": 4, "uint16": 5,
          "uint32": 6, "uint64": 7, "float": 8, "double": 9}
NP = {0: np.int8, 1: np.int16, 2: np.int32, 3: np.int64, 4: np.uint8, 5: np.uint16,
      6: np.uint32, 7: np.uint64, 8: np.float32, 9: np.float64}
PAT_ARITH, PAT_AND, PAT_OR, PAT_XOR = 0, 1, 2, 3
REDUCE_BUFFER_SIZE = 1 << 16  # src/collectives.h:10

_lib = None


def build(force: bool = False) -> Path:
    srcs = [HERE / "oracle.c", HERE / "oracle.h"]
    if force or not LIB_PATH.exists() or any(s.stat().st_mtime > LIB_PATH.stat().st_mtime for s in srcs):
        subprocess.run(["make", "-s", "-C", str(HERE), "-B", "liboracle.so"], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(str(LIB_PATH))
        vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        L.oracle_combine.argtypes = [i, i, vp, vp, sz]
        L.oracle_reduce_fold.argtypes = [i, i, ctypes.POINTER(vp), i, i, vp, sz]
        L.oracle_host_proxy_reduce.argtypes = [i, i, ctypes.POINTER(vp), ctypes.POINTER(vp), i, sz]
        L.oracle_host_proxy_time.argtypes = [i, i, sz, i, i]
        L.oracle_host_proxy_time.restype = ctypes.c_double
        L.oracle_host_bounce_time.argtypes = [i, i, sz, i, i, ctypes.c_char_p, vp, vp, vp, i]
        L.oracle_host_bounce_time.restype = ctypes.c_double
        L.oracle_pattern_source.argtypes = [i, i, i, sz, vp]
        L.oracle_pattern_check.argtypes = [i, i, i, i, sz, vp]
        L.oracle_fill_random.argtypes = [i, ctypes.c_uint64, ctypes.c_double, ctypes.c_double, sz, vp]
        L.oracle_fill_random.restype = None
        L.oracle_valid.argtypes = [i, i]
        _lib = L
    return _lib


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def valid(op: int, dt: int) -> bool:
    return bool(lib().oracle_valid(op, dt))


def reduce_fold(op: int, dt: int, srcs: list[np.ndarray], me: int = 0) -> np.ndarray:
    """Reference device fold for PE `me` (reduce_impl.h:232-256, :288-289).  me=0 is the
    canonical team-order fold the HIP path reproduces on every PE."""
    srcs = [np.ascontiguousarray(s) for s in srcs]
    out = np.empty_like(srcs[0])
    r = lib().oracle_reduce_fold(op, dt, _ptrs(srcs), len(srcs), me, out.ctypes.data, out.size)
    if r:
        raise ValueError("oracle_reduce_fold failed")
    return out


def host_proxy_reduce(op: int, dt: int, srcs: list[np.ndarray]) -> list[np.ndarray]:
    """Reference host bounce path (reduce_impl.h:186-228) — results for every PE."""
    srcs = [np.ascontiguousarray(s) for s in srcs]
    outs = [np.empty_like(srcs[0]) for _ in srcs]
    r = lib().oracle_host_proxy_reduce(op, dt, _ptrs(srcs), _ptrs(outs), len(srcs), srcs[0].size)
    if r:
        raise ValueError("oracle_host_proxy_reduce failed")
    return outs


def host_proxy_time(op: int, dt: int, n: int, npes: int, reps: int = 3) -> float:
    """Best wall seconds of the multi-process host-proxy restatement (CPU baseline)."""
    return float(lib().oracle_host_proxy_time(op, dt, n, npes, reps))


def hip_memcpy_fn() -> int:
    """Address of hipMemcpy in the HIP runtime (the copy the reference's host path makes with
    Level Zero, src/memory.cpp:310-321), for oracle_host_bounce_time."""
    for cand in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
        try:
            h = ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
            return ctypes.cast(h.hipMemcpy, ctypes.c_void_p).value
        except OSError:
            continue
    raise OSError("libamdhip64.so not found")


COPY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)


def host_bounce_time(op: int, dt: int, n: int, me: int, npes: int, key: str, dev_src: int,
                     dev_dst: int, reps: int = 1, copy_fn=None) -> float:
    """This member's best wall seconds of the reference's host path with its real synchronous
    64 KiB device<->host copies (oracle_host_bounce_time); every member calls it.  copy_fn
    defaults to hipMemcpy (a COPY_FN callback may stand in for it in CPU tests)."""
    fn = hip_memcpy_fn() if copy_fn is None else ctypes.cast(copy_fn, ctypes.c_void_p).value
    t = float(lib().oracle_host_bounce_time(op, dt, n, me, npes, key.encode(), dev_src, dev_dst,
                                            fn, reps))
    if t < 0:
        raise RuntimeError(f"oracle_host_bounce_time failed ({t})")
    return t


def pattern_source(family: int, dt: int, pe: int, nelems: int) -> np.ndarray:
    out = np.zeros(nelems, dtype=NP[dt])
    if lib().oracle_pattern_source(family, dt, pe, nelems, out.ctypes.data):
        raise ValueError("bad pattern")
    return out


def pattern_check(family: int, op: int, dt: int, npes: int, nelems: int) -> np.ndarray:
    out = np.zeros(nelems, dtype=NP[dt])
    if lib().oracle_pattern_check(family, op, dt, npes, nelems, out.ctypes.data):
        raise ValueError("bad pattern")
    return out


def family_for(op: int) -> int:
    return {0: PAT_AND, 1: PAT_OR, 2: PAT_XOR}.get(op, PAT_ARITH)


def fill_random(dt: int, seed: int, n: int, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    out = np.zeros(n, dtype=NP[dt])
    lib().oracle_fill_random(dt, seed, lo, hi, n, out.ctypes.data)
    return out


def fp_tolerance(dt: int, op: int, srcs: list[np.ndarray], ref: np.ndarray) -> np.ndarray:
    """Order-independent error bound for FP sum/prod of p terms (SURVEY.md §8c parity rule):
    sum: (p-1) * u * sum_i |x_i|;  prod: (p-1) * u * |ref| * (1 + tiny);  u = 2^-24 / 2^-53.
    Any summation order of the p terms stays within it, so it covers MPICH's order, the
    reference's per-PE order and the HIP path's canonical order alike."""
    p = len(srcs)
    u = 2.0 ** -24 if dt == DTYPES["float"] else 2.0 ** -53
    if op == OPS["sum"]:
        mag = np.sum([np.abs(s.astype(np.float64)) for s in srcs], axis=0)
        return (p - 1) * u * mag * 1.0001 + np.finfo(np.float64).tiny
    if op == OPS["prod"]:
        return (p - 1) * u * np.abs(ref.astype(np.float64)) * 1.0001 + np.finfo(np.float64).tiny
    return np.zeros(ref.shape)


# ---- fcollect / collect / scan ----------------------------------------
def scan_fold(dt: int, srcs: list[np.ndarray], me: int, inclusive: bool) -> np.ndarray:
    """Team-order prefix sum for PE `me`: the proxy hands the request to MPI_Scan / MPI_Exscan
    with MPI_SUM (src/runtime/runtime_mpi.cpp:815-835); integers wrap (two's complement), floats
    fold linearly x0+x1+...  Exscan on the first PE yields 0 (test/unit/exscan.cpp:52 checks 0)."""
    t = NP[dt]
    out = np.zeros_like(np.asarray(srcs[0], dtype=t))
    last = me + 1 if inclusive else me
    with np.errstate(over="ignore"):
        for k in range(last):
            out = np.asarray(srcs[k], dtype=t).copy() if k == 0 else (out + np.asarray(srcs[k], dtype=t)).astype(t)
    return out


def _words(nbytes: int) -> np.ndarray:
    return np.arange(nbytes // 8 + 1, dtype=np.int64)


def scan_pattern_source(pe: int, nbytes: int) -> np.ndarray:
    """test/unit/inscan.cpp / exscan.cpp:30-43: long word idx = pe + idx; first nbytes bytes."""
    w = (pe + _words(nbytes)).astype(np.int64)
    return w.view(np.uint8)[:nbytes].copy()


def scan_pattern_check(pe: int, nbytes: int, inclusive: bool) -> np.ndarray:
    """inscan.cpp:46-58 ((pe+i)(pe+i+1)/2 - i(i-1)/2) and exscan.cpp:46-59 ((pe+i)(pe+i-1)/2 -
    i(i-1)/2), evaluated on 64-bit words like the tester."""
    i = _words(nbytes)
    a = pe + i
    w = (a * (a + 1) // 2 if inclusive else a * (a - 1) // 2) - (i * (i - 1)) // 2
    return w.astype(np.int64).view(np.uint8)[:nbytes].copy()


def collect_pattern_source(pe: int, nelems: int, elem_size: int) -> np.ndarray:
    """test/unit/fcollect.cpp:48-62 / collect.cpp:68-82: word idx =
    (nelems<<48) + ((0x80+pe)<<40) + (0xff<<32) + idx; first nelems*elem_size bytes."""
    nbytes = nelems * elem_size
    i = _words(nbytes).astype(np.uint64)
    w = (np.uint64(nelems) << np.uint64(48)) + (np.uint64(0x80 + pe) << np.uint64(40)) + \
        (np.uint64(0xff) << np.uint64(32)) + i
    return w.view(np.uint8)[:nbytes].copy()


def collect_check(counts: list[int], elem_size: int) -> np.ndarray:
    """test/unit/collect.cpp:85-107 (fcollect.cpp the equal-count case): the members' source
    patterns concatenated in team order."""
    return np.concatenate([collect_pattern_source(pe, c, elem_size) for pe, c in enumerate(counts)]
                          + [np.zeros(0, np.uint8)])
