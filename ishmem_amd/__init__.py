"""ishmem_amd — MI355X-native reduction collective with the ishmem API surface.

Python host mirror of the reference's reduce interface (oneapi-src/ishmem v1.5.1,
src/ishmem.h:923-1238, src/ishmemx.h:1172-1803) over the C-ABI in include/ishmem_capi.h.
Names, argument meaning and error behaviour follow the reference: every
``ishmem_<TYPENAME>_<op>_reduce([team,] dest, source, nreduce)`` returns 0 on success and
nonzero on failure (``last_error()`` says why); ``dest``/``source`` are device addresses (ints)
from ``ishmem_malloc`` (symmetric heap) or any device / host address.

The work is done by ishmem_amd/libishmem_amd.so (HIP kernels for gfx950).  There is no Python
or CPU fallback: importing this package fails if the native library cannot be loaded.
"""
from __future__ import annotations

import ctypes
import sys

from ._lib import LIB_PATH, load

_L = load()

# ---- enums (include/ishmem_capi.h) -------------------------------------------------------
OPS = {"and": 0, "or": 1, "xor": 2, "max": 3, "min": 4, "sum": 5, "prod": 6}
DTYPES = {"int8": 0, "int16": 1, "int32": 2, "int64": 3, "uint8": 4, "uint16": 5,
          "uint32": 6, "uint64": 7, "float": 8, "double": 9}
ISHMEM_TEAM_INVALID = -1
ISHMEM_TEAM_WORLD = 0
ISHMEM_TEAM_SHARED = 1
ISHMEMX_TEAM_NODE = 2

# Reference TYPENAME -> canonical fixed-width type (x86-64 / gfx950 LP64, char signed).
# Instantiation lists: src/collectives/reduce.cpp:95-417.
TYPENAMES = {
    "char": "int8", "schar": "int8", "short": "int16", "int": "int32", "long": "int64",
    "longlong": "int64", "ptrdiff": "int64", "uchar": "uint8", "ushort": "uint16",
    "uint": "uint32", "ulong": "uint64", "ulonglong": "uint64", "int8": "int8",
    "int16": "int16", "int32": "int32", "int64": "int64", "uint8": "uint8", "uint16": "uint16",
    "uint32": "uint32", "uint64": "uint64", "size": "uint64", "float": "float", "double": "double",
}
BITWISE_TYPENAMES = ["uchar", "ushort", "uint", "ulong", "ulonglong", "int8", "int16", "int32",
                     "int64", "uint8", "uint16", "uint32", "uint64", "size"]
ARITH_TYPENAMES = ["char", "schar", "short", "int", "long", "longlong", "ptrdiff", "uchar",
                   "ushort", "uint", "ulong", "ulonglong", "int8", "int16", "int32", "int64",
                   "uint8", "uint16", "uint32", "uint64", "size", "float", "double"]
TYPENAMES_FOR_OP = {**{op: BITWISE_TYPENAMES for op in ("and", "or", "xor")},
                    **{op: ARITH_TYPENAMES for op in ("max", "min", "sum", "prod")}}


def lib() -> ctypes.CDLL:
    return _L


def last_error() -> str:
    e = _L.ishmemi_c_last_error()
    return e.decode() if e else ""


def version() -> str:
    return _L.ishmemi_c_version().decode()


# ---- lifecycle ---------------------------------------------------------------------------
def ishmem_init() -> None:
    """ishmem_init (src/ishmem.h:40): PE identity from the launcher (ISHMEM_PE / ISHMEM_NPES,
    torchrun, MPICH hydra / Intel MPI PMI_*, Open MPI OMPI_COMM_WORLD_*, srun SLURM_*; see
    launch_info)."""
    if _L.ishmemi_c_init() != 0:
        raise RuntimeError(f"ishmem_init failed: {last_error()}")


def launch_info() -> dict:
    """What ishmem_init would use, without touching the GPU: pe, npes, device, launcher, key."""
    pe, npes, dev = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    launcher, key = ctypes.create_string_buffer(32), ctypes.create_string_buffer(256)
    rc = _L.ishmemi_c_launch_info(ctypes.byref(pe), ctypes.byref(npes), ctypes.byref(dev), launcher, 32, key, 256)
    if rc != 0:
        raise RuntimeError(f"ishmem launch identity refused: {last_error()}")
    return {"pe": pe.value, "npes": npes.value, "device": dev.value, "launcher": launcher.value.decode(),
            "key": key.value.decode()}


def init(pe: int = 0, npes: int = 1, device: int = -1, key: str | None = None) -> None:
    """Explicit-identity init (ishmemx_init_attr analogue, src/ishmemx.h:21-37)."""
    if _L.ishmemi_c_init_pe(pe, npes, device, (key or "").encode()) != 0:
        raise RuntimeError(f"ishmem init failed: {last_error()}")


def ishmem_init_thread(requested: int) -> tuple[int, int]:
    """ishmem_init_thread (src/ishmem.h:44): returns (status, provided); always
    ISHMEM_THREAD_MULTIPLE (src/ishmem.cpp:409-419)."""
    prov = ctypes.c_int(-1)
    r = _L.ishmemi_c_init_thread(requested, ctypes.byref(prov))
    return r, prov.value


def ishmem_query_thread() -> int:
    prov = ctypes.c_int(-1)
    _L.ishmemi_c_query_thread(ctypes.byref(prov))
    return prov.value


ISHMEM_THREAD_SINGLE, ISHMEM_THREAD_FUNNELED, ISHMEM_THREAD_SERIALIZED, ISHMEM_THREAD_MULTIPLE = 0, 1, 2, 3
ISHMEM_MAJOR_VERSION, ISHMEM_MINOR_VERSION = 1, 5
ISHMEM_VENDOR_STRING = "ishmem_amd (AMD Instinct MI355X, HIP)"
ISHMEM_TEAM_NUM_CONTEXTS = 1


def ishmem_info_get_version() -> tuple[int, int]:
    """(major, minor) of the reference API implemented (src/ishmem.h:17-18, :57)."""
    return ISHMEM_MAJOR_VERSION, ISHMEM_MINOR_VERSION


def ishmem_info_get_name() -> str:
    return ISHMEM_VENDOR_STRING


def ishmem_finalize() -> None:
    _L.ishmemi_c_finalize()


finalize = ishmem_finalize


def initialized() -> bool:
    return bool(_L.ishmemi_c_initialized())


def ishmem_my_pe() -> int:
    return _L.ishmemi_c_my_pe()


def ishmem_n_pes() -> int:
    return _L.ishmemi_c_n_pes()


# ---- symmetric heap ----------------------------------------------------------------------
def ishmem_malloc(size: int) -> int:
    p = _L.ishmemi_c_malloc(size)
    if not p:
        raise MemoryError(f"ishmem_malloc({size}) failed: {last_error()}")
    return p


def ishmem_align(alignment: int, size: int) -> int:
    p = _L.ishmemi_c_align(alignment, size)
    if not p:
        raise MemoryError(f"ishmem_align failed: {last_error()}")
    return p


def ishmem_calloc(count: int, size: int) -> int:
    p = _L.ishmemi_c_calloc(count, size)
    if not p:
        raise MemoryError(f"ishmem_calloc failed: {last_error()}")
    return p


def ishmem_free(ptr: int) -> None:
    _L.ishmemi_c_free(ptr)


def ishmem_ptr(dest: int, pe: int) -> int | None:
    return _L.ishmemi_c_ptr(dest, pe)


# ---- teams / sync ------------------------------------------------------------------------
def ishmem_team_my_pe(team: int) -> int:
    return _L.ishmemi_c_team_my_pe(team)


def ishmem_team_n_pes(team: int) -> int:
    return _L.ishmemi_c_team_n_pes(team)


def ishmem_team_translate_pe(src_team: int, src_pe: int, dest_team: int) -> int:
    return _L.ishmemi_c_team_translate_pe(src_team, src_pe, dest_team)


def ishmem_team_split_strided(parent: int, start: int, stride: int, size: int) -> tuple[int, int]:
    """Returns (status, new_team) — new_team is ISHMEM_TEAM_INVALID on non-members."""
    t = ctypes.c_int(-1)
    r = _L.ishmemi_c_team_split_strided(parent, start, stride, size, ctypes.byref(t))
    return r, t.value


def ishmem_team_split_2d(parent: int, xrange: int) -> tuple[int, int, int]:
    """Returns (status, xaxis_team, yaxis_team) (src/teams.cpp:453-518)."""
    x, y = ctypes.c_int(-1), ctypes.c_int(-1)
    r = _L.ishmemi_c_team_split_2d(parent, xrange, ctypes.byref(x), ctypes.byref(y))
    return r, x.value, y.value


def ishmem_team_destroy(team: int) -> None:
    _L.ishmemi_c_team_destroy(team)


def ishmem_team_get_config(team: int, config_mask: int = ISHMEM_TEAM_NUM_CONTEXTS) -> tuple[int, int]:
    """(status, num_contexts) (src/ishmem.h:78, src/teams.cpp:545-570)."""
    n = ctypes.c_int(0)
    r = _L.ishmemi_c_team_get_config(team, config_mask, ctypes.byref(n))
    return r, n.value


def ishmem_barrier_all() -> int:
    return _L.ishmemi_c_barrier_all()


def resync() -> int:
    """After a device-side timeout: all PEs agree on every team's epoch again (collective)."""
    return _L.ishmemi_c_resync()


def ishmem_sync_all() -> int:
    return _L.ishmemi_c_sync_all()


def ishmem_team_sync(team: int) -> int:
    return _L.ishmemi_c_team_sync(team)


def set_param(name: str, value: int) -> int:
    return _L.ishmemi_c_set_param(name.encode(), int(value))


def chunk_bounds(nitems: int, npes: int, c: int) -> tuple[int, int]:
    """Member c's [begin, end) of the multi-PE partition of `nitems` 16-B items (test hook)."""
    b, e = ctypes.c_uint64(0), ctypes.c_uint64(0)
    if _L.ishmemi_c_chunk_bounds(nitems, npes, c, ctypes.byref(b), ctypes.byref(e)):
        raise ValueError("chunk_bounds: invalid arguments")
    return b.value, e.value


def get_param(name: str) -> int:
    return int(_L.ishmemi_c_get_param(name.encode()))


# ---- the reduction path ------------------------------------------------------------------
def reduce(op: str, dtype: str, dest: int, source: int, nreduce: int, team: int = ISHMEM_TEAM_WORLD) -> int:
    """ishmemi_reduce<T,OP>(team, dest, source, nreduce) (src/collectives/reduce_impl.h:259-317)."""
    return _L.ishmemi_c_reduce(team, OPS[op], DTYPES[dtype], dest, source, nreduce)


def _event_handle(e) -> int | None:
    return getattr(e, "h", e) or None


def reduce_on_stream(op: str, dtype: str, dest: int, source: int, nreduce: int, ret: int | None,
                     stream: int, team: int = ISHMEM_TEAM_WORLD, deps=(), done=None) -> int:
    """ishmemx_*_reduce_on_queue analogue (src/collectives/reduce_impl.h:444-474).  `deps`: HIP
    events (hip.Event or raw handles) the call waits for, as the reference's `deps`; `done`: an
    event recorded after the call, as the sycl::event the reference returns."""
    if deps or done is not None:
        hs = [_event_handle(e) for e in deps]
        arr = (ctypes.c_void_p * len(hs))(*hs) if hs else None
        return _L.ishmemi_c_reduce_on_stream_deps(team, OPS[op], DTYPES[dtype], dest, source, nreduce,
                                                  ret or None, stream or None, arr, len(hs),
                                                  _event_handle(done))
    return _L.ishmemi_c_reduce_on_stream(team, OPS[op], DTYPES[dtype], dest, source, nreduce,
                                         ret or None, stream or None)


def combine(op: str, dtype: str, dst: int, srcs: list[int], n: int, stream: int = 0) -> int:
    """Local combine unit dst = op(srcs...) (vector_reduce, reduce_impl.h:105-183)."""
    arr = (ctypes.c_void_p * len(srcs))(*srcs)
    return _L.ishmemi_c_combine(OPS[op], DTYPES[dtype], dst, arr, len(srcs), n, stream or None)


def pull_probe(dst: int, srcs: list[int], nbytes: int, policy: int, stream: int = 0) -> int:
    """xGMI measurement hook: dst = sum of f32 srcs, loads with cache policy 0 = nt, 1 = sc0 sc1."""
    arr = (ctypes.c_void_p * len(srcs))(*srcs)
    return _L.ishmemi_c_pull_probe(dst, arr, len(srcs), nbytes, policy, stream or None)


def occupy(grid: int, usec: int, stream: int = 0) -> int:
    """Test hook: `grid` workgroups that each hold half a CU for `usec` microseconds."""
    return _L.ishmemi_c_occupy(grid, usec, stream or None)


def _make_blocking(op: str, dt: str):
    def fn(*args):
        # Overloads of the reference: (dest, source, nreduce) and (team, dest, source, nreduce).
        if len(args) == 3:
            team, (dest, source, n) = ISHMEM_TEAM_WORLD, args
        elif len(args) == 4:
            team, dest, source, n = args
        else:
            raise TypeError("expected ([team,] dest, source, nreduce)")
        return _L.ishmemi_c_reduce(team, OPS[op], DTYPES[dt], dest, source, n)
    return fn


def _make_on_stream(op: str, dt: str):
    def fn(*args):
        if len(args) == 5:
            team, (dest, source, n, ret, stream) = ISHMEM_TEAM_WORLD, args
        elif len(args) == 6:
            team, dest, source, n, ret, stream = args
        else:
            raise TypeError("expected ([team,] dest, source, nreduce, ret, stream)")
        return _L.ishmemi_c_reduce_on_stream(team, OPS[op], DTYPES[dt], dest, source, n,
                                             ret or None, stream or None)
    return fn


# ---- fcollect / collect / scan (src/collectives/collect.cpp, scan.cpp) --
def ishmem_fcollectmem(*args) -> int:
    """ishmem_fcollectmem([team,] dest, source, nbytes) -> int (bytes per PE)."""
    team, (dest, source, n) = (ISHMEM_TEAM_WORLD, args) if len(args) == 3 else (args[0], args[1:])
    return _L.ishmemi_c_fcollect(team, dest, source, n)


def ishmem_collectmem(*args) -> int:
    """ishmem_collectmem([team,] dest, source, nbytes) -> int (nbytes may differ per PE)."""
    team, (dest, source, n) = (ISHMEM_TEAM_WORLD, args) if len(args) == 3 else (args[0], args[1:])
    return _L.ishmemi_c_collect(team, dest, source, n)


def collect_on_stream(dest: int, source: int, nbytes: int, ret: int | None, stream: int,
                      team: int = ISHMEM_TEAM_WORLD) -> int:
    """ishmemx_collectmem_on_queue analogue: nbytes may differ per PE; counts meet on the device."""
    return _L.ishmemi_c_collect_on_stream(team, dest, source, nbytes, ret or None, stream or None)


def fcollect_on_stream(dest: int, source: int, nbytes: int, ret: int | None, stream: int,
                       team: int = ISHMEM_TEAM_WORLD) -> int:
    return _L.ishmemi_c_fcollect_on_stream(team, dest, source, nbytes, ret or None, stream or None)


def ishmem_broadcastmem(*args) -> int:
    """ishmem_broadcastmem([team,] dest, source, nbytes, root) -> int (src/ishmem.h:786, :813)."""
    team, (dest, source, n, root) = (ISHMEM_TEAM_WORLD, args) if len(args) == 4 else (args[0], args[1:])
    return _L.ishmemi_c_broadcast(team, dest, source, n, root)


def broadcast_on_stream(dest: int, source: int, nbytes: int, root: int, ret: int | None, stream: int,
                        team: int = ISHMEM_TEAM_WORLD) -> int:
    """ishmemx_broadcastmem_on_queue analogue: symmetric source, the root's bytes into every dest."""
    return _L.ishmemi_c_broadcast_on_stream(team, dest, source, nbytes, root, ret or None, stream or None)


def team_sync_on_stream(team: int, ret: int | None, stream: int) -> int:
    """ishmemx_team_sync_on_queue analogue (src/ishmemx.h:2235)."""
    return _L.ishmemi_c_team_sync_on_stream(team, ret or None, stream or None)


def scan(dtype: str, inclusive: bool, dest: int, source: int, nelems: int,
         team: int = ISHMEM_TEAM_WORLD) -> int:
    return _L.ishmemi_c_scan(team, DTYPES[dtype], 1 if inclusive else 0, dest, source, nelems)


def _make_coll(kind: str, dt: str, size: int):
    def fn(*args):
        if kind == "broadcast":  # ([team,] dest, source, nelems, root)
            team, (dest, source, n, root) = (ISHMEM_TEAM_WORLD, args) if len(args) == 4 else (args[0], args[1:])
            return _L.ishmemi_c_broadcast(team, dest, source, n * size, root)
        team, (dest, source, n) = (ISHMEM_TEAM_WORLD, args) if len(args) == 3 else (args[0], args[1:])
        if kind == "fcollect":
            return _L.ishmemi_c_fcollect(team, dest, source, n * size)
        if kind == "collect":
            return _L.ishmemi_c_collect(team, dest, source, n * size)
        return _L.ishmemi_c_scan(team, DTYPES[dt], 1 if kind == "inscan" else 0, dest, source, n)
    return fn


_SIZES = {"int8": 1, "uint8": 1, "int16": 2, "uint16": 2, "int32": 4, "uint32": 4, "float": 4,
          "int64": 8, "uint64": 8, "double": 8}

_mod = sys.modules[__name__]
for _tn in ARITH_TYPENAMES:  # the reference's fcollect / collect / scan lists = these 23 names
    for _kind, _name in (("fcollect", f"ishmem_{_tn}_fcollect"), ("collect", f"ishmem_{_tn}_collect"),
                         ("inscan", f"ishmem_{_tn}_sum_inscan"), ("exscan", f"ishmem_{_tn}_sum_exscan"),
                         ("broadcast", f"ishmem_{_tn}_broadcast")):
        _f = _make_coll(_kind, TYPENAMES[_tn], _SIZES[TYPENAMES[_tn]])
        _f.__name__ = _name
        setattr(_mod, _name, _f)
del _tn, _kind, _name, _f
API_NAMES: list[str] = []
for _op, _tns in TYPENAMES_FOR_OP.items():
    for _tn in _tns:
        _name = f"ishmem_{_tn}_{_op}_reduce"
        _f = _make_blocking(_op, TYPENAMES[_tn])
        _f.__name__ = _name
        _f.__doc__ = f"{_name}([team,] dest, source, nreduce) -> int  (src/ishmem.h reduce section)"
        setattr(_mod, _name, _f)
        _xname = f"ishmemx_{_tn}_{_op}_reduce_on_stream"
        _g = _make_on_stream(_op, TYPENAMES[_tn])
        _g.__name__ = _xname
        setattr(_mod, _xname, _g)
        API_NAMES += [_name, _xname]
del _op, _tns, _tn, _name, _f, _xname, _g
