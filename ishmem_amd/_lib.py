"""Loader of the native library (ishmem_amd/libishmem_amd.so) with C-ABI prototypes.

The product path is this library and nothing else: if it cannot be loaded the import fails
loudly (there is no Python / CPU fallback).
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libishmem_amd.so"
# A/B measurements only: ISHMEM_AMD_LIB names a variant build of the same library
# (python -m ishmem_amd._build --define ... --out build/ab/<name>.so); never set for results.
_VARIANT = os.environ.get("ISHMEM_AMD_LIB")

# (name, restype, argtypes) for every symbol declared in include/ishmem_capi.h.
_vp, _i, _sz, _ll, _u64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_longlong, ctypes.c_uint64
PROTOTYPES = [
    ("ishmemi_c_init", _i, []),
    ("ishmemi_c_init_pe", _i, [_i, _i, _i, ctypes.c_char_p]),
    ("ishmemi_c_launch_info", _i, [ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.POINTER(_i), ctypes.c_char_p, _sz,
                                   ctypes.c_char_p, _sz]),
    ("ishmemi_c_finalize", _i, []),
    ("ishmemi_c_initialized", _i, []),
    ("ishmemi_c_my_pe", _i, []),
    ("ishmemi_c_n_pes", _i, []),
    ("ishmemi_c_device", _i, []),
    ("ishmemi_c_init_thread", _i, [_i, ctypes.POINTER(_i)]),
    ("ishmemi_c_query_thread", _i, [ctypes.POINTER(_i)]),
    ("ishmemi_c_malloc", _vp, [_sz]),
    ("ishmemi_c_align", _vp, [_sz, _sz]),
    ("ishmemi_c_calloc", _vp, [_sz, _sz]),
    ("ishmemi_c_free", None, [_vp]),
    ("ishmemi_c_ptr", _vp, [_vp, _i]),
    ("ishmemi_c_heap_info", _i, [ctypes.POINTER(_vp), ctypes.POINTER(_sz), ctypes.POINTER(_sz)]),
    ("ishmemi_c_team_my_pe", _i, [_i]),
    ("ishmemi_c_team_n_pes", _i, [_i]),
    ("ishmemi_c_team_translate_pe", _i, [_i, _i, _i]),
    ("ishmemi_c_team_split_strided", _i, [_i, _i, _i, _i, ctypes.POINTER(_i)]),
    ("ishmemi_c_team_split_2d", _i, [_i, _i, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    ("ishmemi_c_team_destroy", None, [_i]),
    ("ishmemi_c_team_get_config", _i, [_i, ctypes.c_long, ctypes.POINTER(_i)]),
    ("ishmemi_c_team_set_config", _i, [_i, ctypes.c_long, _i]),
    ("ishmemi_c_barrier_all", _i, []),
    ("ishmemi_c_sync_all", _i, []),
    ("ishmemi_c_team_sync", _i, [_i]),
    ("ishmemi_c_team_sync_on_stream", _i, [_i, _vp, _vp]),
    ("ishmemi_c_resync", _i, []),
    ("ishmemi_c_reduce", _i, [_i, _i, _i, _vp, _vp, _sz]),
    ("ishmemi_c_reduce_on_stream", _i, [_i, _i, _i, _vp, _vp, _sz, _vp, _vp]),
    ("ishmemi_c_reduce_on_stream_deps", _i, [_i, _i, _i, _vp, _vp, _sz, _vp, _vp, _vp, _sz, _vp]),
    ("ishmemi_c_combine", _i, [_i, _i, _vp, ctypes.POINTER(_vp), _i, _sz, _vp]),
    ("ishmemi_c_pull_probe", _i, [_vp, ctypes.POINTER(_vp), _i, _sz, _i, _vp]),
    ("ishmemi_c_occupy", _i, [_i, ctypes.c_ulonglong, _vp]),
    ("ishmemi_c_produce_u32", _i, [_vp, _vp, _vp, _sz, _vp]),
    ("ishmemi_c_fcollect", _i, [_i, _vp, _vp, _sz]),
    ("ishmemi_c_fcollect_on_stream", _i, [_i, _vp, _vp, _sz, _vp, _vp]),
    ("ishmemi_c_collect_on_stream", _i, [_i, _vp, _vp, _sz, _vp, _vp]),
    ("ishmemi_c_stream_wait_events", _i, [_vp, _vp, _sz]),
    ("ishmemi_c_stream_record_event", _i, [_vp, _vp]),
    ("ishmemi_c_collect", _i, [_i, _vp, _vp, _sz]),
    ("ishmemi_c_scan", _i, [_i, _i, _i, _vp, _vp, _sz]),
    ("ishmemi_c_scan_on_stream", _i, [_i, _i, _i, _vp, _vp, _sz, _vp, _vp]),
    ("ishmemi_c_broadcast", _i, [_i, _vp, _vp, _sz, _i]),
    ("ishmemi_c_broadcast_on_stream", _i, [_i, _vp, _vp, _sz, _i, _vp, _vp]),
    ("ishmemi_c_device_ctx", _vp, []),
    ("ishmemi_c_register_device_ctx_slot", _i, [_vp]),
    ("ishmemi_c_last_error", ctypes.c_char_p, []),
    ("ishmemi_c_set_param", _i, [ctypes.c_char_p, _ll]),
    ("ishmemi_c_get_param", _ll, [ctypes.c_char_p]),
    ("ishmemi_c_phase_times", _i, [ctypes.POINTER(ctypes.c_float)]),
    ("ishmemi_c_error_count", _i, []),
    ("ishmemi_c_dtype_size", _sz, [_i]),
    ("ishmemi_c_op_dtype_valid", _i, [_i, _i]),
    ("ishmemi_c_chunk_bounds", _i, [_u64, _i, _i, ctypes.POINTER(_u64), ctypes.POINTER(_u64)]),
    ("ishmemi_c_path_limits", _i, [_i, _i, ctypes.POINTER(_ll), ctypes.POINTER(_ll)]),
    ("ishmemi_c_bootstrap_selftest", _i, [_i, _i, ctypes.c_char_p, _i, ctypes.POINTER(_i)]),
    ("ishmemi_c_version", ctypes.c_char_p, []),
]

_lib = None


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    """Load (building in-tree first if needed) the native library."""
    global _lib
    if _lib is not None:
        return _lib
    if _VARIANT:
        lib = ctypes.CDLL(str(Path(_VARIANT).resolve()), mode=ctypes.RTLD_GLOBAL)
        for name, res, args in PROTOTYPES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib
    if build_if_missing:
        from . import _build
        if _build.needs_build():
            try:
                _build.build()
            except RuntimeError:
                if not LIB_PATH.exists():
                    raise
    if not LIB_PATH.exists():
        raise ImportError(f"ishmem_amd native library missing: {LIB_PATH} (run __graft_entry__.build())")
    lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    for name, res, args in PROTOTYPES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    _warn_foreign_runtime()
    return lib


def _warn_foreign_runtime() -> None:
    """torch ships its own HIP runtime under the image's soname; when torch was imported first, that
    copy serves this library too.  Every GPU test runs on the image's runtime, and the round-6 N > 1
    rehearsals stalled in the heap's IPC import on torch's copy, so say so once."""
    try:
        with open("/proc/self/maps") as f:
            foreign = any("amdhip64" in line and "/torch/lib/" in line for line in f)
    except OSError:
        return
    if foreign:
        import sys
        print("[ishmem_amd] WARN: the HIP runtime in use is torch's bundled copy (torch was imported "
              "before ishmem_amd); import ishmem_amd first so the image's runtime serves the process",
              file=sys.stderr, flush=True)
