#!/usr/bin/env python3
"""Host-memory end-to-end rate of one PE's reduce (dev tool, round 3): 1 GiB f32 from host source
to host dest through the staged pipeline, pinned and pageable buffers, every word checked.
Run once per ISHMEM_STAGING_SLOTS / ISHMEM_STAGING_SIZE setting; prints one JSON line."""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def main() -> None:
    import ishmem_amd as ish
    from ishmem_amd import hip
    ish.init(0, 1, 0, None)
    n = (1 << 30) // 4
    B = 4 * n
    st = hip.stream_create()
    out = {"slots": ish.get_param("staging_slots"), "staging_MiB": ish.get_param("staging_bytes") >> 20}
    L = hip.lib()
    L.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    L.hipHostUnregister.argtypes = [ctypes.c_void_p]
    for kind in ("pinned", "pageable", "pageable_app_registered"):
        if kind == "pinned":
            hs, hd = hip.host_malloc(B), hip.host_malloc(B)
            xs = np.ctypeslib.as_array((ctypes.c_float * n).from_address(hs))
            xd = np.ctypeslib.as_array((ctypes.c_float * n).from_address(hd))
        else:
            xs, xd = np.zeros(n, np.float32), np.zeros(n, np.float32)
            hs, hd = xs.ctypes.data, xd.ctypes.data
        if kind == "pageable_app_registered":
            out["app_register_rc"] = [L.hipHostRegister(hs, B, 0), L.hipHostRegister(hd, B, 0)]
        xs[:] = np.arange(n, dtype=np.float32)
        ts = []
        for rep in range(4):
            xd.fill(-1)
            t0 = time.perf_counter()
            if ish.ishmemx_float_sum_reduce_on_stream(hd, hs, n, 0, st) != 0:
                raise RuntimeError(ish.last_error())
            hip.stream_synchronize(st)
            ts.append(time.perf_counter() - t0)
            if not np.array_equal(xd, xs):
                raise RuntimeError(f"{kind}: dest differs")
        out[kind] = {"GiBps_best": round(B / (1 << 30) / min(ts[1:]), 2),
                     "GiBps_median": round(B / (1 << 30) / sorted(ts[1:])[1], 2), "first_ms": round(ts[0] * 1e3, 1)}
        # back to back: 4 calls enqueued on the stream, one synchronisation (the bench's shape)
        t0 = time.perf_counter()
        for _ in range(4):
            if ish.ishmemx_float_sum_reduce_on_stream(hd, hs, n, 0, st) != 0:
                raise RuntimeError(ish.last_error())
        hip.stream_synchronize(st)
        out[kind]["back_to_back_GiBps"] = round(4 * B / (1 << 30) / (time.perf_counter() - t0), 2)
        if kind == "pinned":
            del xs, xd
            hip.host_free(hs)
            hip.host_free(hd)
        if kind == "pageable_app_registered":
            L.hipHostUnregister(hs)
            L.hipHostUnregister(hd)
    print(json.dumps(out), flush=True)
    ish.ishmem_finalize()


if __name__ == "__main__":
    main()
