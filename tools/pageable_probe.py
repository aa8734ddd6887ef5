#!/usr/bin/env python3
"""Host <-> HBM copy rates (dev tool, round 3): pageable (malloc'd numpy) and pinned
(hipHostMalloc) buffers, H2D alone, D2H alone, and both at once from two host threads (each
thread's hipMemcpyAsync on its own stream; pageable copies block the calling thread), plus the
cost of pinning a pageable buffer with hipHostRegister.  Decides the host-memory pipeline's shape
for pageable buffers."""
from __future__ import annotations

import ctypes
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from ishmem_amd import hip  # noqa: E402

B = 1 << 30
CH = 64 << 20


def main() -> None:
    L = hip.lib()
    d1, d2 = hip.malloc(B), hip.malloc(B)
    s1, s2 = hip.stream_create(), hip.stream_create()
    out = {}
    L.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    L.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    L.hipHostUnregister.argtypes = [ctypes.c_void_p]
    flags = {"pinned": 0, "pinned_noncoherent": 0x80000000, "pinned_coherent": 0x40000000,
             "pinned_numa_user": 0x20000000}
    for kind in ("pageable", "registered", *flags):
        keep = []
        if kind in ("pageable", "registered"):
            a, b = np.ones(B // 4, np.float32), np.zeros(B // 4, np.float32)
            ha, hb = a.ctypes.data, b.ctypes.data
            keep = [a, b]
            if kind == "registered":
                L.hipHostRegister(ha, B, 0)
                L.hipHostRegister(hb, B, 0)
        else:
            pa, pb = ctypes.c_void_p(), ctypes.c_void_p()
            if L.hipHostMalloc(ctypes.byref(pa), B, flags[kind]) or L.hipHostMalloc(ctypes.byref(pb), B, flags[kind]):
                out[kind] = "hipHostMalloc failed"
                continue
            ha, hb = pa.value, pb.value
            ctypes.memset(ha, 1, B)
            ctypes.memset(hb, 0, B)

        def h2d(chunk=CH):
            for off in range(0, B, chunk):
                hip.memcpy_async(d1 + off, ha + off, chunk, s1)
            hip.stream_synchronize(s1)

        def d2h(chunk=CH):
            for off in range(0, B, chunk):
                hip.memcpy_async(hb + off, d2 + off, chunk, s2)
            hip.stream_synchronize(s2)

        def timed(fn, reps=3):
            fn()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            return (time.perf_counter() - t0) / reps

        def both():
            t = threading.Thread(target=d2h)
            t.start()
            h2d()
            t.join()

        r = {"h2d_GBps": B / timed(h2d) / 1e9, "d2h_GBps": B / timed(d2h) / 1e9,
             "both_threads_GBps_each": B / timed(both) / 1e9}
        r["seq_GBps_each"] = B / timed(lambda: (h2d(), d2h())) / 1e9
        r["h2d_1GiB_GBps"] = B / timed(lambda: h2d(B)) / 1e9
        r["d2h_1GiB_GBps"] = B / timed(lambda: d2h(B)) / 1e9
        out[kind] = {k: round(v, 2) for k, v in r.items()}
        if kind in flags:
            hip.host_free(ha)
            hip.host_free(hb)
        elif kind == "registered":
            L.hipHostUnregister(ha)
            L.hipHostUnregister(hb)
        del keep
    # hipHostRegister / Unregister of a 1 GiB pageable buffer
    c = np.ones(B // 4, np.float32)
    reg, unreg = L.hipHostRegister, L.hipHostUnregister
    t0 = time.perf_counter()
    e = reg(c.ctypes.data, B, 0)
    t1 = time.perf_counter()
    e2 = unreg(c.ctypes.data)
    t2 = time.perf_counter()
    out["host_register_1GiB_ms"] = {"register": round((t1 - t0) * 1e3, 2), "unregister": round((t2 - t1) * 1e3, 2),
                                    "rc": [e, e2]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
