#!/usr/bin/env python3
"""Host-memory leg, one process, interleaved A/B: why did the driver's bench
measure 34.7 GiB/s for application-pinned (hipHostMalloc) buffers against 42.8 GiB/s for malloc'd
buffers the library page-locks itself?  The same 1 GiB f32 sum at 1 PE (the reference's host path,
reduce_impl.h:186-228, :301-315 — here the staged pipeline, runtime.cpp reduce_staged) over four
kinds of host buffer, rounds interleaved A B C D A B C D ...:

  hostmalloc      hipHostMalloc(flags 0)                      what the bench's pinned leg uses
  hostmalloc_nc   hipHostMalloc(hipHostMallocNonCoherent)
  registered      malloc'd numpy + hipHostRegister by the caller (the library sees pinned memory)
  pageable        malloc'd numpy (the library page-locks it for each call)

For each buffer kind and round: the pipeline's end-to-end rate (4 calls, as the bench's e2e leg,
blocking calls and on-stream calls) and the DMA engines' rate on the SAME buffers (hipMemcpyAsync
1 GiB host -> HBM and HBM -> host at once on two streams, as the bench's pcie_probe).  Every word of
dest is checked.  One JSON line per measurement, then a summary line.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time
import uuid
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

GiB = 1 << 30
B = GiB
N = B // 4
HIP_HOST_MALLOC_NONCOHERENT = 0x80000000


def main() -> None:
    import ishmem_amd as ish
    from ishmem_amd import hip
    L = hip.lib()
    L.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    L.hipHostUnregister.argtypes = [ctypes.c_void_p]
    L.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    ish.init(0, 1, 0, f"hf{uuid.uuid4().hex[:8]}")
    st = hip.stream_create()
    d1, d2 = hip.malloc(B), hip.malloc(B)
    s1, s2 = hip.stream_create(), hip.stream_create()
    rounds = int(os.environ.get("AB_ROUNDS", "3"))

    def hostmalloc(flags):
        p = ctypes.c_void_p()
        rc = L.hipHostMalloc(ctypes.byref(p), B, flags)
        if rc != 0:
            raise RuntimeError(f"hipHostMalloc flags {flags:#x}: {rc}")
        return p.value, np.ctypeslib.as_array((ctypes.c_float * N).from_address(p.value))

    bufs = {}
    kinds = os.environ.get("AB_KINDS", "hostmalloc,hostmalloc_nc,registered,pageable").split(",")
    for kind in kinds:
        pair = []
        for _ in range(2):
            if kind == "hostmalloc":
                pair.append(hostmalloc(0))
            elif kind == "hostmalloc_nc":
                pair.append(hostmalloc(HIP_HOST_MALLOC_NONCOHERENT))
            else:
                a = np.zeros(N, np.float32)
                if kind == "registered":
                    rc = L.hipHostRegister(a.ctypes.data, B, 0)
                    if rc != 0:
                        raise RuntimeError(f"hipHostRegister: {rc}")
                pair.append((a.ctypes.data, a))
        bufs[kind] = pair
    src_vals = (np.arange(N, dtype=np.int64) % 1021).astype(np.float32)
    for kind, ((ps, xs), (pd, xd)) in bufs.items():
        xs[:] = src_vals

    def e2e(kind, on_stream):
        (ps, xs), (pd, xd) = bufs[kind]
        call = (lambda: ish.ishmemx_float_sum_reduce_on_stream(pd, ps, N, 0, st)) if on_stream else \
            (lambda: ish.ishmem_float_sum_reduce(pd, ps, N))
        if call() != 0:
            raise RuntimeError(ish.last_error())
        hip.stream_synchronize(st)
        xd.fill(-1.0)
        k = 4
        t0 = time.perf_counter()
        for _ in range(k):
            if call() != 0:
                raise RuntimeError(ish.last_error())
        hip.stream_synchronize(st)
        dt = (time.perf_counter() - t0) / k
        ok = bool(np.array_equal(xd.view(np.uint32), xs.view(np.uint32)))  # 1 PE: reduce = copy
        return B / GiB / dt, ok

    def dma(kind):
        (ps, _), (pd, _) = bufs[kind]
        for _ in range(2):
            hip.memcpy_async(d1, ps, B, s1)
            hip.memcpy_async(pd, d2, B, s2)
            hip.stream_synchronize(s1)
            hip.stream_synchronize(s2)
        t0 = time.perf_counter()
        for _ in range(2):
            hip.memcpy_async(d1, ps, B, s1)
            hip.memcpy_async(pd, d2, B, s2)
        hip.stream_synchronize(s1)
        hip.stream_synchronize(s2)
        return B / ((time.perf_counter() - t0) / 2) / 1e9

    if os.environ.get("AB_MODE") == "warmup":
        # Fresh buffers of each kind, then 10 single on-stream calls in a row: does the rate of
        # application-pinned buffers change with use (first DMA passes over new pages)?
        for kind in [k for k in ("hostmalloc", "registered", "pageable", "hostmalloc") if k in bufs]:
            (ps, xs), (pd, xd) = bufs[kind]
            if kind.startswith("hostmalloc"):  # replace by fresh allocations
                for p, _ in bufs[kind]:
                    hip.host_free(p)
                bufs[kind] = [hostmalloc(0), hostmalloc(0)]
                (ps, xs), (pd, xd) = bufs[kind]
                xs[:] = src_vals
            rates = []
            for it in range(10):
                t0 = time.perf_counter()
                if ish.ishmemx_float_sum_reduce_on_stream(pd, ps, N, 0, st) != 0:
                    raise RuntimeError(ish.last_error())
                hip.stream_synchronize(st)
                rates.append(round(B / GiB / (time.perf_counter() - t0), 2))
            print(json.dumps({"warmup": kind, "GiBps_per_call": rates, "dma_after_GBps": round(dma(kind), 2)}),
                  flush=True)
        ish.ishmem_finalize()
        return
    res = {k: {"blocking": [], "on_stream": [], "dma_concurrent_GBps": []} for k in bufs}
    for rnd in range(rounds):
        for kind in bufs:
            blk, ok1 = e2e(kind, False)
            ons, ok2 = e2e(kind, True)
            dm = dma(kind)
            res[kind]["blocking"].append(round(blk, 2))
            res[kind]["on_stream"].append(round(ons, 2))
            res[kind]["dma_concurrent_GBps"].append(round(dm, 2))
            print(json.dumps({"round": rnd, "kind": kind, "staged_copy_kernel": int(ish.get_param("staged_copy_kernel")), "blocking_GiBps": round(blk, 2),
                              "on_stream_GiBps": round(ons, 2), "dma_concurrent_GBps": round(dm, 2),
                              "pipeline_each_way_GBps": round(ons * GiB / 1e9, 2), "checked": ok1 and ok2}),
                  flush=True)
    summary = {k: {m: {"median": float(np.median(v)), "min": min(v), "max": max(v)} for m, v in r.items()}
               for k, r in res.items()}
    for k in summary:
        summary[k]["frac_of_dma"] = round(np.median(res[k]["on_stream"]) * GiB / 1e9 /
                                          np.median(res[k]["dma_concurrent_GBps"]), 3)
    print(json.dumps({"summary": summary}), flush=True)
    for kind, pair in bufs.items():
        for p, arr in pair:
            if kind.startswith("hostmalloc"):
                hip.host_free(p)
            elif kind == "registered":
                L.hipHostUnregister(p)
    ish.ishmem_finalize()


if __name__ == "__main__":
    main()
