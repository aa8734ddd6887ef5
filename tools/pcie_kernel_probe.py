#!/usr/bin/env python3
"""Dev probe for the host-memory leg: what moves 1 GiB over PCIe fastest, and in
both directions at once?  The staged pipeline (runtime.cpp reduce_staged_pipeline) copies chunks in
(host -> HBM) and out (HBM -> host) with hipMemcpyAsync on two streams, i.e. on the DMA engines,
which give ~57 GB/s one way but ~48.6 GB/s each way when both run.  The alternative is a copy
KERNEL that reads or writes the pinned host buffer directly (the fan-in copy kernel, ishmemi_c_combine
with one source: 16-B nontemporal loads, write-through stores).  One process, pinned hipHostMalloc
buffers, best of 3 per case, GB/s per direction:

  dma_h2d, dma_d2h, dma_both          hipMemcpyAsync alone / both at once (the bench's pcie_probe)
  kern_h2d, kern_d2h                  the copy kernel reading host / writing host, alone
  dma_h2d+kern_d2h, kern_h2d+dma_d2h  one direction each way, concurrently on two streams
"""
from __future__ import annotations

import json
import os
import sys
import time
import uuid
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

B = 1 << 30


def main() -> None:
    import ishmem_amd as ish
    from ishmem_amd import hip
    ish.init(0, 1, 0, f"pk{uuid.uuid4().hex[:8]}")
    d1, d2 = hip.malloc(B), hip.malloc(B)
    hs, hd = hip.host_malloc(B), hip.host_malloc(B)
    s1, s2 = hip.stream_create(), hip.stream_create()
    n = B // 4

    def kcopy(dst, src, st):
        if ish.combine("sum", "float", dst, [src], n, st) != 0:
            raise RuntimeError(ish.last_error())

    jobs = {
        "dma_h2d": [lambda: hip.memcpy_async(d1, hs, B, s1)],
        "dma_d2h": [lambda: hip.memcpy_async(hd, d2, B, s2)],
        "dma_both": [lambda: hip.memcpy_async(d1, hs, B, s1), lambda: hip.memcpy_async(hd, d2, B, s2)],
        "kern_h2d": [lambda: kcopy(d1, hs, s1)],
        "kern_d2h": [lambda: kcopy(hd, d2, s2)],
        "dma_h2d+kern_d2h": [lambda: hip.memcpy_async(d1, hs, B, s1), lambda: kcopy(hd, d2, s2)],
        "kern_h2d+dma_d2h": [lambda: kcopy(d1, hs, s1), lambda: hip.memcpy_async(hd, d2, B, s2)],
        "kern_both": [lambda: kcopy(d1, hs, s1), lambda: kcopy(hd, d2, s2)],
    }
    out = {}
    for rnd in range(2):
        for name, fns in jobs.items():
            best = 0.0
            for k in range(4):
                t0 = time.perf_counter()
                for f in fns:
                    f()
                hip.stream_synchronize(s1)
                hip.stream_synchronize(s2)
                if k:
                    best = max(best, B / (time.perf_counter() - t0) / 1e9)
            out.setdefault(name, []).append(round(best, 2))
            print(json.dumps({"round": rnd, "case": name, "GBps_each_direction": round(best, 2)}), flush=True)
    print(json.dumps({"summary_GBps_each_direction": out}), flush=True)
    ish.ishmem_finalize()


if __name__ == "__main__":
    main()
