#!/usr/bin/env python3
"""Dev tool: run-to-run variance of DMA from page-locked host memory (the host-memory leg swings
between ~17 and ~43 GiB/s with hipHostMalloc buffers).  For each flavour, 5 fresh allocations of
two 1 GiB buffers, each timed as concurrent H2D + D2H hipMemcpyAsync on two streams (GB/s each way,
best of 3 after a warm-up):
  hostmalloc   - hipHostMalloc (default flags)
  mmap_4k      - anonymous mmap, MADV_NOHUGEPAGE, hipHostRegister
  mmap_thp     - anonymous mmap (2 MiB aligned), MADV_HUGEPAGE, touched, hipHostRegister
Also prints the box's transparent-huge-page mode.
"""
from __future__ import annotations

import ctypes
import json
import mmap
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

B = 1 << 30
MADV_HUGEPAGE, MADV_NOHUGEPAGE = 14, 15


def main() -> None:
    from ishmem_amd import hip
    L = hip.lib()
    libc = ctypes.CDLL("libc.so.6", use_errno=True)
    libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    L.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    L.hipHostUnregister.argtypes = [ctypes.c_void_p]
    d1, d2 = hip.malloc(B), hip.malloc(B)
    s1, s2 = hip.stream_create(), hip.stream_create()

    def rate(hs, hd):
        best = 0.0
        for k in range(4):
            t0 = time.perf_counter()
            hip.memcpy_async(d1, hs, B, s1)
            hip.memcpy_async(hd, d2, B, s2)
            hip.stream_synchronize(s1)
            hip.stream_synchronize(s2)
            if k:
                best = max(best, B / (time.perf_counter() - t0) / 1e9)
        return round(best, 1)

    def mmap_buf(thp: bool):
        m = mmap.mmap(-1, B + (2 << 20), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        base = ctypes.addressof(ctypes.c_char.from_buffer(m))
        addr = (base + (2 << 20) - 1) & ~((2 << 20) - 1)
        libc.madvise(addr, B, MADV_HUGEPAGE if thp else MADV_NOHUGEPAGE)
        ctypes.memset(addr, 1, B)
        rc = L.hipHostRegister(addr, B, 0)
        return m, addr, rc

    out = {}
    try:
        out["thp_mode"] = Path("/sys/kernel/mm/transparent_hugepage/enabled").read_text().strip()
    except OSError:
        out["thp_mode"] = None
    # First allocation or first use?  Allocate pair A, then pair B; time B, then A, then B again.
    ha = (hip.host_malloc(B), hip.host_malloc(B))
    hb = (hip.host_malloc(B), hip.host_malloc(B))
    order = {"B_first": rate(*hb), "A_then": rate(*ha), "B_again": rate(*hb)}
    out["first_alloc_vs_first_use"] = order
    print(json.dumps(order), flush=True)
    for p_ in (*ha, *hb):
        hip.host_free(p_)
    for flavour in ("hostmalloc", "mmap_4k", "mmap_thp"):
        rs = []
        for _ in range(5):
            if flavour == "hostmalloc":
                hs, hd = hip.host_malloc(B), hip.host_malloc(B)
                rs.append(rate(hs, hd))
                hip.host_free(hs)
                hip.host_free(hd)
            else:
                (ma, a, ra), (mb, b, rb) = mmap_buf(flavour == "mmap_thp"), mmap_buf(flavour == "mmap_thp")
                rs.append(rate(a, b) if ra == 0 and rb == 0 else f"register rc {ra}/{rb}")
                L.hipHostUnregister(a)
                L.hipHostUnregister(b)
                del ma, mb
        out[flavour] = rs
        print(json.dumps({flavour: rs}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
