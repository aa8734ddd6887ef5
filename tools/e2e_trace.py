#!/usr/bin/env python3
"""Dev tool: the staged host-memory pipeline's copies on a timeline.  1 PE, 1 GiB f32 sum from
pinned host memory (hipHostMalloc) to pinned host memory: 3 warm-up calls, then 4 on-stream calls
back to back (one synchronize, as the bench's e2e leg) and 4 calls each followed by a synchronize.
Run under `rocprofv3 --memory-copy-trace --kernel-trace` to see each 32 MiB chunk's H2D / D2H copy
and whether the two directions overlap.  Prints the rate of each phase.
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
GiB = 1 << 30


def main() -> None:
    import ishmem_amd as ish
    from ishmem_amd import hip
    ish.init(0, 1, 0, f"et{uuid.uuid4().hex[:8]}")
    n = B // 4
    hs, hd = hip.host_malloc(B), hip.host_malloc(B)
    st = hip.stream_create()

    def call():
        if ish.ishmemx_float_sum_reduce_on_stream(hd, hs, n, 0, st) != 0:
            raise RuntimeError(ish.last_error())

    out = {}
    if os.environ.get("E2E_BIG"):
        # One call over a larger payload: do many chunks queued by ONE call slow down like
        # back-to-back calls do?
        nb = int(os.environ["E2E_BIG"]) << 30
        bs, bd = hip.host_malloc(nb), hip.host_malloc(nb)
        rates = []
        for _ in range(4):
            t0 = time.perf_counter()
            if ish.ishmemx_float_sum_reduce_on_stream(bd, bs, nb // 4, 0, st) != 0:
                raise RuntimeError(ish.last_error())
            hip.stream_synchronize(st)
            rates.append(round(nb / GiB / (time.perf_counter() - t0), 2))
        print(json.dumps({f"single_{nb >> 30}GiB_calls": rates}), flush=True)
        hip.host_free(bs)
        hip.host_free(bd)
    for phase in ("warmup", "back_to_back", "synced", "back_to_back_2", "synced_2"):
        rates = []
        if phase.startswith("back_to_back"):
            t0 = time.perf_counter()
            for _ in range(4):
                call()
            hip.stream_synchronize(st)
            rates.append(round(4 * B / GiB / (time.perf_counter() - t0), 2))
        else:
            for _ in range(3 if phase == "warmup" else 4):
                t0 = time.perf_counter()
                call()
                hip.stream_synchronize(st)
                rates.append(round(B / GiB / (time.perf_counter() - t0), 2))
        out[phase] = rates
        print(json.dumps({phase: rates}), flush=True)
    hip.host_free(hs)
    hip.host_free(hd)
    ish.ishmem_finalize()


if __name__ == "__main__":
    main()
