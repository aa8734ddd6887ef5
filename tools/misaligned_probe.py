#!/usr/bin/env python3
"""Dev tool (round 4): 1-PE reduce (the copy) and the two-source combine with operands whose
addresses differ mod 16 (the element-granular path of fanin_kernel) against aligned operands,
256 MiB of f32, HIP events, one JSON line.  No oracle: the timed results are checked against numpy."""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def main() -> None:
    import ishmem_amd as ish
    from ishmem_amd import hip
    ish.init(0, 1, 0, None)
    n = (int(os.environ.get("MISALIGNED_MIB", "256")) << 20) // 4
    B = 4 * n + 64
    a, b, d = ish.ishmem_malloc(B), ish.ishmem_malloc(B), ish.ishmem_malloc(B)
    x = np.random.default_rng(1).standard_normal(n + 16).astype(np.float32)
    hip.upload(a, x)
    hip.upload(b, x[::-1].copy())
    st = hip.stream_create()
    out = {}

    def timed(fn, iters=10):
        fn()
        hip.stream_synchronize(st)
        e0, e1 = hip.Event(), hip.Event()
        e0.record(st)
        for _ in range(iters):
            fn()
        e1.record(st)
        hip.stream_synchronize(st)
        return e0.elapsed_ms(e1) / iters

    for name, so, do in (("aligned", 0, 0), ("src+4B", 4, 0), ("dst+4B", 0, 4), ("src+8B_dst+4B", 8, 4)):
        ms = timed(lambda: ish.reduce_on_stream("sum", "float", d + do, a + so, n, None, st))
        got = hip.download(d + do, n, np.float32)
        ok = bool(np.array_equal(got, x[so // 4: so // 4 + n]))
        out[f"copy_{name}"] = {"ms": round(ms, 4), "GBps": round(2 * 4 * n / ms / 1e6, 1), "ok": ok}
        ms = timed(lambda: ish.combine("sum", "float", d + do, [a + so, b + so], n, st))
        out[f"combine_{name}"] = {"ms": round(ms, 4), "GBps": round(3 * 4 * n / ms / 1e6, 1)}
    print(json.dumps(out))
    ish.ishmem_finalize()


if __name__ == "__main__":
    main()
