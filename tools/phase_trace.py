#!/usr/bin/env python3
"""Per-phase timing of the multi-PE reduce kernel (dev tool).  Launch with torch.distributed.run
(N ranks; ISHMEM_BENCH_SAME_DEVICE=1 puts them on device 0).  For each size, the kernel writes
s_memrealtime stamps per workgroup (set_param "trace_buffer"): entry, start satisfied, RS done,
AG done, finish, and the last workgroup's done handshake.  Prints, per rank, microseconds from
the earliest entry: median / max of each phase boundary over the workgroups."""
from __future__ import annotations

import argparse
import os
import sys
import uuid
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4194304,16777216,268435456")
    ap.add_argument("--lead", type=int, default=20)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import torch.distributed as dist
    dist.init_process_group("gloo")
    obj = [f"pt{uuid.uuid4().hex[:8]}"]
    dist.broadcast_object_list(obj, src=0)
    import ishmem_amd as ish
    from ishmem_amd import hip
    dev = 0 if os.environ.get("ISHMEM_BENCH_SAME_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", "0"))
    ish.init(rank, world, dev, obj[0])
    sizes = [int(x) for x in args.sizes.split(",")]
    nmax = max(sizes) // 4
    src, dst = ish.ishmem_malloc(nmax * 4), ish.ishmem_malloc(nmax * 4)
    tr = hip.malloc(1024 * 8 * 8)
    tr2 = hip.malloc(1024 * 8 * 8)
    st = hip.stream_create()
    for nb in sizes:
        n = nb // 4
        for _ in range(5):
            ish.ishmemx_float_sum_reduce_on_stream(dst, src, n, 0, st)
        hip.stream_synchronize(st)
        dist.barrier()
        hip.memset(tr, 0, 1024 * 64)
        hip.memset(tr2, 0, 1024 * 64)
        hip.synchronize()  # hipMemset is not ordered with the non-blocking stream
        dist.barrier()
        # Steady state: warm calls back to back, then two traced calls in a row (the first
        # traced call's finish against the second's entry shows the gap between launches).
        for _ in range(args.lead):
            ish.ishmemx_float_sum_reduce_on_stream(dst, src, n, 0, st)
        ish.set_param("trace_buffer", tr2)
        ish.ishmemx_float_sum_reduce_on_stream(dst, src, n, 0, st)
        ish.set_param("trace_buffer", tr)
        ish.ishmemx_float_sum_reduce_on_stream(dst, src, n, 0, st)
        ish.set_param("trace_buffer", 0)
        hip.stream_synchronize(st)
        prev = hip.download(tr2, 1024 * 8, np.uint64).reshape(1024, 8).astype(np.int64)
        prev = prev[prev[:, 0] != 0]
        t = hip.download(tr, 1024 * 8, np.uint64).reshape(1024, 8).astype(np.int64)
        t = t[t[:, 0] != 0]
        g = len(t)
        # One clock for every rank (s_memrealtime is device-global): the earliest entry of the
        # second traced call over all ranks.
        import torch
        mins = [None] * world
        dist.all_gather_object(mins, int(t[:, 0].min()))
        base = min(mins)
        prev_end = (prev[:, 4].max() - base) / 100.0
        wait = t[:, 7] / 100.0
        t[:, 7] = base
        t[:, 2] = np.where(t[:, 2] == 0, t[:, 3], t[:, 2])  # workgroups that never reduced
        us = (t - base) / 100.0  # 100 MHz ticks -> us
        last = us[us[:, 5] > 0]
        msg = (f"rank{rank} bytes={nb} wgs={g} | entry med/max {np.median(us[:,0]):.1f}/{us[:,0].max():.1f}"
               f" | epoch {np.median(us[:,6]):.1f}/{us[:,6].max():.1f}"
               f" | start {np.median(us[:,1]):.1f}/{us[:,1].max():.1f} | rs-end {np.median(us[:,2]):.1f}/{us[:,2].max():.1f}"
               f" | ag-end {np.median(us[:,3]):.1f}/{us[:,3].max():.1f} | fin {np.median(us[:,4]):.1f}/{us[:,4].max():.1f}"
               f" | last-wg done {last[0,5] if len(last) else -1:.1f} | prev call's last fin {prev_end:.1f} | ag wait med/max {np.median(wait):.1f}/{wait.max():.1f}")
        for r in range(world):
            dist.barrier()
            if r == rank:
                print(msg, flush=True)
    hip.free(tr)
    hip.free(tr2)
    ish.ishmem_finalize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
