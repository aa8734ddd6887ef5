#!/usr/bin/env python3
"""Dev tool (round 5): fcollect of B + e bytes per PE, e in {0, 4, 1}: the collect kernels pick
16 / 4 / 1-byte units from the alignment of every member's source, dest offset and count, so a
count that is not a multiple of 16 drops the whole call to narrow units.  Run under
torch.distributed.run (ISHMEM_BENCH_SAME_DEVICE=1: every PE on device 0).  One CSV row per case on
rank 0: bytes per PE, us per call (max over ranks), GB/s of dest written per PE, checked."""
from __future__ import annotations

import os
import sys
import uuid
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main() -> None:
    import torch  # noqa: F401
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist.init_process_group("gloo")
    obj = [f"cp{uuid.uuid4().hex[:10]}"]
    dist.broadcast_object_list(obj, src=0)
    import ishmem_amd as ish
    from ishmem_amd import hip
    dev = 0 if os.environ.get("ISHMEM_BENCH_SAME_DEVICE") == "1" else local
    ish.init(rank, world, dev, obj[0])
    ish.set_param("collect_realign", int(os.environ.get("COLLECT_REALIGN", "1")))
    mib = int(os.environ.get("COLLECT_MIB", "64"))
    extras = [int(x) for x in os.environ.get("COLLECT_EXTRA", "0,4,1").split(",")]
    bmax = (mib << 20) + 16
    src = ish.ishmem_malloc(bmax)
    dst = ish.ishmem_malloc(bmax * world)
    st = hip.stream_create()
    rng = np.random.default_rng(rank)
    mine = rng.integers(0, 256, bmax, dtype=np.uint8)
    hip.upload(src, mine)
    allsrc = [np.random.default_rng(r).integers(0, 256, bmax, dtype=np.uint8) for r in range(world)]
    if rank == 0:
        print("bytes_per_pe,us_per_call,GBps_dest_per_pe,checked", flush=True)
    for e in extras:
        nb = (mib << 20) + e
        for _ in range(3):
            ish.fcollect_on_stream(dst, src, nb, 0, st)
        hip.stream_synchronize(st)
        dist.barrier()
        e0, e1 = hip.Event(), hip.Event()
        iters = 10
        e0.record(st)
        for _ in range(iters):
            if ish.fcollect_on_stream(dst, src, nb, 0, st) != 0:
                raise RuntimeError(ish.last_error())
        e1.record(st)
        hip.stream_synchronize(st)
        us = e0.elapsed_ms(e1) * 1000.0 / iters
        t = torch.tensor([us])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        us = float(t[0])
        got = hip.download(dst, nb * world, np.uint8)
        ok = all(np.array_equal(got[r * nb:(r + 1) * nb], allsrc[r][:nb]) for r in range(world))
        if rank == 0:
            print(f"{nb},{us:.2f},{nb * world / (us * 1e-6) / 1e9:.1f},{int(ok)}", flush=True)
    ish.ishmem_finalize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
