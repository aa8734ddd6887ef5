#!/usr/bin/env python3
"""Dev probe: small on-stream reduces before and after the coherence tripwire (host wall per call
and device time per call), to find what a preceding leg leaves behind.  Launch with
torch.distributed.run (2 ranks, ISHMEM_BENCH_SAME_DEVICE=1)."""
from __future__ import annotations

import os
import sys
import time
import uuid
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def main() -> None:
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    import torch.distributed as dist
    dist.init_process_group("gloo")
    obj = [f"ta{uuid.uuid4().hex[:8]}"]
    dist.broadcast_object_list(obj, src=0)
    import ishmem_amd as ish
    from ishmem_amd import hip, selfcheck
    ish.init(rank, world, 0, obj[0])
    src, dst = ish.ishmem_malloc(1 << 20), ish.ishmem_malloc(1 << 20)
    st = hip.stream_create()

    def timed(tag):
        for _ in range(3):
            ish.reduce_on_stream("min", "int32", dst, src, 1024, None, st)
        hip.stream_synchronize(st)
        dist.barrier()
        e0, e1 = hip.Event(), hip.Event()
        t0 = time.perf_counter()
        e0.record(st)
        for _ in range(50):
            ish.reduce_on_stream("min", "int32", dst, src, 1024, None, st)
        e1.record(st)
        t1 = time.perf_counter()
        hip.stream_synchronize(st)
        t2 = time.perf_counter()
        print(f"rank{rank} {tag}: host enqueue {1e6 * (t1 - t0) / 50:.1f} us/call, "
              f"device {1e3 * e0.elapsed_ms(e1) / 50:.1f} us/call, wall {1e6 * (t2 - t0) / 50:.1f}", flush=True)

    import numpy as np

    def words(tag):
        hip.synchronize()
        w = hip.download(ish.get_param("launch_words"), 1184, np.uint32)
        rep = w[16:16 + 64 * 16].reshape(64, 16)
        print(f"rank{rank} {tag}: epoch {w[0]} line0 {list(w[1:8])} replicas {sorted(set(rep[:, 0].tolist()))} "
              f"marks {sorted(set(rep[:, 1].tolist()))} shards {list(w[65*16:74*16:16])}", flush=True)

    timed("before")
    words("before")
    for _ in range(int(os.environ.get("TA_STREAMS", "1"))):
        s2 = hip.stream_create()
        ish.combine("sum", "uint32", dst, [src, src], 1024, s2)
        hip.stream_synchronize(s2)
        hip.stream_destroy(s2)
    timed("after stream churn")
    selfcheck.chain_tripwire(ish, hip, rank, world, nmax=1 << 20, iters=8)
    words("after tripwire")
    timed("after tripwire")
    words("after timed")
    r, t = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 0, 1, world)
    ish.ishmem_team_destroy(t)
    timed("after split+destroy")
    ish.ishmem_finalize()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
