#!/usr/bin/env python3
"""Size sweep of the reduce path (dev tool): f32 sum (or --op/--dtype) over TEAM_WORLD for sizes
4 B .. --max-mib, one process per PE (launch with torch.distributed.run for N>1; set
ISHMEM_BENCH_SAME_DEVICE=1 to put every PE on device 0).  Prints one CSV row per size on rank 0:
bytes, us per call (max over ranks), algbw GiB/s.  Results are checked against the closed form."""
from __future__ import annotations

import argparse
import ctypes
import os
import sys
import uuid
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-mib", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--min-bytes", type=int, default=4)
    ap.add_argument("--factor", type=int, default=4)
    ap.add_argument("--coll", choices=["reduce", "fcollect", "inscan", "broadcast"], default="reduce")
    ap.add_argument("--graph", action="store_true", help="time a hipGraph of --iters captured calls")
    ap.add_argument("--blocking", action="store_true",
                    help="blocking host calls (ishmem_fcollectmem / ishmem_float_sum_inscan / ishmem_float_sum_reduce), "
                         "timed on the host clock")
    ap.add_argument("--src-offset", type=int, default=0, help="reduce: source starts this many bytes (a multiple of 4) past its allocation")
    ap.add_argument("--dst-offset", type=int, default=0, help="reduce: dest starts this many bytes (a multiple of 4) past its allocation")
    ap.add_argument("--phases", action="store_true", help="reduce: after the sweep, one call of the largest size with "
                    "HIP events between the phased path's five launches (rank 0's ms)")
    ap.add_argument("--emulate-share1", action="store_true",
                    help="every PE reports its own device (ISHMEM_TEST_PCI_BUS): the launch shapes of one PE per GPU")
    ap.add_argument("--inplace", action="store_true",
                    help="reduce: source == dest (the values then change every call: ok = -1, not checked)")
    ap.add_argument("--param", action="append", default=[], metavar="NAME=VALUE",
                    help="ishmem set_param before the sweep (every PE alike), repeatable")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    key = f"sw{uuid.uuid4().hex[:10]}"
    if args.emulate_share1:
        os.environ["ISHMEM_TEST_PCI_BUS"] = f"fake-bus-{rank}"
        # The test-hooks build unless an A/B variant (built with ISHMEMI_TEST_HOOKS) is named.
        os.environ.setdefault("ISHMEM_AMD_LIB", str(Path(__file__).resolve().parents[1] / "ishmem_amd/libishmem_amd_testhooks.so"))
    # The library (and the image's HIP runtime with it) before torch, whose own HIP copy would
    # otherwise serve the process (bench.py main, round 6).
    import ishmem_amd as ish
    from ishmem_amd import hip
    hip.lib()
    try:  # and the image's HSA runtime under the name torch's HIP-side libraries ask for
        ctypes.CDLL("libhsa-runtime64.so", mode=ctypes.RTLD_GLOBAL)
    except OSError:
        pass
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")
        obj = [key]
        dist.broadcast_object_list(obj, src=0)
        key = obj[0]
    dev = 0 if os.environ.get("ISHMEM_BENCH_SAME_DEVICE") == "1" else local
    ish.init(rank, world, dev, key)
    for kv in args.param:
        name, val = kv.split("=", 1)
        ish.set_param(name, int(val))
    nmax = (args.max_mib << 20) // 4
    so, do = args.src_offset // 4, args.dst_offset // 4
    src = ish.ishmem_malloc(nmax * 4 + 64)
    dst = ish.ishmem_malloc(nmax * 4 * (world if args.coll == "fcollect" else 1) + 64)
    hip.upload(src, (np.arange(nmax + 16, dtype=np.int64) % 1024).astype(np.float32) + np.float32(rank))
    st = hip.stream_create()
    if rank == 0:
        print(f"# coll={args.coll} graph={args.graph} blocking={args.blocking} pes={world} same_device={os.environ.get('ISHMEM_BENCH_SAME_DEVICE') == '1'} "
              f"ll_max_bytes={ish.get_param('ll_max_bytes')} wait_slots={ish.get_param('wait_slots')} "
              f"device_share={ish.get_param('device_share')} src_offset={args.src_offset} dst_offset={args.dst_offset} params={args.param}")
        print("bytes,us_per_call,algbw_GiBps,ok")
    def call(n):
        if args.blocking:
            if args.coll == "fcollect":
                return ish.ishmem_fcollectmem(dst, src, n * 4)
            if args.coll == "broadcast":
                return ish.ishmem_broadcastmem(dst, src, n * 4, 0)
            if args.coll == "inscan":
                return ish.lib().ishmemi_c_scan(0, ish.DTYPES["float"], 1, dst, src, n)
            return ish.ishmem_float_sum_reduce(dst, src, n)
        if args.coll == "fcollect":
            return ish.fcollect_on_stream(dst, src, n * 4, 0, st)
        if args.coll == "broadcast":
            return ish.broadcast_on_stream(dst, src, n * 4, 0, 0, st)
        if args.coll == "inscan":
            return ish.lib().ishmemi_c_scan_on_stream(0, ish.DTYPES["float"], 1, dst, src, n, None, st)
        if args.inplace:
            return ish.ishmemx_float_sum_reduce_on_stream(src + 4 * so, src + 4 * so, n, 0, st)
        return ish.ishmemx_float_sum_reduce_on_stream(dst + 4 * do, src + 4 * so, n, 0, st)

    def expect(i, n):
        i = i + so
        base = (i % 1024).astype(np.float32)
        if args.coll == "fcollect":  # the last k elements of the dest = PE world-1's tail
            return base + np.float32(world - 1)
        if args.coll == "broadcast":  # root 0's source
            return base
        if args.coll == "inscan":
            return base * (rank + 1) + np.float32(rank * (rank + 1) / 2)
        return base * world + np.float32(world * (world - 1) / 2)

    n = max(1, args.min_bytes // 4)
    while n <= nmax:
        for _ in range(3):
            call(n)
        hip.stream_synchronize(st)
        if dist is not None:
            dist.barrier()
        e0, e1 = hip.Event(), hip.Event()
        iters = args.iters if n < (1 << 24) else max(3, args.iters // 4)
        if args.graph:
            with hip.Graph(st) as g:
                for _ in range(iters):
                    if call(n):
                        raise RuntimeError(ish.last_error())
            g.launch()
            hip.stream_synchronize(st)
            if dist is not None:
                dist.barrier()
            e0.record(st)
            g.launch()
            e1.record(st)
        elif args.blocking:
            import time
            t0 = time.perf_counter()
            for _ in range(iters):
                if call(n):
                    raise RuntimeError(ish.last_error())
            host_us = (time.perf_counter() - t0) * 1e6 / iters
        else:
            e0.record(st)
            for _ in range(iters):
                if call(n):
                    raise RuntimeError(ish.last_error())
            e1.record(st)
        hip.stream_synchronize(st)
        us = host_us if args.blocking else e0.elapsed_ms(e1) * 1000.0 / iters
        if dist is not None:
            t = torch.tensor([us], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            us = float(t[0])
        k = min(n, 64)
        last = n * (world if args.coll == "fcollect" else 1)
        got = hip.download(dst + 4 * do + (last - k) * 4, k, np.float32)
        ok = -1 if args.inplace else int(np.array_equal(got, expect(np.arange(n - k, n), n)))
        if rank == 0:
            print(f"{n * 4},{us:.2f},{n * 4 / 2**30 / (us * 1e-6):.2f},{int(ok)}", flush=True)
        n *= args.factor
    if args.phases and args.coll == "reduce":
        n = n // args.factor
        ish.set_param("phase_events", 1)
        for _ in range(2):
            call(n)
            hip.stream_synchronize(st)
            if dist is not None:
                dist.barrier()
        ms = (ctypes.c_float * 5)()
        r = ish.lib().ishmemi_c_phase_times(ms)
        ish.set_param("phase_events", 0)
        if rank == 0:
            print(f"# phases bytes={n * 4} rc={r} " + " ".join(f"{k}={v:.4f}" for k, v in zip(
                ["start", "rs", "mid", "ag", "end"], list(ms))), flush=True)
    ish.ishmem_finalize()


if __name__ == "__main__":
    main()
