#!/usr/bin/env python3
"""Benchmark of the MI355X-native reduction collective (BASELINE.json metric:
"GiB/s device-resident float32 sum-reduce at 1/2/4/8 PEs vs HBM+xGMI roofline").

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mib 1024]

N=1 (BASELINE configs[1]): ishmem_float_sum_reduce over a 1 GiB symmetric-heap array on one PE
(reference semantics: dest = source, src/collectives/reduce_impl.h:288-289), plus the local
combine unit dst = a + b (the per-step unit of the multi-PE path) at the same size.
N>1 (launched by torch.distributed.run, one process per GPU): the same call over TEAM_WORLD =
direct reduce-scatter + all-gather over xGMI (configs[2..3]); value = N * B / t (whole job).

A "step" = one reduce of B bytes per PE, inputs already resident in HBM.  K steps are timed
between barrier + device synchronize on both sides; ms_per_step is the max over ranks.  The
dominant kernel's duration is measured with HIP events on the stream it runs on.  rank 0 at N=1
also times the reference's host-proxy CPU reduce, restated in oracle/ (cpu_baseline).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time
import uuid
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# Bound every device-side spin to 15 s (library default 60 s): a PE that never arrives ends the
# run with an error line within a minute instead of stalling every queued step for a minute each.
os.environ.setdefault("ISHMEM_TIMEOUT_MS", "15000")

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
XGMI_LINK_GBS = 153.6       # per link, as given by the task brief (may be bidirectional)
GiB = float(1 << 30)


def pmc_traffic(kernel_tag: str, nbytes: int):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), or None."""
    f = ROOT / "profiles" / "pmc_summary.json"
    if not f.exists():
        return None
    try:
        d = json.loads(f.read_text())
        e = d.get(kernel_tag)
        if e and int(e.get("payload_bytes", -1)) == nbytes:
            return float(e["hbm_bytes_per_launch"])
    except Exception:
        return None
    return None


def config5_sweep(ish, hip, src, dst, nbytes_max, world, rank, dist, stream):
    """Config 5: min/max/prod x int32/float64, 4 KiB .. nbytes_max (the bench payload, 1 GiB by
    default) per PE in steps of 4x: us per call (max over ranks), algbw, last 256 results checked
    against the closed form of x_pe[i] = (i mod 1024) + pe."""
    import torch
    out = []
    for dtn, npd in (("int32", np.int32), ("double", np.float64)):
        es = np.dtype(npd).itemsize
        nmax = nbytes_max // es
        x = (np.arange(nmax, dtype=np.int64) % 1024).astype(npd) + npd(rank)
        hip.upload(src, x)
        del x

        def expect(op, idx):
            base = idx % 1024
            if op == "min":
                return base.astype(npd)
            if op == "max":
                return (base + world - 1).astype(npd)
            if npd is np.float64:
                acc = base.astype(np.float64)
                for pe in range(1, world):
                    acc = acc * (base.astype(np.float64) + pe)
                return acc
            acc = base.astype(np.uint32)
            for pe in range(1, world):
                acc = (acc * (base + pe).astype(np.uint32)).astype(np.uint32)
            return acc.view(np.int32)

        for op in ("min", "max", "prod"):
            nb = 4096
            while nb <= nbytes_max:
                n = nb // es
                for _ in range(2):
                    ish.reduce_on_stream(op, dtn, dst, src, n, None, stream)
                hip.stream_synchronize(stream)
                dist.barrier()
                it = 20 if nb < (8 << 20) else 5
                e0, e1 = hip.Event(), hip.Event()
                e0.record(stream)
                for _ in range(it):
                    if ish.reduce_on_stream(op, dtn, dst, src, n, None, stream) != 0:
                        raise RuntimeError(ish.last_error())
                e1.record(stream)
                hip.stream_synchronize(stream)
                us = e0.elapsed_ms(e1) * 1000.0 / it
                t = torch.tensor([us], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                us = float(t[0])
                k = min(n, 256)
                got = hip.download(dst + (n - k) * es, k, npd)
                want = expect(op, np.arange(n - k, n, dtype=np.int64))
                ok = bool(np.array_equal(got.view(np.uint8), want.view(np.uint8)))
                out.append({"op": op, "dtype": dtn, "bytes": nb, "us": round(us, 2),
                            "algbw_GiBps": round(nb / GiB / (us * 1e-6), 2), "checked": ok})
                nb *= 4
    return out


def xgmi_tuning(ish, hip, src, dst, B, world, dist, stream):
    """N>1: the f32 sum again under other launch shapes, set alike on every rank, so the driver's
    multi-GPU run records how the xGMI path responds (data for choosing the defaults; one
    MI355X per PE cannot be rehearsed on a one-GPU box):
      grid  - the payload with the workgroup cap at 128 / 256 / 512 / 1024 (then clamped to the
              resident capacity);
      p2    - two PEs: one-shot fold vs reduce-scatter + all-gather at the payload size;
      ll    - 4 / 16 / 64 KiB with the one-hop granule path on (default) and off."""
    import torch

    def timed(n, iters):
        for _ in range(2):
            ish.ishmemx_float_sum_reduce_on_stream(dst, src, n, 0, stream)
        hip.stream_synchronize(stream)
        dist.barrier()
        e0, e1 = hip.Event(), hip.Event()
        e0.record(stream)
        for _ in range(iters):
            if ish.ishmemx_float_sum_reduce_on_stream(dst, src, n, 0, stream) != 0:
                raise RuntimeError(ish.last_error())
        e1.record(stream)
        hip.stream_synchronize(stream)
        t = torch.tensor([e0.elapsed_ms(e1) / iters], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t[0])

    out = []

    def run(case, param, value, nbytes, iters):
        old = ish.get_param(param)
        ish.set_param(param, value)
        try:
            ms = timed(nbytes // 4, iters)
        finally:
            ish.set_param(param, old)
        out.append({"case": case, param: value, "bytes": nbytes, "us": round(ms * 1e3, 2),
                    "algbw_GiBps": round(nbytes / GiB / (ms * 1e-3), 2)})

    # Several PEs sharing one GPU (ISHMEM_BENCH_SAME_DEVICE rehearsals) must keep their summed
    # grids resident, so there the sweep stays at or below the grid cap the run started with.
    cap = ish.get_param("max_blocks") if os.environ.get("ISHMEM_BENCH_SAME_DEVICE") == "1" else 1024
    for mb in (128, 256, 512, 1024):
        if mb <= cap:
            run("grid", "max_blocks", mb, B, 5)
    if world == 2:
        run("p2_oneshot", "oneshot_p2_max_bytes", 1 << 40, B, 5)
        run("p2_rs_ag", "oneshot_p2_max_bytes", 0, B, 5)
    for nb in (4096, 16384, 65536):
        run("ll_on", "ll_max_bytes", 65536, nb, 50)
        run("ll_off", "ll_max_bytes", 0, nb, 50)
    return out


def rccl_allreduce(dist, device, n, B, world, steps, line, limit_s=240.0):
    """N>1 comparison only: RCCL (torch "nccl" backend) all_reduce of the
    same f32 payload over the same GPUs, after this library has released its heap.  A watchdog
    bounds the leg: if RCCL does not finish within limit_s, rank 0 prints the line already
    measured (marked) and every rank exits, so the main measurement is never lost."""
    import threading

    import torch

    def expire():
        if line is not None:
            line["rccl_allreduce"] = {"error": f"did not finish within {limit_s:.0f} s"}
            print(json.dumps(line), flush=True)
        os._exit(0)

    wd = threading.Timer(limit_s, expire)
    wd.daemon = True
    wd.start()
    try:
        torch.cuda.set_device(device)
        pg = dist.new_group(backend="nccl")
        buf = torch.ones(n, dtype=torch.float32, device="cuda")
        for _ in range(3):
            dist.all_reduce(buf, group=pg)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            dist.all_reduce(buf, group=pg)
        torch.cuda.synchronize()
        tr = time.perf_counter() - t0
        tt = torch.tensor([tr], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        tr = float(tt[0])
        buf.fill_(1.0)
        dist.all_reduce(buf, group=pg)
        ok = bool(torch.all(buf == float(world)).item())
        del buf
        torch.cuda.synchronize()
        dist.destroy_process_group(pg)
        return {"value": world * B / GiB / (tr / steps), "unit": "GiB/s",
                "ms_per_step": tr / steps * 1000.0, "steps": steps, "checked": ok}
    except Exception as ex:
        return {"error": str(ex)}
    finally:
        wd.cancel()


def log(msg: str) -> None:
    """Progress on stderr (rank 0), so a long leg is visibly alive; stdout keeps the one JSON line."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mib", type=int, default=1024, help="payload per PE in MiB (default 1 GiB)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-combine", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-sweep", action="store_true")
    ap.add_argument("--no-probe", action="store_true")
    ap.add_argument("--nelems", type=int, default=0, help="override: float32 elements per PE")
    ap.add_argument("--no-rccl", action="store_true",
                    help="N>1: skip the RCCL all_reduce comparison on the same payload")
    ap.add_argument("--no-tuning", action="store_true", help="N>1: skip the launch-shape sweep")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            sys.exit("bench.py --gpus N>1 must be launched by torch.distributed.run (one rank per GPU)")
    dist = None
    key = f"bench{uuid.uuid4().hex[:10]}"
    if world > 1:
        import torch.distributed as dist  # control plane only (gloo); the data path is ours
        dist.init_process_group("gloo")
        obj = [key]
        dist.broadcast_object_list(obj, src=0)
        key = obj[0]

    import ishmem_amd as ish
    from ishmem_amd import hip

    # ISHMEM_BENCH_SAME_DEVICE=1 (development only): every rank on device 0, to measure kernel
    # overheads of the multi-PE path on a one-GPU box.  Never used for reported numbers.
    device = 0 if os.environ.get("ISHMEM_BENCH_SAME_DEVICE") == "1" else local_rank
    ish.init(rank, world, device, key)
    n = args.nelems if args.nelems > 0 else (args.mib << 20) // 4
    B = n * 4
    src = ish.ishmem_malloc(B)
    dst = ish.ishmem_malloc(B)
    # Synthetic input with an exactly representable sum: x[i] = (i mod 1024) + pe.
    pattern = (np.arange(n, dtype=np.int64) % 1024).astype(np.float32) + np.float32(rank)
    hip.upload(src, pattern)
    del pattern
    stream = hip.stream_create()

    def barrier():
        hip.synchronize()
        if dist is not None:
            dist.barrier()
        hip.synchronize()

    def step():
        r = ish.ishmemx_float_sum_reduce_on_stream(dst, src, n, 0, stream)
        if r != 0:
            raise RuntimeError(f"reduce failed: {ish.last_error()}")

    log("warm-up")
    for _ in range(args.warmup):
        step()
    barrier()
    if ish.lib().ishmemi_c_error_count():
        raise RuntimeError("device barrier timeouts during warm-up (a PE did not arrive)")
    ev0, ev1 = hip.Event(), hip.Event()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    hip.stream_synchronize(stream)
    t1 = time.perf_counter()
    barrier()
    wall_s = t1 - t0
    kern_ms = ev0.elapsed_ms(ev1) / args.steps
    if dist is not None:
        import torch
        t = torch.tensor([wall_s, kern_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall_s, kern_ms = float(t[0]), float(t[1])
    if ish.lib().ishmemi_c_error_count():
        raise RuntimeError("device barrier timeouts during the benchmark")

    # Correctness of the timed buffers (sampled): dest = sum_pe((i mod 1024) + pe).
    idx = np.random.default_rng(0).integers(0, n, 4096)
    got = np.array([hip.download(dst + int(i) * 4, 1, np.float32)[0] for i in idx[:256]])
    exp = (idx[:256] % 1024).astype(np.float32) * world + np.float32(world * (world - 1) / 2)
    if not np.array_equal(got, exp):
        raise RuntimeError("benchmark result check failed")

    ms_per_step = wall_s * 1000.0 / args.steps
    value = world * B / GiB / (ms_per_step / 1000.0)

    if world == 1:
        roof = {"bound": "hbm", "achieved": 2 * B / (kern_ms * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "traffic": pmc_traffic("copy_1pe", B),
                "kernel": "fanin_kernel<uint8,OR,vec> (1-PE reduce = copy, 2B per launch)"}
    else:
        link_bytes = 2.0 * (world - 1) / world * B  # RS + AG ingress per PE over p-1 links
        roof = {"bound": "xgmi", "achieved": link_bytes / (kern_ms * 1e-3) / 1e9,
                "peak": XGMI_LINK_GBS * (world - 1), "unit": "GB/s",
                "traffic": pmc_traffic(f"allreduce_{world}pe", B),
                "kernel": "allreduce_kernel<float,SUM,vec> (per-PE xGMI ingress 2(p-1)/p*B)"}
    roof["frac"] = roof["achieved"] / roof["peak"]

    extra = {}
    log("timed steps done; combine leg")
    if world == 1 and not args.no_combine:
        # Local combine unit dst = a + b at the same size (3B HBM bytes per launch).
        b2 = ish.ishmem_malloc(B)
        hip.memcpy(b2, src, B)
        for _ in range(3):
            ish.combine("sum", "float", dst, [src, b2], n, stream)
        e0, e1 = hip.Event(), hip.Event()
        e0.record(stream)
        for _ in range(args.steps):
            ish.combine("sum", "float", dst, [src, b2], n, stream)
        e1.record(stream)
        hip.stream_synchronize(stream)
        cms = e0.elapsed_ms(e1) / args.steps
        ach = 3 * B / (cms * 1e-3) / 1e9
        extra["combine"] = {"kernel": "fanin_kernel<float,SUM,vec> dst=a+b", "ms": cms,
                            "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": ach / HBM_PEAK_GBS, "traffic": pmc_traffic("combine2_1pe", B)}
        ish.ishmem_free(b2)

    log("host-memory end-to-end leg")
    if not args.no_e2e:
        # The path starts and ends in host memory (north star): pinned host source/dest, the
        # library stages H2D -> device reduce -> D2H through HBM as a 3-stream pipeline.
        try:
            hs, hd = hip.host_malloc(B), hip.host_malloc(B)
            hip.memcpy(hs, src, B)  # same synthetic input as the device-resident run
            def step_e2e():
                return ish.ishmemx_float_sum_reduce_on_stream(hd, hs, n, 0, stream)
            if step_e2e() != 0:  # warm-up (creates the pipeline streams)
                raise RuntimeError(ish.last_error())
            barrier()
            k = max(2, args.steps // 5)
            te0 = time.perf_counter()
            for _ in range(k):
                if step_e2e() != 0:
                    raise RuntimeError(ish.last_error())
            hip.stream_synchronize(stream)
            te = time.perf_counter() - te0
            barrier()
            if dist is not None:
                import torch
                tt = torch.tensor([te], dtype=torch.float64)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                te = float(tt[0])
            chk = (ctypes.c_float * 4).from_address(hd + 4 * 1000)
            ok = [float(x) for x in chk] == [float((1000 + i) % 1024 * world + world * (world - 1) / 2) for i in range(4)]
            extra["e2e_host"] = {"value": world * B / GiB / (te / k), "unit": "GiB/s",
                                 "ms_per_step": te / k * 1000.0, "steps": k, "checked": ok,
                                 "buffers": "pinned host (hipHostMalloc)",
                                 "pipeline": "H2D | reduce | D2H over 2 staging slots"}
            hip.host_free(hs)
            hip.host_free(hd)
        except Exception as ex:  # reported, never fatal for the main measurement
            extra["e2e_host"] = {"error": str(ex)}

    log("xGMI probe")
    if world > 1 and not args.no_probe:
        # Measured link rates (report against the spec AND a measured L).  Plain
        # pulls of a peer's source through the local combine kernel, no barriers inside:
        #   pull1   — every rank copies S bytes from rank+1 (ring: each link busy in one direction)
        #   pullall — every rank folds the sources of all p-1 peers (ingress (p-1)*S per GPU)
        #   push1   — every rank writes S bytes into rank+1's dest (remote stores)
        try:
            S = min(B, 256 << 20)
            ns = S // 4
            peers = [(rank + d) % world for d in range(1, world)]
            probe = {}
            # pull1 / pullall load nontemporal; the *_sc twins issue the system-coherent (sc0 sc1)
            # loads the collectives use on peer memory, so each pair shows what that policy costs.
            cases = (("pull1", [ish.ishmem_ptr(src, peers[0])], dst, 0),
                     ("pull1_sc", [ish.ishmem_ptr(src, peers[0])], dst, 1),
                     ("pullall", [ish.ishmem_ptr(src, j) for j in peers], dst, 0),
                     ("pullall_sc", [ish.ishmem_ptr(src, j) for j in peers], dst, 1),
                     ("push1", [src], ish.ishmem_ptr(dst, peers[0]), None))

            def launch(srcs, out, pol):
                if pol is None:
                    return ish.combine("sum", "float", out, srcs, ns, stream)
                return ish.pull_probe(out, srcs, S, pol, stream)

            for name, srcs, out, pol in cases:
                for _ in range(2):
                    launch(srcs, out, pol)
                barrier()
                k = 10
                e0, e1 = hip.Event(), hip.Event()
                e0.record(stream)
                for _ in range(k):
                    if launch(srcs, out, pol) != 0:
                        raise RuntimeError(ish.last_error())
                e1.record(stream)
                hip.stream_synchronize(stream)
                ms = e0.elapsed_ms(e1) / k
                import torch
                tt = torch.tensor([ms], dtype=torch.float64)
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                ms = float(tt[0])
                gbs = len(srcs) * S / (ms * 1e-3) / 1e9
                probe[name] = {"bytes_per_peer": S, "peers": len(srcs), "ms": round(ms, 4),
                               "ingress_GBps": round(gbs, 1),
                               "per_link_GBps": round(gbs / len(srcs), 1)}
            barrier()
            extra["xgmi_probe"] = probe
            # Same accounting as roof["achieved"], against the measured all-peer ingress.
            roof["peak_measured"] = max(probe["pullall"]["ingress_GBps"], probe["pullall_sc"]["ingress_GBps"])
            roof["frac_measured"] = roof["achieved"] / roof["peak_measured"]
        except Exception as ex:
            extra["xgmi_probe"] = {"error": str(ex)}

    log("launch-shape sweep")
    if world > 1 and not args.no_tuning:
        try:
            extra["xgmi_tuning"] = xgmi_tuning(ish, hip, src, dst, B, world, dist, stream)
        except Exception as ex:
            extra["xgmi_tuning"] = {"error": str(ex)}

    log("config-5 sweep")
    if world > 1 and not args.no_sweep:
        # BASELINE configs[4] (min/max/prod x int32/float64 across the PEs), sizes 4 KiB ..
        # the payload (1 GiB) per PE (the 4 GiB end of that sweep is left to tools/sweep.py).  Inputs
        # x_pe[i] = (i mod 1024) + pe; every result is checked against the canonical fold.
        extra["config5_sweep"] = config5_sweep(ish, hip, src, dst, B, world, rank, dist, stream)

    log("CPU baseline leg")
    cpu = None
    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        import oracle  # CPU baseline leg only: the reference's host-proxy reduce, restated
        reps = 3
        t_cpu = oracle.host_proxy_time(oracle.OPS["sum"], oracle.DTYPES["float"], n, 1, reps)
        cpu = {"value": B / GiB / t_cpu, "unit": "GiB/s", "cores": 1, "kind": "port",
               "sample": f"full workload: 1 PE f32 sum-reduce of {B / 2**20:g} MiB through 64 KiB host "
                         f"bounce chunks (reduce_impl.h:186-228), best of {reps}"}
        # BASELINE configs[0]: int32 sum, 2 PEs, host loopback through the proxy path (no GPU):
        # two processes exchanging 64 KiB bounce chunks over shared memory.
        n1 = 16 << 20
        t1 = oracle.host_proxy_time(oracle.OPS["sum"], oracle.DTYPES["int32"], n1, 2, 3)
        extra["cpu_config1"] = {"value": n1 * 4 / GiB / t1, "unit": "GiB/s", "cores": 2,
                                "kind": "port", "sample": "int32 sum-reduce, 2 PEs (processes), "
                                "64 MiB per PE, 64 KiB bounce chunks, best of 3"}

    ish.ishmem_free(dst)
    ish.ishmem_free(src)
    hip.stream_destroy(stream)
    ish.ishmem_finalize()
    line = None
    if rank == 0:
        line = {
            "metric": "GiB/s device-resident float32 sum-reduce at 1/2/4/8 PEs vs HBM+xGMI roofline",
            "value": value, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": f"float32 sum-reduce, {B / 2**20:g} MiB per PE, {world} PE(s), "
                                   f"symmetric-heap device buffers", "nreduce": n,
                       "bytes_per_pe": B, "pes": world,
                       "parallelism": "1 PE self-reduce" if world == 1 else f"direct RS+AG over {world} PEs"},
            "kernel_ms": kern_ms,
            **({"dev_same_device": True} if os.environ.get("ISHMEM_BENCH_SAME_DEVICE") == "1" else {}), "roofline": roof, "cpu_baseline": cpu, **extra,
        }
    if world > 1 and not args.no_rccl and os.environ.get("ISHMEM_BENCH_SAME_DEVICE") != "1":
        log("RCCL comparison leg")
        rccl = rccl_allreduce(dist, device, n, B, world, args.steps, line)
        if line is not None:
            line["rccl_allreduce"] = rccl
    if line is not None:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except Exception as exc:  # always leave one JSON line for the driver, with the reason
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps({
                "metric": "GiB/s device-resident float32 sum-reduce at 1/2/4/8 PEs vs HBM+xGMI roofline",
                "value": None, "unit": "GiB/s", "n_gpus": int(os.environ.get("WORLD_SIZE", "1")),
                "higher_is_better": True, "error": f"{type(exc).__name__}: {exc}"}))
        sys.stdout.flush()
        raise
