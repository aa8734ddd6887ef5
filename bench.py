#!/usr/bin/env python3
"""Benchmark of the MI355X-native reduction collective (BASELINE.json metric:
"GiB/s device-resident float32 sum-reduce at 1/2/4/8 PEs vs HBM+xGMI roofline").

  python bench.py [--gpus N] [--steps K] [--warmup W] [--mib 1024]

N=1 (BASELINE configs[1]): ishmem_float_sum_reduce over a 1 GiB symmetric-heap array on one PE
(reference semantics: dest = source, src/collectives/reduce_impl.h:288-289), plus the local
combine unit dst = a + b (the per-step unit of the multi-PE path) at the same size.
N>1 (configs[2..3]): one process per GPU; `python bench.py --gpus N` starts the N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU) unless a launcher
already set WORLD_SIZE.  The same call over TEAM_WORLD = direct reduce-scatter + all-gather over
xGMI.

A "step" = one reduce of B bytes per PE, inputs already resident in HBM.  K steps are timed
between barrier + device synchronize on both sides; ms_per_step is the max over ranks.
  value       = N * B / t  (whole job: payload bytes of all PEs per second)
  algbw_GiBps = B / t      (per PE, the reference harness's payload rate,
                            test/include/ishmem_tester.h:1553-1555; SURVEY.md §8(d)'s targets)
The dominant kernel's duration is measured with HIP events on the stream it runs on.  The timed
dest is compared in full on every rank with the team-order fold of the rotating-winner
input pattern (ishmem_amd/selfcheck.py).  Rank 0 (every rank at N>1) also
times the reference's host path — 64 KiB chunks, each through a synchronous device->host copy, the
MPI-style shared-memory allreduce over the p PEs and a synchronous host->device copy
(reduce_impl.h:186-228, memory.cpp:310-321) — restated in oracle/ (cpu_baseline).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import threading
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

METRIC = "GiB/s device-resident float32 sum-reduce at 1/2/4/8 PEs vs HBM+xGMI roofline"
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
XGMI_LINK_GBS = 153.6       # per link, as given by the task brief (may be bidirectional)
GiB = float(1 << 30)
CFG5_MAX_BYTES = 4 << 30    # BASELINE configs[4]: 4 KiB .. 4 GiB per PE


_OUT = None  # where the one JSON line goes (the original stdout; see main)


def emit(line: dict) -> None:
    out = _OUT if _OUT is not None else sys.stdout
    out.write(json.dumps(line) + "\n")
    out.flush()


def log(msg: str) -> None:
    """Progress on stderr (rank 0), so a long leg is visibly alive; stdout keeps the one JSON line."""
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def host_info() -> dict:
    """Core count and CPU model of the box, for the CPU baseline (nproc + lscpu)."""
    model = None
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    return {"nproc": os.cpu_count(), "usable_cores": usable, "cpu_model": model,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def stall_report(what: str) -> None:
    """Where a stalled setup step is: the Python stack of every thread and, per
    native thread, its name, kernel wait channel and current syscall (/proc: nothing attaches to the
    process), on stderr.  Called by a timer; the run continues (or is ended by its own limit)."""
    import faulthandler
    rank = os.environ.get("RANK", "0")
    print(f"[bench rank {rank}] {what} has not finished after its watchdog interval; thread states:",
          file=sys.stderr, flush=True)
    faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
    for t in sorted(Path("/proc/self/task").iterdir(), key=lambda x: int(x.name)):
        def rd(n):
            try:
                return (t / n).read_text().strip().replace("\n", " ")
            except OSError:
                return "?"
        print(f"[bench rank {rank}]   tid {t.name} comm={rd('comm')} wchan={rd('wchan')} syscall={rd('syscall')[:60]}",
              file=sys.stderr, flush=True)


def self_launch(args) -> int:
    """--gpus N > 1 without a launcher: run the N ranks as a child torch.distributed.run (never
    exec: nothing here has touched the GPU, and the parent only relays), rank 0's JSON line
    passes through on stdout; the exit code is the child's."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           str(Path(__file__).resolve()), *sys.argv[1:]]
    log(f"self-launch: {' '.join(cmd[1:])}")
    return subprocess.run(cmd).returncode


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


def multi_pe_kernel(B: int, phased_min: int, world: int = 0, fold_limit: int = -1) -> str:
    """The multi-PE kernels a B-byte f32 sum with disjoint buffers takes (runtime.cpp reduce_heap):
    up to the team's fold bound (get_param "fold_limit_bytes": path_limits, by topology; 0 for
    teams of more than 4) every member folds the whole array between two barriers; the phased
    path's one-shot grids for payloads of at least phased_min bytes (-1: off); else the persistent
    kernel."""
    if world >= 2 and 0 <= B <= fold_limit:
        return (f"rs_phase_kernel<float,SUM,{world}> whole-array fold on every member between 2 one-workgroup "
                "team barriers")
    if phased_min >= 0 and B >= phased_min:
        return "rs_phase_kernel<float,SUM,P> + ag_phase_kernel between 3 one-workgroup team barriers"
    return "allreduce_kernel<float,SUM,vec>"


def roofline(world: int, share: int, B: int, kern_ms: float, kernel: str = "allreduce_kernel<float,SUM,vec>") -> tuple[dict, float]:
    """Roofline of the dominant kernel for one launch of B payload bytes per PE, and the step's
    roofline time t_roof (for the algbw targets).
      world == 1  copy kernel (1-PE reduce = dest = source): 2B of HBM traffic, HBM-bound.
      share > 1   several PEs on one device (rehearsal): the collective never touches xGMI, so the
                  bound is the device's HBM and the achieved rate is the device-total traffic of
                  the `share` co-located PEs, share * (3 - 1/p) * B per launch.
      otherwise   one PE per GPU: per-PE xGMI ingress 2(p-1)/p * B over p-1 links, against the
                  brief's 153.6 GB/s per link (HBM (3 - 1/p) * B enters t_roof too).
    A ratio above 1 means the model is not what bounds the run: the line then says so
    (model_violated, reason) and carries no frac."""
    t = kern_ms * 1e-3
    if world == 1:
        roof = {"bound": "hbm", "achieved": 2 * B / t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "traffic": pmc_traffic("copy_1pe", B),
                "kernel": "fanin_kernel<uint8,OR,vec> (1-PE reduce = copy, 2B per launch)"}
        t_roof = 2 * B / (HBM_PEAK_GBS * 1e9)
    elif share > 1:
        hbm_f = world + 1.0 if "whole-array" in kernel else 3.0 - 1.0 / world  # per PE: reads, then the dest write
        dev_bytes = share * hbm_f * B
        roof = {"bound": "hbm", "achieved": dev_bytes / t / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "pes_per_device": share,
                "traffic": pmc_traffic(f"{'phased' if kernel.startswith('rs_phase') else 'allreduce'}_{world}pe_same_device", B)
                if share == world else None,
                "traffic_note": "device-wide FETCH_SIZE (x2) + WRITE_SIZE per launch, all PEs on one GPU "
                                "(profiles/pmc_summary.json)",
                "kernel": f"{kernel} x {share} co-located PEs "
                          f"(device HBM traffic {share} x {hbm_f:.3g} x B per launch)"}
        t_roof = dev_bytes / (HBM_PEAK_GBS * 1e9)
    else:
        whole = "whole-array" in kernel  # each member pulls every peer's whole source
        link_bytes = (world - 1.0) * B if whole else 2.0 * (world - 1) / world * B  # ingress per PE, p-1 links
        roof = {"bound": "xgmi", "achieved": link_bytes / t / 1e9,
                "peak": XGMI_LINK_GBS * (world - 1), "unit": "GB/s", "traffic": None,
                "traffic_note": "no PMC pass of a one-PE-per-GPU run is committed (the round's GPU "
                                "pool has one GPU per box): HBM traffic per launch unmeasured",
                "kernel": f"{kernel} (per-PE xGMI ingress {'(p-1)*B' if whole else '2(p-1)/p*B'})"}
        hbm_f = world + 1.0 if whole else 3.0 - 1.0 / world
        t_roof = max(hbm_f * B / (HBM_PEAK_GBS * 1e9),
                     (link_bytes / (world - 1)) / (XGMI_LINK_GBS * 1e9))
    frac = roof["achieved"] / roof["peak"]
    if frac > 1.0:
        roof.update(frac=None, frac_raw=frac, model_violated=True,
                    reason=f"achieved {roof['achieved']:.0f} GB/s exceeds the {roof['bound']} peak "
                           f"{roof['peak']:.0f} GB/s: that bound is not what limits this run")
    else:
        roof["frac"] = frac
    return roof, t_roof


def phase_breakdown(ish, B: int, world: int, share: int, dist, step, barrier) -> dict:
    """One more call of the timed step with HIP events between the phased path's five launches
    (set_param "phase_events", ishmemi_c_phase_times): start barrier, reduce-scatter grid, middle
    barrier, all-gather grid, end barrier, each the max over ranks.  Per-PE link ingress of each
    grid is (p - 1)/p * B; on one GPU (share > 1) the device's HBM traffic of the co-located PEs
    is share * (1 + 1/p) * B for the reduce-scatter and share * 2 (p - 1)/p * B for the
    all-gather."""
    import ctypes
    L = ish.lib()
    ish.set_param("phase_events", 1)
    try:
        barrier()
        step()
        ms = (ctypes.c_float * 5)()
        if L.ishmemi_c_phase_times(ms) != 0:
            raise RuntimeError(ish.last_error())
        barrier()
    finally:
        ish.set_param("phase_events", 0)
    t = max_over_ranks(dist, [float(x) for x in ms])
    names = ["start_barrier", "reduce_scatter", "mid_barrier", "all_gather", "end_barrier"]
    out = {"ms": dict(zip(names, t))}
    ingress = (world - 1) / world * B
    out["ingress_GBps_per_pe"] = {"reduce_scatter": ingress / (t[1] * 1e-3) / 1e9,
                                  "all_gather": ingress / (t[3] * 1e-3) / 1e9}
    if share > 1:
        rs_dev = share * (1 + 1 / world) * B
        ag_dev = share * 2 * (world - 1) / world * B
        out["device_hbm_GBps"] = {"reduce_scatter": rs_dev / (t[1] * 1e-3) / 1e9,
                                  "all_gather": ag_dev / (t[3] * 1e-3) / 1e9}
    return out


def max_over_ranks(dist, vals: list[float]) -> list[float]:
    if dist is None:
        return vals
    import torch
    t = torch.tensor(vals, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t]


def device_errors(ish) -> float:
    """Device-side spin timeouts recorded so far on this PE (library error words)."""
    return float(ish.lib().ishmemi_c_error_count())


def legs_healthy(ish, dist) -> bool:
    """Collective over the ranks: True while no PE has recorded a device timeout.  Once one has,
    the team's later collectives could each wait out the device timeout, so the remaining GPU legs
    are skipped on every rank alike and the line already measured is emitted."""
    return max_over_ranks(dist, [device_errors(ish)])[0] == 0


def config5_sweep(ish, hip, world, rank, dist, stream, nbytes_max, share: int = 1):
    """BASELINE configs[4]: min/max/prod x int32/float64, 4 KiB .. nbytes_max per PE in steps of 4x:
    us per call (max over ranks), algbw, and a check of EVERY word of dest on every rank at every
    size (the device checker, tests/cpp/pattern_check.hip) against the team-order fold of the
    rotating-winner pattern (selfcheck.pattern: non-periodic, a different value on every PE, the
    min / max winner rotating over the PEs)."""
    from ishmem_amd import selfcheck as sc
    out = []
    phased_min, fold_limit = ish.get_param("phased_min_bytes"), ish.get_param("fold_limit_bytes")
    for dtn, npd in (("int32", np.int32), ("double", np.float64)):
        es = np.dtype(npd).itemsize
        nmax = nbytes_max // es
        src, dst = ish.ishmem_malloc(nbytes_max), ish.ishmem_malloc(nbytes_max)
        if not (src and dst):
            raise RuntimeError(f"config-5 sweep: {ish.last_error()}")
        sc.upload_pattern(hip, src, npd, rank, world, nmax)
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
                us, errs = max_over_ranks(dist, [e0.elapsed_ms(e1) * 1000.0 / it, device_errors(ish)])
                if errs:  # every rank sees the same max: all stop here together
                    raise RuntimeError(f"device timeouts at {op} {dtn} {nb} B: {ish.last_error()}")
                if sc.checker_kind(npd) == "device" or nb <= (64 << 20):
                    wins = [(0, n)]
                else:  # checker not built: host-side windows (edges of every chunk, the end, random)
                    nitems = nb // 16
                    wins = []
                    for c in range(world):
                        b0, e0_ = ish.chunk_bounds(nitems, world, c)
                        for edge in (b0, e0_):
                            lo = max(0, edge * (16 // es) - 2048)
                            wins.append((lo, min(n, lo + 4096) - lo))
                    wins.append((n - 4096, 4096))
                    wins += [(int(x), 4096) for x in np.random.default_rng(5).integers(0, n - 4096, 8)]
                bad = sum(sc.count_wrong(hip, dst, op, npd, world, lo, m) for lo, m in wins)
                bad = int(max_over_ranks(dist, [float(bad)])[0])
                _, t_roof = roofline(world, share, nb, us * 1e-3,
                                     multi_pe_kernel(nb, phased_min, world, fold_limit))
                out.append({"op": op, "dtype": dtn, "bytes": nb, "us": round(us, 2),
                            "algbw_GiBps": round(nb / GiB / (us * 1e-6), 2),
                            # t_roof / t: the same bound as the line's roofline (xGMI links one PE
                            # per GPU, device HBM when PEs share a GPU); mid sizes are latency-bound
                            "roofline_frac": round(t_roof / (us * 1e-6), 3),
                            "checked": bad == 0, "words_checked": sum(m for _, m in wins),
                            "checker": sc.checker_kind(npd)})
                nb *= 4
        ish.ishmem_free(dst)
        ish.ishmem_free(src)
    return out


def xgmi_tuning(ish, hip, src, dst, B, world, dist, stream):
    """N>1: the f32 sum again under other launch shapes, set alike on every rank, so the driver's
    multi-GPU run records how the xGMI path responds (data for choosing the defaults; one
    MI355X per PE cannot be rehearsed on a one-GPU box):
      wait  - the persistent kernel (phased path off) at 1 / 4 / 16 MiB with wait_slots 4 / 8 / 16 /
              32: each waiting launch may hold 1 / wait_slots of the device (kernels.h, "Waiting
              footprint"; 16 = 64 workgroups is the default) — whether that grid fills the links;
      phased - 2 / 4 / 8 / 16 / 64 MiB and the payload on the phased path (one-shot grids
               between barriers) and on the persistent kernel (the phased threshold, 4 MiB);
      phased_peer_nt - 64 MiB and the payload on the phased path with nontemporal peer loads
               (the collectives issue sc0 sc1 ones; the tripwire_peer_nt leg checks coherence);
      p2    - two PEs: one-shot fold vs reduce-scatter + all-gather at the payload size;
      fold  - 512 KiB - 4 MiB (2 PEs: to 64 MiB): the whole-array fold between two barriers forced
              for this team size against the path without it (granule path off in both);
      ll    - 4 KiB up to the granule ring's capacity (2 MiB / team size) with the one-hop granule
              path on (default) and off."""

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
        ms, errs = max_over_ranks(dist, [e0.elapsed_ms(e1) / iters, device_errors(ish)])
        if errs:
            raise RuntimeError(f"device timeouts at {n * 4} B: {ish.last_error()}")
        return ms

    out = []

    def run(case, param, value, nbytes, iters, also=None):
        params = {param: value, **(also or {})}
        old = {k: ish.get_param(k) for k in params}
        for k, v in params.items():
            ish.set_param(k, v)
        try:
            ms = timed(nbytes // 4, iters)
        finally:
            for k, v in old.items():
                ish.set_param(k, v)
        out.append({"case": case, **params, "bytes": nbytes, "us": round(ms * 1e3, 2),
                    "algbw_GiBps": round(nbytes / GiB / (ms * 1e-3), 2)})

    # Rows that time reduce-scatter + all-gather turn the whole-array fold off (co-located bound
    # oneshot_p2, cross-device bound xgmi_fold_max_bytes: runtime.cpp path_limits).
    no_fold = {"oneshot_p2_max_bytes": 0, "xgmi_fold_max_bytes": 0}
    for ws in (4, 8, 16, 32):
        for nb in (1 << 20, 4 << 20, 16 << 20):
            if nb <= B:
                run("wait", "wait_slots", ws, nb, 20, also={"phased_min_bytes": -1, **no_fold})
    for nb in sorted({2 << 20, 4 << 20, 8 << 20, 16 << 20, 64 << 20, B}):
        if nb <= B:
            run("phased", "phased_min_bytes", 0, nb, 5 if nb == B else 20, also=no_fold)
            run("persistent", "phased_min_bytes", -1, nb, 5 if nb == B else 20, also=no_fold)
    for nb in sorted({64 << 20, B}):
        if nb <= B:  # the phased grids' peer loads nontemporal instead of sc0 sc1 (measurement only)
            run("phased_peer_nt", "phased_peer_nt", 1, nb, 5 if nb == B else 20, also={"phased_min_bytes": 0, **no_fold})
    if world == 2:
        run("p2_oneshot", "oneshot_p2_max_bytes", 1 << 40, B, 5, also={"xgmi_fold_max_bytes": 1 << 40})
        run("p2_rs_ag", "oneshot_p2_max_bytes", 0, B, 5, also={"xgmi_fold_max_bytes": 0})
    # The whole-array fold (two barriers around one grid in which every member folds every
    # member's source) against the default path below it, at mid sizes: decided on one GPU for
    # 2-4 PEs; over xGMI each member pulls (p - 1) * B instead of 2(p - 1)/p * B.
    # Two members: up to 64 MiB as well, so the crossover with reduce-scatter + all-gather is
    # bracketed by measured sizes (the `recommended` block reads the largest size the fold won).
    fold_sizes = [512 << 10, 1 << 20, 2 << 20, 4 << 20] + ([8 << 20, 16 << 20, 32 << 20, 64 << 20] if world == 2 else [])
    for nb in fold_sizes:
        if nb <= B:
            run("fold", "direct_max_pes", max(2, world), nb, 20,
                also={"direct_p2": 1, "oneshot_p2_max_bytes": 1 << 40, "xgmi_fold_max_bytes": 1 << 40,
                      "ll_max_bytes": 0})
            run("no_fold", "direct_p2", 0, nb, 20, also={"ll_max_bytes": 0})
    cap = int(ish.get_param("ll_capacity_bytes"))  # the ring's capacity at this team size (the leg
    # times the granule path up to it, past the default threshold ll_limit_bytes where that is lower)
    for nb in (4096, 16384, 65536, 131072, 262144, 524288):
        if nb <= cap:
            run("ll_on", "ll_max_bytes", cap, nb, 50, also={"xgmi_ll_max_bytes": cap})
            run("ll_off", "ll_max_bytes", 0, nb, 50)
    return out


def recommended(rows: list, world: int, share: int, B: int) -> dict:
    """The path thresholds the xgmi_tuning rows measured, as the environment
    a run on this topology would set, so the node run yields its defaults directly:
      granule path - the largest size up to which ll_on beat ll_off at every measured size;
      fold         - the largest size up to which the whole-array fold beat the path without it at
                     every measured size (2 PEs: past 4 MiB when p2_oneshot also beat p2_rs_ag at B);
      phased       - the smallest size from which phased beat persistent at every larger size.
    share == 1 (one PE per GPU): the cross-device variables (ISHMEM_XGMI_*, runtime.cpp
    path_limits); co-located PEs: the variables of round 5's co-located crossovers."""
    def us(case, nb):
        for r in rows:
            if r.get("case") == case and r.get("bytes") == nb and "us" in r:
                return r["us"]
        return None

    def prefix_limit(a_case, b_case):
        lim, pairs = 0, []
        for nb in sorted({r["bytes"] for r in rows if r.get("case") == a_case}):
            a, b = us(a_case, nb), us(b_case, nb)
            if a is None or b is None:
                break
            pairs.append([nb, a, b])
            if a >= b:
                break
            lim = nb
        return lim, pairs

    env, basis = {}, {}
    cross = share == 1
    ll, basis["ll_on_vs_ll_off_us"] = prefix_limit("ll_on", "ll_off")
    env["ISHMEM_XGMI_LL_MAX_BYTES" if cross else "ISHMEM_LL_MAX_BYTES"] = ll
    fold, basis["fold_vs_no_fold_us"] = prefix_limit("fold", "no_fold")
    fold_sizes = [p[0] for p in basis["fold_vs_no_fold_us"]]
    if world == 2 and fold_sizes and fold == fold_sizes[-1]:
        a, b = us("p2_oneshot", B), us("p2_rs_ag", B)
        basis["p2_oneshot_vs_rs_ag_us_at_payload"] = [B, a, b]
        if a is not None and b is not None and a < b:
            fold = B
    if world <= 4:
        if cross:
            env["ISHMEM_XGMI_FOLD_MAX_BYTES"] = fold
        else:  # co-located: 2 members fold up to oneshot_p2, 3-4 up to oneshot_p2 / 4 / (p - 1)
            env["ISHMEM_ONESHOT_P2_MAX_BYTES"] = fold if world == 2 else fold * 4 * (world - 1)
    thr, pp = None, []
    for nb in sorted({r["bytes"] for r in rows if r.get("case") == "phased"}, reverse=True):
        a, b = us("phased", nb), us("persistent", nb)
        if a is None or b is None:
            break
        pp.append([nb, a, b])
        if a >= b:
            break
        thr = nb
    basis["phased_vs_persistent_us"] = sorted(pp)
    env["ISHMEM_PHASED_MIN_BYTES"] = thr if thr is not None else -1
    return {"env": env, "basis": basis, "topology": "one PE per GPU (cross-device teams)" if cross
            else f"{share} PEs per GPU (co-located teams)"}


def link_topology(hip, device: int, world: int) -> list | dict:
    """Link type and hop count from this GPU to every other rank's GPU (hipExtGetLinkTypeAndHopCount;
    HSA link types: 2 PCIe, 4 xGMI), so an N > 1 line says what the collective ran over."""
    names = {0: "hypertransport", 1: "qpi", 2: "pcie", 3: "infiniband", 4: "xgmi"}
    try:
        L = hip.lib()
        fn = L.hipExtGetLinkTypeAndHopCount
        fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        out = []
        for d in range(world):
            if d == device:
                continue
            lt, hc = ctypes.c_uint32(0), ctypes.c_uint32(0)
            rc = fn(device, d, ctypes.byref(lt), ctypes.byref(hc))
            out.append({"peer_device": d, "link": names.get(lt.value, str(lt.value)) if rc == 0 else None,
                        "hops": hc.value if rc == 0 else None, "rc": rc})
        return out
    except Exception as ex:
        return {"error": str(ex)}


def xgmi_probe(ish, hip, src, dst, B, world, rank, dist, stream, barrier):
    """Measured link rates (report against the spec AND a measured L).  Plain
    pulls of a peer's source through the local combine kernel, no barriers inside:
      pull1   — every rank copies S bytes from rank+1 (ring: each link busy in one direction)
      pullall — every rank folds the sources of all p-1 peers (ingress (p-1)*S per GPU)
      push1   — every rank writes S bytes into rank+1's dest (remote stores)
    pull1 / pullall load nontemporal; the *_sc twins issue the system-coherent (sc0 sc1) loads the
    collectives use on peer memory."""
    S = min(B, 256 << 20)
    ns = S // 4
    peers = [(rank + d) % world for d in range(1, world)]
    probe = {}
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
        ms, errs = max_over_ranks(dist, [e0.elapsed_ms(e1) / k, device_errors(ish)])
        if errs:
            raise RuntimeError(f"device timeouts in probe {name}: {ish.last_error()}")
        gbs = len(srcs) * S / (ms * 1e-3) / 1e9
        probe[name] = {"bytes_per_peer": S, "peers": len(srcs), "ms": round(ms, 4),
                       "ingress_GBps": round(gbs, 1), "per_link_GBps": round(gbs / len(srcs), 1)}
    barrier()
    return probe


def rccl_allreduce(dist, device, n, B, world, steps, line, limit_s=240.0):
    """N>1 comparison only: RCCL (torch "nccl" backend) all_reduce of the
    same f32 payload over the same GPUs, after this library has released its heap.  A watchdog
    bounds the leg: if RCCL does not finish within limit_s, rank 0 prints the line already
    measured (marked) and every rank exits with status 3, so the main measurement is never lost
    and the hung leg still shows as a failed run."""
    import threading

    import torch

    def expire():
        if line is not None:
            line["rccl_allreduce"] = {"error": f"did not finish within {limit_s:.0f} s"}
            emit(line)
        sys.stdout.flush()
        os._exit(3)

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
        tr = max_over_ranks(dist, [time.perf_counter() - t0])[0]
        buf.fill_(1.0)
        dist.all_reduce(buf, group=pg)
        ok = bool(torch.all(buf == float(world)).item())
        del buf
        torch.cuda.synchronize()
        dist.destroy_process_group(pg)
        return {"value": world * B / GiB / (tr / steps), "algbw_GiBps": B / GiB / (tr / steps),
                "unit": "GiB/s", "ms_per_step": tr / steps * 1000.0, "steps": steps, "checked": ok}
    except Exception as ex:
        return {"error": str(ex)}
    finally:
        wd.cancel()


def mpich_baseline(ns: int, pes=(1, 2, 4, 8), device_mod: int = 1) -> list | dict:
    """The same host path with the reference's own runtime call on the host side: MPICH's
    MPI_Allreduce on each 64 KiB bounce chunk (runtime_mpi.cpp:802-812), p processes under
    mpiexec, all on this GPU (oracle/mpi_bounce.c; built by __graft_entry__.build when MPICH is
    installed).  Per-PE GiB/s of the slowest rank, result checked on every rank.  device_mod: the
    MPI ranks use devices rank % device_mod (1: all on this GPU; N>1 runs pass N, one per GPU)."""
    exe, mpiexec = ROOT / "oracle" / "mpi_bounce", Path("/opt/conda/bin/mpiexec")
    if not (exe.exists() and mpiexec.exists()):
        return {"error": "MPICH (/opt/conda) or oracle/mpi_bounce not present"}
    out = []
    for p in pes:
        try:
            r = subprocess.run([str(mpiexec), "-n", str(p), str(exe), str(ns), str(device_mod)], cwd=str(ROOT),
                               capture_output=True, text=True, timeout=120)
            t, nbytes, bad = r.stdout.split()[-3:]
            out.append({"pes": p, "value": int(nbytes) / GiB / float(t), "unit": "GiB/s (per PE)",
                        "cores": p, "checked": r.returncode == 0 and int(bad) == 0,
                        "sample": f"{int(nbytes) >> 20} MiB f32 per PE, MPICH MPI_Allreduce per 64 KiB chunk"})
        except Exception as ex:
            out.append({"pes": p, "error": f"{type(ex).__name__}: {ex}"})
    return out


def cpu_baseline_leg(ish, hip, src, dst, n, B, world, rank, dist, key) -> tuple[dict, dict]:
    """The reference's host path, restated in oracle/ and timed on the host cores
    (reduce_impl.h:186-228 -> memory.cpp:310-321 -> runtime_mpi.cpp:802-812): every 64 KiB chunk
    of the device source goes through a synchronous device->host hipMemcpy, the shared-memory
    allreduce of the p PEs' chunks, and a synchronous host->device hipMemcpy.
      N = 1: this PE alone over the full 1 GiB (p = 1), then p = 2 / 4 / 8 side by side on a
             64 MiB sample (p - 1 helper processes with their own HIP buffers on this GPU, so
             the p members share its PCIe link), the memcpy-only restatement, and BASELINE
             configs[0] (int32 sum, 2 PEs, host loopback, no GPU).
      N > 1: every rank on its own GPU, p = N, over a 64 MiB-per-PE sample of the payload (the
             p-member exchange costs per chunk grow with p; the sample bounds the leg)."""
    import oracle  # CPU baseline leg only: the reference's host path, restated (test infrastructure)
    op, dt = oracle.OPS["sum"], oracle.DTYPES["float"]
    extra = {}
    if world > 1:
        ns = min(n, (64 << 20) // 4)
        t = oracle.host_bounce_time(op, dt, ns, rank, world, key + "cpu", src, dst, reps=3)
        t = max_over_ranks(dist, [t])[0]
        # The same with MPICH's MPI_Allreduce, N processes one per GPU (rank 0 launches them while
        # the bench ranks wait).
        if rank == 0 and os.environ.get("ISHMEM_BENCH_SAME_DEVICE") == "1" and 2 * world > 12:
            # Rehearsal with every rank on one GPU: N MPI processes beside the N ranks would exceed
            # the processes a one-GPU box lets use its GPU at once (16).
            extra["cpu_baseline_mpich"] = {"skipped": f"{world} ranks + {world} MPI processes on one GPU "
                                                      "exceed the box's per-GPU process limit"}
        elif rank == 0:
            extra["cpu_baseline_mpich"] = mpich_baseline(ns, pes=(world,), device_mod=world)
        dist.barrier()
        return ({"value": ns * 4 / GiB / t, "unit": "GiB/s", "cores": world, "kind": "port",
                 "per": "per PE (B/t, compare algbw_GiBps)",
                 "whole_job_GiBps": world * ns * 4 / GiB / t,
                 "sample": f"{world} PEs x {ns * 4 >> 20} MiB f32 sum (a sample of the {B / 2**20:g} "
                           f"MiB payload), one process per GPU, 64 KiB chunks each D2H hipMemcpy -> "
                           f"shm allreduce -> H2D hipMemcpy (reduce_impl.h:186-228), best of 3",
                 "host": host_info()}, extra)
    t1 = oracle.host_bounce_time(op, dt, n, 0, 1, key + "cpu1", src, dst, reps=3)
    cpu = {"value": B / GiB / t1, "unit": "GiB/s", "cores": 1, "kind": "port",
           "sample": f"full workload: 1 PE f32 sum of {B / 2**20:g} MiB, 64 KiB chunks each through "
                     f"a synchronous D2H hipMemcpy, the (1-member) allreduce and a synchronous H2D "
                     f"hipMemcpy (reduce_impl.h:186-228, memory.cpp:310-321), best of 3",
           "host": host_info()}
    side = []
    ns = min(n, (64 << 20) // 4)
    for p in (2, 4, 8):
        k = f"{key}cpu{p}"
        helpers = [subprocess.Popen([sys.executable, "-m", "oracle.bounce_helper", "--me", str(me),
                                     "--npes", str(p), "--key", k, "--n", str(ns)],
                                    cwd=str(ROOT), stdout=subprocess.PIPE, stderr=subprocess.DEVNULL,
                                    text=True) for me in range(1, p)]
        try:
            t = oracle.host_bounce_time(op, dt, ns, 0, p, k, src, dst, reps=1)
            ts = [t] + [float(h.communicate(timeout=120)[0].strip()) for h in helpers]
            side.append({"pes": p, "value": ns * 4 / GiB / max(ts), "unit": "GiB/s (per PE)",
                         "cores": p, "sample": f"{ns * 4 >> 20} MiB f32 per PE, {p} processes on "
                                               f"this one GPU (its PCIe link shared)"})
        except Exception as ex:
            side.append({"pes": p, "error": str(ex)})
        finally:
            for h in helpers:
                if h.poll() is None:
                    h.kill()
    extra["cpu_baseline_pes"] = side
    extra["cpu_baseline_mpich"] = mpich_baseline(ns)
    tm = oracle.host_proxy_time(op, dt, n, 1, 2)
    extra["cpu_baseline_memcpy_only"] = {
        "value": B / GiB / tm, "unit": "GiB/s", "cores": 1, "kind": "port",
        "sample": "round-1 restatement: the same 64 KiB chunking with host memcpys in place of "
                  "the device copies (optimistic), full workload, best of 2"}
    n1 = 16 << 20
    t1 = oracle.host_proxy_time(oracle.OPS["sum"], oracle.DTYPES["int32"], n1, 2, 3)
    extra["cpu_config1"] = {"value": n1 * 4 / GiB / t1, "unit": "GiB/s", "cores": 2, "kind": "port",
                            "sample": "BASELINE configs[0]: int32 sum-reduce, 2 PEs (processes), "
                                      "64 MiB per PE, 64 KiB bounce chunks, host loopback, best of 3"}
    return cpu, extra


def pcie_probe(hip, hs: int, hd: int, B: int, dist) -> dict:
    """hipMemcpyAsync of B bytes pinned host -> HBM and HBM -> pinned host on their own streams:
    each direction alone, then both at once (GB/s, max time over ranks), 2 reps each."""
    d1, d2 = hip.malloc(B), hip.malloc(B)
    s1, s2 = hip.stream_create(), hip.stream_create()
    try:
        def timed(jobs, reps=2):
            for dst, src, st in jobs:  # warm-up
                hip.memcpy_async(dst, src, B, st)
            for _, _, st in jobs:
                hip.stream_synchronize(st)
            t0 = time.perf_counter()
            for _ in range(reps):
                for dst, src, st in jobs:
                    hip.memcpy_async(dst, src, B, st)
            for _, _, st in jobs:
                hip.stream_synchronize(st)
            return max_over_ranks(dist, [(time.perf_counter() - t0) / reps])[0]
        h2d = B / timed([(d1, hs, s1)]) / 1e9
        d2h = B / timed([(hd, d2, s2)]) / 1e9
        both = B / timed([(d1, hs, s1), (hd, d2, s2)]) / 1e9  # each direction's rate while both run
        return {"h2d_GBps": round(h2d, 2), "d2h_GBps": round(d2h, 2), "concurrent_min_GBps": round(both, 2),
                "bytes": B, "note": "hipMemcpyAsync, pinned host <-> HBM; concurrent = H2D and D2H on two streams"}
    except Exception as ex:
        return {"error": str(ex)}
    finally:
        hip.stream_destroy(s1)
        hip.stream_destroy(s2)
        hip.free(d1)
        hip.free(d2)


def e2e_leg(ish, hip, n, B, world, rank, dist, stream, barrier, steps, pinned: bool) -> dict:
    """Host-memory end-to-end rate: the blocking ishmem_float_sum_reduce on host source / dest —
    the reference's host path (reduce_impl.h:186-228, :301-315) is a blocking host call — each
    call returning with dest final; every word of dest checked.  Also timed: the same calls
    issued back to back on a stream (ishmemx_*_on_stream, one synchronize at the end)."""
    from ishmem_amd import selfcheck as sc
    try:
        if pinned:
            hs, hd = hip.host_malloc(B), hip.host_malloc(B)
            xs = np.ctypeslib.as_array((ctypes.c_float * n).from_address(hs))
            xd = np.ctypeslib.as_array((ctypes.c_float * n).from_address(hd))
        else:
            xs, xd = np.zeros(n, np.float32), np.zeros(n, np.float32)  # pages touched before timing
            hs, hd = xs.ctypes.data, xd.ctypes.data
        for lo in range(0, n, 1 << 26):  # same synthetic input as the device-resident run
            m = min(1 << 26, n - lo)
            xs[lo:lo + m] = sc.pattern(rank, world, lo, m, np.float32)

        def step_e2e():
            return ish.ishmem_float_sum_reduce(hd, hs, n)

        def step_on_stream():
            return ish.ishmemx_float_sum_reduce_on_stream(hd, hs, n, 0, stream)
        # Warm-up, each call timed: the first DMA passes over a process's newly pinned memory run
        # slow (round 4, tools/host_flavours_ab.py AB_MODE=warmup: fresh hipHostMalloc buffers
        # 20.9, 32.2, then 43.2 GiB/s per call), so the timed calls below are the steady state and
        # the warm-up rates are reported beside them.
        warm = []
        for _ in range(3):
            tw0 = time.perf_counter()
            if step_e2e() != 0:
                raise RuntimeError(ish.last_error())
            hip.stream_synchronize(stream)
            warm.append(round(max_over_ranks(dist, [time.perf_counter() - tw0])[0], 6))
        k = max(2, steps // 5)
        barrier()
        ts0 = time.perf_counter()
        for _ in range(k):
            if step_on_stream() != 0:
                raise RuntimeError(ish.last_error())
        hip.stream_synchronize(stream)
        ts = max_over_ranks(dist, [time.perf_counter() - ts0])[0]
        xd.fill(-1.0)  # the timed blocking calls must write every word
        barrier()
        te0 = time.perf_counter()
        for _ in range(k):
            if step_e2e() != 0:
                raise RuntimeError(ish.last_error())
        hip.stream_synchronize(stream)
        te = time.perf_counter() - te0
        barrier()
        te = max_over_ranks(dist, [te])[0]
        bad = 0
        for lo in range(0, n, 1 << 26):
            m = min(1 << 26, n - lo)
            want = sc.pattern_expected("sum", np.float32, world, lo, m)
            bad += int(np.count_nonzero(xd[lo:lo + m].view(np.uint32) != want.view(np.uint32)))
        bad = int(max_over_ranks(dist, [float(bad)])[0])
        out = {"value": world * B / GiB / (te / k), "algbw_GiBps": B / GiB / (te / k),
               "unit": "GiB/s", "ms_per_step": te / k * 1000.0, "steps": k,
               "checked": bad == 0, "words_checked": n, "mode": "every word, every rank",
               "warmup_GiBps_per_call": [round(B / GiB / t, 2) for t in warm],
               "calls": "blocking ishmem_float_sum_reduce, each returning with dest final",
               "on_stream_back_to_back_GiBps": round(world * B / GiB / (ts / k), 2),
               "buffers": "pinned host (hipHostMalloc)" if pinned else "pageable host (malloc'd numpy)",
               "pipeline": "H2D | reduce | D2H through the staging slots (ISHMEM_STAGING_SLOTS, default 2 x 64 MiB)"}
        if pinned:
            # What bounds the leg: plain DMA copies of the same B between these pinned buffers and
            # HBM, each direction alone and both at once (the pipeline moves B each way per step).
            out["pcie_probe"] = pcie_probe(hip, hs, hd, B, dist)
            both = out["pcie_probe"].get("concurrent_min_GBps")
            if both:
                out["frac_of_concurrent_dma"] = (B / (te / k) / 1e9) / both
        del xs, xd
        if pinned:
            hip.host_free(hs)
            hip.host_free(hd)
        return out
    except Exception as ex:  # reported, never fatal for the main measurement
        return {"error": str(ex)}


def main() -> int:
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
    ap.add_argument("--no-tripwire", action="store_true")
    ap.add_argument("--no-full-check", action="store_true")
    ap.add_argument("--sweep-max-mib", type=int, default=CFG5_MAX_BYTES >> 20)
    ap.add_argument("--nelems", type=int, default=0, help="override: float32 elements per PE")
    ap.add_argument("--no-rccl", action="store_true",
                    help="N>1: skip the RCCL all_reduce comparison on the same payload")
    ap.add_argument("--no-tuning", action="store_true", help="N>1: skip the launch-shape sweep")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args)
    # Native libraries (gloo, RCCL, HIP) may print to fd 1; keep stdout for the one JSON line by
    # pointing fd 1 at stderr and writing the line to a duplicate of the original stdout.
    global _OUT
    sys.stdout.flush()
    _OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise RuntimeError(f"--gpus {args.gpus} but the launcher started {world} ranks")
    same_device = os.environ.get("ISHMEM_BENCH_SAME_DEVICE") == "1"
    # ISHMEM_BENCH_EMULATE_SHARE1=1 with ISHMEM_BENCH_SAME_DEVICE=1 (development only): every rank
    # reports its own device (the test-hooks library's ISHMEM_TEST_PCI_BUS), so the team counts as
    # one PE per GPU — the cross-device thresholds, launch shapes and `recommended` keys of the node
    # — while the ranks still share this box's one GPU.  Never used for reported numbers.
    emulate_share1 = same_device and os.environ.get("ISHMEM_BENCH_EMULATE_SHARE1") == "1"
    if emulate_share1:
        os.environ["ISHMEM_TEST_PCI_BUS"] = f"fake-bus-{rank}"
        os.environ.setdefault("ISHMEM_AMD_LIB", str(ROOT / "ishmem_amd" / "libishmem_amd_testhooks.so"))
    n = args.nelems if args.nelems > 0 else (args.mib << 20) // 4
    B = n * 4
    sweep_max = min(args.sweep_max_mib << 20, CFG5_MAX_BYTES)
    if world > 1 and "ISHMEM_SYMMETRIC_SIZE" not in os.environ:
        # The config-5 sweep holds a 4 GiB source and dest per PE (plus the 128 MiB staging
        # region): size the symmetric heap for it (288 GB of HBM per GPU).
        os.environ["ISHMEM_SYMMETRIC_SIZE"] = str(max(2 * B, 2 * sweep_max) + (1 << 30))
    # The library and the ctypes HIP bindings are loaded BEFORE torch: torch ships its own copy of
    # the HIP / HSA runtime (ROCm 7.0, same sonames as the image's 7.2), and whichever loads first
    # serves the whole process.  Loaded first, the image's runtime serves the library, the bindings
    # and torch alike — the configuration every GPU test runs in.  With torch first, the library
    # ran on torch's copy, and the 2-PE rehearsal that was a box's first GPU process stalled inside
    # hipIpcOpenMemHandle of the peer's heap (the setup watchdog's thread dump, profiles/r06/init/
    # r06f_bench_local2_stall.txt), as round 5's r05zm run had stalled after HIP's start.
    watchdog = threading.Timer(float(os.environ.get("ISHMEM_BENCH_SETUP_WATCHDOG_S", "45")), stall_report,
                               args=("setup (library load, ishmem init, heap allocation, input upload)",))
    watchdog.daemon = True
    watchdog.start()
    import ishmem_amd as ish
    from ishmem_amd import hip
    hip.lib()
    try:  # and the image's HSA runtime under the name torch's HIP-side libraries ask for
        ctypes.CDLL("libhsa-runtime64.so", mode=ctypes.RTLD_GLOBAL)
    except OSError:
        pass
    dist = None
    key = f"bench{uuid.uuid4().hex[:10]}"
    if world > 1:
        import torch.distributed as dist  # control plane only (gloo); the data path is ours
        dist.init_process_group("gloo")
        obj = [key]
        dist.broadcast_object_list(obj, src=0)
        key = obj[0]


    # ISHMEM_BENCH_SAME_DEVICE=1 (development only): every rank on device 0, to measure kernel
    # overheads of the multi-PE path on a one-GPU box.  Never used for reported numbers.
    device = 0 if same_device else local_rank
    ish.init(rank, world, device, key)
    # Memory kind the PEs agreed on for the flag rows peers store into (runtime.cpp FlagMem).
    flag_memory = ("uncached", "fine-grained", "coarse-grained")[int(ish.get_param("flags_kind"))]
    src = ish.ishmem_malloc(B)
    dst = ish.ishmem_malloc(B)
    if not (src and dst):
        raise RuntimeError(f"heap allocation failed: {ish.last_error()}")
    # Synthetic input with an exactly representable sum that no misrouted tile, segment or
    # skipped member can reproduce: the rotating-winner pattern (ishmem_amd/selfcheck.py).
    from ishmem_amd import selfcheck as sc
    sc.upload_pattern(hip, src, np.float32, rank, world, n)
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

    watchdog.cancel()
    log("warm-up")
    for _ in range(args.warmup):
        step()
    barrier()
    if ish.lib().ishmemi_c_error_count():
        raise RuntimeError("device barrier timeouts during warm-up (a PE did not arrive)")
    hip.memset(dst, 0xFF, B)  # the timed steps must write every word (checked below)
    barrier()
    ev0, ev1 = hip.Event(), hip.Event()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    hip.stream_synchronize(stream)
    t1 = time.perf_counter()
    barrier()
    wall_s, kern_ms = max_over_ranks(dist, [t1 - t0, ev0.elapsed_ms(ev1) / args.steps])
    if ish.lib().ishmemi_c_error_count():
        raise RuntimeError("device barrier timeouts during the benchmark")

    # Correctness of the timed buffers: every word of dest on every rank.
    log("full check of the timed dest")
    if args.no_full_check:
        idx = np.random.default_rng(0).integers(0, n, 256)
        bad = sum(sc.count_wrong(hip, dst, "sum", np.float32, world, int(i), 1) for i in idx)
        checked = {"words": 256, "mode": "sampled"}
    else:
        bad = sc.count_wrong(hip, dst, "sum", np.float32, world, 0, n)
        checked = {"words": n, "mode": "every word, every rank",
                   "input": "rotating-winner pattern (non-periodic, distinct per PE)",
                   "checker": sc.checker_kind(np.float32)}
    bad = int(max_over_ranks(dist, [float(bad)])[0])
    if bad:
        raise RuntimeError(f"benchmark result check failed: {bad} words wrong")
    checked["wrong"] = 0

    ms_per_step = wall_s * 1000.0 / args.steps
    value = world * B / GiB / (ms_per_step / 1000.0)
    algbw = B / GiB / (ms_per_step / 1000.0)

    share = int(ish.get_param("device_share")) if world > 1 else 1
    roof, t_roof = roofline(world, share, B, kern_ms,
                            multi_pe_kernel(B, ish.get_param("phased_min_bytes"), world,
                                            ish.get_param("fold_limit_bytes")) if world > 1 else "")
    algbw_roof = B / GiB / t_roof
    targets = {"algbw_roofline_GiBps": algbw_roof, "algbw_frac_of_roofline": algbw / algbw_roof}
    if algbw > algbw_roof:
        targets.update(algbw_frac_of_roofline=None, model_violated=True)
    if world == 8 and share == 1:
        targets["algbw_target_GiBps"] = 400.0  # >= 70 % of 572 GiB/s
        targets["met"] = algbw >= 400.0

    extra = {}
    unhealthy = []

    def healthy() -> bool:
        # Checked before each N>1 GPU leg (collective: same answer on every rank).
        if not unhealthy and not legs_healthy(ish, dist):
            unhealthy.append(True)
            extra["legs_skipped"] = "a PE recorded a device timeout; later GPU legs skipped"
        return not unhealthy

    if world == 1 and not args.no_combine:
        log("combine leg")
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

    if world > 1 and healthy() and roof["kernel"].startswith("rs_phase"):
        log("phase breakdown")
        try:
            extra["phases"] = phase_breakdown(ish, B, world, share, dist, step, barrier)
        except Exception as ex:
            extra["phases"] = {"error": str(ex)}

    if world > 1 and healthy() and not args.no_probe:
        log("xGMI probe")
        try:
            probe = xgmi_probe(ish, hip, src, dst, B, world, rank, dist, stream, barrier)
            extra["xgmi_probe"] = probe
            # Same accounting as roof["achieved"] (per-PE ingress), against the measured all-peer
            # ingress; only meaningful when the bound is xGMI (one PE per GPU).
            if roof["bound"] == "xgmi":
                roof["peak_measured"] = max(probe["pullall"]["ingress_GBps"], probe["pullall_sc"]["ingress_GBps"])
                roof["frac_measured"] = roof["achieved"] / roof["peak_measured"]
        except Exception as ex:
            extra["xgmi_probe"] = {"error": str(ex)}

    if world > 1 and healthy() and not args.no_tuning:
        log("launch-shape sweep")
        try:
            extra["xgmi_tuning"] = xgmi_tuning(ish, hip, src, dst, B, world, dist, stream)
            extra["recommended"] = recommended(extra["xgmi_tuning"], world, share, B)
        except Exception as ex:
            extra["xgmi_tuning"] = {"error": str(ex)}

    cpu = None
    if not args.no_cpu_baseline and (world > 1 or rank == 0):
        log("CPU baseline leg (reference host path with its 64 KiB device copies)")
        try:
            cpu, more = cpu_baseline_leg(ish, hip, src, dst, n, B, world, rank, dist, key)
            extra.update(more)
        except Exception as ex:
            cpu = {"error": str(ex)}

    ish.ishmem_free(dst)
    ish.ishmem_free(src)

    if world > 1 and healthy() and not args.no_tripwire:
        log("coherence tripwire")
        from ishmem_amd import selfcheck
        try:
            tw = selfcheck.chain_tripwire(ish, hip, rank, world, nmax=16 << 20, iters=8, stream=stream)
            bad = max_over_ranks(dist, [float(sum(tw["mismatches"])), float(not tw["checked"])])
            tw["checked"] = bad[0] == 0 and bad[1] == 0
            tw["mismatches_rank0"] = tw.pop("mismatches")
            tw["mismatches_all_ranks"] = int(bad[0])
            extra["tripwire"] = tw
        except Exception as ex:
            extra["tripwire"] = {"error": str(ex), "checked": False}
        if healthy() and not args.no_tuning:
            # The same chained producer -> reduce check with the phased grids' peer loads
            # nontemporal (measurement mode, phased path forced): does the kernel-boundary acquire
            # alone keep peers' bytes fresh across devices?  Reported, never fatal.
            old_nt, old_min = ish.get_param("phased_peer_nt"), ish.get_param("phased_min_bytes")
            try:
                ish.set_param("phased_peer_nt", 1)
                ish.set_param("phased_min_bytes", 0)
                tw = selfcheck.chain_tripwire(ish, hip, rank, world, nmax=16 << 20, iters=8, stream=stream)
                bad = max_over_ranks(dist, [float(sum(tw["mismatches"])), float(not tw["checked"])])
                extra["tripwire_peer_nt"] = {"checked": bad[0] == 0 and bad[1] == 0,
                                             "mismatches_all_ranks": int(bad[0]), "iters": tw["iters"]}
            except Exception as ex:
                extra["tripwire_peer_nt"] = {"error": str(ex), "checked": False}
            finally:
                ish.set_param("phased_peer_nt", old_nt)
                ish.set_param("phased_min_bytes", old_min)

    if world > 1 and healthy() and not args.no_sweep:
        log("config-5 sweep")
        # BASELINE configs[4] (min/max/prod x int32/float64 across the PEs), 4 KiB .. 4 GiB per PE.
        try:
            extra["config5_sweep"] = config5_sweep(ish, hip, world, rank, dist, stream, sweep_max, share)
        except Exception as ex:
            extra["config5_sweep"] = {"error": str(ex)}

    if not args.no_e2e and (world == 1 or healthy()):
        # Last: its pipeline streams add hardware queues, which oversubscribe the scheduler when
        # several ranks share one GPU (same-device rehearsals) and slow every later leg there.
        log("host-memory end-to-end leg")
        # The path starts and ends in host memory (north star): host source / dest, the library
        # stages H2D -> device reduce -> D2H through HBM as a 3-stream pipeline.  Pinned buffers
        # (hipHostMalloc) and pageable ones (plain malloc'd numpy arrays, the common application
        # case); dest compared in full on every rank.
        extra["e2e_host"] = e2e_leg(ish, hip, n, B, world, rank, dist, stream, barrier, args.steps, pinned=True)
        extra["e2e_host_pageable"] = e2e_leg(ish, hip, n, B, world, rank, dist, stream, barrier,
                                             args.steps, pinned=False)

    hip.stream_destroy(stream)
    ish.ishmem_finalize()
    line = None
    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "value_definition": "whole job: N PEs x B payload bytes / time per step (N*B/t)",
            "algbw_GiBps": algbw,
            "algbw_definition": "per PE: B / time per step (test/include/ishmem_tester.h:1553-1555)",
            "config": {"workload": f"float32 sum-reduce, {B / 2**20:g} MiB per PE, {world} PE(s), "
                                   f"symmetric-heap device buffers", "nreduce": n,
                       "bytes_per_pe": B, "pes": world,
                       "parallelism": "1 PE self-reduce" if world == 1 else f"direct RS+AG over {world} PEs",
                       **({"semantics": "a 1-PE reduce is a copy in the reference (reduce_impl.h:288-289): the "
                                        "timed kernel moves 2 B per payload byte and does no f32 arithmetic; the "
                                        "f32 sum itself is timed in 'combine' (dst = a + b, 3 B per payload byte)"}
                          if world == 1 else {})},
            "kernel_ms": kern_ms, "checked": checked, "targets": targets,
            **({"flag_memory": flag_memory} if world > 1 else {}),
            **({"topology": link_topology(hip, device, world)} if world > 1 and not same_device else {}),
            **({"dev_same_device": True} if same_device else {}),
            **({"dev_emulated_one_pe_per_gpu": True} if emulate_share1 else {}), "roofline": roof,
            "cpu_baseline": cpu, **extra,
        }
    if world > 1 and not args.no_rccl and not same_device:
        log("RCCL comparison leg")
        rccl = rccl_allreduce(dist, device, n, B, world, args.steps, line)
        if line is not None:
            line["rccl_allreduce"] = rccl
    if line is not None:
        emit(line)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    try:
        sys.exit(main())
    except Exception as exc:  # always leave one JSON line for the driver, with the reason
        if int(os.environ.get("RANK", "0")) == 0:
            emit({"metric": METRIC, "value": None, "unit": "GiB/s",
                  "n_gpus": int(os.environ.get("WORLD_SIZE", "1")),
                  "higher_is_better": True, "error": f"{type(exc).__name__}: {exc}"})
        raise
