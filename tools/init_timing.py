#!/usr/bin/env python3
"""Init time by phase: N PEs (processes, all on device 0 of this box) call
ishmem init with ISHMEM_SYMMETRIC_SIZE = each size given, in order; every PE reports the wall time
of its init call, the time from process start to the call (Python + torch-free imports + library
load) and the library's per-phase durations (get_param "init_us_<phase>": hip runtime init, heap
hipMalloc, flag block, bootstrap allgather, heap IPC export/open, flag IPC, teams).  One JSON line
per (size, PE) on stdout.

  python tools/init_timing.py --npes 2 --sizes 1G,4G,9G,1G
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time
import uuid
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PHASES = ("hip", "heap", "flags", "bootstrap", "ipc_heap", "ipc_flags", "teams", "total")


def pe_main(pe, npes, key, size, q, t_spawn, splits=0):
    t_start = time.time()
    os.environ["ISHMEM_SYMMETRIC_SIZE"] = size
    os.environ.setdefault("ISHMEM_DEBUG", "2")
    sys.path.insert(0, str(ROOT))
    import ishmem_amd as ish
    t_imported = time.time()
    t0 = time.perf_counter()
    try:
        ish.init(pe, npes, 0, key)
        ok, err = True, ""
    except RuntimeError as ex:
        ok, err = False, str(ex)
    wall = time.perf_counter() - t0
    rec = {"pe": pe, "npes": npes, "heap": size, "ok": ok, "init_wall_ms": round(wall * 1e3, 1),
           "spawn_to_start_ms": round((t_start - t_spawn) * 1e3, 1),
           "import_ms": round((t_imported - t_start) * 1e3, 1), "err": err}
    if ok:
        rec["phases_ms"] = {p: round(ish.get_param(f"init_us_{p}") / 1e3, 2) for p in PHASES}
        if splits:
            # team_split_strided of WORLD `splits` times (each allocates, exports, exchanges and
            # opens the new team's flag block), then team_destroy of them all: ms per team
            ish.ishmem_barrier_all()
            t1 = time.perf_counter()
            teams = [ish.ishmem_team_split_strided(0, 0, 1, npes)[1] for _ in range(splits)]
            t2 = time.perf_counter()
            for t in teams:
                ish.ishmem_team_destroy(t)
            t3 = time.perf_counter()
            rec["split_ms_per_team"] = round((t2 - t1) * 1e3 / splits, 3)
            rec["destroy_ms_per_team"] = round((t3 - t2) * 1e3 / splits, 3)
            rec["teams_ok"] = sum(t >= 0 for t in teams)
        ish.ishmem_barrier_all()
        ish.ishmem_finalize()
    q.put(rec)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--npes", type=int, default=2)
    ap.add_argument("--sizes", default="1G,4G,9G,1G")
    ap.add_argument("--timeout", type=float, default=120.0)
    ap.add_argument("--splits", type=int, default=0, help="also time this many team splits + destroys (<= 61)")
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    rc = 0
    for size in args.sizes.split(","):
        q = ctx.Queue()
        key = f"it{uuid.uuid4().hex[:10]}"
        t_spawn = time.time()
        procs = [ctx.Process(target=pe_main, args=(pe, args.npes, key, size, q, t_spawn, args.splits)) for pe in range(args.npes)]
        for p in procs:
            p.start()
        got = []
        try:
            for _ in procs:
                got.append(q.get(timeout=args.timeout))
        except Exception as ex:  # a PE that never reports: say so and stop (no retry)
            print(json.dumps({"heap": size, "error": f"a PE did not report within {args.timeout} s: {ex}"}), flush=True)
            rc = 1
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
        for r in sorted(got, key=lambda r: r["pe"]):
            print(json.dumps(r), flush=True)
            rc |= 0 if r["ok"] else 1
        if rc:
            break
    return rc


if __name__ == "__main__":
    sys.exit(main())
