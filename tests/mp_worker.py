"""Worker body of the multi-PE GPU tests: one process = one PE, all PEs on one GPU, symmetric
heaps mapped into each other over HIP IPC — the same code path as one PE per GPU over xGMI.

Each worker regenerates every PE's inputs (deterministic seeds), runs the collective through
the C-ABI and checks its own result against the ORACLE (tests only) and, where the inputs are
the golden ones, against MPICH's MPI_Allreduce output in tests/golden.  Failures are returned
as strings through the queue.
"""
from __future__ import annotations

import os
import time
import traceback
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"


def _bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8))


def run(pe: int, npes: int, key: str, scenarios: list[str], q, env: dict | None = None) -> None:
    fails: list[str] = []
    try:
        for k, v in (env or {}).items():  # a list gives each PE its own value, None removes it
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v[pe] if isinstance(v, list) else v)
        import oracle
        import ishmem_amd as ish
        from ishmem_amd import hip

        if "refuse" in scenarios:
            # Coarse-grained flag memory across devices (ISHMEM_TEST_FLAGS_UNAVAILABLE: as if no
            # uncached / fine-grained VRAM could be shared; ISHMEM_TEST_PCI_BUS: each PE claims its
            # own device): init must fail on every PE with the reason, not warn and continue.
            # With ISHMEM_FLAGS_KIND=2 (a test forcing coarse-grained flags) it must succeed.
            forced = os.environ.get("ISHMEM_FLAGS_KIND") == "2"
            try:
                ish.init(pe, npes, 0, key)
                if not forced:
                    fails.append(f"pe{pe} refuse: init succeeded with coarse-grained flags across devices")
                elif int(ish.get_param("flags_kind")) != 2:
                    fails.append(f"pe{pe} refuse (forced): flags_kind {ish.get_param('flags_kind')}")
                ish.ishmem_finalize()
            except RuntimeError as ex:
                if forced or "coarse-grained" not in str(ex):
                    fails.append(f"pe{pe} refuse: unexpected init outcome: {ex}")
            q.put((pe, fails))
            return

        ish.init(pe, npes, 0, key)
        OPS, DT = oracle.OPS, oracle.DTYPES
        NAMES = {v: k for k, v in DT.items()}
        ONAMES = {v: k for k, v in OPS.items()}

        def heap(n, dt):
            return ish.ishmem_malloc(max(1, n * np.dtype(oracle.NP[dt]).itemsize))

        def check(tag, op, dt, srcs, got, golden=None, me=None):
            me = pe if me is None else me  # this PE's index in the team the srcs belong to
            ref = oracle.reduce_fold(op, dt, srcs, 0)  # canonical team order = every PE's result
            if not _bits_equal(got, ref):
                bad = np.nonzero(got.view(np.uint8) != ref.view(np.uint8))[0]
                fails.append(f"pe{pe} {tag}: {len(bad)} bytes differ from oracle (first byte {bad[:3]})")
                return
            if dt >= 8 and op in (OPS["sum"], OPS["prod"]) and len(srcs) > 1:
                # The reference's own result on THIS PE folds self first, then team order
                # (reduce_impl.h:247-253).  Both folds lie within fp_tolerance of the exact
                # value, so they differ by at most twice that bound.
                own = oracle.reduce_fold(op, dt, srcs, me)
                tol = 2.0 * oracle.fp_tolerance(dt, op, srcs, ref)
                if not np.all(np.abs(own.astype(np.float64) - got.astype(np.float64)) <= tol):
                    fails.append(f"pe{pe} {tag}: outside tolerance of the reference's PE-{me} fold")
            if golden is not None:
                if dt >= 8 and op in (OPS["sum"], OPS["prod"]):
                    tol = oracle.fp_tolerance(dt, op, srcs, ref)
                    if not np.all(np.abs(golden.astype(np.float64) - got.astype(np.float64)) <= tol):
                        fails.append(f"pe{pe} {tag}: outside tolerance vs MPICH golden")
                elif not _bits_equal(golden, got):
                    fails.append(f"pe{pe} {tag}: differs from MPICH golden")

        if "flagkind" in scenarios:
            want = int(os.environ["FLAGKIND_WANT"])
            if int(ish.get_param("flags_kind")) != want:
                fails.append(f"pe{pe} flags_kind {ish.get_param('flags_kind')} != agreed {want}")

        if "arshift0" in scenarios:
            # The persistent kernel's element-granular instantiation for sources on another 16-B
            # phase than dest (set_param "ar_shifted" 0; the default keeps 16-B items and reads
            # the sources with unaligned loads).
            ish.set_param("ar_shifted", 0)

        if "nodirect" in scenarios:
            # Two-member disjoint reduces on the persistent kernel's one-shot mode instead of the
            # barrier-bracketed whole-array fold grid (set_param "direct_p2", alike on every PE).
            ish.set_param("direct_p2", 0)

        if "realigncap" in scenarios:
            # Tests only: at most 3 workgroups for the realigned kernels, so the realigned
            # reduce-scatter's grid-stride loop (edge[] reuse between passes) runs at test sizes.
            ish.set_param("realign_grid_cap", 3)
            # ... and the realigning reduce-scatter kernel (not the default unaligned-load one).
            ish.set_param("phase_unaligned", 0)

        if "teams61" in scenarios:
            # ISHMEM_TEAMS_MAX (src/ishmem/env_defs.h:34, src/teams.cpp:118-121,
            # :369-371): with the default 64 slots a PE holds 61 user teams besides WORLD / SHARED /
            # NODE.  Each split allocates the team's flag block and ring and exchanges them among its
            # members (no longer reserved at init), so: the base footprint is at most round 5's fixed
            # 16-slot block; 61 splits of WORLD succeed, the next fails on every PE naming the
            # variable; reduces on the last team, a middle one and WORLD (granule and fold sizes,
            # int32 bit-exact, in place) match the oracle; destroying them all returns the footprint
            # to the base block, and a second round of splits (slot reuse) works the same.
            W, INV = ish.ISHMEM_TEAM_WORLD, ish.ISHMEM_TEAM_INVALID
            tmax = int(ish.get_param("teams_max"))
            want_max = int(os.environ.get("TEAMS_WANT", 64))
            fb0, fb5 = int(ish.get_param("flag_block_bytes")), int(ish.get_param("flag_block_bytes_round5"))
            if tmax != want_max:
                fails.append(f"pe{pe} teams61: teams_max {tmax} != {want_max}")
            if not 0 < fb0 <= fb5:
                fails.append(f"pe{pe} teams61: base flag footprint {fb0} B exceeds round 5's {fb5} B")
            nmax = 300_000
            s_t, d_t = heap(nmax, DT["int32"]), heap(nmax, DT["int32"])
            for rnd in range(2):
                teams = []
                for k in range(tmax - 3):
                    r, t = ish.ishmem_team_split_strided(W, 0, 1, npes)
                    if r or t == INV:
                        fails.append(f"pe{pe} teams61 round {rnd}: split {k} failed: {ish.last_error()}")
                        break
                    teams.append(t)
                if sorted(teams) != list(range(3, tmax)):
                    fails.append(f"pe{pe} teams61 round {rnd}: slots {sorted(teams)[:4]}.. ({len(teams)})")
                r, t = ish.ishmem_team_split_strided(W, 0, 1, npes)
                if r == 0 or t != INV or "ISHMEM_TEAMS_MAX" not in ish.last_error():
                    fails.append(f"pe{pe} teams61 round {rnd}: split past the table: rc={r} team={t} '{ish.last_error()}'")
                fb = int(ish.get_param("flag_block_bytes"))
                if teams and (fb <= fb0 or (fb - fb0) % len(teams)):
                    fails.append(f"pe{pe} teams61: footprint with {len(teams)} teams {fb} B (base {fb0})")
                for team in ([teams[-1], teams[len(teams) // 2]] if teams else []) + [W]:
                    for n in (1000, nmax):
                        ins = [oracle.fill_random(DT["int32"], 6100 + 31 * rnd + 7 * team + j + n, n) for j in range(npes)]
                        hip.upload(s_t, ins[pe])
                        if ish.ishmem_int32_sum_reduce(team, d_t, s_t, n):
                            fails.append(f"pe{pe} teams61 team {team} n={n}: {ish.last_error()}")
                            continue
                        check(f"teams61 team {team} n={n}", OPS["sum"], DT["int32"], ins, hip.download(d_t, n, np.int32))
                        hip.upload(d_t, ins[pe])  # in place
                        if ish.ishmem_int32_max_reduce(team, d_t, d_t, n):
                            fails.append(f"pe{pe} teams61 in place team {team} n={n}: {ish.last_error()}")
                            continue
                        check(f"teams61 in place team {team} n={n}", OPS["max"], DT["int32"], ins,
                              hip.download(d_t, n, np.int32))
                for t in teams:
                    ish.ishmem_team_destroy(t)
                if int(ish.get_param("flag_block_bytes")) != fb0:
                    fails.append(f"pe{pe} teams61: footprint after destroy {ish.get_param('flag_block_bytes')} != {fb0}")
                # The destroyed teams' blocks stay pooled for reuse: the second round reuses them.
                if int(ish.get_param("flag_block_pool_bytes")) != len(teams) * 8_651_008:
                    fails.append(f"pe{pe} teams61 round {rnd}: pool {ish.get_param('flag_block_pool_bytes')} B "
                                 f"for {len(teams)} teams")
                ish.ishmem_barrier_all()
            ish.ishmem_free(d_t)
            ish.ishmem_free(s_t)

        if "teamchurn" in scenarios:
            # Team churn (round 6): every split allocates, exports and opens a team block, every
            # destroy closes and frees it.  CHURN_ITERS rounds of: split a random strided team of
            # WORLD (and a nested one inside it), reduce on both (random op / type / size up to the
            # fold sizes) against the oracle, destroy both in a random order.  The footprint must
            # come back to the base block, and the device's free memory must not drift (leaked
            # blocks or IPC mappings would show as a steady drop).
            import random
            rng = random.Random(int(os.environ.get("CHURN_SEED", 4242)))
            iters = int(os.environ.get("CHURN_ITERS", 120))
            W, INV = ish.ISHMEM_TEAM_WORLD, ish.ISHMEM_TEAM_INVALID
            fb0 = int(ish.get_param("flag_block_bytes"))
            nmax = 600_000
            s_c, d_c = heap(nmax, DT["double"]), heap(nmax, DT["double"])
            ish.ishmem_barrier_all()
            hip.synchronize()
            free0 = hip.mem_get_info()[0]
            free_mid = None
            for it in range(iters):
                if it == iters // 2:
                    ish.ishmem_barrier_all()
                    hip.synchronize()
                    free_mid = hip.mem_get_info()[0]
                # the same draws on every PE (shared seed)
                stride = rng.choice([1, 1, 2, 3]) if npes >= 3 else 1
                size = rng.randint(1, (npes - 1) // stride + 1)
                start = rng.randint(0, npes - 1 - stride * (size - 1))
                op_n = rng.choice(["sum", "max", "min", "prod", "and", "xor"])
                dt_n = rng.choice(["int32", "int64", "uint8", "float", "double"]) if op_n not in ("and", "xor") else rng.choice(["int32", "uint8", "int64"])
                n = rng.choice([1, 37, 4099, 70_001, 300_000, nmax // 2])
                order = rng.random() < 0.5
                r, t = ish.ishmem_team_split_strided(W, start, stride, size)
                members = [start + k * stride for k in range(size)]
                if r or (t != INV) != (pe in members):
                    fails.append(f"pe{pe} churn {it}: split ({start},{stride},{size}) rc={r} team={t} {ish.last_error()}")
                    break
                t2 = INV
                if t != INV and size >= 2:
                    r2, t2 = ish.ishmem_team_split_strided(t, 0, 1, size - 1)
                    if r2 or (t2 != INV) != (members.index(pe) < size - 1):
                        fails.append(f"pe{pe} churn {it}: nested split rc={r2} team={t2} {ish.last_error()}")
                        break
                for tm, mem in ((t, members), (t2, members[:size - 1])):
                    if tm == INV:
                        continue
                    op, dt = OPS[op_n], DT[dt_n]
                    if not ish.lib().ishmemi_c_op_dtype_valid(op, dt):
                        continue
                    ins = {j: oracle.fill_random(dt, 7700 + 13 * it + j, n) for j in mem}
                    hip.upload(s_c, ins[pe])
                    if ish.reduce(op_n, dt_n, d_c, s_c, n, tm):
                        fails.append(f"pe{pe} churn {it}: reduce {op_n} {dt_n} n={n} team {tm}: {ish.last_error()}")
                        continue
                    check(f"churn {it} {op_n} {dt_n} n={n}", op, dt, [ins[j] for j in mem],
                          hip.download(d_c, n, oracle.NP[dt]), me=mem.index(pe))
                for tm in ((t2, t) if order else (t, t2)):
                    if tm != INV:
                        ish.ishmem_team_destroy(tm)
                if fails:
                    break
            ish.ishmem_barrier_all()
            hip.synchronize()
            fb = int(ish.get_param("flag_block_bytes"))
            free1 = hip.mem_get_info()[0]
            if fb != fb0:
                fails.append(f"pe{pe} churn: flag footprint {fb} after {iters} split / destroy rounds, base {fb0}")
            # Team blocks are pooled (an exported allocation stays allocated after hipFree, runtime.cpp
            # PoolBlock): the pool holds at most the two blocks a round uses, ~10 MiB each after
            # rounding, per PE on this device; a leak of one block per round would lose iters x 10 MiB.
            blocks = int(ish.get_param("flag_block_pool_bytes")) // 8_651_008
            if blocks > 2:
                fails.append(f"pe{pe} churn: {blocks} pooled team blocks for at most 2 teams at a time")
            # Every PE's pool (<= 2 blocks) and the peers' blocks it maps (a few MiB of mapping each,
            # tools/ipc_leak_probe.py export_import) are one-time costs; the second half of the rounds,
            # with the pools warm, must not lose memory beyond a pool growing by one block.
            allowance = npes * 2 * (10 << 20) + npes * (npes - 1) * 2 * (4 << 20) + (64 << 20)  # every PE's pool <= 2
            if free0 - free1 > allowance:
                fails.append(f"pe{pe} churn: device free memory fell by {(free0 - free1) >> 20} MiB over {iters} "
                             f"rounds (pooled blocks allow {allowance >> 20} MiB)")
            if free_mid is not None and free_mid - free1 > npes * (14 << 20) + (24 << 20):
                fails.append(f"pe{pe} churn: device free memory fell by {(free_mid - free1) >> 20} MiB over the "
                             f"second half of the rounds (warm pools)")
            ish.ishmem_free(d_c)
            ish.ishmem_free(s_c)

        if "inplacegraph" in scenarios:
            # the in-place whole-array fold's path no longer depends on stream
            # capture (its scratch is allocated with the team).  PE 0 captures an in-place f32 sum
            # into a hipGraph once and replays it; the other PEs call it eagerly, for 1 MiB and
            # 512 KiB; every result bit-exact against the oracle, each round well within the timeout.
            gst = hip.stream_create()
            ret = ish.ishmem_malloc(4)
            if int(ish.get_param("fold_limit_bytes")) < (1 << 20):
                fails.append(f"pe{pe} inplacegraph: fold_limit_bytes {ish.get_param('fold_limit_bytes')} < 1 MiB")
            for nbytes in (1 << 20, 512 << 10):
                n = nbytes // 4
                buf = heap(n, DT["float"])
                ish.ishmem_barrier_all()
                g = None
                if pe == 0:
                    g = hip.Graph(gst)
                    with g:
                        if ish.ishmemx_float_sum_reduce_on_stream(buf, buf, n, ret, gst):
                            fails.append(f"pe0 inplacegraph capture {nbytes}: {ish.last_error()}")
                for rep in range(4):
                    vals = [oracle.fill_random(DT["float"], 8800 + 10 * rep + j + n, n) for j in range(npes)]
                    hip.upload(buf, vals[pe])
                    hip.memset(ret, 0xFF, 4)
                    ish.ishmem_barrier_all()
                    t0 = time.monotonic()
                    if pe == 0:
                        g.launch()
                    elif ish.ishmemx_float_sum_reduce_on_stream(buf, buf, n, ret, gst):
                        fails.append(f"pe{pe} inplacegraph eager {nbytes}: {ish.last_error()}")
                    hip.stream_synchronize(gst)
                    if time.monotonic() - t0 > 5.0:
                        fails.append(f"pe{pe} inplacegraph {nbytes} rep {rep}: {time.monotonic() - t0:.1f} s")
                    if int(hip.download(ret, 1, np.int32)[0]) != 0:
                        fails.append(f"pe{pe} inplacegraph {nbytes} rep {rep}: ret != 0")
                    check(f"inplacegraph {nbytes} rep {rep}", OPS["sum"], DT["float"], vals, hip.download(buf, n, np.float32))
                del g
                ish.ishmem_free(buf)
            hip.stream_destroy(gst)
            ish.ishmem_free(ret)

        if "mixeddest" in scenarios:
            # the granule fcollect / broadcast no longer choose their path from
            # this PE's dest kind.  PE 0 passes a pinned-host (blocking) or plain device (on a
            # stream) dest, the others a heap dest; granule and pull sizes; every dest checked.
            m_small, m_big = 1000, 300_000
            src_m = ish.ishmem_malloc(4 * m_big)
            dheap = ish.ishmem_malloc(4 * m_big * npes)
            ddev = hip.malloc(4 * m_big * npes)
            hdst = hip.host_malloc(4 * m_big * npes)
            hv = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_int32 * (m_big * npes)).from_address(hdst))
            mst = hip.stream_create()
            ret = ish.ishmem_malloc(4)
            for m in (m_small, m_big):
                vals = [oracle.fill_random(DT["int32"], 9100 + j + m, m) for j in range(npes)]
                hip.upload(src_m, vals[pe])
                want = np.concatenate(vals)
                ish.ishmem_barrier_all()
                dst = hdst if pe == 0 else dheap
                if ish.ishmem_int32_fcollect(dst, src_m, m):
                    fails.append(f"pe{pe} mixeddest fcollect m={m}: {ish.last_error()}")
                else:
                    got = hv[:m * npes].copy() if pe == 0 else hip.download(dheap, m * npes, np.int32)
                    if not np.array_equal(got, want):
                        fails.append(f"pe{pe} mixeddest fcollect m={m} wrong")
                dst = ddev if pe == 0 else dheap
                hip.memset(ret, 0xFF, 4)
                rc = [ish.fcollect_on_stream(dst, src_m, 4 * m, ret, mst)]
                hip.stream_synchronize(mst)
                got = hip.download(dst, m * npes, np.int32)
                if rc[0] or int(hip.download(ret, 1, np.int32)[0]) != 0 or not np.array_equal(got, want):
                    fails.append(f"pe{pe} mixeddest fcollect_on_stream m={m} rc={rc} {ish.last_error()}")
                root = npes - 1
                hip.memset(ret, 0xFF, 4)
                rc = [ish.broadcast_on_stream(dst, src_m, 4 * m, root, ret, mst)]
                hip.stream_synchronize(mst)
                if rc[0] or int(hip.download(ret, 1, np.int32)[0]) != 0 or \
                        not np.array_equal(hip.download(dst, m, np.int32), vals[root]):
                    fails.append(f"pe{pe} mixeddest broadcast_on_stream m={m} rc={rc} {ish.last_error()}")
                dst = hdst if pe == 0 else dheap
                if ish.ishmem_int32_broadcast(dst, src_m, m, root):
                    fails.append(f"pe{pe} mixeddest broadcast m={m}: {ish.last_error()}")
                else:
                    got = hv[:m].copy() if pe == 0 else hip.download(dheap, m, np.int32)
                    if not np.array_equal(got, vals[root]):
                        fails.append(f"pe{pe} mixeddest broadcast m={m} wrong")
            hip.stream_destroy(mst)
            del hv
            hip.host_free(hdst)
            hip.free(ddev)
            for b_ in (ret, dheap, src_m):
                ish.ishmem_free(b_)

        if "hostread" in scenarios:
            # a blocking call returns on a stream-written host word, without
            # hipStreamSynchronize (host_wait).  A pinned-host dest is read by the host at once, a
            # plain device dest copied out at once on another (non-blocking) stream; reduce (granule,
            # fold / staged sizes) and fcollect, new inputs every round.
            nmax = 300_000
            src_h = ish.ishmem_malloc(4 * nmax)
            ddev = hip.malloc(4 * nmax * npes)
            hdst = hip.host_malloc(4 * nmax * npes)
            hout = hip.host_malloc(4 * nmax * npes)
            hv = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_int32 * (nmax * npes)).from_address(hdst))
            ho = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_int32 * (nmax * npes)).from_address(hout))
            nb_st = hip.stream_create()
            for rnd in range(3):
                for n in (1000, nmax):
                    ins = [oracle.fill_random(DT["int32"], 9300 + 17 * rnd + j + n, n) for j in range(npes)]
                    hip.upload(src_h, ins[pe])
                    red = oracle.reduce_fold(OPS["sum"], DT["int32"], ins, 0)
                    ish.ishmem_barrier_all()
                    hv[:n] = -1
                    if ish.ishmem_int32_sum_reduce(hdst, src_h, n):
                        fails.append(f"pe{pe} hostread reduce pinned n={n}: {ish.last_error()}")
                    elif not np.array_equal(hv[:n], red):
                        fails.append(f"pe{pe} hostread reduce into pinned host n={n} round {rnd}: not final at return")
                    if ish.ishmem_int32_sum_reduce(ddev, src_h, n):
                        fails.append(f"pe{pe} hostread reduce device n={n}: {ish.last_error()}")
                    else:
                        hip.memcpy_async(hout, ddev, 4 * n, nb_st)
                        hip.stream_synchronize(nb_st)
                        if not np.array_equal(ho[:n], red):
                            fails.append(f"pe{pe} hostread reduce into device n={n} round {rnd}: not final at return")
                    hv[:n * npes] = -1
                    if ish.ishmem_int32_fcollect(hdst, src_h, n):
                        fails.append(f"pe{pe} hostread fcollect pinned n={n}: {ish.last_error()}")
                    elif not np.array_equal(hv[:n * npes], np.concatenate(ins)):
                        fails.append(f"pe{pe} hostread fcollect into pinned host n={n} round {rnd}: not final at return")
            hip.stream_destroy(nb_st)
            del hv, ho
            hip.host_free(hout)
            hip.host_free(hdst)
            hip.free(ddev)
            ish.ishmem_free(src_h)

        if "pathparam" in scenarios:
            # TEAM_WORLD's thresholds follow its topology — one PE per (emulated)
            # GPU takes the link-byte model's, co-located PEs round 5's measured ones — and agree
            # with the library's own path_limits for that shape.
            import ctypes
            coloc = int(os.environ.get("COLOCATED_WANT", 1))
            if int(ish.get_param("team_colocated")) != coloc:
                fails.append(f"pe{pe} team_colocated {ish.get_param('team_colocated')} != {coloc}")
            ll, fo = ctypes.c_longlong(), ctypes.c_longlong()
            ish.lib().ishmemi_c_path_limits(npes, coloc, ctypes.byref(ll), ctypes.byref(fo))
            if (int(ish.get_param("ll_limit_bytes")), int(ish.get_param("fold_limit_bytes"))) != (ll.value, fo.value):
                fails.append(f"pe{pe} limits {ish.get_param('ll_limit_bytes')}/{ish.get_param('fold_limit_bytes')} "
                             f"!= path_limits {ll.value}/{fo.value}")
            if "LL_LIMIT_WANT" in os.environ and int(ish.get_param("ll_limit_bytes")) != int(os.environ["LL_LIMIT_WANT"]):
                fails.append(f"pe{pe} ll_limit_bytes {ish.get_param('ll_limit_bytes')} != {os.environ['LL_LIMIT_WANT']}")

        if "phaseevents" in scenarios:
            # The measurement hook: a phased reduce with events between its five launches.
            import ctypes
            n = 1 << 20
            s_, d_ = heap(n, DT["float"]), heap(n, DT["float"])
            hip.upload(s_, np.full(n, pe + 1, np.float32))
            ms = (ctypes.c_float * 5)()
            if ish.lib().ishmemi_c_phase_times(ms) == 0:
                fails.append(f"pe{pe} phase_times succeeded before any phased reduce was recorded")
            ish.set_param("phase_events", 1)
            r = ish.ishmem_float_sum_reduce(d_, s_, n)
            rc = ish.lib().ishmemi_c_phase_times(ms)
            ish.set_param("phase_events", 0)
            want = npes * (npes + 1) / 2
            if r or rc or not all(x > 0 for x in ms) or not np.all(hip.download(d_, n, np.float32) == want):
                fails.append(f"pe{pe} phaseevents: rc={r}/{rc} ms={list(ms)} {ish.last_error()}")
            ish.ishmem_free(d_)
            ish.ishmem_free(s_)

        if "phasedparam" in scenarios:
            # The phased threshold agreed at init: the maximum over the PEs (16 MiB by default,
            # whatever the topology; -1 on any PE turns it off).
            want = int(os.environ["PHASED_WANT"])
            if int(ish.get_param("phased_min_bytes")) != want:
                fails.append(f"pe{pe} phased_min_bytes {ish.get_param('phased_min_bytes')} != agreed {want}")

        if "timeout" in scenarios:
            # Failure detection: PE 0 enters collectives PE 1 never joins.  Every device-side
            # spin is bounded, so the call returns nonzero with a diagnostic instead of hanging
            # (LL granule path and three-barrier path).  The team's epochs now disagree until
            # every PE calls resync (below), after which collectives work again.
            ish.set_param("timeout_ms", 300)
            s_b, d_b = heap(1 << 20, DT["float"]), heap(1 << 20, DT["float"])
            ret = ish.ishmem_malloc(4)
            if pe == 0:
                for n in (100, 1 << 20):
                    r = ish.ishmem_float_sum_reduce(d_b, s_b, n)
                    msg = ish.last_error()
                    if r == 0:
                        fails.append(f"pe0 n={n}: expected a timeout error, got success")
                    elif "timed out" not in msg:
                        fails.append(f"pe0 n={n}: unexpected error text: {msg}")
                if ish.lib().ishmemi_c_error_count() != 2:
                    fails.append(f"pe0 error_count {ish.lib().ishmemi_c_error_count()} != 2")
                # On-stream form with a multi-workgroup grid: *ret must report the failure (every
                # failing workgroup ORs into it), also when the call spans several staged chunks.
                st = hip.stream_create()
                for n, host in ((1 << 20, False), (20_000_000, True)):  # host: two 64 MiB staged chunks
                    hip.memset(ret, 0, 4)
                    if host:
                        hs, hd = np.zeros(n, np.float32), np.zeros(n, np.float32)
                        ish.set_param("timeout_ms", 100)
                        r = ish.ishmemx_float_sum_reduce_on_stream(hd.ctypes.data, hs.ctypes.data, n, ret, st)
                    else:
                        r = ish.ishmemx_float_sum_reduce_on_stream(d_b, s_b, n, ret, st)
                    hip.stream_synchronize(st)
                    if int(hip.download(ret, 1, np.int32)[0]) == 0 and r == 0:
                        fails.append(f"pe0 on_stream n={n} host={host}: *ret is 0 after a timed-out launch")
                hip.stream_destroy(st)
            # Recovery: both PEs resynchronise the team epochs, then collectives work again on
            # the three-phase and the granule paths (and the error words are clear).
            ish.set_param("timeout_ms", 20000)
            if ish.resync() != 0:
                fails.append(f"pe{pe} resync failed: {ish.last_error()}")
            for n in (1 << 20, 100):
                ins = [oracle.fill_random(DT["float"], 0x5E + j, n) for j in range(npes)]
                hip.upload(s_b, ins[pe])
                r = ish.ishmem_float_sum_reduce(d_b, s_b, n)
                if r:
                    fails.append(f"pe{pe} after resync n={n}: rc={r} {ish.last_error()}")
                else:
                    check(f"after resync n={n}", OPS["sum"], DT["float"], ins, hip.download(d_b, n, np.float32))
            ish.ishmem_finalize()
            q.put((pe, fails))
            return

        if "setup" in scenarios:
            # The setup surface of src/ishmem.h:23-26, :44-45, :57-58, :78 (threading, version /
            # name, team configuration).
            if ish.ishmem_query_thread() != ish.ISHMEM_THREAD_MULTIPLE:
                fails.append(f"pe{pe} query_thread {ish.ishmem_query_thread()}")
            if ish.ishmem_info_get_version() != (1, 5) or not ish.ishmem_info_get_name():
                fails.append(f"pe{pe} info_get")
            if ish.ishmem_team_get_config(ish.ISHMEM_TEAM_WORLD) != (0, 0):
                fails.append(f"pe{pe} team_get_config WORLD {ish.ishmem_team_get_config(ish.ISHMEM_TEAM_WORLD)}")
            if ish.lib().ishmemi_c_team_get_config(ish.ISHMEM_TEAM_WORLD, 1, None) == 0:
                fails.append(f"pe{pe} team_get_config accepted a NULL config with a nonzero mask")
            if ish.lib().ishmemi_c_team_get_config(ish.ISHMEM_TEAM_WORLD, 0, None) != 0:
                fails.append(f"pe{pe} team_get_config mask 0")
            r, t = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 0, 1, npes)
            if r or ish.lib().ishmemi_c_team_set_config(t, 1, 7) or ish.ishmem_team_get_config(t) != (0, 7):
                fails.append(f"pe{pe} team config round trip {ish.last_error()}")
            ish.ishmem_team_destroy(t)
            if ish.ishmem_team_get_config(t)[0] == 0:
                fails.append(f"pe{pe} team_get_config of a destroyed team succeeded")

        if "bcast" in scenarios:
            # Host broadcast (ishmem_<TN>_broadcast / broadcastmem, src/ishmem.h:761-813): every
            # root, symmetric / device / pinned-host dest, the root's source in host memory
            # (staged) while the others pass a heap address, odd byte counts, 0 bytes (a team
            # sync), a strided team.  Then the blocking fcollect / scan with members passing
            # different kinds of source (they agree on the staged path first), and a member whose
            # dest is not device-writable: every member fails, none hangs.
            n = 70_001
            src_b, dst_b = ish.ishmem_malloc(4 * n + 64), ish.ishmem_malloc(4 * n + 64)
            ddev = hip.malloc(4 * n)
            hdst = hip.host_malloc(4 * n)
            hview = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_int32 * n).from_address(hdst))
            for root in range(npes):
                vals = [oracle.fill_random(DT["int32"], 0xB0 + j, n) for j in range(npes)]
                hip.upload(src_b, vals[pe])
                for kind, dst in (("heap", dst_b), ("device", ddev), ("pinned", hdst)):
                    hip.memset(dst, 0, 4 * n)
                    if ish.ishmem_int32_broadcast(dst, src_b, n, root):
                        fails.append(f"pe{pe} bcast root {root} {kind}: {ish.last_error()}")
                        continue
                    got = hview.copy() if kind == "pinned" else hip.download(dst, n, np.int32)
                    if not np.array_equal(got, vals[root]):
                        fails.append(f"pe{pe} bcast root {root} into {kind} memory wrong")
                hs = np.ascontiguousarray(vals[pe])
                if ish.ishmem_int32_broadcast(dst_b, hs.ctypes.data if pe == root else src_b, n, root) or \
                        not np.array_equal(hip.download(dst_b, n, np.int32), vals[root]):
                    fails.append(f"pe{pe} bcast root {root} from host memory wrong {ish.last_error()}")
            for nb in (1, 7, 1001):
                hip.upload(src_b + 3, np.arange(nb, dtype=np.uint8) + np.uint8(pe))
                if ish.ishmem_broadcastmem(dst_b + 1, src_b + 3, nb, npes - 1) or not np.array_equal(
                        hip.download(dst_b + 1, nb, np.uint8), np.arange(nb, dtype=np.uint8) + np.uint8(npes - 1)):
                    fails.append(f"pe{pe} broadcastmem {nb} B wrong {ish.last_error()}")
            if ish.ishmem_broadcastmem(dst_b, src_b, 0, 0):
                fails.append(f"pe{pe} broadcastmem 0 B {ish.last_error()}")
            r, team = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 0, 2, (npes + 1) // 2)
            if team != ish.ISHMEM_TEAM_INVALID:
                members = list(range(0, npes, 2))
                root = len(members) - 1
                hip.upload(src_b, np.full(100, 1000 + pe, np.int64))
                if ish.ishmem_long_broadcast(team, dst_b, src_b, 100, root) or not np.all(
                        hip.download(dst_b, 100, np.int64) == 1000 + members[root]):
                    fails.append(f"pe{pe} team broadcast wrong {ish.last_error()}")
                ish.ishmem_team_destroy(team)
            # fcollect / scan with mixed source kinds (PE 0's source in host memory).
            m = 50_000
            vals = [oracle.fill_random(DT["int32"], 0xC0 + j, m) for j in range(npes)]
            hip.upload(src_b, vals[pe])
            hsrc = np.ascontiguousarray(vals[pe])
            fdst = ish.ishmem_malloc(4 * m * npes)
            if ish.ishmem_int32_fcollect(fdst, hsrc.ctypes.data if pe == 0 else src_b, m) or not np.array_equal(
                    hip.download(fdst, m * npes, np.int32), np.concatenate(vals)):
                fails.append(f"pe{pe} fcollect with mixed source kinds wrong {ish.last_error()}")
            for inc in (True, False):
                hip.memset(dst_b, 0, 4 * m)
                if ish.scan("int32", inc, dst_b, hsrc.ctypes.data if pe == 0 else src_b, m) or not _bits_equal(
                        hip.download(dst_b, m, np.int32), oracle.scan_fold(DT["int32"], vals, pe, inc)):
                    fails.append(f"pe{pe} scan inc={inc} with mixed source kinds wrong {ish.last_error()}")
            pageable = np.zeros(m * npes, np.int32)
            bad_dst = pageable.ctypes.data if pe == npes - 1 else fdst
            t0 = time.perf_counter()
            if ish.ishmem_int32_fcollect(bad_dst, src_b, m) == 0:
                fails.append(f"pe{pe} fcollect with a member's pageable dest succeeded")
            if ish.ishmem_int32_collect(bad_dst, src_b, m) == 0:
                fails.append(f"pe{pe} collect with a member's pageable dest succeeded")
            if time.perf_counter() - t0 > 5.0:
                fails.append(f"pe{pe} argument failure took {time.perf_counter() - t0:.1f} s (a member waited)")
            # the team still works afterwards (nothing was launched by the failed calls)
            if ish.ishmem_int32_fcollect(fdst, src_b, m) or not np.array_equal(
                    hip.download(fdst, m * npes, np.int32), np.concatenate(vals)):
                fails.append(f"pe{pe} fcollect after the refused call wrong {ish.last_error()}")
            # On a stream (ishmemx_*_broadcast_on_queue / team_sync_on_queue): a reduce, then a
            # broadcast of one member's result block, then a team barrier, chained with no host
            # synchronisation; *ret stays 0.
            st_b = hip.stream_create()
            ret_b = ish.ishmem_malloc(4)
            hip.memset(ret_b, 0x7F, 4)
            vals = [oracle.fill_random(DT["int32"], 0xD0 + j, m) for j in range(npes)]
            hip.upload(src_b, vals[pe])
            ish.ishmem_barrier_all()
            root = npes // 2
            rc = [ish.reduce_on_stream("max", "int32", fdst, src_b, m, ret_b, st_b),
                  ish.broadcast_on_stream(dst_b, src_b, 4 * 1000, root, ret_b, st_b),
                  ish.team_sync_on_stream(ish.ISHMEM_TEAM_WORLD, ret_b, st_b)]
            hip.stream_synchronize(st_b)
            if any(rc) or int(hip.download(ret_b, 1, np.int32)[0]) != 0:
                fails.append(f"pe{pe} on-stream broadcast chain rc={rc} {ish.last_error()}")
            else:
                check("on-stream max before broadcast", OPS["max"], DT["int32"], vals, hip.download(fdst, m, np.int32))
                if not np.array_equal(hip.download(dst_b, 1000, np.int32), vals[root][:1000]):
                    fails.append(f"pe{pe} on-stream broadcast wrong")
            hip.stream_destroy(st_b)
            ish.ishmem_free(ret_b)
            del hview
            hip.host_free(hdst)
            hip.free(ddev)
            for b_ in (fdst, dst_b, src_b):
                ish.ishmem_free(b_)

        if "golden" in scenarios:
            z = np.load(GOLDEN / f"golden_np{npes}.npz") if (GOLDEN / f"golden_np{npes}.npz").exists() else None
            for op in range(7):
                for dt in range(10):
                    if not oracle.valid(op, dt):
                        continue
                    cases = []
                    if z is not None:
                        for nm in (f"rnd_{ONAMES[op]}_{NAMES[dt]}_1001", f"pat_{ONAMES[op]}_{NAMES[dt]}_129",
                                   f"pat_{ONAMES[op]}_{NAMES[dt]}_3"):
                            ins = list(z[nm + "__in"])
                            outs = z[nm + "__out"]
                            cases.append((nm, ins, outs[pe] if len(outs) > 1 else outs[0]))
                    else:
                        lo, hi = (0.5, 2.0) if op == OPS["prod"] else (-1.0, 1.0)
                        ins = [oracle.fill_random(dt, 0x15AE0001 + j, 1001, lo, hi) for j in range(npes)]
                        cases.append((f"rnd_{op}_{dt}", ins, None))
                    for nm, ins, gold in cases:
                        n = len(ins[0])
                        s, d = heap(n, dt), heap(n, dt)
                        hip.upload(s, ins[pe])
                        r = ish.reduce(ONAMES[op], NAMES[dt], d, s, n)
                        if r != 0:
                            fails.append(f"pe{pe} {nm}: rc={r} {ish.last_error()}")
                        else:
                            check(nm, op, dt, ins, hip.download(d, n, oracle.NP[dt]), gold)
                        ish.ishmem_free(d)
                        ish.ishmem_free(s)

        if "inplace" in scenarios:
            for op, dt, n in [(OPS["sum"], DT["float"], 5000), (OPS["max"], DT["int64"], 777),
                              (OPS["xor"], DT["uint8"], 100003), (OPS["prod"], DT["double"], 31)]:
                lo, hi = (0.5, 2.0) if op == OPS["prod"] else (-1.0, 1.0)
                ins = [oracle.fill_random(dt, 77 + j, n, lo, hi) for j in range(npes)]
                b = heap(n, dt)
                hip.upload(b, ins[pe])
                r = ish.reduce(ONAMES[op], NAMES[dt], b, b, n)
                if r:
                    fails.append(f"pe{pe} inplace rc={r} {ish.last_error()}")
                else:
                    check(f"inplace {op} {dt} {n}", op, dt, ins, hip.download(b, n, oracle.NP[dt]))
                ish.ishmem_free(b)
            # Larger in place, dest 4 B off the 16-B grid (head / tail elements): the whole-array
            # fold through the staging region at 2-4 PEs (round 5), the phased path above it.
            for n in (786_435, 3_000_001):
                ins = [oracle.fill_random(DT["float"], 91 + j, n) for j in range(npes)]
                b = heap(n + 8, DT["float"])
                hip.upload(b + 4, ins[pe])
                r = ish.reduce("sum", "float", b + 4, b + 4, n)
                if r:
                    fails.append(f"pe{pe} inplace offset n={n} rc={r} {ish.last_error()}")
                else:
                    check(f"inplace offset sum float {n}", OPS["sum"], DT["float"], ins, hip.download(b + 4, n, np.float32))
                ish.ishmem_free(b)

        if "offsets" in scenarios:
            # The reference tester's offset sweep (ishmem_tester.h:1407-1436): nelems 1..16 x
            # src/dst byte offsets 0..14 step sizeof(T): exercises head/tail and scalar paths.
            for dt in (DT["int8"], DT["int16"], DT["float"], DT["double"]):
                es = np.dtype(oracle.NP[dt]).itemsize
                base_s, base_d = heap(64, dt), heap(64, dt)
                for nelems in (1, 2, 5, 16, 17, 40):
                    for so in range(0, 15, es * 3):
                        for do in range(0, 15, es * 5):
                            op = OPS["sum"] if dt >= 8 else OPS["min"]
                            ins = [oracle.fill_random(dt, 1000 + 7 * j + nelems, nelems) for j in range(npes)]
                            hip.upload(base_s + so, ins[pe])
                            r = ish.reduce(ONAMES[op], NAMES[dt], base_d + do, base_s + so, nelems)
                            if r:
                                fails.append(f"pe{pe} offsets rc={r} {ish.last_error()}")
                                continue
                            check(f"offsets dt{dt} n{nelems} so{so} do{do}", op, dt, ins,
                                  hip.download(base_d + do, nelems, oracle.NP[dt]))
                ish.ishmem_free(base_d)
                ish.ishmem_free(base_s)

        if "offsets_large" in scenarios:
            # Source and dest on different 16-B phases at sizes past the vector threshold: the
            # phased reduce-scatter realigns the sources (rs_phase_kernel, PhaseArgs::shift), the
            # persistent kernel runs element-granular; both against the oracle, the guard bytes
            # around dest untouched.
            for dt in (DT["int8"], DT["float"], DT["double"]):
                es = np.dtype(oracle.NP[dt]).itemsize
                nmax = 262_147
                base_s, base_d = heap(nmax + 64, dt), heap(nmax + 64, dt)
                for nelems in (1027, 70_001, nmax):
                    for so, do in ((es, 0), (0, 3 * es % 16), (8 % 16, 12 % 16), (15 - 15 % es, es)):
                        so, do = so - so % es, do - do % es
                        if (so - do) % 16 == 0:
                            continue
                        op = OPS["sum"] if dt >= 8 else OPS["max"]
                        ins = [oracle.fill_random(dt, 2000 + 11 * j + nelems + so, nelems) for j in range(npes)]
                        hip.upload(base_s + 16 + so, ins[pe])
                        hip.memset(base_d, 0x3C, (nmax + 64) * es)
                        ish.ishmem_barrier_all()
                        r = ish.reduce(ONAMES[op], NAMES[dt], base_d + 16 + do, base_s + 16 + so, nelems)
                        if r:
                            fails.append(f"pe{pe} offsets_large rc={r} {ish.last_error()}")
                            continue
                        check(f"offsets_large dt{dt} n{nelems} so{so} do{do}", op, dt, ins,
                              hip.download(base_d + 16 + do, nelems, oracle.NP[dt]))
                        raw = hip.download(base_d, (nmax + 64) * es, np.uint8)
                        lo, hi = 16 + do, 16 + do + nelems * es
                        if not ((raw[:lo] == 0x3C).all() and (raw[hi:] == 0x3C).all()):
                            fails.append(f"pe{pe} offsets_large dt{dt} n{nelems} so{so} do{do}: guard bytes written")
                ish.ishmem_free(base_d)
                ish.ishmem_free(base_s)

        if "edge" in scenarios:
            s, d = heap(16, DT["float"]), heap(16, DT["float"])
            if ish.ishmem_float_sum_reduce(d, s, 0) != 0:  # nreduce == 0 still synchronises
                fails.append(f"pe{pe} n=0 failed: {ish.last_error()}")
            ins = [np.array([float(j + 1)], np.float32) for j in range(npes)]
            hip.upload(s, ins[pe])
            if ish.ishmem_float_sum_reduce(ish.ISHMEM_TEAM_WORLD, d, s, 1) != 0:
                fails.append(f"pe{pe} n=1 failed")
            else:
                check("n=1", OPS["sum"], DT["float"], ins, hip.download(d, 1, np.float32))
            # examples/5_pi_reduce.cpp shape: in-place size_sum_reduce of one element
            cnt = np.array([1000 + pe], np.uint64)
            hip.upload(s, cnt)
            if ish.ishmem_size_sum_reduce(s, s, 1) != 0:
                fails.append(f"pe{pe} pi-shape failed")
            elif int(hip.download(s, 1, np.uint64)[0]) != sum(1000 + j for j in range(npes)):
                fails.append(f"pe{pe} pi-shape wrong value")
            ish.ishmem_free(d)
            ish.ishmem_free(s)

        if "stream" in scenarios:
            n = 12345
            ins = [oracle.fill_random(DT["int32"], 5 + j, n) for j in range(npes)]
            s, d = heap(n, DT["int32"]), heap(n, DT["int32"])
            ret = ish.ishmem_malloc(4)
            hip.memset(ret, 0xFF, 4)
            hip.upload(s, ins[pe])
            st = hip.stream_create()
            r = ish.ishmemx_int32_sum_reduce_on_stream(d, s, n, ret, st)
            hip.stream_synchronize(st)
            rv = int(hip.download(ret, 1, np.int32)[0])
            if r != 0 or rv != 0:
                fails.append(f"pe{pe} on_stream rc={r} ret={rv} {ish.last_error()}")
            else:
                check("on_stream", OPS["sum"], DT["int32"], ins, hip.download(d, n, np.int32))
            # deps / done (reduce_impl.h:445-472): each PE's source is produced by a copy on
            # another stream, queued behind a kernel of a PE-dependent length; the reduce waits
            # for it through `deps` (a missed dependency would fold the zeroed source).
            ins2 = [oracle.fill_random(DT["int32"], 55 + j, n) for j in range(npes)]
            hx = hip.host_malloc(n * 4)
            np.ctypeslib.as_array((np.ctypeslib.ctypes.c_int32 * n).from_address(hx))[:] = ins2[pe]
            hip.memset(s, 0, n * 4)
            sa, produced, done = hip.stream_create(), hip.Event(), hip.Event()
            ish.ishmem_barrier_all()
            ish.occupy(2, 20_000 * (1 + pe), sa)
            hip.memcpy_async(s, hx, n * 4, sa)
            produced.record(sa)
            r = ish.reduce_on_stream("sum", "int32", d, s, n, ret, st, deps=[produced], done=done)
            done.synchronize()
            if r:
                fails.append(f"pe{pe} on_stream deps rc={r} {ish.last_error()}")
            else:
                check("on_stream deps", OPS["sum"], DT["int32"], ins2, hip.download(d, n, np.int32))
            hip.stream_synchronize(sa)
            hip.stream_destroy(sa)
            hip.host_free(hx)
            hip.stream_destroy(st)
            for p in (ret, d, s):
                ish.ishmem_free(p)

        if "streams" in scenarios:
            # Back-to-back collectives on different streams with no host synchronisation between
            # them (each must follow the previous one: same epochs / flag rows / staging on every
            # PE), the last stream destroyed before a blocking call.  ISHMEM_STREAM_ORDER on.
            ish.set_param("stream_order", 1)
            n = 70_000
            ins = [[oracle.fill_random(DT["int32"], 300 + 10 * r + j, n) for j in range(npes)] for r in range(4)]
            s_b = [heap(n, DT["int32"]) for _ in range(4)]
            d_b = [heap(n, DT["int32"]) for _ in range(4)]
            for r in range(4):
                hip.upload(s_b[r], ins[r][pe])
            sts = [hip.stream_create() for _ in range(3)]
            host_out = np.zeros(n, np.int32)
            host_in = np.ascontiguousarray(ins[3][pe])
            calls = [ish.ishmemx_int32_sum_reduce_on_stream(d_b[0], s_b[0], n, 0, sts[0]),
                     ish.ishmemx_int32_max_reduce_on_stream(d_b[1], s_b[1], n, 0, sts[1]),
                     ish.ishmemx_int32_sum_reduce_on_stream(d_b[2], s_b[2], 1000, 0, sts[2]),  # LL
                     ish.ishmemx_int32_xor_reduce_on_stream(host_out.ctypes.data, host_in.ctypes.data, n, 0, sts[0])]
            hip.stream_destroy(sts[2])
            if any(calls) or ish.ishmem_int32_min_reduce(d_b[3], s_b[3], n):
                fails.append(f"pe{pe} streams rc={calls} {ish.last_error()}")
            hip.synchronize()
            check("streams sum", OPS["sum"], DT["int32"], ins[0], hip.download(d_b[0], n, np.int32))
            check("streams max", OPS["max"], DT["int32"], ins[1], hip.download(d_b[1], n, np.int32))
            check("streams ll", OPS["sum"], DT["int32"], [x[:1000] for x in ins[2]], hip.download(d_b[2], 1000, np.int32))
            check("streams host", OPS["xor"], DT["int32"], ins[3], host_out)
            check("streams min", OPS["min"], DT["int32"], ins[3], hip.download(d_b[3], n, np.int32))
            for st_ in sts[:2]:
                hip.stream_destroy(st_)
            for b in s_b + d_b:
                ish.ishmem_free(b)
            ish.set_param("stream_order", 0)

        if "graph" in scenarios:
            # A captured hipGraph of on_stream collectives (LL path, RS + AG path, fcollect,
            # inscan) replayed several times: kernel epochs come from the device-side counter,
            # so every replay synchronises afresh.  Inputs change between replays.
            st_ = hip.stream_create()
            n_small, n_big = 600, 300_000
            s1, d1 = heap(n_small, DT["double"]), heap(n_small, DT["double"])
            s2, d2 = heap(n_big, DT["float"]), heap(n_big, DT["float"])
            fc = ish.ishmem_malloc(4096 * npes)
            sc = heap(n_big, DT["int32"])
            ret = ish.ishmem_malloc(4)
            ish.ishmem_barrier_all()
            with hip.Graph(st_) as g:
                ish.ishmemx_double_max_reduce_on_stream(d1, s1, n_small, ret, st_)
                ish.ishmemx_float_sum_reduce_on_stream(d2, s2, n_big, ret, st_)
                ish.fcollect_on_stream(fc, s1, 4096, ret, st_)
                ish.lib().ishmemi_c_scan_on_stream(0, DT["int32"], 1, sc, s2, n_big, ret, st_)
            for rep in range(4):
                a = [oracle.fill_random(DT["double"], 900 + 10 * rep + j, n_small) for j in range(npes)]
                b = [oracle.fill_random(DT["float"], 950 + 10 * rep + j, n_big) for j in range(npes)]
                hip.upload(s1, a[pe])
                hip.upload(s2, b[pe])
                hip.memset(ret, 0xFF, 4)
                ish.ishmem_barrier_all()  # everyone's inputs are in place
                g.launch()
                hip.stream_synchronize(st_)
                if int(hip.download(ret, 1, np.int32)[0]) != 0:
                    fails.append(f"pe{pe} graph replay {rep}: ret != 0")
                check(f"graph max {rep}", OPS["max"], DT["double"], a, hip.download(d1, n_small, np.float64))
                check(f"graph sum {rep}", OPS["sum"], DT["float"], b, hip.download(d2, n_big, np.float32))
                want = np.concatenate([x.view(np.uint8)[:4096] for x in a])
                if not _bits_equal(hip.download(fc, 4096 * npes, np.uint8), want):
                    fails.append(f"pe{pe} graph fcollect {rep} wrong")
                ref = oracle.scan_fold(DT["int32"], [x.view(np.int32) for x in b], pe, True)
                if not _bits_equal(hip.download(sc, n_big, np.int32), ref):
                    fails.append(f"pe{pe} graph inscan {rep} wrong")
            del g
            # Pageable host buffers (malloc'd numpy, 2 MiB: above the 1 MiB page-locking threshold)
            # in a captured on-stream reduce: the library must not page-lock them for
            # the call under capture — its synchronize would invalidate the capture and the pages
            # would be unlocked before any replay.  The captured staged copies replay correctly.
            n_h = (2 << 20) // 4
            hsrc, hdst = np.zeros(n_h, np.float32), np.zeros(n_h, np.float32)
            ish.ishmem_barrier_all()
            with hip.Graph(st_) as g2:
                rc_cap = ish.ishmemx_float_sum_reduce_on_stream(hdst.ctypes.data, hsrc.ctypes.data, n_h, ret, st_)
            if rc_cap:
                fails.append(f"pe{pe} graph pageable: captured call failed: {ish.last_error()}")
            else:
                for rep in range(3):
                    vals = [oracle.fill_random(DT["float"], 990 + 10 * rep + j, n_h) for j in range(npes)]
                    hsrc[:] = vals[pe]
                    hdst[:] = 0
                    hip.memset(ret, 0xFF, 4)
                    ish.ishmem_barrier_all()
                    g2.launch()
                    hip.stream_synchronize(st_)
                    if int(hip.download(ret, 1, np.int32)[0]) != 0:
                        fails.append(f"pe{pe} graph pageable replay {rep}: ret != 0")
                    check(f"graph pageable {rep}", OPS["sum"], DT["float"], vals, hdst.copy())
            del g2
            hip.stream_destroy(st_)
            for b_ in (s1, d1, s2, d2, fc, sc, ret):
                ish.ishmem_free(b_)

        if "staged" in scenarios:
            # Host memory and device memory outside the heap go through the staging region.
            n = 300_000
            ins = [oracle.fill_random(DT["double"], 9 + j, n) for j in range(npes)]
            src = np.ascontiguousarray(ins[pe])
            out = np.zeros(n, np.float64)
            r = ish.ishmem_double_max_reduce(out.ctypes.data, src.ctypes.data, n)
            if r:
                fails.append(f"pe{pe} host-staged rc={r} {ish.last_error()}")
            else:
                check("host-staged", OPS["max"], DT["double"], ins, out)
            ds, dd = hip.malloc(n * 8), hip.malloc(n * 8)
            hip.upload(ds, src)
            r = ish.ishmem_double_sum_reduce(dd, ds, n)
            if r:
                fails.append(f"pe{pe} device-staged rc={r} {ish.last_error()}")
            else:
                check("device-staged", OPS["sum"], DT["double"], ins, hip.download(dd, n, np.float64))
            hip.free(ds)
            hip.free(dd)

        if "team" in scenarios and npes >= 2:
            # Strided team of the even PEs (examples/6_team_split_strided.cpp shape).
            size = (npes + 1) // 2
            r, team = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 0, 2, size)
            if r:
                fails.append(f"pe{pe} split rc={r} {ish.last_error()}")
            n = 4099
            members = list(range(0, npes, 2))
            ins = {j: oracle.fill_random(DT["int64"], 40 + j, n) for j in members}
            s, d = heap(n, DT["int64"]), heap(n, DT["int64"])
            if team != ish.ISHMEM_TEAM_INVALID:
                if ish.ishmem_team_my_pe(team) != members.index(pe):
                    fails.append(f"pe{pe} team_my_pe wrong")
                hip.upload(s, ins[pe])
                r = ish.ishmem_int64_sum_reduce(team, d, s, n)
                if r:
                    fails.append(f"pe{pe} team reduce rc={r} {ish.last_error()}")
                else:
                    check("team", OPS["sum"], DT["int64"], [ins[j] for j in members], hip.download(d, n, np.int64))
            elif pe % 2 == 0:
                fails.append(f"pe{pe} should be in the even team")
            # Nested split of the even team (members 0, 2, ...): its second member alone.  All
            # PEs must still agree on team slots afterwards (free-mask AND-reduction).
            if team != ish.ISHMEM_TEAM_INVALID and size >= 2:
                r, solo = ish.ishmem_team_split_strided(team, 1, 1, 1)
                if r or (solo != ish.ISHMEM_TEAM_INVALID) != (pe == 2):
                    fails.append(f"pe{pe} nested split rc={r} team={solo}")
                if solo != ish.ISHMEM_TEAM_INVALID:
                    ish.ishmem_team_destroy(solo)
            if team != ish.ISHMEM_TEAM_INVALID:
                ish.ishmem_team_destroy(team)
            # 2-D split of WORLD (src/teams.cpp:453-518), xrange 2: x-teams {0,1},{2,3},...;
            # y-teams {0,2,..},{1,3,..}; reduce over both axes.
            r, xt, yt = ish.ishmem_team_split_2d(ish.ISHMEM_TEAM_WORLD, 2)
            if r or xt == ish.ISHMEM_TEAM_INVALID or yt == ish.ISHMEM_TEAM_INVALID:
                fails.append(f"pe{pe} split_2d rc={r} x={xt} y={yt} {ish.last_error()}")
            else:
                xm = [j for j in range(npes) if j // 2 == pe // 2]
                ym = [j for j in range(npes) if j % 2 == pe % 2]
                if ish.ishmem_team_n_pes(xt) != len(xm) or ish.ishmem_team_n_pes(yt) != len(ym):
                    fails.append(f"pe{pe} split_2d sizes")
                if ish.ishmem_team_translate_pe(xt, 0, ish.ISHMEM_TEAM_WORLD) != xm[0]:
                    fails.append(f"pe{pe} translate_pe")
                for tm, members in ((xt, xm), (yt, ym)):
                    allin = {j: oracle.fill_random(DT["int64"], 90 + j, n) for j in range(npes)}
                    hip.upload(s, allin[pe])
                    if ish.ishmem_int64_sum_reduce(tm, d, s, n):
                        fails.append(f"pe{pe} 2d reduce failed {ish.last_error()}")
                    else:
                        check("2d", OPS["sum"], DT["int64"], [allin[j] for j in members],
                              hip.download(d, n, np.int64))
                ish.ishmem_team_destroy(xt)
                ish.ishmem_team_destroy(yt)
            ish.ishmem_free(d)
            ish.ishmem_free(s)

        if "teams2" in scenarios and npes >= 2:
            # The reference's team tests, restated.
            W, INV = ish.ISHMEM_TEAM_WORLD, ish.ISHMEM_TEAM_INVALID

            def pat(idx_team, m):  # ((i % (t + 2)) << 16) + i  (team_translate.cpp / team_shared.cpp)
                i = np.arange(m, dtype=np.int64)
                return (((i % (idx_team + 2)) << 16) + i).astype(np.int32)

            m = 1 << 10
            src_b, dst_b = ish.ishmem_malloc(4 * m), ish.ishmem_malloc(4 * m)
            # (1) test/unit/team_negative_stride.cpp: start npes-1, stride -1, size npes; team
            # index of world PE k is npes-1-k; fcollect of each PE's id lands reversed.
            r, rev = ish.ishmem_team_split_strided(W, npes - 1, -1, npes)
            if r or rev == INV:
                fails.append(f"pe{pe} split stride -1 rc={r} team={rev} {ish.last_error()}")
            else:
                if ish.ishmem_team_translate_pe(W, pe, rev) != npes - 1 - pe:
                    fails.append(f"pe{pe} stride -1: translate_pe {ish.ishmem_team_translate_pe(W, pe, rev)}")
                if ish.ishmem_team_my_pe(rev) != npes - 1 - pe or ish.ishmem_team_n_pes(rev) != npes:
                    fails.append(f"pe{pe} stride -1: team_my_pe / n_pes")
                hip.upload(src_b, np.array([pe], np.int32))
                hip.memset(dst_b, 0xFF, 4 * npes)
                if ish.ishmem_int_fcollect(rev, dst_b, src_b, 1):
                    fails.append(f"pe{pe} stride -1 fcollect rc {ish.last_error()}")
                elif not np.array_equal(hip.download(dst_b, npes, np.int32), np.arange(npes - 1, -1, -1)):
                    fails.append(f"pe{pe} stride -1 fcollect: {hip.download(dst_b, npes, np.int32)}")
                # FP fold order on the reversed team is ITS team order: world PE npes-1 first.
                for op, dt, n in ((OPS["sum"], DT["float"], 3001), (OPS["prod"], DT["double"], 777),
                                  (OPS["max"], DT["int64"], 5000)):
                    lo, hi = (0.5, 2.0) if op == OPS["prod"] else (-1.0, 1.0)
                    ins_w = [oracle.fill_random(dt, 0x7E0 + 13 * op + j, n, lo, hi) for j in range(npes)]
                    s, d = heap(n, dt), heap(n, dt)
                    hip.upload(s, ins_w[pe])
                    if ish.reduce(ONAMES[op], NAMES[dt], d, s, n, rev):
                        fails.append(f"pe{pe} stride -1 reduce rc {ish.last_error()}")
                    else:
                        check(f"stride -1 {ONAMES[op]} {NAMES[dt]}", op, dt, ins_w[::-1],
                              hip.download(d, n, oracle.NP[dt]), me=npes - 1 - pe)
                    ish.ishmem_free(d)
                    ish.ishmem_free(s)
                ish.ishmem_team_destroy(rev)
            # (2) test/unit/team_translate.cpp: teams of every 2nd and every 3rd PE; my_pe and
            # translate_pe are -1 exactly off the team; int sum of the per-team-index pattern.
            r2, t2 = ish.ishmem_team_split_strided(W, 0, 2, (npes - 1) // 2 + 1)
            r3, t3 = ish.ishmem_team_split_strided(W, 0, 3, (npes - 1) // 3 + 1)
            if r2 or r3:
                fails.append(f"pe{pe} translate splits rc={r2},{r3} {ish.last_error()}")
            p2 = ish.ishmem_team_my_pe(t2) if t2 != INV else -1
            p3 = ish.ishmem_team_my_pe(t3) if t3 != INV else -1
            x32 = ish.ishmem_team_translate_pe(t3, p3, t2) if t3 != INV else -1
            x23 = ish.ishmem_team_translate_pe(t2, p2, t3) if t2 != INV else -1
            in2, in3 = pe % 2 == 0, pe % 3 == 0
            want = (p2 != -1, p3 != -1, x23 != -1, x32 != -1)
            if want != (in2, in3, in2 and in3, in2 and in3):
                fails.append(f"pe{pe} team_translate: p2={p2} p3={p3} 2->3={x23} 3->2={x32}")
            if in2 and (p2 != pe // 2 or ish.ishmem_team_translate_pe(W, pe, t2) != p2):
                fails.append(f"pe{pe} team_translate: world -> team_2s")
            for tm, tp in ((t2, p2), (t3, p3)):
                if tm == INV:
                    continue
                hip.upload(src_b, pat(tp, m))
                hip.memset(dst_b, 0, 4 * m)
                if ish.ishmem_int_sum_reduce(tm, dst_b, src_b, m):
                    fails.append(f"pe{pe} team_translate reduce rc {ish.last_error()}")
                    continue
                ref = sum(pat(j, m).astype(np.int64) for j in range(ish.ishmem_team_n_pes(tm))).astype(np.int32)
                if not np.array_equal(hip.download(dst_b, m, np.int32), ref):
                    fails.append(f"pe{pe} team_translate: team reduce wrong")
            for tm in (t2, t3):
                if tm != INV:
                    ish.ishmem_team_destroy(tm)
            # (3) test/unit/team_shared.cpp: every PE of the node is in ISHMEM_TEAM_SHARED; int sum
            # over it of the per-world-PE pattern, in-place min of the PE id (the leader, 0), team
            # size fcollect, then the leader team (stride npes / one member) re-reduces in place.
            ns = ish.ishmem_team_n_pes(ish.ISHMEM_TEAM_SHARED)
            if ns != npes or ish.ishmem_team_translate_pe(ish.ISHMEM_TEAM_SHARED, pe, W) != pe:
                fails.append(f"pe{pe} team_shared: n_pes {ns}")
            hip.upload(src_b, pat(pe, m))
            total = sum(pat(j, m).astype(np.int64) for j in range(npes)).astype(np.int32)
            if ish.ishmem_int_sum_reduce(ish.ISHMEM_TEAM_SHARED, dst_b, src_b, m) or not np.array_equal(
                    hip.download(dst_b, m, np.int32), total):
                fails.append(f"pe{pe} team_shared: sum reduce wrong {ish.last_error()}")
            lead = ish.ishmem_malloc(4)
            hip.upload(lead, np.array([pe], np.int32))
            if ish.ishmem_team_sync(ish.ISHMEM_TEAM_SHARED) or ish.ishmem_int_min_reduce(
                    ish.ISHMEM_TEAM_SHARED, lead, lead, 1) or int(hip.download(lead, 1, np.int32)[0]) != 0:
                fails.append(f"pe{pe} team_shared: leader min-reduce {ish.last_error()}")
            hip.upload(src_b + 4 * m - 4, np.array([ns], np.int32))
            sizes = ish.ishmem_malloc(4 * npes)
            if ish.ishmem_int_fcollect(sizes, src_b + 4 * m - 4, 1) or not np.all(
                    hip.download(sizes, npes, np.int32) == ns):
                fails.append(f"pe{pe} team_shared: size fcollect")
            r, leaders = ish.ishmem_team_split_strided(W, 0, npes, npes // ns)
            if r:
                fails.append(f"pe{pe} team_shared: leader split {ish.last_error()}")
            elif leaders != INV:
                if ish.ishmem_int_sum_reduce(leaders, dst_b, dst_b, m) or not np.array_equal(
                        hip.download(dst_b, m, np.int32), total):
                    fails.append(f"pe{pe} team_shared: leader reduce wrong")
                ish.ishmem_team_destroy(leaders)
            elif pe == 0:
                fails.append("pe0 team_shared: PE 0 must lead")
            for b_ in (sizes, lead, dst_b, src_b):
                ish.ishmem_free(b_)

        if "large" in scenarios:
            # f32 sum over 64 Mi elements per PE (256 MiB; 16 Mi beyond 4 PEs, where every
            # process holds all p inputs): full-array comparison.
            n = (64 << 20) if npes <= 4 else (16 << 20)
            s, d = heap(n, DT["float"]), heap(n, DT["float"])
            ins = [oracle.fill_random(DT["float"], 0xABC + j, n) for j in range(npes)]
            hip.upload(s, ins[pe])
            r = ish.ishmem_float_sum_reduce(d, s, n)
            if r:
                fails.append(f"pe{pe} large rc={r} {ish.last_error()}")
            else:
                got = hip.download(d, n, np.float32)
                ref = ins[0].copy()
                for j in range(1, npes):
                    ref += ins[j]  # canonical left-to-right fold, exactly the kernel's order
                if not _bits_equal(got, ref):
                    fails.append(f"pe{pe} large: {int(np.sum(got != ref))} elements differ")
            ish.ishmem_free(d)
            ish.ishmem_free(s)

        if "huge" in scenarios:
            # > 2 GiB per PE with a misaligned start and an odd length: the head, the tail and the
            # 2 GiB descriptor-range boundary are all exercised.  Rotating-winner pattern
            # (selfcheck.pattern: non-periodic, every PE distinct), every word compared.
            from ishmem_amd import selfcheck as sc
            n = (1 << 29) + (1 << 27) + 5  # 2.5 GiB + 20 B of float32
            s_base = ish.ishmem_malloc(n * 4 + 64)
            d_base = ish.ishmem_malloc(n * 4 + 64)
            s, d = s_base + 4, d_base + 4
            sc.upload_pattern(hip, s, np.float32, pe, npes, n)
            r = ish.ishmem_float_sum_reduce(d, s, n)
            if r:
                fails.append(f"pe{pe} huge rc={r} {ish.last_error()}")
            else:
                bad = sc.count_wrong(hip, d, "sum", np.float32, npes, 0, n)
                if bad:
                    fails.append(f"pe{pe} huge: {bad} of {4 * n} bytes wrong")
            ish.ishmem_free(d_base)
            ish.ishmem_free(s_base)

        if "opposite" in scenarios:
            # two teams with the same members (two clones of WORLD), one
            # collective each on its own stream, issued in OPPOSITE orders on the two halves of the
            # PEs with a 20 ms pause between the two issues, so the first-issued kernels already wait
            # for their peers when the second ones are enqueued.  Run with every PE on its own
            # (emulated) device: round 3 sized each persistent / LL grid for the whole device, so the
            # first-issued launches held every CU while waiting for kernels that then could not
            # become resident (device timeouts).  The waiting footprint (kernels.h) keeps each such
            # launch to 1 / wait_slots of the device.  LL (64 KiB), persistent (1, 4 MiB), phased
            # (32 MiB); results checked, and no call may take seconds.
            r1, ta = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 0, 1, npes)
            r2, tb = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 0, 1, npes)
            if r1 or r2:
                fails.append(f"pe{pe} opposite split: {ish.last_error()}")
            else:
                first = pe < max(1, npes // 2)
                nmax = 8 << 20
                sa, da, sb, db = (heap(nmax, DT["float"]) for _ in range(4))
                ret = ish.ishmem_malloc(8)
                sts = [hip.stream_create() for _ in range(2)]
                for n in (1 << 14, 1 << 18, 1 << 20, 8 << 20):
                    for rnd in range(2):
                        a = [oracle.fill_random(DT["float"], 0x5A00 + 64 * rnd + j, n) for j in range(npes)]
                        b = [oracle.fill_random(DT["float"], 0x5B00 + 64 * rnd + j, n) for j in range(npes)]
                        hip.upload(sa, a[pe])
                        hip.upload(sb, b[pe])
                        hip.memset(ret, 0x7F, 8)
                        ish.ishmem_barrier_all()
                        calls = [(da, sa, ret, sts[0], ta), (db, sb, ret + 4, sts[1], tb)]
                        if not first:
                            calls.reverse()
                        t0 = time.monotonic()
                        rc = [ish.reduce_on_stream("sum", "float", calls[0][0], calls[0][1], n, *calls[0][2:])]
                        time.sleep(0.02)
                        rc.append(ish.reduce_on_stream("sum", "float", calls[1][0], calls[1][1], n, *calls[1][2:]))
                        for st_ in sts:
                            hip.stream_synchronize(st_)
                        dt_s = time.monotonic() - t0
                        rets = hip.download(ret, 2, np.int32)
                        if any(rc) or np.any(rets != 0) or dt_s > 5.0:
                            fails.append(f"pe{pe} opposite n={n} round {rnd}: rc={rc} ret={rets} {dt_s:.2f} s "
                                         f"{ish.last_error()}")
                            break
                        check(f"opposite a n={n} {rnd}", OPS["sum"], DT["float"], a, hip.download(da, n, np.float32))
                        check(f"opposite b n={n} {rnd}", OPS["sum"], DT["float"], b, hip.download(db, n, np.float32))
                    if fails:
                        break
                for st_ in sts:
                    hip.stream_destroy(st_)
                for b_ in (ret, db, sb, da, sa):
                    ish.ishmem_free(b_)
                ish.ishmem_team_destroy(ta)
                ish.ishmem_team_destroy(tb)

        if "concurrent" in scenarios and npes >= 4 and npes % 2 == 0:
            # Collectives of different teams in flight at once on different streams (the TP / DP
            # groups of a 2-D split): an x-team and a y-team reduce, each 16 Mi floats, enqueued
            # back to back on two streams with no synchronisation, plus a WORLD LL reduce on a
            # third; every team has its own flag block and launch words, and no kernel needs its
            # grid resident, so they overlap in any interleaving.  Three rounds, inputs redrawn.
            r, xt, yt = ish.ishmem_team_split_2d(ish.ISHMEM_TEAM_WORLD, 2)
            if r:
                fails.append(f"pe{pe} concurrent split: {ish.last_error()}")
            else:
                xm = [j for j in range(npes) if j // 2 == pe // 2]
                ym = [j for j in range(npes) if j % 2 == pe % 2]
                n, nsmall = 16 << 20, 3000
                sx, dx, sy, dy = (heap(n, DT["float"]) for _ in range(4))
                sw, dw = heap(nsmall, DT["int32"]), heap(nsmall, DT["int32"])
                ret = ish.ishmem_malloc(12)
                sts = [hip.stream_create() for _ in range(3)]
                for rnd in range(3):
                    ax = {j: oracle.fill_random(DT["float"], 0xC0 + 16 * rnd + j, n) for j in xm}
                    ay = {j: oracle.fill_random(DT["float"], 0xD0 + 16 * rnd + j, n) for j in ym}
                    aw = [oracle.fill_random(DT["int32"], 0xE0 + 16 * rnd + j, nsmall) for j in range(npes)]
                    hip.upload(sx, ax[pe])
                    hip.upload(sy, ay[pe])
                    hip.upload(sw, aw[pe])
                    hip.memset(ret, 0x7F, 12)
                    ish.ishmem_barrier_all()
                    rc = [ish.reduce_on_stream("sum", "float", dx, sx, n, ret, sts[0], xt),
                          ish.reduce_on_stream("sum", "float", dy, sy, n, ret + 4, sts[1], yt),
                          ish.reduce_on_stream("max", "int32", dw, sw, nsmall, ret + 8, sts[2])]
                    for st_ in sts:
                        hip.stream_synchronize(st_)
                    rets = hip.download(ret, 3, np.int32)
                    if any(rc) or np.any(rets != 0):
                        fails.append(f"pe{pe} concurrent round {rnd}: rc={rc} ret={rets} {ish.last_error()}")
                        break
                    check(f"concurrent x {rnd}", OPS["sum"], DT["float"], [ax[j] for j in xm],
                          hip.download(dx, n, np.float32), me=xm.index(pe))
                    check(f"concurrent y {rnd}", OPS["sum"], DT["float"], [ay[j] for j in ym],
                          hip.download(dy, n, np.float32), me=ym.index(pe))
                    check(f"concurrent world {rnd}", OPS["max"], DT["int32"], aw, hip.download(dw, nsmall, np.int32))
                for st_ in sts:
                    hip.stream_destroy(st_)
                for b_ in (ret, dw, sw, dy, sy, dx, sx):
                    ish.ishmem_free(b_)
                ish.ishmem_team_destroy(xt)
                ish.ishmem_team_destroy(yt)

        if "huge8" in scenarios:
            # More than 2^32 ELEMENTS per PE (4.5 GiB of uint8, xor) from a misaligned start: any
            # 32-bit element index or byte offset in the path would alias chunk k + 256 onto chunk
            # k.  Source: a 16 MiB base block per PE; PE 0's is xor-tagged per 16 MiB chunk so
            # that chunks k and k + 256 of the result differ.
            blk = 16 << 20
            n = (9 << 29) + 5  # 4.5 GiB + 5 B
            s_base = ish.ishmem_malloc(n + 64)
            d_base = ish.ishmem_malloc(n + 64)
            if not (s_base and d_base):
                raise RuntimeError(f"huge8 heap: {ish.last_error()}")
            s, d = s_base + 3, d_base + 3

            def base_of(j):
                i = np.arange(blk, dtype=np.uint32)
                return ((i * 2654435761 + j * 40503) >> 13).astype(np.uint8)

            def tag(k):
                return np.uint8((k * 7 + (k >> 8) * 13 + 1) & 0xFF)

            mine = base_of(pe)
            for k in range((n + blk - 1) // blk):
                m = min(blk, n - k * blk)
                hip.upload(s + k * blk, mine[:m] ^ tag(k) if pe == 0 else mine[:m])  # tag on PE 0 only
            r = ish.reduce("xor", "uint8", d, s, n)
            if r:
                fails.append(f"pe{pe} huge8 rc={r} {ish.last_error()}")
            else:
                allb = np.bitwise_xor.reduce([base_of(j) for j in range(npes)])
                for lo in (0, (1 << 32) - 2048, (1 << 32) + 12345, n - 4096, (256 << 24) + 77):
                    m = min(4096, n - lo)
                    got = hip.download(d + lo, m, np.uint8)
                    idx = np.arange(lo, lo + m)
                    want = allb[idx % blk] ^ np.array([tag(int(k)) for k in idx // blk], np.uint8)
                    if not np.array_equal(got, want):
                        fails.append(f"pe{pe} huge8: wrong bytes near {lo} ({int(np.sum(got != want))})")
                    elif pe == 0:
                        print(f"[huge8] pe0 {m} bytes at {lo} match ({n} B per PE)", flush=True)
            ish.ishmem_free(d_base)
            ish.ishmem_free(s_base)

        if "occupied" in scenarios:
            # Residency independence: PE 0 first enqueues, on another stream, a kernel holding all
            # but 16 CUs (two 1024-work-item, 80 KiB-LDS workgroups per CU) for 4 s; then the PEs
            # run a 64 MiB f32 sum, PE 0 with a 1024-workgroup grid of which only a fraction can
            # be resident, the others with 16 workgroups (all PEs share this one GPU: a peer's
            # full grid of waiting workgroups would otherwise take the free CUs PE 0 needs, which
            # cannot happen across GPUs).  Nothing in the collective pairs workgroups across PEs,
            # so it completes on the free CUs, correct, long before the occupying kernel ends.
            ish.set_param("max_blocks", 1024 if pe == 0 else 16)
            n = 16 << 20
            ins = [oracle.fill_random(DT["float"], 0x0CC + j, n) for j in range(npes)]
            s, d = heap(n, DT["float"]), heap(n, DT["float"])
            ret = ish.ishmem_malloc(4)
            hip.upload(s, ins[pe])
            hip.memset(ret, 0x7F, 4)
            occ, st = hip.stream_create(), hip.stream_create()
            ish.ishmem_barrier_all()
            if pe == 0:
                cus = int(ish.get_param("cu_count"))
                if ish.occupy(2 * max(1, cus - 16), 4_000_000, occ) != 0:
                    fails.append(f"pe0 occupy failed {ish.last_error()}")
                time.sleep(0.05)  # the occupying workgroups are resident before the reduce starts
            t0 = time.perf_counter()
            r = ish.ishmemx_float_sum_reduce_on_stream(d, s, n, ret, st)
            hip.stream_synchronize(st)
            dt_s = time.perf_counter() - t0
            rv = int(hip.download(ret, 1, np.int32)[0])
            if r or rv:
                fails.append(f"pe{pe} occupied: rc={r} ret={rv} {ish.last_error()}")
            else:
                check("occupied", OPS["sum"], DT["float"], ins, hip.download(d, n, np.float32))
            if dt_s > 3.0:
                fails.append(f"pe{pe} occupied: reduce took {dt_s:.2f} s, i.e. it waited for the occupied CUs")
            hip.stream_synchronize(occ)
            hip.stream_destroy(occ)
            hip.stream_destroy(st)
            for b_ in (ret, d, s):
                ish.ishmem_free(b_)
            ish.set_param("max_blocks", int(os.environ.get("ISHMEM_MAX_BLOCKS", 1024)))

        if "blockread" in scenarios:
            # Blocking calls return once a stream write after their launches has reached host
            # memory (runtime.cpp host_wait, block_spin 2, the default): dest must then be final
            # for work on ANY stream — read here right away through a non-blocking stream (not
            # ordered after the null stream), new inputs every round, granule / fold / phased
            # sizes, reduce / fcollect / scan / broadcast.
            nbst = hip.stream_create()
            cases = [(n, kind) for n in (100, 70_001, 1_000_003) for kind in ("reduce", "fcollect", "inscan", "broadcast")]
            nmax = 1_000_003
            src_r = ish.ishmem_malloc(4 * nmax)
            dst_r = ish.ishmem_malloc(4 * nmax * npes)
            hbuf = hip.host_malloc(4 * nmax * npes)
            hv = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_int32 * (nmax * npes)).from_address(hbuf))
            for rnd in range(3):
                for n, kind in cases:
                    ins = [oracle.fill_random(DT["int32"], 7000 + 97 * rnd + 13 * j + n, n) for j in range(npes)]
                    hip.upload(src_r, ins[pe])
                    ish.ishmem_barrier_all()
                    if kind == "reduce":
                        r, want = ish.ishmem_int32_sum_reduce(dst_r, src_r, n), oracle.reduce_fold(OPS["sum"], DT["int32"], ins, 0)
                    elif kind == "fcollect":
                        r, want = ish.ishmem_int32_fcollect(dst_r, src_r, n), np.concatenate(ins)
                    elif kind == "inscan":
                        r, want = ish.scan("int32", True, dst_r, src_r, n), oracle.scan_fold(DT["int32"], ins, pe, True)
                    else:
                        root = rnd % npes
                        r, want = ish.ishmem_int32_broadcast(dst_r, src_r, n, root), ins[root]
                    if r:
                        fails.append(f"pe{pe} blockread {kind} n={n}: rc={r} {ish.last_error()}")
                        continue
                    hip.memcpy_async(hbuf, dst_r, 4 * want.size, nbst)
                    hip.stream_synchronize(nbst)
                    if not np.array_equal(hv[:want.size], want.view(np.int32)):
                        fails.append(f"pe{pe} blockread {kind} n={n} round {rnd}: dest not final when the call returned")
            hip.stream_destroy(nbst)
            hip.host_free(hbuf)
            ish.ishmem_free(dst_r)
            ish.ishmem_free(src_r)

        if "llchain" in scenarios:
            # Granule-path collectives back to back on one stream with no host synchronisation
            # (round 5: reduce, fcollect, inclusive / exclusive scan, broadcast share the rings, whose two
            # parities alternate by epoch): 32 calls of random kind and size up to the granule
            # threshold, each with its own source and dest, PEs enqueueing with random host delays
            # so the device-side skew varies; every dest then checked against the oracle.
            import time as _t
            rng = np.random.default_rng(4242)
            cap = int(ish.get_param("ll_limit_bytes"))  # the granule path's threshold for this team size
            K = 32
            plan = []
            for k in range(K):
                kind = ["reduce", "fcollect", "inscan", "exscan", "broadcast"][int(rng.integers(5))]
                dt = [DT["int32"], DT["float"], DT["uint64"], DT["double"]][int(rng.integers(4))]
                es = np.dtype(oracle.NP[dt]).itemsize
                limit = cap // 2 if kind in ("fcollect", "broadcast") else cap
                n = max(1, int(np.exp(rng.uniform(0.0, np.log(limit // es)))))
                op = OPS["sum"] if kind != "reduce" else [OPS["sum"], OPS["max"], OPS["min"]][int(rng.integers(3))]
                if kind == "broadcast":
                    op = int(rng.integers(npes))  # the root
                plan.append((kind, dt, es, n, op))
            bufs = []
            for k, (kind, dt, es, n, op) in enumerate(plan):
                ins = [oracle.fill_random(dt, 9000 + 31 * k + j, n) for j in range(npes)]
                sb = ish.ishmem_malloc(n * es)
                db = ish.ishmem_malloc(n * es * (npes if kind == "fcollect" else 1))
                hip.upload(sb, ins[pe])
                bufs.append((sb, db, ins))
            st_c = hip.stream_create()
            ret_c = ish.ishmem_malloc(4)
            hip.memset(ret_c, 0, 4)
            ish.ishmem_barrier_all()
            delays = np.random.default_rng(77 + pe).uniform(0, 2e-4, K)
            for k, (kind, dt, es, n, op) in enumerate(plan):
                _t.sleep(float(delays[k]))
                sb, db, _ = bufs[k]
                if kind == "reduce":
                    r = ish.reduce_on_stream(ONAMES[op], NAMES[dt], db, sb, n, ret_c, st_c)
                elif kind == "fcollect":
                    r = ish.fcollect_on_stream(db, sb, n * es, ret_c, st_c)
                elif kind == "broadcast":
                    r = ish.broadcast_on_stream(db, sb, n * es, op, ret_c, st_c)
                else:
                    r = ish.lib().ishmemi_c_scan_on_stream(0, dt, 1 if kind == "inscan" else 0, db, sb, n, ret_c, st_c)
                if r:
                    fails.append(f"pe{pe} llchain k={k} {kind}: rc={r} {ish.last_error()}")
                    break
            hip.stream_synchronize(st_c)
            if int(hip.download(ret_c, 1, np.int32)[0]) != 0:
                fails.append(f"pe{pe} llchain: *ret set")
            for k, (kind, dt, es, n, op) in enumerate(plan):
                sb, db, ins = bufs[k]
                tag = f"llchain k={k} {kind} dt={NAMES[dt]} n={n}"
                if kind == "reduce":
                    check(tag, op, dt, ins, hip.download(db, n, oracle.NP[dt]))
                elif kind == "fcollect":
                    if not _bits_equal(hip.download(db, n * npes, oracle.NP[dt]), np.concatenate(ins)):
                        fails.append(f"pe{pe} {tag} wrong")
                elif kind == "broadcast":
                    if not _bits_equal(hip.download(db, n, oracle.NP[dt]), ins[op]):
                        fails.append(f"pe{pe} {tag} root={op} wrong")
                else:
                    if not _bits_equal(hip.download(db, n, oracle.NP[dt]), oracle.scan_fold(dt, ins, pe, kind == "inscan")):
                        fails.append(f"pe{pe} {tag} wrong")
                ish.ishmem_free(db)
                ish.ishmem_free(sb)
            ish.ishmem_free(ret_c)
            hip.stream_destroy(st_c)

        if "stress" in scenarios:
            # Randomised protocol stress: every iteration draws (same draw on every PE) an
            # (op, type), a length from 1 element to 4 Mi (log-uniform: granule path, one-shot,
            # RS + AG with many segments), an element offset, in place or not, a team, a grid
            # cap per PE, and whether one PE first fills the GPU with an occupying kernel on
            # another stream (residency perturbation: announce fallback, claims, steals).  The
            # collectives are chained on one stream with *ret; each window is compared with the
            # oracle's canonical fold and the guard words around it must be untouched.
            iters = int(os.environ.get("STRESS_ITERS", 40))
            seed = int(os.environ.get("STRESS_SEED", 1234))
            nmax, pad = 4 << 20, 64
            combos = [(op, dt) for op in range(7) for dt in (DT["int32"], DT["uint64"], DT["float"], DT["double"], DT["uint8"])
                      if oracle.valid(op, dt)]
            teams = [(ish.ISHMEM_TEAM_WORLD, list(range(npes)))]
            if npes >= 3:
                r_, t_ = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 0, 2, (npes + 1) // 2)
                if r_:
                    fails.append(f"pe{pe} stress split: {ish.last_error()}")
                else:
                    teams.append((t_, list(range(0, npes, 2))))
                r_, t_ = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 1, 1, npes - 1)
                if r_:
                    fails.append(f"pe{pe} stress split: {ish.last_error()}")
                else:
                    teams.append((t_, list(range(1, npes))))
            S = ish.ishmem_malloc((nmax + 2 * pad) * 8)
            D = ish.ishmem_malloc((nmax + 2 * pad) * 8)
            ret = ish.ishmem_malloc(4)
            st, occ = hip.stream_create(), hip.stream_create()
            cus = int(ish.get_param("cu_count"))
            done_iters, occupied, kinds = 0, 0, set()
            for k in range(iters):
                rng = np.random.default_rng(seed * 7919 + k)
                op, dt = combos[int(rng.integers(len(combos)))]
                es = np.dtype(oracle.NP[dt]).itemsize
                n = int(np.exp(rng.uniform(0.0, np.log(nmax))))
                n = max(1, min(n, nmax))
                o = int(rng.integers(0, 4))
                inplace = bool(rng.random() < 0.25)
                # Source offset drawn separately (round 5): sources on another 16-B phase than dest
                # take the realigned reduce-scatter (phased sizes) or the element-granular path.
                so = o if rng.random() < 0.5 else int(rng.integers(0, 4))
                th, members = teams[int(rng.integers(len(teams)))]
                occupier = int(rng.integers(npes)) if rng.random() < 0.2 else -1
                cap = [int(rng.choice([16, 64, 256, 1024])) for _ in range(npes)]
                tag = (f"stress k={k} op={ONAMES[op]} dt={NAMES[dt]} n={n} o={o} so={so} inplace={inplace} "
                       f"team={members} occ={occupier} cap={cap[pe]}")
                ish.set_param("max_blocks", cap[pe])
                lo, hi = (0.5, 2.0) if op == OPS["prod"] else (-1.0, 1.0)
                ins = [oracle.fill_random(dt, (seed << 20) + k * 64 + j, n, lo, hi) for j in range(len(members))]
                # Guards: the whole dest region (and the source region in place) holds 0xA5 bytes.
                hip.memset(D, 0xA5, (nmax + 2 * pad) * 8)
                hip.synchronize()
                dbase = D + pad * 8 + o * es
                sbase = dbase if inplace else S + pad * 8 + so * es
                if pe in members:
                    hip.upload(sbase, ins[members.index(pe)])
                ish.ishmem_barrier_all()
                if pe == occupier:
                    ish.occupy(2 * cus, 300, occ)
                if pe in members:
                    hip.memset(ret, 0, 4)
                    r = ish.reduce_on_stream(ONAMES[op], NAMES[dt], dbase, sbase, n, ret, st, th)
                    hip.stream_synchronize(st)
                    rv = int(hip.download(ret, 1, np.int32)[0])
                    if r or rv:
                        fails.append(f"pe{pe} {tag}: rc={r} ret={rv} {ish.last_error()}")
                        break
                    whole = hip.download(D, (nmax + 2 * pad) * 8, np.uint8)
                    lo_b, hi_b = pad * 8 + o * es, pad * 8 + o * es + n * es
                    got = whole[lo_b:hi_b].view(oracle.NP[dt])
                    nf = len(fails)
                    check(tag, op, dt, ins, got, me=members.index(pe))
                    if np.any(whole[:lo_b] != 0xA5) or np.any(whole[hi_b:] != 0xA5):
                        fails.append(f"pe{pe} {tag}: guard bytes around dest overwritten")
                    if len(fails) > nf:
                        break
                hip.stream_synchronize(occ)
                done_iters += 1
                ll_cap = min(int(ish.get_param("ll_max_bytes")), (2 << 20) // len(members))  # about kernels.h ll_capacity
                kinds.add("ll" if n * es <= ll_cap else ("big" if n * es > (1 << 20) else "mid"))
                occupied += occupier >= 0
            if pe == 0:
                print(f"[stress] pe0: {done_iters}/{iters} iterations, {occupied} with an occupier, "
                      f"sizes {sorted(kinds)}", flush=True)
            hip.stream_destroy(occ)
            hip.stream_destroy(st)
            for th, _m in teams[1:]:
                ish.ishmem_team_destroy(th)
            for b_ in (ret, D, S):
                ish.ishmem_free(b_)
            ish.set_param("max_blocks", int(os.environ.get("ISHMEM_MAX_BLOCKS", 1024)))

        if "tripwire" in scenarios:
            from ishmem_amd import selfcheck
            res = selfcheck.chain_tripwire(ish, hip, pe, npes, nmax=int(os.environ.get("TRIPWIRE_N", 1 << 20)),
                                           iters=int(os.environ.get("TRIPWIRE_ITERS", 12)))
            if not res["checked"]:
                fails.append(f"pe{pe} tripwire: {res}")

        if "cfg3" in scenarios or "cfg4" in scenarios:
            # BASELINE configs[2] (2 PEs) / configs[3] (8 PEs) at their own size: float32 sum-reduce
            # of 1 GiB per PE, every word of dest compared on every PE with the team-order fold of
            # the rotating-winner pattern (selfcheck.pattern).
            from ishmem_amd import selfcheck as sc
            n = 256 << 20
            s, d = ish.ishmem_malloc(n * 4), ish.ishmem_malloc(n * 4)
            if not (s and d):
                raise RuntimeError(f"cfg3/4 heap: {ish.last_error()}")
            sc.upload_pattern(hip, s, np.float32, pe, npes, n)
            hip.memset(d, 0xFF, n * 4)
            r = ish.ishmem_float_sum_reduce(d, s, n)
            if r:
                fails.append(f"pe{pe} cfg3/4 rc={r} {ish.last_error()}")
            else:
                bad = sc.count_wrong(hip, d, "sum", np.float32, npes, 0, n)
                if bad:
                    fails.append(f"pe{pe} cfg3/4: {bad} of {4 * n} bytes wrong")
                elif pe == 0:
                    print(f"[cfg] pe0: {npes} PEs x 1 GiB f32 sum, every word matches", flush=True)
            ish.ishmem_free(d)
            ish.ishmem_free(s)

        if "cfg1" in scenarios:
            # BASELINE configs[0]: int32 sum-reduce over HOST buffers (the reference's host path,
            # reduce_impl.h:301-315), full-range seeded int32 (oracle.fill_random), n from the
            # examples/5_pi_reduce.cpp single element to 16 Mi; pageable (numpy) and pinned
            # buffers, in place and not; bit-exact vs the oracle fold on every PE.
            for n in (1, 1 << 10, (1 << 16) + 3, 1 << 20, 16 << 20):
                ins = [oracle.fill_random(DT["int32"], 0x15AE0001 + j, n) for j in range(npes)]
                src = np.ascontiguousarray(ins[pe])
                out = np.zeros(n, np.int32)
                r = ish.ishmem_int32_sum_reduce(out.ctypes.data, src.ctypes.data, n)
                if r:
                    fails.append(f"pe{pe} cfg1 pageable n={n} rc={r} {ish.last_error()}")
                else:
                    check(f"cfg1 pageable n={n}", OPS["sum"], DT["int32"], ins, out)
                hin, hout = hip.host_malloc(n * 4), hip.host_malloc(n * 4)
                hv = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_int32 * n).from_address(hin))
                hv[:] = ins[pe]
                r = ish.ishmem_int_sum_reduce(hout, hin, n)
                got = np.ctypeslib.as_array((np.ctypeslib.ctypes.c_int32 * n).from_address(hout)).copy()
                if r:
                    fails.append(f"pe{pe} cfg1 pinned n={n} rc={r} {ish.last_error()}")
                else:
                    check(f"cfg1 pinned n={n}", OPS["sum"], DT["int32"], ins, got)
                r = ish.ishmem_int_sum_reduce(hin, hin, n)  # in place on host memory
                got = hv.copy()
                if r:
                    fails.append(f"pe{pe} cfg1 pinned in place n={n} rc={r} {ish.last_error()}")
                else:
                    check(f"cfg1 pinned in place n={n}", OPS["sum"], DT["int32"], ins, got)
                del hv
                hip.host_free(hin)
                hip.host_free(hout)

        if "cfg5" in scenarios:
            # BASELINE configs[4]: min / max / prod x int32 / float64 at 4 KiB * 4^k up to
            # CFG5_MAX_BYTES (4 GiB) per PE, rotating-winner pattern (selfcheck.pattern), EVERY
            # word of dest on every PE compared at every size by the device checker
            # (tests/cpp/pattern_check.hip; int: bit-exact; f64 min / max exact, prod folded in team
            # order like the kernels: bit-exact), as the reference's tester compares every element
            # (test/include/ishmem_tester.h:1178-1281).
            from ishmem_amd import selfcheck as sc
            maxb = int(os.environ.get("CFG5_MAX_BYTES", 4 << 30))
            for dtn, npd in (("int32", np.int32), ("double", np.float64)):
                if sc.checker_kind(npd) != "device":
                    raise RuntimeError("cfg5: the device pattern checker (build/libpattern_check.so) is not built")
                es = np.dtype(npd).itemsize
                nmax = maxb // es
                s, d = ish.ishmem_malloc(maxb), ish.ishmem_malloc(maxb)
                if not (s and d):
                    raise RuntimeError(f"cfg5 heap: {ish.last_error()}")
                sc.upload_pattern(hip, s, npd, pe, npes, nmax)
                for op in ("min", "max", "prod"):
                    nb = 4096
                    while nb <= maxb:
                        n = nb // es
                        hip.memset(d, 0xA5, min(nb + 64, maxb))
                        r = ish.reduce(op, dtn, d, s, n)
                        if r:
                            fails.append(f"pe{pe} cfg5 {op} {dtn} {nb} B rc={r} {ish.last_error()}")
                            nb *= 4
                            continue
                        bad = sc.count_wrong(hip, d, op, npd, npes, 0, n, device=True)
                        if bad:
                            fails.append(f"pe{pe} cfg5 {op} {dtn} {nb} B: {bad} bytes wrong")
                        # the poisoned bytes past n must stay untouched
                        if nb < maxb and int(np.count_nonzero(hip.download(d + nb, 64, np.uint8) != 0xA5)):
                            fails.append(f"pe{pe} cfg5 {op} {dtn} {nb} B: wrote past dest's end")
                        nb *= 4
                ish.ishmem_free(d)
                ish.ishmem_free(s)

        if "collect" in scenarios:
            # fcollect.cpp / collect.cpp testers: per-PE word pattern, dest = the members' blocks
            # concatenated in team order; offsets 0..14 in steps of sizeof(T) like
            # collect.cpp:109-141; collect counts drawn per PE (collect.cpp:120-124).
            rng = np.random.default_rng(4242)
            for tn, es in (("uchar", 1), ("short", 2), ("float", 4), ("double", 8)):
                for nelems in (1, 3, 1000, 40_001):
                    counts_c = [int(c) for c in rng.integers(1, nelems + 1, npes)]
                    for so, do in ((0, 0), (es, 3 * es), (7 * es if es < 2 else 2 * es, 0)):
                        src_b = ish.ishmem_malloc(nelems * es + 64)
                        dst_b = ish.ishmem_malloc(npes * nelems * es + 64)
                        hip.upload(src_b + so, oracle.collect_pattern_source(pe, nelems, es))
                        fn = getattr(ish, f"ishmem_{tn}_fcollect")
                        r = fn(dst_b + do, src_b + so, nelems)
                        want = oracle.collect_check([nelems] * npes, es)
                        if r:
                            fails.append(f"pe{pe} fcollect {tn} n{nelems} rc={r} {ish.last_error()}")
                        elif not _bits_equal(hip.download(dst_b + do, want.size, np.uint8), want):
                            fails.append(f"pe{pe} fcollect {tn} n{nelems} so{so} do{do} wrong")
                        c = counts_c[pe]
                        hip.upload(src_b + so, oracle.collect_pattern_source(pe, c, es))
                        r = getattr(ish, f"ishmem_{tn}_collect")(dst_b + do, src_b + so, c)
                        want = oracle.collect_check(counts_c, es)
                        if r:
                            fails.append(f"pe{pe} collect {tn} rc={r} {ish.last_error()}")
                        elif not _bits_equal(hip.download(dst_b + do, want.size, np.uint8), want):
                            fails.append(f"pe{pe} collect {tn} counts{counts_c} so{so} do{do} wrong")
                        ish.ishmem_free(dst_b)
                        ish.ishmem_free(src_b)
            # Sources outside the heap (the reference's intra-node collect copies from any local
            # source, collect_impl.h:93-114): staged through the symmetric staging region, in
            # segments when larger than it (ISHMEM_STAGING_SIZE = 4M here: 5 MiB -> 2 segments);
            # dest in plain device memory; a collect where only PE 0's source is host memory.
            for nb_f in (4000, 5 << 20):
                dsrc = hip.malloc(nb_f)
                src_pat = oracle.collect_pattern_source(pe, nb_f // 4, 4)
                hip.upload(dsrc, src_pat)
                dd = ish.ishmem_malloc(npes * nb_f + 64)
                want = oracle.collect_check([nb_f // 4] * npes, 4)
                if ish.ishmem_int32_fcollect(dd, dsrc, nb_f // 4) or not _bits_equal(
                        hip.download(dd, want.size, np.uint8), want):
                    fails.append(f"pe{pe} fcollect from device memory {nb_f} B wrong {ish.last_error()}")
                ddev = hip.malloc(npes * nb_f)
                if ish.ishmem_int32_fcollect(ddev, dsrc, nb_f // 4) or not _bits_equal(
                        hip.download(ddev, want.size, np.uint8), want):
                    fails.append(f"pe{pe} fcollect into device memory {nb_f} B wrong {ish.last_error()}")
                hip.free(ddev)
                hip.free(dsrc)
                ish.ishmem_free(dd)
            cnts = [int(x) for x in rng.integers(1, 3_000_000, npes)]  # up to 12 MiB: several segments
            mine_h = np.ascontiguousarray(oracle.collect_pattern_source(pe, cnts[pe], 4))
            hsrc = ish.ishmem_malloc(cnts[pe] * 4 + 64)
            hip.upload(hsrc, mine_h)
            dd = ish.ishmem_malloc(sum(cnts) * 4 + 64)
            srcp = mine_h.ctypes.data if pe == 0 else hsrc
            want = oracle.collect_check(cnts, 4)
            if ish.ishmem_int32_collect(dd, srcp, cnts[pe]) or not _bits_equal(
                    hip.download(dd, want.size, np.uint8), want):
                fails.append(f"pe{pe} collect with PE 0's source in host memory wrong {ish.last_error()}")
            ish.ishmem_free(dd)
            ish.ishmem_free(hsrc)
            # collect on a stream (ishmemx_<TN>_collect_on_queue): the counts meet on the device.
            # Three calls chained on one stream with no host synchronisation, counts redrawn per
            # call (a count slot reused before a peer read it would show), one member empty,
            # byte / 4-B / 16-B units by alignment; then every dest is compared.
            st_c = hip.stream_create()
            ret_c = ish.ishmem_malloc(4)
            calls = []
            for c_i, (es_c, so, do) in enumerate(((4, 0, 0), (1, 3, 5), (16, 0, 16))):
                cnts = [int(x) for x in rng.integers(0, 3000, npes)]
                cnts[c_i % npes] = 0 if c_i == 1 else cnts[c_i % npes]
                src_c = ish.ishmem_malloc(3000 * es_c + 64)
                dst_c = ish.ishmem_malloc(sum(cnts) * es_c + 64)
                if cnts[pe]:
                    hip.upload(src_c + so, oracle.collect_pattern_source(pe, cnts[pe], es_c))
                calls.append((cnts, es_c, so, do, src_c, dst_c))
            hip.memset(ret_c, 0x7F, 4)
            ish.ishmem_barrier_all()
            for cnts, es_c, so, do, src_c, dst_c in calls:
                if ish.collect_on_stream(dst_c + do, src_c + so, cnts[pe] * es_c, ret_c, st_c) != 0:
                    fails.append(f"pe{pe} collect_on_stream enqueue {ish.last_error()}")
            hip.stream_synchronize(st_c)
            if int(hip.download(ret_c, 1, np.int32)[0]) != 0:
                fails.append(f"pe{pe} collect_on_stream *ret != 0")
            for cnts, es_c, so, do, src_c, dst_c in calls:
                want = oracle.collect_check(cnts, es_c)
                if want.size and not _bits_equal(hip.download(dst_c + do, want.size, np.uint8), want):
                    fails.append(f"pe{pe} collect_on_stream es{es_c} counts{cnts} wrong")
                ish.ishmem_free(dst_c)
                ish.ishmem_free(src_c)
            hip.stream_destroy(st_c)
            ish.ishmem_free(ret_c)
            # fcollectmem of odd byte counts; nelems 0 (still a team sync)
            src_b, dst_b = ish.ishmem_malloc(4096), ish.ishmem_malloc(4096 * npes)
            hip.upload(src_b, oracle.collect_pattern_source(pe, 1001, 1))
            if ish.ishmem_fcollectmem(dst_b, src_b, 1001) or not _bits_equal(
                    hip.download(dst_b, 1001 * npes, np.uint8), oracle.collect_check([1001] * npes, 1)):
                fails.append(f"pe{pe} fcollectmem 1001 B wrong {ish.last_error()}")
            if ish.ishmem_int_fcollect(dst_b, src_b, 0) or ish.ishmem_collectmem(dst_b, src_b, 0):
                fails.append(f"pe{pe} fcollect n=0 failed {ish.last_error()}")
            # on a strided team (even PEs) via the team overload
            if npes >= 2:
                r, team = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 0, 2, (npes + 1) // 2)
                if team != ish.ISHMEM_TEAM_INVALID:
                    members = list(range(0, npes, 2))
                    hip.upload(src_b, oracle.collect_pattern_source(members.index(pe), 333, 4))
                    want = oracle.collect_check([333] * len(members), 4)
                    if ish.ishmem_int32_fcollect(team, dst_b, src_b, 333) or not _bits_equal(
                            hip.download(dst_b, want.size, np.uint8), want):
                        fails.append(f"pe{pe} team fcollect wrong {ish.last_error()}")
                    ish.ishmem_team_destroy(team)
            ish.ishmem_free(dst_b)
            ish.ishmem_free(src_b)

        if "scan" in scenarios:
            # inscan.cpp / exscan.cpp testers (word pattern pe+idx, closed-form check) over the
            # reference's scan_types, then seeded random inputs vs the oracle's team-order fold.
            for tn in ("short", "int", "long", "ushort", "uint", "size", "int16", "uint64", "float", "double"):
                dt = DT[ish.TYPENAMES[tn]]
                es = np.dtype(oracle.NP[dt]).itemsize
                for nelems in (1, 5, 4096 + 3, 70_001):
                    nb = nelems * es
                    s_b, d_b = ish.ishmem_malloc(nb + 64), ish.ishmem_malloc(nb + 64)
                    hip.upload(s_b, oracle.scan_pattern_source(pe, nb))
                    for inc in (True, False):
                        fn = getattr(ish, f"ishmem_{tn}_sum_{'inscan' if inc else 'exscan'}")
                        hip.memset(d_b, 0xA5, nb)
                        r = fn(d_b, s_b, nelems)
                        if r:
                            fails.append(f"pe{pe} {tn} scan rc={r} {ish.last_error()}")
                            continue
                        got = hip.download(d_b, nb, np.uint8)
                        srcs = [oracle.scan_pattern_source(j, nb).view(oracle.NP[dt]) for j in range(npes)]
                        if not _bits_equal(got, oracle.scan_fold(dt, srcs, pe, inc)):
                            fails.append(f"pe{pe} {tn} {'in' if inc else 'ex'}scan n{nelems} != oracle")
                        # The tester's closed form holds while no lane carries (its word sums
                        # stay below 2^(8*sizeof T)); beyond that the oracle above is the check.
                        if nelems <= 4099 and not _bits_equal(got, oracle.scan_pattern_check(pe, nb, inc)):
                            fails.append(f"pe{pe} {tn} {'in' if inc else 'ex'}scan n{nelems} != tester check pattern")
                    ish.ishmem_free(d_b)
                    ish.ishmem_free(s_b)
            for dt in (DT["int8"], DT["int32"], DT["uint64"], DT["float"], DT["double"]):
                n = 123_457
                ins = [oracle.fill_random(dt, 600 + j, n) for j in range(npes)]
                if dt >= 8:
                    ins[0][:3] = -0.0  # first term passes through unchanged (sign of zero kept)
                s_b, d_b = heap(n, dt), heap(n, dt)
                hip.upload(s_b, ins[pe])
                for inc in (True, False):
                    r = ish.scan(NAMES[dt], inc, d_b, s_b, n)
                    ref = oracle.scan_fold(dt, ins, pe, inc)
                    got = hip.download(d_b, n, oracle.NP[dt])
                    if r:
                        fails.append(f"pe{pe} scan dt{dt} rc={r} {ish.last_error()}")
                    elif not _bits_equal(got, ref):
                        fails.append(f"pe{pe} scan dt{dt} inc={inc}: "
                                     f"{int(np.sum(got.view(np.uint8) != ref.view(np.uint8)))} bytes differ")
                ish.ishmem_free(d_b)
                ish.ishmem_free(s_b)
            # host buffers (the reference proxies them to MPI_Scan / MPI_Exscan): staged through
            # symmetric temporaries
            for dt in (DT["int32"], DT["double"]):
                n = 77_777
                ins = [oracle.fill_random(dt, 680 + j, n) for j in range(npes)]
                hs = np.ascontiguousarray(ins[pe])
                for inc in (True, False):
                    hd = np.zeros(n, oracle.NP[dt])
                    r = ish.scan(NAMES[dt], inc, hd.ctypes.data, hs.ctypes.data, n)
                    if r or not _bits_equal(hd, oracle.scan_fold(dt, ins, pe, inc)):
                        fails.append(f"pe{pe} host-buffer scan dt{dt} inc={inc} wrong {ish.last_error()}")
            # element-granular path: 4-B aligned (not 16-B) buffers, odd length
            n = 50_001
            ins = [oracle.fill_random(DT["int32"], 650 + j, n) for j in range(npes)]
            s_b, d_b = heap(n + 8, DT["int32"]), heap(n + 8, DT["int32"])
            hip.upload(s_b + 4, ins[pe])
            for inc in (True, False):
                r = ish.scan("int32", inc, d_b + 12, s_b + 4, n)
                if r or not _bits_equal(hip.download(d_b + 12, n, np.int32), oracle.scan_fold(DT["int32"], ins, pe, inc)):
                    fails.append(f"pe{pe} misaligned scan inc={inc} wrong {ish.last_error()}")
            ish.ishmem_free(d_b)
            ish.ishmem_free(s_b)
            # several staging-sized segments (ISHMEM_STAGING_SIZE small in the test env)
            n = 3 * (ish.get_param("staging_bytes") // 4) + 17
            ins = [oracle.fill_random(DT["int32"], 700 + j, n) for j in range(npes)]
            s_b, d_b = heap(n, DT["int32"]), heap(n, DT["int32"])
            hip.upload(s_b, ins[pe])
            if ish.ishmem_int32_sum_inscan(d_b, s_b, n) or not _bits_equal(
                    hip.download(d_b, n, np.int32), oracle.scan_fold(DT["int32"], ins, pe, True)):
                fails.append(f"pe{pe} multi-segment scan wrong {ish.last_error()}")
            ish.ishmem_free(d_b)
            ish.ishmem_free(s_b)

        if ish.lib().ishmemi_c_error_count() != 0:
            fails.append(f"pe{pe} device barrier timeouts: {ish.lib().ishmemi_c_error_count()}")
        ish.ishmem_barrier_all()
        ish.ishmem_finalize()
    except Exception:
        fails.append(f"pe{pe} exception: {traceback.format_exc()}")
    q.put((pe, fails))
