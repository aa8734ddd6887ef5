"""Cross-PE coherence tripwire of the reduction path (used by bench.py at N > 1 and by the GPU
tests).  Everything runs through the C-ABI; the expected values come from a host simulation of
every PE's state in wrapping int32 arithmetic, so every checked word is exact.

Each iteration k, on one stream, with no host synchronisation between producer and collective:
  1. a producer kernel with ORDINARY (write-back) stores, like a user's, rewrites this PE's
     source window from the previous iteration's dest: S[o:o+n] = D[o:o+n] + base_pe[:n];
  2. ishmemx_int32_sum_reduce_on_stream(D + o, S + o, n) over team T_k.
The window offset o (0..3 elements: aligned and misaligned heads/tails), the length n (large
windows for reduce-scatter + all-gather, every fourth one small enough for the one-hop granule
path) and the team (WORLD, then a second team with its own flag block) change every iteration,
and dest of step k feeds source of step k+1.  A peer that read a stale source line, a reduced
segment published before its bytes landed, or a flag row reused across teams would show up as a
wrong word in the FULL window, which every PE downloads and compares every iteration.
"""
from __future__ import annotations

import numpy as np


def _base(pe: int, n: int) -> np.ndarray:
    # Deterministic full-range int32 words per PE (xorshift-multiply hash of the index).
    i = np.arange(n, dtype=np.uint64)
    x = (i + np.uint64(0x9E3779B97F4A7C15) * np.uint64(pe + 1)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    x ^= x >> np.uint64(29)
    x = (x * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    x ^= x >> np.uint64(32)
    return (x & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def chain_tripwire(ish, hip, pe: int, npes: int, nmax: int = 1 << 20, iters: int = 8,
                   small: int = 1500, stream: int | None = None) -> dict:
    """Runs the chained producer -> reduce iterations described above on every PE (collective:
    every PE calls it with the same arguments).  Returns {"iters", "elems", "mismatches": [per
    iteration words wrong on this PE], "checked": all zero, "teams"}.  `stream`: the caller's
    stream (default: a stream created and destroyed here).  PEs sharing one GPU should pass theirs:
    every extra HIP stream is another hardware queue, and with more queues than the scheduler
    keeps mapped, cross-process collectives on one device pay queue-switch latency (measured: a
    4 KiB two-PE reduce goes from ~4 to ~28 us per call after one stream_create per process)."""
    pad = 8
    S = ish.ishmem_malloc((nmax + pad) * 4)
    D = ish.ishmem_malloc((nmax + pad) * 4)
    B = ish.ishmem_malloc((nmax + pad) * 4)
    if not (S and D and B):
        raise RuntimeError(f"tripwire: heap allocation failed: {ish.last_error()}")
    bases = [_base(j, nmax + pad) for j in range(npes)]
    hip.upload(B, bases[pe])
    hip.memset(D, 0, (nmax + pad) * 4)
    dsim = [np.zeros(nmax + pad, np.uint32) for _ in range(npes)]
    m = max(2, npes // 2) if npes > 1 else 1
    r, team2 = ish.ishmem_team_split_strided(ish.ISHMEM_TEAM_WORLD, 0, 1, m)
    if r:
        raise RuntimeError(f"tripwire: team split failed: {ish.last_error()}")
    teams = [(ish.ISHMEM_TEAM_WORLD, list(range(npes))), (team2, list(range(m)))]
    own = stream is None
    st = hip.stream_create() if own else stream
    ish.ishmem_barrier_all()
    mism = []
    try:
        for k in range(iters):
            o = k % 4
            n = small + k if k % 4 == 3 else nmax - 3 * k
            th, members = teams[k % 2]
            if pe in members:
                if ish.lib().ishmemi_c_produce_u32(S + 4 * o, D + 4 * o, B, n, st) != 0:
                    raise RuntimeError(f"tripwire: producer failed: {ish.last_error()}")
                if ish.reduce_on_stream("sum", "int32", D + 4 * o, S + 4 * o, n, None, st, th) != 0:
                    raise RuntimeError(f"tripwire: reduce failed: {ish.last_error()}")
            hip.stream_synchronize(st)
            acc = np.zeros(n, np.uint32)
            for j in members:
                acc += dsim[j][o:o + n] + bases[j][:n]  # wraps mod 2^32, like the int32 sum
            for j in members:
                dsim[j][o:o + n] = acc
            got = hip.download(D, nmax + pad, np.uint32)
            mism.append(int(np.count_nonzero(got != dsim[pe])))
            # No host barrier here: PEs drift apart and the next launches are ordered by the
            # device protocol alone (a peer reads this PE's new source only after this PE's
            # next launch has announced itself).
    finally:
        if own:
            hip.stream_destroy(st)
        if team2 != ish.ISHMEM_TEAM_INVALID:
            ish.ishmem_team_destroy(team2)
        for b in (B, D, S):
            ish.ishmem_free(b)
    errs = ish.lib().ishmemi_c_error_count()
    return {"iters": iters, "elems": nmax, "mismatches": mism, "device_errors": errs,
            "checked": all(x == 0 for x in mism) and errs == 0, "teams": [npes, m]}
