"""CPU tests of the ORACLE (test infrastructure): pin it before trusting it.

1. The oracle's fold of the reference testers' source patterns equals the reference testers'
   own check patterns (test/unit/reduce_{sum,prod,min,max,and,or,xor}.cpp), restated in
   oracle/oracle.c, for every valid (op, dtype), npes 1..8 and the tester's power-of-two sizes.
2. The oracle agrees with MPICH's MPI_Allreduce (the reference host path's arithmetic backend,
   src/runtime/runtime_mpi.cpp:802-812) on the committed golden vectors tests/golden/*.npz:
   bit-exact for integer types and FP min/max, within the order-independent bound for FP sum/prod.
3. The host bounce path restatement (64 KiB chunks, reduce_impl.h:186-228) equals the fold.
"""
from pathlib import Path

import numpy as np
import pytest

import oracle

GOLDEN = Path(__file__).resolve().parent / "golden"
VALID = [(op, dt) for op in range(7) for dt in range(10) if oracle.valid(op, dt)]


def test_validity_matrix():
    # docs/source/collectives.rst:910-936: 3 bitwise ops x 8 int types + 4 ops x 10 types
    assert len(VALID) == 3 * 8 + 4 * 10
    assert not oracle.valid(oracle.OPS["and"], oracle.DTYPES["float"])
    assert oracle.valid(oracle.OPS["max"], oracle.DTYPES["double"])


@pytest.mark.parametrize("npes", [1, 2, 3, 4, 8])
def test_fold_of_reference_patterns_matches_reference_check(npes):
    for op, dt in VALID:
        fam = oracle.family_for(op)
        for nelems in [1, 2, 4, 16, 128, 1024, 4096]:
            srcs = [oracle.pattern_source(fam, dt, pe, nelems) for pe in range(npes)]
            got = oracle.reduce_fold(op, dt, srcs, 0)
            chk = oracle.pattern_check(fam, op, dt, npes, nelems)
            assert np.array_equal(got.view(np.uint8), chk.view(np.uint8)), (op, dt, npes, nelems)


def test_device_fold_order_per_pe_fp_can_differ_but_ints_never():
    # The reference folds "self first, then team order" (reduce_impl.h:247-253): FP sums can
    # differ between PEs (docs/source/collectives.rst:1241-1244); integer results never do.
    rng = np.random.default_rng(7)
    srcs = [rng.uniform(-1, 1, 4096).astype(np.float32) for _ in range(4)]
    outs = [oracle.reduce_fold(oracle.OPS["sum"], oracle.DTYPES["float"], srcs, me) for me in range(4)]
    assert any(not np.array_equal(outs[0], o) for o in outs[1:])
    tol = oracle.fp_tolerance(oracle.DTYPES["float"], oracle.OPS["sum"], srcs, outs[0])
    for o in outs:
        assert np.all(np.abs(o.astype(np.float64) - outs[0]) <= 2 * tol)
    isrcs = [rng.integers(-2**31, 2**31, 4096, dtype=np.int64).astype(np.int32) for _ in range(4)]
    iouts = [oracle.reduce_fold(oracle.OPS["sum"], oracle.DTYPES["int32"], isrcs, me) for me in range(4)]
    assert all(np.array_equal(iouts[0], o) for o in iouts)


def _golden_cases(npes):
    z = np.load(GOLDEN / f"golden_np{npes}.npz")
    names = sorted({k.rsplit("__", 1)[0] for k in z.files})
    for nm in names:
        op, dt, n = (int(x) for x in z[nm + "__meta"])
        yield nm, op, dt, n, list(z[nm + "__in"]), z[nm + "__out"]


@pytest.mark.parametrize("npes", [2, 4, 8])
def test_oracle_matches_mpich_golden(npes):
    count = 0
    for nm, op, dt, n, ins, outs in _golden_cases(npes):
        ref = oracle.reduce_fold(op, dt, ins, 0)
        if dt >= 8 and op in (oracle.OPS["sum"], oracle.OPS["prod"]):
            tol = oracle.fp_tolerance(dt, op, ins, ref)
            assert np.all(np.abs(outs.astype(np.float64) - ref.astype(np.float64)) <= tol), nm
        else:
            for o in outs:
                assert np.array_equal(o.view(np.uint8), ref.view(np.uint8)), nm
        count += 1
    assert count == 384


@pytest.mark.parametrize("npes", [2, 4, 8])
def test_golden_inputs_are_the_reference_patterns_and_seeds(npes):
    for nm, op, dt, n, ins, outs in _golden_cases(npes):
        for pe, x in enumerate(ins):
            if nm.startswith("pat_"):
                exp = oracle.pattern_source(oracle.family_for(op), dt, pe, n)
            else:
                lo, hi = (0.5, 2.0) if op == oracle.OPS["prod"] else (-1.0, 1.0)
                exp = oracle.fill_random(dt, 0x15AE0001 + pe, n, lo, hi)
            assert np.array_equal(exp.view(np.uint8), x.view(np.uint8)), (nm, pe)


@pytest.mark.parametrize("op,dt", [(5, 2), (5, 8), (3, 9), (6, 9), (2, 7), (4, 0)])
def test_host_proxy_restatement_equals_fold(op, dt):
    # Sizes straddling the 64 KiB chunk boundary of ISHMEM_REDUCE_BUFFER_SIZE.
    es = np.dtype(oracle.NP[dt]).itemsize
    for n in [0, 1, oracle.REDUCE_BUFFER_SIZE // es - 1, oracle.REDUCE_BUFFER_SIZE // es + 3, 50_000]:
        srcs = [oracle.fill_random(dt, 100 + pe, n, 0.5, 2.0) for pe in range(3)]
        outs = oracle.host_proxy_reduce(op, dt, srcs)
        ref = oracle.reduce_fold(op, dt, srcs, 0) if n else srcs[0]
        for o in outs:
            assert np.array_equal(o.view(np.uint8), ref.view(np.uint8))


def test_long_reduce_known_answer():
    # test/unit/long_reduce.cpp:78-79,120-127: source = (1 << (40+pe)) + idx,
    # expected = ((1 << npes) - 1) << 40 + idx * npes.
    for npes in (1, 2, 8):
        n = 1000
        idx = np.arange(n, dtype=np.int64)
        srcs = [(np.int64(1) << np.int64(40 + pe)) + idx for pe in range(npes)]
        got = oracle.reduce_fold(oracle.OPS["sum"], oracle.DTYPES["int64"], srcs, 0)
        exp = (np.int64((1 << npes) - 1) << np.int64(40)) + idx * npes
        assert np.array_equal(got, exp)


def test_host_proxy_timer_runs():
    t = oracle.host_proxy_time(oracle.OPS["sum"], oracle.DTYPES["int32"], 1 << 16, 2, 2)
    assert 0 < t < 10


def test_scan_fold_reproduces_reference_tester_check_patterns():
    # inscan.cpp:46-58 / exscan.cpp:46-59 closed forms vs the oracle's team-order prefix fold on
    # the testers' source pattern, for every dtype (FP words are exact denormal sums).
    for dt in range(10):
        es = np.dtype(oracle.NP[dt]).itemsize
        for p in (1, 2, 3, 4, 8):
            for nb in (es, 8 * es, 41 * es):
                srcs = [oracle.scan_pattern_source(pe, nb).view(oracle.NP[dt]) for pe in range(p)]
                for me in range(p):
                    for inc in (True, False):
                        got = oracle.scan_fold(dt, srcs, me, inc).view(np.uint8)
                        assert np.array_equal(got, oracle.scan_pattern_check(me, nb, inc)), (dt, p, nb, me, inc)


def test_collect_check_is_concatenation_of_sources():
    src = [oracle.collect_pattern_source(pe, c, 2) for pe, c in enumerate([3, 1, 5])]
    chk = oracle.collect_check([3, 1, 5], 2)
    assert np.array_equal(chk, np.concatenate(src))
    w = oracle.collect_pattern_source(1, 4, 8).view(np.uint64)
    assert int(w[2]) == (4 << 48) + (0x81 << 40) + (0xff << 32) + 2  # fcollect.cpp:54-55


def _bounce_member(me, npes, key, n, q):
    import ctypes

    import numpy as np

    import oracle
    src = oracle.fill_random(oracle.DTYPES["int32"], 0xB0 + me, n)
    dst = np.zeros(n, np.int32)
    calls = []

    def copy(d, s, nb, kind):  # stands in for hipMemcpy: host arrays play the device buffers
        calls.append(kind)
        ctypes.memmove(d, s, nb)
        return 0
    fn = oracle.COPY_FN(copy)
    t = oracle.host_bounce_time(oracle.OPS["sum"], oracle.DTYPES["int32"], n, me, npes, key,
                                src.ctypes.data, dst.ctypes.data, reps=2, copy_fn=fn)
    q.put((me, t, dst, calls.count(2), calls.count(1)))


@pytest.mark.parametrize("npes", [1, 3])
def test_host_bounce_restatement_reduces_through_64KiB_device_copies(npes):
    # oracle_host_bounce_time (the CPU baseline with the reference's synchronous 64 KiB copies,
    # reduce_impl.h:186-228): every member ends with the rank-order fold, and makes exactly one
    # device->host and one host->device copy per chunk and repetition.
    import multiprocessing as mp
    import uuid
    n = 100_003
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    key = f"tb{uuid.uuid4().hex[:8]}"
    ps = [ctx.Process(target=_bounce_member, args=(me, npes, key, n, q)) for me in range(npes)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(npes)]
    for p in ps:
        p.join(timeout=30)
    srcs = [oracle.fill_random(oracle.DTYPES["int32"], 0xB0 + j, n) for j in range(npes)]
    want = oracle.reduce_fold(oracle.OPS["sum"], oracle.DTYPES["int32"], srcs, 0)
    chunks = -(-n * 4 // oracle.REDUCE_BUFFER_SIZE)
    for me, t, dst, d2h, h2d in res:
        assert t > 0
        assert np.array_equal(dst, want), f"member {me}"
        assert d2h == 2 * chunks and h2d == 2 * chunks
