"""GPU parity of the single-GPU pieces of the path, through the C-ABI:
  * the local combine unit dst = op(src_0..src_{k-1}) for every valid (op, dtype), ragged sizes
    and misaligned operands, bit-exact against the oracle's fold (same left-to-right order);
  * the 1-PE reduce (reference semantics: dest = source, reduce_impl.h:288-289) on heap, device
    and host buffers, in place and via the stream API;
  * the 1 GiB f32 combine (BASELINE config 2) compared in full.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

VALID = [(op, dt) for op in range(7) for dt in range(10) if oracle.valid(op, dt)]
ONAMES = {v: k for k, v in oracle.OPS.items()}
DNAMES = {v: k for k, v in oracle.DTYPES.items()}


@pytest.fixture(scope="module")
def ish():
    import ishmem_amd
    ishmem_amd.init(0, 1, 0, None)
    yield ishmem_amd
    ishmem_amd.ishmem_finalize()


def _bits_equal(a, b):
    return np.array_equal(np.ascontiguousarray(a).view(np.uint8), np.ascontiguousarray(b).view(np.uint8))


@pytest.mark.parametrize("op,dt", VALID)
def test_combine_parity_all_ops_types(ish, op, dt):
    from ishmem_amd import hip
    es = np.dtype(oracle.NP[dt]).itemsize
    lo, hi = (0.5, 2.0) if op == oracle.OPS["prod"] else (-1.0, 1.0)
    for k, n in [(1, 1000), (2, 1), (2, 17), (3, 4097), (8, 33333), (16, 1000)]:
        srcs = [oracle.fill_random(dt, 31 * j + n, n, lo, hi) for j in range(k)]
        dptrs = [hip.malloc(n * es) for _ in range(k)]
        for p, s in zip(dptrs, srcs):
            hip.upload(p, s)
        dst = hip.malloc(n * es)
        assert ish.combine(ONAMES[op], DNAMES[dt], dst, dptrs, n) == 0, ish.last_error()
        hip.synchronize()
        got = hip.download(dst, n, oracle.NP[dt])
        ref = oracle.reduce_fold(op, dt, srcs, 0)
        assert _bits_equal(got, ref), (op, dt, k, n)
        for p in dptrs + [dst]:
            hip.free(p)


@pytest.mark.parametrize("dt", [0, 1, 2, 3, 8, 9])
def test_combine_misaligned_operands(ish, dt):
    from ishmem_amd import hip
    es = np.dtype(oracle.NP[dt]).itemsize
    op = oracle.OPS["sum"]
    base = [hip.malloc(4096) for _ in range(3)]
    for n in (1, 3, 16, 41, 200):
        for offs in [(0, 0, 0), (es, es, es), (0, es, 2 * es), (3 * es, 0, 3 * es), (8, 8, 8)]:
            offs = [o - (o % es) for o in offs]
            srcs = [oracle.fill_random(dt, n + i, n) for i in range(2)]
            hip.upload(base[0] + offs[0], srcs[0])
            hip.upload(base[1] + offs[1], srcs[1])
            assert ish.combine("sum", DNAMES[dt], base[2] + offs[2], [base[0] + offs[0], base[1] + offs[1]], n) == 0
            hip.synchronize()
            got = hip.download(base[2] + offs[2], n, oracle.NP[dt])
            assert _bits_equal(got, oracle.reduce_fold(op, dt, srcs, 0)), (dt, n, offs)
    for p in base:
        hip.free(p)


@pytest.mark.parametrize("dt", [0, 2, 3, 8, 9])
def test_combine_realigned_operands(ish, dt):
    # Sources whose addresses differ from dest's mod 16 take the realigned kernel from 1 KiB
    # (fanin_realign_kernel: aligned loads, a DPP wave shift + LDS edges and a funnel shift per source).
    # Every element-aligned shift of dest and of each source, ragged sizes; bit-exact against the
    # oracle's fold, and the bytes around dest untouched.
    from ishmem_amd import hip
    es = np.dtype(oracle.NP[dt]).itemsize
    op = oracle.OPS["sum"]
    offs_all = list(range(0, 16, es))
    n_max = 70_001
    pad = 64
    base = [hip.malloc(n_max * es + 2 * pad) for _ in range(3)]
    rng = np.random.default_rng(dt)
    # 1024 // es (+1): the realigned kernel's 1 KiB entry point, where the 256-B head peel leaves a
    # short body and a ragged tail; 8 KiB +- a few: one 512-thread workgroup's span.
    for n in (256 // es + 3, 1024 // es, 1024 // es + 1, 8192 // es - 3, 8192 // es + 21, 4099, n_max):
        for _ in range(6):
            o = [int(rng.choice(offs_all)) for _ in range(3)]
            srcs = [oracle.fill_random(dt, n + 7 * i + o[i], n) for i in range(2)]
            hip.upload(base[0] + pad + o[0], srcs[0])
            hip.upload(base[1] + pad + o[1], srcs[1])
            hip.memset(base[2], 0xA5, n_max * es + 2 * pad)
            assert ish.combine("sum", DNAMES[dt], base[2] + pad + o[2],
                               [base[0] + pad + o[0], base[1] + pad + o[1]], n) == 0, ish.last_error()
            hip.synchronize()
            got = hip.download(base[2] + pad + o[2], n, oracle.NP[dt])
            assert _bits_equal(got, oracle.reduce_fold(op, dt, srcs, 0)), (dt, n, o)
            raw = hip.download(base[2], n_max * es + 2 * pad, np.uint8)
            lo, hi = pad + o[2], pad + o[2] + n * es
            assert (raw[:lo] == 0xA5).all() and (raw[hi:] == 0xA5).all(), (dt, n, o)
    for p in base:
        hip.free(p)


@pytest.mark.parametrize("dtype,es", [("uint8", 1), ("float", 4), ("double", 8)])
def test_single_pe_reduce_realigned_copy(ish, dtype, es):
    # The 1-PE reduce is a copy (reduce_impl.h:288-289); with source and dest on different 16-B
    # phases it is a byte copy through the realigned kernel.  Every (dest, source) phase pair of
    # the element size at two ragged sizes, the bytes around dest untouched.
    from ishmem_amd import hip
    npd = {"uint8": np.uint8, "float": np.float32, "double": np.float64}[dtype]  # np.dtype("float") is f64
    pad = 64
    for n in (1024 // es, 1024 // es + 5, 8192 // es + 1, 300_007):
        nb = n * es + 2 * pad
        s_buf, d_buf = ish.ishmem_malloc(nb), ish.ishmem_malloc(nb)
        x = np.random.default_rng(n).integers(0, 256, n * es, dtype=np.uint8).view(npd)
        for so in range(0, 16, es):
            for do in range(0, 16, es):
                if (so - do) % 16 == 0 and so != 0:
                    continue  # same phase: the vector path, covered elsewhere
                hip.upload(s_buf + pad + so, x)
                hip.memset(d_buf, 0x5A, nb)
                assert ish.reduce_on_stream("sum" if dtype != "uint8" else "or", dtype, d_buf + pad + do,
                                            s_buf + pad + so, n, None, 0) == 0, ish.last_error()
                hip.synchronize()
                raw = hip.download(d_buf, nb, np.uint8)
                got = raw[pad + do: pad + do + n * es]
                assert np.array_equal(got, x.view(np.uint8)), (dtype, n, so, do)
                assert (raw[:pad + do] == 0x5A).all() and (raw[pad + do + n * es:] == 0x5A).all(), (so, do)
        ish.ishmem_free(d_buf)
        ish.ishmem_free(s_buf)


def test_single_pe_reduce_is_copy(ish):
    from ishmem_amd import hip
    n = 1_000_003
    x = oracle.fill_random(oracle.DTYPES["float"], 3, n)
    s = ish.ishmem_malloc(n * 4)
    d = ish.ishmem_malloc(n * 4)
    hip.upload(s, x)
    assert ish.ishmem_float_sum_reduce(d, s, n) == 0
    assert _bits_equal(hip.download(d, n, np.float32), x)
    assert ish.ishmem_float_prod_reduce(s, s, n) == 0  # in place: unchanged
    assert _bits_equal(hip.download(s, n, np.float32), x)
    # host memory on one PE (reference: runtime allreduce on host pointers, reduce_impl.h:301-315)
    out = np.zeros(n, np.float32)
    assert ish.ishmem_float_max_reduce(out.ctypes.data, x.ctypes.data, n) == 0
    assert _bits_equal(out, x)
    # the stream variant writes *ret = 0
    ret = ish.ishmem_malloc(4)
    hip.memset(ret, 0xFF, 4)
    st = hip.stream_create()
    assert ish.ishmemx_float_sum_reduce_on_stream(d, s, n, ret, st) == 0
    hip.stream_synchronize(st)
    assert int(hip.download(ret, 1, np.int32)[0]) == 0
    hip.stream_destroy(st)
    for p in (ret, d, s):
        ish.ishmem_free(p)


def test_invalid_pairs_fail_cleanly(ish):
    s = ish.ishmem_malloc(64)
    assert ish.reduce("and", "float", s, s, 4) != 0
    assert "invalid" in ish.last_error()
    assert ish.lib().ishmemi_c_reduce(99, 5, 8, s, s, 4) != 0
    ish.ishmem_free(s)


def test_combine_1GiB_f32_sum_full_compare(ish):
    from ishmem_amd import hip
    n = 1 << 28  # 1 GiB of float32 (BASELINE config 2)
    a = oracle.fill_random(oracle.DTYPES["float"], 11, n)
    b = oracle.fill_random(oracle.DTYPES["float"], 12, n)
    pa, pb, pd = hip.malloc(n * 4), hip.malloc(n * 4), hip.malloc(n * 4)
    hip.upload(pa, a)
    hip.upload(pb, b)
    assert ish.combine("sum", "float", pd, [pa, pb], n) == 0
    hip.synchronize()
    got = hip.download(pd, n, np.float32)
    assert _bits_equal(got, a + b)
    # self-reduce (copy) at the same size
    s = ish.ishmem_malloc(n * 4)
    d = ish.ishmem_malloc(n * 4)
    hip.memcpy(s, pa, n * 4)
    assert ish.ishmem_float_sum_reduce(d, s, n) == 0
    assert _bits_equal(hip.download(d, n, np.float32), a)
    for p in (pa, pb, pd):
        hip.free(p)
    ish.ishmem_free(d)
    ish.ishmem_free(s)


def test_on_stream_deps_and_done_event(ish):
    """ishmemx_*_reduce_on_queue's `deps` and returned event (reduce_impl.h:445-472) as HIP events:
    the producer of the source is a copy on ANOTHER stream, queued behind a 100 ms kernel; the
    reduce on its own stream must wait for it (deps) and `done` must follow the reduce."""
    from ishmem_amd import hip
    n = 4 << 20
    x = oracle.fill_random(oracle.DTYPES["float"], 21, n)
    hx = hip.host_malloc(n * 4)
    np.ctypeslib.as_array((np.ctypeslib.ctypes.c_float * n).from_address(hx))[:] = x
    s, d, ret = ish.ishmem_malloc(n * 4), ish.ishmem_malloc(n * 4), ish.ishmem_malloc(4)
    hip.memset(s, 0, n * 4)
    hip.memset(d, 0xFF, n * 4)
    hip.memset(ret, 0xFF, 4)
    sa, sb = hip.stream_create(), hip.stream_create()
    produced, done = hip.Event(), hip.Event()
    assert ish.occupy(4, 100_000, sa) == 0
    hip.memcpy_async(s, hx, n * 4, sa)
    produced.record(sa)
    assert ish.reduce_on_stream("sum", "float", d, s, n, ret, sb, deps=[produced], done=done) == 0, ish.last_error()
    done.synchronize()
    assert _bits_equal(hip.download(d, n, np.float32), x)  # 1 PE: dest = the produced source
    assert int(hip.download(ret, 1, np.int32)[0]) == 0
    # `done` alone (no deps), and the NULL-deps error
    hip.memset(d, 0, n * 4)
    assert ish.reduce_on_stream("max", "float", d, s, n, None, sb, done=done) == 0
    done.synchronize()
    assert _bits_equal(hip.download(d, n, np.float32), x)
    assert ish.lib().ishmemi_c_reduce_on_stream_deps(0, 4, 8, d, s, n, None, sb, None, 2, None) != 0
    assert "deps" in ish.last_error()
    hip.stream_synchronize(sa)
    for st in (sa, sb):
        hip.stream_destroy(st)
    for p in (ret, d, s):
        ish.ishmem_free(p)
    hip.host_free(hx)


@pytest.mark.parametrize("npd", [np.int32, np.float64])
def test_device_pattern_checker_counts_wrong_bytes(ish, npd):
    """Negative control of the device checker that compares configs[2..4] in every word
    (tests/cpp/pattern_check.hip via selfcheck.count_wrong): a dest holding the expected fold
    counts 0 wrong bytes, and exactly the bytes corrupted afterwards are counted — also past 2^32
    elements of index (the hash's high word) — and the device's answer equals the host check."""
    from ishmem_amd import hip, selfcheck as sc
    assert sc.checker_kind(npd) == "device"
    es = np.dtype(npd).itemsize
    n = 3_000_001
    d = ish.ishmem_malloc(n * es)
    try:
        for lo in (0, (1 << 32) - 1000):
            # d holds elements lo .. lo + n of the array, so the array itself starts lo elements
            # before d (count_wrong checks [lo, lo + m) of the array at `base`).
            base = d - lo * es
            # p = 1: the fold of one member is its own pattern (sum / min / max / prod alike)
            if lo == 0:
                sc.upload_pattern(hip, d, npd, 0, 1, n)
            else:
                hip.upload(d, sc.pattern(0, 1, lo, n, npd))
            for op in ("sum", "min", "max", "prod"):
                assert sc.count_wrong(hip, base, op, npd, 1, lo, n) == 0, (op, lo)
            assert sc.count_wrong(hip, base, "sum", npd, 2, lo, n) > 0  # another team size: wrong
            hip.memset(d + 5 * es + 1, 0xEE, 3)  # three bytes of element 5
            hip.memset(d + (n - 1) * es, 0x00, 1)  # the last element's first byte
            dev = sc.count_wrong(hip, base, "max", npd, 1, lo, n)
            host = sc.count_wrong(hip, base, "max", npd, 1, lo, n, device=False)
            assert dev == host and 3 <= dev <= 4, (dev, host)
    finally:
        ish.ishmem_free(d)


@pytest.mark.parametrize("dt", [0, 2, 9])
def test_realigned_kernels_grid_stride_loop(ish, dt):
    """The realigned fan-in's grid-stride loop (with the LDS edge slots reused between passes)
    otherwise runs only past 2^31 items; set_param("realign_grid_cap") caps its grid at 1 / 3 / 7
    workgroups so every workgroup makes several passes.  Copy and a + b, sources on other 16-B
    phases than dest, bit-exact against the oracle, bytes around dest untouched."""
    from ishmem_amd import hip
    es = np.dtype(oracle.NP[dt]).itemsize
    n = (8192 * 9 + 4099) // es + 3
    pad = 64
    base = [hip.malloc(n * es + 2 * pad) for _ in range(3)]
    try:
        for cap in (1, 3, 7):
            assert ish.set_param("realign_grid_cap", cap) == 0
            for o in ((es, 0, 2 * es % 16), (0, 3 * es % 16, es)):
                srcs = [oracle.fill_random(dt, 100 * cap + 7 * i + o[i], n) for i in range(2)]
                for i in range(2):
                    hip.upload(base[i] + pad + o[i], srcs[i])
                for k in (1, 2):
                    hip.memset(base[2], 0xA5, n * es + 2 * pad)
                    assert ish.combine("sum" if dt != 0 else "or", DNAMES[dt], base[2] + pad + o[2],
                                       [base[i] + pad + o[i] for i in range(k)], n) == 0, ish.last_error()
                    hip.synchronize()
                    got = hip.download(base[2] + pad + o[2], n, oracle.NP[dt])
                    op = oracle.OPS["sum"] if dt != 0 else oracle.OPS["or"]
                    assert _bits_equal(got, oracle.reduce_fold(op, dt, srcs[:k], 0)), (dt, cap, o, k)
                    raw = hip.download(base[2], n * es + 2 * pad, np.uint8)
                    lo, hi = pad + o[2], pad + o[2] + n * es
                    assert (raw[:lo] == 0xA5).all() and (raw[hi:] == 0xA5).all(), (dt, cap, o, k)
    finally:
        ish.set_param("realign_grid_cap", 0)
        for b in base:
            hip.free(b)
