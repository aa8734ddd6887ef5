"""CPU tests of the large-size parity checker (ishmem_amd/selfcheck.py: rotating-winner pattern).

At BASELINE's sizes (1 GiB .. 4 GiB per PE, up to 8 PEs) the GPU tests and bench.py cannot fold p
full arrays through the oracle, so they compare dest with a closed form.  These tests pin that
closed form to an explicit team-order fold and show that it catches the routing faults a periodic
input hides: a swapped 16 KiB tile / reduce-scatter segment, a member skipped or counted twice, a
truncated 64-bit tile base (4 GiB alias)."""
import numpy as np
import pytest

from ishmem_amd import selfcheck as sc

TILE_BYTES = 16 << 10  # kernels.h: kBlock 256 x kUnroll 4 x 16 B, the RS / AG unit


def fold(op, npd, xs):
    acc = xs[0].copy()
    with np.errstate(over="ignore"):
        for x in xs[1:]:
            if op == "sum":
                acc = (acc + x).astype(npd)
            elif op == "prod":
                acc = (acc * x).astype(npd)
            elif op == "min":
                acc = np.minimum(acc, x)
            else:
                acc = np.maximum(acc, x)
    return acc


def old_closed_form_inputs(p, lo, m, npd):
    """Round 2's x_pe[i] = (i mod 1024) + pe (kept here only to show what it missed)."""
    i = np.arange(lo, lo + m, dtype=np.int64)
    return [((i % 1024) + pe).astype(npd) for pe in range(p)]


@pytest.mark.parametrize("op,npd", [("sum", np.float32), ("sum", np.int32), ("sum", np.float64),
                                    ("min", np.int32), ("max", np.float64), ("prod", np.int32),
                                    ("prod", np.float64)])
@pytest.mark.parametrize("p", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("lo,m", [(0, 5000), ((1 << 32) - 1000, 3000), (12_345_678_901, 777)])
def test_expected_equals_team_order_fold(op, npd, p, lo, m):
    xs = [sc.pattern(pe, p, lo, m, npd) for pe in range(p)]
    want = fold(op, npd, xs)
    got = sc.pattern_expected(op, npd, p, lo, m)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_pattern_is_blockwise_consistent_and_non_periodic():
    # Any split of the range gives the same values (chunked uploads / checks).
    a = sc.pattern(2, 8, (1 << 32) - 10, (1 << 20) + 20, np.int32)
    b = np.concatenate([sc.pattern(2, 8, (1 << 32) - 10, 10, np.int32),
                        sc.pattern(2, 8, 1 << 32, (1 << 20) + 10, np.int32)])
    assert np.array_equal(a, b)
    # No two 16 KiB tiles of an f32 array are equal; every PE's value differs at every index.
    n = 64 * TILE_BYTES // 4
    x = sc.pattern(0, 8, 0, n, np.float32).reshape(64, -1)
    assert len({row.tobytes() for row in x}) == 64
    xs = np.stack([sc.pattern(pe, 8, 0, 4096, np.int32) for pe in range(8)])
    assert all(len(set(xs[:, i])) == 8 for i in range(4096))
    # The min / max winner rotates over every PE.
    assert set(np.argmin(xs, axis=0)) == set(range(8)) == set(np.argmax(xs, axis=0))


@pytest.mark.parametrize("p", [2, 8])
def test_checker_catches_swapped_tile(p):
    # An all-gather that pulls segment s' instead of s (or an RS that stores into the wrong
    # segment): the result's tiles 3 and 5 swapped.
    n = 8 * TILE_BYTES // 4
    good = sc.pattern_expected("sum", np.float32, p, 0, n)
    bad = good.copy().reshape(8, -1)
    bad[[3, 5]] = bad[[5, 3]]
    assert np.count_nonzero(bad.ravel() != good) > 0
    # Round 2's periodic input could not see it: every tile of its result is identical.
    old = fold("sum", np.float32, old_closed_form_inputs(p, 0, n, np.float32)).reshape(8, -1)
    old_bad = old.copy()
    old_bad[[3, 5]] = old_bad[[5, 3]]
    assert np.array_equal(old, old_bad)


@pytest.mark.parametrize("op", ["min", "max", "sum"])
def test_checker_catches_skipped_or_duplicated_member(op):
    p, n = 8, 10_000
    xs = [sc.pattern(pe, p, 0, n, np.float64) for pe in range(p)]
    want = sc.pattern_expected(op, np.float64, p, 0, n)
    skipped = fold(op, np.float64, [xs[0], xs[-1]])                 # members 1..p-2 skipped
    dup = fold(op, np.float64, [xs[0]] + [xs[0]] + xs[2:])          # member 0 twice, 1 missing
    assert np.count_nonzero(skipped != want) > n // 2
    if op == "sum":
        assert np.all(dup != want)
    olds = old_closed_form_inputs(p, 0, n, np.float64)
    if op in ("min", "max"):  # old form: min always PE 0's, max PE p-1's -> a skip passed
        assert np.array_equal(fold(op, np.float64, [olds[0], olds[-1]]), fold(op, np.float64, olds))


def test_checker_catches_truncated_64bit_tile_base():
    # A 32-bit byte offset: element i + 2^30 (4 GiB of f32 further on) read from element i.
    p, m = 8, 4096
    hi = sc.pattern_expected("sum", np.float32, p, 1 << 30, m)
    lo = sc.pattern_expected("sum", np.float32, p, 0, m)
    assert np.count_nonzero(hi != lo) > m // 2


NPD_CODES = {np.int32: 2, np.int64: 3, np.uint32: 6, np.uint64: 7, np.float32: 8, np.float64: 9}


@pytest.fixture(scope="module")
def checker():
    from tests.test_gpu_cpp import build_pattern_check
    build_pattern_check()
    sc._checker = None
    lib = sc.device_checker()
    assert lib is not None
    return lib


@pytest.mark.parametrize("npd", [np.int32, np.uint32, np.int64, np.float32, np.float64])
@pytest.mark.parametrize("p", [1, 2, 3, 8])
@pytest.mark.parametrize("lo,m", [(0, 3000), ((1 << 32) - 700, 1500), (12_345_678_901, 777)])
def test_device_checker_host_twins_equal_numpy(checker, npd, p, lo, m):
    """The device checker's pattern and expected fold (tests/cpp/pattern_check.hip, compiled for the
    host as well) equal selfcheck's numpy, which test_expected_equals_team_order_fold pins to an
    explicit fold.  int64 products: the true wrap mod 2^64 (selfcheck's numpy only serves 32-bit
    integer products, the configs[4] dtypes), checked against an explicit int64 fold."""
    import ctypes
    code = NPD_CODES[npd]
    for pe in range(p):
        got = np.empty(m, npd)
        assert checker.pc_host_pattern(got.ctypes.data_as(ctypes.c_void_p), code, pe, p, lo, m) == 0
        assert np.array_equal(got, sc.pattern(pe, p, lo, m, npd))
    for op, opc in (("sum", 5), ("min", 4), ("max", 3), ("prod", 6)):
        got = np.empty(m, npd)
        assert checker.pc_host_expected(got.ctypes.data_as(ctypes.c_void_p), opc, code, p, lo, m) == 0
        if op == "prod" and np.dtype(npd).itemsize == 8 and np.issubdtype(npd, np.integer):
            want = fold(op, npd, [sc.pattern(pe, p, lo, m, npd) for pe in range(p)])
        else:
            want = sc.pattern_expected(op, npd, p, lo, m)
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (op, npd, p, lo)
