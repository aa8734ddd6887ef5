"""Path thresholds by team topology (CPU, no GPU).

ishmemi_c_path_limits(p, colocated) returns the two thresholds that pick a multi-PE reduce's path
below the phased one (runtime.cpp path_limits): the granule path's (ll) and the whole-array fold's
(fold).  Co-located teams (every member on one GPU) keep round 5's measured crossovers; teams
whose members sit on different GPUs take them from the link-byte model, restated here:
    t_ll(B)   = a_ll(p)   + 1 hop  + 2B / L
    t_fold(B) = a_fold(p) + 2 hops + B / L
    t_rsag(B) = a_rsag(p) + 3 hops + 2B / (p L)
The share parameter follows the bench's vocabulary: share = p PEs per GPU (co-located), share = 1
(one PE per GPU).
"""
import ctypes
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
KIB = 1 << 10
LL_DEFAULT, ONESHOT_P2 = 512 * KIB, 32 << 20
UNLIMITED = (1 << 63) - 1
L = 76.8e9  # bytes/s per link and direction
HOP = 1.0


def ll_capacity(p):
    return ((8 << 20) // 8 // (2 * p) & ~127) * 4


def model(p):
    ll = (4.5 + 0.5 * (p - 2) + HOP, 2e6 / L)
    fold = (9.0 + 0.75 * (p - 2) + 2 * HOP, 1e6 / L)
    rsag = (9.5 + 2.5 * (p - 2) + 3 * HOP, 2e6 / (p * L))
    return ll, fold, rsag


def crossover(f, g):
    if f[0] > g[0]:
        return 0
    if f[1] <= g[1]:
        return UNLIMITED
    return int((g[0] - f[0]) / (f[1] - g[1]))


def expected(p, colocated, direct_max_pes=4):
    cap = min(LL_DEFAULT, ll_capacity(p))
    fold_team = p <= direct_max_pes
    if colocated:
        ll = min(cap, (768 * KIB) // p) if p >= 3 and fold_team else cap
        fold = ONESHOT_P2 if p == 2 else ONESHOT_P2 // 4 // (p - 1)
    else:
        mll, mfold, mrsag = model(p)
        ll = crossover(mll, mrsag)
        if fold_team:
            ll = min(ll, crossover(mll, mfold))
        ll = min(cap, ll)
        fold = crossover(mfold, mrsag)
    return ll, fold if fold_team else 0


def limits(L_, p, colocated):
    ll, fold = ctypes.c_longlong(-7), ctypes.c_longlong(-7)
    assert L_.ishmemi_c_path_limits(p, int(colocated), ctypes.byref(ll), ctypes.byref(fold)) == 0
    return ll.value, fold.value


@pytest.fixture(scope="module")
def lib():
    from ishmem_amd import _lib
    return _lib.load(build_if_missing=False)


@pytest.mark.parametrize("p", [2, 3, 4, 8])
@pytest.mark.parametrize("share", ["1", "p"])
def test_path_limits_by_team_size_and_device_share(lib, p, share):
    colocated = share == "p"
    got = limits(lib, p, colocated)
    assert got == expected(p, colocated), (p, share, got, expected(p, colocated))


def test_cross_device_limits_follow_the_link_bytes(lib):
    # The granules move 2 link bytes per payload byte: across GPUs the granule path stops earlier
    # than co-located at 2 PEs; the fold pulls (p - 1) B per member against 2(p - 1)/p B, so across
    # GPUs its bound shrinks at 3-4 members, while at 2 the link bytes tie and the fold (one barrier
    # and one grid fewer) wins at every size.
    assert limits(lib, 2, False)[0] < limits(lib, 2, True)[0]
    assert limits(lib, 2, False)[1] == UNLIMITED
    for p in (3, 4):
        assert 0 < limits(lib, p, False)[1] < limits(lib, p, True)[1]
    for p in (2, 3, 4, 8):
        assert 0 < limits(lib, p, False)[0] <= ll_capacity(p)
    assert limits(lib, 8, False)[1] == 0 and limits(lib, 8, True)[1] == 0  # > direct_max_pes: no fold


OVERRIDE_PROBE = r'''
import ctypes, sys
sys.path.insert(0, sys.argv[1])
from ishmem_amd import _lib
L = _lib.load(build_if_missing=False)
L.ishmemi_c_init_pe(0, 1, 0, b"pathprobe")  # fails without a GPU, after the variables are read
ll, fold = ctypes.c_longlong(), ctypes.c_longlong()
out = []
for p in (2, 4):
    for c in (0, 1):
        L.ishmemi_c_path_limits(p, c, ctypes.byref(ll), ctypes.byref(fold))
        out.append(f"{p}{c}:{ll.value},{fold.value}")
print(" ".join(out))
'''


def test_xgmi_overrides_apply_to_cross_device_teams_only():
    """ISHMEM_XGMI_LL_MAX_BYTES / ISHMEM_XGMI_FOLD_MAX_BYTES (e.g. the node run's `recommended`
    crossovers) replace the model's values for teams across GPUs; co-located teams keep theirs."""
    import os
    env = {k: v for k, v in os.environ.items() if not k.startswith("ISHMEM_")}
    env.update(ISHMEM_XGMI_LL_MAX_BYTES="64K", ISHMEM_XGMI_FOLD_MAX_BYTES="1M")
    out = subprocess.run([sys.executable, "-c", OVERRIDE_PROBE, str(ROOT)], env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = dict(kv.split(":") for kv in out.stdout.split())
    assert got["20"] == f"{64 * KIB},{1 << 20}" and got["40"] == f"{64 * KIB},{1 << 20}"
    assert got["21"] == "%d,%d" % expected(2, True) and got["41"] == "%d,%d" % expected(4, True)
