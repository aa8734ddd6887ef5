"""ORACLE — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg): one extra member of the
reference host-path timing (oracle_host_bounce_time) in a process of its own, on its own HIP
allocations, so a one-GPU box can time the p-member host path side by side.

  python -m oracle.bounce_helper --me K --npes P --key KEY --n N [--dtype 8] [--op 5] [--reps 1]

Prints this member's best seconds.  The device is only the source / dest of the copies; nothing
of the product library is loaded.
"""
from __future__ import annotations

import argparse
import ctypes
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import oracle  # noqa: E402


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--me", type=int, required=True)
    ap.add_argument("--npes", type=int, required=True)
    ap.add_argument("--key", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--dtype", type=int, default=oracle.DTYPES["float"])
    ap.add_argument("--op", type=int, default=oracle.OPS["sum"])
    ap.add_argument("--reps", type=int, default=1)
    a = ap.parse_args()
    hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
    nbytes = a.n * oracle.NP[a.dtype]().itemsize
    src, dst = ctypes.c_void_p(), ctypes.c_void_p()
    if hip.hipMalloc(ctypes.byref(src), ctypes.c_size_t(nbytes)) or \
            hip.hipMalloc(ctypes.byref(dst), ctypes.c_size_t(nbytes)):
        print("hipMalloc failed", file=sys.stderr)
        return 1
    hip.hipMemset(src, ctypes.c_int(0), ctypes.c_size_t(nbytes))
    t = oracle.host_bounce_time(a.op, a.dtype, a.n, a.me, a.npes, a.key, src.value, dst.value, a.reps)
    print(f"{t:.6f}")
    hip.hipFree(src)
    hip.hipFree(dst)
    return 0


if __name__ == "__main__":
    sys.exit(main())
