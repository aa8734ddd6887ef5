#!/usr/bin/env python3
"""Does device memory come back after a team block's life cycle (round 6, the team-churn test saw
~8 MiB per split team and PE stay allocated)?  Raw HIP through ctypes, no library: each case runs
ROUNDS cycles on 8.25 MiB blocks and reports the drop in hipMemGetInfo's free bytes.
  alloc_free        - hipExtMallocWithFlags(uncached) + hipFree
  export_free       - the same with hipIpcGetMemHandle before the free
  export_import     - process A allocates and exports, process B opens and closes the handle, A frees
                      (the order of a team destroy: every member closes the others' blocks, frees its own)
  export_import_late - as export_import, but B closes only after A has freed
One JSON line per case.

  python tools/ipc_leak_probe.py [rounds]
"""
from __future__ import annotations

import ctypes
import json
import multiprocessing as mp
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
BYTES = 8_651_008
UNCACHED = 0x3


class Handle(ctypes.Structure):  # hipIpcMemHandle_t, passed by value to hipIpcOpenMemHandle
    _fields_ = [("reserved", ctypes.c_char * 64)]


def hip():
    from ishmem_amd import hip as h
    return h.lib()


def free_bytes(L) -> int:
    f, t = ctypes.c_size_t(), ctypes.c_size_t()
    assert L.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)) == 0
    return f.value


def alloc(L) -> ctypes.c_void_p:
    p = ctypes.c_void_p()
    assert L.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(BYTES), ctypes.c_uint(UNCACHED)) == 0
    return p


def single(case: str, rounds: int, q) -> None:
    L = hip()
    L.hipSetDevice(0)
    L.hipDeviceSynchronize()
    f0 = free_bytes(L)
    for _ in range(rounds):
        p = alloc(L)
        if case == "export_free":
            h = Handle()
            assert L.hipIpcGetMemHandle(ctypes.byref(h), p) == 0
        assert L.hipFree(p) == 0
    L.hipDeviceSynchronize()
    q.put({"case": case, "rounds": rounds, "drop_MiB": (f0 - free_bytes(L)) / 2**20})


def exporter(rounds: int, late: bool, conn, q) -> None:
    libc = ctypes.CDLL(None)
    libc.prctl(0x59616d61, ctypes.c_ulong(-1 & 0xFFFFFFFFFFFFFFFF), 0, 0, 0)  # PR_SET_PTRACER_ANY
    L = hip()
    L.hipSetDevice(0)
    f0 = free_bytes(L)
    for _ in range(rounds):
        p = alloc(L)
        h = Handle()
        assert L.hipIpcGetMemHandle(ctypes.byref(h), p) == 0
        conn.send(bytes(h))
        if not late:
            assert conn.recv() == "closed"
        assert L.hipFree(p) == 0
        if late:
            conn.send("freed")
            assert conn.recv() == "closed"
    L.hipDeviceSynchronize()
    q.put({"side": "exporter", "drop_MiB": (f0 - free_bytes(L)) / 2**20})


def importer(rounds: int, late: bool, conn, q) -> None:
    L = hip()
    L.hipSetDevice(0)
    for _ in range(rounds):
        hb = conn.recv()
        h = Handle.from_buffer_copy(hb)
        p = ctypes.c_void_p()
        L.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), Handle, ctypes.c_uint]
        rc = L.hipIpcOpenMemHandle(ctypes.byref(p), h, ctypes.c_uint(1))
        if rc != 0:
            q.put({"side": "importer", "error": f"hipIpcOpenMemHandle rc={rc}"})
            return
        if late:
            assert conn.recv() == "freed"
        assert L.hipIpcCloseMemHandle(p) == 0
        conn.send("closed")
    L.hipDeviceSynchronize()
    q.put({"side": "importer", "ok": True})


def pair(case: str, rounds: int) -> dict:
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    a, b = ctx.Pipe()
    late = case == "export_import_late"
    pa = ctx.Process(target=exporter, args=(rounds, late, a, q))
    pb = ctx.Process(target=importer, args=(rounds, late, b, q))
    pa.start()
    pb.start()
    got = [q.get(timeout=120), q.get(timeout=120)]
    pa.join(30)
    pb.join(30)
    L = hip()
    L.hipSetDevice(0)
    out = {"case": case, "rounds": rounds}
    for g in got:
        out.update({f"{g['side']}_{k}": v for k, v in g.items() if k != "side"})
    return out


def main() -> int:
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    ctx = mp.get_context("spawn")
    for case in ("alloc_free", "export_free"):
        q = ctx.Queue()
        p = ctx.Process(target=single, args=(case, rounds, q))
        p.start()
        print(json.dumps(q.get(timeout=120)), flush=True)
        p.join(30)
    for case in ("export_import", "export_import_late"):
        print(json.dumps(pair(case, rounds)), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
