"""CPU multi-process tests of the N>1 host logic (no GPU needed).

* The native node-local bootstrap (ishmem_amd/csrc/bootstrap.cpp — replaces the MPI/PMI runtime's
  role of exchanging heap IPC handles, src/ipc.cpp:123-233) with 2 and 4 processes.
* torch.distributed `gloo`, world size 2: the key exchange bench.py uses (rank 0 draws the key,
  broadcast), then the native bootstrap keyed by it, then the multi-PE RS + AG schedule executed
  on the CPU with the library's own partition (ishmemi_c_chunk_bounds) and gloo all_gather —
  every rank's result must equal the oracle's canonical fold.
"""
import ctypes
import multiprocessing as mp
import os
import socket
import uuid

import numpy as np
import pytest


def _selftest(pe, npes, key, q):
    import ishmem_amd as ish
    out = (ctypes.c_int * npes)()
    r = ish.lib().ishmemi_c_bootstrap_selftest(pe, npes, key.encode(), 10 * pe + 1, out)
    q.put((pe, r, list(out), ish.last_error()))


@pytest.mark.parametrize("npes", [2, 4])
def test_native_bootstrap_allgather(npes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    key = f"cpu{uuid.uuid4().hex[:10]}"
    ps = [ctx.Process(target=_selftest, args=(pe, npes, key, q)) for pe in range(npes)]
    for p in ps:
        p.start()
    res = [q.get(timeout=60) for _ in range(npes)]
    for p in ps:
        p.join(timeout=30)
    for pe, r, out, err in res:
        assert r == 0, err
        assert out == [10 * j + 1 for j in range(npes)]
    assert not any(f.startswith("ishmem_amd_" + key) for f in os.listdir("/dev/shm"))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world))
        import torch
        import torch.distributed as dist

        import ishmem_amd as ish
        import oracle
        dist.init_process_group("gloo", rank=rank, world_size=world)
        obj = [f"gloo{uuid.uuid4().hex[:10]}"]
        dist.broadcast_object_list(obj, src=0)  # the bench.py key exchange
        out = (ctypes.c_int * world)()
        r = ish.lib().ishmemi_c_bootstrap_selftest(rank, world, obj[0].encode(), rank + 7, out)
        assert r == 0, ish.last_error()
        assert list(out) == [j + 7 for j in range(world)]

        # RS + AG schedule of allreduce_kernel on the CPU with the library's partition.
        dt, op = oracle.DTYPES["float"], oracle.OPS["sum"]
        n = 10_007
        mine = oracle.fill_random(dt, 0x15AE0001 + rank, n)
        nvec = n // 4  # 16-B vectors of float32
        srcs = [torch.zeros(n, dtype=torch.float32) for _ in range(world)]
        dist.all_gather(srcs, torch.from_numpy(mine))
        srcs = [s.numpy() for s in srcs]
        b, e = ctypes.c_uint64(), ctypes.c_uint64()
        ish.lib().ishmemi_c_chunk_bounds(nvec, world, rank, ctypes.byref(b), ctypes.byref(e))
        lo, hi = 4 * b.value, 4 * e.value
        my_chunk = oracle.reduce_fold(op, dt, [s[lo:hi] for s in srcs], 0)  # RS: canonical order
        tail = oracle.reduce_fold(op, dt, [s[4 * nvec:] for s in srcs], 0)  # owned by member p-1
        chunks = [None] * world
        dist.all_gather_object(chunks, (lo, hi, my_chunk))                  # AG
        res = np.empty(n, np.float32)
        for lo_, hi_, c in chunks:
            res[lo_:hi_] = c
        res[4 * nvec:] = tail
        ref = oracle.reduce_fold(op, dt, srcs, 0)
        assert np.array_equal(res.view(np.uint32), ref.view(np.uint32))
        dist.destroy_process_group()
        q.put((rank, None))
    except Exception as ex:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc() + str(ex)))


def test_gloo_world2_key_exchange_and_schedule():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in ps:
        p.join(timeout=30)
    errs = [e for _, e in res if e]
    assert not errs, "\n".join(errs)
