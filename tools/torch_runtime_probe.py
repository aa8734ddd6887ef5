#!/usr/bin/env python3
"""Which HIP / HSA runtime serves a process that loads ishmem_amd before torch, as bench.py and
tools/sweep.py now do (round 6), and does torch still work on it: one ishmem reduce, then a torch
matmul and a 1-rank RCCL all_reduce (the bench's N > 1 comparison leg runs RCCL after the library
has finalized).  Prints one JSON line.

  python tools/torch_runtime_probe.py
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def runtimes() -> list[str]:
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l})


def main() -> int:
    import numpy as np

    import ishmem_amd as ish
    from ishmem_amd import hip
    hip.lib()
    ctypes.CDLL("libhsa-runtime64.so", mode=ctypes.RTLD_GLOBAL)
    import torch
    import torch.distributed as dist
    out = {"runtimes_after_torch_import": runtimes()}
    ish.init(0, 1, 0, "torchprobe")
    n = 1 << 20
    s, d = ish.ishmem_malloc(4 * n), ish.ishmem_malloc(4 * n)
    hip.upload(s, np.arange(n, dtype=np.float32))
    out["ishmem_reduce_ok"] = ish.ishmem_float_sum_reduce(d, s, n) == 0 and bool(
        np.array_equal(hip.download(d, n, np.float32), np.arange(n, dtype=np.float32)))
    ish.ishmem_free(d)
    ish.ishmem_free(s)
    ish.ishmem_finalize()
    a = torch.randn(1024, 1024, device="cuda")
    out["torch_matmul_ok"] = bool(torch.allclose((a @ torch.eye(1024, device="cuda")).cpu(), a.cpu()))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29611")
    dist.init_process_group("nccl", rank=0, world_size=1)
    x = torch.ones(1 << 20, device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    out["rccl_allreduce_ok"] = bool(torch.all(x == 1.0).item())
    dist.destroy_process_group()
    out["runtimes_at_end"] = runtimes()
    print(json.dumps(out), flush=True)
    return 0 if out["ishmem_reduce_ok"] and out["torch_matmul_ok"] and out["rccl_allreduce_ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
