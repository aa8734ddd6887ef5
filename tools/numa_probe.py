#!/usr/bin/env python3
"""Dev tool: does the NUMA node of pinned host memory explain the host-memory leg's variance?

For each NUMA node of the box: pin this process to that node's CPUs (before allocating), allocate
two 1 GiB pinned buffers with hipHostMalloc, and time hipMemcpyAsync H2D and D2H at once on two
streams (the staged pipeline's shape), 3 reps.  Prints one JSON line with the GPU's own NUMA node.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def node_cpus() -> dict[int, set[int]]:
    out = {}
    for d in sorted(Path("/sys/devices/system/node").glob("node[0-9]*")):
        cpus = set()
        for part in (d / "cpulist").read_text().strip().split(","):
            lo, _, hi = part.partition("-")
            cpus.update(range(int(lo), int(hi or lo) + 1))
        out[int(d.name[4:])] = cpus
    return out


def main() -> None:
    nodes = node_cpus()
    from ishmem_amd import hip
    L = hip.lib()
    bus = ctypes.create_string_buffer(64)
    L.hipDeviceGetPCIBusId(bus, 64, 0)
    busid = bus.value.decode().lower()
    try:
        gpu_node = int(Path(f"/sys/bus/pci/devices/{busid}/numa_node").read_text())
    except OSError:
        gpu_node = None
    B = 1 << 30
    res = {"gpu_pci_bus": busid, "gpu_numa_node": gpu_node, "nodes": {}}
    d1, d2 = hip.malloc(B), hip.malloc(B)
    s1, s2 = hip.stream_create(), hip.stream_create()
    for node, cpus in nodes.items():
        os.sched_setaffinity(0, cpus)
        hs, hd = hip.host_malloc(B), hip.host_malloc(B)
        ctypes.memset(hs, 1, B)  # touch from this node
        ctypes.memset(hd, 2, B)
        rates = []
        for _ in range(4):  # the first is a warm-up
            t0 = time.perf_counter()
            hip.memcpy_async(d1, hs, B, s1)
            hip.memcpy_async(hd, d2, B, s2)
            hip.stream_synchronize(s1)
            hip.stream_synchronize(s2)
            rates.append(round(B / (time.perf_counter() - t0) / 1e9, 2))
        res["nodes"][node] = {"concurrent_each_GBps": rates[1:]}
        hip.host_free(hs)
        hip.host_free(hd)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
