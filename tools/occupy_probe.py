"""Does a kernel on stream B run while an occupying kernel holds CUs on stream A?  (One process,
one PE.)  Prints, per occupier grid, how long a 64 MiB local combine on another stream took."""
from __future__ import annotations

import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import ishmem_amd as ish  # noqa: E402
from ishmem_amd import hip  # noqa: E402


def main() -> None:
    ish.init(0, 1, 0, None)
    cus = int(ish.get_param("cu_count"))
    n = 16 << 20
    a, d = ish.ishmem_malloc(4 * n), ish.ishmem_malloc(4 * n)
    occ, st = hip.stream_create(), hip.stream_create()
    for grid in (0, cus // 2, cus - 16, cus, 2 * (cus - 16), 2 * cus - 8):
        if grid:
            ish.occupy(grid, 1_000_000, occ)
            time.sleep(0.05)
        t0 = time.perf_counter()
        ish.combine("sum", "float", d, [a, a], n, st)
        hip.stream_synchronize(st)
        t1 = time.perf_counter()
        hip.stream_synchronize(occ)
        t2 = time.perf_counter()
        print(f"cus={cus} occupier_grid={grid}: combine {1e3 * (t1 - t0):.2f} ms, occupier done after "
              f"{1e3 * (t2 - t0):.0f} ms", flush=True)
    ish.ishmem_finalize()


if __name__ == "__main__":
    main()
