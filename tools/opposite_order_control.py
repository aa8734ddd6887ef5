"""Negative control of tests/test_gpu_multi.py::test_opposite_order_collectives_of_two_teams_*:
the same "opposite" scenario (two teams, two streams, opposite issue orders on the two halves of
the PEs, every PE on its own emulated device) with the round-3 footprint — every waiting launch
allowed the whole device (ISHMEM_WAIT_SLOTS=1) — and a short device timeout, to show the scenario
does catch the hazard the waiting footprint removes.  Expected: the 4 MiB step fails with device
timeouts (bounded spins, ISHMEM_TIMEOUT_MS), not a hang.  Prints one JSON line.

    python tools/opposite_order_control.py [npes] [wait_slots]
"""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from tests.test_gpu_multi import run_pes  # noqa: E402


def main() -> int:
    npes = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    env = {"ISHMEM_AMD_LIB": str(Path(__file__).resolve().parents[1] / "ishmem_amd/libishmem_amd_testhooks.so"),
           "ISHMEM_TEST_PCI_BUS": [f"fake-bus-{i}" for i in range(npes)], "ISHMEM_MAX_BLOCKS": 1024,
           "ISHMEM_PHASED_MIN_BYTES": "", "ISHMEM_WAIT_SLOTS": slots, "ISHMEM_TIMEOUT_MS": 3000}
    t0 = time.monotonic()
    try:
        run_pes(npes, ["opposite"], env=env, timeout=240)
        outcome, detail = "passed", ""
    except AssertionError as ex:
        outcome, detail = "failed", str(ex)[:1500]
    print(json.dumps({"npes": npes, "wait_slots": slots, "outcome": outcome, "seconds": round(time.monotonic() - t0, 1),
                      "detail": detail}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
