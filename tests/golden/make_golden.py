"""Generate tests/golden/golden_np{2,4,8}.npz — TEST FIXTURES (data only).

Runs oracle/mpi_golden (MPI_Allreduce of MPICH 3.3.2 under /opt/conda: the arithmetic backend
of the reference's host path, src/runtime/runtime_mpi.cpp:802-812) with mpiexec -n N on the
reference testers' source patterns and on seeded xorshift64* inputs, and packs every rank's
input and output.  Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
import oracle  # noqa: E402  (test infrastructure)

MPIEXEC = os.environ.get("MPIEXEC", "/opt/conda/bin/mpiexec")


def parse(path: Path):
    data = path.read_bytes()
    off = 0
    while off < len(data):
        name = data[off:off + 64].split(b"\0", 1)[0].decode()
        op, dt = np.frombuffer(data, np.int32, 2, off + 64)
        n = int(np.frombuffer(data, np.uint64, 1, off + 72)[0])
        es = np.dtype(oracle.NP[int(dt)]).itemsize
        off += 80
        inp = np.frombuffer(data, oracle.NP[int(dt)], n, off).copy()
        off += n * es
        out = np.frombuffer(data, oracle.NP[int(dt)], n, off).copy()
        off += n * es
        yield name, int(op), int(dt), inp, out


def main() -> None:
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle"), "mpi_golden"], check=True)
    for npes in (2, 4, 8):
        with tempfile.TemporaryDirectory() as td:
            subprocess.run([MPIEXEC, "-n", str(npes), str(ROOT / "oracle" / "mpi_golden"), td],
                           check=True, timeout=600)
            cases: dict[str, dict] = {}
            for pe in range(npes):
                for name, op, dt, inp, out in parse(Path(td) / f"golden_np{npes}_pe{pe}.bin"):
                    c = cases.setdefault(name, {"op": op, "dt": dt, "in": [], "out": []})
                    c["in"].append(inp)
                    c["out"].append(out)
        arrays = {}
        for name, c in cases.items():
            ins, outs = np.stack(c["in"]), np.stack(c["out"])
            arrays[f"{name}__meta"] = np.array([c["op"], c["dt"], ins.shape[1]], dtype=np.int64)
            arrays[f"{name}__in"] = ins
            same = all(np.array_equal(outs[0].view(np.uint8), o.view(np.uint8)) for o in outs)
            # Store every rank's output only where MPICH's ranks disagree (fp order effects).
            arrays[f"{name}__out"] = outs[:1] if same else outs
        dst = ROOT / "tests" / "golden" / f"golden_np{npes}.npz"
        np.savez_compressed(dst, **arrays)
        print(dst, len(cases), "cases", dst.stat().st_size, "bytes")


if __name__ == "__main__":
    main()
