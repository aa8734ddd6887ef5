#!/usr/bin/env python3
"""Same-device multi-PE PMC summary (round 3): reads the FETCH_SIZE / WRITE_SIZE passes of
scripts/prof_multi.sh (rocprofv3 over bench.py --gpus N with every PE on the box's one GPU) and
adds `allreduce_{N}pe_same_device` (persistent kernel) or `phased_{N}pe_same_device` (the
phased path's two grids) to profiles/pmc_summary.json.  The counters are device-wide,
so a traced dispatch's window holds every co-located PE's traffic; FETCH_SIZE is doubled
(gfx950, MI355X_MICROARCH.md §HBM), WRITE_SIZE is exact.

  python tools/summarize_multi_pmc.py gpurun_out/<tag> NPES <round-tag> [payload_bytes]
"""
from __future__ import annotations

import csv
import json
import shutil
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def values(path: Path, counter: str, kernel: str) -> list[float]:
    return [float(r["Counter_Value"]) for r in csv.DictReader(path.open())
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]


# Kernel families of a multi-PE f32 sum call: the persistent kernel (one launch per call), or the
# phased path's two one-shot grids (their per-call traffic is the sum of the two medians).
FAMILIES = {"allreduce": ["allreduce_kernel<float, 5, true"],
            "phased": ["rs_phase_kernel<float, 5", "ag_phase_kernel"]}


def main() -> None:
    src, npes, tag = Path(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 30
    dst = ROOT / "profiles" / "r03" / "multi"
    dst.mkdir(parents=True, exist_ok=True)
    f_csv = src / "pmc_FETCH_SIZE" / "run_counter_collection.csv"
    w_csv = src / "pmc_WRITE_SIZE" / "run_counter_collection.csv"
    for p, name in ((f_csv, "pmc_FETCH_SIZE.csv"), (w_csv, "pmc_WRITE_SIZE.csv"),
                    (src / "trace" / "run_kernel_stats.csv", "kernel_stats.csv"),
                    (src / "trace" / "run_kernel_trace.csv", "kernel_trace.csv")):
        if p.exists():
            shutil.copy(p, dst / f"{tag}_p{npes}_{name}")
    fam = "phased" if values(f_csv, "FETCH_SIZE", "rs_phase_kernel<float, 5") else "allreduce"
    fs = [values(f_csv, "FETCH_SIZE", k) for k in FAMILIES[fam]]
    ws = [values(w_csv, "WRITE_SIZE", k) for k in FAMILIES[fam]]
    fk, wk = sum(statistics.median(v) for v in fs), sum(statistics.median(v) for v in ws)
    rd, wr = 2.0 * fk * 1024.0, wk * 1024.0
    alg_r, alg_w = npes * (2.0 - 1.0 / npes) * B, npes * B
    summ = json.loads((ROOT / "profiles" / "pmc_summary.json").read_text())
    key = f"{fam}_{npes}pe_same_device"
    summ[key] = {
        "kernel": ("allreduce_kernel<float, 5, true, P>" if fam == "allreduce" else
                   "rs_phase_kernel<float, 5, P> + ag_phase_kernel (per call: sum of the two medians)")
                  + " (every PE on the one GPU)", "payload_bytes": B,
        "pes": npes, "dispatches_traced": len(fs[0]), "fetch_size_kb_median_raw": fk, "write_size_kb_median": wk,
        "hbm_bytes_per_launch": rd + wr, "algorithmic_bytes_per_launch": alg_r + alg_w,
        "traffic_over_algorithmic": (rd + wr) / (alg_r + alg_w),
        "read_over_algorithmic": rd / alg_r, "write_over_algorithmic": wr / alg_w,
        "correction": "FETCH_SIZE x2 (gfx950, 16 B/lane streams)",
        "scope": "device-wide counters over one traced rank's dispatch window; all PEs share the one GPU "
                 "(not an xGMI run)", "source": f"profiles/r03/multi/{tag}_p{npes}_pmc_*.csv"}
    (ROOT / "profiles" / "pmc_summary.json").write_text(json.dumps(summ, indent=2) + "\n")
    print(json.dumps(summ[key], indent=2))


if __name__ == "__main__":
    main()
