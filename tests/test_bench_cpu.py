"""bench.py's N>1 entry without an external launcher (CPU): `python bench.py --gpus 2` starts the
two ranks itself (torch.distributed.run as a child process), and exactly one JSON line — rank 0's —
reaches stdout.  Without a GPU the ranks fail at init, so the line carries the error; its n_gpus
comes from the WORLD_SIZE the child launcher set, which shows the relay path ran."""
import json
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def test_bench_self_launches_ranks_and_relays_one_json_line():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"],
                       cwd=str(ROOT), capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout + r.stderr[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2
    assert d["metric"].startswith("GiB/s device-resident float32 sum-reduce")
    if "error" in d:  # no GPU in this container
        assert r.returncode != 0
    else:
        assert r.returncode == 0 and d["value"] > 0 and "algbw_GiBps" in d
