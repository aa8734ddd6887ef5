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


def _bench():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_roofline_same_device_is_hbm_bound_and_at_most_one():
    # Round-2 rehearsal numbers: 2 PEs on one GPU, 1 GiB each, 1.0 ms per launch.  Against the
    # xGMI spec this read 6.17x "peak"; against the device's HBM it is a fraction below 1.
    b = _bench()
    B = 1 << 30
    roof, t_roof = b.roofline(2, 2, B, 1.0)
    assert roof["bound"] == "hbm" and roof["pes_per_device"] == 2
    assert abs(roof["achieved"] - 2 * 2.5 * B / 1e-3 / 1e9) < 1e-6
    assert 0 < roof["frac"] <= 1 and "model_violated" not in roof
    assert roof["traffic"] is not None  # committed same-device PMC entry (profiles/pmc_summary.json)
    assert B / t_roof >= B / 1e-3  # the step cannot beat its roofline
    roof8, _ = b.roofline(8, 8, B, 4.5)
    assert roof8["bound"] == "hbm" and roof8["frac"] <= 1


def test_roofline_one_pe_per_gpu_is_xgmi_and_flags_a_violated_model():
    b = _bench()
    B = 1 << 30
    roof, t_roof = b.roofline(8, 1, B, 2.0)  # 1.75 GiB of ingress per PE in 2 ms
    assert roof["bound"] == "xgmi" and roof["peak"] == b.XGMI_LINK_GBS * 7
    assert roof["traffic"] is None and "traffic_note" in roof
    assert 0 < roof["frac"] <= 1
    fast, _ = b.roofline(2, 1, B, 1.0)  # faster than the per-link spec allows
    assert fast["frac"] is None and fast["model_violated"] and fast["frac_raw"] > 1 and fast["reason"]
    one, t1 = b.roofline(1, 1, B, 0.3174)
    assert one["bound"] == "hbm" and abs(one["frac"] - 2 * B / 0.3174e-3 / 1e9 / 8000) < 1e-9
    assert abs(t1 - 2 * B / 8e12) < 1e-12


def test_multi_pe_kernel_follows_the_phased_threshold():
    # runtime.cpp reduce_heap: payloads of at least phased_min_bytes take the phased path's two
    # one-shot grids (-1: off); the roofline names them, and a same-device line then looks up the
    # phased path's PMC entry (the persistent kernel's would not describe the kernels that ran).
    b = _bench()
    B = 1 << 30
    k = b.multi_pe_kernel(B, 128 << 20)
    assert k.startswith("rs_phase_kernel")
    assert b.multi_pe_kernel(B, -1).startswith("allreduce_kernel")
    assert b.multi_pe_kernel(64 << 20, 128 << 20).startswith("allreduce_kernel")
    # Up to the team's fold bound (get_param "fold_limit_bytes": co-located 2 PEs 32 MiB): the
    # whole-array fold between two barriers (HBM 3B per PE).
    k2 = b.multi_pe_kernel(16 << 20, 4 << 20, 2, 32 << 20)
    assert "whole-array" in k2 and b.multi_pe_kernel(64 << 20, 4 << 20, 2, 32 << 20).startswith("rs_phase_kernel<float,SUM,P>")
    r2, t2 = b.roofline(2, 2, 16 << 20, 0.02, k2)
    assert "2 x 3 x B" in r2["kernel"] and abs(t2 - 2 * 3 * (16 << 20) / 8e12) < 1e-12
    # Four members (co-located bound 32 MiB / 4 / 3); every member pulls (p - 1) * B.
    k4 = b.multi_pe_kernel(2 << 20, 4 << 20, 4, (32 << 20) // 12)
    assert "whole-array" in k4 and "whole-array" not in b.multi_pe_kernel(4 << 20, 4 << 20, 4, (32 << 20) // 12)
    assert "whole-array" not in b.multi_pe_kernel(1 << 10, 4 << 20, 8, 0)  # no fold past 4 members
    r4, t4 = b.roofline(4, 1, 2 << 20, 0.02, k4)
    assert "(p-1)*B" in r4["kernel"] and abs(t4 - max(5 * (2 << 20) / 8e12, (2 << 20) / 153.6e9)) < 1e-12
    roof, _ = b.roofline(2, 2, B, 0.84, k)
    assert roof["kernel"].startswith("rs_phase_kernel") and 0 < roof["frac"] <= 1


def test_recommended_thresholds_from_the_tuning_rows():
    # the N > 1 line turns its xgmi_tuning rows into the environment a run on
    # that topology would set (cross-device variables when one PE per GPU).
    b = _bench()
    rows = [{"case": "ll_on", "bytes": 4096, "us": 4.0}, {"case": "ll_off", "bytes": 4096, "us": 9.0},
            {"case": "ll_on", "bytes": 65536, "us": 6.0}, {"case": "ll_off", "bytes": 65536, "us": 9.5},
            {"case": "ll_on", "bytes": 262144, "us": 12.0}, {"case": "ll_off", "bytes": 262144, "us": 10.0},
            {"case": "fold", "bytes": 1 << 20, "us": 9.0}, {"case": "no_fold", "bytes": 1 << 20, "us": 11.0},
            {"case": "fold", "bytes": 4 << 20, "us": 12.0}, {"case": "no_fold", "bytes": 4 << 20, "us": 13.0},
            {"case": "p2_oneshot", "bytes": 1 << 30, "us": 800.0}, {"case": "p2_rs_ag", "bytes": 1 << 30, "us": 840.0},
            {"case": "phased", "bytes": 2 << 20, "us": 15.0}, {"case": "persistent", "bytes": 2 << 20, "us": 14.0},
            {"case": "phased", "bytes": 4 << 20, "us": 16.0}, {"case": "persistent", "bytes": 4 << 20, "us": 17.0},
            {"case": "phased", "bytes": 1 << 30, "us": 850.0}, {"case": "persistent", "bytes": 1 << 30, "us": 990.0}]
    r = b.recommended(rows, 2, 1, 1 << 30)
    assert r["env"] == {"ISHMEM_XGMI_LL_MAX_BYTES": 65536, "ISHMEM_XGMI_FOLD_MAX_BYTES": 1 << 30,
                        "ISHMEM_PHASED_MIN_BYTES": 4 << 20}, r
    r8 = b.recommended([x for x in rows if not x["case"].startswith(("fold", "no_fold", "p2"))], 8, 8, 1 << 30)
    assert r8["env"] == {"ISHMEM_LL_MAX_BYTES": 65536, "ISHMEM_PHASED_MIN_BYTES": 4 << 20}, r8
