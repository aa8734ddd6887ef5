"""The reference's example programs as HIP programs (examples/*.hip): every ishmem call is the
reference's own, unchanged (host calls, and the device calls from inside kernels with no context
argument: ishmem_my_pe(), ishmem_int_sum_reduce(team, ...), ishmemx_int_sum_reduce_work_group(...,
grp), ishmem_barrier_all(), ishmem_int_broadcast(...)); only the SYCL launch / queue syntax is HIP.
Built on the CPU (here and by __graft_entry__.build()); run and result-checked on the GPU, PEs as
processes sharing the box's GPU."""
import os
import shutil
import subprocess
import uuid
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
EXAMPLES = ["pi_reduce", "library_apis", "team_split_strided"]  # ref: examples/5_, 3_, 6_*.cpp
HEADERS = [ROOT / "include" / h for h in ("ishmem.h", "ishmemx.h", "ishmem_capi.h", "ishmemx_device.h")]
MPIEXEC = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"
TORCHRUN_VARS = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT", "MASTER_ADDR",
                 "TORCHELASTIC_RUN_ID")


def build_example(name: str) -> Path:
    src = ROOT / "examples" / f"{name}.hip"
    exe = ROOT / "build" / "examples" / name
    lib = ROOT / "ishmem_amd" / "libishmem_amd.so"
    deps = [src, lib, *HEADERS]
    if exe.exists() and all(d.stat().st_mtime <= exe.stat().st_mtime for d in deps):
        return exe
    exe.parent.mkdir(parents=True, exist_ok=True)
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O2", "-std=c++20", f"-I{ROOT / 'include'}", str(src),
                    f"-L{lib.parent}", "-lishmem_amd", f"-Wl,-rpath,{lib.parent}", "-o", str(exe)], check=True)
    return exe


def run_example(exe: Path, npes: int, timeout: float = 180) -> list[str]:
    key = f"ex{uuid.uuid4().hex[:10]}"
    procs = []
    for pe in range(npes):
        env = {**os.environ, "ISHMEM_PE": str(pe), "ISHMEM_NPES": str(npes), "ISHMEM_DEVICE": "0",
               "ISHMEM_BOOTSTRAP_KEY": key, "ISHMEM_MAX_BLOCKS": "32", "ISHMEM_TIMEOUT_MS": "20000",
               "ISHMEM_SYMMETRIC_SIZE": "512M"}
        env.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)  # set by the library when it loads
        procs.append(subprocess.Popen([str(exe)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append((p.returncode, out))
    for pe, (rc, out) in enumerate(outs):
        assert rc == 0, f"PE {pe} rc={rc}\n{out[-3000:]}"
        assert f"PE#{pe} SUCCESS" in out, out[-3000:]
    return [o for _, o in outs]


@pytest.mark.parametrize("name", EXAMPLES)
def test_example_builds(name):
    assert build_example(name).exists()


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2, 3])
def test_pi_reduce(npes):
    outs = run_example(build_example("pi_reduce"), npes)
    assert "Value of pi from this experiment" in outs[0]


@pytest.mark.gpu
@pytest.mark.skipif(not Path(MPIEXEC).exists(), reason="no mpiexec (MPICH hydra)")
@pytest.mark.parametrize("wrapped", [False, True], ids=["direct", "via_wrapper_script"])
def test_pi_reduce_under_mpiexec(wrapped):
    """The reference's launch path (`mpirun -n N scripts/ishmrun ./app`, test/cmake/common.cmake:28-43):
    `mpiexec -n 2 ./pi_reduce` with no ISHMEM_* or torchrun variable.  The launcher starts both
    processes before any GPU call; ishmem_init takes PE identity from PMI_RANK / PMI_SIZE /
    MPI_LOCALRANKID (runtime_mpi.cpp:1256-1282's role) and both PEs must see npes == 2 — before
    this, each rank became a one-PE world that "reduced" by copying and still printed SUCCESS."""
    exe = build_example("pi_reduce")
    # Nothing but the launcher: no ISHMEM_*, no torchrun variable and no HSA_ENABLE_IPC_MODE_LEGACY
    # (the box exports it; libishmem_amd sets it when the program loads it).
    env = {k: v for k, v in os.environ.items()
           if not k.startswith("ISHMEM_") and k not in TORCHRUN_VARS and k != "HSA_ENABLE_IPC_MODE_LEGACY"}
    cmd = [str(exe)] if not wrapped else ["sh", "-c", '"$0"; exit $?', str(exe)]
    out = subprocess.run([MPIEXEC, "-n", "2", *cmd], env=env, capture_output=True, text=True, timeout=240)
    text = out.stdout + out.stderr
    assert out.returncode == 0, text[-3000:]
    for pe in range(2):
        assert f"PE#{pe} SUCCESS" in text, text[-3000:]
    assert text.count(" npes 2") == 2, text[-3000:]
    assert "Value of pi from this experiment" in text


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2, 4])
def test_library_apis(npes):
    run_example(build_example("library_apis"), npes)


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2, 3, 4])
def test_team_split_strided(npes):
    run_example(build_example("team_split_strided"), npes)
