"""PE identity under the launchers the reference's programs are started with (CPU, no GPU).

The reference's ishmem_init takes rank and size from its MPI / PMI runtime
(src/runtime/runtime_mpi.cpp:1256-1282); its tests and examples run as
`mpirun -n N scripts/ishmrun ./app` (test/cmake/common.cmake:28-43).  ishmemi_c_init reads the
same identity from the launcher's environment (ishmem_amd/csrc/runtime.cpp launch_info) and the
C++ header's ishmem_init exits on failure like the reference's (src/ishmem.cpp:396-407,
src/ishmem/err.h:105-110).  The GPU side (the reference's pi example under mpiexec) is
tests/test_examples.py::test_pi_reduce_under_mpiexec.
"""
import ctypes
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

from ishmem_amd import _lib

ROOT = Path(__file__).resolve().parents[1]
INCLUDE = ROOT / "include"
MPIEXEC = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"
LAUNCH_VARS = ("ISHMEM_PE", "ISHMEM_NPES", "ISHMEM_DEVICE", "ISHMEM_BOOTSTRAP_KEY", "RANK", "WORLD_SIZE",
               "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT", "TORCHELASTIC_RUN_ID", "PMI_RANK", "PMI_SIZE",
               "MPI_LOCALRANKID", "MPI_LOCALNRANKS", "OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE",
               "OMPI_COMM_WORLD_LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_SIZE", "SLURM_PROCID", "SLURM_NTASKS",
               "SLURM_NPROCS", "SLURM_LOCALID", "SLURM_JOB_ID", "SLURM_STEP_ID", "SLURM_NTASKS_PER_NODE",
               "SLURM_STEP_NUM_TASKS", "SLURM_STEP_NUM_NODES", "ISHMEM_ENABLE_GPU_IPC",
               "ISHMEM_ENABLE_ACCESSIBLE_HOST_HEAP", "ISHMEM_WAIT_SLOTS", "ISHMEM_TEST_PCI_BUS",
               "ISHMEM_TEST_FLAGS_UNAVAILABLE", "GPU_MAX_HW_QUEUES", "ISHMEM_BARRIER_KIND", "ISHMEM_DEBUG",
               "ISHMEM_TEAMS_MAX", "ISHMEM_XGMI_LL_MAX_BYTES", "ISHMEM_XGMI_FOLD_MAX_BYTES")

# One process: what ishmemi_c_init would use, then (optionally) the native bootstrap's allgather
# among the PEs it names.
PROBE = r'''
import ctypes, sys
sys.path.insert(0, sys.argv[1])
from ishmem_amd import _lib
L = _lib.load(build_if_missing=False)
pe, npes, dev = ctypes.c_int(-9), ctypes.c_int(-9), ctypes.c_int(-9)
launcher, key = ctypes.create_string_buffer(32), ctypes.create_string_buffer(256)
rc = L.ishmemi_c_launch_info(ctypes.byref(pe), ctypes.byref(npes), ctypes.byref(dev), launcher, 32, key, 256)
line = f"rc={rc} pe={pe.value} npes={npes.value} dev={dev.value} launcher={launcher.value.decode()}"
if rc:
    line += " err=" + L.ishmemi_c_last_error().decode().replace(" ", "_")
elif len(sys.argv) > 2 and npes.value > 1:
    out = (ctypes.c_int * npes.value)()
    r = L.ishmemi_c_bootstrap_selftest(pe.value, npes.value, key.value, 10 * pe.value + 1, out)
    line += f" boot={r} got={','.join(str(v) for v in out)}"
print(line, flush=True)
'''


def clean_env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in LAUNCH_VARS}
    env.update({k: str(v) for k, v in extra.items()})
    return env


def probe(env, boot=False):
    args = [sys.executable, "-c", PROBE, str(ROOT)] + (["boot"] if boot else [])
    out = subprocess.run(args, env=env, capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    return dict(kv.split("=", 1) for kv in out.stdout.split())


def test_launch_info_reads_each_launcher_family():
    assert probe(clean_env()) == {"rc": "0", "pe": "0", "npes": "1", "dev": "0", "launcher": "none"}
    got = probe(clean_env(ISHMEM_PE=2, ISHMEM_NPES=4, ISHMEM_DEVICE=1))
    assert (got["pe"], got["npes"], got["dev"], got["launcher"]) == ("2", "4", "1", "ishmem")
    got = probe(clean_env(RANK=1, WORLD_SIZE=8, LOCAL_RANK=5, MASTER_PORT=29500))
    assert (got["pe"], got["npes"], got["dev"], got["launcher"]) == ("1", "8", "5", "torchrun")
    got = probe(clean_env(PMI_RANK=3, PMI_SIZE=8, MPI_LOCALRANKID=3, MPI_LOCALNRANKS=8))
    assert (got["pe"], got["npes"], got["dev"], got["launcher"]) == ("3", "8", "3", "pmi")
    got = probe(clean_env(OMPI_COMM_WORLD_RANK=6, OMPI_COMM_WORLD_SIZE=8, OMPI_COMM_WORLD_LOCAL_RANK=6,
                          OMPI_COMM_WORLD_LOCAL_SIZE=8))
    assert (got["pe"], got["npes"], got["dev"], got["launcher"]) == ("6", "8", "6", "openmpi")
    got = probe(clean_env(SLURM_PROCID=7, SLURM_NTASKS=8, SLURM_STEP_NUM_TASKS=8, SLURM_STEP_ID=0,
                          SLURM_STEP_NUM_NODES=1, SLURM_LOCALID=7, SLURM_JOB_ID=42))
    assert (got["pe"], got["npes"], got["dev"], got["launcher"]) == ("7", "8", "7", "slurm")
    # Explicit variables override the launcher's, one by one.
    got = probe(clean_env(PMI_RANK=1, PMI_SIZE=2, MPI_LOCALRANKID=1, ISHMEM_DEVICE=0))
    assert (got["pe"], got["npes"], got["dev"], got["launcher"]) == ("1", "2", "0", "pmi")


def test_launch_info_refuses_multi_node_and_bad_ranks():
    got = probe(clean_env(PMI_RANK=0, PMI_SIZE=4, MPI_LOCALRANKID=0, MPI_LOCALNRANKS=2))
    assert got["rc"] == "1" and "one_node" in got["err"], got
    got = probe(clean_env(ISHMEM_PE=3, ISHMEM_NPES=2))
    assert got["rc"] == "1", got
    # `srun -N2 -n8` without --ntasks-per-node: refused by the step's node count.
    got = probe(clean_env(SLURM_PROCID=0, SLURM_NTASKS=8, SLURM_STEP_NUM_TASKS=8, SLURM_STEP_ID=3,
                          SLURM_STEP_NUM_NODES=2, SLURM_LOCALID=0, SLURM_JOB_ID=42))
    assert got["rc"] == "1" and "2_nodes" in got["err"], got


@pytest.mark.parametrize("step", ["batch", "interactive", "extern", None])
def test_slurm_batch_step_is_a_one_pe_world(step):
    """inside `sbatch -n 8` the batch script's environment has SLURM_PROCID=0 and
    SLURM_NTASKS=8 for the allocation; a program started there without srun is one process and must
    be a 1-PE world, not PE 0 of 8 waiting in the bootstrap for peers that never start.  Only an srun
    task step (numeric SLURM_STEP_ID, SLURM_STEP_NUM_TASKS) names a multi-PE world."""
    env = dict(SLURM_PROCID=0, SLURM_NTASKS=8, SLURM_NPROCS=8, SLURM_LOCALID=0, SLURM_JOB_ID=42,
               SLURM_NTASKS_PER_NODE=8)
    if step is not None:
        env["SLURM_STEP_ID"] = step
    got = probe(clean_env(**env))
    assert (got["rc"], got["pe"], got["npes"], got["launcher"]) == ("0", "0", "1", "none"), got


@pytest.mark.parametrize("name,value", [("ISHMEM_PE", "abc"), ("ISHMEM_NPES", "2x"), ("PMI_RANK", "1.0"),
                                        ("OMPI_COMM_WORLD_SIZE", "8 8"), ("ISHMEM_DEVICE", "")])
def test_launch_identity_variables_parse_strictly(name, value):
    """the identity variables pick the bootstrap world, so a malformed one fails
    with its name instead of parsing as a prefix (ISHMEM_NPES='2x' -> 2, ISHMEM_PE='abc' -> 0).
    An empty value counts as unset, as for every other variable."""
    base = {"ISHMEM_PE": dict(ISHMEM_PE=0, ISHMEM_NPES=2), "ISHMEM_NPES": dict(ISHMEM_PE=0, ISHMEM_NPES=2),
            "PMI_RANK": dict(PMI_RANK=0, PMI_SIZE=2), "OMPI_COMM_WORLD_SIZE": dict(OMPI_COMM_WORLD_RANK=0),
            "ISHMEM_DEVICE": dict(ISHMEM_PE=0, ISHMEM_NPES=1)}[name]
    got = probe(clean_env(**{**base, name: value}))
    if value:
        assert got["rc"] == "1" and name in got["err"] and "not_an_integer" in got["err"], got
    else:
        assert got["rc"] == "0", got


@pytest.mark.skipif(not Path(MPIEXEC).exists(), reason="no mpiexec (MPICH hydra)")
@pytest.mark.parametrize("wrapped", [False, True], ids=["direct", "via_wrapper_script"])
def test_mpiexec_two_ranks_form_one_world(wrapped):
    """`mpiexec -n 2` with no ISHMEM_* / torchrun variables: both ranks resolve PE 0 / 1 of 2 and
    meet in the native bootstrap (allgather + barrier).  Wrapped: each rank runs under its own shell,
    like the reference's `mpirun -n N scripts/ishmrun ./app`, and the key still agrees (the hydra
    proxy, found by walking up the process tree)."""
    cmd = [sys.executable, "-c", PROBE, str(ROOT), "boot"]
    if wrapped:  # sh stays the rank's process (no exec), python its child
        cmd = ["sh", "-c", f'"{sys.executable}" -c "$0" "$@"; exit $?', PROBE, str(ROOT), "boot"]
    out = subprocess.run([MPIEXEC, "-n", "2", *cmd], env=clean_env(), capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    lines = sorted(l for l in out.stdout.splitlines() if l.startswith("rc="))
    assert len(lines) == 2, out.stdout + out.stderr
    got = [dict(kv.split("=", 1) for kv in l.split()) for l in lines]
    assert [g["pe"] for g in got] == ["0", "1"]
    for g in got:
        assert (g["rc"], g["npes"], g["launcher"], g["boot"], g["got"]) == ("0", "2", "pmi", "0", "1,11"), g


def test_cxx_ishmem_init_failure_exits_like_the_reference(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    src = tmp_path / "t.cpp"
    src.write_text('#include <ishmem.h>\n#include <cstdio>\n'
                   'int main() { ishmem_init(); std::printf("after init\\n"); return 0; }\n')
    exe = tmp_path / "t"
    subprocess.run([gxx, "-std=c++17", f"-I{INCLUDE}", str(src), "-o", str(exe),
                    f"-L{_lib.LIB_PATH.parent}", f"-Wl,-rpath,{_lib.LIB_PATH.parent}", "-lishmem_amd"], check=True)
    # PE 3 of 2: refused before any GPU call, on any machine.
    out = subprocess.run([str(exe)], env=clean_env(ISHMEM_PE=3, ISHMEM_NPES=2), capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 1, (out.returncode, out.stdout, out.stderr)
    assert "after init" not in out.stdout
    assert "ishmem_init failed" in out.stderr and "PE 3 of 2" in out.stderr, out.stderr


def test_launch_info_is_declared_and_bound():
    L = _lib.load()
    assert L.ishmemi_c_launch_info.restype is ctypes.c_int


ENV_PROBE = r'''
import sys
sys.path.insert(0, sys.argv[1])
from ishmem_amd import _lib
L = _lib.load(build_if_missing=False)
rc = L.ishmemi_c_init_pe(0, 1, 0, b"envprobe")
print("rc=%d|%s" % (rc, L.ishmemi_c_last_error().decode()))
'''


@pytest.mark.parametrize("name,value,bad", [
    ("ISHMEM_PHASED_MIN_BYTES", "16MB x", True), ("ISHMEM_PHASED_MIN_BYTES", "abc", True),
    ("ISHMEM_LL_MAX_BYTES", "64KQ", True), ("ISHMEM_SYMMETRIC_SIZE", "-4G", True),
    ("ISHMEM_STAGING_SIZE", "nan", True), ("ISHMEM_PHASED_MIN_BYTES", "1e30", False),
    ("ISHMEM_PHASED_MIN_BYTES", " 16MiB ", False), ("ISHMEM_LL_MAX_BYTES", "64kb", False),
    ("ISHMEM_SYMMETRIC_SIZE", "2T", False), ("ISHMEM_PHASED_MIN_BYTES", "-1", False),
    # integer variables: the same rule (a prefix such as "16x" -> 16 used to pass silently)
    ("ISHMEM_WAIT_SLOTS", "16x", True), ("ISHMEM_STAGING_SLOTS", "four", True),
    # the waiting-footprint floor: below GPU_MAX_HW_QUEUES (4) fails init
    ("ISHMEM_WAIT_SLOTS", "1", True), ("ISHMEM_WAIT_SLOTS", "3", True), ("ISHMEM_WAIT_SLOTS", "4", False),
    # reference switches this IPC-only path cannot honour, refused by name
    ("ISHMEM_ENABLE_GPU_IPC", "0", True), ("ISHMEM_ENABLE_GPU_IPC", "false", True),
    ("ISHMEM_ENABLE_GPU_IPC", "1", False), ("ISHMEM_ENABLE_ACCESSIBLE_HOST_HEAP", "1", True),
    ("ISHMEM_ENABLE_ACCESSIBLE_HOST_HEAP", "FALSE", False), ("ISHMEM_ENABLE_ACCESSIBLE_HOST_HEAP", "0", False),
    # ISHMEM_DEBUG is the reference's boolean (env_utils.cpp:138-149): "true" / "yes" are valid
    ("ISHMEM_DEBUG", "true", False), ("ISHMEM_DEBUG", "yes", False), ("ISHMEM_DEBUG", "2", False),
    # the team-barrier kind: the kernel only since round 6 (the stream-memory-op barrier was removed,
    # DESIGN.md §7); "stream" is refused by name rather than silently ignored
    ("ISHMEM_BARRIER_KIND", "stream", True), ("ISHMEM_BARRIER_KIND", "Kernel", False),
    ("ISHMEM_BARRIER_KIND", "cp", True),
    # the team table's size: the reference's variable, default 64, at most 64
    # (src/ishmem/env_defs.h:34, src/teams.cpp:245-248); below 3 it is raised to 3 (teams.cpp:119)
    ("ISHMEM_TEAMS_MAX", "abc", True), ("ISHMEM_TEAMS_MAX", "65", True), ("ISHMEM_TEAMS_MAX", "64x", True),
    ("ISHMEM_TEAMS_MAX", "-1", True), ("ISHMEM_TEAMS_MAX", "64", False), ("ISHMEM_TEAMS_MAX", "1", False),
    # cross-device thresholds: byte counts, -1 = the link-byte model
    ("ISHMEM_XGMI_LL_MAX_BYTES", "256K", False), ("ISHMEM_XGMI_LL_MAX_BYTES", "lots", True),
    ("ISHMEM_XGMI_FOLD_MAX_BYTES", "-1", False), ("ISHMEM_XGMI_FOLD_MAX_BYTES", "8MiBs", True),
    # test hooks exist only in libishmem_amd_testhooks.so
    ("ISHMEM_TEST_PCI_BUS", "fake-bus-0", True), ("ISHMEM_TEST_FLAGS_UNAVAILABLE", "1", True),
    ("ISHMEM_TIMEOUT_MS", "99999999999999999999", True), ("ISHMEM_FLAGS_KIND", "1.5", True),
    ("ISHMEM_MAX_BLOCKS", " 256 ", False), ("ISHMEM_TIMEOUT_MS", "-5", False)])
def test_byte_count_variables_parse_strictly(name, value, bad):
    """byte-count variables choose kernel paths every PE must agree on, so a typo
    fails init with the variable named instead of parsing as something else; values past LLONG_MAX
    clamp.  Integer ISHMEM_* variables (grid caps, slots, timeouts, test hooks) are held to the same
    rule.  Checked before any GPU call (here the init then fails for want of a device, or not at
    all on a GPU box — either way not on the variable)."""
    out = subprocess.run([sys.executable, "-c", ENV_PROBE, str(ROOT)], env=clean_env(**{name: value}),
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    line = out.stdout.strip().splitlines()[-1]
    if bad:
        assert line.startswith("rc=1|") and name in line, line
    else:
        assert name not in line, line


def test_wait_slots_floor_follows_hw_queues():
    """The floor is GPU_MAX_HW_QUEUES: with 8 queues per process, 6 slots are refused."""
    out = subprocess.run([sys.executable, "-c", ENV_PROBE, str(ROOT)],
                         env=clean_env(ISHMEM_WAIT_SLOTS=6, GPU_MAX_HW_QUEUES=8), capture_output=True, text=True,
                         timeout=120)
    line = out.stdout.strip().splitlines()[-1]
    assert line.startswith("rc=1|") and "ISHMEM_WAIT_SLOTS=6 is below 8" in line, line


IPC_ENV_PROBE = r'''
import ctypes, os, sys
sys.path.insert(0, sys.argv[1])
from ishmem_amd import _lib
_lib.load(build_if_missing=False)
libc = ctypes.CDLL(None)
libc.getenv.restype = ctypes.c_char_p
v = libc.getenv(b"HSA_ENABLE_IPC_MODE_LEGACY")
print("value=" + (v.decode() if v is not None else "unset"))
'''


@pytest.mark.parametrize("preset,want", [(None, "0"), ("1", "1"), ("0", "0")])
def test_library_sets_ipc_mode_when_loaded(preset, want):
    """the drop-in program launched the reference's way sets no HSA variable, and
    this node's driver shares device memory as dma-buf only; the library's constructor sets
    HSA_ENABLE_IPC_MODE_LEGACY=0 when it is loaded (before any HIP call of a program linked against
    it) and leaves a user's own value alone.  The GPU side: test_pi_reduce_under_mpiexec and
    test_gpu_multi.py::test_two_pes_without_ipc_mode_variable run with the variable removed."""
    env = clean_env()
    env.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    if preset is not None:
        env["HSA_ENABLE_IPC_MODE_LEGACY"] = preset
    out = subprocess.run([sys.executable, "-c", IPC_ENV_PROBE, str(ROOT)], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().splitlines()[-1] == f"value={want}", out.stdout


def test_unknown_ishmem_variable_warns_like_the_reference():
    """The reference warns about an ISHMEM_* name it does not define and carries on
    (src/env_utils.cpp:193-196); so does ishmemi_c_init.  The reference's own variables that this
    path has no use for (ISHMEM_NBI_COUNT, ...) are accepted silently."""
    out = subprocess.run([sys.executable, "-c", ENV_PROBE, str(ROOT)],
                         env=clean_env(ISHMEM_NO_SUCH_KNOB="1", ISHMEM_NBI_COUNT="8"), capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "Environment variable 'ISHMEM_NO_SUCH_KNOB' is not a supported variable" in out.stderr
    assert "ISHMEM_NBI_COUNT" not in out.stderr
    assert "ISHMEM_NO_SUCH_KNOB" not in out.stdout.strip().splitlines()[-1]  # a warning, not an init error
