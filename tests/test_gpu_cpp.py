"""The C++ drop-in API (include/ishmem.h, include/ishmemx.h) exercised like the reference's own
reduce tests (tests/cpp/reduce_patterns.cpp): 2 PEs as processes on the test box's GPU, the
reference testers' source/check patterns, aligned power-of-two sizes and the offset sweep."""
import os
import subprocess
import uuid
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "build" / "reduce_patterns"
DEV_EXE = ROOT / "build" / "device_wg"
HEADERS = [ROOT / "include/ishmem.h", ROOT / "include/ishmemx.h", ROOT / "include/ishmem_capi.h",
           ROOT / "include/ishmemx_device.h", ROOT / "oracle/oracle.c", ROOT / "oracle/oracle.h"]


def build_exe(src: Path = ROOT / "tests/cpp/reduce_patterns.cpp", exe: Path = EXE) -> Path:
    """hipcc the test program against include/ and libishmem_amd.so; link the oracle (checker)."""
    deps = [src, *HEADERS, ROOT / "ishmem_amd/libishmem_amd.so"]
    if exe.exists() and all(s.stat().st_mtime <= exe.stat().st_mtime for s in deps if s.exists()):
        return exe
    exe.parent.mkdir(parents=True, exist_ok=True)
    obj = exe.parent / "oracle_for_cpp_test.o"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-c", str(ROOT / "oracle/oracle.c"), "-o", str(obj)],
                   check=True)
    tobj = exe.with_suffix(".o")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O2", "-std=c++20", "-Wno-unused-value",
                    f"-I{ROOT / 'include'}", f"-I{ROOT / 'oracle'}", "-c", str(src), "-o", str(tobj)],
                   check=True)
    subprocess.run(["hipcc", "--offload-arch=gfx950", str(tobj), str(obj), f"-L{ROOT / 'ishmem_amd'}",
                    "-lishmem_amd", "-lm", "-lpthread", f"-Wl,-rpath,{ROOT / 'ishmem_amd'}", "-o", str(exe)],
                   check=True)
    return exe


CHECK_LIB = ROOT / "build" / "libpattern_check.so"


def build_pattern_check() -> Path:
    """The device pattern checker of the large-size parity checks (tests/cpp/pattern_check.hip ->
    build/libpattern_check.so, loaded by ishmem_amd/selfcheck.py)."""
    src = ROOT / "tests/cpp/pattern_check.hip"
    if CHECK_LIB.exists() and src.stat().st_mtime <= CHECK_LIB.stat().st_mtime:
        return CHECK_LIB
    CHECK_LIB.parent.mkdir(parents=True, exist_ok=True)
    tmp = CHECK_LIB.with_suffix(".so.tmp")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-ffp-contract=off", "-fPIC", "-shared",
                    str(src), "-o", str(tmp)], check=True)
    os.replace(tmp, CHECK_LIB)
    return CHECK_LIB


def base_env() -> dict:
    """The test's environment without HSA_ENABLE_IPC_MODE_LEGACY, which the box exports: the
    library sets it when a program loads it (runtime.cpp ipc_mode_default)."""
    return {k: v for k, v in os.environ.items() if k != "HSA_ENABLE_IPC_MODE_LEGACY"}


def run_exe(exe: Path, npes: int, timeout: float = 600) -> None:
    key = f"cpp{uuid.uuid4().hex[:10]}"
    procs = []
    for pe in range(npes):
        env = {**base_env(), "ISHMEM_PE": str(pe), "ISHMEM_NPES": str(npes), "ISHMEM_DEVICE": "0",
               "ISHMEM_BOOTSTRAP_KEY": key, "ISHMEM_MAX_BLOCKS": "32", "ISHMEM_TIMEOUT_MS": "20000",
               "ISHMEM_SYMMETRIC_SIZE": "512M"}
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
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "PASS errors 0" in out


def test_cpp_test_program_builds():
    assert build_exe().exists()


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2])
def test_cpp_reference_style_reduce_tests(npes):
    run_exe(build_exe(), npes)


def test_device_api_program_builds():
    assert build_exe(ROOT / "tests/cpp/device_wg.hip", DEV_EXE).exists()


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2, 3])
def test_device_initiated_work_group_reduce(npes):
    """ishmemx_*_reduce_work_group called from a user kernel (include/ishmemx_device.h), including the
    reference's device_multi_wg mode: k = 1..4 work-groups of one kernel on k clones of TEAM_WORLD."""
    run_exe(build_exe(ROOT / "tests/cpp/device_wg.hip", DEV_EXE), npes)


BW_EXE = ROOT / "build" / "reduce_bw"


def test_reduce_bw_harness_builds():
    assert build_exe(ROOT / "tests/cpp/reduce_bw.cpp", BW_EXE).exists()


@pytest.mark.gpu
def test_reduce_bw_harness_runs_and_checks():
    """The reference's reduce_bw shape (test/performance/reduce_bw.cpp): every mode, result-checked."""
    key = f"bw{uuid.uuid4().hex[:10]}"
    exe = build_exe(ROOT / "tests/cpp/reduce_bw.cpp", BW_EXE)
    procs = []
    for pe in range(2):
        env = {**base_env(), "ISHMEM_PE": str(pe), "ISHMEM_NPES": "2", "ISHMEM_DEVICE": "0",
               "ISHMEM_BOOTSTRAP_KEY": key, "ISHMEM_MAX_BLOCKS": "32", "ISHMEM_TIMEOUT_MS": "20000",
               "ISHMEM_SYMMETRIC_SIZE": "512M"}
        procs.append(subprocess.Popen([str(exe), "--csv", "-m", "1024"], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=300)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs[0][-2000:] + outs[1][-2000:]
    assert "PASS errors 0" in outs[0]
    assert outs[0].count("csv,reduce_bw,") >= 4 * 8
    # device_multi_wg (ishmem_tester.h:1344-1360): rows for 1, 2, 4 and 8 work-groups.
    for groups in (1, 2, 4, 8):
        assert f",device_multi_wg,{groups},1024," in outs[0], outs[0][-2000:]
