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


def build_exe() -> Path:
    srcs = [ROOT / "tests/cpp/reduce_patterns.cpp", ROOT / "oracle/oracle.c", ROOT / "oracle/oracle.h",
            ROOT / "include/ishmem.h", ROOT / "include/ishmemx.h", ROOT / "include/ishmem_capi.h"]
    if EXE.exists() and all(s.stat().st_mtime <= EXE.stat().st_mtime for s in srcs):
        return EXE
    EXE.parent.mkdir(parents=True, exist_ok=True)
    obj = EXE.parent / "oracle_for_cpp_test.o"
    subprocess.run(["gcc", "-O2", "-std=gnu11", "-fPIC", "-c", str(ROOT / "oracle/oracle.c"), "-o", str(obj)],
                   check=True)
    tobj = EXE.parent / "reduce_patterns.o"
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O2", "-std=c++20", "-Wno-unused-value",
                    f"-I{ROOT / 'include'}", f"-I{ROOT / 'oracle'}", "-c",
                    str(ROOT / "tests/cpp/reduce_patterns.cpp"), "-o", str(tobj)], check=True)
    subprocess.run(["hipcc", "--offload-arch=gfx950", str(tobj), str(obj), f"-L{ROOT / 'ishmem_amd'}",
                    "-lishmem_amd", "-lm", "-lpthread", f"-Wl,-rpath,{ROOT / 'ishmem_amd'}", "-o", str(EXE)],
                   check=True)
    return EXE


def test_cpp_test_program_builds():
    assert build_exe().exists()


@pytest.mark.gpu
@pytest.mark.parametrize("npes", [2])
def test_cpp_reference_style_reduce_tests(npes):
    exe = build_exe()
    key = f"cpp{uuid.uuid4().hex[:10]}"
    procs = []
    for pe in range(npes):
        env = {**os.environ, "ISHMEM_PE": str(pe), "ISHMEM_NPES": str(npes), "ISHMEM_DEVICE": "0",
               "ISHMEM_BOOTSTRAP_KEY": key, "ISHMEM_MAX_BLOCKS": "32", "ISHMEM_TIMEOUT_MS": "20000",
               "ISHMEM_SYMMETRIC_SIZE": "512M", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
        procs.append(subprocess.Popen([str(exe)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=600)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append((p.returncode, out))
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "PASS errors 0" in out
