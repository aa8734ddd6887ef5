"""CPU tests of the C-ABI boundary: the library loads, exports every declared symbol, the host
logic (validity matrix, dtype sizes, partition) is right, and the C++ header with the
reference's names compiles and links.  No compute calls (there is no GPU here)."""
import ctypes
import re
import shutil
import subprocess
from pathlib import Path

import pytest

import ishmem_amd as ish
from ishmem_amd import _lib

ROOT = Path(__file__).resolve().parents[1]
INCLUDE = ROOT / "include"


def declared_symbols():
    text = (INCLUDE / "ishmem_capi.h").read_text()
    return sorted(set(re.findall(r"\b(ishmemi_c_\w+)\s*\(", text)))


def test_every_declared_symbol_is_exported_and_bound():
    lib = ish.lib()
    syms = declared_symbols()
    assert len(syms) >= 30
    bound = {name for name, _, _ in _lib.PROTOTYPES}
    for s in syms:
        assert hasattr(lib, s), s
        assert s in bound, f"{s} has no ctypes prototype"
    nm = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True)
    exported = set(re.findall(r" T (ishmemi_c_\w+)", nm.stdout))
    assert set(syms) <= exported


def test_library_has_gfx950_code_object():
    out = subprocess.run(["strings", str(_lib.LIB_PATH)], capture_output=True, text=True).stdout
    assert "gfx950" in out


def test_not_initialized_calls_fail_cleanly():
    lib = ish.lib()
    assert lib.ishmemi_c_initialized() == 0
    assert lib.ishmemi_c_my_pe() == -1
    assert lib.ishmemi_c_reduce(0, 5, 8, None, None, 0) != 0
    assert "not initialized" in ish.last_error()
    assert lib.ishmemi_c_malloc(16) is None


def test_dtype_sizes_and_validity():
    lib = ish.lib()
    sizes = [lib.ishmemi_c_dtype_size(d) for d in range(10)]
    assert sizes == [1, 2, 4, 8, 1, 2, 4, 8, 4, 8]
    assert lib.ishmemi_c_dtype_size(10) == 0
    for op in range(7):
        for dt in range(10):
            fp = dt >= 8
            assert lib.ishmemi_c_op_dtype_valid(op, dt) == (0 if (fp and op <= 2) else 1)
    assert lib.ishmemi_c_op_dtype_valid(7, 0) == 0


def test_api_names_match_reference_instantiations():
    # src/collectives/reduce.cpp:95-417: 14 typenames x {and,or,xor} + 23 x {max,min,sum,prod}
    blocking = [n for n in ish.API_NAMES if n.startswith("ishmem_")]
    assert len(blocking) == 14 * 3 + 23 * 4
    for n in ["ishmem_float_sum_reduce", "ishmem_size_sum_reduce", "ishmem_int32_prod_reduce",
              "ishmem_ulonglong_xor_reduce", "ishmem_double_min_reduce", "ishmem_char_max_reduce"]:
        assert callable(getattr(ish, n))
    assert not hasattr(ish, "ishmem_float_and_reduce")
    assert not hasattr(ish, "ishmem_schar_and_reduce")  # declared, never defined in the reference
    assert callable(ish.ishmemx_float_sum_reduce_on_stream)


@pytest.mark.parametrize("nitems", [0, 1, 63, 64, 65, 1000, 4096 * 7 + 5, 1 << 26])
@pytest.mark.parametrize("npes", [1, 2, 3, 4, 8])
def test_partition_covers_exactly_once(nitems, npes):
    lib = ish.lib()
    b, e = ctypes.c_uint64(), ctypes.c_uint64()
    prev_end = 0
    for c in range(npes):
        assert lib.ishmemi_c_chunk_bounds(nitems, npes, c, ctypes.byref(b), ctypes.byref(e)) == 0
        assert b.value == prev_end
        assert e.value >= b.value
        if npes > 1 and e.value < nitems:
            assert b.value % 64 == 0 and e.value % 64 == 0  # line-aligned chunk edges
        prev_end = e.value
    assert prev_end == nitems


def test_cxx_header_compiles_and_links(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include "ishmemx.h"
#include <cstdio>
int main() {
    float *d = nullptr; const float *s = nullptr;
    int r1 = ishmem_float_sum_reduce(d, s, 0);             // not initialised -> nonzero
    int r2 = ishmem_sum_reduce(ISHMEM_TEAM_WORLD, d, s, 0);  // generic template overload
    size_t *z = nullptr;
    int r3 = ishmem_size_and_reduce(z, z, 0);
    int r4 = ishmemx_double_max_reduce_on_stream((double*)nullptr, nullptr, 0, nullptr, nullptr);
    hipEvent_t deps[1] = {nullptr};
    int r5 = ishmemx_int_sum_reduce_on_stream(ISHMEM_TEAM_WORLD, (int*)nullptr, nullptr, 0, nullptr,
                                              nullptr, deps, 0, nullptr);  // deps / done overload
    int r7 = ishmemx_int_fcollect_on_stream(ISHMEM_TEAM_WORLD, (int*)nullptr, nullptr, 0, nullptr, nullptr,
                                            deps, 0, nullptr);  // deps / done form of the collectives
    long *lp = nullptr;
    int r6 = ishmemx_sum_reduce_on_stream(lp, (const long*)lp, 0, nullptr, nullptr);  // generic
    std::printf("%d %d %d %d %d %d %d %d\n", r1 != 0, r2 != 0, r3 != 0, r4 != 0, r5 != 0, r6 != 0, r7 != 0, ishmem_my_pe());
    return 0;
}
''')
    exe = tmp_path / "t"
    subprocess.run([gxx, "-std=c++17", f"-I{INCLUDE}", str(src), "-o", str(exe),
                    f"-L{_lib.LIB_PATH.parent}", f"-Wl,-rpath,{_lib.LIB_PATH.parent}", "-lishmem_amd"],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["1", "1", "1", "1", "1", "1", "1", "-1"]


def test_c_header_is_plain_c(tmp_path):
    gcc = shutil.which("gcc")
    if gcc is None:
        pytest.skip("no gcc")
    src = tmp_path / "t.c"
    src.write_text('#include "ishmem_capi.h"\nint main(void){return ishmemi_c_n_pes() == -1 ? 0 : 1;}\n')
    subprocess.run([gcc, "-std=c99", "-Wall", "-Werror", f"-I{INCLUDE}", "-c", str(src), "-o",
                    str(tmp_path / "t.o")], check=True)


def test_setup_surface_of_the_reference_header_compiles(tmp_path):
    # src/ishmem.h:17-26 (version, thread levels), :44-45 (init_thread / query_thread), :57-58
    # (info_get_*), :63-67 / :78 (team config), :761-813 (broadcast) — with host g++, no GPU.
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    src = tmp_path / "t.cpp"
    src.write_text(r'''
#include <ishmem.h>
#include <ishmemx.h>
#include <cstdio>
#include <cstring>
int main() {
    int major = 0, minor = 0, provided = -1;
    char name[ISHMEM_MAX_NAME_LEN];
    ishmem_info_get_version(&major, &minor);
    ishmem_info_get_name(name);
    ishmem_query_thread(&provided);
    ishmem_team_config_t cfg = {3};
    ishmem_team_config_t *config = NULL;
    ishmem_team_t t = ISHMEM_TEAM_INVALID;
    int r1 = ishmem_team_get_config(ISHMEM_TEAM_WORLD, ISHMEM_TEAM_NUM_CONTEXTS, &cfg);  // not initialised
    int r2 = ishmem_team_split_strided(ISHMEM_TEAM_WORLD, 0, 2, 1, config, 0, &t);
    int r3 = ishmem_int_broadcast((int *) nullptr, nullptr, 0, 0);
    int r4 = ishmem_broadcastmem(ISHMEM_TEAM_WORLD, nullptr, nullptr, 0, 0);
    std::printf("%d %d %d %s %d %d %d %d %d\n", major, minor, provided, std::strlen(name) > 0 ? "named" : "-",
                r1 != 0, r2 != 0, r3 != 0, r4 != 0, ISHMEM_THREAD_MULTIPLE);
    return 0;
}
''')
    exe = tmp_path / "t"
    subprocess.run([gxx, "-std=c++17", f"-I{INCLUDE}", str(src), "-o", str(exe),
                    f"-L{_lib.LIB_PATH.parent}", f"-Wl,-rpath,{_lib.LIB_PATH.parent}", "-lishmem_amd"],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split() == ["1", "5", "3", "named", "1", "1", "1", "1", "3"]


def test_device_api_compiles_without_a_context_argument(tmp_path):
    # The reference's device calls, verbatim, inside HIP kernels (hipcc, gfx950; compile only).
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists():
        pytest.skip("no hipcc")
    src = tmp_path / "t.hip"
    src.write_text(r'''
#include <hip/hip_cooperative_groups.h>
#include <ishmem.h>
#include <ishmemx.h>
namespace cg = cooperative_groups;
__global__ void k(int *dst_sum, int *reduce_src, int *dst, int *src, ishmem_team_t team, double *fd, double *fs) {
    auto grp = cg::this_thread_block();
    auto wave = cg::tiled_partition<64>(grp);
    int my_dev_pe = ishmem_my_pe(), my_dev_npes = ishmem_n_pes();
    if (grp.thread_rank() == 0) ishmem_barrier_all();
    ishmemx_barrier_all_work_group(grp);
    ishmemx_sync_all_work_group(grp);
    ishmemx_team_sync_work_group(team, grp);
    if (grp.thread_rank() == 0) ishmem_int_sum_reduce(dst_sum, reduce_src, 1);
    ishmemx_int_sum_reduce_work_group(dst_sum, reduce_src, 1, grp);
    ishmemx_int_sum_reduce_work_group(team, dst_sum, reduce_src, 1, grp);
    ishmemx_double_prod_reduce_work_group(fd, fs, 8, wave);
    ishmemx_sum_reduce_work_group(fd, fs, 8, grp);          // generic
    ishmemx_broadcastmem_work_group(dst, src, 4, 0, grp);
    ishmemx_int_fcollect_work_group(dst, src, 1, grp);
    ishmemx_int_sum_inscan_work_group(team, dst, src, 1, grp);
    if (grp.thread_rank() == 0) {
        ishmem_int_sum_reduce(team, dst_sum, reduce_src, 1);
        ishmem_int_broadcast(team, dst, src, 1, 0);
        ishmem_team_sync(ISHMEM_TEAM_WORLD);
        ishmem_sync_all();
        int t = ishmem_team_my_pe(team) + ishmem_team_n_pes(team) + ishmem_team_translate_pe(team, 0, ISHMEM_TEAM_WORLD);
        void *p = ishmem_ptr(dst, (my_dev_pe + 1) % my_dev_npes);
        int mj, mn;
        ishmem_info_get_version(&mj, &mn);
        if (!p || t < 0) ishmemx_print("unexpected\n", ishmemx_print_msg_type_t::ERROR);
    }
}
int main() { return 0; }
''')
    subprocess.run([hipcc, "--offload-arch=gfx950", "-std=c++20", f"-I{INCLUDE}", "-c", str(src), "-o",
                    str(tmp_path / "t.o")], check=True)
