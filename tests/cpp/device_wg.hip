// Device-initiated reductions through include/ishmemx_device.h, in the shape of the reference's
// test/unit/long_reduce.cpp (source produced on the device, reduced from inside the kernel by one
// work-group per PE, checked against the closed form ((1 << npes) - 1) << 40 + idx * npes) and
// of its reduce_*.cpp pattern tests (sources = reference source patterns, checked against the
// reference check patterns restated in oracle/oracle.c, linked here as the CHECKER).
// Also: a wavefront (sub_group) caller and a single work-item device-side ishmem_int_sum_reduce,
// the reference's device_multi_wg mode (k work-groups of one kernel, each on its own team clone),
// and the device-side fcollect / collect / sum_inscan / sum_exscan (closed-form checks).
// Every device call is the reference's context-free form (the library's device state reaches the
// kernels through include/ishmemx_device.h's per-code-object context slot); groups are HIP
// cooperative groups (thread_block for sycl::group, a 64-lane thread_block_tile for sub_group) or
// the library's tags.
// Launch: ISHMEM_PE=<pe> ISHMEM_NPES=<n> ISHMEM_DEVICE=0 ISHMEM_BOOTSTRAP_KEY=<k> ./device_wg
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "ishmem.h"
#include "ishmemx.h"

namespace cg = cooperative_groups;

extern "C" {
#include "oracle.h"
}

static int errors = 0;

// long_reduce.cpp:78-79 / :120-127 — produce, then reduce, in one kernel.
__global__ void long_reduce_kernel(long *dest, long *source,
                                   size_t n, int my_pe, int *rc)
{
    for (size_t i = threadIdx.x; i < n; i += blockDim.x) source[i] = (1L << (40 + my_pe)) + (long) i;
    const int r = ishmemx_long_sum_reduce_work_group(dest, (const long *) source, n, cg::this_thread_block());
    if (threadIdx.x == 0) *rc = r;
}

template <typename T, int OPC>
__global__ void pattern_kernel(int team, T *dest, const T *source,
                               size_t n, int *rc)
{
    int r;
    if constexpr (OPC == ISHMEMI_OP_SUM) r = ishmemx_sum_reduce_work_group(team, dest, source, n, cg::this_thread_block());
    else if constexpr (OPC == ISHMEMI_OP_MAX) r = ishmemx_max_reduce_work_group(team, dest, source, n, cg::this_thread_block());
    else if constexpr (OPC == ISHMEMI_OP_MIN) r = ishmemx_min_reduce_work_group(team, dest, source, n, cg::this_thread_block());
    else if constexpr (OPC == ISHMEMI_OP_PROD) r = ishmemx_prod_reduce_work_group(team, dest, source, n, cg::this_thread_block());
    else if constexpr (OPC == ISHMEMI_OP_AND) r = ishmemx_and_reduce_work_group(team, dest, source, n, cg::this_thread_block());
    else if constexpr (OPC == ISHMEMI_OP_OR) r = ishmemx_or_reduce_work_group(team, dest, source, n, cg::this_thread_block());
    else r = ishmemx_xor_reduce_work_group(team, dest, source, n, cg::this_thread_block());
    if (threadIdx.x == 0) *rc = r;
}

// The reference CTest's "device" mode (test/unit/CMakeLists.txt:35, ishmem_tester.h:1229-1232):
// the blocking ishmem_<op>_reduce called by ONE work-item inside a kernel.
template <typename T, int OPC>
__global__ void device_mode_kernel(T *dest, const T *source, size_t n,
                                   int *rc)
{
    int r;
    if constexpr (OPC == ISHMEMI_OP_SUM) r = ishmem_sum_reduce(dest, source, n);
    else if constexpr (OPC == ISHMEMI_OP_MAX) r = ishmem_max_reduce(dest, source, n);
    else if constexpr (OPC == ISHMEMI_OP_MIN) r = ishmem_min_reduce(dest, source, n);
    else if constexpr (OPC == ISHMEMI_OP_PROD) r = ishmem_prod_reduce(dest, source, n);
    else if constexpr (OPC == ISHMEMI_OP_AND) r = ishmem_and_reduce(dest, source, n);
    else if constexpr (OPC == ISHMEMI_OP_OR) r = ishmem_or_reduce(dest, source, n);
    else r = ishmem_xor_reduce(dest, source, n);
    *rc = r;
}

// long_reduce.cpp:145-186: the in-place variant (source == dest) of the produce-then-reduce kernel.
__global__ void long_reduce_inplace_kernel(long *buf, size_t n, int my_pe,
                                           int *rc)
{
    for (size_t i = threadIdx.x; i < n; i += blockDim.x) buf[i] = (1L << (40 + my_pe)) + (long) i;
    const int r = ishmemx_long_sum_reduce_work_group(buf, (const long *) buf, n, ishmemx_dev::work_group);
    if (threadIdx.x == 0) *rc = r;
}

// sub_group analogue: only the second wavefront of the work-group takes part.
__global__ void wave_kernel(float *dest, const float *source, size_t n,
                            int *rc)
{
    if (threadIdx.x / warpSize != 1) return;
    const int r = ishmemx_float_sum_reduce_work_group(dest, source, n, ishmemx_dev::wavefront);
    if (__lane_id() == 0) *rc = r;
}

// device_multi_wg (ishmem_tester.h:117, :299-304, :1256-1260; team_reduce_test.h:119-137): k
// work-groups of ONE kernel, work-group g reducing its own slice [g * per, (g + 1) * per) on its
// own clone of TEAM_WORLD (ishmem_team_split_strided(WORLD, 0, 1, npes), ishmem_tester.h:299-304),
// the division of the tester's bandwidth runs (nelems /= groups, ishmem_tester.h:1292, :1344-1347).
// k collectives of k different teams in flight inside one kernel; each team has its own device
// flag rows and epoch counter.
struct WgTeams {
    int t[8];
};

template <typename T, int OPC>
__global__ void multi_wg_kernel(WgTeams teams, T *dest, const T *source, size_t per, int *rc)
{
    const size_t off = (size_t) blockIdx.x * per;
    const int team = teams.t[blockIdx.x];
    int r;
    if constexpr (OPC == ISHMEMI_OP_SUM) r = ishmemx_sum_reduce_work_group(team, dest + off, source + off, per, cg::this_thread_block());
    else if constexpr (OPC == ISHMEMI_OP_MIN) r = ishmemx_min_reduce_work_group(team, dest + off, source + off, per, cg::this_thread_block());
    else if constexpr (OPC == ISHMEMI_OP_PROD) r = ishmemx_prod_reduce_work_group(team, dest + off, source + off, per, cg::this_thread_block());
    else r = ishmemx_xor_reduce_work_group(team, dest + off, source + off, per, cg::this_thread_block());
    if (threadIdx.x == 0) rc[blockIdx.x] = r;
}

// Device-side blocking call by one work-item (the reference's single_task shape).
__global__ void single_kernel(int *dest, const int *source, size_t n,
                              int *rc)
{
    *rc = ishmem_int_sum_reduce(ISHMEM_TEAM_WORLD, dest, source, n);
}

// Device-side fcollect / collect / sum-scan (src/ishmemx.h *_work_group): the source is produced
// in the same kernel, then the collective runs by the work-group (or one wavefront / one item).
template <int MODE>  // 0 fcollect, 1 collect, 2 inscan, 3 exscan, 4 fcollect by a wavefront,
                     // 5 inscan by one work-item
__global__ void coll_kernel(long *dest, long *source, size_t n, int my_pe,
                            int *rc)
{
    const size_t mine = MODE == 1 ? n + 37 * (size_t) my_pe : n;  // collect: counts differ per PE
    for (size_t i = threadIdx.x; i < mine; i += blockDim.x) source[i] = ((long) (my_pe + 1) << 32) + (long) i;
    int r = 0;
    if constexpr (MODE == 0) r = ishmemx_long_fcollect_work_group(dest, (const long *) source, n, cg::this_thread_block());
    else if constexpr (MODE == 1) r = ishmemx_long_collect_work_group(dest, (const long *) source, mine, cg::this_thread_block());
    else if constexpr (MODE == 2) r = ishmemx_long_sum_inscan_work_group(dest, (const long *) source, n, cg::this_thread_block());
    else if constexpr (MODE == 3) r = ishmemx_long_sum_exscan_work_group(dest, (const long *) source, n, cg::this_thread_block());
    else if constexpr (MODE == 4) {
        __syncthreads();  // every wave's source stores are done before one wavefront publishes them
        auto wave = cg::tiled_partition<64>(cg::this_thread_block());  // sub_group analogue
        if (threadIdx.x / warpSize != 0) return;
        r = ishmemx_long_fcollect_work_group(dest, (const long *) source, n, wave);
        if (__lane_id() == 0) *rc = r;
        return;
    } else {
        __syncthreads();
        if (threadIdx.x != 0) return;
        r = ishmem_long_sum_inscan(ISHMEM_TEAM_WORLD, dest, (const long *) source, n);
        *rc = r;
        return;
    }
    if (threadIdx.x == 0) *rc = r;
}

template <int MODE>
static void coll_case(size_t n, int block, char *sb, char *db, int *rc)
{
    const int pe = ishmem_my_pe(), npes = ishmem_n_pes();
    auto val = [](int j, size_t i) { return ((long) (j + 1) << 32) + (long) i; };
    std::vector<long> want;
    if (MODE == 0 || MODE == 1 || MODE == 4) {
        for (int j = 0; j < npes; ++j) {
            const size_t c = MODE == 1 ? n + 37 * (size_t) j : n;
            for (size_t i = 0; i < c; ++i) want.push_back(val(j, i));
        }
    } else {
        const int last = (MODE == 3) ? pe - 1 : pe;
        for (size_t i = 0; i < n; ++i) {
            long acc = 0;
            for (int k = 0; k <= last; ++k) acc += val(k, i);
            want.push_back(acc);
        }
    }
    (void) hipMemset(db, 0xA5, want.size() * sizeof(long) + 64);
    (void) hipMemset(rc, 0xff, sizeof(int));
    hipLaunchKernelGGL(coll_kernel<MODE>, dim3(1), dim3(block), 0, 0, (long *) db, (long *) sb, n, pe, rc);
    (void) hipDeviceSynchronize();
    int r = -1;
    std::vector<long> got(want.size() + 8);
    (void) hipMemcpy(&r, rc, sizeof(int), hipMemcpyDeviceToHost);
    (void) hipMemcpy(got.data(), db, got.size() * sizeof(long), hipMemcpyDeviceToHost);
    size_t bad = 0;
    for (size_t i = 0; i < want.size(); ++i) bad += got[i] != want[i];
    const long guard = (long) 0xA5A5A5A5A5A5A5A5ull;
    for (size_t i = want.size(); i < got.size(); ++i) bad += got[i] != guard;
    if (r != 0 || bad) {
        if (++errors <= 16) printf("[%d] FAIL device collective mode %d n %zu block %d rc %d bad %zu\n", pe, MODE, n,
                                   block, r, bad);
    }
}

template <typename K, typename T, int OPC, int ODT>
static void group_case(const char *what, K kernel, int block, size_t n,
                       char *sb, char *db, int *rc)
{
    const int pe = ishmem_my_pe(), npes = ishmem_n_pes();
    std::vector<T> src(n), chk(n), got(n);
    oracle_pattern_source(PAT_ARITH, ODT, pe, n, src.data());
    oracle_pattern_check(PAT_ARITH, OPC, ODT, npes, n, chk.data());
    (void) hipMemcpy(sb, src.data(), n * sizeof(T), hipMemcpyHostToDevice);
    (void) hipMemset(db, 0, n * sizeof(T));
    (void) hipMemset(rc, 0xff, sizeof(int));
    hipLaunchKernelGGL(kernel, dim3(1), dim3(block), 0, 0, (T *) db, (const T *) sb, n, rc);
    (void) hipDeviceSynchronize();
    int r = -1;
    (void) hipMemcpy(&r, rc, sizeof(int), hipMemcpyDeviceToHost);
    (void) hipMemcpy(got.data(), db, n * sizeof(T), hipMemcpyDeviceToHost);
    if (r != 0 || memcmp(got.data(), chk.data(), n * sizeof(T)) != 0) {
        if (++errors <= 16) printf("[%d] FAIL %s n %zu rc %d\n", pe, what, n, r);
    }
}

template <typename T, int OPC, int ODT>
static void pattern_case(size_t n, dim3 block, char *sb, char *db,
                         int *rc, bool single_item = false)
{
    const int pe = ishmem_my_pe(), npes = ishmem_n_pes();
    const int fam = OPC == OR_AND ? PAT_AND : OPC == OR_OR ? PAT_OR : OPC == OR_XOR ? PAT_XOR : PAT_ARITH;
    std::vector<T> src(n), chk(n), got(n);
    oracle_pattern_source(fam, ODT, pe, n, src.data());
    oracle_pattern_check(fam, OPC, ODT, npes, n, chk.data());
    (void) hipMemcpy(sb, src.data(), n * sizeof(T), hipMemcpyHostToDevice);
    (void) hipMemset(db, 0, n * sizeof(T));
    if (single_item)
        hipLaunchKernelGGL((device_mode_kernel<T, OPC>), dim3(1), dim3(1), 0, 0, (T *) db, (const T *) sb,
                           n, rc);
    else
        hipLaunchKernelGGL((pattern_kernel<T, OPC>), dim3(1), block, 0, 0, ISHMEM_TEAM_WORLD,
                           (T *) db, (const T *) sb, n, rc);
    (void) hipDeviceSynchronize();
    int r = -1;
    (void) hipMemcpy(&r, rc, sizeof(int), hipMemcpyDeviceToHost);
    (void) hipMemcpy(got.data(), db, n * sizeof(T), hipMemcpyDeviceToHost);
    if (r != 0 || memcmp(got.data(), chk.data(), n * sizeof(T)) != 0) {
        if (++errors <= 16)
            printf("[%d] FAIL device pattern op %d dt %d n %zu block %ux%ux%u single %d rc %d\n", pe, OPC, ODT, n,
                   block.x, block.y, block.z, (int) single_item, r);
    }
}

template <typename T, int OPC, int ODT>
static void multi_wg_case(const WgTeams &teams, int k, size_t n, int block, char *sb, char *db, int *rc)
{
    const int pe = ishmem_my_pe(), npes = ishmem_n_pes();
    const int fam = OPC == OR_XOR ? PAT_XOR : PAT_ARITH;
    const size_t per = n / (size_t) k, covered = per * (size_t) k;
    std::vector<T> src(n), chk(n), got(n);
    oracle_pattern_source(fam, ODT, pe, n, src.data());
    oracle_pattern_check(fam, OPC, ODT, npes, n, chk.data());
    (void) hipMemcpy(sb, src.data(), n * sizeof(T), hipMemcpyHostToDevice);
    (void) hipMemset(db, 0x5A, n * sizeof(T));
    (void) hipMemset(rc, 0xff, 8 * sizeof(int));
    ishmem_barrier_all();  // every PE's source is in place (ishmem_sync_all in TEST_MULTI_WG_FN)
    hipLaunchKernelGGL((multi_wg_kernel<T, OPC>), dim3(k), dim3(block), 0, 0, teams, (T *) db, (const T *) sb, per,
                       rc);
    (void) hipDeviceSynchronize();
    int r[8];
    (void) hipMemcpy(r, rc, sizeof(r), hipMemcpyDeviceToHost);
    (void) hipMemcpy(got.data(), db, n * sizeof(T), hipMemcpyDeviceToHost);
    int rbad = 0;
    for (int g = 0; g < k; ++g) rbad += r[g] != 0;
    size_t bad = 0;
    for (size_t i = 0; i < covered; ++i) bad += memcmp(&got[i], &chk[i], sizeof(T)) != 0;
    std::vector<T> guard(1);
    memset(guard.data(), 0x5A, sizeof(T));
    for (size_t i = covered; i < n; ++i) bad += memcmp(&got[i], guard.data(), sizeof(T)) != 0;  // untouched
    if (rbad || bad) {
        if (++errors <= 16)
            printf("[%d] FAIL device_multi_wg op %d dt %d k %d n %zu block %d rc-fail %d bad %zu\n", pe, OPC, ODT, k,
                   n, block, rbad, bad);
    }
}

// Device-side broadcast (ishmemx_broadcastmem_work_group / ishmem_<TN>_broadcast, the reference's
// intra-node pull): the source is produced in the kernel, every member pulls the root's bytes.
__global__ void bcast_kernel(char *dest, char *source, size_t nbytes, int root, int my_pe, int mode, int *rc)
{
    for (size_t i = threadIdx.x; i < nbytes; i += blockDim.x) source[i] = (char) (i * 7 + my_pe * 31 + 1);
    int r;
    if (mode == 0) {
        r = ishmemx_broadcastmem_work_group(dest, source, nbytes, root, cg::this_thread_block());
    } else {
        __syncthreads();
        if (threadIdx.x != 0) return;
        r = ishmem_long_broadcast(ISHMEM_TEAM_WORLD, (long *) dest, (const long *) source, nbytes / 8, root);
    }
    if (threadIdx.x == 0) *rc = r;
}

// Device queries and barriers (src/ishmem.h:54-58, :74-77, :1555-1559).
__global__ void query_kernel(int *out, char *buf, const char *nonsym)
{
    auto grp = cg::this_thread_block();
    int r = 0;
    for (int k = 0; k < 5; ++k) ishmemx_team_sync_work_group(ISHMEM_TEAM_WORLD, grp);
    ishmemx_barrier_all_work_group(grp);
    ishmemx_sync_all_work_group(grp);
    if (grp.thread_rank() == 0) {
        for (int k = 0; k < 5; ++k) r |= ishmem_team_sync(ISHMEM_TEAM_WORLD);
        ishmem_barrier_all();
        ishmem_sync_all();
        const int pe = ishmem_my_pe(), n = ishmem_n_pes();
        int mj = 0, mn = 0;
        ishmem_info_get_version(&mj, &mn);
        char name[ISHMEM_MAX_NAME_LEN];
        ishmem_info_get_name(name);
        out[0] = pe;
        out[1] = n;
        out[2] = ishmem_team_my_pe(ISHMEM_TEAM_WORLD);
        out[3] = ishmem_team_n_pes(ISHMEM_TEAM_WORLD);
        out[4] = ishmem_team_translate_pe(ISHMEM_TEAM_WORLD, (pe + 1) % n, ISHMEM_TEAM_SHARED);
        out[5] = ishmem_ptr(buf, (pe + 1) % n) != nullptr && ishmem_ptr(buf, n) == nullptr &&
                 ishmem_ptr(nonsym, 0) == nullptr;
        out[6] = mj * 10 + mn;
        out[7] = name[0] != 0;
        out[8] = r;
        out[9] = ishmem_team_my_pe(ISHMEMI_C_MAX_TEAMS - 1);  // an unused team slot: -1
    }
}

int main()
{
    ishmem_init();
    const int pe = ishmem_my_pe(), npes = ishmem_n_pes();
    if (pe < 0) {
        printf("init failed: %s\n", ishmemi_c_last_error());
        return 2;
    }
    const size_t maxn = 1 << 17;
    char *sb = (char *) ishmem_malloc(maxn * 8);
    char *db = (char *) ishmem_malloc(maxn * 8);
    int *rc = (int *) ishmem_malloc(8 * sizeof(int));

    for (size_t n = 1; n <= maxn; n <<= 2) {
        for (int block : {64, 256, 1024}) {
            hipLaunchKernelGGL(long_reduce_kernel, dim3(1), dim3(block), 0, 0, (long *) db, (long *) sb,
                               n, pe, rc);
            (void) hipDeviceSynchronize();
            std::vector<long> got(n);
            int r = -1;
            (void) hipMemcpy(&r, rc, sizeof(int), hipMemcpyDeviceToHost);
            (void) hipMemcpy(got.data(), db, n * sizeof(long), hipMemcpyDeviceToHost);
            const long mask = ((1L << npes) - 1) << 40;
            size_t bad = 0;
            for (size_t i = 0; i < n; ++i) bad += got[i] != mask + (long) i * npes;
            if (r != 0 || bad) {
                if (++errors <= 16) printf("[%d] FAIL long_reduce n %zu block %d rc %d bad %zu\n", pe, n, block, r, bad);
            }
        }
    }
    for (size_t n : {1, 7, 64, 1000, 4097}) {
        pattern_case<float, OR_SUM, OD_FLOAT>(n, 256, sb, db, rc);
        pattern_case<double, OR_PROD, OD_DOUBLE>(n, 256, sb, db, rc);
        pattern_case<int32_t, OR_MIN, OD_INT32>(n, 128, sb, db, rc);
        pattern_case<int8_t, OR_MAX, OD_INT8>(n, 256, sb, db, rc);
        pattern_case<int16_t, OR_SUM, OD_INT16>(n, 64, sb, db, rc);
        pattern_case<uint64_t, OR_XOR, OD_UINT64>(n, 512, sb, db, rc);
        pattern_case<uint8_t, OR_AND, OD_UINT8>(n, 256, sb, db, rc);
        pattern_case<uint32_t, OR_OR, OD_UINT32>(n, 256, sb, db, rc);
    }
    // In place (long_reduce.cpp:145-186).
    for (size_t n : {1, 100, 4096, 65536}) {
        hipLaunchKernelGGL(long_reduce_inplace_kernel, dim3(1), dim3(256), 0, 0, (long *) sb, n, pe, rc);
        (void) hipDeviceSynchronize();
        std::vector<long> got(n);
        int r = -1;
        (void) hipMemcpy(&r, rc, sizeof(int), hipMemcpyDeviceToHost);
        (void) hipMemcpy(got.data(), sb, n * sizeof(long), hipMemcpyDeviceToHost);
        const long mask = ((1L << npes) - 1) << 40;
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i) bad += got[i] != mask + (long) i * npes;
        if (r != 0 || bad) {
            if (++errors <= 16) printf("[%d] FAIL long_reduce in place n %zu rc %d bad %zu\n", pe, n, r, bad);
        }
    }
    // "device" mode (one work-item) over every valid (op, dtype) with the testers' patterns.
    for (size_t n : {1, 17, 129}) {
#define DM(T, OPC, ODT) pattern_case<T, OPC, ODT>(n, dim3(1), sb, db, rc, true);
#define DM_INT(OPC) DM(int8_t, OPC, OD_INT8) DM(int16_t, OPC, OD_INT16) DM(int32_t, OPC, OD_INT32) \
    DM(int64_t, OPC, OD_INT64) DM(uint8_t, OPC, OD_UINT8) DM(uint16_t, OPC, OD_UINT16) DM(uint32_t, OPC, OD_UINT32) \
    DM(uint64_t, OPC, OD_UINT64)
#define DM_ALL(OPC) DM_INT(OPC) DM(float, OPC, OD_FLOAT) DM(double, OPC, OD_DOUBLE)
        DM_INT(OR_AND) DM_INT(OR_OR) DM_INT(OR_XOR)
        DM_ALL(OR_MAX) DM_ALL(OR_MIN) DM_ALL(OR_SUM) DM_ALL(OR_PROD)
#undef DM_ALL
#undef DM_INT
#undef DM
    }
    // device_grp2 / device_grp3: 2-D and 3-D work-groups (team_reduce_test.h TEST_GRP2_FN / GRP3).
    for (size_t n : {1, 1000, 4097}) {
        pattern_case<float, OR_SUM, OD_FLOAT>(n, dim3(16, 16), sb, db, rc);
        pattern_case<int64_t, OR_MAX, OD_INT64>(n, dim3(8, 4, 8), sb, db, rc);
        pattern_case<uint16_t, OR_XOR, OD_UINT16>(n, dim3(32, 2, 2), sb, db, rc);
    }
    for (size_t n : {1, 63, 64, 1000, 20000}) {
        group_case<decltype(&wave_kernel), float, OR_SUM, OD_FLOAT>("wavefront float sum", wave_kernel, 256, n, sb,
                                                                    db, rc);
        group_case<decltype(&single_kernel), int, OR_SUM, OD_INT32>("single-thread int sum", single_kernel, 1, n,
                                                                    sb, db, rc);
    }
    // device_multi_wg: k = 1..4 work-groups of one kernel on k clones of TEAM_WORLD.
    {
        WgTeams teams{};
        for (int g = 0; g < 4; ++g) {
            teams.t[g] = ISHMEM_TEAM_INVALID;
            if (ishmem_team_split_strided(ISHMEM_TEAM_WORLD, 0, 1, npes, nullptr, 0, &teams.t[g]) != 0 ||
                teams.t[g] == ISHMEM_TEAM_INVALID) {
                if (++errors <= 16) printf("[%d] FAIL team clone %d: %s\n", pe, g, ishmemi_c_last_error());
            }
        }
        for (int k = 1; k <= 4; ++k) {
            for (size_t n : {(size_t) k, (size_t) 1000, (size_t) 4097, (size_t) 65536}) {
                multi_wg_case<float, OR_SUM, OD_FLOAT>(teams, k, n, 256, sb, db, rc);
                multi_wg_case<int32_t, OR_MIN, OD_INT32>(teams, k, n, 1024, sb, db, rc);
                multi_wg_case<double, OR_PROD, OD_DOUBLE>(teams, k, n, 128, sb, db, rc);
                multi_wg_case<uint64_t, OR_XOR, OD_UINT64>(teams, k, n, 64, sb, db, rc);
            }
        }
        for (int g = 0; g < 4; ++g)
            if (teams.t[g] != ISHMEM_TEAM_INVALID) ishmem_team_destroy(teams.t[g]);
    }
    // fcollect / collect / inscan / exscan from inside a kernel (dest room: npes * (n + 37 npes)).
    for (size_t n : {1, 5, 64, 1000, 4099}) {
        if ((size_t) npes * (n + 37 * (size_t) npes) + 16 > maxn) continue;
        coll_case<0>(n, 256, sb, db, rc);
        coll_case<1>(n, 256, sb, db, rc);
        coll_case<2>(n, 256, sb, db, rc);
        coll_case<3>(n, 1024, sb, db, rc);
        coll_case<4>(n, 128, sb, db, rc);
        coll_case<5>(n, 64, sb, db, rc);
    }
    // Broadcast from every root, work-group and one-work-item forms, odd and even byte counts.
    for (int root = 0; root < npes; ++root) {
        for (size_t nb : {(size_t) 8, (size_t) 1000, (size_t) 77777 * 8}) {
            for (int mode = 0; mode < 2; ++mode) {
                (void) hipMemset(db, 0, nb + 64);
                (void) hipMemset(rc, 0xff, sizeof(int));
                hipLaunchKernelGGL(bcast_kernel, dim3(1), dim3(256), 0, 0, db, sb, nb, root, pe, mode, rc);
                (void) hipDeviceSynchronize();
                std::vector<char> got(nb);
                int r = -1;
                (void) hipMemcpy(&r, rc, sizeof(int), hipMemcpyDeviceToHost);
                (void) hipMemcpy(got.data(), db, nb, hipMemcpyDeviceToHost);
                size_t bad = 0;
                for (size_t i = 0; i < nb; ++i) bad += got[i] != (char) (i * 7 + root * 31 + 1);
                if (r != 0 || bad) {
                    if (++errors <= 16)
                        printf("[%d] FAIL device broadcast root %d nbytes %zu mode %d rc %d bad %zu\n", pe, root, nb,
                               mode, r, bad);
                }
            }
        }
    }
    {  // queries and barriers
        int *out = (int *) ishmem_malloc(16 * sizeof(int));
        char *nonsym = nullptr;
        (void) hipMalloc(&nonsym, 64);
        hipLaunchKernelGGL(query_kernel, dim3(1), dim3(256), 0, 0, out, db, nonsym);
        (void) hipDeviceSynchronize();
        int q[10];
        (void) hipMemcpy(q, out, sizeof(q), hipMemcpyDeviceToHost);
        const int want[10] = {pe, npes, pe, npes, (pe + 1) % npes, 1, 15, 1, 0, -1};
        for (int k = 0; k < 10; ++k)
            if (q[k] != want[k] && ++errors <= 16) printf("[%d] FAIL device query %d: %d != %d\n", pe, k, q[k], want[k]);
        ishmem_free(out);
        (void) hipFree(nonsym);
    }
    ishmem_free(rc);
    ishmem_free(db);
    ishmem_free(sb);
    ishmem_barrier_all();
    if (ishmemi_c_error_count()) ++errors;
    printf("[%d] %s errors %d\n", pe, errors ? "FAIL" : "PASS", errors);
    ishmem_finalize();
    return errors ? 1 : 0;
}
