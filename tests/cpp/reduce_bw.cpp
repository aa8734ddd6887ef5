// Reduce bandwidth harness in the shape of the reference's test/performance/reduce_bw.cpp driven
// by ishmem_tester::run_bw_tests (test/include/ishmem_tester.h:1478-1581): long sum-reduce over
// TEAM_WORLD for nelems = 1, 2, 4, ..., max_nelems; for each size the iteration count doubles
// (up to 16384) until one timed run takes > 2 ms, then the best of 10 runs is kept;
// latency = duration / iterations, bw = sizeof(long) * nelems * iterations / duration (MB/s).
// Same CSV columns as the reference (print_bw_result, :1448-1477).  Modes:
//   host_device_device  blocking ishmem_long_sum_reduce on symmetric-heap buffers
//   on_queue            ishmemx_long_sum_reduce_on_stream (the on_queue analogue), one sync
//   device_grp1         ishmemx_long_sum_reduce_work_group from a user kernel, 1024-thread group
//   device_subgroup     the same with one wavefront (sub_group analogue)
//   device_multi_wg     1 / 2 / 4 / 8 work-groups of 1024 threads in one kernel, each reducing
//                       nelems / groups elements on its own clone of TEAM_WORLD (groups column)
// Every PE runs the same schedule; the iteration count is agreed with a max-reduce of the
// durations (the reference broadcasts PE 0's command instead).
// Launch: ISHMEM_PE / ISHMEM_NPES / ISHMEM_DEVICE / ISHMEM_BOOTSTRAP_KEY per process, or torchrun.
//   ./reduce_bw [--csv] [-m max_nelems]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "ishmem.h"
#include "ishmemx.h"
#include "ishmemx_device.h"

template <typename G>
__global__ void wg_loop(long *dest, const long *src, size_t n,
                        size_t iters, int *rc)
{
    int bad = 0;
    for (size_t i = 0; i < iters; ++i) bad |= ishmemx_long_sum_reduce_work_group(dest, src, n, G());
    if (threadIdx.x == 0) *rc = bad;
}

// device_multi_wg (ishmem_tester.h:1344-1360): `groups` work-groups of one kernel, group g reducing
// its slice [g * per, (g + 1) * per) on its own clone of TEAM_WORLD (:299-304).
struct WgTeams {
    int t[8];
};

__global__ void multi_wg_loop(WgTeams teams, long *dest, const long *src, size_t per,
                              size_t iters, int *rc)
{
    const size_t off = (size_t) blockIdx.x * per;
    int bad = 0;
    for (size_t i = 0; i < iters; ++i)
        bad |= ishmemx_long_sum_reduce_work_group(teams.t[blockIdx.x], dest + off, src + off, per,
                                                  ishmemx_dev::work_group);
    if (threadIdx.x == 0 && bad) *rc = bad;
}

static double now_s()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    bool csv = false;
    size_t max_nelems = 1ul << 16;  // the tester's default (ishmem_tester.h:217)
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--csv") || !strcmp(argv[i], "-c")) csv = true;
        else if ((!strcmp(argv[i], "-m") || !strcmp(argv[i], "--max_nelems")) && i + 1 < argc)
            max_nelems = strtoul(argv[++i], nullptr, 0);
    }
    ishmem_init();
    if (!ishmemi_c_initialized()) {
        fprintf(stderr, "init failed: %s\n", ishmemi_c_last_error());
        return 1;
    }
    const int me = ishmem_my_pe(), npes = ishmem_n_pes();
    long *src = (long *) ishmem_malloc(max_nelems * sizeof(long) + 4096);
    long *dst = (long *) ishmem_malloc(max_nelems * sizeof(long) + 4096);
    double *agree = (double *) ishmem_malloc(sizeof(double));
    int *rc = nullptr;
    (void) hipMalloc(&rc, sizeof(int));
    hipStream_t st;
    (void) hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    (void) hipMemset(src, 1, max_nelems * sizeof(long));
    if (csv && me == 0) printf("csv,testname,ipc,npes,type,op,mode,groups,threads,bytes,pe,latency_us,bw_mb\n");

    WgTeams teams{};
    for (int g = 0; g < 8; ++g)
        if (ishmem_team_split_strided(ISHMEM_TEAM_WORLD, 0, 1, npes, nullptr, 0, &teams.t[g]) != 0) {
            fprintf(stderr, "team clone %d: %s\n", g, ishmemi_c_last_error());
            return 1;
        }
    // (mode, groups): the multi-work-group mode at 1, 2, 4 and 8 groups of 1024 threads.
    const struct {
        const char *mode;
        int groups;
    } runs[] = {{"host_device_device", 1}, {"on_queue", 1},        {"device_grp1", 1},     {"device_subgroup", 1},
                {"device_multi_wg", 1},    {"device_multi_wg", 2}, {"device_multi_wg", 4}, {"device_multi_wg", 8}};
    int failures = 0;
    for (const auto &rr : runs) {
        const char *mode = rr.mode;
        const int groups = rr.groups;
        const bool wave = !strcmp(mode, "device_subgroup"), grp = !strcmp(mode, "device_grp1");
        const bool multi = !strcmp(mode, "device_multi_wg");
        for (size_t n = multi ? (size_t) groups : 1; n <= max_nelems; n <<= 1) {
            auto run = [&](size_t iters) -> double {
                ishmem_barrier_all();
                const double t0 = now_s();
                if (!strcmp(mode, "host_device_device")) {
                    for (size_t i = 0; i < iters; ++i)
                        failures += ishmem_long_sum_reduce(ISHMEM_TEAM_WORLD, dst, src, n) != 0;
                } else if (!strcmp(mode, "on_queue")) {
                    for (size_t i = 0; i < iters; ++i)
                        failures += ishmemx_long_sum_reduce_on_stream(dst, src, n, nullptr, st) != 0;
                    (void) hipStreamSynchronize(st);
                } else if (multi) {
                    (void) hipMemset(rc, 0, sizeof(int));
                    hipLaunchKernelGGL(multi_wg_loop, dim3(groups), dim3(1024), 0, st, teams, dst, (const long *) src,
                                       n / (size_t) groups, iters, rc);
                    (void) hipStreamSynchronize(st);
                    int r = 0;
                    (void) hipMemcpy(&r, rc, sizeof(int), hipMemcpyDeviceToHost);
                    failures += r != 0;
                } else {
                    if (wave)
                        hipLaunchKernelGGL(wg_loop<ishmemx_dev::wavefront_t>, dim3(1), dim3(64), 0, st,
                                           dst, (const long *) src, n, iters, rc);
                    else
                        hipLaunchKernelGGL(wg_loop<ishmemx_dev::work_group_t>, dim3(1), dim3(1024), 0, st,
                                           dst, (const long *) src, n, iters, rc);
                    (void) hipStreamSynchronize(st);
                    int r = 0;
                    (void) hipMemcpy(&r, rc, sizeof(int), hipMemcpyDeviceToHost);
                    failures += r != 0;
                }
                double d = now_s() - t0;
                // Every PE takes the same decision: agree on the slowest PE's duration.
                (void) hipMemcpy(agree, &d, sizeof(double), hipMemcpyHostToDevice);
                ishmem_double_max_reduce(agree, agree, 1);
                (void) hipMemcpy(&d, agree, sizeof(double), hipMemcpyDeviceToHost);
                return d;
            };
            size_t iters = 1;
            double dur = run(iters);
            while (dur <= 0.002 && iters < 16384) {
                iters <<= 1;
                dur = run(iters);
            }
            const bool tested = dur > 0.002;
            for (int b = 0; b < 10; ++b) {
                const double t = run(iters);
                if (t < dur) dur = t;
            }
            if (tested && me == 0) {
                const double lat = dur / (double) iters * 1e6;
                const double bw = (double) sizeof(long) * (double) n * (double) iters / (dur * 1e6);
                const size_t threads = (grp || multi) ? 1024 : wave ? 64 : 1;
                if (csv)
                    printf("csv,reduce_bw,1,%d,long,sum,%s,%d,%zu,%zu,%s,%f,%f\n", npes, mode, groups, threads, n,
                           npes > 1 ? "xe" : "self", lat, bw);
                else
                    printf("test reduce_bw n_pes %d type long op sum mode %s groups %d threads %zu nelems %zu "
                           "latency %f us bw %f MB/s\n", npes, mode, groups, threads, n, lat, bw);
                fflush(stdout);
            }
        }
    }
    // Result check of the last call: every element of src is 0x0101010101010101.
    long *host = (long *) malloc(max_nelems * sizeof(long));
    (void) hipMemcpy(host, dst, max_nelems * sizeof(long), hipMemcpyDeviceToHost);
    const unsigned long want = 0x0101010101010101ul * (unsigned long) npes;
    size_t wrong = 0;
    for (size_t i = 0; i < max_nelems; ++i) wrong += (unsigned long) host[i] != want;
    free(host);
    if (me == 0) printf("%s errors %d wrong %zu\n", (failures || wrong) ? "FAIL" : "PASS", failures, wrong);
    for (int g = 0; g < 8; ++g) ishmem_team_destroy(teams.t[g]);
    (void) hipFree(rc);
    (void) hipStreamDestroy(st);
    ishmem_free(agree);
    ishmem_free(dst);
    ishmem_free(src);
    ishmem_finalize();
    return (failures || wrong) ? 1 : 0;
}
