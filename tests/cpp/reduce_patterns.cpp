// Parity test in the shape of the reference's test/unit/reduce_{sum,prod,min,max,and,or,xor}.cpp:
// every PE fills its source with the reference tester's source pattern, calls the typed
// ishmem_<TYPENAME>_<op>_reduce through include/ishmem.h (the drop-in C++ API), copies dest back
// and compares it with the reference tester's check pattern (restated in oracle/oracle.c, which
// this TEST links as the checker).  Sizes 1, 2, 4, ..., max_nelems like run_aligned_tests
// (test/include/ishmem_tester.h:1373-1395) plus the offset sweep of run_offset_tests (:1407-1436).
// Launch: ISHMEM_PE=<pe> ISHMEM_NPES=<n> ISHMEM_DEVICE=0 ISHMEM_BOOTSTRAP_KEY=<k> ./reduce_patterns
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "ishmem.h"
#include "ishmemx.h"

extern "C" {
#include "oracle.h"
}

static int errors = 0;

template <typename T>
static int dt_of()
{
    return ishmemi_cxx::dtype_of<T>();
}

// One (type, op) test at nelems with source/dest byte offsets (both multiples of sizeof(T)).
template <typename T, typename F>
static void run_case(const char *tn, const char *opn, int op, F reduce_fn, size_t nelems, size_t so,
                     size_t od, char *src_base, char *dst_base)
{
    const int pe = ishmem_my_pe(), npes = ishmem_n_pes();
    const int dt = dt_of<T>();
    const int fam = op == OR_AND ? PAT_AND : op == OR_OR ? PAT_OR : op == OR_XOR ? PAT_XOR : PAT_ARITH;
    std::vector<T> src(nelems), chk(nelems), got(nelems);
    oracle_pattern_source(fam, dt, pe, nelems, src.data());
    oracle_pattern_check(fam, op, dt, npes, nelems, chk.data());
    T *s = (T *) (src_base + so), *d = (T *) (dst_base + od);
    hipMemcpy(s, src.data(), nelems * sizeof(T), hipMemcpyHostToDevice);
    hipMemset(d, 0, nelems * sizeof(T));
    const int r = reduce_fn(d, s, nelems);
    hipMemcpy(got.data(), d, nelems * sizeof(T), hipMemcpyDeviceToHost);
    if (r != 0 || memcmp(got.data(), chk.data(), nelems * sizeof(T)) != 0) {
        if (++errors <= 16)
            printf("[%d] FAIL %s_%s_reduce nelems %zu os %zu od %zu rc %d\n", pe, tn, opn, nelems, so,
                   od, r);
    }
}

template <typename T, typename F>
static void run_type(const char *tn, const char *opn, int op, F fn, size_t max_nelems, char *sb,
                     char *db)
{
    for (size_t n = 1; n <= max_nelems; n <<= 1) run_case<T>(tn, opn, op, fn, n, 0, 0, sb, db);
    for (size_t n = 1; n <= 16; ++n)
        for (size_t so = 0; so < 15; so += sizeof(T) * 3)
            for (size_t od = 0; od < 15; od += sizeof(T) * 2)
                run_case<T>(tn, opn, op, fn, n, so, od, sb, db);
}

int main()
{
    ishmem_init();
    const int pe = ishmem_my_pe(), npes = ishmem_n_pes();
    if (pe < 0) {
        printf("init failed: %s\n", ishmemi_c_last_error());
        return 2;
    }
    const size_t max_nelems = 1 << 16;  // ishmem_tester.h:217 default
    char *sb = (char *) ishmem_malloc(max_nelems * 8 + 64);
    char *db = (char *) ishmem_malloc(max_nelems * 8 + 64);
#define T_(TN, TYPE, OPN, OPC)                                                                     \
    run_type<TYPE>(#TN, #OPN, OPC,                                                                 \
                   [](TYPE *d, const TYPE *s, size_t n) { return ishmem_##TN##_##OPN##_reduce(d, s, n); }, \
                   max_nelems, sb, db);
    T_(int, int, sum, OR_SUM)
    T_(float, float, sum, OR_SUM)
    T_(double, double, sum, OR_SUM)
    T_(long, long, sum, OR_SUM)
    T_(short, short, prod, OR_PROD)
    T_(double, double, prod, OR_PROD)
    T_(int8, int8_t, min, OR_MIN)
    T_(float, float, min, OR_MIN)
    T_(uint64, uint64_t, max, OR_MAX)
    T_(double, double, max, OR_MAX)
    T_(uchar, unsigned char, and, OR_AND)
    T_(uint32, uint32_t, or, OR_OR)
    T_(size, size_t, xor, OR_XOR)
    T_(ulonglong, unsigned long long, xor, OR_XOR)
#undef T_
    // Team overload + generic template (src/ishmem.h:1136, :1162).
    {
        std::vector<int> src(1000), chk(1000), got(1000);
        oracle_pattern_source(PAT_ARITH, OD_INT32, pe, 1000, src.data());
        oracle_pattern_check(PAT_ARITH, OR_SUM, OD_INT32, npes, 1000, chk.data());
        hipMemcpy(sb, src.data(), 4000, hipMemcpyHostToDevice);
        const int r = ishmem_sum_reduce(ISHMEM_TEAM_WORLD, (int *) db, (const int *) sb, 1000);
        hipMemcpy(got.data(), db, 4000, hipMemcpyDeviceToHost);
        if (r || memcmp(got.data(), chk.data(), 4000)) {
            ++errors;
            printf("[%d] FAIL generic team sum_reduce\n", pe);
        }
    }
    // Stream variant with *ret (ishmemx_*_reduce_on_queue analogue).
    {
        int *ret = (int *) ishmem_malloc(sizeof(int));
        hipMemset(ret, 0xff, sizeof(int));
        hipStream_t st;
        hipStreamCreate(&st);
        const int r = ishmemx_float_max_reduce_on_stream((float *) db, (const float *) sb, 1000, ret, st);
        hipStreamSynchronize(st);
        int rv = -1;
        hipMemcpy(&rv, ret, sizeof(int), hipMemcpyDeviceToHost);
        if (r || rv) {
            ++errors;
            printf("[%d] FAIL on_stream rc %d ret %d\n", pe, r, rv);
        }
        hipStreamDestroy(st);
        ishmem_free(ret);
    }
    // fcollect (fcollect.cpp:48-62 pattern) and exscan on a stream (exscan.cpp:30-59 closed form).
    {
        const size_t n = 1000;
        std::vector<long> src(n), got(n * npes);
        for (size_t i = 0; i < n; ++i) src[i] = (long) (((long) n << 48) + ((0x80L + pe) << 40) + (0xffL << 32) + (long) i);
        hipMemcpy(sb, src.data(), n * 8, hipMemcpyHostToDevice);
        int r = ishmem_long_fcollect((long *) db, (const long *) sb, n);
        hipMemcpy(got.data(), db, n * 8 * npes, hipMemcpyDeviceToHost);
        for (int j = 0; j < npes && !r; ++j)
            for (size_t i = 0; i < n; ++i)
                if (got[j * n + i] != (long) (((long) n << 48) + ((0x80L + j) << 40) + (0xffL << 32) + (long) i)) r = -1;
        if (r) {
            ++errors;
            printf("[%d] FAIL long_fcollect rc %d\n", pe, r);
        }
        for (size_t i = 0; i < n; ++i) src[i] = (long) pe + (long) i;
        hipMemcpy(sb, src.data(), n * 8, hipMemcpyHostToDevice);
        hipStream_t st;
        hipStreamCreate(&st);
        int *ret = (int *) ishmem_malloc(sizeof(int));
        hipMemset(ret, 0xff, sizeof(int));
        r = ishmemx_long_sum_exscan_on_stream((long *) db, (const long *) sb, n, ret, st);
        hipStreamSynchronize(st);
        int rv = -1;
        hipMemcpy(&rv, ret, sizeof(int), hipMemcpyDeviceToHost);
        hipMemcpy(got.data(), db, n * 8, hipMemcpyDeviceToHost);
        for (size_t i = 0; i < n && !r; ++i) {
            const long a = pe + (long) i, ii = (long) i;
            if (got[i] != a * (a - 1) / 2 - ii * (ii - 1) / 2) r = -1;
        }
        if (r || rv) {
            ++errors;
            printf("[%d] FAIL long_sum_exscan_on_stream rc %d ret %d\n", pe, r, rv);
        }
        hipStreamDestroy(st);
        ishmem_free(ret);
    }
    ishmem_free(db);
    ishmem_free(sb);
    ishmem_barrier_all();
    printf("[%d] %s errors %d\n", pe, errors ? "FAIL" : "PASS", errors);
    ishmem_finalize();
    return errors ? 1 : 0;
}
