/* ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's reduction-collective semantics (oneapi-src/ishmem v1.5.1),
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the CHECKER.  The
 * product path (ishmem_amd/libishmem_amd.so) never links, loads or calls anything here.
 *
 * Parity pinning:
 *   1. oracle_pattern_{source,check} restate the reference's own known-answer generators
 *      (test/unit/reduce_{sum,prod,min,max,and,or,xor}.cpp create_*_pattern); the oracle's fold
 *      of the source patterns must equal the reference's check pattern (tests/test_oracle.py).
 *   2. tests/golden/golden_np<N>.npz hold MPI_Allreduce outputs of MPICH 3.3.2 (the arithmetic backend the
 *      reference's host path calls, src/runtime/runtime_mpi.cpp:802-812) produced by
 *      oracle/mpi_golden.c on the reference patterns and seeded inputs; the oracle must agree.
 * The reference itself (SYCL + Level Zero) cannot be compiled in this image.
 *
 * Enum values are those of include/ishmem_capi.h (op: AND..PROD = 0..6; dtype: INT8..DOUBLE).
 */
#ifndef ISHMEM_AMD_ORACLE_H
#define ISHMEM_AMD_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { OR_AND = 0, OR_OR, OR_XOR, OR_MAX, OR_MIN, OR_SUM, OR_PROD };
enum {
    OD_INT8 = 0, OD_INT16, OD_INT32, OD_INT64, OD_UINT8, OD_UINT16, OD_UINT32, OD_UINT64,
    OD_FLOAT, OD_DOUBLE
};
/* Pattern families of the reference tests. */
enum { PAT_ARITH = 0, PAT_AND = 1, PAT_OR = 2, PAT_XOR = 3 };

size_t oracle_dtype_size(int dt);
int oracle_valid(int op, int dt);

/* dst[i] = reduce_op(dst[i], src[i]) — src/collectives/reduce_impl.h:83-102 */
int oracle_combine(int op, int dt, void *dst, const void *src, size_t n);

/* The reference's device fold for PE `me` (src/collectives/reduce_impl.h:288-289 then
 * ishmemi_sub_reduce :232-256): dst = srcs[me]; for pe in team order, pe != me: combine. */
int oracle_reduce_fold(int op, int dt, const void *const *srcs, int npes, int me, void *dst,
                       size_t n);

/* The reference's host path (src/collectives/reduce_impl.h:186-228): 64 KiB chunks
 * (src/collectives.h:10), each copied to a bounce buffer, all-reduced across PEs with
 * MPI_Allreduce semantics (rank-order fold), copied back.  Writes the result for every PE into
 * dsts[pe] (host memory). */
int oracle_host_proxy_reduce(int op, int dt, const void *const *srcs, void *const *dsts, int npes,
                             size_t n);

/* Multi-process timing of the host-proxy path restatement: `npes` processes (fork) over shared
 * memory, 64 KiB chunks: memcpy in -> reduce-scatter + all-gather fold through shared bounce
 * buffers (the MPI shared-memory allreduce) -> memcpy out.  Returns best wall seconds over
 * `reps` repetitions of one reduce of n elements; -1 on failure. */
double oracle_host_proxy_time(int op, int dt, size_t n, int npes, int reps);

/* The same host path with its real device copies (CPU baseline of bench.py): called by each of
 * `npes` processes (member `me`, rendezvous by `key`) on its own DEVICE source / dest; every
 * 64 KiB chunk is copied device->host with copy_fn(dst, src, bytes, 2), all-reduced through
 * shared memory, and copied host->device with copy_fn(dst, src, bytes, 1) — both synchronous,
 * like ishmemi_copy (src/memory.cpp:310-321).  copy_fn is hipMemcpy, bound by the caller.
 * Returns this member's best wall seconds over `reps`; < 0 on failure. */
typedef int (*oracle_copy_fn)(void *dst, const void *src, size_t bytes, int kind);
double oracle_host_bounce_time(int op, int dt, size_t n, int me, int npes, const char *key,
                               const void *dev_src, void *dev_dst, oracle_copy_fn copy_fn,
                               int reps);

/* Reference known-answer patterns (test/unit/reduce_*.cpp).  `out` receives nelems elements
 * (nelems * size bytes, built from the 64-bit word pattern exactly like the tester). */
int oracle_pattern_source(int family, int dt, int pe, size_t nelems, void *out);
int oracle_pattern_check(int family, int op, int dt, int npes, size_t nelems, void *out);

/* xorshift64* fill (SURVEY.md §8d seeds): ints full range, fp uniform [lo, hi). */
void oracle_fill_random(int dt, uint64_t seed, double lo, double hi, size_t n, void *out);

#ifdef __cplusplus
}
#endif
#endif
