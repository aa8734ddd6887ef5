/* ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).  Plain C restatement of the reference's
 * reduction semantics; each function cites the reference file:line it follows. */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <pthread.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

/* ISHMEM_REDUCE_BUFFER_SIZE, src/collectives.h:10 */
#define REDUCE_BUFFER_SIZE (1L << 16)

size_t oracle_dtype_size(int dt)
{
    static const size_t sz[] = {1, 2, 4, 8, 1, 2, 4, 8, 4, 8};
    return (dt >= 0 && dt <= OD_DOUBLE) ? sz[dt] : 0;
}

/* docs/source/collectives.rst:910-936: bitwise ops on integer types only. */
int oracle_valid(int op, int dt)
{
    if (op < OR_AND || op > OR_PROD || dt < OD_INT8 || dt > OD_DOUBLE) return 0;
    if ((dt == OD_FLOAT || dt == OD_DOUBLE) && op <= OR_XOR) return 0;
    return 1;
}

/* reduce_op<T,OP> (src/collectives/reduce_impl.h:83-102).  FP max/min are sycl::fmax/fmin
 * (= C fmax/fmin); integer + and * wrap modulo 2^bits (done on unsigned to avoid C UB, which
 * gives the two's-complement bits the device computes). */
#define INT_CASES(T, UT)                                                                           \
    {                                                                                              \
        T *d = (T *) dst;                                                                          \
        const T *s = (const T *) src;                                                              \
        for (size_t i = 0; i < n; ++i) {                                                           \
            switch (op) {                                                                          \
                case OR_AND: d[i] = (T) (d[i] & s[i]); break;                                      \
                case OR_OR: d[i] = (T) (d[i] | s[i]); break;                                       \
                case OR_XOR: d[i] = (T) (d[i] ^ s[i]); break;                                      \
                case OR_MAX: d[i] = (d[i] < s[i]) ? s[i] : d[i]; break;                            \
                case OR_MIN: d[i] = (s[i] < d[i]) ? s[i] : d[i]; break;                            \
                case OR_SUM: d[i] = (T) (UT) ((uint64_t) (UT) d[i] + (uint64_t) (UT) s[i]); break; \
                case OR_PROD: d[i] = (T) (UT) ((uint64_t) (UT) d[i] * (uint64_t) (UT) s[i]); break;\
            }                                                                                      \
        }                                                                                          \
    }                                                                                              \
    break;

#define FP_CASES(T, MAXF, MINF)                                                                    \
    {                                                                                              \
        T *d = (T *) dst;                                                                          \
        const T *s = (const T *) src;                                                              \
        for (size_t i = 0; i < n; ++i) {                                                           \
            switch (op) {                                                                          \
                case OR_MAX: d[i] = MAXF(d[i], s[i]); break;                                       \
                case OR_MIN: d[i] = MINF(d[i], s[i]); break;                                       \
                case OR_SUM: d[i] = d[i] + s[i]; break;                                            \
                case OR_PROD: d[i] = d[i] * s[i]; break;                                           \
            }                                                                                      \
        }                                                                                          \
    }                                                                                              \
    break;

int oracle_combine(int op, int dt, void *dst, const void *src, size_t n)
{
    if (!oracle_valid(op, dt)) return 1;
    switch (dt) {
        case OD_INT8: INT_CASES(int8_t, uint8_t)
        case OD_INT16: INT_CASES(int16_t, uint16_t)
        case OD_INT32: INT_CASES(int32_t, uint32_t)
        case OD_INT64: INT_CASES(int64_t, uint64_t)
        case OD_UINT8: INT_CASES(uint8_t, uint8_t)
        case OD_UINT16: INT_CASES(uint16_t, uint16_t)
        case OD_UINT32: INT_CASES(uint32_t, uint32_t)
        case OD_UINT64: INT_CASES(uint64_t, uint64_t)
        case OD_FLOAT: FP_CASES(float, fmaxf, fminf)
        case OD_DOUBLE: FP_CASES(double, fmax, fmin)
    }
    return 0;
}

/* vec_copy_push(dest, source) then ishmemi_sub_reduce: fold every other PE in team order
 * (src/collectives/reduce_impl.h:247-253, :288-289). */
int oracle_reduce_fold(int op, int dt, const void *const *srcs, int npes, int me, void *dst,
                       size_t n)
{
    if (!oracle_valid(op, dt) || npes < 1 || me < 0 || me >= npes) return 1;
    const size_t es = oracle_dtype_size(dt);
    memmove(dst, srcs[me], n * es);
    for (int pe = 0; pe < npes; ++pe) {
        if (pe == me) continue;
        oracle_combine(op, dt, dst, srcs[pe], n);
    }
    return 0;
}

/* ishmemi_generic_op_reduce (src/collectives/reduce_impl.h:186-228) with the MPI runtime's
 * reduce (src/runtime/runtime_mpi.cpp:802-812) restated as a rank-order fold. */
int oracle_host_proxy_reduce(int op, int dt, const void *const *srcs, void *const *dsts, int npes,
                             size_t n)
{
    if (!oracle_valid(op, dt) || npes < 1) return 1;
    const size_t es = oracle_dtype_size(dt);
    const size_t max_reduce = REDUCE_BUFFER_SIZE / es;
    char *bounce_src = malloc((size_t) npes * REDUCE_BUFFER_SIZE);
    char *bounce_dst = malloc(REDUCE_BUFFER_SIZE);
    if (!bounce_src || !bounce_dst) {
        free(bounce_src);
        free(bounce_dst);
        return 1;
    }
    for (size_t off = 0; off < n; off += max_reduce) {
        const size_t m = (n - off < max_reduce) ? n - off : max_reduce;
        for (int pe = 0; pe < npes; ++pe) /* ishmemi_copy(team.source <- src chunk), :196 */
            memcpy(bounce_src + (size_t) pe * REDUCE_BUFFER_SIZE,
                   (const char *) srcs[pe] + off * es, m * es);
        /* MPI_Allreduce(team.source -> team.dest) */
        memcpy(bounce_dst, bounce_src, m * es);
        for (int pe = 1; pe < npes; ++pe)
            oracle_combine(op, dt, bounce_dst, bounce_src + (size_t) pe * REDUCE_BUFFER_SIZE, m);
        for (int pe = 0; pe < npes; ++pe) /* ishmemi_copy(dest chunk <- team.dest), :218 */
            memcpy((char *) dsts[pe] + off * es, bounce_dst, m * es);
    }
    free(bounce_src);
    free(bounce_dst);
    return 0;
}

/* ---------------------------------------------------------------------------------------------
 * Multi-process timing harness of the host-proxy path (reported CPU baseline, not a target).
 * ------------------------------------------------------------------------------------------- */
static double wall(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double) ts.tv_sec + 1e-9 * (double) ts.tv_nsec;
}

struct shm_ctl {
    pthread_barrier_t bar;
    double best;
    int failed;
};

double oracle_host_proxy_time(int op, int dt, size_t n, int npes, int reps)
{
    if (!oracle_valid(op, dt) || npes < 1 || reps < 1) return -1.0;
    const size_t es = oracle_dtype_size(dt);
    const size_t chunk = REDUCE_BUFFER_SIZE / es;
    const size_t arr = ((n * es + 4095) / 4096) * 4096;
    const size_t total = 4096 + (size_t) npes * 2 * arr + (size_t) npes * REDUCE_BUFFER_SIZE +
                         REDUCE_BUFFER_SIZE;
    char *base = mmap(NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (base == MAP_FAILED) return -1.0;
    struct shm_ctl *ctl = (struct shm_ctl *) base;
    pthread_barrierattr_t ba;
    pthread_barrierattr_init(&ba);
    pthread_barrierattr_setpshared(&ba, PTHREAD_PROCESS_SHARED);
    pthread_barrier_init(&ctl->bar, &ba, (unsigned) npes);
    ctl->best = 1e30;
    ctl->failed = 0;
    char *src0 = base + 4096;
    char *dst0 = src0 + (size_t) npes * arr;
    char *bsrc = dst0 + (size_t) npes * arr;
    char *bres = bsrc + (size_t) npes * REDUCE_BUFFER_SIZE;
    for (int pe = 0; pe < npes; ++pe)
        oracle_fill_random(dt, 0x15AE0001ull + (uint64_t) pe, 0.5, 2.0, n, src0 + (size_t) pe * arr);

    pid_t kids[64];
    int nk = 0;
    int me = 0;
    for (int pe = 1; pe < npes && pe < 64; ++pe) {
        pid_t k = fork();
        if (k == 0) {
            prctl(PR_SET_PDEATHSIG, SIGKILL);
            me = pe;
            break;
        }
        kids[nk++] = k;
    }
    char *src = src0 + (size_t) me * arr, *dst = dst0 + (size_t) me * arr;
    char *mybounce = bsrc + (size_t) me * REDUCE_BUFFER_SIZE;
    for (int r = 0; r < reps; ++r) {
        pthread_barrier_wait(&ctl->bar);
        const double t0 = wall();
        for (size_t off = 0; off < n; off += chunk) {
            const size_t m = (n - off < chunk) ? n - off : chunk;
            memcpy(mybounce, src + off * es, m * es); /* device -> host bounce */
            pthread_barrier_wait(&ctl->bar);
            /* MPI shared-memory allreduce: reduce-scatter over the PEs' bounce buffers ... */
            const size_t part = (m + (size_t) npes - 1) / (size_t) npes;
            const size_t lo = (size_t) me * part < m ? (size_t) me * part : m;
            const size_t hi = lo + part < m ? lo + part : m;
            if (hi > lo) {
                memcpy(bres + lo * es, bsrc + lo * es, (hi - lo) * es);
                for (int pe = 1; pe < npes; ++pe)
                    oracle_combine(op, dt, bres + lo * es,
                                   bsrc + (size_t) pe * REDUCE_BUFFER_SIZE + lo * es, hi - lo);
            }
            pthread_barrier_wait(&ctl->bar);
            memcpy(dst + off * es, bres, m * es); /* ... all-gather, host bounce -> device */
            pthread_barrier_wait(&ctl->bar);
        }
        const double t1 = wall();
        if (me == 0 && t1 - t0 < ctl->best) ctl->best = t1 - t0;
    }
    if (me != 0) _exit(0);
    for (int i = 0; i < nk; ++i) waitpid(kids[i], NULL, 0);
    const double best = ctl->best;
    pthread_barrier_destroy(&ctl->bar);
    munmap(base, total);
    return best;
}

/* ---------------------------------------------------------------------------------------------
 * The reference's host path INCLUDING its device copies, for the CPU baseline: each PE is a
 * process of its own (the caller), its source / dest are device memory, and every 64 KiB chunk
 * goes through a synchronous device->host copy into this PE's bounce buffer
 * (ishmemi_copy(team.source, src), src/collectives/reduce_impl.h:196 -> src/memory.cpp:310-321,
 * a synchronous immediate command list), the MPI shared-memory allreduce of the p bounce buffers
 * (runtime_mpi.cpp:802-812: reduce-scatter + all-gather through shared memory, restated as
 * above), and a synchronous host->device copy back (:218).  The copies go through `copy_fn`,
 * which the caller binds to hipMemcpy (kind 2 = device->host, 1 = host->device), so this file
 * stays free of any GPU header.  The p processes meet in a POSIX shared-memory segment named by
 * `key`; member 0 creates it.  Returns this member's best seconds over `reps`; < 0 on failure.
 * ------------------------------------------------------------------------------------------- */
#include <errno.h>
#include <fcntl.h>
#include <stdio.h>
#include <sys/stat.h>

struct bounce_ctl {
    int magic, count, gen, pad;
};
#define BOUNCE_MAGIC 0x1B0C0E5

/* Shared-memory spin barrier (what an MPI shared-memory transport polls), bounded: returns
 * nonzero if the other members do not arrive within 60 s (a member that died). */
static int bounce_barrier(struct bounce_ctl *c, int npes)
{
    const int g = __atomic_load_n(&c->gen, __ATOMIC_ACQUIRE);
    if (__atomic_fetch_add(&c->count, 1, __ATOMIC_ACQ_REL) == npes - 1) {
        __atomic_store_n(&c->count, 0, __ATOMIC_RELAXED);
        __atomic_fetch_add(&c->gen, 1, __ATOMIC_RELEASE);
        return 0;
    }
    const double t0 = wall();
    for (unsigned it = 0; __atomic_load_n(&c->gen, __ATOMIC_ACQUIRE) == g; ++it)
        if ((it & 1023) == 1023 && wall() - t0 > 60.0) return 1;
    return 0;
}

double oracle_host_bounce_time(int op, int dt, size_t n, int me, int npes, const char *key,
                               const void *dev_src, void *dev_dst, oracle_copy_fn copy_fn,
                               int reps)
{
    if (!oracle_valid(op, dt) || npes < 1 || me < 0 || me >= npes || reps < 1 || !copy_fn || !key)
        return -1.0;
    const size_t es = oracle_dtype_size(dt);
    const size_t chunk = REDUCE_BUFFER_SIZE / es;
    const size_t total = 4096 + (size_t) npes * REDUCE_BUFFER_SIZE + REDUCE_BUFFER_SIZE;
    char name[256];
    snprintf(name, sizeof(name), "/ishmem_oracle_bounce_%s", key);
    int fd = -1;
    const double t_attach = wall();
    if (me == 0) {
        shm_unlink(name);
        fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd < 0 || ftruncate(fd, (off_t) total) != 0) return -2.0;
    } else {
        while ((fd = shm_open(name, O_RDWR, 0600)) < 0) {
            if (wall() - t_attach > 60.0) return -3.0;
            usleep(1000);
        }
        struct stat st;
        while (fstat(fd, &st) == 0 && (size_t) st.st_size < total) {
            if (wall() - t_attach > 60.0) return -3.0;
            usleep(1000);
        }
    }
    char *base = mmap(NULL, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (base == MAP_FAILED) return -4.0;
    struct bounce_ctl *ctl = (struct bounce_ctl *) base;
    if (me == 0) {
        ctl->count = 0;
        ctl->gen = 0;
        __atomic_store_n(&ctl->magic, BOUNCE_MAGIC, __ATOMIC_RELEASE);
    } else {
        while (__atomic_load_n(&ctl->magic, __ATOMIC_ACQUIRE) != BOUNCE_MAGIC) {
            if (wall() - t_attach > 60.0) {
                munmap(base, total);
                return -3.0;
            }
            usleep(1000);
        }
    }
    char *bsrc = base + 4096;
    char *bres = bsrc + (size_t) npes * REDUCE_BUFFER_SIZE;
    char *mine = bsrc + (size_t) me * REDUCE_BUFFER_SIZE;
    double best = 1e30;
    int failed = 0;
    for (int r = 0; r < reps && !failed; ++r) {
        failed |= bounce_barrier(ctl, npes);
        const double t0 = wall();
        for (size_t off = 0; off < n && !failed; off += chunk) {
            const size_t m = (n - off < chunk) ? n - off : chunk;
            failed |= copy_fn(mine, (const char *) dev_src + off * es, m * es, 2) != 0;
            failed |= bounce_barrier(ctl, npes);
            const size_t part = (m + (size_t) npes - 1) / (size_t) npes;
            const size_t lo = (size_t) me * part < m ? (size_t) me * part : m;
            const size_t hi = lo + part < m ? lo + part : m;
            if (hi > lo) {
                memcpy(bres + lo * es, bsrc + lo * es, (hi - lo) * es);
                for (int pe = 1; pe < npes; ++pe)
                    oracle_combine(op, dt, bres + lo * es,
                                   bsrc + (size_t) pe * REDUCE_BUFFER_SIZE + lo * es, hi - lo);
            }
            failed |= bounce_barrier(ctl, npes);
            failed |= copy_fn((char *) dev_dst + off * es, bres, m * es, 1) != 0;
            failed |= bounce_barrier(ctl, npes);
        }
        const double t1 = wall();
        if (t1 - t0 < best) best = t1 - t0;
    }
    if (!failed) failed |= bounce_barrier(ctl, npes);
    if (me == 0) shm_unlink(name);
    munmap(base, total);
    return failed ? -5.0 : best;
}

/* ---------------------------------------------------------------------------------------------
 * Reference known-answer patterns.
 * ------------------------------------------------------------------------------------------- */

/* Integer source word of the arithmetic tests (test/unit/reduce_sum.cpp:180-189; identical in
 * reduce_prod.cpp / reduce_min.cpp / reduce_max.cpp). */
static uint64_t arith_word(int pe, size_t idx)
{
    const size_t m = (size_t) pe + 2;
    return ((uint64_t) (idx % m) << 48) + ((uint64_t) ((idx + 1) % m) << 40) +
           ((uint64_t) ((idx + 2) % m) << 32) + (uint64_t) ((idx + 3) % m);
}

/* Bitwise tests' source word (test/unit/reduce_and.cpp:34-37, reduce_or.cpp, reduce_xor.cpp). */
static uint64_t bitwise_word(int pe, size_t nelems, size_t idx)
{
    return ((uint64_t) nelems << 48) + ((uint64_t) (0x80L + pe) << 40) + ((uint64_t) 0xffL << 32) +
           (uint64_t) idx;
}

static double arith_fp(int pe, size_t idx) { return ((double) pe) * 100.0 + ((double) idx / 128.0); }

int oracle_pattern_source(int family, int dt, int pe, size_t nelems, void *out)
{
    const size_t es = oracle_dtype_size(dt);
    if (!es) return 1;
    if (family == PAT_ARITH && dt == OD_FLOAT) {
        for (size_t i = 0; i < nelems; ++i) ((float *) out)[i] = (float) arith_fp(pe, i);
        return 0;
    }
    if (family == PAT_ARITH && dt == OD_DOUBLE) {
        for (size_t i = 0; i < nelems; ++i) ((double *) out)[i] = arith_fp(pe, i);
        return 0;
    }
    const size_t words = (nelems * es) / 8 + 1;
    uint64_t *w = malloc(words * 8);
    if (!w) return 1;
    for (size_t idx = 0; idx < words; ++idx)
        w[idx] = family == PAT_ARITH ? arith_word(pe, idx) : bitwise_word(pe, nelems, idx);
    memcpy(out, w, nelems * es);
    free(w);
    return 0;
}

/* tsum/tprod/tmin/tmax of the testers (e.g. test/unit/reduce_sum.cpp:13-136): lane `lane` of
 * the two 64-bit words as type dt, combined, truncated to the lane width. */
static uint64_t lane_op(uint64_t a, uint64_t b, int op, int dt, size_t lane)
{
    const size_t es = oracle_dtype_size(dt);
    unsigned char ra[8], rb[8];
    memcpy(ra, &a, 8);
    memcpy(rb, &b, 8);
    unsigned char res[8] = {0};
    oracle_combine(op, dt, ra + lane * es, rb + lane * es, 1);
    memcpy(res, ra + lane * es, es);
    uint64_t r = 0;
    memcpy(&r, res, 8);
    return r;
}

int oracle_pattern_check(int family, int op, int dt, int npes, size_t nelems, void *out)
{
    const size_t es = oracle_dtype_size(dt);
    if (!oracle_valid(op, dt) || npes < 1) return 1;
    if (family == PAT_ARITH && (dt == OD_FLOAT || dt == OD_DOUBLE)) {
        /* reduce_sum.cpp:203-224 / reduce_prod.cpp / reduce_min.cpp / reduce_max.cpp: start from
         * 0 (sum) / 1 (prod) / PE 0's value (min, max) and fold PEs in order, in T. */
        for (size_t idx = 0; idx < nelems; ++idx) {
            if (dt == OD_FLOAT) {
                float acc = op == OR_SUM ? 0.0f : op == OR_PROD ? 1.0f : (float) arith_fp(0, idx);
                for (int i = (op == OR_SUM || op == OR_PROD) ? 0 : 1; i < npes; ++i) {
                    float v = (float) arith_fp(i, idx);
                    if (op == OR_SUM) acc += v;
                    else if (op == OR_PROD) acc *= v;
                    else if (op == OR_MIN) acc = (v < acc) ? v : acc; /* std::min */
                    else acc = (acc < v) ? v : acc;                   /* std::max */
                }
                ((float *) out)[idx] = acc;
            } else {
                double acc = op == OR_SUM ? 0.0 : op == OR_PROD ? 1.0 : arith_fp(0, idx);
                for (int i = (op == OR_SUM || op == OR_PROD) ? 0 : 1; i < npes; ++i) {
                    double v = arith_fp(i, idx);
                    if (op == OR_SUM) acc += v;
                    else if (op == OR_PROD) acc *= v;
                    else if (op == OR_MIN) acc = (v < acc) ? v : acc;
                    else acc = (acc < v) ? v : acc;
                }
                ((double *) out)[idx] = acc;
            }
        }
        return 0;
    }
    const size_t words = (nelems * es) / 8 + 1;
    uint64_t *w = malloc(words * 8);
    if (!w) return 1;
    if (family == PAT_ARITH) {
        /* reduce_sum.cpp:225-258: per 64-bit word, per lane j, fold the PEs' lanes with tsum. */
        const size_t lanes = 8 / es;
        for (size_t idx = 0; idx < words; ++idx) {
            uint64_t expected = 0;
            for (size_t j = 0; j < lanes; ++j) {
                const size_t lane = lanes - (j + 1);
                uint64_t mask = (es == 8) ? ~0ull : (((1ull << (es * 8)) - 1) << (lane * es * 8));
                uint64_t cur = arith_word(0, idx);
                for (int i = 1; i < npes; ++i) {
                    cur = lane_op(cur, arith_word(i, idx), op, dt, lane);
                    cur <<= lane * es * 8;
                }
                expected |= cur & mask;
            }
            w[idx] = expected;
        }
    } else {
        /* reduce_and.cpp:48-63 / reduce_or.cpp / reduce_xor.cpp:49-71 */
        uint64_t a = nelems, b = 0x80, c = 0xff;
        for (int i = 1; i < npes; ++i) {
            if (family == PAT_AND) b &= (uint64_t) (0x80 + i);
            else if (family == PAT_OR) b |= (uint64_t) (0x80 + i);
            else {
                a ^= nelems;
                b ^= (uint64_t) (0x80 + i);
                c ^= 0xff;
            }
        }
        for (size_t idx = 0; idx < words; ++idx) {
            uint64_t d = idx;
            if (family == PAT_XOR)
                for (int i = 1; i < npes; ++i) d ^= idx;
            w[idx] = (a << 48) + (b << 40) + (c << 32) + d;
        }
    }
    memcpy(out, w, nelems * es);
    free(w);
    return 0;
}

static uint64_t xs64(uint64_t *s)
{
    uint64_t x = *s;
    x ^= x >> 12;
    x ^= x << 25;
    x ^= x >> 27;
    *s = x;
    return x * 0x2545F4914F6CDD1Dull;
}

void oracle_fill_random(int dt, uint64_t seed, double lo, double hi, size_t n, void *out)
{
    uint64_t s = seed ? seed : 0x9E3779B97F4A7C15ull;
    const size_t es = oracle_dtype_size(dt);
    for (size_t i = 0; i < n; ++i) {
        const uint64_t r = xs64(&s);
        if (dt == OD_FLOAT) {
            ((float *) out)[i] = (float) (lo + (hi - lo) * ((double) (r >> 11) * 0x1.0p-53));
        } else if (dt == OD_DOUBLE) {
            ((double *) out)[i] = lo + (hi - lo) * ((double) (r >> 11) * 0x1.0p-53);
        } else {
            memcpy((char *) out + i * es, &r, es);
        }
    }
}
