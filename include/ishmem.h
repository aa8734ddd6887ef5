/* ishmem_amd — C++ API of the reduction-collective path with the reference's names.
 *
 * Source-compatible with the reduce section of oneapi-src/ishmem's public header
 * (src/ishmem.h:923-1238) and its setup calls (src/ishmem.h:40-86, :1555-1559): every
 *   int ishmem_<TYPENAME>_<op>_reduce([ishmem_team_t team,] TYPE *dest, const TYPE *source,
 *                                      size_t nreduce)
 * and the generic  template <typename T> int ishmem_<op>_reduce([team,] T*, const T*, size_t)
 * are header-only inline wrappers over the C-ABI in ishmem_capi.h (link -lishmem_amd).
 * TYPENAME x op matrix = src/collectives/reduce.cpp:95-417 (bitwise ops on unsigned and
 * fixed-width integer types only; schar bitwise is declared by the reference but never defined,
 * reduce.cpp:97-110, so it is not provided here either).
 *
 * Host-callable.  The stream-ordered variant is in ishmemx.h; the device-callable work-group
 * reductions (the reference's SYCL_EXTERNAL *_work_group overloads) are in ishmemx_device.h.
 */
#ifndef ISHMEM_AMD_ISHMEM_H
#define ISHMEM_AMD_ISHMEM_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <type_traits>

#include "ishmem_capi.h"

/* ---- version, threading (src/ishmem.h:17-26) ---------------------------------------------- */
#define ISHMEM_MAJOR_VERSION ISHMEMI_C_SPEC_MAJOR
#define ISHMEM_MINOR_VERSION ISHMEMI_C_SPEC_MINOR
#define ISHMEM_PATCH_VERSION ISHMEMI_C_SPEC_PATCH
#define ISHMEM_MAX_NAME_LEN  ISHMEMI_C_MAX_NAME_LEN
#define ISHMEM_VENDOR_STRING ISHMEMI_C_VENDOR_STRING

#define ISHMEM_THREAD_SINGLE     ISHMEMI_C_THREAD_SINGLE
#define ISHMEM_THREAD_FUNNELED   ISHMEMI_C_THREAD_FUNNELED
#define ISHMEM_THREAD_SERIALIZED ISHMEMI_C_THREAD_SERIALIZED
#define ISHMEM_THREAD_MULTIPLE   ISHMEMI_C_THREAD_MULTIPLE

typedef int ishmem_team_t; /* src/ishmem.h:61 */
typedef struct {           /* src/ishmem.h:63-65 */
    int num_contexts;
} ishmem_team_config_t;
#define ISHMEM_TEAM_NUM_CONTEXTS 1L
#define ISHMEM_TEAM_INVALID ISHMEMI_C_TEAM_INVALID
#define ISHMEM_TEAM_WORLD   ISHMEMI_C_TEAM_WORLD
#define ISHMEM_TEAM_SHARED  ISHMEMI_C_TEAM_SHARED

/* ---- setup (src/ishmem.h:40-58) ---------------------------------------------------------- */
/* A failed initialisation is fatal, as in the reference: ishmem_init raises the error and exits
 * (src/ishmem.cpp:396-407, RAISE_ERROR_MSG src/ishmem/err.h:105-110), a second ishmem_init too. */
inline void ishmemi_cxx_init_or_exit(void)
{
    if (ishmemi_c_initialized()) {
        fprintf(stderr, "[ishmem_amd] ERROR: Attempt to re-initialize library\n");
        exit(1);
    }
    if (ishmemi_c_init() != 0) {
        fprintf(stderr, "[ishmem_amd] ERROR: ishmem_init failed: %s\n", ishmemi_c_last_error());
        exit(1);
    }
}
inline void ishmem_init(void) { ishmemi_cxx_init_or_exit(); }
inline void ishmem_finalize(void) { (void) ishmemi_c_finalize(); }
inline int ishmem_init_thread(int requested, int *provided)
{
    (void) requested; /* ISHMEM_THREAD_MULTIPLE is always provided (src/ishmem.cpp:409-419) */
    ishmemi_cxx_init_or_exit();
    if (provided) *provided = ISHMEM_THREAD_MULTIPLE;
    return 0;
}
inline void ishmem_query_thread(int *provided) { (void) ishmemi_c_query_thread(provided); }
inline void ishmem_info_get_version(int *major, int *minor)
{
    *major = ISHMEM_MAJOR_VERSION;
    *minor = ISHMEM_MINOR_VERSION;
}
inline void ishmem_info_get_name(char *name)
{
    const char *v = ISHMEM_VENDOR_STRING;
    while (*v) *name++ = *v++;
    *name = '\0';
}
inline int ishmem_my_pe(void) { return ishmemi_c_my_pe(); }
inline int ishmem_n_pes(void) { return ishmemi_c_n_pes(); }
inline void *ishmem_malloc(size_t size) { return ishmemi_c_malloc(size); }
inline void *ishmem_align(size_t alignment, size_t size) { return ishmemi_c_align(alignment, size); }
inline void *ishmem_calloc(size_t count, size_t size) { return ishmemi_c_calloc(count, size); }
inline void ishmem_free(void *ptr) { ishmemi_c_free(ptr); }
inline void *ishmem_ptr(const void *dest, int pe) { return ishmemi_c_ptr(dest, pe); }

/* ---- teams (src/ishmem.h:74-86) ---------------------------------------------------------- */
inline int ishmem_team_my_pe(ishmem_team_t team) { return ishmemi_c_team_my_pe(team); }
inline int ishmem_team_n_pes(ishmem_team_t team) { return ishmemi_c_team_n_pes(team); }
inline int ishmem_team_translate_pe(ishmem_team_t src_team, int src_pe, ishmem_team_t dest_team)
{
    return ishmemi_c_team_translate_pe(src_team, src_pe, dest_team);
}
/* The config / config_mask arguments (src/ishmem.h:78-85): the only option, num_contexts, is
 * stored on the new team and reported by ishmem_team_get_config (contexts do not exist on this
 * path; nothing else depends on it). */
inline int ishmem_team_get_config(ishmem_team_t team, long config_mask, ishmem_team_config_t *config)
{
    return ishmemi_c_team_get_config(team, config_mask, config ? &config->num_contexts : (int *) 0);
}
inline int ishmem_team_split_strided(ishmem_team_t parent_team, int start, int stride, int size,
                                     const ishmem_team_config_t *config, long config_mask,
                                     ishmem_team_t *new_team)
{
    const int r = ishmemi_c_team_split_strided(parent_team, start, stride, size, new_team);
    if (r == 0 && new_team && *new_team != ISHMEM_TEAM_INVALID && config && config_mask)
        return ishmemi_c_team_set_config(*new_team, config_mask, config->num_contexts);
    return r;
}
inline int ishmem_team_split_2d(ishmem_team_t parent_team, int xrange, const ishmem_team_config_t *xaxis_config,
                                long xaxis_mask, ishmem_team_t *xaxis_team,
                                const ishmem_team_config_t *yaxis_config, long yaxis_mask,
                                ishmem_team_t *yaxis_team)
{
    int r = ishmemi_c_team_split_2d(parent_team, xrange, xaxis_team, yaxis_team);
    if (r == 0 && xaxis_team && *xaxis_team != ISHMEM_TEAM_INVALID && xaxis_config && xaxis_mask)
        r = ishmemi_c_team_set_config(*xaxis_team, xaxis_mask, xaxis_config->num_contexts);
    if (r == 0 && yaxis_team && *yaxis_team != ISHMEM_TEAM_INVALID && yaxis_config && yaxis_mask)
        r = ishmemi_c_team_set_config(*yaxis_team, yaxis_mask, yaxis_config->num_contexts);
    return r;
}
inline void ishmem_team_destroy(ishmem_team_t team) { ishmemi_c_team_destroy(team); }

/* ---- synchronisation (src/ishmem.h:1555-1559) -------------------------------------------- */
inline void ishmem_barrier_all(void) { (void) ishmemi_c_barrier_all(); }
inline void ishmem_sync_all(void) { (void) ishmemi_c_sync_all(); }
inline int ishmem_team_sync(ishmem_team_t team) { return ishmemi_c_team_sync(team); }

/* ---- reductions ---------------------------------------------------------------------------- */
namespace ishmemi_cxx {
/* C type -> canonical dtype (the reference's ishmemi_union_get_base_type, src/ishmem/util.h:452-479) */
template <typename T>
constexpr int dtype_of()
{
    static_assert(std::is_arithmetic_v<T> && sizeof(T) <= 8, "unsupported reduction type");
    if constexpr (std::is_same_v<T, float>) return ISHMEMI_DT_FLOAT;
    else if constexpr (std::is_same_v<T, double>) return ISHMEMI_DT_DOUBLE;
    else if constexpr (std::is_signed_v<T>)
        return sizeof(T) == 1 ? ISHMEMI_DT_INT8 : sizeof(T) == 2 ? ISHMEMI_DT_INT16
               : sizeof(T) == 4 ? ISHMEMI_DT_INT32 : ISHMEMI_DT_INT64;
    else
        return sizeof(T) == 1 ? ISHMEMI_DT_UINT8 : sizeof(T) == 2 ? ISHMEMI_DT_UINT16
               : sizeof(T) == 4 ? ISHMEMI_DT_UINT32 : ISHMEMI_DT_UINT64;
}
template <typename T>
inline int reduce(ishmem_team_t team, int op, T *dest, const T *source, size_t nreduce)
{
    return ishmemi_c_reduce(team, op, dtype_of<T>(), (void *) dest, (const void *) source, nreduce);
}
}  // namespace ishmemi_cxx

#define ISHMEMI_CXX_GENERIC(OPNAME, OPC)                                                            \
    template <typename T>                                                                          \
    inline int ishmem_##OPNAME##_reduce(T *dest, const T *source, size_t nreduce)                  \
    {                                                                                              \
        return ishmemi_cxx::reduce<T>(ISHMEM_TEAM_WORLD, OPC, dest, source, nreduce);              \
    }                                                                                              \
    template <typename T>                                                                          \
    inline int ishmem_##OPNAME##_reduce(ishmem_team_t team, T *dest, const T *source,              \
                                        size_t nreduce)                                            \
    {                                                                                              \
        return ishmemi_cxx::reduce<T>(team, OPC, dest, source, nreduce);                           \
    }

ISHMEMI_CXX_GENERIC(and, ISHMEMI_OP_AND)
ISHMEMI_CXX_GENERIC(or, ISHMEMI_OP_OR)
ISHMEMI_CXX_GENERIC(xor, ISHMEMI_OP_XOR)
ISHMEMI_CXX_GENERIC(max, ISHMEMI_OP_MAX)
ISHMEMI_CXX_GENERIC(min, ISHMEMI_OP_MIN)
ISHMEMI_CXX_GENERIC(sum, ISHMEMI_OP_SUM)
ISHMEMI_CXX_GENERIC(prod, ISHMEMI_OP_PROD)

#define ISHMEMI_CXX_TYPED(TYPENAME, TYPE, OPNAME, OPC)                                              \
    inline int ishmem_##TYPENAME##_##OPNAME##_reduce(TYPE *dest, const TYPE *source,               \
                                                     size_t nreduce)                               \
    {                                                                                              \
        return ishmemi_cxx::reduce<TYPE>(ISHMEM_TEAM_WORLD, OPC, dest, source, nreduce);           \
    }                                                                                              \
    inline int ishmem_##TYPENAME##_##OPNAME##_reduce(ishmem_team_t team, TYPE *dest,               \
                                                     const TYPE *source, size_t nreduce)           \
    {                                                                                              \
        return ishmemi_cxx::reduce<TYPE>(team, OPC, dest, source, nreduce);                        \
    }

/* bitwise: src/collectives/reduce.cpp:95-147, :257-309 */
#define ISHMEMI_CXX_BITWISE_TYPES(X, OPNAME, OPC)                                                   \
    X(uchar, unsigned char, OPNAME, OPC)                                                           \
    X(ushort, unsigned short, OPNAME, OPC)                                                         \
    X(uint, unsigned int, OPNAME, OPC)                                                             \
    X(ulong, unsigned long, OPNAME, OPC)                                                           \
    X(ulonglong, unsigned long long, OPNAME, OPC)                                                  \
    X(int8, int8_t, OPNAME, OPC)                                                                   \
    X(int16, int16_t, OPNAME, OPC)                                                                 \
    X(int32, int32_t, OPNAME, OPC)                                                                 \
    X(int64, int64_t, OPNAME, OPC)                                                                 \
    X(uint8, uint8_t, OPNAME, OPC)                                                                 \
    X(uint16, uint16_t, OPNAME, OPC)                                                               \
    X(uint32, uint32_t, OPNAME, OPC)                                                               \
    X(uint64, uint64_t, OPNAME, OPC)                                                               \
    X(size, size_t, OPNAME, OPC)

/* max/min/sum/prod: src/collectives/reduce.cpp:149-255, :311-417 */
#define ISHMEMI_CXX_ARITH_TYPES(X, OPNAME, OPC)                                                     \
    X(char, char, OPNAME, OPC)                                                                     \
    X(schar, signed char, OPNAME, OPC)                                                             \
    X(short, short, OPNAME, OPC)                                                                   \
    X(int, int, OPNAME, OPC)                                                                       \
    X(long, long, OPNAME, OPC)                                                                     \
    X(longlong, long long, OPNAME, OPC)                                                            \
    X(ptrdiff, ptrdiff_t, OPNAME, OPC)                                                             \
    X(uchar, unsigned char, OPNAME, OPC)                                                           \
    X(ushort, unsigned short, OPNAME, OPC)                                                         \
    X(uint, unsigned int, OPNAME, OPC)                                                             \
    X(ulong, unsigned long, OPNAME, OPC)                                                           \
    X(ulonglong, unsigned long long, OPNAME, OPC)                                                  \
    X(int8, int8_t, OPNAME, OPC)                                                                   \
    X(int16, int16_t, OPNAME, OPC)                                                                 \
    X(int32, int32_t, OPNAME, OPC)                                                                 \
    X(int64, int64_t, OPNAME, OPC)                                                                 \
    X(uint8, uint8_t, OPNAME, OPC)                                                                 \
    X(uint16, uint16_t, OPNAME, OPC)                                                               \
    X(uint32, uint32_t, OPNAME, OPC)                                                               \
    X(uint64, uint64_t, OPNAME, OPC)                                                               \
    X(size, size_t, OPNAME, OPC)                                                                   \
    X(float, float, OPNAME, OPC)                                                                   \
    X(double, double, OPNAME, OPC)

ISHMEMI_CXX_BITWISE_TYPES(ISHMEMI_CXX_TYPED, and, ISHMEMI_OP_AND)
ISHMEMI_CXX_BITWISE_TYPES(ISHMEMI_CXX_TYPED, or, ISHMEMI_OP_OR)
ISHMEMI_CXX_BITWISE_TYPES(ISHMEMI_CXX_TYPED, xor, ISHMEMI_OP_XOR)
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_TYPED, max, ISHMEMI_OP_MAX)
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_TYPED, min, ISHMEMI_OP_MIN)
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_TYPED, sum, ISHMEMI_OP_SUM)
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_TYPED, prod, ISHMEMI_OP_PROD)

/* ---- fcollect / collect / scan (src/ishmem.h:894-921 and the scan section) ---- */
inline int ishmem_fcollectmem(void *dest, const void *source, size_t nbytes)
{
    return ishmemi_c_fcollect(ISHMEM_TEAM_WORLD, dest, source, nbytes);
}
inline int ishmem_fcollectmem(ishmem_team_t team, void *dest, const void *source, size_t nbytes)
{
    return ishmemi_c_fcollect(team, dest, source, nbytes);
}
inline int ishmem_collectmem(void *dest, const void *source, size_t nbytes)
{
    return ishmemi_c_collect(ISHMEM_TEAM_WORLD, dest, source, nbytes);
}
inline int ishmem_collectmem(ishmem_team_t team, void *dest, const void *source, size_t nbytes)
{
    return ishmemi_c_collect(team, dest, source, nbytes);
}
template <typename T>
inline int ishmem_fcollect(ishmem_team_t team, T *dest, const T *source, size_t nelems)
{
    return ishmemi_c_fcollect(team, (void *) dest, (const void *) source, nelems * sizeof(T));
}
template <typename T>
inline int ishmem_fcollect(T *dest, const T *source, size_t nelems)
{
    return ishmem_fcollect(ISHMEM_TEAM_WORLD, dest, source, nelems);
}
template <typename T>
inline int ishmem_collect(ishmem_team_t team, T *dest, const T *source, size_t nelems)
{
    return ishmemi_c_collect(team, (void *) dest, (const void *) source, nelems * sizeof(T));
}
template <typename T>
inline int ishmem_collect(T *dest, const T *source, size_t nelems)
{
    return ishmem_collect(ISHMEM_TEAM_WORLD, dest, source, nelems);
}
template <typename T>
inline int ishmem_sum_inscan(ishmem_team_t team, T *dest, const T *source, size_t nelems)
{
    return ishmemi_c_scan(team, ishmemi_cxx::dtype_of<T>(), 1, (void *) dest, (const void *) source, nelems);
}
template <typename T>
inline int ishmem_sum_inscan(T *dest, const T *source, size_t nelems)
{
    return ishmem_sum_inscan(ISHMEM_TEAM_WORLD, dest, source, nelems);
}
template <typename T>
inline int ishmem_sum_exscan(ishmem_team_t team, T *dest, const T *source, size_t nelems)
{
    return ishmemi_c_scan(team, ishmemi_cxx::dtype_of<T>(), 0, (void *) dest, (const void *) source, nelems);
}
template <typename T>
inline int ishmem_sum_exscan(T *dest, const T *source, size_t nelems)
{
    return ishmem_sum_exscan(ISHMEM_TEAM_WORLD, dest, source, nelems);
}

#define ISHMEMI_CXX_COLL_TYPED(TYPENAME, TYPE, UNUSED1, UNUSED2)                                    \
    inline int ishmem_##TYPENAME##_fcollect(TYPE *d, const TYPE *s, size_t n) { return ishmem_fcollect(d, s, n); } \
    inline int ishmem_##TYPENAME##_fcollect(ishmem_team_t t, TYPE *d, const TYPE *s, size_t n)     \
    {                                                                                              \
        return ishmem_fcollect(t, d, s, n);                                                        \
    }                                                                                              \
    inline int ishmem_##TYPENAME##_collect(TYPE *d, const TYPE *s, size_t n) { return ishmem_collect(d, s, n); } \
    inline int ishmem_##TYPENAME##_collect(ishmem_team_t t, TYPE *d, const TYPE *s, size_t n)      \
    {                                                                                              \
        return ishmem_collect(t, d, s, n);                                                         \
    }                                                                                              \
    inline int ishmem_##TYPENAME##_sum_inscan(TYPE *d, const TYPE *s, size_t n) { return ishmem_sum_inscan(d, s, n); } \
    inline int ishmem_##TYPENAME##_sum_inscan(ishmem_team_t t, TYPE *d, const TYPE *s, size_t n)   \
    {                                                                                              \
        return ishmem_sum_inscan(t, d, s, n);                                                      \
    }                                                                                              \
    inline int ishmem_##TYPENAME##_sum_exscan(TYPE *d, const TYPE *s, size_t n) { return ishmem_sum_exscan(d, s, n); } \
    inline int ishmem_##TYPENAME##_sum_exscan(ishmem_team_t t, TYPE *d, const TYPE *s, size_t n)   \
    {                                                                                              \
        return ishmem_sum_exscan(t, d, s, n);                                                      \
    }

/* fcollect / collect / inscan / exscan typename lists = src/collectives/collect.cpp:44-66,
 * :129-151 and scan.cpp:28-74: the same 23 names as max/min/sum/prod. */
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_COLL_TYPED, _, _)

/* ---- broadcast (src/ishmem.h:761-813; the reference's intra-node pull, broadcast_impl.h) ----- */
inline int ishmem_broadcastmem(ishmem_team_t team, void *dest, const void *source, size_t nbytes, int root)
{
    return ishmemi_c_broadcast(team, dest, source, nbytes, root);
}
inline int ishmem_broadcastmem(void *dest, const void *source, size_t nbytes, int root)
{
    return ishmemi_c_broadcast(ISHMEM_TEAM_WORLD, dest, source, nbytes, root);
}
template <typename T>
inline int ishmem_broadcast(ishmem_team_t team, T *dest, const T *source, size_t nelems, int root)
{
    return ishmemi_c_broadcast(team, (void *) dest, (const void *) source, nelems * sizeof(T), root);
}
template <typename T>
inline int ishmem_broadcast(T *dest, const T *source, size_t nelems, int root)
{
    return ishmem_broadcast(ISHMEM_TEAM_WORLD, dest, source, nelems, root);
}
#define ISHMEMI_CXX_BCAST_TYPED(TYPENAME, TYPE, UNUSED1, UNUSED2)                                   \
    inline int ishmem_##TYPENAME##_broadcast(ishmem_team_t t, TYPE *d, const TYPE *s, size_t n, int root) \
    {                                                                                              \
        return ishmem_broadcast(t, d, s, n, root);                                                 \
    }                                                                                              \
    inline int ishmem_##TYPENAME##_broadcast(TYPE *d, const TYPE *s, size_t n, int root)            \
    {                                                                                              \
        return ishmem_broadcast(d, s, n, root);                                                    \
    }
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_BCAST_TYPED, _, _)

/* Compiled as HIP: the device-callable half of this API (the reference's SYCL_EXTERNAL functions:
 * ishmem_my_pe / ishmem_<TN>_<op>_reduce / ... from inside a kernel, ishmemx_*_work_group). */
#if defined(__HIP__)
#include "ishmemx_device.h"
#endif

#endif /* ISHMEM_AMD_ISHMEM_H */
