/* ishmem_amd — extension API of the reduction path (reference: src/ishmemx.h).
 *
 * The reference's queue-ordered variant
 *   sycl::event ishmemx_<TYPENAME>_<op>_reduce_on_queue([team,] dest, source, nreduce, int *ret,
 *                                                       sycl::queue &q, deps = {})
 * (src/ishmemx.h:1172-1803, src/collectives/reduce_impl.h:444-474) becomes the HIP-stream
 * variant below: enqueue on `stream`, return immediately (0 = enqueued); *ret (device-visible
 * int, may be nullptr) is zeroed in stream order at the call's start and set nonzero by any of the
 * call's launches that fails, so it reads 0 after completion exactly when the call succeeded.
 * The reference's `deps` and returned sycl::event map to the overloads taking
 * (const hipEvent_t *deps, size_t ndeps, hipEvent_t done): the call waits for every dep and
 * records `done` (if not NULL) after its last launch.
 */
#ifndef ISHMEM_AMD_ISHMEMX_H
#define ISHMEM_AMD_ISHMEMX_H

#include "ishmem.h"

#define ISHMEMX_TEAM_NODE ISHMEMI_C_TEAM_NODE /* src/ishmemx.h:11 */

/* After a device-side timeout, all PEs agree on the teams' epochs again (collective over all PEs;
 * no reference counterpart — the reference aborts, src/proxy.cpp:79-84). */
inline int ishmemx_resync(void) { return ishmemi_c_resync(); }

#ifndef __HIP__
typedef struct ihipStream_t *hipStream_t; /* identical to HIP's own typedefs */
typedef struct ihipEvent_t *hipEvent_t;
#endif

namespace ishmemi_cxx {
template <typename T>
inline int reduce_on_stream(ishmem_team_t team, int op, T *dest, const T *source, size_t nreduce,
                            int *ret, hipStream_t stream)
{
    return ishmemi_c_reduce_on_stream(team, op, dtype_of<T>(), (void *) dest, (const void *) source,
                                      nreduce, ret, (void *) stream);
}
template <typename T>
inline int reduce_on_stream(ishmem_team_t team, int op, T *dest, const T *source, size_t nreduce,
                            int *ret, hipStream_t stream, const hipEvent_t *deps, size_t ndeps,
                            hipEvent_t done)
{
    return ishmemi_c_reduce_on_stream_deps(team, op, dtype_of<T>(), (void *) dest,
                                           (const void *) source, nreduce, ret, (void *) stream,
                                           (void *const *) deps, ndeps, (void *) done);
}
}  // namespace ishmemi_cxx

/* Generic forms, as the reference's template <typename T> ishmemx_<op>_reduce_on_queue
 * (src/ishmemx.h:1173, :1191 and the same for every op). */
#define ISHMEMI_CXX_GENERIC_ON_STREAM(OPNAME, OPC)                                                  \
    template <typename T>                                                                          \
    inline int ishmemx_##OPNAME##_reduce_on_stream(T *dest, const T *source, size_t nreduce,        \
                                                   int *ret, hipStream_t stream)                   \
    {                                                                                              \
        return ishmemi_cxx::reduce_on_stream<T>(ISHMEM_TEAM_WORLD, OPC, dest, source, nreduce, ret, \
                                                stream);                                           \
    }                                                                                              \
    template <typename T>                                                                          \
    inline int ishmemx_##OPNAME##_reduce_on_stream(ishmem_team_t team, T *dest, const T *source,    \
                                                   size_t nreduce, int *ret, hipStream_t stream)   \
    {                                                                                              \
        return ishmemi_cxx::reduce_on_stream<T>(team, OPC, dest, source, nreduce, ret, stream);     \
    }                                                                                              \
    template <typename T>                                                                          \
    inline int ishmemx_##OPNAME##_reduce_on_stream(ishmem_team_t team, T *dest, const T *source,    \
                                                   size_t nreduce, int *ret, hipStream_t stream,   \
                                                   const hipEvent_t *deps, size_t ndeps,           \
                                                   hipEvent_t done)                                \
    {                                                                                              \
        return ishmemi_cxx::reduce_on_stream<T>(team, OPC, dest, source, nreduce, ret, stream,      \
                                                deps, ndeps, done);                                \
    }

ISHMEMI_CXX_GENERIC_ON_STREAM(and, ISHMEMI_OP_AND)
ISHMEMI_CXX_GENERIC_ON_STREAM(or, ISHMEMI_OP_OR)
ISHMEMI_CXX_GENERIC_ON_STREAM(xor, ISHMEMI_OP_XOR)
ISHMEMI_CXX_GENERIC_ON_STREAM(max, ISHMEMI_OP_MAX)
ISHMEMI_CXX_GENERIC_ON_STREAM(min, ISHMEMI_OP_MIN)
ISHMEMI_CXX_GENERIC_ON_STREAM(sum, ISHMEMI_OP_SUM)
ISHMEMI_CXX_GENERIC_ON_STREAM(prod, ISHMEMI_OP_PROD)

#define ISHMEMI_CXX_ON_STREAM(TYPENAME, TYPE, OPNAME, OPC)                                          \
    inline int ishmemx_##TYPENAME##_##OPNAME##_reduce_on_stream(                                   \
        TYPE *dest, const TYPE *source, size_t nreduce, int *ret, hipStream_t stream)              \
    {                                                                                              \
        return ishmemi_cxx::reduce_on_stream<TYPE>(ISHMEM_TEAM_WORLD, OPC, dest, source, nreduce,  \
                                                   ret, stream);                                   \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_##OPNAME##_reduce_on_stream(                                   \
        ishmem_team_t team, TYPE *dest, const TYPE *source, size_t nreduce, int *ret,              \
        hipStream_t stream)                                                                        \
    {                                                                                              \
        return ishmemi_cxx::reduce_on_stream<TYPE>(team, OPC, dest, source, nreduce, ret, stream); \
    }                                                                                              \
    /* the reference's `deps` / returned event: wait for deps[0..ndeps), then record `done` */     \
    inline int ishmemx_##TYPENAME##_##OPNAME##_reduce_on_stream(                                   \
        ishmem_team_t team, TYPE *dest, const TYPE *source, size_t nreduce, int *ret,              \
        hipStream_t stream, const hipEvent_t *deps, size_t ndeps, hipEvent_t done)                 \
    {                                                                                              \
        return ishmemi_cxx::reduce_on_stream<TYPE>(team, OPC, dest, source, nreduce, ret, stream,  \
                                                   deps, ndeps, done);                             \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_##OPNAME##_reduce_on_stream(                                   \
        TYPE *dest, const TYPE *source, size_t nreduce, int *ret, hipStream_t stream,              \
        const hipEvent_t *deps, size_t ndeps, hipEvent_t done)                                     \
    {                                                                                              \
        return ishmemi_cxx::reduce_on_stream<TYPE>(ISHMEM_TEAM_WORLD, OPC, dest, source, nreduce,  \
                                                   ret, stream, deps, ndeps, done);                \
    }

ISHMEMI_CXX_BITWISE_TYPES(ISHMEMI_CXX_ON_STREAM, and, ISHMEMI_OP_AND)
ISHMEMI_CXX_BITWISE_TYPES(ISHMEMI_CXX_ON_STREAM, or, ISHMEMI_OP_OR)
ISHMEMI_CXX_BITWISE_TYPES(ISHMEMI_CXX_ON_STREAM, xor, ISHMEMI_OP_XOR)
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_ON_STREAM, max, ISHMEMI_OP_MAX)
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_ON_STREAM, min, ISHMEMI_OP_MIN)
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_ON_STREAM, sum, ISHMEMI_OP_SUM)
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_ON_STREAM, prod, ISHMEMI_OP_PROD)

/* fcollect / collect / scan on a stream (src/ishmemx.h fcollect/collect/inscan/exscan _on_queue). */
inline int ishmemx_fcollectmem_on_stream(ishmem_team_t team, void *dest, const void *source,
                                         size_t nbytes, int *ret, hipStream_t stream)
{
    return ishmemi_c_fcollect_on_stream(team, dest, source, nbytes, ret, (void *) stream);
}
inline int ishmemx_fcollectmem_on_stream(void *dest, const void *source, size_t nbytes, int *ret,
                                         hipStream_t stream)
{
    return ishmemx_fcollectmem_on_stream(ISHMEM_TEAM_WORLD, dest, source, nbytes, ret, stream);
}

namespace ishmemi_cxx {
/* deps -> call -> done around any stream-ordered call (the reference's _on_queue deps / event). */
template <typename F>
inline int with_events(hipStream_t stream, const hipEvent_t *deps, size_t ndeps, hipEvent_t done, F &&call)
{
    if (ishmemi_c_stream_wait_events((void *) stream, (void *const *) deps, ndeps)) return 1;
    if (call()) return 1;
    return ishmemi_c_stream_record_event((void *) stream, (void *) done);
}
}  // namespace ishmemi_cxx

/* collect with per-PE counts on a stream (src/ishmemx.h collectmem / <TN>_collect _on_queue). */
inline int ishmemx_collectmem_on_stream(ishmem_team_t team, void *dest, const void *source,
                                        size_t nbytes, int *ret, hipStream_t stream)
{
    return ishmemi_c_collect_on_stream(team, dest, source, nbytes, ret, (void *) stream);
}
inline int ishmemx_collectmem_on_stream(void *dest, const void *source, size_t nbytes, int *ret,
                                        hipStream_t stream)
{
    return ishmemx_collectmem_on_stream(ISHMEM_TEAM_WORLD, dest, source, nbytes, ret, stream);
}

#define ISHMEMI_CXX_COLL_ON_STREAM(TYPENAME, TYPE, UNUSED1, UNUSED2)                                 \
    inline int ishmemx_##TYPENAME##_fcollect_on_stream(ishmem_team_t team, TYPE *dest,              \
                                                       const TYPE *source, size_t nelems, int *ret, \
                                                       hipStream_t stream)                          \
    {                                                                                              \
        return ishmemi_c_fcollect_on_stream(team, (void *) dest, (const void *) source,             \
                                            nelems * sizeof(TYPE), ret, (void *) stream);           \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_fcollect_on_stream(TYPE *dest, const TYPE *source,              \
                                                       size_t nelems, int *ret, hipStream_t stream) \
    {                                                                                              \
        return ishmemx_##TYPENAME##_fcollect_on_stream(ISHMEM_TEAM_WORLD, dest, source, nelems,    \
                                                       ret, stream);                               \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_collect_on_stream(ishmem_team_t team, TYPE *dest,               \
                                                      const TYPE *source, size_t nelems, int *ret,  \
                                                      hipStream_t stream)                           \
    {                                                                                              \
        return ishmemi_c_collect_on_stream(team, (void *) dest, (const void *) source,              \
                                           nelems * sizeof(TYPE), ret, (void *) stream);            \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_collect_on_stream(TYPE *dest, const TYPE *source, size_t nelems, \
                                                      int *ret, hipStream_t stream)                 \
    {                                                                                              \
        return ishmemx_##TYPENAME##_collect_on_stream(ISHMEM_TEAM_WORLD, dest, source, nelems, ret, \
                                                      stream);                                     \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_sum_inscan_on_stream(ishmem_team_t team, TYPE *dest,            \
                                                         const TYPE *source, size_t nelems,         \
                                                         int *ret, hipStream_t stream)              \
    {                                                                                              \
        return ishmemi_c_scan_on_stream(team, ishmemi_cxx::dtype_of<TYPE>(), 1, (void *) dest,      \
                                        (const void *) source, nelems, ret, (void *) stream);       \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_sum_inscan_on_stream(TYPE *dest, const TYPE *source,            \
                                                         size_t nelems, int *ret,                   \
                                                         hipStream_t stream)                        \
    {                                                                                              \
        return ishmemx_##TYPENAME##_sum_inscan_on_stream(ISHMEM_TEAM_WORLD, dest, source, nelems,  \
                                                         ret, stream);                             \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_sum_exscan_on_stream(ishmem_team_t team, TYPE *dest,            \
                                                         const TYPE *source, size_t nelems,         \
                                                         int *ret, hipStream_t stream)              \
    {                                                                                              \
        return ishmemi_c_scan_on_stream(team, ishmemi_cxx::dtype_of<TYPE>(), 0, (void *) dest,      \
                                        (const void *) source, nelems, ret, (void *) stream);       \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_sum_exscan_on_stream(TYPE *dest, const TYPE *source,            \
                                                         size_t nelems, int *ret,                   \
                                                         hipStream_t stream)                        \
    {                                                                                              \
        return ishmemx_##TYPENAME##_sum_exscan_on_stream(ISHMEM_TEAM_WORLD, dest, source, nelems,  \
                                                         ret, stream);                             \
    }

ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_COLL_ON_STREAM, _, _)

/* The same four with the reference's deps / returned event (team form). */
#define ISHMEMI_CXX_COLL_ON_STREAM_EV(TYPENAME, TYPE, UNUSED1, UNUSED2)                              \
    inline int ishmemx_##TYPENAME##_fcollect_on_stream(ishmem_team_t team, TYPE *dest,              \
        const TYPE *source, size_t nelems, int *ret, hipStream_t stream, const hipEvent_t *deps,    \
        size_t ndeps, hipEvent_t done)                                                             \
    {                                                                                              \
        return ishmemi_cxx::with_events(stream, deps, ndeps, done, [&] {                           \
            return ishmemx_##TYPENAME##_fcollect_on_stream(team, dest, source, nelems, ret, stream); \
        });                                                                                        \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_collect_on_stream(ishmem_team_t team, TYPE *dest,               \
        const TYPE *source, size_t nelems, int *ret, hipStream_t stream, const hipEvent_t *deps,    \
        size_t ndeps, hipEvent_t done)                                                             \
    {                                                                                              \
        return ishmemi_cxx::with_events(stream, deps, ndeps, done, [&] {                           \
            return ishmemx_##TYPENAME##_collect_on_stream(team, dest, source, nelems, ret, stream); \
        });                                                                                        \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_sum_inscan_on_stream(ishmem_team_t team, TYPE *dest,            \
        const TYPE *source, size_t nelems, int *ret, hipStream_t stream, const hipEvent_t *deps,    \
        size_t ndeps, hipEvent_t done)                                                             \
    {                                                                                              \
        return ishmemi_cxx::with_events(stream, deps, ndeps, done, [&] {                           \
            return ishmemx_##TYPENAME##_sum_inscan_on_stream(team, dest, source, nelems, ret, stream); \
        });                                                                                        \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_sum_exscan_on_stream(ishmem_team_t team, TYPE *dest,            \
        const TYPE *source, size_t nelems, int *ret, hipStream_t stream, const hipEvent_t *deps,    \
        size_t ndeps, hipEvent_t done)                                                             \
    {                                                                                              \
        return ishmemi_cxx::with_events(stream, deps, ndeps, done, [&] {                           \
            return ishmemx_##TYPENAME##_sum_exscan_on_stream(team, dest, source, nelems, ret, stream); \
        });                                                                                        \
    }

ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_COLL_ON_STREAM_EV, _, _)

/* broadcast / team barrier on a stream (src/ishmemx.h:846-954, :2228-2235). */
inline int ishmemx_broadcastmem_on_stream(ishmem_team_t team, void *dest, const void *source, size_t nbytes,
                                          int root, int *ret, hipStream_t stream)
{
    return ishmemi_c_broadcast_on_stream(team, dest, source, nbytes, root, ret, (void *) stream);
}
inline int ishmemx_broadcastmem_on_stream(void *dest, const void *source, size_t nbytes, int root, int *ret,
                                          hipStream_t stream)
{
    return ishmemi_c_broadcast_on_stream(ISHMEM_TEAM_WORLD, dest, source, nbytes, root, ret, (void *) stream);
}
template <typename T>
inline int ishmemx_broadcast_on_stream(ishmem_team_t team, T *dest, const T *source, size_t nelems, int root,
                                       int *ret, hipStream_t stream)
{
    return ishmemi_c_broadcast_on_stream(team, (void *) dest, (const void *) source, nelems * sizeof(T), root, ret,
                                         (void *) stream);
}
template <typename T>
inline int ishmemx_broadcast_on_stream(T *dest, const T *source, size_t nelems, int root, int *ret,
                                       hipStream_t stream)
{
    return ishmemx_broadcast_on_stream(ISHMEM_TEAM_WORLD, dest, source, nelems, root, ret, stream);
}
#define ISHMEMI_CXX_BCAST_ON_STREAM(TYPENAME, TYPE, UNUSED1, UNUSED2)                               \
    inline int ishmemx_##TYPENAME##_broadcast_on_stream(ishmem_team_t team, TYPE *dest,             \
                                                        const TYPE *source, size_t nelems, int root, \
                                                        int *ret, hipStream_t stream)              \
    {                                                                                              \
        return ishmemx_broadcast_on_stream(team, dest, source, nelems, root, ret, stream);         \
    }                                                                                              \
    inline int ishmemx_##TYPENAME##_broadcast_on_stream(TYPE *dest, const TYPE *source,             \
                                                        size_t nelems, int root, int *ret,         \
                                                        hipStream_t stream)                        \
    {                                                                                              \
        return ishmemx_broadcast_on_stream(dest, source, nelems, root, ret, stream);               \
    }
ISHMEMI_CXX_ARITH_TYPES(ISHMEMI_CXX_BCAST_ON_STREAM, _, _)
inline int ishmemx_team_sync_on_stream(ishmem_team_t team, int *ret, hipStream_t stream)
{
    return ishmemi_c_team_sync_on_stream(team, ret, (void *) stream);
}
inline int ishmemx_sync_all_on_stream(hipStream_t stream)
{
    return ishmemi_c_team_sync_on_stream(ISHMEM_TEAM_WORLD, nullptr, (void *) stream);
}
/* barrier_all = quiet + sync_all; stream order already completes the stream's earlier work. */
inline int ishmemx_barrier_all_on_stream(hipStream_t stream)
{
    return ishmemi_c_team_sync_on_stream(ISHMEM_TEAM_WORLD, nullptr, (void *) stream);
}

/* Explicit-identity init (the role of ishmemx_init_attr, src/ishmemx.h:21-37). */
inline int ishmemx_init_pe(int pe, int npes, int device, const char *bootstrap_key)
{
    return ishmemi_c_init_pe(pe, npes, device, bootstrap_key);
}

#endif /* ISHMEM_AMD_ISHMEMX_H */
