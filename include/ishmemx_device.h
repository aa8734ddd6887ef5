/* ishmem_amd — device-callable collectives, header-only HIP (included by ishmem.h / ishmemx.h
 * when the translation unit is compiled as HIP, so a kernel sees the reference's device API).
 *
 * Analogue of the reference's SYCL_EXTERNAL device API, called exactly as the reference calls it:
 *   ishmemx_<TYPENAME>_<op>_reduce_work_group([team,] dest, source, nreduce, grp)
 *       (src/ishmemx.h:1209-1803, src/collectives/reduce_impl.h:386-418, :505-518) — every thread
 *       of the group `grp` calls, on every PE of the team;
 *   ishmem_<TYPENAME>_<op>_reduce([team,] dest, source, nreduce) from ONE work-item (the
 *       reference's device-side blocking call, e.g. in a single_task: examples/6_team_split_strided.cpp:67);
 *   fcollect / collect / sum_inscan / sum_exscan / broadcast in the same forms;
 *   ishmem_my_pe / n_pes / team_my_pe / team_n_pes / team_translate_pe / ptr / info_get_*,
 *   ishmem_barrier_all / sync_all / team_sync and their *_work_group forms, ishmemx_print.
 * `grp` is a HIP cooperative group — cooperative_groups::thread_block (the reference's
 * sycl::group) or a 64-lane cooperative_groups::thread_block_tile (its sycl::sub_group) — or one of
 * the tags ishmemx_dev::work_group / wavefront.
 *
 *   __global__ void k(int *dst, const int *src, size_t n) {
 *       auto grp = cooperative_groups::this_thread_block();
 *       ... produce src ...
 *       int rc = ishmemx_int_sum_reduce_work_group(dst, src, n, grp);
 *   }
 *
 * The library's device state reaches the kernel without an argument: every translation unit
 * that includes this header owns a device pointer to the library's context and registers it with
 * the library from a static initializer; ishmem_init fills every registered copy (a code object
 * loaded later is filled when it registers).  This is what SYCL device globals give the reference.
 *
 * Algorithm: the same direct reduce-scatter + all-gather as the host-launched kernel, executed by
 * the calling group (member c folds chunk c of every member's source in canonical team order
 * with system-coherent loads, stores it write-through, team barrier, then pulls the other chunks).
 * `source` must have been written by the calling group or by earlier kernels (the start barrier
 * releases this group's own writes).  Returns 0, or nonzero if the library is not initialised or
 * a peer did not arrive within the library's timeout.  dest/source must be symmetric-heap
 * addresses; source and dest identical or disjoint (reduce), disjoint (scan, collect).
 */
#ifndef ISHMEM_AMD_ISHMEMX_DEVICE_H
#define ISHMEM_AMD_ISHMEMX_DEVICE_H

#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#include <type_traits>

#include "ishmem_capi.h"

namespace ishmemx_dev {

// This translation unit's pointer to the library's device context (see the header comment).
static __device__ const ishmemi_c_device_ctx_t *g_ctx = nullptr;
[[maybe_unused]] static const int g_ctx_registered = ishmemi_c_register_device_ctx_slot((const void *) &g_ctx);

__device__ __forceinline__ const ishmemi_c_device_ctx_t *ctx() { return g_ctx; }

template <typename T, int OP>
__device__ __forceinline__ T op1(T a, T b)
{
    using W = std::conditional_t<(sizeof(T) == 8), uint64_t, uint32_t>;
    if constexpr (OP == ISHMEMI_OP_AND) return (T) (a & b);
    else if constexpr (OP == ISHMEMI_OP_OR) return (T) (a | b);
    else if constexpr (OP == ISHMEMI_OP_XOR) return (T) (a ^ b);
    else if constexpr (OP == ISHMEMI_OP_MAX) {
        if constexpr (std::is_floating_point_v<T>) return fmax(a, b);
        else return (a < b) ? b : a;
    } else if constexpr (OP == ISHMEMI_OP_MIN) {
        if constexpr (std::is_floating_point_v<T>) return fmin(a, b);
        else return (b < a) ? b : a;
    } else if constexpr (OP == ISHMEMI_OP_SUM) {
        if constexpr (std::is_floating_point_v<T>) return a + b;
        else return (T) (std::make_unsigned_t<T>) ((W) (std::make_unsigned_t<T>) a + (W) (std::make_unsigned_t<T>) b);
    } else {
        if constexpr (std::is_floating_point_v<T>) return a * b;
        else return (T) (std::make_unsigned_t<T>) ((W) (std::make_unsigned_t<T>) a * (W) (std::make_unsigned_t<T>) b);
    }
}

// System-coherent element access (sc0 sc1): bypasses L1 / non-coherent L2 copies.
template <typename T>
__device__ __forceinline__ T sys_load(const T *p)
{
    using U = std::conditional_t<sizeof(T) == 8, uint64_t, std::conditional_t<sizeof(T) == 4, uint32_t,
              std::conditional_t<sizeof(T) == 2, uint16_t, uint8_t>>>;
    const U v = __hip_atomic_load((const U *) p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return __builtin_bit_cast(T, v);
}

template <typename T>
__device__ __forceinline__ void sys_store(T *p, T x)
{
    using U = std::conditional_t<sizeof(T) == 8, uint64_t, std::conditional_t<sizeof(T) == 4, uint32_t,
              std::conditional_t<sizeof(T) == 2, uint16_t, uint8_t>>>;
    __hip_atomic_store((U *) p, __builtin_bit_cast(U, x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ char *peer_addr(const ishmemi_c_device_ctx_t *c, const void *p, int pe)
{
    return c->peer_heap[pe] + ((const char *) p - c->heap_base);
}

// 16 bytes of T, the unit of the vectorised fold.
template <typename T>
struct alignas(16) Vec16 {
    T e[16 / sizeof(T)];
};
constexpr int kUnroll = 4;  // 16-B items in flight per thread and member
// The group's reduce-scatter loads this many members' items before folding them (a run-time loop
// over members would wait for each member's loads before issuing the next member's: 4 x 16 B per
// thread in flight), and the all-gather pulls this many 16-B items per thread per step.
#ifndef ISHMEMX_DEV_MEMBER_BATCH
#define ISHMEMX_DEV_MEMBER_BATCH 4
#endif
#ifndef ISHMEMX_DEV_AG_UNROLL
#define ISHMEMX_DEV_AG_UNROLL 8
#endif
constexpr int kMemberBatch = ISHMEMX_DEV_MEMBER_BATCH;
constexpr int kAgUnroll = ISHMEMX_DEV_AG_UNROLL;

template <typename T, int OP>
__device__ __forceinline__ Vec16<T> op16(const Vec16<T> &a, const Vec16<T> &b)
{
    Vec16<T> r;
#pragma unroll
    for (int i = 0; i < (int) (16 / sizeof(T)); ++i) r.e[i] = op1<T, OP>(a.e[i], b.e[i]);
    return r;
}

// A pointer every calling thread holds with the same value, moved to scalar registers (buffer
// descriptors need a uniform base; the group's threads all compute the same address).
__device__ __forceinline__ const char *group_uniform(const char *p)
{
    const uint64_t v = (uint64_t) p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t) v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t) (v >> 32));
    return (const char *) (((uint64_t) hi << 32) | lo);
}

// System-coherent (sc0 sc1) 16-B load / write-through store through a buffer descriptor based at
// `base`; off < 2 GiB.
template <typename T>
__device__ __forceinline__ Vec16<T> sys_load16(const char *base, uint32_t off)
{
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), (short) 0, 0x7FFFFFFF, 0x00020000);
    return __builtin_bit_cast(Vec16<T>, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 17));
}

template <typename T>
__device__ __forceinline__ void sys_store16(char *base, uint32_t off, const Vec16<T> &v)
{
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short) 0, 0x7FFFFFFF, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 17);
}

// Execution groups that can call a device collective (the reference's `const Group &grp`:
// sycl::group<1..3> and sycl::sub_group, plus the single work-item of a device-side blocking
// call).  Every member of the group calls with identical arguments.
struct work_group_t {  // every thread of the work-group
    __device__ static int rank() { return threadIdx.x + blockDim.x * (threadIdx.y + blockDim.y * threadIdx.z); }
    __device__ static int size() { return blockDim.x * blockDim.y * blockDim.z; }
    __device__ static void sync() { __syncthreads(); }
    __device__ static uint32_t bcast(uint32_t v)
    {
        __shared__ uint32_t s_v;
        __syncthreads();
        if (rank() == 0) s_v = v;
        __syncthreads();
        return s_v;
    }
};
struct wavefront_t {  // one full 64-lane wavefront (sub_group analogue)
    __device__ static int rank() { return (int) __lane_id(); }
    __device__ static int size() { return warpSize; }
    __device__ static void sync() { __builtin_amdgcn_wave_barrier(); }
    __device__ static uint32_t bcast(uint32_t v) { return (uint32_t) __shfl((int) v, 0); }
};
struct thread_t {  // one work-item (device-side ishmem_<TN>_<op>_reduce)
    __device__ static int rank() { return 0; }
    __device__ static int size() { return 1; }
    __device__ static void sync() {}
    __device__ static uint32_t bcast(uint32_t v) { return v; }
};
inline constexpr work_group_t work_group{};
inline constexpr wavefront_t wavefront{};
inline constexpr thread_t thread{};

// Group argument -> execution tag: the library's tags, and HIP cooperative groups in the roles of
// the reference's sycl::group (thread_block) and sycl::sub_group (a 64-lane tile).
template <typename G>
struct exec_of {
    static_assert(std::is_same_v<G, work_group_t> || std::is_same_v<G, wavefront_t> || std::is_same_v<G, thread_t>,
                  "group: cooperative_groups::thread_block, thread_block_tile<64>, or an ishmemx_dev tag");
    using type = G;
};
template <>
struct exec_of<cooperative_groups::thread_block> {
    using type = work_group_t;
};
template <unsigned N, typename P>
struct exec_of<cooperative_groups::thread_block_tile<N, P>> {
    static_assert(N == 64, "a sub-group collective needs the whole 64-lane wavefront (thread_block_tile<64>)");
    using type = wavefront_t;
};
template <typename G>
using exec_t = typename exec_of<std::remove_cv_t<std::remove_reference_t<G>>>::type;

// Team barrier among the calling groups (one per member): the group's leader stores the epoch
// into its slot of every peer's row and polls its own row; bounded by the library timeout.
template <typename G>
__device__ inline bool group_barrier(const ishmemi_c_device_ctx_t *c, int team, int phase,
                                     uint32_t epoch, bool release)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    G::sync();
    uint32_t ok = 1;
    if (G::rank() == 0) {
        const int size = c->team_size[team], me = c->team_my_idx[team];
        const size_t row = ((size_t) team * ISHMEMI_C_DEV_PHASES + phase) * ISHMEMI_C_MAX_PES;
        if (release) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        for (int j = 0; j < size; ++j) {
            if (j == me) continue;
            const int gpe = c->team_start[team] + j * c->team_stride[team];
            __hip_atomic_store(c->peer_dflags[gpe] + row + me, epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (int j = 0; j < size && ok; ++j) {
            if (j == me) continue;
            while ((int32_t) (__hip_atomic_load(c->my_dflags + row + j, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > c->timeout_ticks) {
                    ok = 0;
                    __hip_atomic_fetch_or(c->err, 1u << phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    return G::bcast(ok) != 0;
}

template <typename G, typename T, int OP>
__device__ int reduce_group(const ishmemi_c_device_ctx_t *c, int team, T *dest, const T *source,
                            size_t nreduce)
{
    if (!c || team < 0 || team >= ISHMEMI_C_MAX_TEAMS) return 1;  // not initialised / bad handle
    const int tid = G::rank(), nthr = G::size();
    const int size = c->team_size[team], me = c->team_my_idx[team];
    if (size <= 0 || me < 0) return 1;
    uint32_t epoch = 0;
    if (tid == 0)
        epoch = __hip_atomic_fetch_add(c->epochs + team, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    epoch = G::bcast(epoch);
    if (size == 1) {  // one PE: dest = source (reduce_impl.h:288-289)
        if (dest != source)
            for (size_t i = tid; i < nreduce; i += nthr) dest[i] = source[i];
        G::sync();
        return 0;
    }
    // Start: every member's source is complete (this group's own writes released).
    if (!group_barrier<G>(c, team, 0, epoch, true)) return 1;
    const size_t per = ((nreduce + size - 1) / size + 63) & ~(size_t) 63;
    const size_t cs = (size_t) me * per < nreduce ? (size_t) me * per : nreduce;
    const size_t ce = cs + per < nreduce ? cs + per : nreduce;
    const int start = c->team_start[team], stride = c->team_stride[team];
    // 16-B items when both arrays are 16-B aligned (chunk edges are multiples of 64 elements, and
    // every heap is mapped at the same offsets, so peers' addresses share the residue); the few
    // elements of the last chunk past its last whole item, and misaligned arrays, go element-wise.
    constexpr size_t E = 16 / sizeof(T);
    const bool vec = ((((uintptr_t) dest) | ((uintptr_t) source)) & 15) == 0;
    const size_t nv = vec ? (ce - cs) / E : 0;
    for (size_t v0 = 0; v0 < nv; v0 += (size_t) nthr * kUnroll) {
        Vec16<T> acc[kUnroll];
        for (int j0 = 0; j0 < size; j0 += kMemberBatch) {
            Vec16<T> x[kMemberBatch][kUnroll];
#pragma unroll
            for (int b = 0; b < kMemberBatch; ++b) {
                const int j = j0 + b;
                if (j >= size) break;
                const int gpe = start + j * stride;
                const char *base = (j == me) ? (const char *) (source + cs) : peer_addr(c, source + cs, gpe);
                const char *step = group_uniform(base + v0 * 16);
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const size_t k = (size_t) u * nthr + tid;
                    if (v0 + k < nv) x[b][u] = sys_load16<T>(step, (uint32_t) (k * 16));
                }
            }
#pragma unroll
            for (int b = 0; b < kMemberBatch; ++b) {
                if (j0 + b >= size) break;
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) acc[u] = (j0 + b == 0) ? x[b][u] : op16<T, OP>(acc[u], x[b][u]);
            }
        }
        char *dstep = (char *) group_uniform((const char *) (dest + cs) + v0 * 16);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const size_t k = (size_t) u * nthr + tid;
            if (v0 + k < nv) sys_store16<T>(dstep, (uint32_t) (k * 16), acc[u]);  // write-through
        }
    }
    for (size_t i = cs + nv * E + tid; i < ce; i += nthr) {
        T acc = T();
        for (int j = 0; j < size; ++j) {
            const int gpe = start + j * stride;
            const T x = (j == me) ? source[i] : sys_load((const T *) peer_addr(c, source + i, gpe));
            acc = (j == 0) ? x : op1<T, OP>(acc, x);
        }
        sys_store(dest + i, acc);  // write-through: peers pull it after the next barrier
    }
    if (!group_barrier<G>(c, team, 1, epoch, true)) return 1;
    for (int k = 1; k < size; ++k) {
        const int j = (me + k) % size;
        const int gpe = start + j * stride;
        const size_t js = (size_t) j * per < nreduce ? (size_t) j * per : nreduce;
        const size_t je = js + per < nreduce ? js + per : nreduce;
        const size_t jv = vec ? (je - js) / E : 0;
        const char *pbase = peer_addr(c, dest + js, gpe);
        for (size_t v0 = 0; v0 < jv; v0 += (size_t) nthr * kAgUnroll) {
            const char *step = group_uniform(pbase + v0 * 16);
            Vec16<T> x[kAgUnroll];
#pragma unroll
            for (int u = 0; u < kAgUnroll; ++u) {
                const size_t q = (size_t) u * nthr + tid;
                if (v0 + q < jv) x[u] = sys_load16<T>(step, (uint32_t) (q * 16));
            }
            Vec16<T> *dp = (Vec16<T> *) (dest + js) + v0;
#pragma unroll
            for (int u = 0; u < kAgUnroll; ++u) {
                const size_t q = (size_t) u * nthr + tid;
                if (v0 + q < jv) dp[q] = x[u];
            }
        }
        for (size_t i = js + jv * E + tid; i < je; i += nthr)
            dest[i] = sys_load((const T *) peer_addr(c, dest + i, gpe));
    }
    // End: no member returns while a peer may still read its dest.
    return group_barrier<G>(c, team, 2, epoch, false) ? 0 : 1;
}

template <typename T, int OP>
__device__ int reduce_work_group(const ishmemi_c_device_ctx_t *c, int team, T *dest, const T *source,
                                 size_t nreduce)
{
    return reduce_group<work_group_t, T, OP>(c, team, dest, source, nreduce);
}

// ---- fcollect / collect / sum-scan from inside a kernel ------------------------------------
// The reference's ishmemx_<TN>_{fcollect,collect,sum_inscan,sum_exscan}_work_group and their
// device-side blocking forms (src/ishmemx.h, src/collectives/collect_impl.h, scan_impl.h), on the
// reduce's machinery: start barrier (every member's source final, this group's writes released),
// pulls with system-coherent loads into the local dest, end barrier (no member returns while a
// peer may still read its source).

// `nbytes` from `src` (a peer's when `remote`) to the local `dst` by the group: 16-B items when
// both addresses and the length allow, 4-B or single bytes otherwise.
template <typename G>
__device__ inline void group_copy(const char *src, char *dst, size_t nbytes, bool remote)
{
    const int tid = G::rank(), nthr = G::size();
    const uintptr_t al = (uintptr_t) src | (uintptr_t) dst | (uintptr_t) nbytes;
    if ((al & 15) == 0) {
        const size_t nv = nbytes / 16;
        for (size_t v0 = 0; v0 < nv; v0 += (size_t) nthr * kUnroll) {
            const char *step = group_uniform(src + v0 * 16);
            Vec16<uint32_t> x[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const size_t k = (size_t) u * nthr + tid;
                if (v0 + k < nv)
                    x[u] = remote ? sys_load16<uint32_t>(step, (uint32_t) (k * 16)) : ((const Vec16<uint32_t> *) step)[k];
            }
            Vec16<uint32_t> *dp = (Vec16<uint32_t> *) (dst + v0 * 16);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const size_t k = (size_t) u * nthr + tid;
                if (v0 + k < nv) dp[k] = x[u];
            }
        }
    } else if ((al & 3) == 0) {
        for (size_t i = tid; i < nbytes / 4; i += nthr)
            ((uint32_t *) dst)[i] = remote ? sys_load((const uint32_t *) src + i) : ((const uint32_t *) src)[i];
    } else {
        for (size_t i = tid; i < nbytes; i += nthr)
            dst[i] = remote ? (char) sys_load((const uint8_t *) src + i) : src[i];
    }
}

template <typename G>
__device__ inline uint32_t group_epoch(const ishmemi_c_device_ctx_t *c, int team)
{
    uint32_t epoch = 0;
    if (G::rank() == 0)
        epoch = __hip_atomic_fetch_add(c->epochs + team, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    return G::bcast(epoch);
}

// fcollect (equal counts) when counts == nullptr; collect otherwise: this member contributes
// `mybytes`, published in its symmetric count slot before the start barrier and read by every
// member after it (pull: no peer stores into this PE's coarse-grained heap).
template <typename G>
__device__ inline int collect_group(const ishmemi_c_device_ctx_t *c, int team, void *dest, const void *source,
                                    size_t mybytes, bool equal)
{
    if (!c || team < 0 || team >= ISHMEMI_C_MAX_TEAMS) return 1;  // not initialised / bad handle
    const int size = c->team_size[team], me = c->team_my_idx[team];
    if (size <= 0 || me < 0) return 1;
    const uint32_t epoch = group_epoch<G>(c, team);
    if (size == 1) {
        if (dest != source) group_copy<G>((const char *) source, (char *) dest, mybytes, false);
        G::sync();
        return 0;
    }
    uint64_t *slot = c->dev_counts + (size_t) team * 8;
    if (!equal && G::rank() == 0) sys_store(slot, (uint64_t) mybytes);  // write-through; barrier drains it
    if (!group_barrier<G>(c, team, 0, epoch, true)) return 1;
    const int start = c->team_start[team], stride = c->team_stride[team];
    size_t off = 0;
    for (int j = 0; j < size; ++j) {
        const int gpe = start + j * stride;
        const size_t nb = equal ? mybytes : (size_t) sys_load((const uint64_t *) peer_addr(c, slot, gpe));
        if (nb) {
            const char *src = j == me ? (const char *) source : peer_addr(c, source, gpe);
            group_copy<G>(src, (char *) dest + off, nb, j != me);
        }
        off += nb;
    }
    return group_barrier<G>(c, team, 2, epoch, false) ? 0 : 1;
}

// Prefix sum in team order: member me folds members 0..me (inclusive) or 0..me-1 (exclusive;
// member 0 gets 0) element by element — the first term passes through unchanged, as in the host
// scan.  dest must not overlap source (a peer may still be reading it).
template <typename G, typename T>
__device__ inline int scan_group(const ishmemi_c_device_ctx_t *c, int team, T *dest, const T *source,
                                 size_t nelems, bool inclusive)
{
    if (!c || team < 0 || team >= ISHMEMI_C_MAX_TEAMS) return 1;  // not initialised / bad handle
    const int tid = G::rank(), nthr = G::size();
    const int size = c->team_size[team], me = c->team_my_idx[team];
    // dest and source must be disjoint: a peer may still be reading this PE's source.
    const bool overlap = (const char *) dest < (const char *) (source + nelems) &&
                         (const char *) source < (const char *) (dest + nelems);
    if (size <= 0 || me < 0 || (size > 1 && nelems && overlap)) return 1;
    const uint32_t epoch = group_epoch<G>(c, team);
    if (size > 1 && !group_barrier<G>(c, team, 0, epoch, true)) return 1;
    const int last = inclusive ? me : me - 1;
    const int start = c->team_start[team], stride = c->team_stride[team];
    constexpr size_t E = 16 / sizeof(T);
    const bool vec = ((((uintptr_t) dest) | ((uintptr_t) source)) & 15) == 0;
    const size_t nv = vec ? nelems / E : 0;
    for (size_t v0 = 0; v0 < nv; v0 += (size_t) nthr * kUnroll) {
        Vec16<T> acc[kUnroll] = {};
        for (int k = 0; k <= last; ++k) {
            const char *base = k == me ? (const char *) source : peer_addr(c, source, start + k * stride);
            const char *step = group_uniform(base + v0 * 16);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const size_t q = (size_t) u * nthr + tid;
                if (v0 + q < nv) {
                    const Vec16<T> x = sys_load16<T>(step, (uint32_t) (q * 16));
                    acc[u] = k == 0 ? x : op16<T, ISHMEMI_OP_SUM>(acc[u], x);
                }
            }
        }
        Vec16<T> *dp = (Vec16<T> *) dest + v0;
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const size_t q = (size_t) u * nthr + tid;
            if (v0 + q < nv) dp[q] = acc[u];
        }
    }
    for (size_t i = nv * E + tid; i < nelems; i += nthr) {
        T acc = T();
        for (int k = 0; k <= last; ++k) {
            const T x = k == me ? source[i] : sys_load((const T *) peer_addr(c, source + i, start + k * stride));
            acc = k == 0 ? x : op1<T, ISHMEMI_OP_SUM>(acc, x);
        }
        dest[i] = acc;
    }
    if (size == 1) {
        G::sync();
        return 0;
    }
    return group_barrier<G>(c, team, 2, epoch, false) ? 0 : 1;
}

// Team barrier from inside a kernel (ishmem_team_sync / sync_all / barrier_all and their
// *_work_group forms, src/collectives/sync_impl.h:30-69): the group's writes are released, then
// every member's group meets on the team's phase-3 row.  There is no RMA in this library, so
// barrier_all's quiet has nothing further to complete.
template <typename G>
__device__ inline int team_sync_group(const ishmemi_c_device_ctx_t *c, int team)
{
    if (!c || team < 0 || team >= ISHMEMI_C_MAX_TEAMS) return 1;
    const int size = c->team_size[team], me = c->team_my_idx[team];
    if (size <= 0 || me < 0) return 1;
    if (size == 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        G::sync();
        return 0;
    }
    const uint32_t epoch = group_epoch<G>(c, team);
    return group_barrier<G>(c, team, 3, epoch, true) ? 0 : 1;
}

// Broadcast (src/collectives/broadcast_impl.h, its intra-node pull variant): start barrier (the
// root's source is final), every member including the root pulls `nbytes` of the root's source
// into its dest, end barrier (the root may reuse its source).
template <typename G>
__device__ inline int broadcast_group(const ishmemi_c_device_ctx_t *c, int team, void *dest,
                                      const void *source, size_t nbytes, int root)
{
    if (!c || team < 0 || team >= ISHMEMI_C_MAX_TEAMS) return 1;
    const int size = c->team_size[team], me = c->team_my_idx[team];
    if (size <= 0 || me < 0 || root < 0 || root >= size) return 1;
    const uint32_t epoch = group_epoch<G>(c, team);
    if (size == 1) {
        if (dest != source) group_copy<G>((const char *) source, (char *) dest, nbytes, false);
        G::sync();
        return 0;
    }
    if (!group_barrier<G>(c, team, 0, epoch, true)) return 1;
    const int groot = c->team_start[team] + root * c->team_stride[team];
    if (root != me) group_copy<G>(peer_addr(c, source, groot), (char *) dest, nbytes, true);
    else if (dest != source) group_copy<G>((const char *) source, (char *) dest, nbytes, false);
    return group_barrier<G>(c, team, 2, epoch, false) ? 0 : 1;
}

template <typename T>
constexpr bool is_canon()
{
    return std::is_arithmetic_v<T> && sizeof(T) <= 8;
}

}  // namespace ishmemx_dev

/* ---- library queries from a kernel (src/ishmem.h:54-58, :74-77: host and device) ------------ */
__device__ inline int ishmem_my_pe(void)
{
    const ishmemi_c_device_ctx_t *c = ishmemx_dev::ctx();
    return c ? c->pe : -1;
}
__device__ inline int ishmem_n_pes(void)
{
    const ishmemi_c_device_ctx_t *c = ishmemx_dev::ctx();
    return c ? c->npes : -1;
}
__device__ inline void *ishmem_ptr(const void *dest, int pe)
{
    const ishmemi_c_device_ctx_t *c = ishmemx_dev::ctx();
    if (!c || pe < 0 || pe >= c->npes) return nullptr;
    const uint64_t off = (uint64_t) ((const char *) dest - c->heap_base);
    return off < c->heap_size ? (void *) (c->peer_heap[pe] + off) : nullptr;
}
__device__ inline int ishmem_team_my_pe(int team)
{
    const ishmemi_c_device_ctx_t *c = ishmemx_dev::ctx();
    if (!c || team < 0 || team >= ISHMEMI_C_MAX_TEAMS || c->team_size[team] <= 0) return -1;
    return c->team_my_idx[team];
}
__device__ inline int ishmem_team_n_pes(int team)
{
    const ishmemi_c_device_ctx_t *c = ishmemx_dev::ctx();
    if (!c || team < 0 || team >= ISHMEMI_C_MAX_TEAMS || c->team_size[team] <= 0) return -1;
    return c->team_size[team];
}
__device__ inline int ishmem_team_translate_pe(int src_team, int src_pe, int dest_team)
{
    const ishmemi_c_device_ctx_t *c = ishmemx_dev::ctx();
    if (!c || src_team < 0 || src_team >= ISHMEMI_C_MAX_TEAMS || dest_team < 0 ||
        dest_team >= ISHMEMI_C_MAX_TEAMS || c->team_size[src_team] <= 0 || c->team_size[dest_team] <= 0 ||
        src_pe < 0 || src_pe >= c->team_size[src_team])
        return -1;
    const int d = c->team_start[src_team] + src_pe * c->team_stride[src_team] - c->team_start[dest_team];
    const int st = c->team_stride[dest_team];
    if (st == 0 || d % st) return -1;
    return (d / st >= 0 && d / st < c->team_size[dest_team]) ? d / st : -1;
}
__device__ inline void ishmem_info_get_version(int *major, int *minor)
{
    *major = ISHMEMI_C_SPEC_MAJOR;
    *minor = ISHMEMI_C_SPEC_MINOR;
}
__device__ inline void ishmem_info_get_name(char *name)
{
    const char *v = ISHMEMI_C_VENDOR_STRING;
    while (*v) *name++ = *v++;
    *name = '\0';
}

/* ---- synchronisation from a kernel (src/ishmem.h:1555-1559, src/ishmemx.h:2228-2239) -------- */
__device__ inline void ishmem_barrier_all(void)
{
    (void) ishmemx_dev::team_sync_group<ishmemx_dev::thread_t>(ishmemx_dev::ctx(), ISHMEMI_C_TEAM_WORLD);
}
__device__ inline void ishmem_sync_all(void)
{
    (void) ishmemx_dev::team_sync_group<ishmemx_dev::thread_t>(ishmemx_dev::ctx(), ISHMEMI_C_TEAM_WORLD);
}
__device__ inline int ishmem_team_sync(int team)
{
    return ishmemx_dev::team_sync_group<ishmemx_dev::thread_t>(ishmemx_dev::ctx(), team);
}
template <typename Group>
__device__ inline void ishmemx_barrier_all_work_group(const Group &)
{
    (void) ishmemx_dev::team_sync_group<ishmemx_dev::exec_t<Group>>(ishmemx_dev::ctx(), ISHMEMI_C_TEAM_WORLD);
}
template <typename Group>
__device__ inline void ishmemx_sync_all_work_group(const Group &)
{
    (void) ishmemx_dev::team_sync_group<ishmemx_dev::exec_t<Group>>(ishmemx_dev::ctx(), ISHMEMI_C_TEAM_WORLD);
}
template <typename Group>
__device__ inline void ishmemx_team_sync_work_group(int team, const Group &)
{
    (void) ishmemx_dev::team_sync_group<ishmemx_dev::exec_t<Group>>(ishmemx_dev::ctx(), team);
}

/* ---- device print (src/ishmemx.h:2256-2271; the reference sends it to a host proxy thread, a
 *      HIP kernel prints directly) --------------------------------------------------------------- */
typedef enum { DEBUG, WARNING, ERROR, STDOUT, STDERR } ishmemx_print_msg_type_t;
__device__ inline void ishmemx_print(const char *file, long int line, const char *func, const char *out,
                                     ishmemx_print_msg_type_t msg_type)
{
    const char *kind = msg_type == DEBUG ? "DEBUG" : msg_type == WARNING ? "WARN" : msg_type == ERROR ? "ERROR" : "";
    if (file) printf("[%d] %s %s:%ld %s: %s", ishmem_my_pe(), kind, file, line, func ? func : "", out);
    else printf("[%d] %s%s%s", ishmem_my_pe(), kind, *kind ? ": " : "", out);
}
__device__ inline void ishmemx_print(const char *out, ishmemx_print_msg_type_t msg_type)
{
    ishmemx_print(nullptr, 0, nullptr, out, msg_type);
}
__device__ inline void ishmemx_print(const char *out) { ishmemx_print(nullptr, 0, nullptr, out, DEBUG); }

/* ---- reductions ------------------------------------------------------------------------------ */
#define ISHMEMX_DEV_GENERIC(OPNAME, OPC)                                                           \
    template <typename T, typename Group>                                                          \
    __device__ inline int ishmemx_##OPNAME##_reduce_work_group(T *dest, const T *source,           \
                                                               size_t nreduce, const Group &)      \
    {                                                                                              \
        return ishmemx_dev::reduce_group<ishmemx_dev::exec_t<Group>, T, OPC>(                      \
            ishmemx_dev::ctx(), ISHMEMI_C_TEAM_WORLD, dest, source, nreduce);                      \
    }                                                                                              \
    template <typename T, typename Group>                                                          \
    __device__ inline int ishmemx_##OPNAME##_reduce_work_group(int team, T *dest, const T *source, \
                                                               size_t nreduce, const Group &)      \
    {                                                                                              \
        return ishmemx_dev::reduce_group<ishmemx_dev::exec_t<Group>, T, OPC>(ishmemx_dev::ctx(),   \
                                                                             team, dest, source,   \
                                                                             nreduce);             \
    }                                                                                              \
    template <typename T>                                                                          \
    __device__ inline int ishmem_##OPNAME##_reduce(T *dest, const T *source, size_t nreduce)       \
    {                                                                                              \
        return ishmemx_dev::reduce_group<ishmemx_dev::thread_t, T, OPC>(                           \
            ishmemx_dev::ctx(), ISHMEMI_C_TEAM_WORLD, dest, source, nreduce);                      \
    }                                                                                              \
    template <typename T>                                                                          \
    __device__ inline int ishmem_##OPNAME##_reduce(int team, T *dest, const T *source,             \
                                                   size_t nreduce)                                 \
    {                                                                                              \
        return ishmemx_dev::reduce_group<ishmemx_dev::thread_t, T, OPC>(ishmemx_dev::ctx(), team,  \
                                                                        dest, source, nreduce);    \
    }

ISHMEMX_DEV_GENERIC(and, ISHMEMI_OP_AND)
ISHMEMX_DEV_GENERIC(or, ISHMEMI_OP_OR)
ISHMEMX_DEV_GENERIC(xor, ISHMEMI_OP_XOR)
ISHMEMX_DEV_GENERIC(max, ISHMEMI_OP_MAX)
ISHMEMX_DEV_GENERIC(min, ISHMEMI_OP_MIN)
ISHMEMX_DEV_GENERIC(sum, ISHMEMI_OP_SUM)
ISHMEMX_DEV_GENERIC(prod, ISHMEMI_OP_PROD)

#define ISHMEMX_DEV_TYPED(TYPENAME, TYPE, OPNAME, OPC)                                              \
    template <typename Group>                                                                      \
    __device__ inline int ishmemx_##TYPENAME##_##OPNAME##_reduce_work_group(                       \
        TYPE *dest, const TYPE *source, size_t nreduce, const Group &grp)                          \
    {                                                                                              \
        return ishmemx_##OPNAME##_reduce_work_group<TYPE>(dest, source, nreduce, grp);             \
    }                                                                                              \
    template <typename Group>                                                                      \
    __device__ inline int ishmemx_##TYPENAME##_##OPNAME##_reduce_work_group(                       \
        int team, TYPE *dest, const TYPE *source, size_t nreduce, const Group &grp)                \
    {                                                                                              \
        return ishmemx_##OPNAME##_reduce_work_group<TYPE>(team, dest, source, nreduce, grp);       \
    }                                                                                              \
    __device__ inline int ishmem_##TYPENAME##_##OPNAME##_reduce(TYPE *dest, const TYPE *source,    \
                                                                size_t nreduce)                    \
    {                                                                                              \
        return ishmem_##OPNAME##_reduce<TYPE>(dest, source, nreduce);                              \
    }                                                                                              \
    __device__ inline int ishmem_##TYPENAME##_##OPNAME##_reduce(int team, TYPE *dest,              \
                                                                const TYPE *source, size_t nreduce) \
    {                                                                                              \
        return ishmem_##OPNAME##_reduce<TYPE>(team, dest, source, nreduce);                        \
    }

/* ---- fcollect / collect / sum_inscan / sum_exscan / broadcast --------------------------------- */
template <typename T, typename Group>
__device__ inline int ishmemx_fcollect_work_group(int team, T *dest, const T *source, size_t nelems, const Group &)
{
    return ishmemx_dev::collect_group<ishmemx_dev::exec_t<Group>>(ishmemx_dev::ctx(), team, dest, source,
                                                                  nelems * sizeof(T), true);
}
template <typename T, typename Group>
__device__ inline int ishmemx_collect_work_group(int team, T *dest, const T *source, size_t nelems, const Group &)
{
    return ishmemx_dev::collect_group<ishmemx_dev::exec_t<Group>>(ishmemx_dev::ctx(), team, dest, source,
                                                                  nelems * sizeof(T), false);
}
template <typename T, typename Group>
__device__ inline int ishmemx_sum_inscan_work_group(int team, T *dest, const T *source, size_t nelems, const Group &)
{
    return ishmemx_dev::scan_group<ishmemx_dev::exec_t<Group>, T>(ishmemx_dev::ctx(), team, dest, source, nelems,
                                                                  true);
}
template <typename T, typename Group>
__device__ inline int ishmemx_sum_exscan_work_group(int team, T *dest, const T *source, size_t nelems, const Group &)
{
    return ishmemx_dev::scan_group<ishmemx_dev::exec_t<Group>, T>(ishmemx_dev::ctx(), team, dest, source, nelems,
                                                                  false);
}
template <typename T, typename Group>
__device__ inline int ishmemx_broadcast_work_group(int team, T *dest, const T *source, size_t nelems, int root,
                                                   const Group &)
{
    return ishmemx_dev::broadcast_group<ishmemx_dev::exec_t<Group>>(ishmemx_dev::ctx(), team, dest, source,
                                                                    nelems * sizeof(T), root);
}
#define ISHMEMX_DEV_COLL_WORLD(NAME)                                                                \
    template <typename T, typename Group>                                                          \
    __device__ inline int ishmemx_##NAME##_work_group(T *dest, const T *source, size_t nelems,      \
                                                      const Group &grp)                            \
    {                                                                                              \
        return ishmemx_##NAME##_work_group<T>(ISHMEMI_C_TEAM_WORLD, dest, source, nelems, grp);    \
    }                                                                                              \
    template <typename T>                                                                          \
    __device__ inline int ishmem_##NAME(int team, T *dest, const T *source, size_t nelems)         \
    {                                                                                              \
        return ishmemx_##NAME##_work_group<T>(team, dest, source, nelems, ishmemx_dev::thread);    \
    }                                                                                              \
    template <typename T>                                                                          \
    __device__ inline int ishmem_##NAME(T *dest, const T *source, size_t nelems)                   \
    {                                                                                              \
        return ishmemx_##NAME##_work_group<T>(ISHMEMI_C_TEAM_WORLD, dest, source, nelems,          \
                                              ishmemx_dev::thread);                                \
    }
ISHMEMX_DEV_COLL_WORLD(fcollect)
ISHMEMX_DEV_COLL_WORLD(collect)
ISHMEMX_DEV_COLL_WORLD(sum_inscan)
ISHMEMX_DEV_COLL_WORLD(sum_exscan)
template <typename T, typename Group>
__device__ inline int ishmemx_broadcast_work_group(T *dest, const T *source, size_t nelems, int root, const Group &grp)
{
    return ishmemx_broadcast_work_group<T>(ISHMEMI_C_TEAM_WORLD, dest, source, nelems, root, grp);
}
template <typename T>
__device__ inline int ishmem_broadcast(int team, T *dest, const T *source, size_t nelems, int root)
{
    return ishmemx_broadcast_work_group<T>(team, dest, source, nelems, root, ishmemx_dev::thread);
}
template <typename T>
__device__ inline int ishmem_broadcast(T *dest, const T *source, size_t nelems, int root)
{
    return ishmemx_broadcast_work_group<T>(ISHMEMI_C_TEAM_WORLD, dest, source, nelems, root, ishmemx_dev::thread);
}

/* Typed forms for the reference's 23 arithmetic typenames (collect.cpp:44-66, :129-151,
 * scan.cpp:28-74, broadcast.cpp): work-group and one-work-item, with and without a team. */
#define ISHMEMX_DEV_COLL_TYPED_ONE(TYPENAME, TYPE, NAME)                                             \
    template <typename Group>                                                                      \
    __device__ inline int ishmemx_##TYPENAME##_##NAME##_work_group(int team, TYPE *dest,            \
                                                                   const TYPE *source,              \
                                                                   size_t nelems, const Group &grp) \
    {                                                                                              \
        return ishmemx_##NAME##_work_group<TYPE>(team, dest, source, nelems, grp);                 \
    }                                                                                              \
    template <typename Group>                                                                      \
    __device__ inline int ishmemx_##TYPENAME##_##NAME##_work_group(TYPE *dest, const TYPE *source,  \
                                                                   size_t nelems, const Group &grp) \
    {                                                                                              \
        return ishmemx_##NAME##_work_group<TYPE>(dest, source, nelems, grp);                       \
    }                                                                                              \
    __device__ inline int ishmem_##TYPENAME##_##NAME(int team, TYPE *dest, const TYPE *source,      \
                                                     size_t nelems)                                \
    {                                                                                              \
        return ishmem_##NAME<TYPE>(team, dest, source, nelems);                                    \
    }                                                                                              \
    __device__ inline int ishmem_##TYPENAME##_##NAME(TYPE *dest, const TYPE *source, size_t nelems) \
    {                                                                                              \
        return ishmem_##NAME<TYPE>(dest, source, nelems);                                          \
    }
#define ISHMEMX_DEV_COLL(TYPENAME, TYPE, UNUSED1, UNUSED2)                                          \
    ISHMEMX_DEV_COLL_TYPED_ONE(TYPENAME, TYPE, fcollect)                                            \
    ISHMEMX_DEV_COLL_TYPED_ONE(TYPENAME, TYPE, collect)                                             \
    ISHMEMX_DEV_COLL_TYPED_ONE(TYPENAME, TYPE, sum_inscan)                                          \
    ISHMEMX_DEV_COLL_TYPED_ONE(TYPENAME, TYPE, sum_exscan)                                          \
    template <typename Group>                                                                      \
    __device__ inline int ishmemx_##TYPENAME##_broadcast_work_group(                               \
        int team, TYPE *dest, const TYPE *source, size_t nelems, int root, const Group &grp)       \
    {                                                                                              \
        return ishmemx_broadcast_work_group<TYPE>(team, dest, source, nelems, root, grp);          \
    }                                                                                              \
    template <typename Group>                                                                      \
    __device__ inline int ishmemx_##TYPENAME##_broadcast_work_group(                               \
        TYPE *dest, const TYPE *source, size_t nelems, int root, const Group &grp)                 \
    {                                                                                              \
        return ishmemx_broadcast_work_group<TYPE>(dest, source, nelems, root, grp);                \
    }                                                                                              \
    __device__ inline int ishmem_##TYPENAME##_broadcast(int team, TYPE *dest, const TYPE *source,   \
                                                        size_t nelems, int root)                   \
    {                                                                                              \
        return ishmem_broadcast<TYPE>(team, dest, source, nelems, root);                           \
    }                                                                                              \
    __device__ inline int ishmem_##TYPENAME##_broadcast(TYPE *dest, const TYPE *source,             \
                                                        size_t nelems, int root)                   \
    {                                                                                              \
        return ishmem_broadcast<TYPE>(dest, source, nelems, root);                                 \
    }

/* byte forms: fcollectmem / collectmem / broadcastmem */
template <typename Group>
__device__ inline int ishmemx_fcollectmem_work_group(int team, void *dest, const void *source, size_t nbytes,
                                                     const Group &)
{
    return ishmemx_dev::collect_group<ishmemx_dev::exec_t<Group>>(ishmemx_dev::ctx(), team, dest, source, nbytes,
                                                                  true);
}
template <typename Group>
__device__ inline int ishmemx_fcollectmem_work_group(void *dest, const void *source, size_t nbytes, const Group &grp)
{
    return ishmemx_fcollectmem_work_group(ISHMEMI_C_TEAM_WORLD, dest, source, nbytes, grp);
}
template <typename Group>
__device__ inline int ishmemx_collectmem_work_group(int team, void *dest, const void *source, size_t nbytes,
                                                    const Group &)
{
    return ishmemx_dev::collect_group<ishmemx_dev::exec_t<Group>>(ishmemx_dev::ctx(), team, dest, source, nbytes,
                                                                  false);
}
template <typename Group>
__device__ inline int ishmemx_collectmem_work_group(void *dest, const void *source, size_t nbytes, const Group &grp)
{
    return ishmemx_collectmem_work_group(ISHMEMI_C_TEAM_WORLD, dest, source, nbytes, grp);
}
template <typename Group>
__device__ inline int ishmemx_broadcastmem_work_group(int team, void *dest, const void *source, size_t nbytes,
                                                      int root, const Group &)
{
    return ishmemx_dev::broadcast_group<ishmemx_dev::exec_t<Group>>(ishmemx_dev::ctx(), team, dest, source, nbytes,
                                                                    root);
}
template <typename Group>
__device__ inline int ishmemx_broadcastmem_work_group(void *dest, const void *source, size_t nbytes, int root,
                                                      const Group &grp)
{
    return ishmemx_broadcastmem_work_group(ISHMEMI_C_TEAM_WORLD, dest, source, nbytes, root, grp);
}
__device__ inline int ishmem_fcollectmem(int team, void *dest, const void *source, size_t nbytes)
{
    return ishmemx_fcollectmem_work_group(team, dest, source, nbytes, ishmemx_dev::thread);
}
__device__ inline int ishmem_fcollectmem(void *dest, const void *source, size_t nbytes)
{
    return ishmemx_fcollectmem_work_group(ISHMEMI_C_TEAM_WORLD, dest, source, nbytes, ishmemx_dev::thread);
}
__device__ inline int ishmem_collectmem(int team, void *dest, const void *source, size_t nbytes)
{
    return ishmemx_collectmem_work_group(team, dest, source, nbytes, ishmemx_dev::thread);
}
__device__ inline int ishmem_collectmem(void *dest, const void *source, size_t nbytes)
{
    return ishmemx_collectmem_work_group(ISHMEMI_C_TEAM_WORLD, dest, source, nbytes, ishmemx_dev::thread);
}
__device__ inline int ishmem_broadcastmem(int team, void *dest, const void *source, size_t nbytes, int root)
{
    return ishmemx_broadcastmem_work_group(team, dest, source, nbytes, root, ishmemx_dev::thread);
}
__device__ inline int ishmem_broadcastmem(void *dest, const void *source, size_t nbytes, int root)
{
    return ishmemx_broadcastmem_work_group(ISHMEMI_C_TEAM_WORLD, dest, source, nbytes, root, ishmemx_dev::thread);
}

/* Same TYPENAME x op matrix as the host API (src/collectives/reduce.cpp:95-417). */
#define ISHMEMX_DEV_BITWISE_TYPES(X, OPNAME, OPC)                                                   \
    X(uchar, unsigned char, OPNAME, OPC) X(ushort, unsigned short, OPNAME, OPC)                    \
    X(uint, unsigned int, OPNAME, OPC) X(ulong, unsigned long, OPNAME, OPC)                        \
    X(ulonglong, unsigned long long, OPNAME, OPC) X(int8, int8_t, OPNAME, OPC)                     \
    X(int16, int16_t, OPNAME, OPC) X(int32, int32_t, OPNAME, OPC) X(int64, int64_t, OPNAME, OPC)   \
    X(uint8, uint8_t, OPNAME, OPC) X(uint16, uint16_t, OPNAME, OPC)                                \
    X(uint32, uint32_t, OPNAME, OPC) X(uint64, uint64_t, OPNAME, OPC) X(size, size_t, OPNAME, OPC)
#define ISHMEMX_DEV_ARITH_TYPES(X, OPNAME, OPC)                                                     \
    X(char, char, OPNAME, OPC) X(schar, signed char, OPNAME, OPC) X(short, short, OPNAME, OPC)     \
    X(int, int, OPNAME, OPC) X(long, long, OPNAME, OPC) X(longlong, long long, OPNAME, OPC)        \
    X(ptrdiff, ptrdiff_t, OPNAME, OPC) X(uchar, unsigned char, OPNAME, OPC)                        \
    X(ushort, unsigned short, OPNAME, OPC) X(uint, unsigned int, OPNAME, OPC)                      \
    X(ulong, unsigned long, OPNAME, OPC) X(ulonglong, unsigned long long, OPNAME, OPC)             \
    X(int8, int8_t, OPNAME, OPC) X(int16, int16_t, OPNAME, OPC) X(int32, int32_t, OPNAME, OPC)     \
    X(int64, int64_t, OPNAME, OPC) X(uint8, uint8_t, OPNAME, OPC) X(uint16, uint16_t, OPNAME, OPC) \
    X(uint32, uint32_t, OPNAME, OPC) X(uint64, uint64_t, OPNAME, OPC) X(size, size_t, OPNAME, OPC) \
    X(float, float, OPNAME, OPC) X(double, double, OPNAME, OPC)

ISHMEMX_DEV_BITWISE_TYPES(ISHMEMX_DEV_TYPED, and, ISHMEMI_OP_AND)
ISHMEMX_DEV_BITWISE_TYPES(ISHMEMX_DEV_TYPED, or, ISHMEMI_OP_OR)
ISHMEMX_DEV_BITWISE_TYPES(ISHMEMX_DEV_TYPED, xor, ISHMEMI_OP_XOR)
ISHMEMX_DEV_ARITH_TYPES(ISHMEMX_DEV_TYPED, max, ISHMEMI_OP_MAX)
ISHMEMX_DEV_ARITH_TYPES(ISHMEMX_DEV_TYPED, min, ISHMEMI_OP_MIN)
ISHMEMX_DEV_ARITH_TYPES(ISHMEMX_DEV_TYPED, sum, ISHMEMI_OP_SUM)
ISHMEMX_DEV_ARITH_TYPES(ISHMEMX_DEV_TYPED, prod, ISHMEMI_OP_PROD)
ISHMEMX_DEV_ARITH_TYPES(ISHMEMX_DEV_COLL, _, _)

#endif /* ISHMEM_AMD_ISHMEMX_DEVICE_H */
