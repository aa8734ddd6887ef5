// ishmem_amd — HIP kernels of the reduction-collective hot path (gfx950 / MI355X).
// Templates only: instantiated per reduction op by kernels_op.hip (one translation unit per op,
// compiled in parallel) and dispatched by kernels.hip.
//
// What the reference does (src/collectives/reduce_impl.h):
//   * reduce_op<T,OP> (:62-102): FP max/min = fmax/fmin, sum +=, prod *=; ints & | ^ max min + *.
//   * vector_reduce / vector_reduce_work_group (:105-183): d[i] = op(d[i], s[i]) with 16-wide
//     vectors, run by ONE work-item or ONE work-group.
//   * ishmemi_sub_reduce (:232-256): team barrier, then for every other PE in team order fold
//     that PE's whole source into dest (p-1 full passes, each over the peer link), barrier.
//
// What this file does instead (MI355X-first, not a translation):
//   * fanin_kernel: dst = op(src_0, ..., src_{k-1}) over 16-B vectors, every CU busy, all sources
//     streamed once (the local combine unit; with k = 1 it is the p = 1 self-reduce copy).
//   * allreduce_kernel: ONE launch per collective, direct reduce-scatter + all-gather across the
//     team.  PE c folds chunk c of every member's source (pulled over xGMI with system-coherent
//     loads) in canonical team order 0..p-1 and writes its own dest; as each segment of it is
//     published every PE pulls it from that PE's dest.  Each PE's link
//     ingress is 2(p-1)/p * B spread over p-1 links, vs (p-1) * B serialised over peers in the
//     reference loop.  Folding in canonical order makes every PE's result bit-identical (the
//     reference's results differ between PEs for FP, docs/source/collectives.rst:1241-1244) and
//     equal to the reference's PE-0 result and to its tester's check pattern
//     (test/unit/reduce_sum.cpp:203-224).
//   * The barriers replace ishmemi_team_sync's psync counters (src/collectives/sync_impl.h:30-69)
//     with epoch-tagged flags in fine-grained memory: one "started" flag per member, one
//     "ready" flag per reduced segment (the RS -> AG hand-off) and one "done reading" flag per
//     member, exchanged by whichever workgroup gets there; work is grabbed from per-launch
//     counters, so no workgroup ever waits for a particular peer workgroup and the launch
//     completes whatever part of the grid is resident.  All remote data accesses are LOADS
//     (pull), so no PE's L2 can hold stale copies of bytes a peer wrote.
#pragma once
#include <algorithm>
#include <map>
#include <mutex>
#include <type_traits>

#include "kernels.h"

namespace ishmemi {
namespace {

// sc0|sc1 cache policy on gfx950 buffer instructions = system-coherent access.
constexpr int kSysCoherent = 17;
constexpr uint64_t kTile = (uint64_t) kBlock * kUnroll;  // items per tile

template <typename T>
struct alignas(16) Vec {
    T e[16 / sizeof(T)];
};

template <typename T>
struct WideOf {
    using type = uint32_t;
};
template <>
struct WideOf<uint64_t> {
    using type = uint64_t;
};

// reduce_op semantics of src/collectives/reduce_impl.h:83-102 on canonical types.
template <typename T, int OP>
__device__ __forceinline__ T op1(T a, T b)
{
    if constexpr (OP == ISHMEMI_OP_AND) return (T) (a & b);
    else if constexpr (OP == ISHMEMI_OP_OR) return (T) (a | b);
    else if constexpr (OP == ISHMEMI_OP_XOR) return (T) (a ^ b);
    else if constexpr (OP == ISHMEMI_OP_MAX) {
        if constexpr (std::is_same_v<T, float>) return fmaxf(a, b);
        else if constexpr (std::is_same_v<T, double>) return fmax(a, b);
        else return (a < b) ? b : a;
    } else if constexpr (OP == ISHMEMI_OP_MIN) {
        if constexpr (std::is_same_v<T, float>) return fminf(a, b);
        else if constexpr (std::is_same_v<T, double>) return fmin(a, b);
        else return (b < a) ? b : a;
    } else if constexpr (OP == ISHMEMI_OP_SUM) {
        if constexpr (std::is_floating_point_v<T>) return a + b;
        else return (T) ((typename WideOf<T>::type) a + (typename WideOf<T>::type) b);
    } else {
        if constexpr (std::is_floating_point_v<T>) return a * b;
        else return (T) ((typename WideOf<T>::type) a * (typename WideOf<T>::type) b);
    }
}

template <typename T, int OP>
__device__ __forceinline__ Vec<T> op1(const Vec<T> &a, const Vec<T> &b)
{
    Vec<T> r;
#pragma unroll
    for (int i = 0; i < (int) (16 / sizeof(T)); ++i) r.e[i] = op1<T, OP>(a.e[i], b.e[i]);
    return r;
}

__device__ __forceinline__ const char *uniform_ptr(const char *p)
{
    const uint64_t v = (uint64_t) p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t) v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t) (v >> 32));
    return (const char *) (((uint64_t) hi << 32) | lo);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const char *uniform_base)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(uniform_base), (short) 0,
                                             0x7FFFFFFF, 0x00020000);
}

// System-coherent (sc0 sc1) load of one item from a peer's memory.
template <typename I>
__device__ __forceinline__ I cload(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    if constexpr (sizeof(I) == 16) {
        return __builtin_bit_cast(I, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSysCoherent));
    } else if constexpr (sizeof(I) == 8) {
        return __builtin_bit_cast(I, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kSysCoherent));
    } else if constexpr (sizeof(I) == 4) {
        return __builtin_bit_cast(I, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, kSysCoherent));
    } else if constexpr (sizeof(I) == 2) {
        return __builtin_bit_cast(I, __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, kSysCoherent));
    } else {
        return __builtin_bit_cast(I, __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, kSysCoherent));
    }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// Streaming store that does not keep the line in L2 / Infinity Cache (output is not re-read).
template <typename I>
__device__ __forceinline__ void nt_store(I *p, const I &v)
{
    if constexpr (sizeof(I) == 16) __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), (u32x4 *) p);
    else __builtin_nontemporal_store(v, p);
}

// System-coherent write-through store (sc0 sc1): the line is not left dirty in this XCD's L2, so
// the release before the hand-off flag is cheap and peers' coherent loads see memory.
template <typename I>
__device__ __forceinline__ void wt_store(__amdgpu_buffer_rsrc_t r, uint32_t off, const I &v)
{
    if constexpr (sizeof(I) == 16) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, kSysCoherent);
    else if constexpr (sizeof(I) == 8) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, kSysCoherent);
    else if constexpr (sizeof(I) == 4) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, kSysCoherent);
    else if constexpr (sizeof(I) == 2) __builtin_amdgcn_raw_buffer_store_b16(__builtin_bit_cast(uint16_t, v), r, off, 0, kSysCoherent);
    else __builtin_amdgcn_raw_buffer_store_b8(__builtin_bit_cast(uint8_t, v), r, off, 0, kSysCoherent);
}

// Kernel epochs live on the device: every workgroup of a launch reads the team's counter at
// its start (epoch = counter + 1) and the last workgroup to finish stores the new value.
// Collectives of a team are stream-ordered, so the next launch sees it; a captured hipGraph
// therefore replays with fresh epochs every time.  0 is the flags' initial value and never an
// epoch; at the wrap the sequence goes 0xFFFFFFFF -> 2, so consecutive epochs always differ in
// parity (the small-message rings are indexed by epoch parity).
template <typename A>
__device__ __forceinline__ uint32_t kernel_epoch(const A &a)
{
    __shared__ uint32_t s_ep;
    if (threadIdx.x == 0) {
        const uint32_t e =
            __hip_atomic_load(a.ep_ctr + kEpEpoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
        s_ep = e == 0 ? 2u : e;
    }
    __syncthreads();
    return s_ep;
}

template <typename A>
__device__ __forceinline__ void kernel_epoch_done(const A &a, uint32_t ep)
{
    if (threadIdx.x == 0) {
        if (__hip_atomic_fetch_add(a.ep_ctr + kEpDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) ==
            gridDim.x - 1) {
            __hip_atomic_store(a.ep_ctr + kEpDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(a.ep_ctr + kEpEpoch, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__device__ __forceinline__ uint32_t *flag_slot(uint32_t *base, int phase, int slot)
{
    return base + ((size_t) phase * kMaxBlocks + (size_t) slot) * kMaxPes;
}

// One lane: store epoch `ep` into this member's slot of row (phase, slot) on every other member
// (and on itself when `self`) — system-scope stores over xGMI into fine-grained memory.
template <typename A>
__device__ __forceinline__ void push_flag(const A &a, int phase, int slot, uint32_t ep, bool self)
{
    for (int j = 0; j < a.p; ++j) {
        if (j == a.me && !self) continue;
        uint32_t *f = flag_slot(j == a.me ? a.my_flags : a.peer_flags[j], phase, slot) + a.me;
        __hip_atomic_store(f, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// All threads: every wave's stores (all payload stores are write-through sc0 sc1) are
// acknowledged before the workgroup barrier (Guideline 16, R1).
__device__ __forceinline__ void drain_block()
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

// One lane, before a hand-off flag: system-scope release.  Nothing of ours is dirty (write-through
// payload stores), so it only orders the drained stores before the flag; the asm wait guards the
// compiler dropping the wait after buffer_wbl2 (MI355X_MICROARCH.md, compiler hazard).
__device__ __forceinline__ void release_system()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <typename A>
__device__ __forceinline__ void launch_fail(const A &a, int phase)
{
    __hip_atomic_store(a.ep_ctr + kEpFail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_or(a.err, 1u << phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// All threads call.  Wave 0 polls row (phase, slot) of the local flag block until the slot of
// every member selected by `who` holds `ep` or a later epoch (wrap-safe): who = -1 every other
// member, -2 every member including this one, >= 0 that member only.  Bounded: false on timeout
// (recorded in the team's error word) or once another workgroup of this launch has timed out.
// No acquire instruction follows: every load of bytes another PE produced is a system-coherent
// (sc0 sc1) load, which neither L1 nor a stale L2 line can satisfy; the wavefront fence only
// keeps the compiler from hoisting those loads above the poll (cdna_hip_programming.md
// Guideline 16).
template <typename A>
__device__ bool block_wait(const A &a, uint32_t ep, int phase, int slot, int who)
{
    __shared__ int s_ok;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        bool done = lane >= a.p || (who == -1 && lane == a.me) || (who >= 0 && lane != who);
        const uint32_t *row = flag_slot(a.my_flags, phase, slot);
        bool ok = true;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (uint32_t it = 0;; ++it) {
            if (!done) {
                const uint32_t v = __hip_atomic_load(row + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                done = (int32_t) (v - ep) >= 0;
            }
            if (__all(done)) break;
            if ((it & 15) == 15) {
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                    if (lane == 0) launch_fail(a, phase);
                    ok = false;
                    break;
                }
                if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(
                        a.ep_ctr + kEpFail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0) {
                    ok = false;
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

// All threads call: one returning device-scope add on a launch word, broadcast to the block
// (the dequeue primitive of MI355X_MICROARCH.md's price list).
template <typename A>
__device__ __forceinline__ uint32_t block_grab(const A &a, int word)
{
    __shared__ uint32_t s_v;
    __syncthreads();  // every thread has read the previous value
    if (threadIdx.x == 0)
        s_v = __hip_atomic_fetch_add(a.ep_ctr + word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return s_v;
}

// Start of a collective launch (replaces the start half of ishmemi_team_sync,
// src/collectives/sync_impl.h:30-69).  The first workgroup to run announces the launch to every
// other member — this member's source is final, since the launch runs after everything before it
// on the stream — and every workgroup waits until every member has announced the same launch.
// No workgroup waits for a particular peer workgroup, so residency never matters.
template <typename A>
__device__ bool launch_start(const A &a, uint32_t ep)
{
    if (threadIdx.x == 0 &&
        __hip_atomic_fetch_add(a.ep_ctr + kEpStarted, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0)
        push_flag(a, kPhaseStart, 0, ep, false);
    return block_wait(a, ep, kPhaseStart, 0, -1);
}

// End of a collective launch; every workgroup calls it once.  The last workgroup to finish
// tells every member that this member has finished reading their memory and waits until every
// member has said the same, so neither a member's next launch nor its caller can overwrite bytes
// a peer still reads (the end half of ishmemi_team_sync).  It then ORs a failure into *ret
// (the caller zeroed it before the call: sticky over the launches of one call), resets the
// launch words and publishes the epoch.
template <typename A>
__device__ void launch_finish(const A &a, uint32_t ep)
{
    __shared__ int s_last;
    drain_block();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(a.ep_ctr + kEpDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 gridDim.x - 1;
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x == 0) push_flag(a, kPhaseEnd, 0, ep, false);
    const bool ok = block_wait(a, ep, kPhaseEnd, 0, -1);
    if (threadIdx.x == 0) {
        uint32_t *w = a.ep_ctr;
        const bool failed =
            !ok || __hip_atomic_load(w + kEpFail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        if (failed && a.ret) __hip_atomic_fetch_or(a.ret, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int k = kEpDone; k < kEpWords; ++k)
            __hip_atomic_store(w + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(w + kEpEpoch, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Standalone barrier of one workgroup (team_sync_kernel): member me stores the call's epoch into
// its own slot of every peer's row, then polls its local row.
template <typename A>
__device__ bool pe_barrier(const A &a, uint32_t ep, int phase, int slot)
{
    drain_block();
    if (threadIdx.x == 0) push_flag(a, phase, slot, ep, false);
    return block_wait(a, ep, phase, slot, -1);
}

// One reduce-scatter tile for a compile-time team size P and load rotation R: slot k holds member
// (R + k) mod P, every register index is a compile-time constant (no scratch), the P loads of a
// half tile are all in flight before the canonical-order fold.
template <typename T, int OP, bool VEC, int P, int R>
__device__ __forceinline__ void rs_tile(const ReduceArgs &a, uint64_t t0, uint64_t ce,
                                        uint64_t head_bytes)
{
    using Item = std::conditional_t<VEC, Vec<T>, T>;
    constexpr uint64_t IB = sizeof(Item);
    constexpr int H = sizeof(T) >= 4 ? 2 : 1;  // items per thread per step: P * H staged in registers
    const int tid = threadIdx.x;
#pragma unroll
    for (int h = 0; h < kUnroll / H; ++h) {
        Item x[H][P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const int j = (R + k) % P;
            const char *base = uniform_ptr(a.src[j] + head_bytes + t0 * IB);
            if (j == a.me) {
                const Item *lp = (const Item *) base;
#pragma unroll
                for (int u = 0; u < H; ++u) {
                    const uint64_t e = (uint64_t) (h * H + u) * kBlock + tid;
                    if (t0 + e < ce) x[u][k] = lp[e];
                }
            } else {
                const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
#pragma unroll
                for (int u = 0; u < H; ++u) {
                    const uint64_t e = (uint64_t) (h * H + u) * kBlock + tid;
                    if (t0 + e < ce) x[u][k] = cload<Item>(r, (uint32_t) (e * IB));
                }
            }
        }
        const __amdgpu_buffer_rsrc_t dr = make_rsrc(uniform_ptr(a.dst + head_bytes + t0 * IB));
#pragma unroll
        for (int u = 0; u < H; ++u) {
            Item acc = x[u][(P - R) % P];  // member 0
#pragma unroll
            for (int j = 1; j < P; ++j) acc = op1<T, OP>(acc, x[u][(j - R + P) % P]);
            const uint64_t e = (uint64_t) (h * H + u) * kBlock + tid;
            if (t0 + e < ce) wt_store(dr, (uint32_t) (e * IB), acc);
        }
    }
}

// Wave-uniform run-time rotation -> compile-time rs_tile<R> (a uniform branch per tile).
template <typename T, int OP, bool VEC, int P, int R = 0>
__device__ __forceinline__ void rs_tile_dispatch(const ReduceArgs &a, int rot, uint64_t t0,
                                                 uint64_t ce, uint64_t head_bytes)
{
    if constexpr (R == P - 1) {
        rs_tile<T, OP, VEC, P, R>(a, t0, ce, head_bytes);
    } else {
        if (rot == R) rs_tile<T, OP, VEC, P, R>(a, t0, ce, head_bytes);
        else rs_tile_dispatch<T, OP, VEC, P, R + 1>(a, rot, t0, ce, head_bytes);
    }
}

// Run-time team size: the fold is rotated only where the op is order-insensitive (integers,
// min, max — bit-identical in any order), otherwise loaded and folded in team order.
template <typename T, int OP, bool VEC>
__device__ __forceinline__ void rs_tile_any(const ReduceArgs &a, int rot, uint64_t t0, uint64_t ce,
                                            uint64_t head_bytes)
{
    using Item = std::conditional_t<VEC, Vec<T>, T>;
    constexpr uint64_t IB = sizeof(Item);
    constexpr bool kOrderFree =
        !(std::is_floating_point_v<T> && (OP == ISHMEMI_OP_SUM || OP == ISHMEMI_OP_PROD));
    const int tid = threadIdx.x, p = a.p;
    Item acc[kUnroll];
    for (int k = 0; k < p; ++k) {
        const int j = kOrderFree ? (rot + k) % p : k;
        const char *base = uniform_ptr(a.src[j] + head_bytes + t0 * IB);
        Item x[kUnroll];
        if (j == a.me) {
            const Item *lp = (const Item *) base;
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint64_t e = (uint64_t) u * kBlock + tid;
                if (t0 + e < ce) x[u] = lp[e];
            }
        } else {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint64_t e = (uint64_t) u * kBlock + tid;
                if (t0 + e < ce) x[u] = cload<Item>(r, (uint32_t) (e * IB));
            }
        }
        if (k == 0) {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) acc[u] = x[u];
        } else {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) acc[u] = op1<T, OP>(acc[u], x[u]);
        }
    }
    const __amdgpu_buffer_rsrc_t dr = make_rsrc(uniform_ptr(a.dst + head_bytes + t0 * IB));
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
        const uint64_t e = (uint64_t) u * kBlock + tid;
        if (t0 + e < ce) wt_store(dr, (uint32_t) (e * IB), acc[u]);
    }
}

// Member c's chunk of the reduce-scatter partition, [begin, end) in items.
__device__ __forceinline__ void chunk_of(const ReduceArgs &a, int c, uint64_t &cs, uint64_t &ce)
{
    cs = min((uint64_t) c * a.items_per_chunk, a.nitems);
    ce = min(cs + a.items_per_chunk, a.nitems);
}

// Segments of a chunk of `len` items: at least one, so an empty chunk (tiny arrays) still
// hands off its head / tail and a consumer never waits for a segment nobody publishes.
__device__ __forceinline__ uint32_t nsegs(uint64_t len, uint64_t seg)
{
    return (uint32_t) max<uint64_t>(1, (len + seg - 1) / seg);
}

// ---------------------------------------------------------------------------------------------
// Multi-PE reduce-scatter + all-gather (one launch per collective).
//   start    - launch_start: every member has announced this launch (sources final).
//   RS       - workgroups grab segments of chunk `me` from a work counter, fold each segment of
//              every member's source in canonical team order (peers via sc0 sc1 loads), store
//              it write-through into own dest, drain, and push "segment s ready" to every peer.
//   AG       - workgroups grab (peer j, segment s) items, round-robin over the peers so every
//              link is busy, wait for j's "segment s ready" in the LOCAL flag row and pull it
//              from j's dest.  In place, the AG store into chunk j overwrites bytes member j
//              read in its RS of segment s, which it had finished before publishing s.
//   finish   - launch_finish: the last workgroup exchanges "done reading" with every member.
// Every workgroup grabs RS work before AG work, so any workgroup waiting in AG implies that all
// RS segments are held by running workgroups that wait for nothing but the start flags: the
// launch completes whatever subset of its grid (and of its peers' grids) is resident.
// ---------------------------------------------------------------------------------------------
template <typename T, int OP, bool VEC, int P>
__global__ __launch_bounds__(kBlock) __attribute__((flatten)) void allreduce_kernel(ReduceArgs a)
{
    using Item = std::conditional_t<VEC, Vec<T>, T>;
    constexpr uint64_t IB = sizeof(Item);
    const int tid = threadIdx.x;
    const int p = a.p, me = a.me;
    const uint64_t head_bytes = VEC ? a.head * sizeof(T) : 0;
    const uint64_t seg = a.seg_items;
    const bool one = a.oneshot != 0;
    const uint32_t ep = kernel_epoch(a);
    bool ok = launch_start(a, ep);

    // ---- reduce-scatter of chunk `me` (one-shot: the whole array) ----
    uint64_t cs = 0, ce = a.nitems;
    if (!one) chunk_of(a, me, cs, ce);
    const uint32_t nseg = nsegs(ce - cs, seg);
    while (ok) {
        const uint32_t s = block_grab(a, kEpRsHead);
        if (s >= nseg) break;
        const uint64_t ss = cs + (uint64_t) s * seg, se = min(ss + seg, ce);
        // Load order rotated by segment: concurrently folded segments read from all members
        // (all links) at once; the fold order stays canonical 0..p-1.
        const int rot = (int) (s % (uint32_t) p);
        for (uint64_t t0 = ss; t0 < se; t0 += kTile) {
            if constexpr (P > 0) rs_tile_dispatch<T, OP, VEC, P>(a, rot, t0, se, head_bytes);
            else rs_tile_any<T, OP, VEC>(a, rot, t0, se, head_bytes);
        }
        // Unaligned head (owned by member 0) and tail (owned by member p-1; one-shot: both by
        // every member), element-wise, with segment 0.  Descriptors are based at the region
        // (offsets < 16 B), never at the array start (a > 2 GiB array exceeds a descriptor).
        if (VEC && s == 0) {
            const uint64_t tail_off = a.head + a.nitems * (16 / sizeof(T));
            for (int region = 0; region < 2; ++region) {
                const bool owner = one || (region == 0 ? me == 0 : me == p - 1);
                const uint64_t cnt = region == 0 ? a.head : a.tail;
                if (!owner || (uint64_t) tid >= cnt) continue;
                const uint64_t rbase = (region == 0 ? 0 : tail_off) * sizeof(T);
                const uint32_t off = (uint32_t) (tid * sizeof(T));
                T acc = T();
                for (int j = 0; j < p; ++j) {
                    T x;
                    if (j == me) x = ((const T *) (a.src[j] + rbase))[tid];
                    else x = cload<T>(make_rsrc(uniform_ptr(a.src[j] + rbase)), off);
                    acc = (j == 0) ? x : op1<T, OP>(acc, x);
                }
                wt_store(make_rsrc(uniform_ptr(a.dst + rbase)), off, acc);
            }
        }
        if (!one) {
            drain_block();
            if (tid == 0) {
                release_system();
                push_flag(a, kPhaseMid, (int) s, ep, false);
            }
        }
    }

    // ---- all-gather: pull every other member's reduced segments from its dest ----
    if (ok && !one) {
        const uint32_t per_peer = nsegs(min(a.items_per_chunk, a.nitems), seg);  // chunk 0 is the largest
        const uint32_t total = (uint32_t) (p - 1) * per_peer;
        for (;;) {
            const uint32_t i = block_grab(a, kEpAgHead);
            if (i >= total) break;
            const int j = (me + 1 + (int) (i % (uint32_t) (p - 1))) % p;
            const uint32_t s = i / (uint32_t) (p - 1);
            uint64_t js, je;
            chunk_of(a, j, js, je);
            if (s >= nsegs(je - js, seg)) continue;
            if (!block_wait(a, ep, kPhaseMid, (int) s, j)) {
                ok = false;
                break;
            }
            const uint64_t ss = js + (uint64_t) s * seg, se = min(ss + seg, je);
            for (uint64_t t0 = ss; t0 < se; t0 += kTile) {
                const __amdgpu_buffer_rsrc_t r = make_rsrc(uniform_ptr(a.dstp[j] + head_bytes + t0 * IB));
                Item x[kUnroll];
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const uint64_t k = (uint64_t) u * kBlock + tid;
                    if (t0 + k < se) x[u] = cload<Item>(r, (uint32_t) (k * IB));
                }
                const __amdgpu_buffer_rsrc_t dr = make_rsrc(uniform_ptr(a.dst + head_bytes + t0 * IB));
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const uint64_t k = (uint64_t) u * kBlock + tid;
                    if (t0 + k < se) wt_store(dr, (uint32_t) (k * IB), x[u]);
                }
            }
            if (VEC && s == 0) {
                const uint64_t tail_off = a.head + a.nitems * (16 / sizeof(T));
                const uint64_t rbase = (j == 0 ? 0 : tail_off) * sizeof(T);
                const bool do_head = (j == 0) && ((uint64_t) tid < a.head);
                const bool do_tail = (j == p - 1) && ((uint64_t) tid < a.tail);
                if (do_head || do_tail)
                    ((T *) (a.dst + rbase))[tid] =
                        cload<T>(make_rsrc(uniform_ptr(a.dstp[j] + rbase)), (uint32_t) (tid * sizeof(T)));
            }
        }
    }
    launch_finish(a, ep);
}

// ---------------------------------------------------------------------------------------------
// Local fan-in combine: dst = op(src_0, ..., src_{k-1}), folded in source order.
// Measured on MI355X (tools/stream_variants.hip, 1 GiB operands, profiles/r01_extra/
// stream_variants*.txt): a one-shot grid with ONE 16-B item per thread is the fastest shape;
// persistent grid-stride loops with 4-8 items per thread reached only 63-73 %, an XCD-aware
// contiguous block order 77-80 %.  One-wave workgroups with nontemporal loads and
// system-coherent write-through 16-B stores (sc0 sc1: the line leaves L2 at once, like nt, but
// the store retires sooner) gave copy 84.2 % / a + b 84.7 % of the 8 TB/s HBM peak, against
// 81.8 % / 82.2 % for 128-thread blocks with nt stores.  Element-granular (non-vector) items keep
// nt stores: narrow sc1 stores are one fabric write each (MI355X_MICROARCH.md, store flavours).
// NS = 1 / 2 are specialised so every load is in flight before the fold; NS = 0 handles any
// source count at run time.
// ---------------------------------------------------------------------------------------------
template <typename I>
__device__ __forceinline__ I nt_load(const I *p)
{
    if constexpr (sizeof(I) == 16) return __builtin_bit_cast(I, __builtin_nontemporal_load((const u32x4 *) p));
    else return __builtin_nontemporal_load(p);
}

template <typename T, int OP, bool VEC, int NS>
__global__ __launch_bounds__(kFaninBlock) void fanin_kernel(FaninArgs a)
{
    using Item = std::conditional_t<VEC, Vec<T>, T>;
    constexpr uint64_t IB = sizeof(Item);
    const uint64_t head_bytes = VEC ? a.head * sizeof(T) : 0;
    const uint64_t stride = (uint64_t) gridDim.x * kFaninBlock;
    for (uint64_t i = (uint64_t) blockIdx.x * kFaninBlock + threadIdx.x; i < a.nitems; i += stride) {
        const uint64_t off = head_bytes + i * IB;
        Item acc;
        if constexpr (NS == 1) {
            acc = nt_load((const Item *) (a.src[0] + off));
        } else if constexpr (NS == 2) {
            const Item x0 = nt_load((const Item *) (a.src[0] + off));
            const Item x1 = nt_load((const Item *) (a.src[1] + off));
            acc = op1<T, OP>(x0, x1);
        } else {
            acc = nt_load((const Item *) (a.src[0] + off));
            for (int j = 1; j < a.nsrc; ++j) acc = op1<T, OP>(acc, nt_load((const Item *) (a.src[j] + off)));
        }
        if constexpr (VEC) {
            // Descriptor based at this workgroup's first item (offsets < 1 KiB, any array size).
            const char *wbase = uniform_ptr(a.dst + off - (uint64_t) threadIdx.x * IB);
            wt_store(make_rsrc(wbase), (uint32_t) (threadIdx.x * IB), acc);
        } else {
            nt_store((Item *) (a.dst + off), acc);
        }
    }
    if (VEC && blockIdx.x == 0) {
        const int tid = threadIdx.x;
        const uint64_t tail_off = a.head + a.nitems * (16 / sizeof(T));
        for (int pass = 0; pass < 2; ++pass) {
            if ((uint64_t) tid >= (pass == 0 ? a.head : a.tail)) continue;
            const uint64_t e = pass == 0 ? (uint64_t) tid : tail_off + tid;
            T acc = ((const T *) a.src[0])[e];
            for (int j = 1; j < a.nsrc; ++j) acc = op1<T, OP>(acc, ((const T *) a.src[j])[e]);
            ((T *) a.dst)[e] = acc;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Small-message path: one data hop, no barriers.  Thread t owns 8 payload bytes (item t): it
// pushes them as two {data, epoch} granules into slot `me` of every peer's ring (system-scope
// 8-B atomic stores into fine-grained memory: a granule is its own flag, MI355X_MICROARCH.md
// R2), then polls its own ring until all p-1 peers' granules for item t carry this epoch and
// folds the p items in canonical team order.  Sources are reusable at once (they were copied);
// ring parity = epoch & 1, and a peer can be at most one collective ahead (it cannot finish
// collective e+1 without our e+1 push), so two parities never collide.
// ---------------------------------------------------------------------------------------------
template <typename T, int OP>
__device__ __forceinline__ uint64_t fold8(uint64_t acc, uint64_t x)
{
    constexpr int K = 8 / sizeof(T);
    struct alignas(8) W {
        T e[K];
    };
    W a = __builtin_bit_cast(W, acc), b = __builtin_bit_cast(W, x);
#pragma unroll
    for (int i = 0; i < K; ++i) a.e[i] = op1<T, OP>(a.e[i], b.e[i]);
    return __builtin_bit_cast(uint64_t, a);
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void ll_kernel(LLArgs a)
{
    const uint64_t item = (uint64_t) blockIdx.x * kBlock + threadIdx.x;
    const uint64_t nitems = (a.nbytes + 7) / 8;
    const int p = a.p, me = a.me;
    const uint32_t ep = kernel_epoch(a);
    const uint64_t par = ep & 1u;
    const uint64_t tag = (uint64_t) ep << 32;
    bool ok = true;
    if (item < nitems) {
        const uint64_t off = item * 8;
        const uint64_t valid = a.nbytes - off < 8 ? a.nbytes - off : 8;
        uint64_t mine = 0;
        if (valid == 8) mine = *(const uint64_t *) (a.src + off);
        else memcpy(&mine, a.src + off, valid);
        const uint64_t g0 = tag | (uint32_t) mine, g1 = tag | (uint32_t) (mine >> 32);
        for (int j = 0; j < p; ++j) {
            if (j == me) continue;
            uint64_t *slot = a.peer_ring[j] + (par * kMaxPes + me) * kLLGranules + 2 * item;
            __hip_atomic_store(slot, g0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(slot + 1, g1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        uint64_t acc = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (int j = 0; j < p && ok; ++j) {
            uint64_t x = mine;
            if (j != me) {
                const uint64_t *slot = a.my_ring + (par * kMaxPes + j) * kLLGranules + 2 * item;
                uint64_t h0, h1;
                for (;;) {
                    h0 = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    h1 = __hip_atomic_load(slot + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if ((h0 >> 32) == ep && (h1 >> 32) == ep) break;
                    if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeout_ticks) {
                        ok = false;
                        __hip_atomic_fetch_or(a.err, 1u << 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                x = (h0 & 0xffffffffull) | (h1 << 32);
            }
            acc = (j == 0) ? x : fold8<T, OP>(acc, x);
        }
        if (ok) {
            if (valid == 8) *(uint64_t *) (a.dst + off) = acc;
            else memcpy(a.dst + off, &acc, valid);
        }
    }
    // *ret was zeroed by the caller: any thread that failed marks it (sticky over launches).
    if (!ok && a.ret) __hip_atomic_fetch_or(a.ret, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    kernel_epoch_done(a, ep);
}

template <typename T, int OP>
hipError_t ll_t(const LLArgs &a, hipStream_t s)
{
    const uint64_t nitems = (a.nbytes + 7) / 8;
    const int grid = (int) ((nitems + kBlock - 1) / kBlock);
    hipLaunchKernelGGL((ll_kernel<T, OP>), dim3(grid > 0 ? grid : 1), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

// Standalone team barrier (ishmem_team_sync / barrier_all analogue): one workgroup.
__global__ __launch_bounds__(kBlock) void team_sync_kernel(ReduceArgs a)
{
    const uint32_t ep = kernel_epoch(a);
    const bool ok = pe_barrier(a, ep, kPhaseSync, 0);
    if (threadIdx.x == 0 && !ok && a.ret)
        __hip_atomic_fetch_or(a.ret, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    kernel_epoch_done(a, ep);
}

// Canonical kernel type: MIN/MAX keep the signedness, every other integer op folds on the
// unsigned type of the same width (bit-identical two's-complement results).
template <int OP, typename S, typename U>
using Canon = std::conditional_t<(OP == ISHMEMI_OP_MAX || OP == ISHMEMI_OP_MIN), S, U>;

// Workgroups of `kernel` that are resident at once on this device (cached per kernel address),
// divided among the PEs sharing the device.  The collectives are correct with any residency of
// their own grid (they grab work; nothing is paired); the clamp avoids launching workgroups that
// would find no work left, and keeps co-located PEs' launches from crowding each other out.  One block per CU of margin:
// the occupancy API over-reports by one block per CU for SGPR-heavy 256-thread kernels on
// ROCm 7.2 (MI355X_MICROARCH.md, residency).
inline int resident_blocks_of(const void *kernel)
{
    static std::mutex mu;
    static std::map<const void *, int> cache;
    std::lock_guard<std::mutex> lk(mu);
    auto it = cache.find(kernel);
    if (it != cache.end()) return std::max(1, it->second / device_share());
    int dev = 0, cus = 0, per = 0;
    (void) hipGetDevice(&dev);
    (void) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, kBlock, 0) != hipSuccess) {
        (void) hipGetLastError();
        per = 1;
    }
    const int n = std::max(1, (per > 1 ? per - 1 : 1) * std::max(cus, 1));
    cache[kernel] = n;
    return std::max(1, n / device_share());
}

template <typename K>
int resident_blocks(K kernel)
{
    return resident_blocks_of((const void *) kernel);
}

template <typename K>
hipError_t launch_resident(K kernel, const ReduceArgs &a, int grid, hipStream_t s)
{
    grid = std::min(grid, resident_blocks(kernel));
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <typename T, int OP>
hipError_t ar_t(bool vec, const ReduceArgs &a, int grid, hipStream_t s)
{
    if (!vec) return launch_resident(allreduce_kernel<T, OP, false, 0>, a, grid, s);
    if (a.p == 2) return launch_resident(allreduce_kernel<T, OP, true, 2>, a, grid, s);
    if (a.p == 4) return launch_resident(allreduce_kernel<T, OP, true, 4>, a, grid, s);
    if (a.p == 8) return launch_resident(allreduce_kernel<T, OP, true, 8>, a, grid, s);
    return launch_resident(allreduce_kernel<T, OP, true, 0>, a, grid, s);
}

template <typename T, int OP, bool VEC>
void fi_ns(const FaninArgs &a, int grid, hipStream_t s)
{
    if (a.nsrc == 1) hipLaunchKernelGGL((fanin_kernel<T, OP, VEC, 1>), dim3(grid), dim3(kFaninBlock), 0, s, a);
    else if (a.nsrc == 2) hipLaunchKernelGGL((fanin_kernel<T, OP, VEC, 2>), dim3(grid), dim3(kFaninBlock), 0, s, a);
    else hipLaunchKernelGGL((fanin_kernel<T, OP, VEC, 0>), dim3(grid), dim3(kFaninBlock), 0, s, a);
}

template <typename T, int OP>
hipError_t fi_t(bool vec, const FaninArgs &a, int grid, hipStream_t s)
{
    if (vec) fi_ns<T, OP, true>(a, grid, s);
    else fi_ns<T, OP, false>(a, grid, s);
    return hipGetLastError();
}

template <int OP, typename A, typename L>
hipError_t dispatch_dt(int dt, L &&launch)
{
    constexpr bool fp_ok = OP >= ISHMEMI_OP_MAX;
    switch (dt) {
        case ISHMEMI_DT_INT8: return launch.template operator()<Canon<OP, int8_t, uint8_t>, OP>();
        case ISHMEMI_DT_INT16: return launch.template operator()<Canon<OP, int16_t, uint16_t>, OP>();
        case ISHMEMI_DT_INT32: return launch.template operator()<Canon<OP, int32_t, uint32_t>, OP>();
        case ISHMEMI_DT_INT64: return launch.template operator()<Canon<OP, int64_t, uint64_t>, OP>();
        case ISHMEMI_DT_UINT8: return launch.template operator()<uint8_t, OP>();
        case ISHMEMI_DT_UINT16: return launch.template operator()<uint16_t, OP>();
        case ISHMEMI_DT_UINT32: return launch.template operator()<uint32_t, OP>();
        case ISHMEMI_DT_UINT64: return launch.template operator()<uint64_t, OP>();
        case ISHMEMI_DT_FLOAT:
            if constexpr (fp_ok) return launch.template operator()<float, OP>();
            else return hipErrorInvalidValue;
        case ISHMEMI_DT_DOUBLE:
            if constexpr (fp_ok) return launch.template operator()<double, OP>();
            else return hipErrorInvalidValue;
        default: return hipErrorInvalidValue;
    }
}

template <typename A, typename L>
hipError_t dispatch(int op, int dt, L &&launch)
{
    switch (op) {
        case ISHMEMI_OP_AND: return dispatch_dt<ISHMEMI_OP_AND, A>(dt, launch);
        case ISHMEMI_OP_OR: return dispatch_dt<ISHMEMI_OP_OR, A>(dt, launch);
        case ISHMEMI_OP_XOR: return dispatch_dt<ISHMEMI_OP_XOR, A>(dt, launch);
        case ISHMEMI_OP_MAX: return dispatch_dt<ISHMEMI_OP_MAX, A>(dt, launch);
        case ISHMEMI_OP_MIN: return dispatch_dt<ISHMEMI_OP_MIN, A>(dt, launch);
        case ISHMEMI_OP_SUM: return dispatch_dt<ISHMEMI_OP_SUM, A>(dt, launch);
        case ISHMEMI_OP_PROD: return dispatch_dt<ISHMEMI_OP_PROD, A>(dt, launch);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace
}  // namespace ishmemi
