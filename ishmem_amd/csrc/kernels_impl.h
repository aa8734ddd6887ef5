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
//   * rs_phase_kernel / ag_phase_kernel: the same reduce-scatter + all-gather for large payloads
//     as two one-shot grids (the fan-in kernel's shape) between one-workgroup team barriers —
//     nothing in either grid waits, so it runs at the streaming kernels' rate (round 3).
//   * ll_kernel: small payloads (up to 512 KiB, 2 MiB / p) with no handshake at all: every member
//     pushes its bytes as {4 B data, 32-bit epoch} granules into every peer's ring and folds what
//     it receives; the same exchange carries small fcollect, sum scans and broadcasts (round 5).
//   * The barriers replace ishmemi_team_sync's psync counters (src/collectives/sync_impl.h:30-69)
//     with epoch-tagged flags in fine-grained memory: one "started" flag per member, one
//     "ready" flag per reduced segment (the RS -> AG hand-off) and one "done reading" flag per
//     member, exchanged by whichever workgroup gets there; work is grabbed from per-launch
//     counters, so no workgroup ever waits for a particular peer workgroup and the launch
//     completes whatever part of the grid is resident.  All remote payload accesses outside the
//     granule rings are LOADS (pull), so no PE's L2 can hold stale copies of bytes a peer wrote;
//     the rings are uncached fine-grained memory written and polled with system-scope atomics.
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
constexpr int kNonTemporal = 2;  // buffer aux bits: nt
constexpr uint64_t kTile = (uint64_t) kBlock * kUnroll;  // items per tile
#ifndef ISHMEMI_AR_OCC
#define ISHMEMI_AR_OCC 4  // multi-PE kernel: workgroups per CU (see allreduce_kernel)
#endif


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

// Nontemporal 16-B buffer load (scalar base + 32-bit lane offset).
template <typename I>
__device__ __forceinline__ I bload(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    static_assert(sizeof(I) == 16, "bload: 16-B items");
    return __builtin_bit_cast(I, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kNonTemporal));
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
        const uint32_t *rep = a.ep_ctr + (kEpRepLine + blockIdx.x % kEpReplicas) * kLineWords;
        const uint32_t e = __hip_atomic_load(rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) + 1u;
        s_ep = e == 0 ? 2u : e;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(s_ep);
}

// One whole wave: the team's epoch and its 64 replicas (one per lane, each on its own line).
template <typename A>
__device__ __forceinline__ void publish_epoch_wave(const A &a, uint32_t ep)
{
    const int r = threadIdx.x & 63;
    __hip_atomic_store(a.ep_ctr + (kEpRepLine + r) * kLineWords, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (r == 0) __hip_atomic_store(a.ep_ctr + kEpEpoch, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// End of the small kernels (LL, team sync; grids of a few workgroups): the last workgroup
// publishes the epoch.  All threads call.
template <typename A>
__device__ __forceinline__ void kernel_epoch_done(const A &a, uint32_t ep)
{
    __shared__ int s_last;
    // A one-workgroup grid (the team barrier, which the phased paths launch three times per call)
    // is its own last workgroup: no returning atomic on its critical path.
    if (threadIdx.x == 0)
        s_last = gridDim.x == 1 ||
                 __hip_atomic_fetch_add(a.ep_ctr + kEpDone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                     gridDim.x - 1;
    __syncthreads();
    if (s_last && threadIdx.x < 64) {
        // Every launch word back to zero, the failure word included (a timed-out team sync must
        // not make the team's next collective drain at once), as launch_finish does.
        if (threadIdx.x == 0)
            for (int k = kEpDone; k < kEpWords; ++k)
                __hip_atomic_store(a.ep_ctr + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        publish_epoch_wave(a, ep);
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
// Returns 0 when the flags are there, 1 on timeout / launch failure, 2 when `patience` ticks
// (0 = unlimited) passed first — the caller may then do something else and wait again.
template <typename A>
__device__ int block_wait_ex(const A &a, uint32_t ep, int phase, int slot, int who, uint64_t patience)
{
    __shared__ int s_ok;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        bool done = lane >= a.p || (who == -1 && lane == a.me) || (who >= 0 && lane != who);
        const uint32_t *row = flag_slot(a.my_flags, phase, slot);
        int st = 0;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        // One poll in flight, then a back-off once the wait is long: hundreds of waiting
        // workgroups polling uncached memory back to back take HBM bandwidth from the workgroups
        // still streaming (two polls in flight, tried, slowed 1 GiB at 8 PEs on one GPU by 60 %).
        for (uint32_t it = 0;; ++it) {
            if (!done) {
                const uint32_t v = __hip_atomic_load(row + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                done = (int32_t) (v - ep) >= 0;
            }
            if (__all(done)) break;
            if ((it & 15) == 15) {
                const uint64_t waited = __builtin_amdgcn_s_memrealtime() - t0;
                if (waited > a.timeout_ticks) {
                    if (lane == 0) launch_fail(a, phase);
                    st = 1;
                    break;
                }
                if (patience && waited > patience) {
                    st = 2;
                    break;
                }
                if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(
                        a.ep_ctr + kEpFail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0) {
                    st = 1;
                    break;
                }
            }
            if (it < 32) __builtin_amdgcn_s_sleep(1);
            else __builtin_amdgcn_s_sleep(8);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) s_ok = st;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(s_ok);
}

template <typename A>
__device__ bool block_wait(const A &a, uint32_t ep, int phase, int slot, int who)
{
    return block_wait_ex(a, ep, phase, slot, who, 0) == 0;
}

// Work grabbing with one grab in flight (the dequeue primitive of MI355X_MICROARCH.md's price
// list: a returning device-scope add on a launch word, ~1 us under load).  grab_issue: lane 0
// issues the add and does not wait; grab_take (all threads) waits for it and broadcasts the
// value.  Issued before an item's loads, the add's latency hides behind them.
// Lane roles inside a 256-thread workgroup: wave 0 polls flags, lane kSignalLane (wave 1) stores
// flags to peers, lane kGrabLane (wave 2) issues work grabs.  gfx9-family waves count loads,
// stores and returning atomics in ONE in-order vmcnt, so a poll issued by the wave that just
// stored a flag over xGMI (or issued a grab) would first wait for that store's acknowledgement:
// separate waves keep the three latencies from adding up.
constexpr int kSignalLane = 64, kGrabLane = 128;

template <typename A>
__device__ __forceinline__ void grab_issue(const A &a, int word, uint32_t &pending)
{
    if (threadIdx.x == kGrabLane)
        pending = __hip_atomic_fetch_add(a.ep_ctr + word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t grab_take(uint32_t pending)
{
    __shared__ uint32_t s_v;
    __syncthreads();  // every thread has read the previous value
    if (threadIdx.x == kGrabLane) s_v = pending;
    __syncthreads();
    // Block-uniform: keep it (and everything derived from it) in scalar registers.
    return __builtin_amdgcn_readfirstlane(s_v);
}

template <typename A>
__device__ __forceinline__ uint32_t block_grab(const A &a, int word)
{
    uint32_t pending = 0;
    grab_issue(a, word, pending);
    return grab_take(pending);
}

// Development trace (ReduceArgs::trace, set_param "trace_buffer"): per workgroup, s_memrealtime
// (100 MHz) at kernel entry, start satisfied, RS done, AG done, finish entered, and — for the
// launch's last workgroup — after the done handshake.  8 u64 slots per workgroup.
__device__ __forceinline__ void trace_mark(uint64_t *tr, int k)
{
    if (tr && threadIdx.x == 0) tr[(size_t) blockIdx.x * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

// Start of a collective launch (replaces the start half of ishmemi_team_sync,
// src/collectives/sync_impl.h:30-69).  The first workgroup to run announces the launch to every
// other member — this member's source is final, since the launch runs after everything before it
// on the stream — and every workgroup waits until every member has announced the same launch.
// No workgroup waits for a particular peer workgroup, so residency never matters.
// Workgroup 0 announces at once (no atomic on its path); whichever other workgroup runs first
// announces too (its "started" add returns 0), so the announcement never waits for a particular
// workgroup to be resident.  The duplicate stores the same epoch.
// The announcement is stored into kEpReplicas start slots of every peer (the signalling wave,
// one slot per lane), and workgroup b polls slot b mod kEpReplicas: hundreds of workgroups
// polling one 64-B line would queue on it.
// One whole wave: this member's start announcement into every peer's kEpReplicas start slots,
// then the local mark "announced in epoch ep" (word 1 of every epoch replica line).
template <typename A>
__device__ __forceinline__ void announce_wave(const A &a, uint32_t ep)
{
    const int r = threadIdx.x & 63;
    for (int j = 0; j < a.p; ++j) {
        if (j == a.me) continue;
        __hip_atomic_store(flag_slot(a.peer_flags[j], kPhaseStart, r) + a.me, ep, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __hip_atomic_store(a.ep_ctr + (kEpRepLine + r) * kLineWords + 1, ep, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup 0 announces at once, from the signalling wave (no atomic on any workgroup's path:
// 255 workgroups adding to one "started" word cost ~2.5 us here).  Every other workgroup, once
// it has seen every peer, checks the local "announced" mark and announces itself if it is not
// there yet (its PE must not do work peers depend on while peers still wait for it: workgroup 0
// may be queued behind other work).  A workgroup that has waited kAnnouncePatience without
// seeing every peer announces too — if workgroup 0 is not resident
// (CUs held by other work), any resident workgroup of the launch eventually speaks for it;
// duplicates store the same epoch.
constexpr uint64_t kAnnouncePatience = 2000;  // 20 us of s_memrealtime

template <typename A>
__device__ bool launch_start(const A &a, uint32_t ep)
{
    if (blockIdx.x == 0 && threadIdx.x >= kSignalLane && threadIdx.x < kSignalLane + 64)
        announce_wave(a, ep);
    const int slot = (int) (blockIdx.x % kEpReplicas);
    int st = block_wait_ex(a, ep, kPhaseStart, slot, -1, blockIdx.x == 0 ? 0 : kAnnouncePatience);
    if (st == 2) {
        if (threadIdx.x >= kSignalLane && threadIdx.x < kSignalLane + 64) announce_wave(a, ep);
        st = block_wait_ex(a, ep, kPhaseStart, slot, -1, 0);
    } else if (st == 0 && blockIdx.x != 0 && threadIdx.x >= kSignalLane && threadIdx.x < kSignalLane + 64) {
        const uint32_t mark = __hip_atomic_load(a.ep_ctr + (kEpRepLine + slot) * kLineWords + 1,
                                                __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__builtin_amdgcn_readfirstlane(mark) != ep) announce_wave(a, ep);
    }
    return st == 0;
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
    // No store drain: "done" speaks for this workgroup's LOADS of peer memory, all of which have
    // returned (their values were stored or folded); its own stores complete with the kernel.
    __syncthreads();
    if (threadIdx.x == 0) {
        // Finished count sharded by blockIdx mod kEpShards (~ per XCD under round-robin
        // dispatch); the workgroup completing a shard counts it at the top line.
        const uint32_t k = blockIdx.x % kEpShards;
        const uint32_t in_shard = (gridDim.x - k + kEpShards - 1) / kEpShards;
        int last = 0;
        if (__hip_atomic_fetch_add(a.ep_ctr + (kEpShardLine + k) * kLineWords, 1u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) == in_shard - 1) {
            const uint32_t shards = gridDim.x < (uint32_t) kEpShards ? gridDim.x : (uint32_t) kEpShards;
            last = __hip_atomic_fetch_add(a.ep_ctr + kEpTopLine * kLineWords, 1u, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT) == shards - 1;
        }
        s_last = last;
    }
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(s_last)) return;
    if (threadIdx.x == kSignalLane) push_flag(a, kPhaseEnd, 0, ep, false);
    const bool ok = block_wait(a, ep, kPhaseEnd, 0, -1);
    if constexpr (std::is_same_v<A, ReduceArgs>) trace_mark(a.trace, 5);
    if (threadIdx.x == 0) {
        uint32_t *w = a.ep_ctr;
        const bool failed =
            !ok || __hip_atomic_load(w + kEpFail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        if (failed && a.ret) __hip_atomic_fetch_or(a.ret, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int k = kEpDone; k < kEpWords; ++k)
            __hip_atomic_store(w + k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (int k = 0; k <= kEpShards; ++k)  // the shards and the top line
            __hip_atomic_store(w + (kEpShardLine + k) * kLineWords, 0u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    if (threadIdx.x < 64) publish_epoch_wave(a, ep);
}

// Standalone barrier of one workgroup (team_sync_kernel): member me stores the call's epoch into
// its own slot of every peer's row, then polls its local row.
template <typename A>
__device__ bool pe_barrier(const A &a, uint32_t ep, int phase, int slot)
{
    drain_block();
    if (threadIdx.x == kSignalLane) push_flag(a, phase, slot, ep, false);
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
    // Items per thread per step: P * H = 8 loads staged in registers for P in {2, 4, 8}
    // (MI355X_MICROARCH.md: keep >= 8 loads per lane outstanding on streamed hand-offs; more
    // pushed the kernel past 128 VGPRs, i.e. below 4 workgroups per CU).
#if ISHMEMI_AR_OCC >= 4
    constexpr int H = sizeof(T) >= 4 ? (P <= 2 ? 2 : 1) : 1;
#else
    constexpr int H = sizeof(T) >= 4 ? (P <= 2 ? 4 : P == 4 ? 2 : 1) : 1;
#endif
    const uint32_t tid = threadIdx.x;
    // Items left in this tile (wave-uniform, <= kTile): 32-bit per-lane bounds checks.
    const uint32_t lim = (uint32_t) min<uint64_t>(ce - t0, kTile);
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
                    const uint32_t e = (uint32_t) (h * H + u) * kBlock + tid;
                    if (e < lim) x[u][k] = lp[e];
                }
            } else {
                const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
#pragma unroll
                for (int u = 0; u < H; ++u) {
                    const uint32_t e = (uint32_t) (h * H + u) * kBlock + tid;
                    if (e < lim) x[u][k] = cload<Item>(r, e * (uint32_t) IB);
                }
            }
        }
        const __amdgpu_buffer_rsrc_t dr = make_rsrc(uniform_ptr(a.dst + head_bytes + t0 * IB));
#pragma unroll
        for (int u = 0; u < H; ++u) {
            Item acc = x[u][(P - R) % P];  // member 0
#pragma unroll
            for (int j = 1; j < P; ++j) acc = op1<T, OP>(acc, x[u][(j - R + P) % P]);
            const uint32_t e = (uint32_t) (h * H + u) * kBlock + tid;
            if (e < lim) wt_store(dr, e * (uint32_t) IB, acc);
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
    const uint32_t tid = threadIdx.x;
    const int p = a.p;
    const uint32_t lim = (uint32_t) min<uint64_t>(ce - t0, kTile);
    Item acc[kUnroll];
    for (int k = 0; k < p; ++k) {
        const int j = kOrderFree ? (rot + k) % p : k;
        const char *base = uniform_ptr(a.src[j] + head_bytes + t0 * IB);
        Item x[kUnroll];
        if (j == a.me) {
            const Item *lp = (const Item *) base;
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint32_t e = (uint32_t) u * kBlock + tid;
                if (e < lim) x[u] = lp[e];
            }
        } else {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint32_t e = (uint32_t) u * kBlock + tid;
                if (e < lim) x[u] = cload<Item>(r, e * (uint32_t) IB);
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
        const uint32_t e = (uint32_t) u * kBlock + tid;
        if (e < lim) wt_store(dr, e * (uint32_t) IB, acc[u]);
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
//   start  - launch_start: every member has announced this launch (sources final).
//   RS     - segment b of chunk `me` (contiguous tiles) belongs to workgroup b: it claims it (one
//            uncontended atomic exchange of the launch's epoch into the segment's claim word),
//            folds it from every member's source in canonical team order (peers via sc0 sc1
//            loads), stores it write-through into own dest, drains and pushes "segment b ready"
//            to every peer.  Segments G.. are grabbed from a work counter by whichever workgroup
//            is free (one grab per segment, in flight while the previous segment streams).
//   AG     - item i = (peer j, segment s), round-robin over the peers so every link is busy;
//            item b is workgroup b's, items G.. are grabbed.  It waits for j's "segment s ready"
//            in the LOCAL flag row and pulls the segment from j's dest.  In place, the AG store
//            into chunk j overwrites bytes member j read in its RS of segment s, which it finished
//            before publishing s.
//   finish - launch_finish: the last workgroup exchanges "done reading" with every member.
// Owned first segments cost no contended atomics when every workgroup has one segment (round
// 2's first version grabbed every segment from one counter: 256 workgroups x 2 grabs queued on
// one line, +6 us at 4 MiB); grabbing the rest keeps large arrays balanced when workgroups (or
// co-located PEs) run at uneven speeds (all-static ownership ran 1 GiB at 8 PEs on one GPU in
// 7.2 ms against 3.9 ms grabbed).  Residency: a peer only ever waits for RS segments; grabbed
// ones are held by running workgroups, and an AG waiter that has waited kStealPatience claims and
// reduces any still-unclaimed owned segment of its own PE (owner not resident) — the claim word
// makes every owned segment reduced exactly once.
// ---------------------------------------------------------------------------------------------
// Long enough that launch skew between PEs and ordinary waits never trigger it (a steal scans
// claim words); short against the device timeout.
constexpr uint64_t kStealPatience = 10000;  // 100 us of s_memrealtime

template <typename A>
__device__ __forceinline__ uint32_t *claim_word(const A &a, uint32_t s)
{
    return a.ep_ctr + kEpClaimLine * kLineWords + s;
}

// Lane kGrabLane issues the claim of segment s (old value returned later); claim_take
// broadcasts whether this workgroup won it.
template <typename A>
__device__ __forceinline__ void claim_issue(const A &a, uint32_t ep, uint32_t s, uint32_t &pending)
{
    if (threadIdx.x == kGrabLane)
        pending = __hip_atomic_exchange(claim_word(a, s), ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ bool claim_take(uint32_t pending, uint32_t ep)
{
    return grab_take(pending) != ep;
}

// Steal: wave 2 scans the claim words of [0, nseg) from the END (owners claim in increasing
// order, so unclaimed segments gather there) for one not yet claimed by this launch and claims
// it.  Returns the segment, or nseg if every segment is claimed.  All threads call.
template <typename A>
__device__ uint32_t steal_segment(const A &a, uint32_t ep, uint32_t nseg)
{
    __shared__ uint32_t s_found;
    if (threadIdx.x == kGrabLane) s_found = nseg;
    __syncthreads();
    if (threadIdx.x >= kGrabLane && threadIdx.x < kGrabLane + 64) {
        const uint32_t lane = threadIdx.x - kGrabLane;
        for (uint32_t top = nseg; top > 0; top = top > 64 ? top - 64 : 0) {
            const uint32_t s = top - 1 - lane;
            bool open = false;
            if (lane < top)
                open = __hip_atomic_load(claim_word(a, s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != ep;
            uint64_t mask = __ballot(open);
            bool got = false;
            while (mask && !got) {
                const uint32_t l = (uint32_t) __builtin_ctzll(mask);
                uint32_t old = ep;
                if (lane == l) old = __hip_atomic_exchange(claim_word(a, s), ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                got = __builtin_amdgcn_readlane(old, l) != ep;
                if (got && lane == l) s_found = s;
                mask &= mask - 1;
            }
            if (got) break;
        }
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(s_found);
}

// One reduce-scatter segment: tiles s, s + nseg, ... of [cs, ce), the unaligned head / tail with
// segment 0, then (not one-shot) drain and publish "segment s ready".
template <typename T, int OP, bool VEC, int P>
__device__ __forceinline__ void rs_segment(const ReduceArgs &a, uint32_t ep, uint32_t s, uint32_t nseg,
                                           uint64_t cs, uint64_t ce, uint64_t head_bytes, bool one)
{
    const int tid = threadIdx.x, p = a.p, me = a.me;
    // Load order rotated by segment: concurrently folded segments read from all members (all
    // links) at once; the fold order stays canonical 0..p-1.  A segment is contiguous (each
    // workgroup stays inside one 2 MiB page of every member's array for many tiles: a strided
    // tile set, tried, ran 7 % (2 PEs) to 30 % (8 PEs) slower at 1 GiB).
    const int rot = (int) (s % (uint32_t) p);
    const uint64_t ss = cs + (uint64_t) s * a.seg_items, se = min(ss + a.seg_items, ce);
    for (uint64_t t0 = ss; t0 < se; t0 += kTile) {
        const uint64_t te = min(t0 + kTile, se);
        if constexpr (P > 0) rs_tile_dispatch<T, OP, VEC, P>(a, rot, t0, te, head_bytes);
        else rs_tile_any<T, OP, VEC>(a, rot, t0, te, head_bytes);
    }
    (void) nseg;
    // Unaligned head (owned by member 0) and tail (owned by member p-1; one-shot: both by every
    // member), element-wise, with segment 0.  Descriptors are based at the region (offsets
    // < 16 B), never at the array start (a > 2 GiB array exceeds a descriptor's range).
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
        // Every payload store of the segment is a system-scope write-through store: once drained
        // (vmcnt(0) in every wave) its bytes are past this XCD's L2, so the flag needs no release
        // fence (MI355X_MICROARCH.md: handoff-flag, drained sc1 stores; cdna_hip_programming.md
        // R1).  A system-scope release here is a buffer_wbl2 per segment — 1024 of them per
        // launch, serialised per XCD — and made the reduce-scatter half the speed of the
        // all-gather (same-device trace, 128 MiB: 2.2 against 5.3 TB/s).
        drain_block();
        if (tid == kSignalLane) push_flag(a, kPhaseMid, (int) s, ep, false);
    }
}

// Workgroups per CU of the multi-PE kernel and all-gather tiles per step.  Round 3's A/B
// (profiles/r03/ab_occ/): 4 per CU with 4 loads per lane staged against round 2's
// 3 per CU with 8 — 8 PEs on one GPU 3.90 vs 4.55 ms per 1 GiB call, 2 PEs within noise
// (1.05 vs 1.07 ms).  ISHMEMI_AR_OCC=3 builds the round-2 shape (A/B variants only).
#if ISHMEMI_AR_OCC >= 4
constexpr int kArOcc = 4, kAgTiles = 1;
#else
constexpr int kArOcc = 3, kAgTiles = 2;
#endif
// Workgroups per CU an instantiation is compiled for: 8-bit types and the P = 8 min / max kernels
// take fewer (at 4 per CU they spill 44-152 B per lane; the P = 8 sum kernels spill 12 B at 4 and
// ran 14 % faster there than at 3).
template <typename T, int OP, int P>
constexpr int ar_occ()
{
    if constexpr (sizeof(T) == 1) return 2;
    else if constexpr (P == 8 && (OP == ISHMEMI_OP_MIN || OP == ISHMEMI_OP_MAX)) return 3;
    else return kArOcc;
}

template <typename T, int OP, bool VEC, int P>
__global__ __launch_bounds__(kBlock, (ar_occ<T, OP, P>())) __attribute__((flatten)) void allreduce_kernel(ReduceArgs a)
{
    using Item = std::conditional_t<VEC, Vec<T>, T>;
    constexpr uint64_t IB = sizeof(Item);
    const int tid = threadIdx.x;
    const int p = a.p, me = a.me;
    const uint32_t G = gridDim.x, b = blockIdx.x;
    const uint64_t head_bytes = VEC ? a.head * sizeof(T) : 0;
    const uint64_t seg = a.seg_items;
    const bool one = a.oneshot != 0;
    trace_mark(a.trace, 0);
    const uint32_t ep = kernel_epoch(a);
    trace_mark(a.trace, 6);

    // ---- reduce-scatter of chunk `me` (one-shot: the whole array) ----
    uint64_t cs = 0, ce = a.nitems;
    if (!one) chunk_of(a, me, cs, ce);
    const uint32_t nseg = nsegs(ce - cs, seg);
    uint32_t pending = 0, pclaim = 0;
    if (b < nseg) claim_issue(a, ep, b, pclaim);  // overlaps the start wait
    bool ok = launch_start(a, ep);
    trace_mark(a.trace, 1);

    // One work loop (so the segment body and the all-gather body are each instantiated once):
    //   RS_OWN - segment b, this workgroup's own (claimed, so a stealer can take it if this
    //            workgroup never becomes resident);
    //   RS_DYN - segments G.. grabbed from the head by whoever is free (they balance uneven
    //            workgroup speeds on large arrays; no claim: the head hands each out once);
    //   AG     - item b, then items G.. grabbed; a wait longer than kStealPatience first reduces
    //            an unclaimed owned segment of this PE (its owner is not resident), then resumes.
    enum { kRsOwn, kRsDyn, kAg } state = kRsOwn;
    const bool dyn_rs = nseg > G;
    if (dyn_rs) grab_issue(a, kEpRsHead, pending);
    const uint32_t per_peer = nsegs(min(a.items_per_chunk, a.nitems), seg);  // chunk 0 is the largest
    const uint32_t total = one ? 0 : (uint32_t) (p - 1) * per_peer;
    const bool dyn_ag = total > G;
    uint32_t item = b;          // current all-gather item (valid when have_item)
    bool have_item = false, ag_first = true, may_steal = true;
    uint64_t ag_wait = 0;  // trace only: ticks spent waiting for peers' segments
    while (ok) {
        uint32_t rs = 0xFFFFFFFFu;  // segment to reduce in this pass, if any
        if (state == kRsOwn) {
            state = kRsDyn;
            if (b < nseg && claim_take(pclaim, ep)) rs = b;
        } else if (state == kRsDyn) {
            if (dyn_rs) {
                const uint32_t s = G + grab_take(pending);
                if (s < nseg) {
                    grab_issue(a, kEpRsHead, pending);  // next grab in flight while this streams
                    rs = s;
                }
            }
            if (rs == 0xFFFFFFFFu) {
                state = kAg;
                trace_mark(a.trace, 2);
                if (dyn_ag) grab_issue(a, kEpAgHead, pending);
            }
        } else {
            if (!have_item) {
                if (ag_first) {
                    ag_first = false;
                    item = b;
                } else {
                    if (!dyn_ag) break;
                    item = G + grab_take(pending);
                    if (item < total) grab_issue(a, kEpAgHead, pending);
                }
                if (item >= total) break;
                have_item = true;
            }
            const int j = (me + 1 + (int) (item % (uint32_t) (p - 1))) % p;
            const uint32_t s = item / (uint32_t) (p - 1);
            uint64_t js, je;
            chunk_of(a, j, js, je);
            if (s >= nsegs(je - js, seg)) {
                have_item = false;
                continue;
            }
            const uint64_t w0 = a.trace ? __builtin_amdgcn_s_memrealtime() : 0;
            const int st = block_wait_ex(a, ep, kPhaseMid, (int) s, j, may_steal ? kStealPatience : 0);
            if (a.trace) ag_wait += __builtin_amdgcn_s_memrealtime() - w0;
            if (st == 1) {
                ok = false;
                break;
            }
            if (st == 2) {
                // Waited long: reduce one of this PE's owned segments nobody has claimed, so
                // peers stuck on it progress; then wait for the same item again.
                const uint32_t nown = nseg < G ? nseg : G;
                const uint32_t t = steal_segment(a, ep, nown);
                if (t < nown) rs = t;
                else may_steal = false;
            } else {
                have_item = false;
                // The segment's tiles, two per step: 8 loads per lane in flight.
                const uint64_t ss = js + (uint64_t) s * seg, se = min(ss + seg, je);
                constexpr int U = kAgTiles * kUnroll;
                constexpr uint64_t SI = (uint64_t) U * kBlock;
                auto ag_load = [&](uint64_t t, Item (&x)[U]) {
                    const uint32_t lim = (uint32_t) min<uint64_t>(se - t, SI);
                    const __amdgpu_buffer_rsrc_t r = make_rsrc(uniform_ptr(a.dstp[j] + head_bytes + t * IB));
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t k = (uint32_t) u * kBlock + (uint32_t) tid;
                        if (k < lim) x[u] = cload<Item>(r, k * (uint32_t) IB);
                    }
                };
                auto ag_store = [&](uint64_t t, const Item (&x)[U]) {
                    const uint32_t lim = (uint32_t) min<uint64_t>(se - t, SI);
                    const __amdgpu_buffer_rsrc_t dr = make_rsrc(uniform_ptr(a.dst + head_bytes + t * IB));
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const uint32_t k = (uint32_t) u * kBlock + (uint32_t) tid;
                        if (k < lim) wt_store(dr, k * (uint32_t) IB, x[u]);
                    }
                };
                for (uint64_t t = ss; t < se; t += SI) {
                    Item x[U];
                    ag_load(t, x);
                    ag_store(t, x);
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
        if (rs != 0xFFFFFFFFu) rs_segment<T, OP, VEC, P>(a, ep, rs, nseg, cs, ce, head_bytes, one);
    }
    trace_mark(a.trace, 3);
    if (a.trace && tid == 0) a.trace[(size_t) b * 8 + 7] = ag_wait;
    launch_finish(a, ep);
    trace_mark(a.trace, 4);
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
        } else if constexpr (NS == 2 && VEC) {
            // Buffer loads based at the workgroup's first item (scalar base + 32-bit lane offset):
            // a + b 0.471-0.472 ms against 0.484-0.485 ms with global nt loads, 1 GiB, interleaved
            // A B x3 (profiles/r04/fanin_loads/); the copy (NS = 1) keeps global loads, which were
            // 0.7 % faster there.
            // Source 1's load is issued once source 0's has landed: a + b 0.473 ms against 0.486 ms
            // with both in flight (one process, interleaved, tools/realign_variants.hip "serial",
            // profiles/r05/fanin/) — fewer interleaved request streams per wave; the realigned
            // kernel showed the same (its LDS stores order the sources).
            const uint64_t wo = off - (uint64_t) threadIdx.x * IB;
            const uint32_t lo = (uint32_t) (threadIdx.x * IB);
            const Item x0 = bload<Item>(make_rsrc(uniform_ptr(a.src[0] + wo)), lo);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const Item x1 = bload<Item>(make_rsrc(uniform_ptr(a.src[1] + wo)), lo);
            acc = op1<T, OP>(x0, x1);
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
// Realigned fan-in: 1 or 2 sources whose addresses differ from dst's mod 16, every operand
// element-aligned (runtime.cpp plan_fanin).  The element-granular path moved such operands one
// element per lane — a 1-PE reduce (a byte copy) at 0.6 TB/s, a + b at 3.4 TB/s on 256 MiB
// (tools/misaligned_probe.py).  Here dst is peeled to the 16-B grid (head elements, workgroup 0)
// and every lane loads the ALIGNED 16-B vector of each source at its item, takes its neighbour
// lane's vector with a cross-lane shuffle (lane 63 loads the next vector itself), and funnel-shifts
// the pair by the source's byte shift (uniform: v_alignbyte on word pairs picked by a scalar
// switch) — full-width loads and stores, HBM traffic of the aligned kernel.  The aligned loads
// reach at most up to the source's end rounded up to 16 B (the same 16-B block, so the same page);
// the descriptor's bound there returns zeros for lanes past the body.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_n(const char *uniform_base, uint64_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(uniform_base), (short) 0,
                                             (int) (bytes < 0x7FFFFFFFull ? bytes : 0x7FFFFFFFull), 0x00020000);
}

// Bytes k .. k + 15 of the 32-byte concatenation A | B (k uniform, 0 <= k < 16).
__device__ __forceinline__ u32x4 funnel16(const u32x4 &A, const u32x4 &B, uint32_t k)
{
    const uint32_t r = k & 3;
    auto al = [r](uint32_t hi, uint32_t lo) { return __builtin_amdgcn_alignbyte(hi, lo, r); };
    switch (k >> 2) {
        case 0: return u32x4{al(A.y, A.x), al(A.z, A.y), al(A.w, A.z), al(B.x, A.w)};
        case 1: return u32x4{al(A.z, A.y), al(A.w, A.z), al(B.x, A.w), al(B.y, B.x)};
        case 2: return u32x4{al(A.w, A.z), al(B.x, A.w), al(B.y, B.x), al(B.z, B.y)};
        default: return u32x4{al(B.x, A.w), al(B.y, B.x), al(B.z, B.y), al(B.w, B.z)};
    }
}

// The neighbour exchange of the realigned fan-in.  A source vector straddles two aligned 16-B
// vectors: lane i's own and lane i+1's.  Within a wave lane i+1's comes by a DPP wave shift
// (v_mov_b32_dpp wave_shl:1, four VALU ops, no LDS crossbar traffic); lane 63 takes lane 0 of the
// next wave through LDS, and the workgroup's last lane loads the vector past the workgroup's end.
// Round 4's one-wave workgroups did the same with four ds_bpermute shuffles and a boundary load
// per 1 KiB (0.72 / 0.70 of HBM for copy / a + b at 1 GiB); measured alternatives (tools/
// realign_variants.hip, 1 GiB, shifts 1 / 4 / 12 B, profiles/r05/realign/): shuffles 0.75 / 0.75,
// DPP alone 0.75 / 0.76, two aligned loads per lane 0.73 / 0.71, unaligned 16-B loads 0.79 / 0.76
// (0.80 / 0.82 with an XCD-grouped block order, but 0.77 at a 1-B shift), LDS exchange in 256 /
// 512-thread workgroups 0.83 / 0.82, DPP + LDS edges in 512-thread workgroups 0.835-0.838 /
// 0.822-0.827 (aligned kernel 0.84 / 0.83): the boundary load per 8 KiB instead of per 1 KiB, and
// no shuffle through LDS for 63 of 64 lanes.
__device__ __forceinline__ u32x4 wave_next(const u32x4 &A)
{
    return u32x4{(uint32_t) __builtin_amdgcn_update_dpp(0, (int) A.x, 0x130, 0xF, 0xF, false),
                 (uint32_t) __builtin_amdgcn_update_dpp(0, (int) A.y, 0x130, 0xF, 0xF, false),
                 (uint32_t) __builtin_amdgcn_update_dpp(0, (int) A.z, 0x130, 0xF, 0xF, false),
                 (uint32_t) __builtin_amdgcn_update_dpp(0, (int) A.w, 0x130, 0xF, 0xF, false)};
}

// A realigned load in two steps around a workgroup barrier:
//   realign_issue  - every thread: the aligned vector A of `src` under this lane for the workgroup
//                    whose dest starts `wo` bytes past element 0 (src + wo sits `shift` bytes past
//                    the 16-B grid), its in-wave neighbour B by DPP, each wave's first vector into
//                    edge[wave] and, from the workgroup's last lane, the vector past the
//                    workgroup's end into edge[kRealignWaves].  Loads reach at most the source's
//                    end rounded up to 16 B (the same 16-B block, so the same page); the
//                    descriptor returns zeros past it;
//   realign_finish - lane 63 takes the next wave's first vector, then the 16 bytes this lane's
//                    dest item takes from the source.
// Sources are issued one after the other, each source's LDS stores waiting for its loads: with
// two sources that order ran a + b at 0.489-0.490 ms per GiB against 0.511-0.513 ms with both
// sources' loads issued before any wait (tools/realign_variants.hip var24 / var8, interleaved,
// profiles/r05/realign/).
template <int AUX, int BS = kRealignBlock>
__device__ __forceinline__ void realign_issue(const char *src, uint32_t shift, uint64_t total, uint64_t wo,
                                              u32x4 *edge, u32x4 &A, u32x4 &B)
{
    const uint32_t tid = threadIdx.x;
    const char *sb = uniform_ptr(src + (wo - shift));  // 16-B aligned in memory
    const uint64_t end_al = (((uint64_t) (uintptr_t) src + total + 15) & ~15ull) - (uint64_t) (uintptr_t) sb;
    const __amdgpu_buffer_rsrc_t r = make_rsrc_n(sb, end_al);
    A = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u, 0, AUX);
    if (tid == BS - 1) edge[BS / 64] = __builtin_amdgcn_raw_buffer_load_b128(r, BS * 16u, 0, AUX);
    if ((tid & 63) == 0) edge[tid >> 6] = A;
    B = wave_next(A);
}

__device__ __forceinline__ u32x4 realign_finish(const u32x4 *edge, const u32x4 &A, u32x4 B, uint32_t shift)
{
    if ((threadIdx.x & 63) == 63) B = edge[(threadIdx.x >> 6) + 1];
    return funnel16(A, B, shift);
}

// One 512-item block of the realigned fan-in (every thread; i0 workgroup-uniform).
template <typename T, int OP, int NS>
__device__ __forceinline__ void fanin_realign_block(const FaninArgs &a, u32x4 (*edge)[kRealignWaves + 1], uint64_t i0)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t wo = a.head * sizeof(T) + i0 * 16;  // bytes from element 0 to this block's first item
    u32x4 A[NS], B[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) realign_issue<kNonTemporal>(a.src[j], a.shift[j], a.total, wo, edge[j], A[j], B[j]);
    __syncthreads();
    Vec<T> acc = __builtin_bit_cast(Vec<T>, realign_finish(edge[0], A[0], B[0], a.shift[0]));
    if constexpr (NS == 2)
        acc = op1<T, OP>(acc, __builtin_bit_cast(Vec<T>, realign_finish(edge[1], A[1], B[1], a.shift[1])));
    if (i0 + tid < a.nitems) wt_store(make_rsrc(uniform_ptr(a.dst + wo)), tid * 16u, acc);
}

template <typename T, int OP, int NS>
__global__ __launch_bounds__(kRealignBlock) void fanin_realign_kernel(FaninArgs a)
{
    static_assert(NS == 1 || NS == 2, "realigned fan-in: 1 or 2 sources");
    __shared__ u32x4 edge[NS][kRealignWaves + 1];
    const uint32_t tid = threadIdx.x;
    const uint64_t stride = (uint64_t) gridDim.x * kRealignBlock;
    const uint64_t first = (uint64_t) blockIdx.x * kRealignBlock;
    if (stride >= a.nitems) {
        // One block per workgroup (up to 2^31 items = 32 GiB): the grid-stride loop's bookkeeping
        // cost 1.3 % on the copy (var8, tools/realign_variants.hip).
        if (first < a.nitems) fanin_realign_block<T, OP, NS>(a, edge, first);
    } else {
        for (uint64_t i0 = first; i0 < a.nitems; i0 += stride) {
            fanin_realign_block<T, OP, NS>(a, edge, i0);
            __syncthreads();  // edge[] is rewritten by the next pass
        }
    }
    if (blockIdx.x == 0) {  // head elements (before dst's kRealignPeel boundary) and tail elements
        const uint64_t tail_off = a.head + a.nitems * (16 / sizeof(T));
        for (int pass = 0; pass < 2; ++pass) {
            const uint64_t cnt = pass == 0 ? a.head : a.tail;
            for (uint64_t t = tid; t < cnt; t += kRealignBlock) {
                const uint64_t e = pass == 0 ? t : tail_off + t;
                T acc = ((const T *) a.src[0])[e];
                if constexpr (NS == 2) acc = op1<T, OP>(acc, ((const T *) a.src[1])[e]);
                ((T *) a.dst)[e] = acc;
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Phased reduce-scatter + all-gather for large payloads (runtime.cpp reduce_heap, p > 1, 16-B
// vector body, payload >= ISHMEM_PHASED_MIN_BYTES):
//   team_sync_kernel - every member's source is final;
//   rs_phase_kernel  - dst[chunk me] = fold_j src_j[chunk me] in canonical team order: ONE 16-B
//                      item per thread, one-wave workgroups, a one-shot grid — the fan-in kernel's
//                      shape (83 % of HBM on the same 2-read-1-write traffic) instead of the
//                      persistent kernel's segment loop (4.7 TB/s in its reduce-scatter phase,
//                      DESIGN.md §3); peers' items by system-coherent loads, the load order rotated
//                      per workgroup so concurrently running workgroups pull from every member;
//   team_sync_kernel - every member's chunk is stored (kernel boundary: the write-through stores
//                      have completed) and every member has finished reading the sources;
//   ag_phase_kernel  - dst[chunk j] = dst_j[chunk j] for every j != me;
//   team_sync_kernel - every member has finished reading this member's dest.
// Neither grid ever waits, so any residency works and co-located PEs cannot crowd each other
// out; the only waiters are the three one-workgroup barriers.  In place is safe: member j reads
// chunk j of my source only in its reduce-scatter, and my all-gather (the only writer of chunk j
// here) starts after the middle barrier.  The price is two more launches and two more barrier
// round trips than the persistent kernel (~10 us), so it is used for large payloads only.
// ---------------------------------------------------------------------------------------------
template <typename T, int OP, int P, bool NT, int R>
__device__ __forceinline__ void rs_phase_item(const PhaseArgs &a, uint64_t wb, bool valid)
{
    using Item = Vec<T>;
    const uint32_t off = threadIdx.x * 16u;
    Item x[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int j = (R + k) % P;
        if (!valid) continue;
        // Own chunk (and every chunk in the peer-nt mode): nontemporal buffer loads; global nt
        // loads measured the same here (2 / 4 PEs x 1 GiB, profiles/r04/rs_loads/).
        if (NT || j == a.me) x[k] = bload<Item>(make_rsrc(uniform_ptr(a.src[j] + wb)), off);
        else x[k] = cload<Item>(make_rsrc(uniform_ptr(a.src[j] + wb)), off);
    }
    Item acc = x[(P - R) % P];  // member 0
#pragma unroll
    for (int j = 1; j < P; ++j) acc = op1<T, OP>(acc, x[(j - R + P) % P]);
    if (valid) wt_store(make_rsrc(uniform_ptr(a.dst + wb)), off, acc);
}

template <typename T, int OP, int P, bool NT, int R = 0>
__device__ __forceinline__ void rs_phase_dispatch(const PhaseArgs &a, int rot, uint64_t wb, bool valid)
{
    if constexpr (R == P - 1) {
        rs_phase_item<T, OP, P, NT, R>(a, wb, valid);
    } else {
        if (rot == R) rs_phase_item<T, OP, P, NT, R>(a, wb, valid);
        else rs_phase_dispatch<T, OP, P, NT, R + 1>(a, rot, wb, valid);
    }
}

// P = 0: any team size, loaded and folded in team order.
template <typename T, int OP>
__device__ __forceinline__ void rs_phase_item_any(const PhaseArgs &a, uint64_t wb, bool valid)
{
    using Item = Vec<T>;
    if (!valid) return;
    const uint32_t off = threadIdx.x * 16u;
    Item acc;
    for (int j = 0; j < a.p; ++j) {
        Item x;
        if (j == a.me || a.peer_nt) x = nt_load((const Item *) (a.src[j] + wb + off));
        else x = cload<Item>(make_rsrc(uniform_ptr(a.src[j] + wb)), off);
        acc = j == 0 ? x : op1<T, OP>(acc, x);
    }
    wt_store(make_rsrc(uniform_ptr(a.dst + wb)), off, acc);
}

// Unaligned head (member 0's) and tail (member p-1's), element-wise, by workgroup 0 of the
// reduce-scatter grid; descriptors based at the region (offsets < 16 B).
template <typename T, int OP>
__device__ __forceinline__ void rs_phase_edges(const PhaseArgs &a)
{
    const int p = a.p, me = a.me;
    if (blockIdx.x == 0) {
        const int tid = threadIdx.x;
        const uint64_t tail_off = a.head + a.nitems * (16 / sizeof(T));
        for (int region = 0; region < 2; ++region) {
            const bool owner = a.whole || (region == 0 ? me == 0 : me == p - 1);
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
}

// XCD-grouped block order (round 6): the hardware hands workgroup b to XCD b mod 8, so in a
// one-shot grid neighbouring 1 KiB blocks land on different XCDs, whose L2s are separate.  Within
// each full group of 64 workgroups, XCD x takes logical blocks 8x .. 8x + 7 instead: neighbouring
// blocks share an L2.  For sources read with unaligned 16-B loads (the shifted reduce-scatter) the
// line at each block boundary is then fetched once, not by two XCDs: 1 GiB a + b from sources 4 /
// 12 B off dest's phase, one-wave workgroups, 0.537 / 0.536 ms in block order against 0.484 /
// 0.483 ms grouped (0.75 -> 0.83 of HBM; tools/realign_variants.hip "unal 64 xcd",
// profiles/r06/realign/).  A permutation of [0, grid): the tail past the last full group keeps
// its index.
__device__ __forceinline__ uint64_t xcd_grouped_block(uint64_t b, uint64_t grid)
{
    if (b >= (grid & ~63ull)) return b;
    return (b & ~63ull) | ((b & 7) << 3) | ((b >> 3) & 7);
}

template <typename T, int OP, int P>
__global__ __launch_bounds__(kFaninBlock) void rs_phase_kernel(PhaseArgs a)
{
    const int me = a.me;
    const uint64_t cs = a.whole ? 0 : min((uint64_t) me * a.items_per_chunk, a.nitems);
    const uint64_t ce = a.whole ? a.nitems : min(cs + a.items_per_chunk, a.nitems);
    const uint64_t head_bytes = a.head * sizeof(T);
    const uint64_t stride = (uint64_t) gridDim.x * kFaninBlock;
    const uint64_t blk = a.shift && a.xcd_group ? xcd_grouped_block(blockIdx.x, gridDim.x) : blockIdx.x;
    auto body = [&](auto nt) {
        for (uint64_t i0 = cs + blk * kFaninBlock; i0 < ce; i0 += stride) {
            const bool valid = i0 + threadIdx.x < ce;
            const uint64_t wb = head_bytes + i0 * 16;
            if constexpr (P > 0) rs_phase_dispatch<T, OP, P, decltype(nt)::value>(a, (int) ((i0 / kFaninBlock) % P), wb, valid);
            else rs_phase_item_any<T, OP>(a, wb, valid);
        }
    };
    if (a.peer_nt) {
        body(std::true_type{});
    } else {
        body(std::false_type{});
    }
    rs_phase_edges<T, OP>(a);
}

// The phased reduce-scatter with every member's source on another 16-B phase than dest (the same
// shift on every PE: the offsets are symmetric): the realigned fan-in's loads (realign_issue /
// realign_finish, DPP + LDS edges) per member in kRsRealignBlock-thread workgroups (64: the block
// size A/B above), members taken four at a time and folded in team order.  Round 4 ran this with
// four shuffles per member per vector.  In place never gets here (source == dest has no shift), so
// the loads past the chunk's end read only bytes no member writes during the reduce-scatter.
// One BS-item block of the realigned reduce-scatter (every thread; i0 workgroup-uniform):
// members in groups of G, each member's loads issued after the previous member's LDS store has
// waited for its own, one barrier per group plus one between groups (edge[] reuse).  2 PEs x 1 GiB
// on one GPU, sources 4 B off dest's phase, reduce-scatter grid (`tools/sweep.py --phases`,
// interleaved, profiles/r05/realign_multi/): 64-thread workgroups 0.546-0.547 ms, 256 0.563-0.569,
// 512 0.559-0.594; all members' loads issued before any wait 0.609-0.617 (64) / 0.643-0.671 (512);
// round 4's shuffle version 0.571; aligned operands 0.487-0.493.
template <typename T, int OP, int BS, int G>
__device__ __forceinline__ void rs_realign_block(const PhaseArgs &a, u32x4 (*edge)[BS / 64 + 1], uint64_t i0, uint64_t ce)
{
    const int p = a.p, me = a.me;
    const uint32_t tid = threadIdx.x;
    const uint64_t wb = a.head * sizeof(T) + i0 * 16;
    Vec<T> acc;
    for (int g0 = 0; g0 < p; g0 += G) {
        if (g0) __syncthreads();  // the previous group's edge[] reads are done
        u32x4 A[G], B[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int j = g0 + k;
            if (j >= p) break;
            if (j == me || a.peer_nt) realign_issue<kNonTemporal, BS>(a.src[j], a.shift, a.total, wb, edge[k], A[k], B[k]);
            else realign_issue<kSysCoherent, BS>(a.src[j], a.shift, a.total, wb, edge[k], A[k], B[k]);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int j = g0 + k;
            if (j >= p) break;
            const Vec<T> x = __builtin_bit_cast(Vec<T>, realign_finish(edge[k], A[k], B[k], a.shift));
            acc = j == 0 ? x : op1<T, OP>(acc, x);
        }
    }
    if (i0 + tid < ce) wt_store(make_rsrc(uniform_ptr(a.dst + wb)), tid * 16u, acc);
}

template <typename T, int OP>
__global__ __launch_bounds__(kRsRealignBlock) void rs_phase_realign_kernel(PhaseArgs a)
{
    constexpr int BS = kRsRealignBlock, G = 4;
    __shared__ u32x4 edge[G][BS / 64 + 1];
    const uint64_t cs = a.whole ? 0 : min((uint64_t) a.me * a.items_per_chunk, a.nitems);
    const uint64_t ce = a.whole ? a.nitems : min(cs + a.items_per_chunk, a.nitems);
    const uint64_t stride = (uint64_t) gridDim.x * BS;
    const uint64_t first = cs + (uint64_t) blockIdx.x * BS;
    if (cs + stride >= ce) {
        if (first < ce) rs_realign_block<T, OP, BS, G>(a, edge, first, ce);
    } else {
        for (uint64_t i0 = first; i0 < ce; i0 += stride) {
            rs_realign_block<T, OP, BS, G>(a, edge, i0, ce);
            __syncthreads();  // edge[] is rewritten by the next pass
        }
    }
    rs_phase_edges<T, OP>(a);
}

// Every item outside chunk `me`, pulled from its owner's dest.  Workgroup w takes peer
// k = w mod (p-1) (member (me + 1 + k) mod p) and that member's 64-item block w / (p-1):
// consecutive workgroups — the ones resident together in a one-shot grid — pull from every peer
// at once, so every xGMI link is busy (in chunk order the resident window, a few MiB, would sit
// inside one peer's chunk and load one link at a time).  Chunk edges are multiples of 64 items.
__global__ __launch_bounds__(kFaninBlock) void ag_phase_kernel(PhaseArgs a)
{
    const int p = a.p, me = a.me;
    const uint64_t head_bytes = a.head * a.elem;
    const uint64_t peers = (uint64_t) (p - 1);
    const uint64_t blocks = (a.items_per_chunk + kFaninBlock - 1) / kFaninBlock;  // per chunk
    const uint64_t work = peers * blocks;
    const uint32_t off = threadIdx.x * 16u;
    for (uint64_t w = blockIdx.x; w < work; w += gridDim.x) {
        const int j = (me + 1 + (int) (w % peers)) % p;
        const uint64_t js = min((uint64_t) j * a.items_per_chunk, a.nitems);
        const uint64_t je = min(js + a.items_per_chunk, a.nitems);
        const uint64_t i0 = js + (w / peers) * kFaninBlock;
        if (i0 + threadIdx.x < je) {
            const uint64_t wb = head_bytes + i0 * 16;
            const u32x4 x = a.peer_nt ? nt_load((const u32x4 *) (a.dstp[j] + wb + off))
                                      : cload<u32x4>(make_rsrc(uniform_ptr(a.dstp[j] + wb)), off);
            wt_store(make_rsrc(uniform_ptr(a.dst + wb)), off, x);
        }
    }
    if (blockIdx.x == 0) {
        // Head bytes from member 0, tail bytes from member p-1 (byte copies, < 16 each).
        const uint32_t tid = threadIdx.x;
        const uint64_t tail_b = (uint64_t) a.tail * a.elem;
        const uint64_t tail_base = head_bytes + a.nitems * 16;
        if (me != 0 && tid < head_bytes)
            a.dst[tid] = (char) cload<uint8_t>(make_rsrc(uniform_ptr(a.dstp[0])), tid);
        if (me != p - 1 && tid < tail_b)
            a.dst[tail_base + tid] = (char) cload<uint8_t>(make_rsrc(uniform_ptr(a.dstp[p - 1] + tail_base)), tid);
    }
}

template <typename K>
int phase_grid(K, uint64_t items)
{
    const uint64_t g = (items + kFaninBlock - 1) / kFaninBlock;
    return (int) std::max<uint64_t>(1, std::min<uint64_t>(g, (uint64_t) kFaninMaxGrid));
}

template <typename T, int OP>
hipError_t rs_phase_t(const PhaseArgs &a, hipStream_t s)
{
    const uint64_t cs = a.whole ? 0 : std::min((uint64_t) a.me * a.items_per_chunk, a.nitems);
    const uint64_t len = a.whole ? a.nitems : std::min(cs + a.items_per_chunk, a.nitems) - cs;
    auto go = [&](auto kernel) {
        hipLaunchKernelGGL(kernel, dim3(phase_grid(kernel, len)), dim3(kFaninBlock), 0, s, a);
    };
    if (a.shift && !phase_unaligned()) {
        uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((len + kRsRealignBlock - 1) / kRsRealignBlock,
                                                              (1ull << 31) / kRsRealignBlock));
        if (realign_grid_cap() > 0) g = std::min<uint64_t>(g, (uint64_t) realign_grid_cap());
        hipLaunchKernelGGL((rs_phase_realign_kernel<T, OP>), dim3((unsigned) g), dim3(kRsRealignBlock), 0, s, a);
    } else if (a.p == 2) go(rs_phase_kernel<T, OP, 2>);
    else if (a.p == 4) go(rs_phase_kernel<T, OP, 4>);
    else if (a.p == 8) go(rs_phase_kernel<T, OP, 8>);
    else go(rs_phase_kernel<T, OP, 0>);
    return hipGetLastError();
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

// The grid is capped by the waiting footprint (resident_blocks_of), so a thread may own several
// items (t, t + G*kBlock, ...): it pushes all of them before polling for any.
// Item `off` (8 payload bytes, or the `valid` < 8 of the ragged last item) of the source.  Items
// sit at multiples of 8 bytes from element 0, so elements never straddle them whatever the
// array's address; the address only picks the load width (round 5: 4-B aligned arrays — a float
// array 4 B off an 8-B boundary — took the persistent kernel before, 8.5 vs 4.5 us at 64 KiB).
__device__ __forceinline__ uint64_t ll_load(const LLArgs &a, uint64_t off, uint64_t valid)
{
    const char *p = a.src + off;
    if (valid == 8) {
        if (((uintptr_t) p & 7) == 0) return *(const uint64_t *) p;
        if (((uintptr_t) p & 3) == 0)
            return (uint64_t) ((const uint32_t *) p)[0] | ((uint64_t) ((const uint32_t *) p)[1] << 32);
    }
    // Ragged last item or a byte-aligned array: byte assembly (a variable-length memcpy would go
    // through scratch).
    uint64_t mine = 0;
    for (uint32_t k = 0; k < (uint32_t) valid; ++k) mine |= (uint64_t) (uint8_t) p[k] << (8 * k);
    return mine;
}

__device__ __forceinline__ void ll_store(char *p, uint64_t valid, uint64_t v)
{
    if (valid == 8 && ((uintptr_t) p & 7) == 0) {
        *(uint64_t *) p = v;
    } else if (valid == 8 && ((uintptr_t) p & 3) == 0) {
        ((uint32_t *) p)[0] = (uint32_t) v;
        ((uint32_t *) p)[1] = (uint32_t) (v >> 32);
    } else {
        for (uint32_t k = 0; k < (uint32_t) valid; ++k) p[k] = (char) (v >> (8 * k));
    }
}

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void ll_kernel(LLArgs a)
{
    const uint64_t first = (uint64_t) blockIdx.x * kBlock + threadIdx.x;
    const uint64_t stride = (uint64_t) gridDim.x * kBlock;
    const uint64_t nitems = (a.nbytes + 7) / 8;
    const int p = a.p, me = a.me;
    const uint32_t ep = kernel_epoch(a);
    const uint64_t par = ep & 1u;
    const uint64_t tag = (uint64_t) ep << 32;
    const uint64_t sg = ll_sender_granules(p);  // granules per (parity, sender) slot
    const bool bcast = a.mode == kLLBroadcast;
    const bool has_src = !bcast || me == a.root;  // a broadcast's non-roots read no source
    bool ok = true;
    for (uint64_t item = first; item < nitems; item += stride) {
        if (!has_src && item != 0) break;  // non-root: the item-0 token only
        const uint64_t off = item * 8;
        const uint64_t mine = has_src ? ll_load(a, off, a.nbytes - off < 8 ? a.nbytes - off : 8) : 0;
        const uint64_t g0 = tag | (uint32_t) mine, g1 = tag | (uint32_t) (mine >> 32);
        for (int j = 0; j < p; ++j) {
            if (j == me) continue;
            uint64_t *slot = a.peer_ring[j] + (par * (uint64_t) p + me) * sg;
            __hip_atomic_store(slot + ll_granule(item, 0), g0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(slot + ll_granule(item, 1), g1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // Members folded: all (reduce), 0..me (inclusive scan), 0..me-1 (exclusive scan).
    const int last = a.mode == kLLInscan ? me : a.mode == kLLExscan ? me - 1 : p - 1;
    for (uint64_t item = first; item < nitems && ok; item += stride) {
        const uint64_t off = item * 8;
        const uint64_t valid = a.nbytes - off < 8 ? a.nbytes - off : 8;
        const uint64_t mine = has_src ? ll_load(a, off, valid) : 0;
        uint64_t acc = 0;  // an empty fold (member 0's exclusive scan) stores zeros
        for (int j = 0; j < p && ok; ++j) {
            // Broadcast: the root's items, plus every member's item-0 token.
            if (bcast && j != a.root && j != me && item != 0) continue;
            uint64_t x = mine;
            if (j != me) {
                const uint64_t *slot = a.my_ring + (par * (uint64_t) p + j) * sg;
                uint64_t h0, h1;
                for (;;) {
                    h0 = __hip_atomic_load(slot + ll_granule(item, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    h1 = __hip_atomic_load(slot + ll_granule(item, 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
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
            if (a.mode == kLLCollect) ll_store(a.dst + (uint64_t) j * a.nbytes + off, valid, x);
            else if (bcast) { if (j == a.root) ll_store(a.dst + off, valid, x); }
            else if (j <= last) acc = (j == 0) ? x : fold8<T, OP>(acc, x);
        }
        if (ok && a.mode != kLLCollect && !bcast) ll_store(a.dst + off, valid, acc);
    }
    // *ret was zeroed by the caller: any thread that failed marks it (sticky over launches).
    if (!ok && a.ret) __hip_atomic_fetch_or(a.ret, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    kernel_epoch_done(a, ep);
}

inline int resident_blocks_of(const void *kernel);

template <typename T, int OP>
hipError_t ll_t(const LLArgs &a, hipStream_t s)
{
    const uint64_t nitems = (a.nbytes + 7) / 8;
    const uint64_t want = std::max<uint64_t>(1, (nitems + kBlock - 1) / kBlock);
    const int grid = (int) std::min<uint64_t>(want, (uint64_t) resident_blocks_of((const void *) ll_kernel<T, OP>));
    hipLaunchKernelGGL((ll_kernel<T, OP>), dim3(grid), dim3(kBlock), 0, s, a);
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

// Grid cap of a kernel whose workgroups wait for peers (kernels.h, "Waiting footprint"): the
// workgroups of `kernel` resident at once on this device (occupancy API, cached per kernel
// address; it can over-report by one block per CU for SGPR-heavy kernels, MI355X_MICROARCH.md
// residency, which the division leaves far from mattering) divided by share x wait_slots.  The
// collectives are correct with any residency of their grid (owned work can be stolen, the rest is grabbed or
// strided; nothing is paired), so the cap only bounds how much of the device one waiting launch
// can hold.  Round 3 sized the persistent reduce to the whole device (1024 workgroups, each
// spinning at start): two collectives of different teams issued in opposite orders on two PEs
// then each held their own GPU while waiting for the other's kernel, which could not get a CU —
// the r03zh device timeouts (profiles/r03/phased_share/).
inline int resident_blocks_of(const void *kernel)
{
    static std::mutex mu;  // one instance per translation unit (inline, internal namespace)
    static std::map<const void *, int> cache;
    static int cus = 0;
    std::lock_guard<std::mutex> lk(mu);
    if (cus <= 0) {
        int dev = 0;
        (void) hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
            (void) hipGetLastError();
            cus = 1;
        }
    }
    int per = 0;
    auto it = cache.find(kernel);
    if (it != cache.end()) {
        per = it->second;
    } else {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, kBlock, 0) != hipSuccess) {
            (void) hipGetLastError();
            per = 1;
        }
        per = std::max(per, 1);
        cache[kernel] = per;
    }
    const long long slots = (long long) device_share() * wait_slots();
    return (int) std::max<long long>(1, (long long) per * std::max(cus, 1) / slots);
}

template <typename K>
int resident_blocks(K kernel)
{
    return resident_blocks_of((const void *) kernel);
}

template <typename K>
hipError_t launch_resident(K kernel, const ReduceArgs &a, int grid, hipStream_t s)
{
    // Balanced waves of grabs: the work list (the reduce-scatter segments of one chunk, or the
    // all-gather items when those fit the grid at once) is split into equal waves, so no wave
    // leaves most workgroups idle (1024 segments on a 768-workgroup cap would run one full wave
    // and one a third full: 512 workgroups x 2 instead).
    const uint64_t cap = (uint64_t) std::max(1, std::min(grid, resident_blocks(kernel)));
    const uint64_t len = a.oneshot ? a.nitems : std::min(a.items_per_chunk, a.nitems);
    const uint64_t nseg = std::max<uint64_t>(1, (len + a.seg_items - 1) / a.seg_items);
    const uint64_t ag = a.oneshot ? 0 : nseg * (uint64_t) (a.p - 1);
    const uint64_t work = ag > nseg && ag <= cap ? ag : nseg;
    const uint64_t waves = (work + cap - 1) / cap;
    grid = (int) std::max<uint64_t>(1, (work + waves - 1) / waves);
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
    if (a.realign) {
        if (realign_grid_cap() > 0) grid = std::min(grid, realign_grid_cap());
        if (a.nsrc == 1) hipLaunchKernelGGL((fanin_realign_kernel<T, OP, 1>), dim3(grid), dim3(kRealignBlock), 0, s, a);
        else if (a.nsrc == 2) hipLaunchKernelGGL((fanin_realign_kernel<T, OP, 2>), dim3(grid), dim3(kRealignBlock), 0, s, a);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
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
