// ishmem_amd — fcollect / collect and sum-scan kernels (the collectives
// next to the reduce, built on the same pull + pairwise-barrier machinery; kernels_impl.h).
//
// Reference semantics: fcollect / collect concatenate the members' sources in team order on
// every member (src/collectives/collect_impl.h, docs/source/collectives.rst:687-760);
// ishmem_sum_inscan / exscan compute the inclusive / exclusive prefix sum over the team in team
// order (src/collectives/scan_impl.h, proxied to MPI_Scan / MPI_Exscan,
// src/runtime/runtime_mpi.cpp:816-835).  The exclusive scan's first member receives 0 (MPI leaves
// it undefined).
#include "kernels_impl.h"

namespace ishmemi {
namespace {

// All-gather of the sources: workgroup b copies tiles t == b (mod G) of every member's source,
// member order rotated by workgroup (all links busy), local slot included.  Only remote LOADS;
// between launch_start and launch_finish nothing waits, so the static tile split is safe.
__device__ void collect_member_realign(const char *src, char *dst, uint64_t nb, bool local, uint32_t b, uint64_t G,
                                       u32x4 *edge);

// U = 0: members off the 16-B grid moved with realigned 16-B loads (collect_member_realign).
template <int U>
__global__ __launch_bounds__(kBlock) void collect_kernel(CollectArgs a)
{
    using Item = std::conditional_t<U == 16 || U == 0, Vec<uint32_t>, std::conditional_t<U == 4, uint32_t, uint8_t>>;
    const int tid = threadIdx.x, b = blockIdx.x;
    const uint64_t G = gridDim.x;
    const uint32_t ep = kernel_epoch(a);
    const bool ok = launch_start(a, ep);
    if constexpr (U == 0) {
        __shared__ u32x4 edge[kBlock / 64 + 1];
        if (ok)
            for (int k = 0; k < a.p; ++k) {
                const int j = (a.me + (b + k)) % a.p;
                collect_member_realign(a.src[j], a.dst + a.dst_off[j], a.nbytes[j], j == a.me, (uint32_t) b, G, edge);
            }
        launch_finish(a, ep);
        return;
    }
    if (ok) {
        for (int k = 0; k < a.p; ++k) {
            const int j = (a.me + (b + k)) % a.p;
            const uint64_t nitems = a.nbytes[j] / U;
            for (uint64_t t0 = (uint64_t) b * kTile; t0 < nitems; t0 += G * kTile) {
                Item x[kUnroll];
                const char *base = uniform_ptr(a.src[j] + t0 * U);
                if (j == a.me) {
#pragma unroll
                    for (int u = 0; u < kUnroll; ++u) {
                        const uint64_t e = (uint64_t) u * kBlock + tid;
                        if (t0 + e < nitems) x[u] = ((const Item *) base)[e];
                    }
                } else {
                    const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
#pragma unroll
                    for (int u = 0; u < kUnroll; ++u) {
                        const uint64_t e = (uint64_t) u * kBlock + tid;
                        if (t0 + e < nitems) x[u] = cload<Item>(r, (uint32_t) (e * U));
                    }
                }
                Item *dp = (Item *) (a.dst + a.dst_off[j] + t0 * U);
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const uint64_t e = (uint64_t) u * kBlock + tid;
                    if (t0 + e < nitems) dp[e] = x[u];
                }
            }
        }
    }
    // No member returns while a peer may still read its source.
    launch_finish(a, ep);
}

// Phased fcollect / collect (runtime.cpp collect_launch, total bytes >= ISHMEM_PHASED_MIN_BYTES):
// team_sync_kernel, this one-shot grid, team_sync_kernel — the reduce's phased shape
// (kernels_impl.h).  One 1 KiB block of one member per one-wave workgroup, 16 / U items per
// thread (item k * 64 + lane: every load instruction is one contiguous 64 * U bytes); workgroup w
// takes member (me + 1 + w mod p) mod p and that member's block w / p, so the resident window
// pulls from every member (every link) at once.  Never waits: any residency works.
template <int U>
__global__ __launch_bounds__(kFaninBlock) void collect_phase_kernel(CollectArgs a, uint64_t blocks)
{
    using Item = std::conditional_t<U == 16, Vec<uint32_t>, std::conditional_t<U == 4, uint32_t, uint8_t>>;
    constexpr int K = 16 / U;
    constexpr uint64_t kBlockItems = (uint64_t) kFaninBlock * K;  // 1 KiB
    const int p = a.p;
    const uint32_t lane = threadIdx.x;
    for (uint64_t w = blockIdx.x; w < (uint64_t) p * blocks; w += gridDim.x) {
        const int j = (a.me + 1 + (int) (w % (uint64_t) p)) % p;
        const uint64_t nitems = a.nbytes[j] / U;
        const uint64_t i0 = (w / (uint64_t) p) * kBlockItems;
        if (i0 >= nitems) continue;
        const uint32_t lim = (uint32_t) min<uint64_t>(nitems - i0, kBlockItems);
        const char *base = uniform_ptr(a.src[j] + i0 * U);
        Item x[K];
        if (j == a.me) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t e = (uint32_t) k * kFaninBlock + lane;
                if (e < lim) x[k] = nt_load((const Item *) base + e);
            }
        } else {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint32_t e = (uint32_t) k * kFaninBlock + lane;
                if (e < lim) x[k] = cload<Item>(r, e * (uint32_t) U);
            }
        }
        const __amdgpu_buffer_rsrc_t dr = make_rsrc(uniform_ptr(a.dst + a.dst_off[j] + i0 * U));
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t e = (uint32_t) k * kFaninBlock + lane;
            if (e < lim) wt_store(dr, e * (uint32_t) U, x[k]);
        }
    }
}

// The phased fcollect / collect when some source, dest offset or count is not 16-B aligned
// (round 5): instead of narrowing every member's copy to 4- or 1-byte items (2 PEs x 64 MiB on one
// GPU: 86 us aligned, 179 us with 4-byte items, 345 us with 1-byte items, tools/collect_probe.py),
// member j's dest is peeled to the 16-B grid byte-wise (head, and the tail after the last whole
// vector) and its body is moved in 16-B items with the realigned loads of the fan-in
// (kernels_impl.h realign_issue / realign_finish: aligned source vectors, the in-wave neighbour by
// DPP, the vector past the wave's end loaded by lane 63, a funnel shift by the member's own byte
// shift).  Same block map as collect_phase_kernel: workgroup w, member (me + 1 + w mod p) mod p,
// its 1 KiB block w / p; the member's block 0 also moves the head / tail bytes.
__global__ __launch_bounds__(kFaninBlock) void collect_phase_realign_kernel(CollectArgs a, uint64_t blocks)
{
    __shared__ u32x4 edge[2];
    const int p = a.p;
    const uint32_t lane = threadIdx.x;
    for (uint64_t w = blockIdx.x; w < (uint64_t) p * blocks; w += gridDim.x) {
        const int j = (a.me + 1 + (int) (w % (uint64_t) p)) % p;
        const uint64_t nb = a.nbytes[j];
        char *dj = a.dst + a.dst_off[j];
        const uint64_t h = std::min<uint64_t>(nb, (16 - (uint64_t) (uintptr_t) dj % 16) % 16);
        const uint64_t nitems = (nb - h) / 16;
        const uint64_t tail = nb - h - nitems * 16;
        const uint64_t blk = w / (uint64_t) p;
        const uint64_t i0 = blk * kFaninBlock;
        const bool local = j == a.me;
        if (i0 < nitems) {  // workgroup-uniform
            const uint64_t wo = h + i0 * 16;
            const uint32_t shift = (uint32_t) (((uint64_t) (uintptr_t) a.src[j] + wo) % 16);
            u32x4 A, B;
            if (local) realign_issue<kNonTemporal, kFaninBlock>(a.src[j], shift, nb, wo, edge, A, B);
            else realign_issue<kSysCoherent, kFaninBlock>(a.src[j], shift, nb, wo, edge, A, B);
            __syncthreads();
            const u32x4 x = realign_finish(edge, A, B, shift);
            if (i0 + lane < nitems) wt_store(make_rsrc(uniform_ptr(dj + wo)), lane * 16u, x);
            __syncthreads();  // edge[] is rewritten by this workgroup's next block
        }
        if (blk == 0 && (h || tail)) {
            const uint64_t tb = h + nitems * 16;
            if (lane < h) dj[lane] = (char) (local ? a.src[j][lane] : cload<uint8_t>(make_rsrc(uniform_ptr(a.src[j])), lane));
            if (lane < tail)
                dj[tb + lane] = (char) (local ? a.src[j][tb + lane]
                                              : cload<uint8_t>(make_rsrc(uniform_ptr(a.src[j] + tb)), lane));
        }
    }
}

// Member j's `nbytes` at `src` -> dst (local), U-byte items, tiles b, b + G, ... of workgroup b.
template <int U>
__device__ __forceinline__ void collect_member(const char *src, char *dst, uint64_t nbytes, bool local,
                                               uint32_t b, uint64_t G)
{
    using Item = std::conditional_t<U == 16, Vec<uint32_t>, std::conditional_t<U == 4, uint32_t, uint8_t>>;
    const int tid = threadIdx.x;
    const uint64_t nitems = nbytes / U;
    for (uint64_t t0 = (uint64_t) b * kTile; t0 < nitems; t0 += G * kTile) {
        Item x[kUnroll];
        const char *base = uniform_ptr(src + t0 * U);
        if (local) {
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint64_t e = (uint64_t) u * kBlock + tid;
                if (t0 + e < nitems) x[u] = ((const Item *) base)[e];
            }
        } else {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                const uint64_t e = (uint64_t) u * kBlock + tid;
                if (t0 + e < nitems) x[u] = cload<Item>(r, (uint32_t) (e * U));
            }
        }
        Item *dp = (Item *) (dst + t0 * U);
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint64_t e = (uint64_t) u * kBlock + tid;
            if (t0 + e < nitems) dp[e] = x[u];
        }
    }
}

// Member j's `nb` bytes at `src` -> dst with dst off the 16-B grid relative to src (round 5):
// dst is peeled to the 16-B grid (head bytes, and the tail after the last whole vector, copied by
// workgroup 0), the body moves in 4 KiB blocks b, b + G, ... of 16-B items with the realigned
// loads (kernels_impl.h realign_issue / realign_finish, kBlock threads).  Every thread calls it.
__device__ void collect_member_realign(const char *src, char *dst, uint64_t nb, bool local, uint32_t b, uint64_t G,
                                       u32x4 *edge)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t h = min(nb, (16 - (uint64_t) (uintptr_t) dst % 16) % 16);
    const uint64_t nitems = (nb - h) / 16;
    const uint64_t tail = nb - h - nitems * 16;
    for (uint64_t blk = b; blk * kBlock < nitems; blk += G) {
        const uint64_t i0 = blk * kBlock, wo = h + i0 * 16;
        const uint32_t shift = (uint32_t) (((uint64_t) (uintptr_t) src + wo) % 16);
        u32x4 A, B;
        if (local) realign_issue<kNonTemporal, kBlock>(src, shift, nb, wo, edge, A, B);
        else realign_issue<kSysCoherent, kBlock>(src, shift, nb, wo, edge, A, B);
        __syncthreads();
        const u32x4 x = realign_finish(edge, A, B, shift);
        if (i0 + tid < nitems) *(u32x4 *) (dst + wo + tid * 16u) = x;
        __syncthreads();  // edge[] is rewritten by the next block
    }
    if (b == 0) {
        const uint64_t tb = h + nitems * 16;
        if (tid < h) dst[tid] = (char) (local ? src[tid] : cload<uint8_t>(make_rsrc(uniform_ptr(src)), tid));
        if (tid < tail)
            dst[tb + tid] = (char) (local ? src[tb + tid] : cload<uint8_t>(make_rsrc(uniform_ptr(src + tb)), tid));
    }
}

// Stream-ordered collect (ishmemx_<TN>_collect_on_queue, src/ishmemx.h): the counts are not
// known when the launch is enqueued.  Every workgroup first stores this member's count into its
// symmetric slot (system-scope, drained) — any workgroup may be the one that announces the
// launch — so a peer that has seen the announcement reads a final count.  After the start
// handshake each workgroup reads the p counts (one lane each), derives the team-order offsets
// and copies every member's bytes with the widest unit that divides that member's source
// address, destination offset and length.  The slot is not reused before every peer has
// finished reading it: the next launch starts after this one's "done reading" exchange.
__global__ __launch_bounds__(kBlock) void collect_dyn_kernel(CollectArgs a)
{
    __shared__ uint64_t s_cnt[kMaxPes];
    __shared__ u32x4 edge[kBlock / 64 + 1];  // a.unit == 0: realigned members (collect_member_realign)
    const uint32_t b = blockIdx.x;
    const uint64_t G = gridDim.x;
    const uint32_t ep = kernel_epoch(a);
    if (threadIdx.x == 0)
        __hip_atomic_store(a.my_count_slot, a.my_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    drain_block();
    const bool ok = launch_start(a, ep);
    if (ok) {
        if (threadIdx.x < (unsigned) a.p)
            s_cnt[threadIdx.x] = __hip_atomic_load(a.count_at[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        for (int k = 0; k < a.p; ++k) {
            const int j = (a.me + ((int) b + k)) % a.p;
            uint64_t off = 0;
            for (int i = 0; i < j; ++i) off += s_cnt[i];
            const uint64_t n = s_cnt[j];
            const uint64_t al = (uint64_t) a.src[j] | ((uint64_t) a.dst + off) | n;
            if ((al & 15) == 0) collect_member<16>(a.src[j], a.dst + off, n, j == a.me, b, G);
            else if (a.unit == 0) collect_member_realign(a.src[j], a.dst + off, n, j == a.me, b, G, edge);
            else if ((al & 3) == 0) collect_member<4>(a.src[j], a.dst + off, n, j == a.me, b, G);
            else collect_member<1>(a.src[j], a.dst + off, n, j == a.me, b, G);
        }
    }
    launch_finish(a, ep);
}

// Prefix sum.  Phase 1: member c owns chunk c; for each element it folds the members' values in
// team order and stores every member k's prefix into its own scratch row k (write-through).
// Phase 2 (once every member has published its chunk): each member pulls its row of every
// chunk into dest.
// Items are 16-B vectors when every base is 16-B aligned (chunk sizes are multiples of 64
// elements); the < 16 leftover elements of the last chunk go element by element.  For P in
// {2, 4, 8} the P loads of an item are all issued before the first store (compile-time register
// staging), so a tile costs one round trip instead of P.
template <typename T, typename I>
__device__ __forceinline__ I scan_add(const I &a, const I &b)
{
    return op1<T, ISHMEMI_OP_SUM>(a, b);
}

template <typename T, typename I, int P>
__device__ __forceinline__ void scan_item_fold(const ScanArgs &a, const char *const *base, char *const *row,
                                               uint32_t off, int p, int me, bool ok_item)
{
    if (!ok_item) return;
    I acc{};
    if constexpr (P > 0) {
        I x[P];
#pragma unroll
        for (int k = 0; k < P; ++k) x[k] = cload<I>(make_rsrc(base[k]), off);
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const I incl = k == 0 ? x[0] : scan_add<T, I>(acc, x[k]);  // first term kept (sign of 0)
            wt_store(make_rsrc(row[k]), off, a.inclusive ? incl : acc);
            acc = incl;
        }
    } else {
        for (int k = 0; k < p; ++k) {
            const I x = cload<I>(make_rsrc(base[k]), off);
            const I incl = k == 0 ? x : scan_add<T, I>(acc, x);
            wt_store(make_rsrc(row[k]), off, a.inclusive ? incl : acc);
            acc = incl;
        }
    }
    (void) me;
}

template <typename T, bool VEC, int P>
__global__ __launch_bounds__(kBlock) void scan_kernel(ScanArgs a)
{
    using I = std::conditional_t<VEC, Vec<T>, T>;
    constexpr uint64_t E = sizeof(I) / sizeof(T);
    constexpr int H = (P == 8 || P == 0) ? 2 : kUnroll;
    constexpr uint64_t kT = (uint64_t) kBlock * H;
    const int tid = threadIdx.x, b = blockIdx.x;
    const uint64_t G = gridDim.x;
    const int p = P > 0 ? P : a.p, me = a.me;
    const uint64_t ipc = a.items_per_chunk;
    const uint32_t ep = kernel_epoch(a);
    bool ok = launch_start(a, ep);
    {
        // Phase 1, grabbed piece by piece (tiles of kT items of chunk me; the last piece also
        // folds the < E leftover elements); the workgroup completing the last piece publishes
        // "chunk me ready" to every member, itself included.
        const uint64_t cs = min((uint64_t) me * ipc, a.nelems), ce = min(cs + ipc, a.nelems);
        const uint64_t nI = (ce - cs) / E;
        const uint64_t tail = (ce - cs) - nI * E;  // < E elements, last chunk only
        const uint32_t npieces = (uint32_t) max<uint64_t>(1, (nI + kT - 1) / kT);
        while (ok) {
            const uint32_t piece = block_grab(a, kEpRsHead);
            if (piece >= npieces) break;
            const uint64_t t0 = (uint64_t) piece * kT;
            if (t0 < nI) {
                const char *base[kMaxPes];
                char *row[kMaxPes];
                for (int k = 0; k < p; ++k) {
                    base[k] = uniform_ptr(a.src[k] + (cs + t0 * E) * sizeof(T));
                    row[k] = (char *) uniform_ptr(a.scratch[me] + ((uint64_t) k * ipc + t0 * E) * sizeof(T));
                }
#pragma unroll
                for (int u = 0; u < H; ++u) {
                    const uint64_t e = (uint64_t) u * kBlock + tid;
                    scan_item_fold<T, I, P>(a, base, row, (uint32_t) (e * sizeof(I)), p, me, t0 + e < nI);
                }
            }
            if (tail && piece == npieces - 1 && (uint64_t) tid < tail) {
                const uint64_t el = nI * E + tid;
                const char *base[kMaxPes];
                char *row[kMaxPes];
                for (int k = 0; k < p; ++k) {
                    base[k] = uniform_ptr(a.src[k] + (cs + nI * E) * sizeof(T));
                    row[k] = (char *) uniform_ptr(a.scratch[me] + ((uint64_t) k * ipc + nI * E) * sizeof(T));
                }
                scan_item_fold<T, T, 0>(a, base, row, (uint32_t) ((el - nI * E) * sizeof(T)), p, me, true);
            }
            drain_block();
            if (tid == kSignalLane && __hip_atomic_fetch_add(a.ep_ctr + kEpP1Done, 1u, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT) == npieces - 1) {
                release_system();
                push_flag(a, kPhaseMid, 0, ep, true);
            }
        }
    }
    // Phase 2 may start once every member's chunk is complete.  Every phase-1 piece was grabbed
    // before any workgroup gets here, by workgroups that wait for nothing else: no residency
    // coupling.
    ok = ok && block_wait(a, ep, kPhaseMid, 0, -2);
    if (ok) {
        for (int k = 0; k < p; ++k) {
            const int c = (me + b + k) % p;  // rotated over the members' scratch (links)
            const uint64_t cs = min((uint64_t) c * ipc, a.nelems), ce = min(cs + ipc, a.nelems);
            const uint64_t nI = (ce - cs) / E;
            const char *rowbase = a.scratch[c] + (uint64_t) me * ipc * sizeof(T);
            for (uint64_t t0 = (uint64_t) b * kT; t0 < nI; t0 += G * kT) {
                const __amdgpu_buffer_rsrc_t r = make_rsrc(uniform_ptr(rowbase + t0 * E * sizeof(T)));
                I x[H];
#pragma unroll
                for (int u = 0; u < H; ++u) {
                    const uint64_t e = (uint64_t) u * kBlock + tid;
                    if (t0 + e < nI) x[u] = cload<I>(r, (uint32_t) (e * sizeof(I)));
                }
                I *dp = (I *) (a.dst + (cs + t0 * E) * sizeof(T));
#pragma unroll
                for (int u = 0; u < H; ++u) {
                    const uint64_t e = (uint64_t) u * kBlock + tid;
                    if (t0 + e < nI) nt_store(dp + e, x[u]);
                }
            }
            const uint64_t tail = (ce - cs) - nI * E;
            if (tail && b == (int) ((nI / kT) % G) && (uint64_t) tid < tail) {
                const uint64_t el = nI * E + tid;
                const __amdgpu_buffer_rsrc_t r = make_rsrc(uniform_ptr(rowbase + nI * E * sizeof(T)));
                ((T *) (a.dst + cs * sizeof(T)))[el] = cload<T>(r, (uint32_t) (tid * sizeof(T)));
            }
        }
    }
    launch_finish(a, ep);
}

// Phased scan (runtime.cpp scan_impl, segments of >= ISHMEM_PHASED_MIN_BYTES): per segment
// team_sync_kernel, scan_p1_kernel, team_sync_kernel, scan_p2_kernel, team_sync_kernel — the
// reduce's phased shape (kernels_impl.h).  Phase 1: one item of chunk me per thread of a one-shot
// grid of one-wave workgroups, every member's prefix into this PE's scratch row k; phase 2:
// workgroup w pulls block w / p of its row of member c = (me + 1 + w mod p) mod p's scratch
// (every member, every link, at once).  Neither grid waits; the barriers order the phases, and the
// last one protects the scratch rows from the next segment.
template <typename T, bool VEC, int P>
__global__ __launch_bounds__(kFaninBlock) void scan_p1_kernel(ScanArgs a)
{
    using I = std::conditional_t<VEC, Vec<T>, T>;
    constexpr uint64_t E = sizeof(I) / sizeof(T);
    const int p = P > 0 ? P : a.p, me = a.me;
    const uint64_t ipc = a.items_per_chunk;
    const uint64_t cs = min((uint64_t) me * ipc, a.nelems), ce = min(cs + ipc, a.nelems);
    const uint64_t nI = (ce - cs) / E;
    const uint64_t tail = (ce - cs) - nI * E;  // < E elements, last chunk only
    const uint64_t stride = (uint64_t) gridDim.x * kFaninBlock;
    const uint32_t lane = threadIdx.x;
    for (uint64_t t0 = (uint64_t) blockIdx.x * kFaninBlock; t0 < nI; t0 += stride) {
        const char *base[kMaxPes];
        char *row[kMaxPes];
        for (int k = 0; k < p; ++k) {
            base[k] = uniform_ptr(a.src[k] + (cs + t0 * E) * sizeof(T));
            row[k] = (char *) uniform_ptr(a.scratch[me] + ((uint64_t) k * ipc + t0 * E) * sizeof(T));
        }
        scan_item_fold<T, I, P>(a, base, row, lane * (uint32_t) sizeof(I), p, me, t0 + lane < nI);
    }
    if (tail && blockIdx.x == 0 && lane < tail) {
        const char *base[kMaxPes];
        char *row[kMaxPes];
        for (int k = 0; k < p; ++k) {
            base[k] = uniform_ptr(a.src[k] + (cs + nI * E) * sizeof(T));
            row[k] = (char *) uniform_ptr(a.scratch[me] + ((uint64_t) k * ipc + nI * E) * sizeof(T));
        }
        scan_item_fold<T, T, 0>(a, base, row, lane * (uint32_t) sizeof(T), p, me, true);
    }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(kFaninBlock) void scan_p2_kernel(ScanArgs a, uint64_t blocks)
{
    using I = std::conditional_t<VEC, Vec<T>, T>;
    constexpr uint64_t E = sizeof(I) / sizeof(T);
    const int p = a.p, me = a.me;
    const uint64_t ipc = a.items_per_chunk;
    const uint32_t lane = threadIdx.x;
    for (uint64_t w = blockIdx.x; w < (uint64_t) p * blocks; w += gridDim.x) {
        const int c = (me + 1 + (int) (w % (uint64_t) p)) % p;
        const uint64_t cs = min((uint64_t) c * ipc, a.nelems), ce = min(cs + ipc, a.nelems);
        const uint64_t nI = (ce - cs) / E;
        const uint64_t t0 = (w / (uint64_t) p) * kFaninBlock;
        const char *rowbase = a.scratch[c] + (uint64_t) me * ipc * sizeof(T);
        if (t0 < nI) {
            if (t0 + lane < nI) {
                const I x = cload<I>(make_rsrc(uniform_ptr(rowbase + t0 * E * sizeof(T))), lane * (uint32_t) sizeof(I));
                wt_store(make_rsrc(uniform_ptr(a.dst + (cs + t0 * E) * sizeof(T))), lane * (uint32_t) sizeof(I), x);
            }
        } else if (t0 == ((nI + kFaninBlock - 1) / kFaninBlock) * kFaninBlock) {
            // The block just past the vector body: the chunk's < E leftover elements, if any.
            const uint64_t tail = (ce - cs) - nI * E;
            if (lane < tail)
                ((T *) (a.dst + (cs + nI * E) * sizeof(T)))[lane] =
                    cload<T>(make_rsrc(uniform_ptr(rowbase + nI * E * sizeof(T))), lane * (uint32_t) sizeof(T));
        }
    }
}

// Direct scan (runtime.cpp scan_impl: two members, disjoint dest and source, >= the phased
// threshold): between two team barriers, member me folds members 0..me (inclusive) or 0..me-1
// (exclusive; member 0 gets zeros) straight into its dest — no scratch rows, no second grid.
// Member me pulls me * B over the links, so for two members this equals the two-phase scan's
// ingress (B) with less HBM traffic; for more members the last one would pull (p-1) * B.
template <typename T, bool VEC>
__global__ __launch_bounds__(kFaninBlock) void scan_direct_kernel(ScanArgs a)
{
    using I = std::conditional_t<VEC, Vec<T>, T>;
    constexpr uint64_t E = sizeof(I) / sizeof(T);
    const int me = a.me;
    const int last = a.inclusive ? me : me - 1;  // fold members 0..last (none when last < 0)
    const uint64_t nI = a.nelems / E, tail = a.nelems - nI * E;
    const uint64_t stride = (uint64_t) gridDim.x * kFaninBlock;
    const uint32_t lane = threadIdx.x, off = lane * (uint32_t) sizeof(I);
    for (uint64_t t0 = (uint64_t) blockIdx.x * kFaninBlock; t0 < nI; t0 += stride) {
        if (t0 + lane >= nI) continue;
        const uint64_t wb = t0 * E * sizeof(T);
        I acc{};
        for (int j = 0; j <= last; ++j) {
            const I x = j == me ? *(const I *) (a.src[j] + wb + off) : cload<I>(make_rsrc(uniform_ptr(a.src[j] + wb)), off);
            acc = j == 0 ? x : scan_add<T, I>(acc, x);  // first term kept (sign of zero)
        }
        wt_store(make_rsrc(uniform_ptr(a.dst + wb)), off, acc);
    }
    if (blockIdx.x == 0 && lane < tail) {
        const uint64_t rb = nI * E * sizeof(T);
        const uint32_t eo = lane * (uint32_t) sizeof(T);
        T acc{};
        for (int j = 0; j <= last; ++j) {
            const T x = j == me ? ((const T *) (a.src[j] + rb))[lane] : cload<T>(make_rsrc(uniform_ptr(a.src[j] + rb)), eo);
            acc = j == 0 ? x : scan_add<T, T>(acc, x);
        }
        wt_store(make_rsrc(uniform_ptr(a.dst + rb)), eo, acc);
    }
}

template <typename T>
hipError_t scan_direct_t(const ScanArgs &a, bool vec, hipStream_t s)
{
    const uint64_t E = vec ? 16 / sizeof(T) : 1;
    const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((a.nelems / E + kFaninBlock - 1) / kFaninBlock,
                                                                (uint64_t) kFaninMaxGrid));
    if (vec) hipLaunchKernelGGL((scan_direct_kernel<T, true>), dim3((unsigned) g), dim3(kFaninBlock), 0, s, a);
    else hipLaunchKernelGGL((scan_direct_kernel<T, false>), dim3((unsigned) g), dim3(kFaninBlock), 0, s, a);
    return hipGetLastError();
}

// xGMI measurement hook (bench.py xgmi_probe): the same one-wave, one-item-per-thread shape as
// fanin_kernel, but every source load carries an explicit cache policy so the probe compares
// the collectives' system-coherent pulls (AUX = sc0 sc1) with nontemporal ones (AUX = nt) over
// the same links.  All nsrc loads are issued before the sum.
template <int AUX>
__global__ __launch_bounds__(kFaninBlock) void pull_probe_kernel(FaninArgs a)
{
    using Item = Vec<float>;
    const uint64_t first = (uint64_t) blockIdx.x * kFaninBlock;
    const uint32_t off = (uint32_t) (threadIdx.x * sizeof(Item));
    if (first + threadIdx.x >= a.nitems) return;
    Item x[kMaxFanin];
#pragma unroll
    for (int j = 0; j < kMaxFanin; ++j) {
        if (j < a.nsrc) {
            const __amdgpu_buffer_rsrc_t r = make_rsrc(uniform_ptr(a.src[j] + first * sizeof(Item)));
            x[j] = __builtin_bit_cast(Item, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
        }
    }
    Item acc = x[0];
#pragma unroll
    for (int j = 1; j < kMaxFanin; ++j)
        if (j < a.nsrc) acc = op1<float, ISHMEMI_OP_SUM>(acc, x[j]);
    wt_store(make_rsrc(uniform_ptr(a.dst + first * sizeof(Item))), off, acc);
}

// Test / measurement hook (ishmemi_c_occupy): a workgroup of 1024 work-items holding 80 KiB of
// LDS — two of them fill a CU's 160 KiB of LDS and 32 waves — that sleeps for `ticks` of
// s_memrealtime (100 MHz) and exits: lets a test hold most CUs while a collective runs.  Every
// wave leaves once the time is up (bounded).
constexpr int kOccupyThreads = 1024;
constexpr int kOccupyLdsWords = 80 * 1024 / 4;
__global__ __launch_bounds__(kOccupyThreads) void occupy_kernel(uint64_t ticks, uint32_t *sink)
{
    __shared__ uint32_t lds[kOccupyLdsWords];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int i = threadIdx.x; i < kOccupyLdsWords; i += kOccupyThreads) lds[i] = (uint32_t) i;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
    __syncthreads();
    if (sink && lds[(threadIdx.x * 17) % kOccupyLdsWords] == 0xFFFFFFFFu) *sink = 1;  // keeps LDS live
}

// Test hook (ishmemi_c_produce_u32): dst[i] = a[i] + b[i] over uint32 with ORDINARY loads and
// stores — what a user's producer kernel does — so its results may sit dirty in this device's L2
// when the next kernel on the stream (a collective) starts.  The coherence tripwire uses it
// instead of the library's write-through combine, so a peer reading stale HBM under dirty L2
// lines would show.
__global__ __launch_bounds__(256) void produce_u32_kernel(uint32_t *__restrict__ dst, const uint32_t *__restrict__ a,
                                                          const uint32_t *__restrict__ b, uint64_t n)
{
    for (uint64_t i = (uint64_t) blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t) gridDim.x * 256)
        dst[i] = a[i] + b[i];
}

template <typename K, typename A>
hipError_t launch_res(K kernel, const A &a, int grid, hipStream_t s)
{
    grid = std::min(grid, resident_blocks(kernel));
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_collect(const CollectArgs &a, int grid, hipStream_t s)
{
    if (a.unit == 16) return launch_res(collect_kernel<16>, a, grid, s);
    if (collect_realign()) return launch_res(collect_kernel<0>, a, grid, s);
    if (a.unit == 4) return launch_res(collect_kernel<4>, a, grid, s);
    return launch_res(collect_kernel<1>, a, grid, s);
}

hipError_t launch_collect_phase(const CollectArgs &a, hipStream_t s)
{
    uint64_t maxb = 0;
    for (int j = 0; j < a.p; ++j) maxb = std::max<uint64_t>(maxb, a.nbytes[j]);
    const uint64_t blocks = (maxb + 1023) / 1024;  // 1 KiB blocks of the largest member
    const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t) a.p * blocks, (uint64_t) kFaninMaxGrid));
    if (a.unit == 16) hipLaunchKernelGGL(collect_phase_kernel<16>, dim3((unsigned) g), dim3(kFaninBlock), 0, s, a, blocks);
    else if (collect_realign()) hipLaunchKernelGGL(collect_phase_realign_kernel, dim3((unsigned) g), dim3(kFaninBlock), 0, s, a, blocks);
    else if (a.unit == 4) hipLaunchKernelGGL(collect_phase_kernel<4>, dim3((unsigned) g), dim3(kFaninBlock), 0, s, a, blocks);
    else hipLaunchKernelGGL(collect_phase_kernel<1>, dim3((unsigned) g), dim3(kFaninBlock), 0, s, a, blocks);
    return hipGetLastError();
}

hipError_t launch_collect_dyn(const CollectArgs &a, int grid, hipStream_t s)
{
    CollectArgs b = a;
    b.unit = collect_realign() ? 0 : 1;  // members off the 16-B grid: realigned (0) or narrow items
    return launch_res(collect_dyn_kernel, b, grid, s);
}

hipError_t launch_occupy(int grid, uint64_t usec, hipStream_t s)
{
    if (grid < 1 || usec > 60ull * 1000 * 1000) return hipErrorInvalidValue;
    hipLaunchKernelGGL(occupy_kernel, dim3(grid), dim3(kOccupyThreads), 0, s, usec * 100ull, (uint32_t *) nullptr);
    return hipGetLastError();
}

hipError_t launch_produce_u32(uint32_t *dst, const uint32_t *a, const uint32_t *b, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    const uint64_t g = std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(produce_u32_kernel, dim3((unsigned) g), dim3(256), 0, s, dst, a, b, n);
    return hipGetLastError();
}

hipError_t launch_pull_probe(const FaninArgs &a, int policy, hipStream_t s)
{
    const uint64_t g = (a.nitems + kFaninBlock - 1) / kFaninBlock;
    if (a.nsrc < 1 || a.nsrc > kMaxFanin || g == 0 || g > (uint64_t) kFaninMaxGrid) return hipErrorInvalidValue;
    if (policy == 0)
        hipLaunchKernelGGL(pull_probe_kernel<2>, dim3((unsigned) g), dim3(kFaninBlock), 0, s, a);
    else
        hipLaunchKernelGGL(pull_probe_kernel<kSysCoherent>, dim3((unsigned) g), dim3(kFaninBlock), 0, s, a);
    return hipGetLastError();
}

template <typename T>
hipError_t scan_t(const ScanArgs &a, bool vec, int grid, hipStream_t s)
{
    if (!vec) {
        if (a.p == 2) return launch_res(scan_kernel<T, false, 2>, a, grid, s);
        if (a.p == 4) return launch_res(scan_kernel<T, false, 4>, a, grid, s);
        if (a.p == 8) return launch_res(scan_kernel<T, false, 8>, a, grid, s);
        return launch_res(scan_kernel<T, false, 0>, a, grid, s);
    }
    if (a.p == 2) return launch_res(scan_kernel<T, true, 2>, a, grid, s);
    if (a.p == 4) return launch_res(scan_kernel<T, true, 4>, a, grid, s);
    if (a.p == 8) return launch_res(scan_kernel<T, true, 8>, a, grid, s);
    return launch_res(scan_kernel<T, true, 0>, a, grid, s);
}

template <typename T>
hipError_t scan_phase_t(const ScanArgs &a, bool vec, int phase, hipStream_t s)
{
    const uint64_t E = vec ? 16 / sizeof(T) : 1;
    const uint64_t items = (a.items_per_chunk + E - 1) / E;
    if (phase == 1) {
        const uint64_t cs = std::min((uint64_t) a.me * a.items_per_chunk, a.nelems);
        const uint64_t len = std::min(cs + a.items_per_chunk, a.nelems) - cs;
        const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((len / E + kFaninBlock - 1) / kFaninBlock,
                                                                    (uint64_t) kFaninMaxGrid));
        auto go = [&](auto kernel) { hipLaunchKernelGGL(kernel, dim3((unsigned) g), dim3(kFaninBlock), 0, s, a); };
        if (vec) {
            if (a.p == 2) go(scan_p1_kernel<T, true, 2>);
            else if (a.p == 4) go(scan_p1_kernel<T, true, 4>);
            else if (a.p == 8) go(scan_p1_kernel<T, true, 8>);
            else go(scan_p1_kernel<T, true, 0>);
        } else {
            if (a.p == 2) go(scan_p1_kernel<T, false, 2>);
            else if (a.p == 4) go(scan_p1_kernel<T, false, 4>);
            else if (a.p == 8) go(scan_p1_kernel<T, false, 8>);
            else go(scan_p1_kernel<T, false, 0>);
        }
    } else {
        // Blocks per chunk, plus one for the last chunk's < E leftover elements.
        const uint64_t blocks = (items + kFaninBlock - 1) / kFaninBlock + 1;
        const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t) a.p * blocks, (uint64_t) kFaninMaxGrid));
        if (vec) hipLaunchKernelGGL((scan_p2_kernel<T, true>), dim3((unsigned) g), dim3(kFaninBlock), 0, s, a, blocks);
        else hipLaunchKernelGGL((scan_p2_kernel<T, false>), dim3((unsigned) g), dim3(kFaninBlock), 0, s, a, blocks);
    }
    return hipGetLastError();
}

hipError_t launch_scan_direct(int dt, const ScanArgs &a, bool vec, hipStream_t s)
{
    switch (dt) {
        case ISHMEMI_DT_INT8: case ISHMEMI_DT_UINT8: return scan_direct_t<uint8_t>(a, vec, s);
        case ISHMEMI_DT_INT16: case ISHMEMI_DT_UINT16: return scan_direct_t<uint16_t>(a, vec, s);
        case ISHMEMI_DT_INT32: case ISHMEMI_DT_UINT32: return scan_direct_t<uint32_t>(a, vec, s);
        case ISHMEMI_DT_INT64: case ISHMEMI_DT_UINT64: return scan_direct_t<uint64_t>(a, vec, s);
        case ISHMEMI_DT_FLOAT: return scan_direct_t<float>(a, vec, s);
        case ISHMEMI_DT_DOUBLE: return scan_direct_t<double>(a, vec, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_scan_phase(int dt, const ScanArgs &a, bool vec, int phase, hipStream_t s)
{
    switch (dt) {
        case ISHMEMI_DT_INT8: case ISHMEMI_DT_UINT8: return scan_phase_t<uint8_t>(a, vec, phase, s);
        case ISHMEMI_DT_INT16: case ISHMEMI_DT_UINT16: return scan_phase_t<uint16_t>(a, vec, phase, s);
        case ISHMEMI_DT_INT32: case ISHMEMI_DT_UINT32: return scan_phase_t<uint32_t>(a, vec, phase, s);
        case ISHMEMI_DT_INT64: case ISHMEMI_DT_UINT64: return scan_phase_t<uint64_t>(a, vec, phase, s);
        case ISHMEMI_DT_FLOAT: return scan_phase_t<float>(a, vec, phase, s);
        case ISHMEMI_DT_DOUBLE: return scan_phase_t<double>(a, vec, phase, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_scan(int dt, const ScanArgs &a, bool vec, int grid, hipStream_t s)
{
    switch (dt) {  // sum wraps on the unsigned type of the same width (two's complement)
        case ISHMEMI_DT_INT8: case ISHMEMI_DT_UINT8: return scan_t<uint8_t>(a, vec, grid, s);
        case ISHMEMI_DT_INT16: case ISHMEMI_DT_UINT16: return scan_t<uint16_t>(a, vec, grid, s);
        case ISHMEMI_DT_INT32: case ISHMEMI_DT_UINT32: return scan_t<uint32_t>(a, vec, grid, s);
        case ISHMEMI_DT_INT64: case ISHMEMI_DT_UINT64: return scan_t<uint64_t>(a, vec, grid, s);
        case ISHMEMI_DT_FLOAT: return scan_t<float>(a, vec, grid, s);
        case ISHMEMI_DT_DOUBLE: return scan_t<double>(a, vec, grid, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace ishmemi
