// Dev tool (round 5, not product): variants of the realigned fan-in (a source on another 16-B
// phase than dest) against the aligned copy, 1 GiB, interleaved rounds in one process, every
// variant's output checked against the host.  Which per-item mechanism brings the misaligned
// copy / a + b to the aligned kernel's rate (kernels_impl.h fanin_realign_kernel)?
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/realign_variants.hip -o tools/bin/realign_variants
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kernels_impl.h"  // the product's kernels, launched beside the variants (-Iishmem_amd/csrc -Iinclude)

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            printf("%s failed: %s\n", #x, hipGetErrorString(e_));                                  \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kNT = 2, kSC = 17;

__device__ __forceinline__ const char *uptr(const char *p)
{
    const uint64_t v = (uint64_t) p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t) v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t) (v >> 32));
    return (const char *) (((uint64_t) hi << 32) | lo);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const char *b, uint32_t bytes = 0x7FFFFFFF)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(b), (short) 0, (int) bytes, 0x00020000);
}
__device__ __forceinline__ void wt(const char *base, uint32_t off, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(base), off, 0, kSC);
}
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
__device__ __forceinline__ u32x4 addv(u32x4 a, u32x4 b) { return a + b; }

// XCD-grouped block map: workgroup b runs on XCD b % 8; within each group of 64 workgroups XCD x
// takes logical blocks 8x .. 8x + 7, so neighbouring 1 KiB blocks share an L2.
__device__ __forceinline__ uint64_t lblock(uint64_t b, uint64_t g, bool xcd)
{
    if (!xcd || b >= (g & ~63ull)) return b;
    return (b & ~63ull) | ((b & 7) << 3) | ((b >> 3) & 7);
}

struct Args {
    const char *s[2];  // sources (s + k is element 0)
    char *d;           // dest (16-B aligned)
    uint64_t nitems;   // 16-B dest items
    uint32_t k;        // byte shift of the sources
    uint64_t total;    // bytes
};

// 0: aligned reference (k must be 0): nt global loads, wt stores.
template <int NS>
__global__ __launch_bounds__(64) void k_aligned(Args a)
{
    const uint64_t i = (uint64_t) blockIdx.x * 64 + threadIdx.x;
    if (i >= a.nitems) return;
    u32x4 x = __builtin_nontemporal_load((const u32x4 *) (a.s[0] + i * 16));
    if (NS == 2) x = addv(x, __builtin_nontemporal_load((const u32x4 *) (a.s[1] + i * 16)));
    wt(uptr(a.d + (i - threadIdx.x) * 16), threadIdx.x * 16u, x);
}

// Aligned copy / a + b shapes (round 5): BS threads per workgroup, U 16-B items per thread (all
// loads before the stores), store cache policy SAUX (17 = sc0 sc1 write-through, 2 = nt,
// 1 = sc0, 16 = sc1, 0 = default), buffer loads based at the workgroup's first item.
template <int NS, int BS, int U, int SAUX, bool SERIAL = false>
__global__ __launch_bounds__(BS) void k_al(Args a)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = (uint64_t) blockIdx.x * BS * U;
    if (i0 >= a.nitems) return;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint32_t off = (u * BS + tid) * 16u;
        x[u] = __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[0] + i0 * 16)), off, 0, kNT);
        if (SERIAL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (NS == 2) x[u] = addv(x[u], __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[1] + i0 * 16)), off, 0, kNT));
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (i0 + u * BS + tid < a.nitems)
            __builtin_amdgcn_raw_buffer_store_b128(x[u], rsrc(uptr(a.d + i0 * 16)), (u * BS + tid) * 16u, 0, SAUX);
}

// Neighbour exchange flavours for the aligned-load + funnel family.
enum { X_SHFL = 0, X_DPP = 1, X_TWO = 2 };

template <int X>
__device__ __forceinline__ u32x4 realigned(const char *src, uint64_t total, uint64_t wo, uint32_t k, uint32_t tid)
{
    const char *sb = uptr(src + k + wo - k);  // src + wo is 16-B aligned (src aligned)
    (void) total;
    const auto r = rsrc(sb);
    const u32x4 A = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u, 0, kNT);
    u32x4 B;
    if constexpr (X == X_TWO) {
        B = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u + 16u, 0, kNT);
    } else {
        if constexpr (X == X_SHFL) {
            B.x = __shfl_down(A.x, 1u);
            B.y = __shfl_down(A.y, 1u);
            B.z = __shfl_down(A.z, 1u);
            B.w = __shfl_down(A.w, 1u);
        } else {
            B.x = __builtin_amdgcn_update_dpp(0u, A.x, 0x130, 0xF, 0xF, false);
            B.y = __builtin_amdgcn_update_dpp(0u, A.y, 0x130, 0xF, 0xF, false);
            B.z = __builtin_amdgcn_update_dpp(0u, A.z, 0x130, 0xF, 0xF, false);
            B.w = __builtin_amdgcn_update_dpp(0u, A.w, 0x130, 0xF, 0xF, false);
        }
        if (tid == 63) B = __builtin_amdgcn_raw_buffer_load_b128(r, 64 * 16u, 0, kNT);
    }
    return funnel16(A, B, k);
}

template <int NS, int X, bool XCD>
__global__ __launch_bounds__(64) void k_realign(Args a)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t b = lblock(blockIdx.x, gridDim.x, XCD);
    const uint64_t i0 = b * 64;
    if (i0 >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    // sources are allocated 16-B aligned; element 0 of source j is at s[j] + k.
    u32x4 acc = realigned<X>(a.s[0], a.total, wo, a.k, tid);
    if (NS == 2) acc = addv(acc, realigned<X>(a.s[1], a.total, wo, a.k, tid));
    if (i0 + tid < a.nitems) wt(uptr(a.d + wo), tid * 16u, acc);
}

// Unaligned 16-B loads straight from src + k (buffer or global).
template <int NS, bool BUF, bool XCD>
__global__ __launch_bounds__(64) void k_unal(Args a)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t b = lblock(blockIdx.x, gridDim.x, XCD);
    const uint64_t i0 = b * 64;
    if (i0 + tid >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    u32x4 acc;
    if constexpr (BUF) {
        acc = __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[0] + a.k + wo)), tid * 16u, 0, kNT);
        if (NS == 2) acc = addv(acc, __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[1] + a.k + wo)), tid * 16u, 0, kNT));
    } else {
        acc = __builtin_nontemporal_load((const u32x4 *) (a.s[0] + a.k + wo + tid * 16u));
        if (NS == 2) acc = addv(acc, __builtin_nontemporal_load((const u32x4 *) (a.s[1] + a.k + wo + tid * 16u)));
    }
    wt(uptr(a.d + wo), tid * 16u, acc);
}

// BS-thread workgroups (BS * 16 B of dest): aligned loads, neighbour through LDS, the last lane
// loads the next vector itself (one extra line per BS * 16 B).
template <int NS, int BS, bool XCD>
__global__ __launch_bounds__(BS) void k_lds(Args a)
{
    __shared__ u32x4 sh[NS][BS];
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = lblock(blockIdx.x, gridDim.x, XCD) * BS;
    if (i0 >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    u32x4 A[NS], B[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const auto r = rsrc(uptr(a.s[j] + wo));
        A[j] = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u, 0, kNT);
        if (tid == BS - 1) B[j] = __builtin_amdgcn_raw_buffer_load_b128(r, BS * 16u, 0, kNT);
        sh[j][tid] = A[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NS; ++j)
        if (tid < BS - 1) B[j] = sh[j][tid + 1];
    u32x4 acc = funnel16(A[0], B[0], a.k);
    if (NS == 2) acc = addv(acc, funnel16(A[1], B[1], a.k));
    if (i0 + tid < a.nitems) wt(uptr(a.d + wo), tid * 16u, acc);
}

// As k_lds, but only the wave boundaries go through LDS: within a wave the neighbour comes by a
// DPP wave shift, lane 63 of wave w takes lane 0 of wave w + 1 from LDS.
template <int NS, int BS>
__global__ __launch_bounds__(BS) void k_ldsdpp(Args a)
{
    __shared__ u32x4 sh[NS][BS / 64 + 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint64_t i0 = (uint64_t) blockIdx.x * BS;
    if (i0 >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    u32x4 A[NS], B[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const auto r = rsrc(uptr(a.s[j] + wo));
        A[j] = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u, 0, kNT);
        if (tid == BS - 1) sh[j][BS / 64] = __builtin_amdgcn_raw_buffer_load_b128(r, BS * 16u, 0, kNT);
        if (lane == 0) sh[j][w] = A[j];
        B[j].x = __builtin_amdgcn_update_dpp(0u, A[j].x, 0x130, 0xF, 0xF, false);
        B[j].y = __builtin_amdgcn_update_dpp(0u, A[j].y, 0x130, 0xF, 0xF, false);
        B[j].z = __builtin_amdgcn_update_dpp(0u, A[j].z, 0x130, 0xF, 0xF, false);
        B[j].w = __builtin_amdgcn_update_dpp(0u, A[j].w, 0x130, 0xF, 0xF, false);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NS; ++j)
        if (lane == 63) B[j] = sh[j][w + 1];
    u32x4 acc = funnel16(A[0], B[0], a.k);
    if (NS == 2) acc = addv(acc, funnel16(A[1], B[1], a.k));
    if (i0 + tid < a.nitems) wt(uptr(a.d + wo), tid * 16u, acc);
}

// Two 1 KiB blocks per one-wave workgroup, DPP shift; block 0's lane 63 takes lane 0 of block 1.
template <int NS>
__global__ __launch_bounds__(64) void k_dpp2(Args a)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = (uint64_t) blockIdx.x * 128;
    if (i0 >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    u32x4 acc[2];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const auto r = rsrc(uptr(a.s[j] + wo));
        const u32x4 A0 = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u, 0, kNT);
        const u32x4 A1 = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u + 1024u, 0, kNT);
        u32x4 C;
        if (tid == 63) C = __builtin_amdgcn_raw_buffer_load_b128(r, 2048u, 0, kNT);
        u32x4 B0, B1;
        B0.x = __builtin_amdgcn_update_dpp(0u, A0.x, 0x130, 0xF, 0xF, false);
        B0.y = __builtin_amdgcn_update_dpp(0u, A0.y, 0x130, 0xF, 0xF, false);
        B0.z = __builtin_amdgcn_update_dpp(0u, A0.z, 0x130, 0xF, 0xF, false);
        B0.w = __builtin_amdgcn_update_dpp(0u, A0.w, 0x130, 0xF, 0xF, false);
        B1.x = __builtin_amdgcn_update_dpp(0u, A1.x, 0x130, 0xF, 0xF, false);
        B1.y = __builtin_amdgcn_update_dpp(0u, A1.y, 0x130, 0xF, 0xF, false);
        B1.z = __builtin_amdgcn_update_dpp(0u, A1.z, 0x130, 0xF, 0xF, false);
        B1.w = __builtin_amdgcn_update_dpp(0u, A1.w, 0x130, 0xF, 0xF, false);
        const u32x4 f = {(uint32_t) __builtin_amdgcn_readfirstlane(A1.x), (uint32_t) __builtin_amdgcn_readfirstlane(A1.y),
                         (uint32_t) __builtin_amdgcn_readfirstlane(A1.z), (uint32_t) __builtin_amdgcn_readfirstlane(A1.w)};
        if (tid == 63) {
            B0 = f;
            B1 = C;
        }
        const u32x4 x0 = funnel16(A0, B0, a.k), x1 = funnel16(A1, B1, a.k);
        if (j == 0) {
            acc[0] = x0;
            acc[1] = x1;
        } else {
            acc[0] = addv(acc[0], x0);
            acc[1] = addv(acc[1], x1);
        }
    }
    const char *db = uptr(a.d + wo);
    if (i0 + tid < a.nitems) wt(db, tid * 16u, acc[0]);
    if (i0 + 64 + tid < a.nitems) wt(db, tid * 16u + 1024u, acc[1]);
}

// Round 6: the neighbour within the wave by DPP, lane 63's from its own load of the next vector (no
// LDS, no workgroup barrier); BS-thread workgroups so the extra load hits the line a sibling wave
// of the same workgroup (same CU, same L2) fetches.  SERIAL: source 1's load after source 0's landed.
template <int NS, int BS, bool SERIAL, bool XCD>
__global__ __launch_bounds__(BS) void k_wedge(Args a)
{
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint64_t i0 = lblock(blockIdx.x, gridDim.x, XCD) * BS;
    if (i0 >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    u32x4 acc;
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const auto r = rsrc(uptr(a.s[j] + wo));
        const u32x4 A = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u, 0, kNT);
        u32x4 E = A;
        if (lane == 63) E = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u + 16u, 0, kNT);
        if (SERIAL && j == 0 && NS == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u32x4 B;
        B.x = __builtin_amdgcn_update_dpp(0u, A.x, 0x130, 0xF, 0xF, false);
        B.y = __builtin_amdgcn_update_dpp(0u, A.y, 0x130, 0xF, 0xF, false);
        B.z = __builtin_amdgcn_update_dpp(0u, A.z, 0x130, 0xF, 0xF, false);
        B.w = __builtin_amdgcn_update_dpp(0u, A.w, 0x130, 0xF, 0xF, false);
        if (lane == 63) B = E;
        const u32x4 x = funnel16(A, B, a.k);
        acc = j == 0 ? x : addv(acc, x);
    }
    if (i0 + tid < a.nitems) wt(uptr(a.d + wo), tid * 16u, acc);
}

// Round 6: unaligned 16-B buffer loads (the phased reduce-scatter's shifted path) in BS-thread
// workgroups, optionally XCD-grouped, SERIAL as above.
template <int NS, int BS, bool SERIAL, bool XCD>
__global__ __launch_bounds__(BS) void k_unalw(Args a)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = lblock(blockIdx.x, gridDim.x, XCD) * BS;
    if (i0 + tid >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    u32x4 acc = __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[0] + a.k + wo)), tid * 16u, 0, kNT);
    if (SERIAL && NS == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (NS == 2) acc = addv(acc, __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[1] + a.k + wo)), tid * 16u, 0, kNT));
    wt(uptr(a.d + wo), tid * 16u, acc);
}

// Round 6: items laid out by the SOURCES' phase instead — aligned 16-B source loads, the store
// unaligned (dest + 16 - k + 16 i); the first 16 - k bytes and the last item are not written
// (the check skips them).  SC1: source 1 loaded system-coherent (sc0 sc1), as a peer source is.
template <int NS, bool XCD, bool SC1>
__global__ __launch_bounds__(64) void k_stshift(Args a)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = lblock(blockIdx.x, gridDim.x, XCD) * 64;
    if (i0 + tid + 1 >= a.nitems) return;
    const uint64_t wo = (i0 + 1) * 16;  // source bytes from s[j] (aligned)
    u32x4 acc = __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[0] + wo)), tid * 16u, 0, kNT);
    if (NS == 2) acc = addv(acc, __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[1] + wo)), tid * 16u, 0, SC1 ? 17 : kNT));
    __builtin_amdgcn_raw_buffer_store_b128(acc, rsrc(uptr(a.d + wo - a.k)), tid * 16u, 0, kSC);
}

// The reduce-scatter's current shifted shape with source 1 system-coherent (its peer), for k_stshift.
template <int NS, bool XCD>
__global__ __launch_bounds__(64) void k_unal_sc(Args a)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = lblock(blockIdx.x, gridDim.x, XCD) * 64;
    if (i0 + tid >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    u32x4 acc = __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[0] + a.k + wo)), tid * 16u, 0, kNT);
    if (NS == 2) acc = addv(acc, __builtin_amdgcn_raw_buffer_load_b128(rsrc(uptr(a.s[1] + a.k + wo)), tid * 16u, 0, 17));
    wt(uptr(a.d + wo), tid * 16u, acc);
}

// Round 6 (late): unaligned 16-B loads, one-wave workgroups, each workgroup U CONSECUTIVE 1 KiB
// blocks, so the line straddling two blocks is re-read by the same wave (same CU, same L2) however
// the workgroups are spread over the XCDs — the XCD grouping's effect without depending on the
// dispatch order (which co-located PEs' grids break).  BURST: every block's loads issued before the
// first store; otherwise block by block.
template <int NS, int U, bool BURST>
__global__ __launch_bounds__(64) void k_unalc(Args a)
{
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = (uint64_t) blockIdx.x * 64 * U;
    if (i0 >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    const auto r0 = rsrc(uptr(a.s[0] + a.k + wo)), r1 = rsrc(uptr(a.s[1] + a.k + wo));
    const auto rd = rsrc(uptr(a.d + wo));
    if constexpr (BURST) {
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t off = (u * 64 + tid) * 16u;
            if (i0 + u * 64 + tid < a.nitems) {
                x[u] = __builtin_amdgcn_raw_buffer_load_b128(r0, off, 0, kNT);
                if (NS == 2) x[u] = addv(x[u], __builtin_amdgcn_raw_buffer_load_b128(r1, off, 0, kNT));
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * 64 + tid < a.nitems) __builtin_amdgcn_raw_buffer_store_b128(x[u], rd, (u * 64 + tid) * 16u, 0, kSC);
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t off = (u * 64 + tid) * 16u;
            if (i0 + u * 64 + tid >= a.nitems) break;
            u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r0, off, 0, kNT);
            if (NS == 2) x = addv(x, __builtin_amdgcn_raw_buffer_load_b128(r1, off, 0, kNT));
            __builtin_amdgcn_raw_buffer_store_b128(x, rd, off, 0, kSC);
        }
    }
}

// The product's kernels with FaninArgs built as runtime.cpp plan_fanin builds them.
static ishmemi::FaninArgs prod_args(const Args &a, int ns, bool aligned)
{
    ishmemi::FaninArgs f{};
    f.nsrc = ns;
    for (int j = 0; j < ns; ++j) f.src[j] = a.s[j] + a.k;
    f.dst = a.d;
    f.head = 0;
    f.nitems = a.nitems;
    f.tail = 0;
    f.realign = aligned ? 0 : 1;
    for (int j = 0; j < ns; ++j) f.shift[j] = a.k;
    f.total = a.nitems * 16;
    return f;
}

struct Variant {
    std::string name;
    int ns;
    int block;           // threads per workgroup
    uint64_t per_wg;     // items per workgroup
    bool aligned;        // k = 0
    void (*kern)(Args);
    int prod = 0;  // 1: product aligned fanin_kernel, 2: product fanin_realign_kernel
};

// Product-kernel variants (what makes fanin_realign_kernel slower than k_ldsdpp?):
//   V bit 0: descriptor bound 0x7FFFFFFF instead of the source's end;  bit 1: one shift (shift[0])
//   for both sources;  bit 2: funnel by dynamic register indexing instead of the switch;
//   bit 3: one-shot (early return) instead of the grid-stride loop.
[[maybe_unused]] __device__ __forceinline__ u32x4 funnel_idx(const u32x4 &A, const u32x4 &B, uint32_t k)
{
    const uint32_t W[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
    const uint32_t q = __builtin_amdgcn_readfirstlane(k >> 2), r = k & 3;
    return u32x4{__builtin_amdgcn_alignbyte(W[q + 1], W[q], r), __builtin_amdgcn_alignbyte(W[q + 2], W[q + 1], r),
                 __builtin_amdgcn_alignbyte(W[q + 3], W[q + 2], r), __builtin_amdgcn_alignbyte(W[q + 4], W[q + 3], r)};
}

// var24 of the round-5 ablation: the product structure with each source loaded, its edge vector
// stored to LDS and published before the next source is issued, one-shot (this is the order the
// product kernel now uses; the ablation's other variants are recorded in profiles/r05/realign/).
template <int NS, int V>
__global__ __launch_bounds__(ishmemi::kRealignBlock) void k_prodvar(ishmemi::FaninArgs a)
{
    using namespace ishmemi;
    __shared__ u32x4 edge[NS][kRealignWaves];
    __shared__ u32x4 edge2[NS][1];
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = (uint64_t) blockIdx.x * kRealignBlock;
    if (i0 >= a.nitems) return;
    const uint64_t wo = i0 * 16;
    u32x4 A[NS], B[NS];
    uint32_t sh[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        sh[j] = (V & 2) ? a.shift[0] : a.shift[j];
        const char *sb = uniform_ptr(a.src[j] + (wo - sh[j]));
        const auto r = make_rsrc(sb);
        A[j] = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u, 0, kNonTemporal);
        if (tid == kRealignBlock - 1) edge2[j][0] = __builtin_amdgcn_raw_buffer_load_b128(r, kRealignBlock * 16u, 0, kNonTemporal);
        if ((tid & 63) == 0) edge[j][tid >> 6] = A[j];
        B[j] = wave_next(A[j]);
    }
    __syncthreads();
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        if ((tid & 63) == 63) B[j] = tid == kRealignBlock - 1 ? edge2[j][0] : edge[j][(tid >> 6) + 1];
        acc = acc + ishmemi::funnel16(A[j], B[j], sh[j]);
    }
    if (i0 + tid < a.nitems) wt_store(make_rsrc(uniform_ptr(a.dst + wo)), tid * 16u, acc);
}

static void launch(const Variant &v, const Args &a, hipStream_t st)
{
    const unsigned g = (unsigned) ((a.nitems + v.per_wg - 1) / v.per_wg);
    if (v.prod == 0) {
        hipLaunchKernelGGL(v.kern, dim3(g), dim3(v.block), 0, st, a);
        return;
    }
    const ishmemi::FaninArgs f = prod_args(a, v.ns, v.prod == 1);
    using namespace ishmemi;
    if (v.prod >= 16) {
        const int V = v.prod - 16;
        auto go = [&](auto k1, auto k2) {
            if (v.ns == 1) hipLaunchKernelGGL(k1, dim3(g), dim3(v.block), 0, st, f);
            else hipLaunchKernelGGL(k2, dim3(g), dim3(v.block), 0, st, f);
        };
        switch (V) {
            case 24: go(k_prodvar<1, 24>, k_prodvar<2, 24>); break;
            case 26: go(k_prodvar<1, 26>, k_prodvar<2, 26>); break;
            default: break;
        }
        return;
    }
    if (v.prod == 1) {
        if (v.ns == 1) hipLaunchKernelGGL((fanin_kernel<uint32_t, ISHMEMI_OP_SUM, true, 1>), dim3(g), dim3(v.block), 0, st, f);
        else hipLaunchKernelGGL((fanin_kernel<uint32_t, ISHMEMI_OP_SUM, true, 2>), dim3(g), dim3(v.block), 0, st, f);
    } else {
        if (v.ns == 1) hipLaunchKernelGGL((fanin_realign_kernel<uint32_t, ISHMEMI_OP_SUM, 1>), dim3(g), dim3(v.block), 0, st, f);
        else hipLaunchKernelGGL((fanin_realign_kernel<uint32_t, ISHMEMI_OP_SUM, 2>), dim3(g), dim3(v.block), 0, st, f);
    }
}

int main(int argc, char **argv)
{
    const uint64_t mib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024;
    const int rounds = argc > 2 ? atoi(argv[2]) : 3;
    const int iters = argc > 3 ? atoi(argv[3]) : 10;
    const uint32_t kshift = argc > 4 ? (uint32_t) atoi(argv[4]) : 4;
    const uint64_t bytes = mib << 20, n = bytes / 16;
    char *s0, *s1, *d;
    CK(hipMalloc(&s0, bytes + 4096));
    CK(hipMalloc(&s1, bytes + 4096));
    CK(hipMalloc(&d, bytes + 4096));
    std::vector<uint32_t> h((bytes + 4096) / 4), h1((bytes + 4096) / 4);
    uint32_t x = 12345;
    for (auto &v : h) v = (x = x * 1664525u + 1013904223u);
    for (auto &v : h1) v = (x = x * 1664525u + 1013904223u);
    CK(hipMemcpy(s0, h.data(), bytes + 4096, hipMemcpyHostToDevice));
    CK(hipMemcpy(s1, h1.data(), bytes + 4096, hipMemcpyHostToDevice));
    std::vector<Variant> vs = {
        {"a+b product aligned", 2, 64, 64, true, nullptr, 1},
        {"a+b unal 64 (rs now)", 2, 64, 64, false, k_unalw<2, 64, false, false>},
        {"a+b unal 64 xcd", 2, 64, 64, false, k_unalw<2, 64, false, true>},
        {"a+b unalc 2 loop", 2, 64, 128, false, k_unalc<2, 2, false>},
        {"a+b unalc 4 loop", 2, 64, 256, false, k_unalc<2, 4, false>},
        {"a+b unalc 8 loop", 2, 64, 512, false, k_unalc<2, 8, false>},
        {"a+b unalc 16 loop", 2, 64, 1024, false, k_unalc<2, 16, false>},
        {"a+b unalc 2 burst", 2, 64, 128, false, k_unalc<2, 2, true>},
        {"a+b unalc 4 burst", 2, 64, 256, false, k_unalc<2, 4, true>},
        {"a+b unalc 8 burst", 2, 64, 512, false, k_unalc<2, 8, true>},
        {"copy product aligned", 1, 64, 64, true, nullptr, 1},
        {"copy product realign", 1, 512, 512, false, nullptr, 2},
        {"copy unal 64", 1, 64, 64, false, k_unalw<1, 64, false, false>},
        {"copy unalc 4 loop", 1, 64, 256, false, k_unalc<1, 4, false>},
        {"copy unalc 8 burst", 1, 64, 512, false, k_unalc<1, 8, true>},
    };
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint32_t> got(n * 4);
    std::vector<std::vector<float>> ms(vs.size());
    printf("size %llu MiB, shift %u B, %d rounds x %d iterations\n", (unsigned long long) mib, kshift, rounds, iters);
    for (size_t v = 0; v < vs.size(); ++v) {  // correctness, once per variant
        Args a{{s0, s1}, d, n, vs[v].aligned ? 0u : kshift, bytes};
        CK(hipMemset(d, 0, bytes));
        launch(vs[v], a, st);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(got.data(), d, bytes, hipMemcpyDeviceToHost));
        const uint32_t k = a.k;
        uint64_t bad = 0;
        const bool st = vs[v].name.find("stshift") != std::string::npos;
        for (uint64_t w = 0; w < n * 4; ++w) {
            if (st && (4 * w < 16 - k || 4 * w + 4 > 16 * (n - 1) + 16 - k)) continue;
            uint32_t e0w, e1w;
            memcpy(&e0w, (const char *) h.data() + k + 4 * w, 4);
            memcpy(&e1w, (const char *) h1.data() + k + 4 * w, 4);
            const uint32_t want = vs[v].ns == 2 ? e0w + e1w : e0w;
            bad += got[w] != want;
        }
        printf("check %-28s %s (%llu bad words)\n", vs[v].name.c_str(), bad ? "FAIL" : "ok", (unsigned long long) bad);
    }
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            Args a{{s0, s1}, d, n, vs[v].aligned ? 0u : kshift, bytes};
            launch(vs[v], a, st);
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; ++i) launch(vs[v], a, st);
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[v].push_back(t / iters);
        }
    }
    for (size_t v = 0; v < vs.size(); ++v) {
        auto m = ms[v];
        std::sort(m.begin(), m.end());
        const double med = m[m.size() / 2];
        const double tb = (vs[v].ns + 1.0) * bytes / (med * 1e-3) / 1e12;
        printf("%-28s med %.4f ms  min %.4f max %.4f  %.2f TB/s  frac %.3f\n", vs[v].name.c_str(), med, m.front(),
               m.back(), tb, tb / 8.0);
    }
    return 0;
}
