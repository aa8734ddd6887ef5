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

// 256-thread workgroups (4 KiB of dest): aligned loads, neighbour through LDS, lane 255 loads.
template <int NS>
__global__ __launch_bounds__(256) void k_lds(Args a)
{
    __shared__ u32x4 sh[NS][256];
    const uint32_t tid = threadIdx.x;
    const uint64_t i0 = (uint64_t) blockIdx.x * 256;
    const uint64_t wo = i0 * 16;
    u32x4 A[NS], B[NS];
#pragma unroll
    for (int j = 0; j < NS; ++j) {
        const auto r = rsrc(uptr(a.s[j] + wo));
        A[j] = __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16u, 0, kNT);
        if (tid == 255) B[j] = __builtin_amdgcn_raw_buffer_load_b128(r, 256 * 16u, 0, kNT);
        sh[j][tid] = A[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < NS; ++j)
        if (tid < 255) B[j] = sh[j][tid + 1];
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

struct Variant {
    std::string name;
    int ns;
    int block;           // threads per workgroup
    uint64_t per_wg;     // items per workgroup
    bool aligned;        // k = 0
    void (*kern)(Args);
};

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
        {"copy aligned", 1, 64, 64, true, k_aligned<1>},
        {"copy shfl", 1, 64, 64, false, k_realign<1, X_SHFL, false>},
        {"copy dpp", 1, 64, 64, false, k_realign<1, X_DPP, false>},
        {"copy two-loads", 1, 64, 64, false, k_realign<1, X_TWO, false>},
        {"copy shfl xcd8", 1, 64, 64, false, k_realign<1, X_SHFL, true>},
        {"copy dpp xcd8", 1, 64, 64, false, k_realign<1, X_DPP, true>},
        {"copy unaligned buf", 1, 64, 64, false, k_unal<1, true, false>},
        {"copy unaligned glb", 1, 64, 64, false, k_unal<1, false, false>},
        {"copy unaligned buf xcd8", 1, 64, 64, false, k_unal<1, true, true>},
        {"copy lds256", 1, 256, 256, false, k_lds<1>},
        {"copy dpp2", 1, 64, 128, false, k_dpp2<1>},
        {"a+b aligned", 2, 64, 64, true, k_aligned<2>},
        {"a+b shfl", 2, 64, 64, false, k_realign<2, X_SHFL, false>},
        {"a+b dpp", 2, 64, 64, false, k_realign<2, X_DPP, false>},
        {"a+b two-loads", 2, 64, 64, false, k_realign<2, X_TWO, false>},
        {"a+b dpp xcd8", 2, 64, 64, false, k_realign<2, X_DPP, true>},
        {"a+b unaligned buf", 2, 64, 64, false, k_unal<2, true, false>},
        {"a+b unaligned glb", 2, 64, 64, false, k_unal<2, false, false>},
        {"a+b unaligned buf xcd8", 2, 64, 64, false, k_unal<2, true, true>},
        {"a+b lds256", 2, 256, 256, false, k_lds<2>},
        {"a+b dpp2", 2, 64, 128, false, k_dpp2<2>},
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
        const unsigned g = (unsigned) ((n + vs[v].per_wg - 1) / vs[v].per_wg);
        hipLaunchKernelGGL(vs[v].kern, dim3(g), dim3(vs[v].block), 0, st, a);
        CK(hipStreamSynchronize(st));
        CK(hipMemcpy(got.data(), d, bytes, hipMemcpyDeviceToHost));
        const uint32_t k = a.k;
        uint64_t bad = 0;
        for (uint64_t w = 0; w < n * 4; ++w) {
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
            const unsigned g = (unsigned) ((n + vs[v].per_wg - 1) / vs[v].per_wg);
            hipLaunchKernelGGL(vs[v].kern, dim3(g), dim3(vs[v].block), 0, st, a);
            CK(hipEventRecord(e0, st));
            for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(vs[v].kern, dim3(g), dim3(vs[v].block), 0, st, a);
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
