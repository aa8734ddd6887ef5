// Dev tool (not product): sweep of streaming-kernel variants for the local combine / copy unit
// on MI355X.  Interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/stream_variants.hip -o build/stream_variants
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e = (x);                                                                        \
        if (e != hipSuccess) {                                                                     \
            printf("%s failed: %s\n", #x, hipGetErrorString(e));                                   \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ f4 ld(const f4 *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(f4 *p, f4 v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// NSRC sources -> dst, U 16-B items per thread per iteration.
// CONTIG: each block owns a contiguous range; else tiles interleave over blocks.
template <int NSRC, int U, int BS, bool NTL, bool NTS, bool CONTIG>
__global__ __launch_bounds__(BS) void kern(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                           f4 *__restrict__ d, long n)
{
    const long TI = (long) BS * U;
    long start, end, stride;
    if (CONTIG) {
        const long per = ((n + gridDim.x - 1) / gridDim.x + TI - 1) / TI * TI;
        start = (long) blockIdx.x * per;
        end = min(start + per, n);
        stride = TI;
    } else {
        start = (long) blockIdx.x * TI;
        end = n;
        stride = (long) gridDim.x * TI;
    }
    for (long t = start; t < end; t += stride) {
        f4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = t + (long) u * BS + threadIdx.x;
            if (i < end) {
                x[u] = ld<NTL>(a + i);
                if (NSRC == 2) y[u] = ld<NTL>(b + i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = t + (long) u * BS + threadIdx.x;
            if (i < end) st<NTS>(d + i, NSRC == 2 ? x[u] + y[u] : x[u]);
        }
    }
}

// One-shot: no loop, grid covers n exactly (the dispatcher does the scheduling).
template <int NSRC, int U, int BS, bool NTL, bool NTS>
__global__ __launch_bounds__(BS) void oneshot(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                              f4 *__restrict__ d, long n)
{
    const long t = (long) blockIdx.x * BS * U;
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = t + (long) u * BS + threadIdx.x;
        if (i < n) {
            x[u] = ld<NTL>(a + i);
            if (NSRC == 2) y[u] = ld<NTL>(b + i);
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = t + (long) u * BS + threadIdx.x;
        if (i < n) st<NTS>(d + i, NSRC == 2 ? x[u] + y[u] : x[u]);
    }
}

// Read-only ceiling: xor-accumulate, one store per thread.
template <int U, int BS, bool NTL>
__global__ __launch_bounds__(BS) void readonly(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                               f4 *__restrict__ d, long n)
{
    const long t = (long) blockIdx.x * BS * U;
    f4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = t + (long) u * BS + threadIdx.x;
        if (i < n) acc += ld<NTL>(a + i);
    }
    if (acc.x == 12345.f) d[threadIdx.x] = acc;
}

// Write-only ceiling.
template <int U, int BS, bool NTS>
__global__ __launch_bounds__(BS) void writeonly(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                                f4 *__restrict__ d, long n)
{
    const long t = (long) blockIdx.x * BS * U;
    const f4 v = {1, 2, 3, 4};
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = t + (long) u * BS + threadIdx.x;
        if (i < n) st<NTS>(d + i, v);
    }
}

// LDS-DMA copy: each wave moves 1 KiB per global_load_lds_dwordx4 into its own LDS slot, then
// ds_read_b128 + global store.
template <int U, int BS, bool NTL, bool NTS>
__global__ __launch_bounds__(BS) void ldsdma_copy(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                                  f4 *__restrict__ d, long n)
{
    __shared__ __attribute__((aligned(16))) f4 buf[U * BS];
    const long t = (long) blockIdx.x * BS * U;
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = t + (long) u * BS + threadIdx.x;
        __builtin_amdgcn_global_load_lds((const void *) (a + (i < n ? i : 0)),
                                         (__attribute__((address_space(3))) void *) &buf[u * BS + wave * 64],
                                         16, 0, NTL ? 2 : 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const long i = t + (long) u * BS + threadIdx.x;
        f4 v = buf[u * BS + wave * 64 + lane];
        if (i < n) st<NTS>(d + i, v);
    }
}

struct Variant {
    std::string name;
    void (*launch)(const f4 *, const f4 *, f4 *, long, int, hipStream_t);
    int grid;
    int nsrc;
};

template <int NSRC, int U, int BS, bool NTL, bool NTS, bool CONTIG>
void L(const f4 *a, const f4 *b, f4 *d, long n, int grid, hipStream_t s)
{
    hipLaunchKernelGGL((kern<NSRC, U, BS, NTL, NTS, CONTIG>), dim3(grid), dim3(BS), 0, s, a, b, d, n);
}

template <int NSRC, int U, int BS, bool NTL, bool NTS>
void O(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    const long g = (n + (long) BS * U - 1) / ((long) BS * U);
    hipLaunchKernelGGL((oneshot<NSRC, U, BS, NTL, NTS>), dim3(g), dim3(BS), 0, s, a, b, d, n);
}
template <int U, int BS, bool NTL>
void RO(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    const long g = (n + (long) BS * U - 1) / ((long) BS * U);
    hipLaunchKernelGGL((readonly<U, BS, NTL>), dim3(g), dim3(BS), 0, s, a, b, d, n);
}
template <int U, int BS, bool NTS>
void WO(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    const long g = (n + (long) BS * U - 1) / ((long) BS * U);
    hipLaunchKernelGGL((writeonly<U, BS, NTS>), dim3(g), dim3(BS), 0, s, a, b, d, n);
}
template <int U, int BS, bool NTL, bool NTS>
void LD(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    const long g = (n + (long) BS * U - 1) / ((long) BS * U);
    hipLaunchKernelGGL((ldsdma_copy<U, BS, NTL, NTS>), dim3(g), dim3(BS), 0, s, a, b, d, n);
}

void MC(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    (void) hipMemcpyAsync(d, a, n * 16, hipMemcpyDeviceToDevice, s);
}

#define V(NS, U, BS, NTL, NTS, C, G)                                                               \
    vs.push_back({"ns" #NS " U" #U " bs" #BS " ntl" #NTL " nts" #NTS " contig" #C " g" #G,          \
                  L<NS, U, BS, NTL, NTS, C>, G, NS})

int main(int argc, char **argv)
{
    const long bytes = 1l << 30;
    const long n = bytes / 16;
    f4 *a, *b, *d;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    std::vector<Variant> vs;
    vs.push_back({"oneshot ns1 U1 bs256 nt/nt", O<1, 1, 256, true, true>, 0, 1});
    vs.push_back({"oneshot ns1 U1 bs256 nt/plain", O<1, 1, 256, true, false>, 0, 1});
    vs.push_back({"oneshot ns1 U1 bs128 nt/nt", O<1, 1, 128, true, true>, 0, 1});
    vs.push_back({"oneshot ns1 U1 bs512 nt/nt", O<1, 1, 512, true, true>, 0, 1});
    vs.push_back({"oneshot ns1 U1 bs1024 nt/nt", O<1, 1, 1024, true, true>, 0, 1});
    vs.push_back({"oneshot ns1 U2 bs128 nt/nt", O<1, 2, 128, true, true>, 0, 1});
    vs.push_back({"oneshot ns1 U4 bs256 nt/nt", O<1, 4, 256, true, true>, 0, 1});
    vs.push_back({"oneshot ns1 U4 bs64 nt/nt", O<1, 4, 64, true, true>, 0, 1});
    vs.push_back({"oneshot ns2 U1 bs256 nt/nt", O<2, 1, 256, true, true>, 0, 2});
    vs.push_back({"oneshot ns2 U1 bs256 nt/plain", O<2, 1, 256, true, false>, 0, 2});
    vs.push_back({"oneshot ns2 U1 bs128 nt/nt", O<2, 1, 128, true, true>, 0, 2});
    vs.push_back({"oneshot ns2 U1 bs512 nt/nt", O<2, 1, 512, true, true>, 0, 2});
    vs.push_back({"oneshot ns2 U1 bs1024 nt/nt", O<2, 1, 1024, true, true>, 0, 2});
    vs.push_back({"oneshot ns2 U2 bs128 nt/nt", O<2, 2, 128, true, true>, 0, 2});
    vs.push_back({"oneshot ns2 U2 bs256 nt/nt", O<2, 2, 256, true, true>, 0, 2});
    vs.push_back({"writeonly U1 plain (traffic=1B)", WO<1, 256, false>, 0, 0});
    vs.push_back({"writeonly U1 nt (traffic=1B)", WO<1, 256, true>, 0, 0});
    vs.push_back({"writeonly U2 nt bs512 (traffic=1B)", WO<2, 512, true>, 0, 0});
    vs.push_back({"readonly U1 nt (traffic=1B)", RO<1, 256, true>, 0, 0});
    vs.push_back({"readonly U2 nt (traffic=1B)", RO<2, 256, true>, 0, 0});
    vs.push_back({"hipMemcpyAsync D2D", MC, 0, 1});
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int rounds = argc > 1 ? atoi(argv[1]) : 5, iters = 10;
    std::vector<std::vector<float>> ms(vs.size());
    for (auto &v : vs) v.launch(a, b, d, n, v.grid, s);  // warm
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < rounds; ++r) {
        for (size_t k = 0; k < vs.size(); ++k) {
            auto &v = vs[k];
            v.launch(a, b, d, n, v.grid, s);
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < iters; ++i) v.launch(a, b, d, n, v.grid, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            ms[k].push_back(t / iters);
        }
    }
    for (size_t k = 0; k < vs.size(); ++k) {
        auto m = ms[k];
        std::sort(m.begin(), m.end());
        const double med = m[m.size() / 2], best = m[0];
        const double traffic = (double) bytes * (vs[k].nsrc == 0 ? 1 : vs[k].nsrc + 1);
        printf("%-48s med %.4f ms  %.0f GB/s (%.1f%%)  best %.0f GB/s\n", vs[k].name.c_str(), med,
               traffic / med / 1e6, traffic / med / 1e6 / 80.0, traffic / best / 1e6);
    }
    return 0;
}
