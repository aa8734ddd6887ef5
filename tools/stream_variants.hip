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

// One-shot with an XCD-aware block order: workgroups are dispatched round-robin over the 8 XCDs
// (block b runs on XCD b % 8), so the remap gives each XCD one contiguous eighth of the array.
template <int NSRC, int BS, bool NTL, bool NTS>
__global__ __launch_bounds__(BS) void oneshot_xcd(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                                  f4 *__restrict__ d, long n)
{
    const long per = gridDim.x / 8;  // grid is a multiple of 8
    const long lb = (long) (blockIdx.x % 8) * per + blockIdx.x / 8;
    const long i = lb * BS + threadIdx.x;
    if (i < n) {
        f4 x = ld<NTL>(a + i);
        if (NSRC == 2) x += ld<NTL>(b + i);
        st<NTS>(d + i, x);
    }
}

// One-shot with system-coherent write-through stores (buffer_store ... sc0 sc1).
template <int BS>
__global__ __launch_bounds__(BS) void oneshot_wt(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                                 f4 *__restrict__ d, long n)
{
    const long base = (long) blockIdx.x * BS;
    const long i = base + threadIdx.x;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc((void *) (d + base), (short) 0, 0x7FFFFFFF, 0x00020000);
    if (i < n) {
        const f4 x = __builtin_nontemporal_load(a + i);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, x),
                                               r, threadIdx.x * 16, 0, 17);
    }
}

// One-shot with buffer loads / stores and explicit cache-policy bits on both (gfx950 aux:
// 1 = sc0, 2 = nt, 16 = sc1).
typedef unsigned u4 __attribute__((ext_vector_type(4)));
template <int NSRC, int BS, int LAUX, int SAUX>
__global__ __launch_bounds__(BS) void oneshot_aux(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                                  f4 *__restrict__ d, long n)
{
    const long base = (long) blockIdx.x * BS;
    const __amdgpu_buffer_rsrc_t ra =
        __builtin_amdgcn_make_buffer_rsrc((void *) (a + base), (short) 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rb =
        __builtin_amdgcn_make_buffer_rsrc((void *) (b + base), (short) 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc((void *) (d + base), (short) 0, 0x7FFFFFFF, 0x00020000);
    if (base + threadIdx.x < n) {
        f4 x = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, threadIdx.x * 16, 0, LAUX));
        if (NSRC == 2) x += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rb, threadIdx.x * 16, 0, LAUX));
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x), rd, threadIdx.x * 16, 0, SAUX);
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

// Copy with a second, far item per thread: items i and i + n/2 (two DRAM regions in flight per
// wave), nt loads, write-through stores.
template <int BS>
__global__ __launch_bounds__(BS) void split_halves(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                                   f4 *__restrict__ d, long n)
{
    const long h = n / 2;
    const long i = (long) blockIdx.x * BS + threadIdx.x;
    const __amdgpu_buffer_rsrc_t r0 =
        __builtin_amdgcn_make_buffer_rsrc((void *) (d + (long) blockIdx.x * BS), (short) 0, 0x7FFFFFFF, 0x00020000);
    const __amdgpu_buffer_rsrc_t r1 =
        __builtin_amdgcn_make_buffer_rsrc((void *) (d + h + (long) blockIdx.x * BS), (short) 0, 0x7FFFFFFF, 0x00020000);
    if (i < h) {
        const f4 x = __builtin_nontemporal_load(a + i);
        const f4 y = __builtin_nontemporal_load(a + h + i);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, x), r0, threadIdx.x * 16, 0, 17);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, y), r1, threadIdx.x * 16, 0, 17);
    }
}

// Round 3: the multi-PE kernel's reduce-scatter shape — persistent grid, each workgroup a
// contiguous range, U 16-B items per thread per step from NSRC sources (nt buffer loads), the fold
// stored write-through (sc0 sc1).  gfx9 waves count loads and stores in ONE in-order vmcnt, so a
// step that waits for its loads also waits for the previous step's stores to be acknowledged.
// PIPE: the next step's loads are issued before this step's stores (ping-pong register sets), so
// the store acknowledgements overlap the next loads.
template <int NSRC, int U, int BS, bool PIPE>
__global__ __launch_bounds__(BS) void persist_wt(const f4 *__restrict__ a, const f4 *__restrict__ b,
                                                 f4 *__restrict__ d, long n)
{
    const long TI = (long) BS * U;
    const long per = ((n + gridDim.x - 1) / gridDim.x + TI - 1) / TI * TI;
    const long start = (long) blockIdx.x * per, end = min(start + per, n);
    auto rs = [](const void *p) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short) 0, 0x7FFFFFFF, 0x00020000);
    };
    auto load = [&](long t, f4 (&x)[U][2]) {
        const __amdgpu_buffer_rsrc_t ra = rs(a + t), rb = rs(b + t);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t off = (uint32_t) (u * BS + threadIdx.x) * 16;
            if (t + u * BS + threadIdx.x < end) {
                x[u][0] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 2));
                if (NSRC == 2) x[u][1] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 2));
            }
        }
    };
    auto store = [&](long t, const f4 (&x)[U][2]) {
        const __amdgpu_buffer_rsrc_t rd = rs(d + t);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t off = (uint32_t) (u * BS + threadIdx.x) * 16;
            const f4 v = NSRC == 2 ? x[u][0] + x[u][1] : x[u][0];
            if (t + u * BS + threadIdx.x < end) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, v), rd, off, 0, 17);
        }
    };
    f4 xa[U][2], xb[U][2];
    if (!PIPE) {
        for (long t = start; t < end; t += TI) {
            load(t, xa);
            store(t, xa);
        }
        return;
    }
    long t = start;
    if (t < end) load(t, xa);
    while (t < end) {
        if (t + TI < end) load(t + TI, xb);
        store(t, xa);
        t += TI;
        if (t >= end) break;
        if (t + TI < end) load(t + TI, xa);
        store(t, xb);
        t += TI;
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

template <int NSRC, int BS, bool NTL, bool NTS>
void OX(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    const long g = ((n + BS - 1) / BS + 7) / 8 * 8;
    hipLaunchKernelGGL((oneshot_xcd<NSRC, BS, NTL, NTS>), dim3(g), dim3(BS), 0, s, a, b, d, n);
}
template <int BS>
void OW(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    const long g = (n + BS - 1) / BS;
    hipLaunchKernelGGL((oneshot_wt<BS>), dim3(g), dim3(BS), 0, s, a, b, d, n);
}

template <int NSRC, int BS, int LAUX, int SAUX>
void OA(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    const long g = (n + BS - 1) / BS;
    hipLaunchKernelGGL((oneshot_aux<NSRC, BS, LAUX, SAUX>), dim3(g), dim3(BS), 0, s, a, b, d, n);
}

// The product copy shape with `lds` bytes of dynamic LDS per workgroup: caps workgroups (waves)
// per CU, i.e. requests in flight per CU.
template <int NSRC, int BS, int LAUX, int SAUX, int LDS>
void OAL(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    const long g = (n + BS - 1) / BS;
    hipLaunchKernelGGL((oneshot_aux<NSRC, BS, LAUX, SAUX>), dim3(g), dim3(BS), LDS, s, a, b, d, n);
}
template <int BS>
void SH(const f4 *a, const f4 *b, f4 *d, long n, int, hipStream_t s)
{
    const long g = (n / 2 + BS - 1) / BS;
    hipLaunchKernelGGL((split_halves<BS>), dim3(g), dim3(BS), 0, s, a, b, d, n);
}

template <int NSRC, int U, int BS, bool PIPE>
void PW(const f4 *a, const f4 *b, f4 *d, long n, int grid, hipStream_t s)
{
    hipLaunchKernelGGL((persist_wt<NSRC, U, BS, PIPE>), dim3(grid), dim3(BS), 0, s, a, b, d, n);
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
    const std::string layout = argc > 3 ? argv[3] : "separate";
    if (layout == "separate") {
        CK(hipMalloc(&a, bytes));
        CK(hipMalloc(&b, bytes));
        CK(hipMalloc(&d, bytes));
    } else if (layout.rfind("dskew:", 0) == 0) {
        // Round 4: operands packed in one heap, each next operand `gap` bytes past the end of the
        // previous one (the library's 2 MiB-aligned large allocations have gap 0): does moving
        // dest off the source's DRAM channel / bank phase change the copy's rate?
        const long gap = atol(layout.c_str() + 6);
        char *h;
        CK(hipMalloc(&h, 4l << 30));
        a = (f4 *) (h + (128l << 20));
        d = (f4 *) ((char *) a + bytes + gap);
        b = (f4 *) ((char *) d + bytes + gap);
    } else {
        // One heap like the library's symmetric heap: operands at `skew` bytes past 128 MiB and
        // packed back to back (heap = 256-B aligned first fit after the staging region).
        const long skew = layout == "heap256" ? 256 : 0;
        char *h;
        CK(hipMalloc(&h, 4l << 30));
        a = (f4 *) (h + (128l << 20) + skew);
        d = (f4 *) ((char *) a + bytes);
        b = (f4 *) ((char *) d + bytes);
    }
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    std::vector<Variant> vs;
    const std::string set = argc > 2 ? argv[2] : "all";
    if (set == "all") {
        vs.push_back({"oneshot ns1 U1 bs256 nt/nt", O<1, 1, 256, true, true>, 0, 1});
        vs.push_back({"oneshot ns1 U1 bs256 nt/plain", O<1, 1, 256, true, false>, 0, 1});
        vs.push_back({"oneshot ns1 U1 bs512 nt/nt", O<1, 1, 512, true, true>, 0, 1});
        vs.push_back({"oneshot ns1 U1 bs1024 nt/nt", O<1, 1, 1024, true, true>, 0, 1});
        vs.push_back({"oneshot ns1 U2 bs128 nt/nt", O<1, 2, 128, true, true>, 0, 1});
        vs.push_back({"oneshot ns1 U4 bs256 nt/nt", O<1, 4, 256, true, true>, 0, 1});
        vs.push_back({"oneshot ns1 U4 bs64 nt/nt", O<1, 4, 64, true, true>, 0, 1});
        vs.push_back({"oneshot ns2 U1 bs256 nt/nt", O<2, 1, 256, true, true>, 0, 2});
        vs.push_back({"oneshot ns2 U1 bs256 nt/plain", O<2, 1, 256, true, false>, 0, 2});
        vs.push_back({"oneshot ns2 U1 bs512 nt/nt", O<2, 1, 512, true, true>, 0, 2});
        vs.push_back({"oneshot ns2 U1 bs1024 nt/nt", O<2, 1, 1024, true, true>, 0, 2});
        vs.push_back({"oneshot ns2 U2 bs128 nt/nt", O<2, 2, 128, true, true>, 0, 2});
        vs.push_back({"oneshot ns2 U2 bs256 nt/nt", O<2, 2, 256, true, true>, 0, 2});
        vs.push_back({"writeonly U2 nt bs512 (traffic=1B)", WO<2, 512, true>, 0, 0});
        vs.push_back({"readonly U2 nt (traffic=1B)", RO<2, 256, true>, 0, 0});
        vs.push_back({"hipMemcpyAsync D2D", MC, 0, 1});
    }
    if (set == "aux") {
        vs.push_back({"oneshot ns1 U1 bs128 nt/nt", O<1, 1, 128, true, true>, 0, 1});
        vs.push_back({"aux ns1 bs64  ld nt / st sc0sc1", OA<1, 64, 2, 17>, 0, 1});
        vs.push_back({"aux ns1 bs128 ld nt / st sc0sc1", OA<1, 128, 2, 17>, 0, 1});
        vs.push_back({"aux ns1 bs256 ld nt / st sc0sc1", OA<1, 256, 2, 17>, 0, 1});
        vs.push_back({"aux ns1 bs128 ld nt / st sc1", OA<1, 128, 2, 16>, 0, 1});
        vs.push_back({"aux ns1 bs128 ld nt / st nt sc1", OA<1, 128, 2, 18>, 0, 1});
        vs.push_back({"aux ns1 bs128 ld nt / st nt", OA<1, 128, 2, 2>, 0, 1});
        vs.push_back({"aux ns1 bs128 ld nt / st nt sc0 sc1", OA<1, 128, 2, 19>, 0, 1});
        vs.push_back({"aux ns1 bs128 ld sc0sc1 / st sc0sc1", OA<1, 128, 17, 17>, 0, 1});
        vs.push_back({"aux ns1 bs128 ld nt sc0sc1 / st sc0sc1", OA<1, 128, 19, 17>, 0, 1});
        vs.push_back({"aux ns1 bs64  ld nt / st nt", OA<1, 64, 2, 2>, 0, 1});
        vs.push_back({"aux ns1 bs64  ld nt / st sc1", OA<1, 64, 2, 16>, 0, 1});
        vs.push_back({"oneshot ns2 U1 bs128 nt/nt", O<2, 1, 128, true, true>, 0, 2});
        vs.push_back({"aux ns2 bs64  ld nt / st sc0sc1", OA<2, 64, 2, 17>, 0, 2});
        vs.push_back({"aux ns2 bs128 ld nt / st sc0sc1", OA<2, 128, 2, 17>, 0, 2});
        vs.push_back({"aux ns2 bs128 ld nt / st nt", OA<2, 128, 2, 2>, 0, 2});
        vs.push_back({"aux ns2 bs64  ld nt / st nt", OA<2, 64, 2, 2>, 0, 2});
        vs.push_back({"aux ns2 bs256 ld nt / st sc0sc1", OA<2, 256, 2, 17>, 0, 2});
    }
    // Current product shape (fanin_kernel: one 16-B item per thread, 128-thread blocks) and the
    // round-1b candidates around it.
    if (set == "all" || set == "new") {
    vs.push_back({"oneshot ns1 U1 bs128 nt/nt", O<1, 1, 128, true, true>, 0, 1});
    vs.push_back({"oneshot ns1 U1 bs64 nt/nt", O<1, 1, 64, true, true>, 0, 1});
    vs.push_back({"oneshot ns1 U1 bs128 plain/nt", O<1, 1, 128, false, true>, 0, 1});
    vs.push_back({"oneshot ns1 U1 bs128 plain/plain", O<1, 1, 128, false, false>, 0, 1});
    vs.push_back({"xcd-remap ns1 bs128 nt/nt", OX<1, 128, true, true>, 0, 1});
    vs.push_back({"xcd-remap ns1 bs256 nt/nt", OX<1, 256, true, true>, 0, 1});
    vs.push_back({"wt-store ns1 bs128 nt/sc0sc1", OW<128>, 0, 1});
    vs.push_back({"lds-dma ns1 U1 bs128 nt/nt", LD<1, 128, true, true>, 0, 1});
    vs.push_back({"lds-dma ns1 U4 bs256 nt/nt", LD<4, 256, true, true>, 0, 1});
    vs.push_back({"oneshot ns2 U1 bs128 nt/nt", O<2, 1, 128, true, true>, 0, 2});
    vs.push_back({"xcd-remap ns2 bs128 nt/nt", OX<2, 128, true, true>, 0, 2});
    vs.push_back({"writeonly U1 plain (traffic=1B)", WO<1, 256, false>, 0, 0});
    vs.push_back({"writeonly U1 nt (traffic=1B)", WO<1, 256, true>, 0, 0});
    vs.push_back({"readonly U1 nt (traffic=1B)", RO<1, 256, true>, 0, 0});
    }
    if (set == "r2") {  // round 2: requests in flight per CU, and two DRAM regions per wave
        vs.push_back({"aux ns1 bs64 ld nt / st sc0sc1 (product)", OA<1, 64, 2, 17>, 0, 1});
        vs.push_back({"  + 4 KiB LDS (<=40 wg/CU)", OAL<1, 64, 2, 17, 4096>, 0, 1});
        vs.push_back({"  + 8 KiB LDS (<=20 wg/CU)", OAL<1, 64, 2, 17, 8192>, 0, 1});
        vs.push_back({"  + 16 KiB LDS (<=10 wg/CU)", OAL<1, 64, 2, 17, 16384>, 0, 1});
        vs.push_back({"  + 32 KiB LDS (<=5 wg/CU)", OAL<1, 64, 2, 17, 32768>, 0, 1});
        vs.push_back({"split halves bs64 nt / sc0sc1", SH<64>, 0, 1});
        vs.push_back({"split halves bs128 nt / sc0sc1", SH<128>, 0, 1});
        vs.push_back({"aux ns2 bs64 ld nt / st sc0sc1 (product a+b)", OA<2, 64, 2, 17>, 0, 2});
        vs.push_back({"  a+b + 8 KiB LDS", OAL<2, 64, 2, 17, 8192>, 0, 2});
        vs.push_back({"  a+b + 16 KiB LDS", OAL<2, 64, 2, 17, 16384>, 0, 2});
    }
    if (set == "prod") {  // round 4: the product shapes only (layout A/B)
        vs.push_back({"aux ns1 bs64 ld nt / st sc0sc1 (product copy)", OA<1, 64, 2, 17>, 0, 1});
        vs.push_back({"aux ns2 bs64 ld nt / st sc0sc1 (product a+b)", OA<2, 64, 2, 17>, 0, 2});
    }
    if (set == "r3") {  // round 3: store acknowledgements on the persistent kernel's critical path
        vs.push_back({"aux ns2 bs64 ld nt / st sc0sc1 (product a+b)", OA<2, 64, 2, 17>, 0, 2});
        vs.push_back({"persist a+b U2 bs256 g1024 plain", PW<2, 2, 256, false>, 1024, 2});
        vs.push_back({"persist a+b U2 bs256 g1024 PIPE", PW<2, 2, 256, true>, 1024, 2});
        vs.push_back({"persist a+b U4 bs256 g1024 plain", PW<2, 4, 256, false>, 1024, 2});
        vs.push_back({"persist a+b U4 bs256 g1024 PIPE", PW<2, 4, 256, true>, 1024, 2});
        vs.push_back({"persist a+b U2 bs256 g512 PIPE", PW<2, 2, 256, true>, 512, 2});
        vs.push_back({"persist a+b U2 bs256 g2048 PIPE", PW<2, 2, 256, true>, 2048, 2});
        vs.push_back({"aux ns1 bs64 ld nt / st sc0sc1 (product copy)", OA<1, 64, 2, 17>, 0, 1});
        vs.push_back({"persist copy U4 bs256 g1024 plain", PW<1, 4, 256, false>, 1024, 1});
        vs.push_back({"persist copy U4 bs256 g1024 PIPE", PW<1, 4, 256, true>, 1024, 1});
    }
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
