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
// member order rotated by workgroup (all links busy), local slot included.  Only remote LOADS.
template <int U>
__global__ __launch_bounds__(kBlock) void collect_kernel(CollectArgs a)
{
    using Item = std::conditional_t<U == 16, Vec<uint32_t>, std::conditional_t<U == 4, uint32_t, uint8_t>>;
    const int tid = threadIdx.x, b = blockIdx.x;
    const uint64_t G = gridDim.x;
    bool ok = pe_barrier<false>(a, kPhaseStart, b);
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
    ok = ok && pe_barrier<false>(a, kPhaseEnd, b);
    if (b == 0 && tid == 0 && a.ret) *a.ret = ok ? 0 : 1;
}

// Prefix sum.  Phase 1: member c owns chunk c; for each element it folds the members' values in
// team order and stores every member k's prefix into its own scratch row k (write-through).
// Phase 2 (after the mid barrier): each member pulls its row of every chunk into dest.
template <typename T>
__global__ __launch_bounds__(kBlock) void scan_kernel(ScanArgs a)
{
    const int tid = threadIdx.x, b = blockIdx.x;
    const uint64_t G = gridDim.x;
    const int p = a.p, me = a.me;
    const uint64_t ipc = a.items_per_chunk;
    bool ok = pe_barrier<false>(a, kPhaseStart, b);
    if (ok) {
        const uint64_t cs = min((uint64_t) me * ipc, a.nelems), ce = min(cs + ipc, a.nelems);
        for (uint64_t t0 = cs + (uint64_t) b * kTile; t0 < ce; t0 += G * kTile) {
            T acc[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) acc[u] = T(0);
            for (int k = 0; k < p; ++k) {
                T x[kUnroll];
                const char *base = uniform_ptr(a.src[k] + t0 * sizeof(T));
                if (k == me) {
#pragma unroll
                    for (int u = 0; u < kUnroll; ++u) {
                        const uint64_t e = (uint64_t) u * kBlock + tid;
                        if (t0 + e < ce) x[u] = ((const T *) base)[e];
                    }
                } else {
                    const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
#pragma unroll
                    for (int u = 0; u < kUnroll; ++u) {
                        const uint64_t e = (uint64_t) u * kBlock + tid;
                        if (t0 + e < ce) x[u] = cload<T>(r, (uint32_t) (e * sizeof(T)));
                    }
                }
                // Row k of the scratch holds member k's result for this chunk.
                const __amdgpu_buffer_rsrc_t wr =
                    make_rsrc(uniform_ptr(a.scratch[me] + ((uint64_t) k * ipc + (t0 - cs)) * sizeof(T)));
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const uint64_t e = (uint64_t) u * kBlock + tid;
                    const T incl = k == 0 ? x[u] : op1<T, ISHMEMI_OP_SUM>(acc[u], x[u]);  // keeps -0.0
                    if (t0 + e < ce) wt_store(wr, (uint32_t) (e * sizeof(T)), a.inclusive ? incl : acc[u]);
                    acc[u] = incl;
                }
            }
        }
    }
    ok = ok && pe_barrier<true>(a, kPhaseMid, b);
    if (ok) {
        for (int k = 0; k < p; ++k) {
            const int c = (me + b + k) % p;  // rotated over the members' scratch (links)
            const uint64_t cs = min((uint64_t) c * ipc, a.nelems), ce = min(cs + ipc, a.nelems);
            for (uint64_t t0 = cs + (uint64_t) b * kTile; t0 < ce; t0 += G * kTile) {
                const char *base = uniform_ptr(a.scratch[c] + ((uint64_t) me * ipc + (t0 - cs)) * sizeof(T));
                const __amdgpu_buffer_rsrc_t r = make_rsrc(base);
                T x[kUnroll];
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const uint64_t e = (uint64_t) u * kBlock + tid;
                    if (t0 + e < ce) x[u] = cload<T>(r, (uint32_t) (e * sizeof(T)));
                }
                T *dp = (T *) (a.dst + t0 * sizeof(T));
#pragma unroll
                for (int u = 0; u < kUnroll; ++u) {
                    const uint64_t e = (uint64_t) u * kBlock + tid;
                    if (t0 + e < ce) dp[e] = x[u];
                }
            }
        }
    }
    ok = ok && pe_barrier<false>(a, kPhaseEnd, b);
    if (b == 0 && tid == 0 && a.ret) *a.ret = ok ? 0 : 1;
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
    if (a.unit == 4) return launch_res(collect_kernel<4>, a, grid, s);
    return launch_res(collect_kernel<1>, a, grid, s);
}

hipError_t launch_scan(int dt, const ScanArgs &a, int grid, hipStream_t s)
{
    switch (dt) {  // sum wraps on the unsigned type of the same width (two's complement)
        case ISHMEMI_DT_INT8: case ISHMEMI_DT_UINT8: return launch_res(scan_kernel<uint8_t>, a, grid, s);
        case ISHMEMI_DT_INT16: case ISHMEMI_DT_UINT16: return launch_res(scan_kernel<uint16_t>, a, grid, s);
        case ISHMEMI_DT_INT32: case ISHMEMI_DT_UINT32: return launch_res(scan_kernel<uint32_t>, a, grid, s);
        case ISHMEMI_DT_INT64: case ISHMEMI_DT_UINT64: return launch_res(scan_kernel<uint64_t>, a, grid, s);
        case ISHMEMI_DT_FLOAT: return launch_res(scan_kernel<float>, a, grid, s);
        case ISHMEMI_DT_DOUBLE: return launch_res(scan_kernel<double>, a, grid, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace ishmemi
