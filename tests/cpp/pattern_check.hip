// Test / bench infrastructure (not product): the rotating-winner input pattern of
// ishmem_amd/selfcheck.py generated and checked ON THE DEVICE, so BASELINE configs[4] (up to
// 4 GiB per PE, 8 PEs) can be compared in every word on every PE, as the reference's tester does
// (test/include/ishmem_tester.h:1178-1281), instead of in host-side windows.
//
//   x_pe[i] = 1 + h(i) + 1024 * ((i + pe) mod p),  h(i) = mix32(lo32(i) ^ k(hi(i))) >> 22
//
// with k(0) = 0, k(hi) = mix32((hi * 0x9E3779B9 + 0x632BE5AB) mod 2^32) — selfcheck._hash_lo —
// and the expected team-order fold over PEs 0..p-1 per op (selfcheck._expected_block): sum and
// min / max in closed form, prod folded in team order in the array's own type (integers wrap).
// The same functions are compiled for the host and exported (pc_host_*), and a CPU test pins
// them to selfcheck's numpy (tests/test_patterns.py), which is itself pinned to an explicit fold.
//
// Build (tests/test_gpu_cpp.py build_pattern_check, __graft_entry__.build()):
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -fPIC -shared
//         tests/cpp/pattern_check.hip -o build/libpattern_check.so
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <type_traits>

namespace {

// ishmem_capi.h dtype / op codes (the subset the large-size checks use).
enum { DT_INT32 = 2, DT_INT64 = 3, DT_UINT32 = 6, DT_UINT64 = 7, DT_FLOAT = 8, DT_DOUBLE = 9 };
enum { OP_MAX = 3, OP_MIN = 4, OP_SUM = 5, OP_PROD = 6 };

__host__ __device__ inline uint32_t mix32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}

__host__ __device__ inline uint32_t hash10(uint64_t i)
{
    const uint32_t hi = (uint32_t) (i >> 32);
    uint32_t key = (uint32_t) i;
    if (hi) key ^= mix32((uint32_t) ((uint64_t) hi * 0x9E3779B9ull + 0x632BE5ABull));
    return mix32(key) >> 22;
}

__host__ __device__ inline uint32_t value_u32(uint64_t i, int pe, int p)
{
    return 1u + hash10(i) + 1024u * (uint32_t) ((i + (uint64_t) pe) % (uint64_t) p);
}

template <typename T>
__host__ __device__ inline T expected(int op, int p, uint64_t i)
{
    const uint32_t h = hash10(i);
    if (op == OP_SUM) return (T) ((uint64_t) p * (h + 1u) + 1024ull * (uint64_t) p * (uint64_t) (p - 1) / 2);
    if (op == OP_MIN) return (T) (h + 1u);
    if (op == OP_MAX) return (T) (h + 1u + 1024u * (uint32_t) (p - 1));
    // prod, team order 0..p-1 in T (unsigned wrap for the integer types)
    if constexpr (std::is_integral_v<T> && sizeof(T) == 4) {
        uint32_t acc = 1;
        for (int pe = 0; pe < p; ++pe) acc *= value_u32(i, pe, p);
        T r;
        memcpy(&r, &acc, 4);
        return r;
    } else if constexpr (std::is_integral_v<T> && sizeof(T) == 8) {
        uint64_t acc = 1;
        for (int pe = 0; pe < p; ++pe) acc *= (uint64_t) value_u32(i, pe, p);
        T r;
        memcpy(&r, &acc, 8);
        return r;
    } else {
        T acc = (T) value_u32(i, 0, p);
        for (int pe = 1; pe < p; ++pe) acc = acc * (T) value_u32(i, pe, p);
        return acc;
    }
}

template <typename T>
__global__ void fill_kernel(T *dst, int pe, int p, uint64_t lo, uint64_t n)
{
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    for (uint64_t t = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride)
        dst[t] = (T) value_u32(lo + t, pe, p);
}

// Bytes of dst[0..n) that differ from the expected fold at indices lo..lo+n.
template <typename T>
__global__ void count_kernel(const T *dst, int op, int p, uint64_t lo, uint64_t n, unsigned long long *bad)
{
    const uint64_t stride = (uint64_t) gridDim.x * blockDim.x;
    unsigned long long mine = 0;
    for (uint64_t t = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x; t < n; t += stride) {
        const T want = expected<T>(op, p, lo + t);
        const T got = dst[t];
        unsigned char a[sizeof(T)], b[sizeof(T)];
        memcpy(a, &want, sizeof(T));
        memcpy(b, &got, sizeof(T));
#pragma unroll
        for (int k = 0; k < (int) sizeof(T); ++k) mine += a[k] != b[k];
    }
    if (mine) atomicAdd(bad, mine);
}

unsigned long long *g_counter = nullptr;

template <typename F>
int by_dtype(int dtype, F &&f)
{
    switch (dtype) {
        case DT_INT32: return f((int32_t *) nullptr);
        case DT_UINT32: return f((uint32_t *) nullptr);
        case DT_INT64: return f((int64_t *) nullptr);
        case DT_UINT64: return f((uint64_t *) nullptr);
        case DT_FLOAT: return f((float *) nullptr);
        case DT_DOUBLE: return f((double *) nullptr);
        default: return -1;
    }
}

unsigned grid_for(uint64_t n)
{
    const uint64_t g = (n + 255) / 256;
    return (unsigned) (g < 8192 ? (g ? g : 1) : 8192);
}

}  // namespace

extern "C" {

// dst[0..n) = x_pe[lo .. lo + n) as `dtype`; 0 on success.
int pc_fill(void *dst, int dtype, int pe, int p, unsigned long long lo, unsigned long long n)
{
    if (p < 1 || pe < 0 || pe >= p) return -1;
    const int r = by_dtype(dtype, [&](auto *tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        if (n) hipLaunchKernelGGL(fill_kernel<T>, dim3(grid_for(n)), dim3(256), 0, 0, (T *) dst, pe, p, (uint64_t) lo, (uint64_t) n);
        return 0;
    });
    if (r) return r;
    return hipDeviceSynchronize() == hipSuccess && hipGetLastError() == hipSuccess ? 0 : -2;
}

// Bytes of dst[0..n) (device) that differ from the team-order fold of x_0..x_{p-1} at
// [lo, lo + n); negative on error.
long long pc_count_wrong(const void *dst, int op, int dtype, int p, unsigned long long lo, unsigned long long n)
{
    if (p < 1 || (op != OP_MAX && op != OP_MIN && op != OP_SUM && op != OP_PROD)) return -1;
    if (!g_counter && hipMalloc((void **) &g_counter, sizeof(unsigned long long)) != hipSuccess) return -2;
    if (hipMemset(g_counter, 0, sizeof(unsigned long long)) != hipSuccess) return -2;
    const int r = by_dtype(dtype, [&](auto *tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        if (n) hipLaunchKernelGGL(count_kernel<T>, dim3(grid_for(n)), dim3(256), 0, 0, (const T *) dst, op, p, (uint64_t) lo, (uint64_t) n, g_counter);
        return 0;
    });
    if (r) return r;
    unsigned long long bad = 0;
    if (hipMemcpy(&bad, g_counter, sizeof(bad), hipMemcpyDeviceToHost) != hipSuccess || hipGetLastError() != hipSuccess)
        return -2;
    return (long long) bad;
}

// Host twins of the device functions (CPU test pins them to selfcheck.py's numpy).
int pc_host_pattern(void *out, int dtype, int pe, int p, unsigned long long lo, unsigned long long n)
{
    if (p < 1 || pe < 0 || pe >= p) return -1;
    return by_dtype(dtype, [&](auto *tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        for (uint64_t t = 0; t < n; ++t) ((T *) out)[t] = (T) value_u32(lo + t, pe, p);
        return 0;
    });
}

int pc_host_expected(void *out, int op, int dtype, int p, unsigned long long lo, unsigned long long n)
{
    if (p < 1 || (op != OP_MAX && op != OP_MIN && op != OP_SUM && op != OP_PROD)) return -1;
    return by_dtype(dtype, [&](auto *tag) {
        using T = std::remove_pointer_t<decltype(tag)>;
        for (uint64_t t = 0; t < n; ++t) ((T *) out)[t] = expected<T>(op, p, lo + t);
        return 0;
    });
}

}  // extern "C"
