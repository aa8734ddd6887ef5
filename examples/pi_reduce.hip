// HIP version of the reference's examples/5_pi_reduce.cpp: Monte-Carlo estimate of pi where every
// PE counts the points of its own stream that fall inside the quarter circle, then the PEs add up
// their counts with ONE host call, unchanged from the reference:
//     ishmem_size_sum_reduce(inside, inside, 1)        (in place, symmetric heap, 1 element)
// Only the SYCL parts differ: the sycl::reduction kernel becomes a HIP kernel with an atomic add,
// oneapi::dpl::minstd_rand becomes the same Lehmer generator (x <- 48271 x mod 2^31-1) written out,
// and q.memcpy becomes hipMemcpy.  The program also checks the reduced count against the counts
// every PE's stream gives when replayed on the host (exact), and prints SUCCESS / FAILURE.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>

#include <ishmem.h>
#include <ishmemx.h>

constexpr size_t npoints = 100000;

// Lehmer / minstd: state in [1, 2^31 - 2]; stream `seed`, point `k` starts from a skipped-ahead
// state (seed mixed with the point index), two draws per point.
__host__ __device__ inline uint32_t minstd_next(uint32_t x) { return (uint32_t) ((uint64_t) x * 48271u % 2147483647u); }
__host__ __device__ inline double unit(uint32_t x) { return (double) (x - 1) / 2147483646.0; }
__host__ __device__ inline bool inside_circle(uint32_t seed, uint64_t k)
{
    uint32_t s = (uint32_t) ((seed * 2654435761u + k * 40503u) % 2147483646u) + 1u;
    s = minstd_next(s);
    const double x = unit(s);
    s = minstd_next(s);
    const double y = unit(s);
    return x * x + y * y < 1.0;
}

__global__ void count_points(size_t *inside, uint32_t seed, size_t n)
{
    const size_t k = blockIdx.x * (size_t) blockDim.x + threadIdx.x;
    if (k < n && inside_circle(seed, k)) atomicAdd((unsigned long long *) inside, 1ull);
}

int main()
{
    ishmem_init();
    const int my_pe = ishmem_my_pe();
    const int npes = ishmem_n_pes();

    const uint32_t seed = (uint32_t) my_pe + 1;  // every PE its own stream
    size_t *inside = (size_t *) ishmem_calloc(1, sizeof(size_t));

    hipLaunchKernelGGL(count_points, dim3((npoints + 255) / 256), dim3(256), 0, 0, inside, seed, npoints);
    if (hipDeviceSynchronize() != hipSuccess) return EXIT_FAILURE;

    if (ishmem_size_sum_reduce(inside, inside, 1)) {
        std::cerr << "ishmem reduce failed, exiting" << std::endl;
        ishmem_free(inside);
        return EXIT_FAILURE;
    }

    size_t total = 0;
    (void) hipMemcpy(&total, inside, sizeof(size_t), hipMemcpyDeviceToHost);

    size_t want = 0;  // the same streams replayed on the host
    for (int pe = 0; pe < npes; ++pe)
        for (size_t k = 0; k < npoints; ++k) want += inside_circle((uint32_t) pe + 1, k);

    if (my_pe == 0) {
        const double pi_appx = 4.0 * (double) total / (double) (npoints * (size_t) npes);
        std::cout << "Value of pi from this experiment = " << pi_appx << std::endl;
        std::cout << "Relative error (%) = " << (pi_appx - M_PI) * 100 / M_PI << " %" << std::endl;
    }
    const bool ok = total == want && std::fabs(4.0 * (double) total / (double) (npoints * (size_t) npes) - M_PI) < 0.05;
    std::cout << "PE#" << my_pe << (ok ? " SUCCESS" : " FAILURE") << " inside " << total << " expected " << want
              << " npes " << npes << std::endl;

    ishmem_free(inside);
    ishmem_finalize();
    return ok ? EXIT_SUCCESS : EXIT_FAILURE;
}
