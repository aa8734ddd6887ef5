// HIP version of the parts of the reference's examples/3_library_apis.cpp that belong to this
// library (the reduction path and the calls around it): device-side queries, barriers,
// broadcast and sum reduction, each called from inside a kernel both by the group leader alone
// and by the whole work-group, exactly as the reference calls them:
//     if (grp.leader()) ishmem_barrier_all();          ishmemx_barrier_all_work_group(grp);
//     if (grp.leader()) ishmem_broadcastmem(...);      ishmemx_broadcastmem_work_group(..., grp);
//     if (grp.leader()) ishmem_int_sum_reduce(...);    ishmemx_int_sum_reduce_work_group(..., grp);
// SYCL's nd_item / group become HIP's cooperative groups (grp = this_thread_block(),
// grp.leader() -> grp.thread_rank() == 0, sycl::group_barrier -> grp.sync()).  The reference's
// put / get / atomic / wait_until calls are RMA and AMO, which this library does not provide
// (out of scope), so they are not part of this program.
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <iostream>

#include <ishmem.h>
#include <ishmemx.h>

namespace cg = cooperative_groups;

constexpr int array_size = 10;
constexpr int chunk_size = 2;

__global__ void init_kernel(int my_pe, int *src, int *src_bcast, int *reduce_src)
{
    reduce_src[0] = my_pe;
    for (int i = 0; i < array_size; i++) src[i] = (my_pe + 1) * (1 << i);
    if (my_pe == 0) src_bcast[0] = 42;
}

__global__ void test_kernel(int *dst_bcast, const int *src_bcast, int *dst_sum, const int *reduce_src, int *seen)
{
    const int my_dev_pe = ishmem_my_pe();
    const int my_dev_npes = ishmem_n_pes();
    auto grp = cg::this_thread_block();
    if (grp.thread_rank() == 0) {
        seen[0] = my_dev_pe;
        seen[1] = my_dev_npes;
    }

    grp.sync();
    if (grp.thread_rank() == 0) ishmem_barrier_all();
    grp.sync();
    ishmemx_barrier_all_work_group(grp);

    if (grp.thread_rank() == 0) ishmem_broadcastmem(dst_bcast, src_bcast, sizeof(int), 0);
    ishmemx_broadcastmem_work_group(dst_bcast, src_bcast, sizeof(int), 0, grp);

    ishmemx_barrier_all_work_group(grp);

    if (grp.thread_rank() == 0) ishmem_int_sum_reduce(dst_sum, reduce_src, 1);
    ishmemx_int_sum_reduce_work_group(dst_sum, reduce_src, 1, grp);
}

__global__ void verify_kernel(int my_pe, int npes, const int *dst_bcast, const int *dst_sum, const int *seen,
                              int *errors)
{
    if (*dst_bcast != 42) *errors += 1;
    if (*dst_sum != npes * (npes - 1) / 2) *errors += 1;
    if (seen[0] != my_pe || seen[1] != npes) *errors += 1;
}

int main()
{
    int dev = 0;
    hipDeviceProp_t prop;
    (void) hipGetDevice(&dev);
    (void) hipGetDeviceProperties(&prop, dev);
    std::cout << "Selected device: " << prop.name << std::endl;

    ishmem_init();
    const int my_pe = ishmem_my_pe();
    const int npes = ishmem_n_pes();
    std::cout << "Hello from PE " << my_pe << std::endl;
    const int num_threads = array_size / chunk_size;

    int *src = (int *) ishmem_malloc(array_size * sizeof(int));
    int *dst_sum = (int *) ishmem_calloc(1, sizeof(int));
    int *src_bcast = (int *) ishmem_malloc(sizeof(int));
    int *dst_bcast = (int *) ishmem_malloc(sizeof(int));
    int *reduce_src = (int *) ishmem_calloc(1, sizeof(int));
    int *seen = (int *) ishmem_calloc(2, sizeof(int));

    int *errors = nullptr;  // host memory the kernels can write (sycl::malloc_host)
    if (hipHostMalloc((void **) &errors, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return 1;
    *errors = 0;

    hipLaunchKernelGGL(init_kernel, dim3(1), dim3(1), 0, 0, my_pe, src, src_bcast, reduce_src);
    (void) hipDeviceSynchronize();
    ishmem_barrier_all();

    hipLaunchKernelGGL(test_kernel, dim3(1), dim3(num_threads), 0, 0, dst_bcast, src_bcast, dst_sum, reduce_src,
                       seen);
    (void) hipDeviceSynchronize();
    ishmem_barrier_all();

    hipLaunchKernelGGL(verify_kernel, dim3(1), dim3(1), 0, 0, my_pe, npes, dst_bcast, dst_sum, seen, errors);
    (void) hipDeviceSynchronize();

    if (*errors == 0) std::cout << "PE#" << my_pe << " SUCCESS - verified query/barrier/broadcast/reduce" << std::endl;
    else std::cout << "PE#" << my_pe << " FAILURE - Error count: " << *errors << std::endl;
    const int nerr = *errors;

    ishmem_free(seen);
    ishmem_free(reduce_src);
    ishmem_free(dst_bcast);
    ishmem_free(src_bcast);
    ishmem_free(dst_sum);
    ishmem_free(src);
    (void) hipHostFree(errors);
    ishmem_finalize();
    return nerr ? 1 : 0;
}
