// HIP version of the reference's examples/6_team_split_strided.cpp (itself from the OpenSHMEM 1.5
// team_split_strided example): a team of the even PEs, a sum reduce and a broadcast on it called
// from INSIDE a kernel by one work-item, a host broadcast, then a copy of the world team and a
// device-side team_sync + reduce + barrier_all on it.  Every ishmem call is the reference's, with
// the reference's arguments; only the SYCL parts differ (q.submit/single_task -> a one-thread
// kernel, sycl::malloc_host -> hipHostMalloc, captures -> kernel arguments).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <iostream>

#include <ishmem.h>
#include <ishmemx.h>

__global__ void even_team_kernel(ishmem_team_t even_team, int t_pe, int t_size, int *dev_buf, int *dev_sum,
                                 int *errors)
{
    *dev_buf = t_pe;
    if (even_team != ISHMEM_TEAM_INVALID) {
        ishmem_int_sum_reduce(even_team, dev_sum, dev_buf, 1);
        if (*dev_sum != (t_size * (t_size - 1) / 2)) {
            *errors += 1;
            ishmemx_print("Wrong reduce on even_team (device)\n", ishmemx_print_msg_type_t::ERROR);
        }
        ishmem_int_broadcast(even_team, dev_buf, dev_sum, 1, 0);
        if (*dev_buf != (t_size * (t_size - 1) / 2)) {
            *errors += 1;
            ishmemx_print("Wrong broadcast on even_team (device)\n", ishmemx_print_msg_type_t::ERROR);
        }
        *dev_sum = 123;
    }
}

__global__ void check_host_broadcast(int *dev_buf, int *errors)
{
    if (*dev_buf != 123) {
        *errors += 1;
        ishmemx_print("Wrong broadcast on even_team (host)\n", ishmemx_print_msg_type_t::ERROR);
    }
}

__global__ void world_copy_kernel(ishmem_team_t world_team_copy, int rank, int npes, int *dev_buf, int *dev_sum,
                                  int *errors)
{
    *dev_sum = 0;
    *dev_buf = rank;
    const int my_team_pe = ishmem_team_my_pe(world_team_copy);
    if (my_team_pe != rank) *errors += 1;
    ishmem_team_sync(ISHMEM_TEAM_WORLD);
    ishmem_int_sum_reduce(world_team_copy, dev_sum, dev_buf, 1);
    ishmem_barrier_all();
    if (*dev_sum != (npes * (npes - 1) / 2)) {
        *errors += 1;
        ishmemx_print("Wrong reduce on world_team (device)\n", ishmemx_print_msg_type_t::ERROR);
    }
}

int main()
{
    ishmem_team_t even_team;
    ishmem_team_config_t *config = NULL;

    ishmem_init();
    const int rank = ishmem_my_pe();
    const int npes = ishmem_n_pes();
    if (npes < 2) {
        fprintf(stderr, "ERR - Requires at least 2 PEs\n");
        ishmem_finalize();
        return 0;
    }

    int ret = ishmem_team_split_strided(ISHMEM_TEAM_WORLD, 0, 2, (npes + 1) / 2, config, 0, &even_team);
    if (ret != 0) {
        ishmem_finalize();
        return EXIT_FAILURE;
    }
    const int t_size = ishmem_team_n_pes(even_team);
    const int t_pe = ishmem_team_my_pe(even_team);

    int *errors = nullptr;
    if (hipHostMalloc((void **) &errors, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
        return EXIT_FAILURE;
    *errors = 0;

    if (even_team != ISHMEM_TEAM_INVALID) {
        if ((rank % 2 != 0) || (rank / 2 != t_pe) || ((npes + 1) / 2 != t_size)) {
            printf("[%d] Error on even_team\n", rank);
            return EXIT_FAILURE;
        }
    } else if ((rank % 2 == 0) || (t_pe != -1) || (t_size != -1)) {
        printf("[%d] Error on non even_team\n", rank);
        return EXIT_FAILURE;
    }

    int *dev_buf = (int *) ishmem_malloc(sizeof(int));
    int *dev_sum = (int *) ishmem_calloc(1, sizeof(int));

    hipLaunchKernelGGL(even_team_kernel, dim3(1), dim3(1), 0, 0, even_team, t_pe, t_size, dev_buf, dev_sum, errors);
    (void) hipDeviceSynchronize();

    if (even_team != ISHMEM_TEAM_INVALID) {  // host broadcast on device memory
        ishmem_int_broadcast(even_team, dev_buf, dev_sum, 1, 0);
        hipLaunchKernelGGL(check_host_broadcast, dim3(1), dim3(1), 0, 0, dev_buf, errors);
        (void) hipDeviceSynchronize();
    }

    ishmem_barrier_all();

    ishmem_team_t world_team_copy;
    ret = ishmem_team_split_strided(ISHMEM_TEAM_WORLD, 0, 1, npes, config, 0, &world_team_copy);
    if (ret != 0) {
        ishmem_finalize();
        return EXIT_FAILURE;
    }
    ishmem_team_sync(world_team_copy);

    hipLaunchKernelGGL(world_copy_kernel, dim3(1), dim3(1), 0, 0, world_team_copy, rank, npes, dev_buf, dev_sum,
                       errors);
    (void) hipDeviceSynchronize();

    if (*errors == 0) std::cout << "PE#" << rank << " SUCCESS - verified" << std::endl;
    else std::cout << "PE#" << rank << " FAILURE - Error count: " << *errors << std::endl;
    const int nerr = *errors;

    ishmem_team_destroy(even_team);
    ishmem_team_destroy(world_team_copy);
    ishmem_free(dev_buf);
    ishmem_free(dev_sum);
    (void) hipHostFree(errors);
    ishmem_finalize();
    return nerr ? EXIT_FAILURE : 0;
}
