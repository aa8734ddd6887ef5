/* ORACLE — TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).  The reference's host path for
 * a reduce on symmetric-heap device buffers, with the reference's OWN runtime call on the host
 * side: ishmemi_generic_op_reduce (src/collectives/reduce_impl.h:186-228) walks the array in
 * ISHMEM_REDUCE_BUFFER_SIZE = 64 KiB chunks (src/collectives.h:10); each chunk is a synchronous
 * device-to-host copy into a host bounce buffer (ishmemi_copy -> memory.cpp:310-321), one runtime
 * all-reduce — MPI_Allreduce with the op / datatype mapping of runtime_mpi.cpp:358-398, 802-812 —
 * and a synchronous host-to-device copy back.  Run under MPICH's mpiexec, one process per PE;
 * float32 sum.  Prints (rank 0) one line: "<seconds> <bytes per PE>" for the slowest rank.
 *
 *   mpiexec -n P ./mpi_bounce NFLOATS [DEVICE_MOD]
 *
 * Every rank uses HIP device (rank % DEVICE_MOD) (default: the number of visible devices). */
#include <hip/hip_runtime_api.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHUNK_BYTES (64 * 1024) /* src/collectives.h:10 */

static int check(hipError_t e, const char *what)
{
    if (e != hipSuccess) {
        fprintf(stderr, "mpi_bounce: %s failed: %s\n", what, hipGetErrorString(e));
        return 1;
    }
    return 0;
}

int main(int argc, char **argv)
{
    MPI_Init(&argc, &argv);
    int rank = 0, np = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &np);
    const size_t n = argc > 1 ? (size_t) strtoull(argv[1], NULL, 10) : (size_t) 1 << 24;
    int ndev = 1;
    if (check(hipGetDeviceCount(&ndev), "hipGetDeviceCount")) MPI_Abort(MPI_COMM_WORLD, 2);
    const int mod = argc > 2 ? atoi(argv[2]) : ndev;
    if (check(hipSetDevice(rank % (mod > 0 ? mod : 1) % ndev), "hipSetDevice")) MPI_Abort(MPI_COMM_WORLD, 2);
    float *src = NULL, *dst = NULL;
    float *host = (float *) malloc(n * sizeof(float));
    float *bounce = (float *) malloc(CHUNK_BYTES);
    if (!host || !bounce) MPI_Abort(MPI_COMM_WORLD, 2);
    if (check(hipMalloc((void **) &src, n * sizeof(float)), "hipMalloc") ||
        check(hipMalloc((void **) &dst, n * sizeof(float)), "hipMalloc"))
        MPI_Abort(MPI_COMM_WORLD, 2);
    for (size_t i = 0; i < n; ++i) host[i] = (float) (i % 1024) + (float) rank;
    if (check(hipMemcpy(src, host, n * sizeof(float), hipMemcpyHostToDevice), "upload")) MPI_Abort(MPI_COMM_WORLD, 2);
    const size_t chunk = CHUNK_BYTES / sizeof(float);
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    int failed = 0;
    for (size_t off = 0; off < n && !failed; off += chunk) {
        const size_t m = n - off < chunk ? n - off : chunk;
        failed |= check(hipMemcpy(bounce, src + off, m * sizeof(float), hipMemcpyDeviceToHost), "D2H");
        failed |= MPI_Allreduce(MPI_IN_PLACE, bounce, (int) m, MPI_FLOAT, MPI_SUM, MPI_COMM_WORLD) != MPI_SUCCESS;
        failed |= check(hipMemcpy(dst + off, bounce, m * sizeof(float), hipMemcpyHostToDevice), "H2D");
    }
    double t = MPI_Wtime() - t0, tmax = 0.0;
    MPI_Allreduce(&t, &tmax, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
    /* Check the result (exact: small integers) on every rank. */
    size_t bad = 0;
    if (!failed && hipMemcpy(host, dst, n * sizeof(float), hipMemcpyDeviceToHost) == hipSuccess) {
        for (size_t i = 0; i < n; ++i)
            bad += host[i] != (float) (i % 1024) * (float) np + (float) (np * (np - 1) / 2);
    } else {
        bad = 1;
    }
    unsigned long long bad_all = 0, bad_me = (unsigned long long) bad;
    MPI_Allreduce(&bad_me, &bad_all, 1, MPI_UNSIGNED_LONG_LONG, MPI_SUM, MPI_COMM_WORLD);
    if (rank == 0) printf("%.6f %zu %llu\n", tmax, n * sizeof(float), bad_all);
    (void) hipFree(src);
    (void) hipFree(dst);
    free(host);
    free(bounce);
    MPI_Finalize();
    return bad_all ? 1 : 0;
}
