/* ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * Golden-vector generator: runs the reference host path's arithmetic backend, MPI_Allreduce
 * (src/runtime/runtime_mpi.cpp:802-812, datatype/op mapping :358-398), under MPICH 3.3.2
 * (/opt/conda, a third-party library in this image, not part of the reference) on
 *   (a) the reference testers' source patterns (oracle_pattern_source), and
 *   (b) seeded xorshift64* inputs (seed 0x15AE0001 + pe),
 * and writes, per rank, one record per case: {name[64], op, dtype, n, input bytes, output bytes}.
 * tests/golden/make_golden.py runs it with mpiexec -n {2,4,8} and packs the records into .npz.
 */
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static MPI_Datatype mpi_dt(int dt)
{
    switch (dt) {
        case OD_INT8: return MPI_INT8_T;
        case OD_INT16: return MPI_INT16_T;
        case OD_INT32: return MPI_INT32_T;
        case OD_INT64: return MPI_INT64_T;
        case OD_UINT8: return MPI_UINT8_T;
        case OD_UINT16: return MPI_UINT16_T;
        case OD_UINT32: return MPI_UINT32_T;
        case OD_UINT64: return MPI_UINT64_T;
        case OD_FLOAT: return MPI_FLOAT;
        default: return MPI_DOUBLE;
    }
}

static MPI_Op mpi_op(int op)
{
    static MPI_Op t[7];
    t[OR_AND] = MPI_BAND;
    t[OR_OR] = MPI_BOR;
    t[OR_XOR] = MPI_BXOR;
    t[OR_MAX] = MPI_MAX;
    t[OR_MIN] = MPI_MIN;
    t[OR_SUM] = MPI_SUM;
    t[OR_PROD] = MPI_PROD;
    return t[op];
}

static void record(FILE *f, const char *name, int op, int dt, size_t n, const void *in,
                   const void *out)
{
    char nm[64] = {0};
    strncpy(nm, name, 63);
    int32_t hdr[2] = {op, dt};
    uint64_t nn = n;
    fwrite(nm, 1, 64, f);
    fwrite(hdr, 4, 2, f);
    fwrite(&nn, 8, 1, f);
    const size_t es = oracle_dtype_size(dt);
    fwrite(in, es, n, f);
    fwrite(out, es, n, f);
}

static void run(FILE *f, const char *name, int op, int dt, size_t n, void *in)
{
    const size_t es = oracle_dtype_size(dt);
    void *out = calloc(n ? n : 1, es);
    MPI_Allreduce(in, out, (int) n, mpi_dt(dt), mpi_op(op), MPI_COMM_WORLD);
    record(f, name, op, dt, n, in, out);
    free(out);
}

int main(int argc, char **argv)
{
    MPI_Init(&argc, &argv);
    int rank, npes;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &npes);
    if (argc < 2) {
        if (!rank) fprintf(stderr, "usage: mpi_golden OUTDIR\n");
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    char path[4096];
    snprintf(path, sizeof path, "%s/golden_np%d_pe%d.bin", argv[1], npes, rank);
    FILE *f = fopen(path, "wb");
    if (!f) MPI_Abort(MPI_COMM_WORLD, 2);
    static const size_t sizes[] = {1, 3, 16, 129, 1000};
    static const char *opn[] = {"and", "or", "xor", "max", "min", "sum", "prod"};
    static const char *dtn[] = {"int8", "int16", "int32", "int64", "uint8",
                                "uint16", "uint32", "uint64", "float", "double"};
    char name[64];
    for (int op = 0; op < 7; ++op) {
        for (int dt = 0; dt < 10; ++dt) {
            if (!oracle_valid(op, dt)) continue;
            const size_t es = oracle_dtype_size(dt);
            const int fam = op == OR_AND ? PAT_AND : op == OR_OR ? PAT_OR : op == OR_XOR ? PAT_XOR : PAT_ARITH;
            for (size_t k = 0; k < sizeof sizes / sizeof sizes[0]; ++k) {
                const size_t n = sizes[k];
                void *in = calloc(n, es);
                oracle_pattern_source(fam, dt, rank, n, in);
                snprintf(name, sizeof name, "pat_%s_%s_%zu", opn[op], dtn[dt], n);
                run(f, name, op, dt, n, in);
                free(in);
            }
            const size_t n = 1001;
            void *in = calloc(n, es);
            const double lo = op == OR_PROD ? 0.5 : -1.0, hi = op == OR_PROD ? 2.0 : 1.0;
            oracle_fill_random(dt, 0x15AE0001ull + (uint64_t) rank, lo, hi, n, in);
            snprintf(name, sizeof name, "rnd_%s_%s_%zu", opn[op], dtn[dt], n);
            run(f, name, op, dt, n, in);
            free(in);
        }
    }
    fclose(f);
    MPI_Finalize();
    return 0;
}
