// Dev tool (round 5, not product): can a team barrier be built from stream memory operations
// (hipStreamWriteValue32 / hipStreamWaitValue32: the command processor waits, no workgroup is
// held) and what does one cost against the one-workgroup barrier kernel?  One process, two
// streams standing in for two PEs; for each memory kind of the flag word:
//   accepts  - whether HIP accepts a wait / write on that memory at all;
//   self     - write then wait on the same stream (a wait that is already satisfied): per pair;
//   pingpong - streams A and B each write their own word and wait for the other's, n rounds:
//              per round = one two-party barrier;
//   kernel   - the same ping-pong with a one-workgroup kernel per barrier (the product shape:
//              store own flag, spin on the peer's).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/streamop_probe.hip -o tools/bin/streamop_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            printf("%s failed: %s\n", #x, hipGetErrorString(e_));                                  \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

__global__ void kbarrier(uint32_t *mine, const uint32_t *theirs, uint32_t ep)
{
    if (threadIdx.x == 0) {
        __hip_atomic_store(mine, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while ((int32_t) (__hip_atomic_load(theirs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - ep) < 0)
            if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) break;  // 5 s bound
    }
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 2000;
    int attr = 0;
    CK(hipDeviceGetAttribute(&attr, hipDeviceAttributeCanUseStreamWaitValue, 0));
    printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", attr);
    hipStream_t A, B;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&B, hipStreamNonBlocking));
    struct Kind {
        const char *name;
        unsigned flags;  // hipExtMallocWithFlags flags, ~0u = hipMalloc
    } kinds[] = {{"hipMalloc", ~0u},
                 {"uncached", hipDeviceMallocUncached},
                 {"fine-grained", hipDeviceMallocFinegrained},
                 {"signal", hipMallocSignalMemory}};
    for (const Kind &k : kinds) {
        uint32_t *w = nullptr;
        const size_t bytes = k.flags == hipMallocSignalMemory ? 8 : 256;
        hipError_t e = k.flags == ~0u ? hipMalloc((void **) &w, bytes) : hipExtMallocWithFlags((void **) &w, bytes, k.flags);
        if (e != hipSuccess) {
            printf("%-13s alloc failed: %s\n", k.name, hipGetErrorString(e));
            (void) hipGetLastError();
            continue;
        }
        CK(hipMemset(w, 0, bytes));
        CK(hipDeviceSynchronize());
        uint32_t *wa = w, *wb = k.flags == hipMallocSignalMemory ? nullptr : w + 16;
        // accepts
        hipError_t ew = hipStreamWriteValue32(A, wa, 1, 0);
        (void) hipGetLastError();
        hipError_t ev = hipStreamWaitValue32(A, wa, 1, hipStreamWaitValueGte, 0xFFFFFFFFu);
        (void) hipGetLastError();
        hipError_t es = hipStreamSynchronize(A);
        printf("%-13s write %s, wait %s, sync %s\n", k.name, hipGetErrorString(ew), hipGetErrorString(ev),
               hipGetErrorString(es));
        if (ew != hipSuccess || ev != hipSuccess || es != hipSuccess) {
            (void) hipFree(w);
            continue;
        }
        // self: write + satisfied wait on one stream
        uint32_t ep = 1;
        double t0 = now_us();
        for (int r = 0; r < rounds; ++r) {
            ++ep;
            CK(hipStreamWriteValue32(A, wa, ep, 0));
            CK(hipStreamWaitValue32(A, wa, ep, hipStreamWaitValueGte, 0xFFFFFFFFu));
        }
        CK(hipStreamSynchronize(A));
        const double self_us = (now_us() - t0) / rounds;
        double pp_us = -1, kk_us = -1;
        if (wb) {
            CK(hipMemset(w, 0, bytes));
            CK(hipDeviceSynchronize());
            t0 = now_us();
            for (uint32_t r = 1; r <= (uint32_t) rounds; ++r) {
                CK(hipStreamWriteValue32(A, wa, r, 0));
                CK(hipStreamWriteValue32(B, wb, r, 0));
                CK(hipStreamWaitValue32(A, wb, r, hipStreamWaitValueGte, 0xFFFFFFFFu));
                CK(hipStreamWaitValue32(B, wa, r, hipStreamWaitValueGte, 0xFFFFFFFFu));
            }
            CK(hipStreamSynchronize(A));
            CK(hipStreamSynchronize(B));
            pp_us = (now_us() - t0) / rounds;
            CK(hipMemset(w, 0, bytes));
            CK(hipDeviceSynchronize());
            t0 = now_us();
            for (uint32_t r = 1; r <= (uint32_t) rounds; ++r) {
                hipLaunchKernelGGL(kbarrier, dim3(1), dim3(64), 0, A, wa, wb, r);
                hipLaunchKernelGGL(kbarrier, dim3(1), dim3(64), 0, B, wb, wa, r);
            }
            CK(hipStreamSynchronize(A));
            CK(hipStreamSynchronize(B));
            kk_us = (now_us() - t0) / rounds;
        }
        // hipStreamBatchMemOp: the write and the wait of one side as ONE call (one submission).
        double bb_us = -1, bs_us = -1;
        if (wb) {
            CK(hipMemset(w, 0, bytes));
            CK(hipDeviceSynchronize());
            hipError_t eb = hipSuccess;
            t0 = now_us();
            for (uint32_t r = 1; r <= (uint32_t) rounds && eb == hipSuccess; ++r) {
                hipStreamBatchMemOpParams pa[2], pb[2];
                memset(pa, 0, sizeof(pa));
                memset(pb, 0, sizeof(pb));
                pa[0].writeValue.operation = hipStreamMemOpWriteValue32;
                pa[0].writeValue.address = (hipDeviceptr_t) wa;
                pa[0].writeValue.value = r;
                pa[1].waitValue.operation = hipStreamMemOpWaitValue32;
                pa[1].waitValue.address = (hipDeviceptr_t) wb;
                pa[1].waitValue.value = r;
                pa[1].waitValue.flags = hipStreamWaitValueGte;
                pb[0] = pa[0];
                pb[0].writeValue.address = (hipDeviceptr_t) wb;
                pb[1] = pa[1];
                pb[1].waitValue.address = (hipDeviceptr_t) wa;
                eb = hipStreamBatchMemOp(A, 2, pa, 0);
                if (eb == hipSuccess) eb = hipStreamBatchMemOp(B, 2, pb, 0);
            }
            if (eb != hipSuccess) {
                printf("%-13s hipStreamBatchMemOp: %s\n", k.name, hipGetErrorString(eb));
                (void) hipGetLastError();
            } else {
                CK(hipStreamSynchronize(A));
                CK(hipStreamSynchronize(B));
                bb_us = (now_us() - t0) / rounds;
            }
            // self: one batch of a write and a satisfied wait on one stream
            t0 = now_us();
            for (uint32_t r = 1; r <= (uint32_t) rounds && eb == hipSuccess; ++r) {
                hipStreamBatchMemOpParams pa[2];
                memset(pa, 0, sizeof(pa));
                pa[0].writeValue.operation = hipStreamMemOpWriteValue32;
                pa[0].writeValue.address = (hipDeviceptr_t) wa;
                pa[0].writeValue.value = (uint32_t) rounds + r;
                pa[1].waitValue.operation = hipStreamMemOpWaitValue32;
                pa[1].waitValue.address = (hipDeviceptr_t) wa;
                pa[1].waitValue.value = (uint32_t) rounds + r;
                pa[1].waitValue.flags = hipStreamWaitValueGte;
                eb = hipStreamBatchMemOp(A, 2, pa, 0);
            }
            if (eb == hipSuccess) {
                CK(hipStreamSynchronize(A));
                bs_us = (now_us() - t0) / rounds;
            }
        }
        printf("%-13s self %.2f us/pair  pingpong %.2f us/barrier  kernel pingpong %.2f us/barrier  "
               "batch pingpong %.2f us/barrier  batch self %.2f us\n", k.name, self_us, pp_us, kk_us, bb_us, bs_us);
        CK(hipFree(w));
    }
    return 0;
}
