// Dev tool (not product): host-side completion latency of one tiny kernel under the ways a
// blocking collective can wait for it (null stream vs an internal non-blocking stream; stream
// sync vs event sync vs spinning on hipEventQuery).  Interleaved rounds in one process.
// Build: hipcc --offload-arch=gfx950 -O3 tools/sync_latency.hip -o tools/bin/sync_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void tiny(int *p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
    int *d;
    (void) hipMalloc(&d, 4096);
    hipStream_t nb, bl;
    (void) hipStreamCreateWithFlags(&nb, hipStreamNonBlocking);
    (void) hipStreamCreate(&bl);
    hipEvent_t ev, evs;
    (void) hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    (void) hipEventCreateWithFlags(&evs, hipEventDisableTiming | hipEventBlockingSync);
    const char *names[] = {"null stream + hipStreamSynchronize(0)", "null stream + hipDeviceSynchronize",
                           "nonblocking stream + hipStreamSynchronize", "nonblocking + event record + hipEventSynchronize",
                           "nonblocking + event record + spin hipEventQuery", "nonblocking + blocking-sync event",
                           "null-stream event -> nonblocking wait -> launch -> spin hipEventQuery",
                           "blocking stream + hipStreamSynchronize"};
    const int V = 8, R = 7, I = 200;
    std::vector<std::vector<double>> t(V);
    for (int r = 0; r < R; ++r) {
        for (int v = 0; v < V; ++v) {
            const double t0 = now_us();
            for (int i = 0; i < I; ++i) {
                switch (v) {
                    case 0: hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, 0, d); (void) hipStreamSynchronize(0); break;
                    case 1: hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, 0, d); (void) hipDeviceSynchronize(); break;
                    case 2: hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, nb, d); (void) hipStreamSynchronize(nb); break;
                    case 3:
                        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, nb, d);
                        (void) hipEventRecord(ev, nb);
                        (void) hipEventSynchronize(ev);
                        break;
                    case 4:
                        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, nb, d);
                        (void) hipEventRecord(ev, nb);
                        while (hipEventQuery(ev) == hipErrorNotReady) {}
                        break;
                    case 5:
                        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, nb, d);
                        (void) hipEventRecord(evs, nb);
                        (void) hipEventSynchronize(evs);
                        break;
                    case 6:
                        (void) hipEventRecord(evs, 0);
                        (void) hipStreamWaitEvent(nb, evs, 0);
                        hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, nb, d);
                        (void) hipEventRecord(ev, nb);
                        while (hipEventQuery(ev) == hipErrorNotReady) {}
                        break;
                    default: hipLaunchKernelGGL(tiny, dim3(1), dim3(64), 0, bl, d); (void) hipStreamSynchronize(bl); break;
                }
            }
            t[v].push_back((now_us() - t0) / I);
        }
    }
    for (int v = 0; v < V; ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("%-72s med %.2f us  min %.2f us\n", names[v], t[v][R / 2], t[v][0]);
    }
    return 0;
}
