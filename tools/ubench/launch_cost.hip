// Host cost of a kernel launch on this runtime: plain hipLaunchKernelGGL, and one hipGraphLaunch
// of a 6-node chain (the C2 frame's launch count). Prints microseconds per launch / per graph.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ void k_empty(int* p, int v) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && v < 0) p[0] = v;
}

int main() {
    int* d;
    (void)hipMalloc(&d, 64);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    auto now = [] { return std::chrono::steady_clock::now(); };
    for (int rep = 0; rep < 3; rep++) {
        const int n = 600;
        (void)hipStreamSynchronize(s);
        auto t0 = now();
        for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s, d, i);
        auto t1 = now();
        (void)hipStreamSynchronize(s);
        auto t2 = now();
        std::printf("launch: host %.2f us/launch, drain %.2f us/launch\n",
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
                    std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < 6; i++) hipLaunchKernelGGL(k_empty, dim3(64), dim3(256), 0, s, d, i);
    (void)hipStreamEndCapture(s, &g);
    (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    for (int rep = 0; rep < 3; rep++) {
        const int n = 100;
        (void)hipStreamSynchronize(s);
        auto t0 = now();
        for (int i = 0; i < n; i++) (void)hipGraphLaunch(ge, s);
        auto t1 = now();
        (void)hipStreamSynchronize(s);
        auto t2 = now();
        std::printf("graph(6 nodes): host %.2f us/graph, drain %.2f us/graph\n",
                    std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
                    std::chrono::duration<double, std::micro>(t2 - t0).count() / n);
    }
    {
        const int n = 100000;
        auto t0 = now();
        int hits = 0;
        for (int i = 0; i < n; i++) hits += std::getenv("ORBHIP_GRAPH") != nullptr;
        auto t1 = now();
        std::printf("getenv: %.3f us/call (%d hits)\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / n,
                    hits);
        hipEvent_t ev;
        (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        hipStream_t s2;
        (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
        const int m = 2000;
        t0 = now();
        for (int i = 0; i < m; i++) (void)hipEventRecord(ev, s);
        t1 = now();
        std::printf("hipEventRecord (no timing): %.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / m);
        t0 = now();
        for (int i = 0; i < m; i++) (void)hipStreamWaitEvent(s2, ev, 0);
        t1 = now();
        std::printf("hipStreamWaitEvent: %.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / m);
        (void)hipStreamSynchronize(s2);
    }
    return 0;
}
