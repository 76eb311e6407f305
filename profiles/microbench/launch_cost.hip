// Host cost of a kernel launch vs the GPU time of short dependent kernels
// (the engine's build is ~100 launches of 1-30 us kernels): is the host or
// the GPU the bottleneck of such a chain?  Prints one JSON line.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_empty() {}
__global__ void k_touch(unsigned *p, unsigned n) {
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] += 1u;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    unsigned *p;
    const unsigned n = 1u << 20;   // 4 MB, 4096 blocks: a 1M-row elementwise pass
    hipMalloc(&p, n * 4);
    hipMemset(p, 0, n * 4);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int N = 2000;
    for (int i = 0; i < 200; i++) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
    hipStreamSynchronize(s);
    // 1. host cost per launch (queue never drains: empty kernels)
    double t0 = now_us();
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
    double host_empty = (now_us() - t0) / N;
    hipStreamSynchronize(s);
    // 2. GPU time per dependent 1M-element pass when queued ahead (events)
    hipEventRecord(a, s);
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_touch, dim3(n / 256), dim3(256), 0, s, p, n);
    hipEventRecord(b, s);
    hipStreamSynchronize(s);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    double gpu_touch = ms * 1e3 / N;
    // 3. launches right after a host wait (the queue is empty): time to the end of 8 kernels
    double after_sync = 0;
    for (int r = 0; r < 50; r++) {
        hipStreamSynchronize(s);
        double t1 = now_us();
        for (int i = 0; i < 8; i++) hipLaunchKernelGGL(k_touch, dim3(n / 256), dim3(256), 0, s, p, n);
        hipStreamSynchronize(s);
        after_sync += now_us() - t1;
    }
    after_sync /= 50;
    // 4. the same 8 kernels captured in a graph
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < 8; i++) hipLaunchKernelGGL(k_touch, dim3(n / 256), dim3(256), 0, s, p, n);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    double graph8 = 0;
    for (int r = 0; r < 50; r++) {
        hipStreamSynchronize(s);
        double t1 = now_us();
        hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        graph8 += now_us() - t1;
    }
    graph8 /= 50;
    std::printf("{\"host_us_per_launch\": %.2f, \"gpu_us_per_1M_pass_queued\": %.2f, "
                "\"us_8_passes_after_sync\": %.1f, \"us_8_passes_graph\": %.1f}\n",
                host_empty, gpu_touch, after_sync, graph8);
    return 0;
}
