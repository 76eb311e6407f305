// Is the emission's store bandwidth a property of the buffer's placement?
// bench.py's k_vtx_tile runs at 0.836 or 0.95 ms per 5.86 GB launch, the mode
// changing from process to process with the same code (r05 w29).  Here: eight
// allocations in one process, each written by a 24 KiB-block non-temporal
// store kernel (k_vtx_tile's shape) at three start addresses inside it — as
// returned, rounded up to 2 MiB and to 1 GiB — with the address printed.
//   hipcc --offload-arch=gfx950 -O3 -o store_align store_align.hip && ./store_align
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void __launch_bounds__(256) k_block(v4f *out, size_t n) {
    const v4f v = {1.0f, 2.0f, 3.0f, 4.0f};
    const size_t b = (size_t)blockIdx.x * (256 * 6);
#pragma unroll
    for (int k = 0; k < 6; k++) {
        const size_t i = b + k * 256 + threadIdx.x;
        if (i < n) __builtin_nontemporal_store(v, out + i);
    }
}

int main() {
    const size_t bytes = 5856279118ull & ~(size_t)15, n = bytes / 16;
    const size_t slack = (size_t)1 << 30;
    hipEvent_t a, b;
    CHECK(hipEventCreateWithFlags(&a, hipEventReleaseToDevice));
    CHECK(hipEventCreateWithFlags(&b, hipEventReleaseToDevice));
    const unsigned grid = (unsigned)((n + 1535) / 1536);
    for (int trial = 0; trial < 8; trial++) {
        char *base;
        CHECK(hipMalloc(&base, bytes + slack));
        const uintptr_t u = (uintptr_t)base;
        const uintptr_t starts[3] = {u, (u + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1), (u + slack - 1) & ~(uintptr_t)(slack - 1)};
        const char *names[3] = {"as returned", "2 MiB aligned", "1 GiB aligned"};
        for (int s = 0; s < 3; s++) {
            v4f *out = (v4f *)starts[s];
            for (int w = 0; w < 2; w++) hipLaunchKernelGGL(k_block, dim3(grid), dim3(256), 0, 0, out, n);
            CHECK(hipDeviceSynchronize());
            float sum = 0.0f, best = 1e30f;
            for (int r = 0; r < 6; r++) {
                CHECK(hipEventRecord(a));
                hipLaunchKernelGGL(k_block, dim3(grid), dim3(256), 0, 0, out, n);
                CHECK(hipEventRecord(b));
                CHECK(hipEventSynchronize(b));
                float ms = 0.0f;
                CHECK(hipEventElapsedTime(&ms, a, b));
                sum += ms;
                best = ms < best ? ms : best;
            }
            printf("{\"trial\": %d, \"start\": \"%s\", \"addr\": \"0x%llx\", \"addr_mod_1GiB_MiB\": %llu, \"avg_ms\": %.4f, \"best_ms\": %.4f, \"avg_TBps\": %.3f}\n",
                   trial, names[s], (unsigned long long)starts[s], (unsigned long long)((starts[s] & (slack - 1)) >> 20), sum / 6,
                   best, bytes / (sum / 6 * 1e-3) / 1e12);
            fflush(stdout);
        }
        // keep every other allocation so later ones land elsewhere
        if (trial & 1) CHECK(hipFree(base));
    }
    return 0;
}
