// Store-bandwidth ceiling on this GPU for the vertex-emission roofline
// (DESIGN.md §3): how fast can a kernel that only writes 16-B vectors fill a
// buffer the size of one k_vtx_tile launch (5.86 GB)?  Variants: plain and
// non-temporal stores, grid-stride and one contiguous 48 KiB block per
// workgroup (k_vtx_tile's shape), 256 threads per workgroup.
//   hipcc --offload-arch=gfx950 -O3 -o store_ceiling store_ceiling.hip && ./store_ceiling
#include <hip/hip_runtime.h>
#include <cstring>

#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

template <bool NT>
__global__ void __launch_bounds__(256) k_stride(v4f *out, size_t n) {
    const v4f v = {1.0f, 2.0f, 3.0f, 4.0f};
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (NT) __builtin_nontemporal_store(v, out + i);
        else out[i] = v;
    }
}

// one contiguous block per workgroup (R rounds of 256 lanes x 16 B: R = 12 is
// 48 KiB, R = 6 is 24 KiB — k_vtx_tile's tile shapes)
template <bool NT, int R>
__global__ void __launch_bounds__(256) k_block(v4f *out, size_t n) {
    const v4f v = {1.0f, 2.0f, 3.0f, 4.0f};
    const size_t b = (size_t)blockIdx.x * (256 * R);
#pragma unroll
    for (int k = 0; k < R; k++) {
        const size_t i = b + k * 256 + threadIdx.x;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(v, out + i);
            else out[i] = v;
        }
    }
}

int main(int argc, char **argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 5856279118ull) & ~(size_t)15;   // (argv[1]: another launch size, e.g. C4's 15.67 GB)
    const size_t n = bytes / 16;
    v4f *out;
    CHECK(hipMalloc(&out, bytes));
    hipEvent_t a, b;
    // STORE_EVENTS=device: timing events with a device-scope release (as
    // bench.py's since r03n); default: HIP's system-scope fence
    const char *ev_env = getenv("STORE_EVENTS");
    const unsigned ev_flags = (ev_env && !strcmp(ev_env, "device")) ? hipEventReleaseToDevice : hipEventDefault;
    CHECK(hipEventCreateWithFlags(&a, ev_flags));
    CHECK(hipEventCreateWithFlags(&b, ev_flags));
    struct V { const char *name; void (*launch)(v4f *, size_t); };
    auto run = [&](const char *name, auto launch) {
        for (int w = 0; w < 2; w++) launch();
        CHECK(hipDeviceSynchronize());
        float best = 1e30f, sum = 0.0f;
        const int reps = 10;
        for (int r = 0; r < reps; r++) {
            CHECK(hipEventRecord(a));
            launch();
            CHECK(hipEventRecord(b));
            CHECK(hipEventSynchronize(b));
            float ms = 0.0f;
            CHECK(hipEventElapsedTime(&ms, a, b));
            best = ms < best ? ms : best;
            sum += ms;
        }
        printf("{\"variant\": \"%s\", \"bytes\": %zu, \"best_ms\": %.4f, \"avg_ms\": %.4f, \"best_TBps\": %.3f, \"avg_TBps\": %.3f}\n",
               name, bytes, best, sum / reps, bytes / (best * 1e-3) / 1e12, bytes / (sum / reps * 1e-3) / 1e12);
    };
    const unsigned grid_stride = 256 * 32;
    const unsigned g48 = (unsigned)((n + 3071) / 3072), g24 = (unsigned)((n + 1535) / 1536), g12 = (unsigned)((n + 767) / 768);
    run("grid-stride plain", [&] { hipLaunchKernelGGL(k_stride<false>, dim3(grid_stride), dim3(256), 0, 0, out, n); });
    run("grid-stride nontemporal", [&] { hipLaunchKernelGGL(k_stride<true>, dim3(grid_stride), dim3(256), 0, 0, out, n); });
    run("48KiB-block plain", [&] { hipLaunchKernelGGL((k_block<false, 12>), dim3(g48), dim3(256), 0, 0, out, n); });
    run("48KiB-block nontemporal", [&] { hipLaunchKernelGGL((k_block<true, 12>), dim3(g48), dim3(256), 0, 0, out, n); });
    run("24KiB-block plain", [&] { hipLaunchKernelGGL((k_block<false, 6>), dim3(g24), dim3(256), 0, 0, out, n); });
    run("24KiB-block nontemporal", [&] { hipLaunchKernelGGL((k_block<true, 6>), dim3(g24), dim3(256), 0, 0, out, n); });
    run("12KiB-block plain", [&] { hipLaunchKernelGGL((k_block<false, 3>), dim3(g12), dim3(256), 0, 0, out, n); });
    run("12KiB-block nontemporal", [&] { hipLaunchKernelGGL((k_block<true, 3>), dim3(g12), dim3(256), 0, 0, out, n); });
    CHECK(hipFree(out));
    return 0;
}
