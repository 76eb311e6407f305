// Store-bandwidth sweep beyond store_ceiling.hip: does the MAPPING of
// workgroups to output tiles, or the workgroup size, move the write ceiling
// of a k_vtx_tile-shaped kernel (5.86 GB of 16-B vectors, one contiguous
// tile per workgroup)?  Variants:
//   dispatch   tile = blockIdx.x (k_vtx_tile today; blocks are dealt to the 8
//              XCDs round-robin, so neighbouring tiles come from different XCDs)
//   xcd-split  tile = (b % 8) * (T / 8) + b / 8: each XCD writes one contiguous
//              eighth of the buffer
//   persist-s  2048 workgroups, tile-strided loop (t += grid)
//   persist-c  2048 workgroups, each a contiguous run of tiles
// with 256 / 512 threads and 12 / 24 / 48 KiB tiles, plain and non-temporal.
//   hipcc --offload-arch=gfx950 -O3 -o store_sweep store_sweep.hip && ./store_sweep
#include <hip/hip_runtime.h>
#include <cstring>

#include <cstdio>
#include <cstdlib>

typedef float v4f __attribute__((ext_vector_type(4)));
#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

enum { MAP_DISPATCH = 0, MAP_XCD = 1, MAP_PERSIST_STRIDE = 2, MAP_PERSIST_CONTIG = 3, MAP_XCD_STAGGER = 4, MAP_XCD_DYN = 5, MAP_XCD_PERSIST = 6 };

template <bool NT, int R, int TH>
__device__ __forceinline__ void write_tile(v4f *out, size_t n, size_t t) {
    const v4f v = {1.0f, 2.0f, 3.0f, 4.0f};
    const size_t b = t * (size_t)(TH * R);
#pragma unroll
    for (int k = 0; k < R; k++) {
        const size_t i = b + (size_t)k * TH + threadIdx.x;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(v, out + i);
            else out[i] = v;
        }
    }
}

template <bool NT, int R, int TH, int MAP>
__global__ void __launch_bounds__(TH) k_tiles(v4f *out, size_t n, size_t ntiles, unsigned *ctr) {
    const size_t g = gridDim.x, b = blockIdx.x;
    if (MAP == MAP_XCD_DYN) {
        // XCD x's workgroups claim the tiles of its eighth in order (one counter
        // per XCD); once that eighth is taken they claim from the others'
        __shared__ unsigned s_t;
        const size_t per = (ntiles + 7) / 8;
        if (threadIdx.x == 0) {
            const unsigned x = (unsigned)(b % 8);
            unsigned t = ~0u;
            for (unsigned k = 0; k < 8 && t == ~0u; k++) {
                const unsigned xx = (x + k) % 8;
                const unsigned i = atomicAdd(&ctr[xx * 32], 1u);
                if (i < per && xx * per + i < ntiles) t = (unsigned)(xx * per + i);
            }
            s_t = t;
        }
        __syncthreads();
        if (s_t != ~0u) write_tile<NT, R, TH>(out, n, s_t);
        return;
    }
    if (MAP == MAP_DISPATCH) {
        write_tile<NT, R, TH>(out, n, b);
    } else if (MAP == MAP_XCD) {
        const size_t per = (ntiles + 7) / 8;
        const size_t t = (b % 8) * per + b / 8;
        if (t < ntiles) write_tile<NT, R, TH>(out, n, t);
    } else if (MAP == MAP_XCD_STAGGER) {
        // as MAP_XCD, but XCD x starts its eighth x/8 of the way in (and wraps):
        // the eight write streams sit at different phases of their regions
        const size_t per = (ntiles + 7) / 8, x = b % 8;
        const size_t t = x * per + (b / 8 + x * per / 8) % per;
        if (b / 8 < per && t < ntiles) write_tile<NT, R, TH>(out, n, t);
    } else if (MAP == MAP_XCD_PERSIST) {
        // persistent, XCD-split: XCD x's g / 8 workgroups stride through its
        // contiguous eighth (the workgroups of one XCD write neighbouring tiles
        // at any moment, as the one-tile xcd-split does)
        const size_t per = (ntiles + 7) / 8, x = b % 8, k = g / 8;
        for (size_t j = b / 8; j < per; j += k)
            if (x * per + j < ntiles) write_tile<NT, R, TH>(out, n, x * per + j);
    } else if (MAP == MAP_PERSIST_STRIDE) {
        for (size_t t = b; t < ntiles; t += g) write_tile<NT, R, TH>(out, n, t);
    } else {
        const size_t per = (ntiles + g - 1) / g;
        for (size_t t = b * per; t < (b + 1) * per && t < ntiles; t++) write_tile<NT, R, TH>(out, n, t);
    }
}

int main(int argc, char **argv) {
    // optional argv[1]: bytes written per launch (default: the 1M-row wide16 vertex buffer)
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 5856279118ull) & ~(size_t)15;
    const size_t n = bytes / 16;
    v4f *out;
    CHECK(hipMalloc(&out, bytes));
    unsigned *ctr;
    CHECK(hipMalloc(&ctr, 8 * 32 * 4));
    hipEvent_t a, b;
    // STORE_EVENTS=device: timing events with a device-scope release (as
    // bench.py's since r03n); default: HIP's system-scope fence
    const char *ev_env = getenv("STORE_EVENTS");
    const unsigned ev_flags = (ev_env && !strcmp(ev_env, "device")) ? hipEventReleaseToDevice : hipEventDefault;
    CHECK(hipEventCreateWithFlags(&a, ev_flags));
    CHECK(hipEventCreateWithFlags(&b, ev_flags));
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
        fflush(stdout);
    };
#define V(NT, R, TH, MAP, GRID, NAME)                                                                          \
    {                                                                                                          \
        const size_t nt_ = (n + (size_t)TH * R - 1) / ((size_t)TH * R);                                        \
        size_t grid_ = (GRID) ? (size_t)(GRID) : nt_;                                                          \
        if (MAP == MAP_XCD || MAP == MAP_XCD_STAGGER) grid_ = ((nt_ + 7) / 8) * 8;                                                       \
        if (MAP == MAP_XCD_DYN) grid_ = nt_;                                                                   \
        run(NAME, [&] {                                                                                        \
            if (MAP == MAP_XCD_DYN) CHECK(hipMemsetAsync(ctr, 0, 8 * 32 * 4, 0));                              \
            hipLaunchKernelGGL((k_tiles<NT, R, TH, MAP>), dim3((unsigned)grid_), dim3(TH), 0, 0, out, n, nt_, ctr); \
        });                                                                                                    \
    }
    V(true, 6, 256, MAP_XCD, 0, "24KiB/256 nt xcd-split");
    V(true, 6, 256, MAP_XCD_PERSIST, 2048, "24KiB/256 nt xcd-persist 2048");
    V(true, 6, 256, MAP_XCD_PERSIST, 4096, "24KiB/256 nt xcd-persist 4096");
    V(true, 6, 256, MAP_XCD_PERSIST, 8192, "24KiB/256 nt xcd-persist 8192");
    V(true, 6, 256, MAP_XCD_DYN, 0, "24KiB/256 nt xcd-dynamic");
    V(true, 3, 256, MAP_XCD, 0, "12KiB/256 nt xcd-split");
    V(true, 3, 256, MAP_XCD_DYN, 0, "12KiB/256 nt xcd-dynamic");
    V(true, 6, 256, MAP_DISPATCH, 0, "24KiB/256 nt dispatch");
    V(false, 6, 256, MAP_DISPATCH, 0, "24KiB/256 plain dispatch");
    V(true, 6, 256, MAP_XCD, 0, "24KiB/256 nt xcd-split");
    V(true, 6, 256, MAP_XCD_STAGGER, 0, "24KiB/256 nt xcd-stagger");
    V(false, 6, 256, MAP_XCD, 0, "24KiB/256 plain xcd-split");
    V(true, 3, 256, MAP_XCD, 0, "12KiB/256 nt xcd-split");
    V(true, 3, 256, MAP_DISPATCH, 0, "12KiB/256 nt dispatch");
    V(true, 6, 256, MAP_PERSIST_STRIDE, 2048, "24KiB/256 nt persist-stride 2048");
    V(true, 6, 256, MAP_PERSIST_STRIDE, 4096, "24KiB/256 nt persist-stride 4096");
    V(true, 6, 256, MAP_PERSIST_CONTIG, 2048, "24KiB/256 nt persist-contig 2048");
    V(true, 3, 512, MAP_DISPATCH, 0, "24KiB/512 nt dispatch");
    V(true, 6, 512, MAP_DISPATCH, 0, "48KiB/512 nt dispatch");
    V(true, 3, 512, MAP_XCD, 0, "24KiB/512 nt xcd-split");
    V(true, 12, 256, MAP_XCD, 0, "48KiB/256 nt xcd-split");
    V(false, 12, 256, MAP_XCD, 0, "48KiB/256 plain xcd-split");
    V(true, 18, 256, MAP_XCD, 0, "72KiB/256 nt xcd-split");
    CHECK(hipFree(out));
    CHECK(hipFree(ctr));
    return 0;
}
