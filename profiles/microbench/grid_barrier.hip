// Is a grid-wide barrier inside one kernel cheaper than a kernel boundary?
// The small-list step (C1 10k, C3 100k rows) is a chain of ~30 dependent
// kernels, most at the ~5 us floor of a dependent launch; fusing a chain into
// one kernel pays a grid barrier per phase instead.  Measured here, each
// phase a pass over n words that reads another workgroup's previous writes
// (so the barrier's release / acquire must make them visible across XCDs):
//   chain:   R dependent launches of that pass (grid = n / 256 blocks)
//   barrier: one launch of G workgroups doing R phases, a counter barrier
//            between them (agent-scope release fence, one atomic add per
//            workgroup, acquire loads until the phase's count is reached;
//            bounded spin: a workgroup that waits too long raises an error
//            word and leaves, so no wave can hang)
// Results are checked against the host.  Prints one JSON line per variant.
//   hipcc --offload-arch=gfx950 -O3 -o grid_barrier grid_barrier.hip && ./grid_barrier
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr uint32_t SHIFT = 4099;   // a word written by another workgroup (another XCD)

__device__ __forceinline__ void pass(const uint32_t *in, uint32_t *out, uint32_t n, uint32_t i0, uint32_t stride) {
    for (uint32_t i = i0; i < n; i += stride) {
        uint32_t j = i + SHIFT;
        if (j >= n) j -= n;
        out[i] = in[j] * 3u + 1u;
    }
}

__global__ void __launch_bounds__(256) k_pass(const uint32_t *in, uint32_t *out, uint32_t n) {
    pass(in, out, n, blockIdx.x * 256u + threadIdx.x, gridDim.x * 256u);
}

// every workgroup arrives once per phase: the phase is over when the counter
// reaches (phase + 1) * G
__device__ __forceinline__ bool grid_sync(uint32_t *count, uint32_t target, uint32_t *err) {
    __syncthreads();
    __shared__ uint32_t s_ok;
    if (threadIdx.x == 0) {
        __atomic_thread_fence(__ATOMIC_RELEASE);   // (agent scope below: the writes of this workgroup)
        __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t spins = 0, ok = 1;
        while (__hip_atomic_load(count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            if (++spins > (1u << 22)) {   // bounded: raise the error word and leave
                __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        s_ok = ok;
    }
    __syncthreads();
    return s_ok != 0;
}

__global__ void __launch_bounds__(256) k_fused(uint32_t *a, uint32_t *b, uint32_t n, uint32_t rounds, uint32_t *count,
                                               uint32_t *err) {
    const uint32_t G = gridDim.x;
    for (uint32_t r = 0; r < rounds; r++) {
        const uint32_t *in = (r & 1) ? b : a;
        uint32_t *out = (r & 1) ? a : b;
        pass(in, out, n, blockIdx.x * 256u + threadIdx.x, G * 256u);
        if (!grid_sync(count, (r + 1) * G, err)) return;
    }
}

static std::vector<uint32_t> host_ref(uint32_t n, uint32_t rounds) {
    std::vector<uint32_t> x(n), y(n);
    for (uint32_t i = 0; i < n; i++) x[i] = i * 2654435761u;
    for (uint32_t r = 0; r < rounds; r++) {
        for (uint32_t i = 0; i < n; i++) {
            uint32_t j = i + SHIFT;
            if (j >= n) j -= n;
            y[i] = x[j] * 3u + 1u;
        }
        x.swap(y);
    }
    return x;
}

int main() {
    const uint32_t ns[3] = {10000, 100000, 400000};
    const uint32_t R = 64;
    uint32_t *a, *b, *cnt, *err;
    CHECK(hipMalloc(&a, 400000 * 4));
    CHECK(hipMalloc(&b, 400000 * 4));
    CHECK(hipMalloc(&cnt, 64));
    CHECK(hipMalloc(&err, 64));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<uint32_t> init(400000), got(400000);
    for (uint32_t i = 0; i < 400000; i++) init[i] = i * 2654435761u;
    for (uint32_t n : ns) {
        const std::vector<uint32_t> want = host_ref(n, R);
        // chain of dependent launches
        for (int rep = 0; rep < 3; rep++) {
            CHECK(hipMemcpy(a, init.data(), n * 4, hipMemcpyHostToDevice));
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0, s));
            for (uint32_t r = 0; r < R; r++)
                hipLaunchKernelGGL(k_pass, dim3((n + 255) / 256), dim3(256), 0, s, (r & 1) ? b : a, (r & 1) ? a : b, n);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            CHECK(hipMemcpy(got.data(), (R & 1) ? b : a, n * 4, hipMemcpyDeviceToHost));
            const bool okv = std::equal(want.begin(), want.end(), got.begin());
            if (rep == 2) printf("{\"variant\": \"chain\", \"n\": %u, \"phases\": %u, \"us_per_phase\": %.2f, \"exact\": %s}\n", n, R,
                                 ms * 1000.0f / R, okv ? "true" : "false");
        }
        for (uint32_t G : {32u, 64u, 128u, 256u, 512u}) {
            for (int rep = 0; rep < 3; rep++) {
                CHECK(hipMemcpy(a, init.data(), n * 4, hipMemcpyHostToDevice));
                CHECK(hipMemset(cnt, 0, 64));
                CHECK(hipMemset(err, 0, 64));
                CHECK(hipDeviceSynchronize());
                CHECK(hipEventRecord(e0, s));
                hipLaunchKernelGGL(k_fused, dim3(G), dim3(256), 0, s, a, b, n, R, cnt, err);
                CHECK(hipEventRecord(e1, s));
                CHECK(hipEventSynchronize(e1));
                float ms = 0;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                uint32_t e = 0;
                CHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
                CHECK(hipMemcpy(got.data(), (R & 1) ? b : a, n * 4, hipMemcpyDeviceToHost));
                const bool okv = std::equal(want.begin(), want.end(), got.begin());
                if (rep == 2)
                    printf("{\"variant\": \"barrier\", \"n\": %u, \"workgroups\": %u, \"phases\": %u, \"us_per_phase\": %.2f, "
                           "\"exact\": %s, \"timeout\": %u}\n", n, G, R, ms * 1000.0f / R, okv ? "true" : "false", e);
                if (e) break;
            }
        }
    }
    return 0;
}
