// Cost per event of an exact single-wave lane replay (wg_lanes_serial.hip's
// design, measured before it went into the engine).
//
// Lane l of the wave owns slot l (word w of a lane: slot 64 w + l) and holds
// D = the time its holder dies (0 = never held; leaked = 0x7FFFFFFF).  Event k
// (time k + 1) is one record {lo, width, dv}: the slots it selects are those
// with D - lo < width (ALLOC: lo 0, width k + 1 = free before k; MIN: lo
// k + 1, width 1 = the waiters dying at k; FREE: width 0 = nothing), its slot is
// the lowest selected one, and that lane's D becomes dv (ALLOC / MIN that
// occupies: its own death time; otherwise k + 1).  The host builds a random
// event stream from a reference greedy (lowest free slot; MIN keeps the
// lowest waiter) and checks the kernel's slots against it.
//
// usage: serial_replay [events] [live]   -> one JSON line per variant
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__device__ __forceinline__ int ff1(uint64_t m) {   // s_ff1: lowest set bit, -1 for none
    int x;
    asm volatile("s_ff1_i32_b64 %0, %1" : "=s"(x) : "s"(m));
    return x;
}
template <int J>
__device__ __forceinline__ void wlc(uint32_t &v, int val) {   // v[J] = val
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(v) : "s"(val), "n"(J));
}

// MODE 0: NW words, update by compare + cndmask on every word
// MODE 1: update by v_writelane with the lane select in M0 (NW = 1: the whole
//         step in one asm block; NW > 1: a uniform branch on the word)
template <int NW, int MODE, int J>
__device__ __forceinline__ void step(uint32_t (&D)[NW], uint32_t lane, uint32_t &o, uint4 r) {
    if (MODE == 1 && NW == 1) {
        uint32_t t;
        uint64_t m;
        asm volatile(
            "v_subrev_u32 %[t], %[lo], %[D]\n\t"
            "v_cmp_gt_u32_e64 %[m], %[wid], %[t]\n\t"
            "s_ff1_i32_b64 m0, %[m]\n\t"
            "v_writelane_b32 %[D], %[dv], m0\n\t"
            "v_writelane_b32 %[o], m0, %[j]"
            : [D] "+v"(D[0]), [o] "+v"(o), [t] "=&v"(t), [m] "=&s"(m)
            : [lo] "s"(r.x), [wid] "s"(r.y), [dv] "s"(r.z), [j] "n"(J)
            : "m0", "scc");
        return;
    }
    int x = -1;
#pragma unroll
    for (int w = NW - 1; w >= 0; w--) {
        const uint64_t m = __ballot(D[w] - r.x < r.y);
        const int f = ff1(m);
        if (NW == 1) x = f;
        else x = m ? 64 * w + f : x;
    }
    if (MODE == 0) {
#pragma unroll
        for (int w = 0; w < NW; w++) D[w] = (lane + 64u * w == (uint32_t)x) ? r.z : D[w];
    } else {
        const int w = x >> 6;
#pragma unroll
        for (int q = 0; q < NW; q++)
            if (w == q) asm volatile("s_mov_b32 m0, %1\n\tv_writelane_b32 %0, %2, m0" : "+v"(D[q]) : "s"(x & 63), "s"(r.z) : "m0", "scc");
    }
    wlc<J>(o, x);
}

// MODE 2 (NW = 1): software-pipelined — event j+1's compare runs on D before
// event j's lane write, which the scalar unit patches in (rec.w = Y: 0 when
// the previous event's lane, with its new D, is selected, else 63).  PIPE 0:
// the scalar patch first (in-order issue holds the next compare behind it);
// PIPE 1: the lane write and the next compare first.
template <int J, int PIPE>
__device__ __forceinline__ void pstep(uint32_t &D, uint32_t &o, uint64_t &M, uint64_t &Mn, uint32_t Y, uint32_t dvp,
                                      uint32_t lo1, uint32_t wid1) {
    uint32_t y, T;
    if (PIPE == 0)
        asm volatile(
            "s_or_b32 %[y], m0, %[Y]\n\t"
            "s_bitset0_b64 %[M], m0\n\t"
            "s_bitset1_b64 %[M], %[y]\n\t"
            "v_writelane_b32 %[D], %[dvp], m0\n\t"
            "s_ff1_i32_b64 m0, %[M]\n\t"
            "v_writelane_b32 %[o], m0, %[j]\n\t"
            "v_subrev_u32 %[T], %[lo1], %[D]\n\t"
            "v_cmp_gt_u32_e64 %[Mn], %[wid1], %[T]"
            : [D] "+v"(D), [o] "+v"(o), [M] "+s"(M), [Mn] "=s"(Mn), [y] "=&s"(y), [T] "=&v"(T)
            : [Y] "s"(Y), [dvp] "s"(dvp), [lo1] "s"(lo1), [wid1] "s"(wid1), [j] "n"(J)
            : "m0", "scc");
    else
        asm volatile(
            "v_writelane_b32 %[D], %[dvp], m0\n\t"
            "v_subrev_u32 %[T], %[lo1], %[D]\n\t"
            "v_cmp_gt_u32_e64 %[Mn], %[wid1], %[T]\n\t"
            "s_or_b32 %[y], m0, %[Y]\n\t"
            "s_bitset0_b64 %[M], m0\n\t"
            "s_bitset1_b64 %[M], %[y]\n\t"
            "s_ff1_i32_b64 m0, %[M]\n\t"
            "v_writelane_b32 %[o], m0, %[j]"
            : [D] "+v"(D), [o] "+v"(o), [M] "+s"(M), [Mn] "=s"(Mn), [y] "=&s"(y), [T] "=&v"(T)
            : [Y] "s"(Y), [dvp] "s"(dvp), [lo1] "s"(lo1), [wid1] "s"(wid1), [j] "n"(J)
            : "m0", "scc");
}
template <int G, int PIPE>
__device__ __forceinline__ void pgroup(uint32_t &D, uint32_t &o, uint64_t &Ma, uint64_t &Mb, uint32_t &dvp,
                                       const uint4 (&cur)[8], const uint4 &n0) {
    pstep<G + 0, PIPE>(D, o, Ma, Mb, cur[0].w, dvp, cur[1].x, cur[1].y);
    pstep<G + 1, PIPE>(D, o, Mb, Ma, cur[1].w, cur[0].z, cur[2].x, cur[2].y);
    pstep<G + 2, PIPE>(D, o, Ma, Mb, cur[2].w, cur[1].z, cur[3].x, cur[3].y);
    pstep<G + 3, PIPE>(D, o, Mb, Ma, cur[3].w, cur[2].z, cur[4].x, cur[4].y);
    pstep<G + 4, PIPE>(D, o, Ma, Mb, cur[4].w, cur[3].z, cur[5].x, cur[5].y);
    pstep<G + 5, PIPE>(D, o, Mb, Ma, cur[5].w, cur[4].z, cur[6].x, cur[6].y);
    pstep<G + 6, PIPE>(D, o, Ma, Mb, cur[6].w, cur[5].z, cur[7].x, cur[7].y);
    pstep<G + 7, PIPE>(D, o, Mb, Ma, cur[7].w, cur[6].z, n0.x, n0.y);
    dvp = cur[7].z;
}
template <int PIPE>
__global__ void __launch_bounds__(64) k_pipe(const uint4 *__restrict__ rec, uint64_t n, uint16_t *__restrict__ out,
                                             unsigned long long *cyc) {
    const uint32_t lane = threadIdx.x;
    uint32_t D = lane == 63 ? 0x7FFFFFFFu : 0u;
    uint64_t Ma, Mb;
    uint32_t dvp = 0x7FFFFFFFu;
    uint4 cur[8], nxt[8];
#pragma unroll
    for (int i = 0; i < 8; i++) cur[i] = rec[i];
    const unsigned long long t0 = clock64();
    {
        uint32_t T;
        asm volatile("s_mov_b32 m0, 63\n\tv_subrev_u32 %[T], %[lo], %[D]\n\tv_cmp_gt_u32_e64 %[M], %[wid], %[T]"
                     : [M] "=s"(Ma), [T] "=&v"(T) : [D] "v"(D), [lo] "s"(cur[0].x), [wid] "s"(cur[0].y) : "m0", "scc");
    }
    for (uint64_t base = 0; base < n; base += 64) {
        uint32_t o = 0xFFFFu;
#define PG(G) { _Pragma("unroll") for (int i = 0; i < 8; i++) nxt[i] = rec[base + G + 8 + i]; \
                pgroup<G, PIPE>(D, o, Ma, Mb, dvp, cur, nxt[0]); \
                _Pragma("unroll") for (int i = 0; i < 8; i++) cur[i] = nxt[i]; }
        PG(0) PG(8) PG(16) PG(24) PG(32) PG(40) PG(48) PG(56)
#undef PG
        out[base + lane] = (uint16_t)o;
    }
    if (lane == 0) *cyc = clock64() - t0;
}

template <int J, int NW, int MODE>
__device__ __forceinline__ void group(uint32_t (&D)[NW], uint32_t lane, uint32_t &o, const uint4 (&cur)[8]) {
    step<NW, MODE, J + 0>(D, lane, o, cur[0]);
    step<NW, MODE, J + 1>(D, lane, o, cur[1]);
    step<NW, MODE, J + 2>(D, lane, o, cur[2]);
    step<NW, MODE, J + 3>(D, lane, o, cur[3]);
    step<NW, MODE, J + 4>(D, lane, o, cur[4]);
    step<NW, MODE, J + 5>(D, lane, o, cur[5]);
    step<NW, MODE, J + 6>(D, lane, o, cur[6]);
    step<NW, MODE, J + 7>(D, lane, o, cur[7]);
}

template <int NW, int MODE>
__global__ void __launch_bounds__(64) k_serial(const uint4 *__restrict__ rec, uint64_t n, uint16_t *__restrict__ out,
                                               unsigned long long *cyc) {
    const uint32_t lane = threadIdx.x;
    uint32_t D[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) D[w] = 0;
    const unsigned long long t0 = clock64();
    uint4 cur[8], nxt[8];
#pragma unroll
    for (int i = 0; i < 8; i++) cur[i] = rec[i];
    for (uint64_t base = 0; base < n; base += 64) {
        uint32_t o = 0xFFFFu;
#define G(J) { _Pragma("unroll") for (int i = 0; i < 8; i++) nxt[i] = rec[base + J + 8 + i]; \
               group<J, NW, MODE>(D, lane, o, cur); \
               _Pragma("unroll") for (int i = 0; i < 8; i++) cur[i] = nxt[i]; }
        G(0) G(8) G(16) G(24) G(32) G(40) G(48) G(56)
#undef G
        out[base + lane] = (uint16_t)o;
    }
    if (lane == 0) *cyc = clock64() - t0;
}

struct Ev { int kind; uint32_t t0, t1; bool occ; };   // kind 0 ALLOC, 1 MIN, 2 FREE

int main(int argc, char **argv) {
    const uint64_t N = argc > 1 ? strtoull(argv[1], 0, 10) : 65536;
    const int LIVE = argc > 2 ? atoi(argv[2]) : 40;
    std::mt19937_64 rng(12345);
    // random stream: keep about LIVE tokens alive; a few leak
    std::vector<Ev> ev(N);
    std::vector<uint32_t> live;
    for (uint64_t k = 0; k < N; k++) {
        const double u = std::uniform_real_distribution<double>(0, 1)(rng);
        if (live.size() < 2 || (live.size() < (size_t)LIVE && u < 0.6) || u < 0.45) {
            ev[k] = {0, 0, 0, u > 0.01};
            if (ev[k].occ) live.push_back((uint32_t)k);
        } else if (u < 0.95) {
            std::swap(live[rng() % live.size()], live.back());
            const uint32_t a = live.back(); live.pop_back();
            std::swap(live[rng() % live.size()], live.back());
            const uint32_t b = live.back(); live.pop_back();
            ev[k] = {1, a, b, u < 0.93};
            if (ev[k].occ) live.push_back((uint32_t)k);
        } else {
            std::swap(live[rng() % live.size()], live.back());
            const uint32_t a = live.back(); live.pop_back();
            ev[k] = {2, a, a, false};
        }
    }
    // reference greedy with token -> slot
    std::vector<uint16_t> ref(N, 0xFFFF);
    std::vector<int64_t> holder(1024, -1);
    std::vector<uint32_t> death(N, 0x7FFFFFFFu);
    int maxslot = 0;
    for (uint64_t k = 0; k < N; k++) {
        const Ev &e = ev[k];
        if (e.kind == 0) {
            int s = 0;
            while (holder[s] >= 0) s++;
            ref[k] = (uint16_t)s;
            maxslot = std::max(maxslot, s);
            if (e.occ) holder[s] = (int64_t)k;
        } else {
            death[e.t0] = (uint32_t)k + 1;
            death[e.t1] = (uint32_t)k + 1;
            const int a = ref[e.t0], b = ref[e.t1];
            holder[a] = -1;
            holder[b] = -1;
            const int m = std::min(a, b);
            ref[k] = (uint16_t)m;
            if (e.kind == 1 && e.occ) holder[m] = (int64_t)k;
        }
    }
    const uint64_t NP = (N + 63) / 64 * 64;
    std::vector<uint4> rec(NP + 64, make_uint4(0u, 0u, 0u, 0u));   // (+64: the last group's prefetch)
    for (uint64_t k = 0; k < N; k++) {
        const Ev &e = ev[k];
        const uint32_t t = (uint32_t)k + 1;
        if (e.kind == 0) rec[k] = make_uint4(0u, t, e.occ ? death[k] : t, 0u);
        else if (e.kind == 1) rec[k] = make_uint4(t, 1u, e.occ ? death[k] : t, 0u);
        else rec[k] = make_uint4(0u, t, t, 0u);   // FREE: a probe that takes no slot (its result is ignored)
    }
    for (uint64_t k = N; k < NP + 64; k++) rec[k] = make_uint4(0u, 0u, 0x7FFFFFFFu, 63u);   // no-ops (the pipelined kernels)
    // Y: does event k select the previous event's lane with its new D?
    for (uint64_t k = 0; k < N; k++) {
        const uint32_t dvp = k ? rec[k - 1].z : 0x7FFFFFFFu;
        rec[k].w = (k && dvp - rec[k].x < rec[k].y) ? 0u : 63u;
    }
    uint4 *d_rec; uint16_t *d_out; unsigned long long *d_cyc;
    CK(hipMalloc(&d_rec, (NP + 64) * 16));
    CK(hipMalloc(&d_out, NP * 2));
    CK(hipMalloc(&d_cyc, 8));
    CK(hipMemcpy(d_rec, rec.data(), (NP + 64) * 16, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto run = [&](const char *name, int nw, auto kern) -> int {
        for (int rep = 0; rep < 3; rep++) {
            CK(hipMemset(d_out, 0xFF, NP * 2));
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, (const uint4 *)d_rec, NP, d_out, d_cyc);
            CK(hipGetLastError());
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
        }
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        unsigned long long cyc = 0;
        CK(hipMemcpy(&cyc, d_cyc, 8, hipMemcpyDeviceToHost));
        std::vector<uint16_t> o(NP);
        CK(hipMemcpy(o.data(), d_out, NP * 2, hipMemcpyDeviceToHost));
        uint64_t bad = 0;
        for (uint64_t k = 0; k < N; k++) if (ev[k].kind != 2 && o[k] != ref[k]) bad++;
        printf("{\"variant\": \"%s\", \"nw\": %d, \"events\": %lu, \"max_slot\": %d, \"ms\": %.4f, \"ns_per_event\": %.2f, "
               "\"clock64_per_event\": %.2f, \"mismatch\": %lu}\n",
               name, nw, (unsigned long)N, maxslot, ms, ms * 1e6 / N, (double)cyc / NP, (unsigned long)bad);
        fflush(stdout);
        return 0;
    };
    if (maxslot < 63 && run("pipe_salu_first", 1, k_pipe<0>)) return 1;
    if (maxslot < 63 && run("pipe_valu_first", 1, k_pipe<1>)) return 1;
    if (maxslot < 64 && run("cnd", 1, k_serial<1, 0>)) return 1;
    if (maxslot < 64 && run("wl", 1, k_serial<1, 1>)) return 1;
    if (maxslot < 128 && run("cnd", 2, k_serial<2, 0>)) return 1;
    if (maxslot < 128 && run("wl", 2, k_serial<2, 1>)) return 1;
    if (maxslot < 192 && run("cnd", 3, k_serial<3, 0>)) return 1;
    if (maxslot < 192 && run("wl", 3, k_serial<3, 1>)) return 1;
    if (run("cnd", 4, k_serial<4, 0>)) return 1;
    if (run("wl", 4, k_serial<4, 1>)) return 1;
    return 0;
}
