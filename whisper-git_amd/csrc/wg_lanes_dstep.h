// wg_lanes_dstep.h — the D-state lane step shared by the exact serial replay
// (wg_lanes_serial.hip) and the compacted chunked replay (wg_lanes_dchunk.hip).
//
// Lane l of a wave owns slot 64 w + l (word w) and holds D = the time its
// holder's chain is consumed (event k has time k + 1; 0 = never held;
// WG_SER_INF = held for good).  An event selects "the lowest slot with D - lo
// < wid" (ALLOC: lo 0, wid its time = free before it, lowest_free_lane,
// commit_graph.rs:414-423; MIN / FREE: lo its time, wid 1 = the waiters it
// consumes, :287-291) and sets that slot's D to dv.  The helpers take a batch
// of 64 records {lo, wid, dv} held one per lane and write each event's slot
// into lane J of `out` (0xFFFFFFFF: nothing selected).
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

namespace {

constexpr uint32_t WG_SER_INF = 0x7FFFFFFFu;

// One word (63 slots + the sentinel lane 63).  One event: T = D - lo, the
// lanes with T < wid, the lowest into M0, its D := dv, the output lane J :=
// it.  A single wave issues about one instruction per 6-9 cycles
// (profiles/microbench/chain_latency.hip), so the step is its instruction
// count: these five plus the three v_readlane of the record.  Nothing
// selected: M0 = -1 addresses lane 63, the sentinel (its D := dv).
template <int J>
__device__ __forceinline__ void ser_step1(uint32_t &D, uint32_t &out, uint32_t lo, uint32_t wid, uint32_t dv) {
    uint32_t T;
    uint64_t M;
    asm volatile(
        "v_subrev_u32 %[T], %[lo], %[D]\n\t"
        "v_cmp_gt_u32_e64 %[M], %[wid], %[T]\n\t"
        "s_ff1_i32_b64 m0, %[M]\n\t"
        "v_writelane_b32 %[D], %[dv], m0\n\t"
        "v_writelane_b32 %[o], m0, %[j]"
        : [D] "+v"(D), [o] "+v"(out), [M] "=&s"(M), [T] "=&v"(T)
        : [lo] "s"(lo), [wid] "s"(wid), [dv] "s"(dv), [j] "n"(J)
        : "m0", "scc");
}

template <int J>
__device__ __forceinline__ void ser_quad1(uint32_t &D, uint32_t &out, const uint4 &R) {
#define WG_SER_RL(v, j) (uint32_t)__builtin_amdgcn_readlane((int)(v), (j))
    ser_step1<J + 0>(D, out, WG_SER_RL(R.x, J + 0), WG_SER_RL(R.y, J + 0), WG_SER_RL(R.z, J + 0));
    ser_step1<J + 1>(D, out, WG_SER_RL(R.x, J + 1), WG_SER_RL(R.y, J + 1), WG_SER_RL(R.z, J + 1));
    ser_step1<J + 2>(D, out, WG_SER_RL(R.x, J + 2), WG_SER_RL(R.y, J + 2), WG_SER_RL(R.z, J + 2));
    ser_step1<J + 3>(D, out, WG_SER_RL(R.x, J + 3), WG_SER_RL(R.y, J + 3), WG_SER_RL(R.z, J + 3));
#undef WG_SER_RL
}


// Wider occupancies (64 NW - 1 slots): per event one compare per word, the
// lowest selected slot over the words (s_ff1 of each word, tagged with the
// word, unsigned minimum: an empty word's -1 stays the largest), the lane
// write by compare + select on every word (its word is not a compile-time
// register).  Nothing selected: x = 0xFFFFFFFF, no lane written.
template <int NW>
__device__ __forceinline__ uint32_t ser_first_w(const uint64_t (&m)[NW]);
template <>
__device__ __forceinline__ uint32_t ser_first_w<1>(const uint64_t (&m)[1]) {
    uint32_t x;
    asm volatile("s_ff1_i32_b64 %[x], %[m0]" : [x] "=s"(x) : [m0] "s"(m[0]));
    return x;
}
template <>
__device__ __forceinline__ uint32_t ser_first_w<2>(const uint64_t (&m)[2]) {
    uint32_t x, f1;   // (as the four-word form)
    asm volatile(
        "s_ff1_i32_b64 %[x], %[m0]\n\t"
        "s_ff1_i32_b64 %[f1], %[m1]\n\t"
        "s_or_b32 %[f1], %[f1], 64\n\t"
        "s_min_u32 %[x], %[x], %[f1]"
        : [x] "=&s"(x), [f1] "=&s"(f1)
        : [m0] "s"(m[0]), [m1] "s"(m[1])
        : "scc");
    return x;
}
template <>
__device__ __forceinline__ uint32_t ser_first_w<4>(const uint64_t (&m)[4]) {
    uint32_t x, f1, f2, f3;   // (wave-uniform scalar arithmetic kept in one asm block: the
                              // compiler takes asm results for divergent and would move it to VALU)
    asm volatile(
        "s_ff1_i32_b64 %[x], %[m0]\n\t"
        "s_ff1_i32_b64 %[f1], %[m1]\n\t"
        "s_ff1_i32_b64 %[f2], %[m2]\n\t"
        "s_ff1_i32_b64 %[f3], %[m3]\n\t"
        "s_or_b32 %[f1], %[f1], 64\n\t"
        "s_or_b32 %[f2], %[f2], 0x80\n\t"
        "s_or_b32 %[f3], %[f3], 0xc0\n\t"
        "s_min_u32 %[x], %[x], %[f1]\n\t"
        "s_min_u32 %[f2], %[f2], %[f3]\n\t"
        "s_min_u32 %[x], %[x], %[f2]"
        : [x] "=&s"(x), [f1] "=&s"(f1), [f2] "=&s"(f2), [f3] "=&s"(f3)
        : [m0] "s"(m[0]), [m1] "s"(m[1]), [m2] "s"(m[2]), [m3] "s"(m[3])
        : "scc");
    return x;
}
template <>
__device__ __forceinline__ uint32_t ser_first_w<3>(const uint64_t (&m)[3]) {
    uint32_t x, f1, f2;   // (as the four-word form)
    asm volatile(
        "s_ff1_i32_b64 %[x], %[m0]\n\t"
        "s_ff1_i32_b64 %[f1], %[m1]\n\t"
        "s_ff1_i32_b64 %[f2], %[m2]\n\t"
        "s_or_b32 %[f1], %[f1], 64\n\t"
        "s_or_b32 %[f2], %[f2], 0x80\n\t"
        "s_min_u32 %[x], %[x], %[f1]\n\t"
        "s_min_u32 %[x], %[x], %[f2]"
        : [x] "=&s"(x), [f1] "=&s"(f1), [f2] "=&s"(f2)
        : [m0] "s"(m[0]), [m1] "s"(m[1]), [m2] "s"(m[2])
        : "scc");
    return x;
}
template <>
__device__ __forceinline__ uint32_t ser_first_w<8>(const uint64_t (&m)[8]) {
    uint32_t x = 0xFFFFFFFFu;
#pragma unroll
    for (int w = 7; w >= 0; w--) {
        uint32_t f;
        asm volatile("s_ff1_i32_b64 %[f], %[m]\n\t"
                     "s_or_b32 %[f], %[f], %[tag]\n\t"
                     "s_min_u32 %[x], %[x], %[f]"
                     : [x] "+s"(x), [f] "=&s"(f) : [m] "s"(m[w]), [tag] "n"(64 * w) : "scc");
    }
    return x;
}
template <>
__device__ __forceinline__ uint32_t ser_first_w<16>(const uint64_t (&m)[16]) {
    uint32_t x = 0xFFFFFFFFu;
#pragma unroll
    for (int w = 15; w >= 0; w--) {
        uint32_t f;
        asm volatile("s_ff1_i32_b64 %[f], %[m]\n\t"
                     "s_or_b32 %[f], %[f], %[tag]\n\t"
                     "s_min_u32 %[x], %[x], %[f]"
                     : [x] "+s"(x), [f] "=&s"(f) : [m] "s"(m[w]), [tag] "n"(64 * w) : "scc");
    }
    return x;
}

template <int NW, int J>
__device__ __forceinline__ void ser_step_w(uint32_t (&D)[NW], uint32_t &out, uint32_t lane, uint32_t lo, uint32_t wid,
                                           uint32_t dv) {
    uint64_t m[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) m[w] = __ballot(D[w] - lo < wid);
    const uint32_t x = ser_first_w<NW>(m);   // 0xFFFFFFFF: nothing selected (an overflow)
#pragma unroll
    for (int w = 0; w < NW; w++) D[w] = (lane + 64u * w == x) ? dv : D[w];
    asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(out) : "s"(x), "n"(J));
}

template <int NW, int J>
__device__ __forceinline__ void ser_quad_w(uint32_t (&D)[NW], uint32_t &out, uint32_t lane, const uint4 &R) {
#define WG_SER_RL(v, j) (uint32_t)__builtin_amdgcn_readlane((int)(v), (j))
    ser_step_w<NW, J + 0>(D, out, lane, WG_SER_RL(R.x, J + 0), WG_SER_RL(R.y, J + 0), WG_SER_RL(R.z, J + 0));
    ser_step_w<NW, J + 1>(D, out, lane, WG_SER_RL(R.x, J + 1), WG_SER_RL(R.y, J + 1), WG_SER_RL(R.z, J + 1));
    ser_step_w<NW, J + 2>(D, out, lane, WG_SER_RL(R.x, J + 2), WG_SER_RL(R.y, J + 2), WG_SER_RL(R.z, J + 2));
    ser_step_w<NW, J + 3>(D, out, lane, WG_SER_RL(R.x, J + 3), WG_SER_RL(R.y, J + 3), WG_SER_RL(R.z, J + 3));
#undef WG_SER_RL
}


}  // namespace
