// wg_lanes_serial.hip — exact single-wave replay of the lane events
// (wg_lanes_fast.hip's event stream) for the lists whose greedy state does not
// forget: GraphLayout::build's lane loop (commit_graph.rs:276-295, 401-471)
// leaks a slot for every parent at an earlier row (:441-446, clock skew after
// commit_graph_with_orphans re-sorts by time, git/mod.rs:767-772) and keeps
// long-lived lanes, so a chunk replayed from a guessed entry state is wrong
// until the guess is exact, and the chunked fixed point of wg_lanes_replay.hip
// advances by about one chunk per iteration (profiles/r04_replay_shapes.jsonl:
// 562 iterations for the 128-event chunks of the skewed 1M-row list).  This
// replay is exact in one pass: no fixed point, no guess.
//
// State: lane l of the wave owns slot l (word w of a lane: slot 64 w + l) and
// holds D = the time its holder's chain is consumed (event k has time k + 1;
// 0 = never held; WG_SER_INF = leaked, never consumed).  A token's consumption
// event is structural (the MIN / FREE event that lists it), so it is known
// before the replay, and the replay never looks a token's slot up:
//   ALLOC at k    the slots free at k are those with D < k + 1 (their holder
//                 was consumed before k): the lowest (lowest_free_lane,
//                 :414-423) takes the token; its D = the token's consumption
//                 time (or k + 1 if it does not occupy: a probe allocation)
//   MIN / FREE    the waiters are the slots with D == k + 1 (every token the
//                 event consumes); the lowest keeps the new chain (:287-291 with
//                 find_or_assign_lane's lowest waiter) with the event's own
//                 consumption time, the others are free from now on
// Both are "the lowest lane with D - lo < wid" for a per-event {lo, wid}, so
// one event is a subtract, a compare, a find-first-set and a lane write.
// max_lane (update_peak, :462-471) is the highest slot an occupying event
// took (every occupied slot was taken by an occupying allocation first);
// n_slots the highest slot any allocation took, plus one.
//
// The one-wave kernel is bound by its instruction issue: 8 instructions per
// event (profiles/microbench/chain_latency.hip, serial_replay.hip).
#include "wg_internal.h"
#include "wg_lanes_dstep.h"

namespace {

enum : uint32_t { F_A = 1u, F_O = 2u, F_C = 4u, F_M = 8u };
constexpr int SER_PAD = 128;   // no-op records after the last event (the last batch and the prefetch)

// Per event record rec[k] = {lo, wid, dv, 0}: lanes with D - lo < wid are
// selected (ALLOC: lo 0, wid its time k + 1 = free before it; MIN / FREE: lo
// its time, wid 1 = consumed at it); the lowest selected lane's D becomes dv
// (an occupying event: the time of the event that consumes its token, filled
// in by k_ser_death; otherwise its own time: free after it).  Past the last
// event: no-ops (select nothing; the sentinel slot takes them, its lane stays
// leaked).
__global__ void k_ser_rec(uint64_t nev_cap, const uint32_t *__restrict__ nev_dev, const uint32_t *__restrict__ gate,
                          const uint4 *__restrict__ ev, uint4 *__restrict__ rec) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nev_cap + SER_PAD) return;
    if (gate && *gate) return;   // not well formed: nothing is replayed
    const uint64_t nev = nev_dev ? (uint64_t)*nev_dev : nev_cap;
    uint4 o = make_uint4(0u, 0u, WG_SER_INF, 0u);
    if (k < nev) {
        const uint32_t f = ev[k].x, t = (uint32_t)k + 1u;
        if (f & F_A) { o.x = 0u; o.y = t; }
        else { o.x = t; o.y = 1u; }
        o.z = (f & F_O) ? WG_SER_INF : t;
    }
    rec[k] = o;
}

// consumption times: every MIN / FREE event k writes its time k + 1 as the
// new D of the tokens it consumes (after k_ser_rec; tokens never consumed
// keep WG_SER_INF: leaked)
__global__ void k_ser_death(uint64_t nev_cap, const uint32_t *__restrict__ nev_dev, const uint32_t *__restrict__ gate,
                            const uint4 *__restrict__ ev, const uint32_t *__restrict__ aux, uint4 *__restrict__ rec) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gate && *gate) return;
    const uint64_t nev = nev_dev ? (uint64_t)*nev_dev : nev_cap;
    if (k >= nev) return;
    const uint4 r = ev[k];
    if (!(r.x & F_C)) return;
    const uint32_t t = (uint32_t)k + 1u;
    if (r.x & F_M) {   // (a token past the events is not written through)
        const uint32_t n = aux[r.w];
        for (uint32_t q = 0; q < n; q++) {
            const uint32_t tk = aux[r.w + 1 + q];
            if (tk < nev) rec[tk].z = t;
        }
    } else {
        if (r.y < nev) rec[r.y].z = t;
        if (r.z < nev) rec[r.z].z = t;
    }
}

// ---- the one-wave replay, up to 63 slots (slot 63 is the sentinel) --------
// The D-step of wg_lanes_dstep.h: the batch's records sit one per lane, loaded
// a batch ahead (scalar loads return out of order and any wait for one waits
// for all).  Software-pipelining the next event's compare ahead of this lane
// write needs a scalar patch and a fourth record word: 12 instructions,
// slower (profiles/r04_serial_variants.md).
//
// the batch's outputs: slots, and the running maxima (occupying events /
// allocations; a slot at the sentinel or beyond is an overflow)
__device__ __forceinline__ void ser_flush(uint64_t base, uint64_t nev, uint32_t lane, uint32_t x, const uint4 *__restrict__ ev,
                                          uint16_t *__restrict__ slot, uint32_t cap, uint32_t &ml, uint32_t &ms, uint32_t &ovf) {
    const uint64_t k = base + lane;
    if (k >= nev) return;
    slot[k] = (uint16_t)x;
    const uint32_t f = ev[k].x;
    if (x >= cap) { ovf = 1u; return; }
    if (f & F_O) ml = x > ml ? x : ml;       // occupying
    if (f & F_A) ms = x > ms ? x : ms;       // allocation
}

__device__ __forceinline__ void ser_finish(uint32_t lane, uint32_t ml, uint32_t ms, uint32_t ovf, uint32_t cap,
                                           uint32_t *__restrict__ stats, uint32_t *__restrict__ flags,
                                           uint32_t *__restrict__ scal) {
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t a = (uint32_t)__shfl_xor((int)ml, d, 64), b = (uint32_t)__shfl_xor((int)ms, d, 64),
                       o = (uint32_t)__shfl_xor((int)ovf, d, 64);
        ml = a > ml ? a : ml;
        ms = b > ms ? b : ms;
        ovf |= o;
    }
    if (lane == 0) {
        // one "chunk" (wg_lanes_replay.hip's replay_finish reduces these): max_lane,
        // the highest allocated slot (the sentinel when the occupancy overflowed)
        stats[0] = ml;
        stats[1] = ovf ? cap : ms;
        flags[0] = 1u;   // "iteration 1 changed something, iteration 2 nothing": converged
        flags[1] = 0u;
        // the lane scalars as replay_finish leaves them: max_lane, slots, overflow, first still iteration
        scal[0] = ml;
        scal[1] = (ovf ? cap : ms) + 1u;
        scal[2] = ovf;
        scal[3] = 1u;
    }
}

__global__ void __launch_bounds__(64) k_ser_replay1(const uint4 *__restrict__ rec, const uint4 *__restrict__ ev,
                                                    uint64_t nev_cap, const uint32_t *__restrict__ nev_dev,
                                                    const uint32_t *__restrict__ gate, uint16_t *__restrict__ slot,
                                                    uint32_t *__restrict__ stats, uint32_t *__restrict__ flags,
                                                    uint32_t *__restrict__ scal) {
    if (gate && *gate) return;
    const uint32_t lane = threadIdx.x;
    const uint64_t nev = nev_dev ? (uint64_t)*nev_dev : nev_cap;
    uint32_t ml = 0, ms = 0, ovf = 0;
    uint32_t D = lane == 63 ? WG_SER_INF : 0u;   // the sentinel slot is held for good
    uint4 R = rec[lane];
    for (uint64_t base = 0; base < nev; base += 64) {
        const uint4 Rn = rec[base + 64 + lane];   // the next batch (no-ops past the last event)
        uint32_t out = 0xFFFFu;
        ser_quad1<0>(D, out, R);   ser_quad1<4>(D, out, R);   ser_quad1<8>(D, out, R);   ser_quad1<12>(D, out, R);
        ser_quad1<16>(D, out, R);  ser_quad1<20>(D, out, R);  ser_quad1<24>(D, out, R);  ser_quad1<28>(D, out, R);
        ser_quad1<32>(D, out, R);  ser_quad1<36>(D, out, R);  ser_quad1<40>(D, out, R);  ser_quad1<44>(D, out, R);
        ser_quad1<48>(D, out, R);  ser_quad1<52>(D, out, R);  ser_quad1<56>(D, out, R);  ser_quad1<60>(D, out, R);
        ser_flush(base, nev, lane, out, ev, slot, 63u, ml, ms, ovf);
        R = Rn;
    }
    ser_finish(lane, ml, ms, ovf, 63u, stats, flags, scal);
}

// ---- wider occupancies (64 NW - 1 slots, NW = 3, 4, 8 or 16): slot 64 w + l
// is lane l of word w (ser_step_w, wg_lanes_dstep.h).  Records as the
// one-word kernel's: a batch per lane, read out with v_readlane.
template <int NW>
__global__ void __launch_bounds__(64) k_ser_replay_w(const uint4 *__restrict__ rec, const uint4 *__restrict__ ev,
                                                     uint64_t nev_cap, const uint32_t *__restrict__ nev_dev,
                                                     const uint32_t *__restrict__ gate, uint16_t *__restrict__ slot,
                                                     uint32_t *__restrict__ stats, uint32_t *__restrict__ flags,
                                                     uint32_t *__restrict__ scal) {
    if (gate && *gate) return;
    const uint32_t lane = threadIdx.x;
    const uint64_t nev = nev_dev ? (uint64_t)*nev_dev : nev_cap;
    constexpr uint32_t cap = 64u * NW - 1u;
    uint32_t ml = 0, ms = 0, ovf = 0;
    uint32_t D[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) D[w] = (w == NW - 1 && lane == 63) ? WG_SER_INF : 0u;
    uint4 R = rec[lane];
    for (uint64_t base = 0; base < nev; base += 64) {
        const uint4 Rn = rec[base + 64 + lane];
        uint32_t out = 0xFFFFu;
        ser_quad_w<NW, 0>(D, out, lane, R);   ser_quad_w<NW, 4>(D, out, lane, R);
        ser_quad_w<NW, 8>(D, out, lane, R);   ser_quad_w<NW, 12>(D, out, lane, R);
        ser_quad_w<NW, 16>(D, out, lane, R);  ser_quad_w<NW, 20>(D, out, lane, R);
        ser_quad_w<NW, 24>(D, out, lane, R);  ser_quad_w<NW, 28>(D, out, lane, R);
        ser_quad_w<NW, 32>(D, out, lane, R);  ser_quad_w<NW, 36>(D, out, lane, R);
        ser_quad_w<NW, 40>(D, out, lane, R);  ser_quad_w<NW, 44>(D, out, lane, R);
        ser_quad_w<NW, 48>(D, out, lane, R);  ser_quad_w<NW, 52>(D, out, lane, R);
        ser_quad_w<NW, 56>(D, out, lane, R);  ser_quad_w<NW, 60>(D, out, lane, R);
        ser_flush(base, nev, lane, out, ev, slot, cap, ml, ms, ovf);
        R = Rn;
    }
    ser_finish(lane, ml, ms, ovf, cap, stats, flags, scal);
}

// ---- more than 1023 slots: a workgroup of MW_WAVES waves ------------------
// Wave v holds slots [256 v, 256 v + 256) as four words (the four-word step's
// compare and scalar selection); per event every wave offers its lowest
// selected slot to one LDS word (ds_min), a barrier, every wave reads the
// winner, its owner writes the lane's D and wave 0 the output lane.  Three
// words in turn: event k's winner word is read by every wave before barrier
// k + 1, and thread 0 resets it for event k + 3 after barrier k + 1.
constexpr int MW_WAVES = 16, MW_NW = 4;   // 4096 slots, the last one the sentinel
__global__ void __launch_bounds__(64 * MW_WAVES) k_ser_replay_mw(const uint4 *__restrict__ rec, const uint4 *__restrict__ ev,
                                                                uint64_t nev_cap, const uint32_t *__restrict__ nev_dev,
                                                                const uint32_t *__restrict__ gate, uint16_t *__restrict__ slot,
                                                                uint32_t *__restrict__ stats, uint32_t *__restrict__ flags,
                                                                uint32_t *__restrict__ scal) {
    __shared__ uint32_t cb[3];
    if (gate && *gate) return;   // (uniform over the block)
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t nev = nev_dev ? (uint64_t)*nev_dev : nev_cap;
    constexpr uint32_t cap = 64u * MW_NW * MW_WAVES - 1u;
    uint32_t ml = 0, ms = 0, ovf = 0;
    uint32_t D[MW_NW];
#pragma unroll
    for (int w = 0; w < MW_NW; w++) D[w] = (wv == MW_WAVES - 1 && w == MW_NW - 1 && lane == 63) ? WG_SER_INF : 0u;
    if (threadIdx.x < 3) cb[threadIdx.x] = 0xFFFFFFFFu;
    __syncthreads();
    uint4 R = rec[lane];
    uint32_t k3 = 0;
    for (uint64_t base = 0; base < nev; base += 64) {
        const uint4 Rn = rec[base + 64 + lane];
        uint32_t out = 0xFFFFu;
        for (uint32_t J = 0; J < 64; J++) {
            const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)R.x, (int)J);
            const uint32_t wid = (uint32_t)__builtin_amdgcn_readlane((int)R.y, (int)J);
            const uint32_t dv = (uint32_t)__builtin_amdgcn_readlane((int)R.z, (int)J);
            uint64_t m[MW_NW];
#pragma unroll
            for (int w = 0; w < MW_NW; w++) m[w] = __ballot(D[w] - lo < wid);
            const uint32_t x = ser_first_w<MW_NW>(m);
            if (x != 0xFFFFFFFFu && lane == 0) atomicMin(&cb[k3], x + 256u * wv);
            __syncthreads();
            uint32_t g = (uint32_t)__builtin_amdgcn_readfirstlane((int)cb[k3]);
            if (threadIdx.x == 0) cb[k3 == 0 ? 2u : k3 - 1u] = 0xFFFFFFFFu;   // event k - 1's word, for event k + 2
            if (g == 0xFFFFFFFFu) g = cap;   // nothing selected: the sentinel (an overflow, or a padding no-op)
            if ((g >> 8) == wv) {
                const uint32_t l = g & 255u;
#pragma unroll
                for (int w = 0; w < MW_NW; w++) D[w] = (lane + 64u * (uint32_t)w == l) ? dv : D[w];
            }
            asm volatile("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(out) : "s"(g), "s"(J) : "m0");
            k3 = k3 == 2u ? 0u : k3 + 1u;
        }
        if (wv == 0) ser_flush(base, nev, lane, out, ev, slot, cap, ml, ms, ovf);
        R = Rn;
    }
    if (wv == 0) ser_finish(lane, ml, ms, ovf, cap, stats, flags, scal);
}

// ---- the chunked replay's first iteration (wg_lanes_replay.hip) -----------
// Every chunk restarts `warm` events early from an empty table, so its replay
// is the serial step over [ew, e1) with this wave's own table: one wave per
// chunk, the records built in registers from the event flags and the
// consumption times (R.death).  A merge whose waiters were allocated before
// the warm-up finds fewer of them (none: x = -1, whose lane write lands on the
// sentinel): a guess, as the general kernel's zero-filled one is; iteration 1
// is never a fixed point.  Writes the chunk's slots and its exit occupancy
// (the lanes alive after it, the sentinel excluded).
__global__ void __launch_bounds__(64) k_lf_replay_first(const uint4 *__restrict__ ev, const uint32_t *__restrict__ death,
                                                        uint64_t nev_cap, const uint32_t *__restrict__ nev_dev,
                                                        const uint32_t *__restrict__ gate, uint32_t chunk, uint32_t warm,
                                                        uint16_t *__restrict__ slot_next,
                                                        unsigned long long *__restrict__ occ_next, uint32_t *__restrict__ changed) {
    if (gate && *gate) return;
    const uint64_t nev = nev_dev ? (uint64_t)*nev_dev : nev_cap;
    const uint64_t c = blockIdx.x, e0 = c * chunk;
    if (e0 >= nev) return;
    const uint64_t e1 = e0 + chunk < nev ? e0 + chunk : nev;
    const uint64_t ew = e0 > warm ? e0 - warm : 0;
    const uint32_t lane = threadIdx.x;
    uint32_t D = lane == 63 ? WG_SER_INF : 0u;
    for (uint64_t base = ew; base < e1; base += 64) {
        const uint64_t k = base + lane;
        const uint32_t t = (uint32_t)k + 1u;
        uint4 R = make_uint4(0u, 0u, WG_SER_INF, 0u);   // past the chunk: selects nothing
        if (k < e1) {
            const uint32_t f = ev[k].x;
            R.x = (f & F_A) ? 0u : t;
            R.y = (f & F_A) ? t : 1u;
            R.z = (f & F_O) ? death[k] : t;
        }
        uint32_t out = 0xFFFFu;
        ser_quad1<0>(D, out, R);   ser_quad1<4>(D, out, R);   ser_quad1<8>(D, out, R);   ser_quad1<12>(D, out, R);
        ser_quad1<16>(D, out, R);  ser_quad1<20>(D, out, R);  ser_quad1<24>(D, out, R);  ser_quad1<28>(D, out, R);
        ser_quad1<32>(D, out, R);  ser_quad1<36>(D, out, R);  ser_quad1<40>(D, out, R);  ser_quad1<44>(D, out, R);
        ser_quad1<48>(D, out, R);  ser_quad1<52>(D, out, R);  ser_quad1<56>(D, out, R);  ser_quad1<60>(D, out, R);
        if (base >= e0 && k < e1) slot_next[k] = (uint16_t)out;
    }
    const uint64_t alive = __ballot(lane != 63 && D > (uint32_t)e1);   // consumed after the chunk, or never
    if (lane == 0) {
        occ_next[c] = alive;
        changed[1] = 1u;   // a warm-started iteration is never the fixed point
    }
}

}  // namespace

// Serial replay of nev events (nev_dev: the count on the device, nev its
// upper bound; gate: nonzero = not well formed, nothing replayed) at
// occupancy width nw (1, 4, 16 words; 64: the 16-wave workgroup); slots into R.slots_a, which becomes
// the run's result (R.sp_prev); the run looks like a one-chunk replay that
// converged at iteration 1 (stats / flags / it), so the lane and scalar
// kernels of wg_lanes_replay.hip finish it unchanged.
hipError_t wg_replay_serial(hipStream_t s, ReplayRun &R, uint4 *rec) {
    R.nch = 1;
    R.chunk = 0xFFFFFFFFu;   // (replay_finish: one chunk holds every event)
    R.it = 1;
    R.sp_prev = R.slots_a;
    R.sp_next = R.slots_b;
    const uint64_t n = R.nev + SER_PAD;
    hipLaunchKernelGGL(k_ser_rec, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, R.nev, R.nev_dev, R.gate, R.ev, rec);
    if (R.nev)
        hipLaunchKernelGGL(k_ser_death, dim3((uint32_t)((R.nev + 255) / 256)), dim3(256), 0, s, R.nev, R.nev_dev, R.gate, R.ev,
                           R.aux, rec);
    const uint4 *r = rec;
    if (R.nw <= 1)
        hipLaunchKernelGGL(k_ser_replay1, dim3(1), dim3(64), 0, s, r, R.ev, R.nev, R.nev_dev, R.gate, R.slots_a, R.stats, R.flags,
                           R.scal);
    else if (R.nw <= 4 && R.ser_w3)
        hipLaunchKernelGGL(k_ser_replay_w<3>, dim3(1), dim3(64), 0, s, r, R.ev, R.nev, R.nev_dev, R.gate, R.slots_a, R.stats,
                           R.flags, R.scal);
    else if (R.nw <= 4)
        hipLaunchKernelGGL(k_ser_replay_w<4>, dim3(1), dim3(64), 0, s, r, R.ev, R.nev, R.nev_dev, R.gate, R.slots_a, R.stats,
                           R.flags, R.scal);
    else if (R.nw <= 16 && R.ser_w8)
        hipLaunchKernelGGL(k_ser_replay_w<8>, dim3(1), dim3(64), 0, s, r, R.ev, R.nev, R.nev_dev, R.gate, R.slots_a, R.stats,
                           R.flags, R.scal);
    else if (R.nw <= 16)
        hipLaunchKernelGGL(k_ser_replay_w<16>, dim3(1), dim3(64), 0, s, r, R.ev, R.nev, R.nev_dev, R.gate, R.slots_a, R.stats,
                           R.flags, R.scal);
    else
        hipLaunchKernelGGL(k_ser_replay_mw, dim3(1), dim3(64 * MW_WAVES), 0, s, r, R.ev, R.nev, R.nev_dev, R.gate, R.slots_a,
                           R.stats, R.flags, R.scal);
    return hipGetLastError();
}

uint64_t wg_replay_serial_rec_bytes(uint64_t nev) { return (nev + SER_PAD + 64) * sizeof(uint4); }

hipError_t wg_replay_first(hipStream_t s, const ReplayRun &R, uint16_t *slot_next, unsigned long long *occ_next) {
    hipLaunchKernelGGL(k_lf_replay_first, dim3((uint32_t)R.nch), dim3(64), 0, s, R.ev, R.death, R.nev, R.nev_dev, R.gate,
                       R.chunk, R.warm, slot_next, occ_next, R.flags);
    return hipGetLastError();
}
