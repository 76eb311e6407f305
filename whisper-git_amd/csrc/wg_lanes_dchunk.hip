// wg_lanes_dchunk.hip — the lane events replayed as a chunked fixed point on
// the D-state, with the leaked slots compacted out (r05).
//
// GraphLayout::build's lane loop (commit_graph.rs:276-295, 401-471) on the
// lists commit_graph_with_orphans delivers (git/mod.rs:767-772: reflog orphans
// re-sorted by time, so a child older than a clock-skewed parent sits below
// it) leaks a slot for every parent at an earlier row: the slot set to wait
// for it is never freed (:441-446, :287-291 only runs at the parent's own
// row).  A chunk replayed from an empty table does not know those slots, so
// its "lowest free slot" is wrong for the rest of the list, and the chunked
// fixed point of wg_lanes_replay.hip advances about one chunk per iteration
// (profiles/r04_replay_shapes.jsonl).  Here:
//
//  * positions instead of slots: a leaked slot stays occupied for good, so the
//    lowest free slot is the lowest free one among the never-leaked slots.
//    The replay runs on the ranks of the non-leaked slots ("positions"): an
//    event that leaks its slot (an occupying event whose token no event
//    consumes — known before the replay) removes its position, the positions
//    above it move down by one.  The greedy on positions is the greedy on
//    slots with the leaked ones struck out, order preserved.
//  * the D-state (wg_lanes_dstep.h): a position holds the time its holder is
//    consumed, so a chunk's state is one D-vector and a replay needs no token
//    lookups.  Iteration 1 replays every chunk from an empty table `warm`
//    events early (one wave per chunk); iteration i > 1 starts chunk c from
//    chunk c - 1's exit D-vector of iteration i - 1.  Free positions are
//    normalised to 0 at the exit, so a warm-started exit that found the live
//    holders equals the exact one.  An iteration that changes no position and
//    no exit vector is the fixed point (chunk 0 is exact, and by induction
//    every chunk's replay from its predecessor's exact exit is exact).  With
//    the leaked slots struck out the state forgets within a few thousand
//    events: profiles/replay_sim.c `compact` reaches the fixed point at
//    iteration 2 with an 8192-event warm-up on the skewed 1M- and 8M-row lists
//    and the Linux shape (r05_compact_sim.jsonl).
//  * slots from positions afterwards: after j leaks the non-leaked slots in
//    order are S_j (S_0 = identity; a leak at position x drops S[x], the top
//    position gets the next unused slot).  k_dc_snap builds every S_j in one
//    pass over the leaks (their positions are final); the slot of event k is
//    S_{leaks before k}[position of k] (k_dc_fix, one thread per event, with
//    max_lane / n_slots, :462-471).
#include <utility>

#include "wg_internal.h"
#include "wg_lanes_dstep.h"

namespace {

enum : uint32_t { F_A = 1u, F_O = 2u, F_C = 4u };
constexpr uint32_t DC_NEVER = 0xFFFFFFFFu;   // death[]: the token is never consumed (a leak if it occupies)
constexpr uint32_t DC_FIX_T = WG_DC_FIX_T;   // k_dc_fix: events per block (one stats record each)

struct DcArgs {
    const uint4 *ev;              // event records (flags in .x)
    const uint32_t *death;        // per event: the time of the event consuming its token, or DC_NEVER
    uint64_t nev;                 // events (the bound when nev_dev is set)
    const uint32_t *nev_dev;      // speculative build: the event count on the device
    const uint32_t *gate;         // speculative build: nonzero = not well formed, replay nothing
    uint32_t chunk, warm, iter;
    uint32_t *changed;            // [iter] = 1: iteration iter changed something
    const uint32_t *dprev;        // exit D-vectors of iteration iter - 1, [chunk][64 NW]
    uint32_t *dnext;
    const uint16_t *pprev;        // positions per event, iteration iter - 1
    uint16_t *pnext;
    unsigned long long *lkmask;   // per 64-event batch: the events that leak (written by iteration 1)
};

// the record of event k for the D-step {lo, wid, dv}; past e1: selects nothing
__device__ __forceinline__ uint4 dc_record(uint64_t k, uint64_t e1, uint32_t f, uint32_t dth, bool &leak) {
    leak = false;
    uint4 R = make_uint4(0u, 0u, WG_SER_INF, 0u);
    if (k < e1) {
        const uint32_t t = (uint32_t)k + 1u;
        R.x = (f & F_A) ? 0u : t;
        R.y = (f & F_A) ? t : 1u;
        if (f & F_O) {
            leak = dth == DC_NEVER;
            R.z = leak ? WG_SER_INF : dth;
        } else {
            R.z = t;   // not occupying: free after this event
        }
    }
    return R;
}

// drop position x (< 64 NW - 1): positions above move down one, the top
// regular position (64 NW - 2) becomes a free never-used slot; the sentinel
// (64 NW - 1) stays held
template <int NW>
__device__ __forceinline__ void dc_remove(uint32_t (&D)[NW], uint32_t x, uint32_t lane) {
    uint32_t nx[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) {
        uint32_t v = (uint32_t)__shfl_down((int)D[w], 1, 64);   // lane l <- lane l + 1
        const uint32_t carry = (w + 1 < NW) ? (uint32_t)__builtin_amdgcn_readfirstlane((int)D[w + 1 < NW ? w + 1 : w]) : 0u;
        if (lane == 63) v = carry;
        nx[w] = v;
    }
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const uint32_t p = 64u * w + lane;
        if (p == 64u * NW - 2u) D[w] = 0u;
        else if (p >= x && p < 64u * NW - 2u) D[w] = nx[w];
    }
}

// a batch holding a leaking event: the events one at a time, the leaks removed
template <int NW>
__device__ __forceinline__ void dc_batch_slow(uint32_t (&D)[NW], uint32_t &out, uint32_t lane, const uint4 &R,
                                           unsigned long long lkm) {
    constexpr uint32_t cap = 64u * NW - 1u;
    for (uint32_t J = 0; J < 64; J++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)R.x, (int)J);
        const uint32_t wid = (uint32_t)__builtin_amdgcn_readlane((int)R.y, (int)J);
        const uint32_t dv = (uint32_t)__builtin_amdgcn_readlane((int)R.z, (int)J);
        uint64_t m[NW];
#pragma unroll
        for (int w = 0; w < NW; w++) m[w] = __ballot(D[w] - lo < wid);
        uint32_t x = 0xFFFFFFFFu;
#pragma unroll
        for (int w = NW - 1; w >= 0; w--)
            if (m[w]) x = 64u * w + (uint32_t)__builtin_ctzll(m[w]);
        if (x < cap && ((lkm >> J) & 1ull)) dc_remove<NW>(D, x, lane);
        else if (x != 0xFFFFFFFFu) {
#pragma unroll
            for (int w = 0; w < NW; w++) D[w] = (lane + 64u * w == x) ? dv : D[w];
        }
        out = (lane == J) ? x : out;
    }
}

template <int NW>
__device__ __forceinline__ void dc_batch_fast(uint32_t (&D)[NW], uint32_t &out, uint32_t lane, const uint4 &R) {
    if constexpr (NW == 1) {
        ser_quad1<0>(D[0], out, R);   ser_quad1<4>(D[0], out, R);   ser_quad1<8>(D[0], out, R);   ser_quad1<12>(D[0], out, R);
        ser_quad1<16>(D[0], out, R);  ser_quad1<20>(D[0], out, R);  ser_quad1<24>(D[0], out, R);  ser_quad1<28>(D[0], out, R);
        ser_quad1<32>(D[0], out, R);  ser_quad1<36>(D[0], out, R);  ser_quad1<40>(D[0], out, R);  ser_quad1<44>(D[0], out, R);
        ser_quad1<48>(D[0], out, R);  ser_quad1<52>(D[0], out, R);  ser_quad1<56>(D[0], out, R);  ser_quad1<60>(D[0], out, R);
    } else {
        ser_quad_w<NW, 0>(D, out, lane, R);   ser_quad_w<NW, 4>(D, out, lane, R);
        ser_quad_w<NW, 8>(D, out, lane, R);   ser_quad_w<NW, 12>(D, out, lane, R);
        ser_quad_w<NW, 16>(D, out, lane, R);  ser_quad_w<NW, 20>(D, out, lane, R);
        ser_quad_w<NW, 24>(D, out, lane, R);  ser_quad_w<NW, 28>(D, out, lane, R);
        ser_quad_w<NW, 32>(D, out, lane, R);  ser_quad_w<NW, 36>(D, out, lane, R);
        ser_quad_w<NW, 40>(D, out, lane, R);  ser_quad_w<NW, 44>(D, out, lane, R);
        ser_quad_w<NW, 48>(D, out, lane, R);  ser_quad_w<NW, 52>(D, out, lane, R);
        ser_quad_w<NW, 56>(D, out, lane, R);  ser_quad_w<NW, 60>(D, out, lane, R);
    }
}

// One iteration, one wave per chunk.  FIRST: from an empty table `warm`
// events before the chunk (never the fixed point); else from chunk c - 1's
// exit of the previous iteration.
template <int NW, bool FIRST>
__global__ void __launch_bounds__(64) k_dc_iter(DcArgs A) {
    constexpr uint32_t top = 64u * NW - 1u;   // the sentinel position
    if (!FIRST && A.changed[A.iter - 1] == 0) return;   // the previous iteration was the fixed point
    if (A.gate && *A.gate) return;
    const uint64_t nev = A.nev_dev ? (uint64_t)*A.nev_dev : A.nev;
    const uint64_t c = blockIdx.x, e0 = c * A.chunk;
    if (e0 >= nev) return;
    const uint64_t e1 = e0 + A.chunk < nev ? e0 + A.chunk : nev;
    const uint64_t ew = FIRST ? (e0 > A.warm ? e0 - A.warm : 0) : e0;
    const uint32_t lane = threadIdx.x;
    uint32_t D[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const uint32_t p = 64u * w + lane;
        D[w] = (FIRST || c == 0) ? 0u : A.dprev[(c - 1) * (64u * NW) + p];
        if (p == top) D[w] = WG_SER_INF;
    }
    // records two batches ahead (the warm-up streams thousands of events)
    uint32_t f1 = 0, d1 = 0, f2 = 0, d2 = 0;
    if (ew + lane < e1) { f1 = A.ev[ew + lane].x; d1 = A.death[ew + lane]; }
    if (ew + 64 + lane < e1) { f2 = A.ev[ew + 64 + lane].x; d2 = A.death[ew + 64 + lane]; }
    bool diff = false;
    for (uint64_t base = ew; base < e1; base += 64) {
        const uint64_t k = base + lane;
        bool leak;
        const uint4 R = dc_record(k, e1, f1, d1, leak);
        f1 = f2; d1 = d2;
        if (base + 128 + lane < e1) { f2 = A.ev[base + 128 + lane].x; d2 = A.death[base + 128 + lane]; }
        const unsigned long long lkm = __ballot(leak);
        uint32_t out = 0xFFFFFFFFu;
        if (lkm) dc_batch_slow<NW>(D, out, lane, R, lkm);
        else dc_batch_fast<NW>(D, out, lane, R);
        if (base >= e0) {
            if (k < e1) {
                A.pnext[k] = (uint16_t)out;
                if (!FIRST) diff |= A.pprev[k] != (uint16_t)out;
            }
            if (FIRST && lane == 0) A.lkmask[base >> 6] = lkm;
        }
    }
    // the exit: free positions read 0, the sentinel held
    bool dchg = false;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const uint32_t p = 64u * w + lane;
        uint32_t v = D[w] <= (uint32_t)e1 ? 0u : D[w];
        if (p == top) v = WG_SER_INF;
        A.dnext[c * (64u * NW) + p] = v;
        if (!FIRST) dchg |= A.dprev[c * (64u * NW) + p] != v;
    }
    if (FIRST || __any(diff || dchg)) A.changed[A.iter] = 1u;
}

// After the fixed point: the leaks' prefix per 64-event batch (bpre), the
// leak list, and S_j for every j (snap[j][position], u16).  One block.
// scal[5] = leaks; more than leak_cap: scal[6] = 1 (the snapshots would not
// fit; the caller replays serially).
template <int NW>
__global__ void __launch_bounds__(1024) k_dc_snap(uint64_t nev_cap, const uint32_t *__restrict__ nev_dev,
                                                  const uint32_t *__restrict__ gate, const unsigned long long *__restrict__ lkmask,
                                                  const uint16_t *__restrict__ pos, uint32_t *__restrict__ bpre,
                                                  uint32_t *__restrict__ lklist, uint16_t *__restrict__ snap, uint32_t leak_cap,
                                                  uint32_t *__restrict__ scal) {
    constexpr uint32_t W = 64u * NW, cap = W - 1u;
    __shared__ uint32_t ws[16];
    __shared__ uint32_t carry_s;
    __shared__ uint16_t lpos[1024];
    if (gate && *gate) return;
    const uint64_t nev = nev_dev ? (uint64_t)*nev_dev : nev_cap;
    const uint64_t nb = (nev + 63) / 64;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    // 1. exclusive prefix of the batch popcounts; the leak list in event order
    for (uint64_t b0 = 0; b0 < nb; b0 += 1024) {
        const uint64_t b = b0 + tid;
        const unsigned long long m = b < nb ? lkmask[b] : 0ull;
        const uint32_t v = (uint32_t)__builtin_popcountll(m);
        const uint32_t inc = wg_wave_scan(v, 0u, [](uint32_t a, uint32_t q) { return a + q; });
        if (lane == 63) ws[wv] = inc;
        __syncthreads();
        uint32_t before = carry_s;
        for (uint32_t q = 0; q < wv; q++) before += ws[q];
        const uint32_t ex = before + inc - v;
        if (b < nb) {
            bpre[b] = ex;
            unsigned long long mm = m;
            for (uint32_t q = ex; mm; q++) {
                const uint32_t bit = (uint32_t)__builtin_ctzll(mm);
                mm &= mm - 1;
                if (q < leak_cap) lklist[q] = (uint32_t)(b * 64 + bit);
            }
        }
        __syncthreads();
        if (tid == 1023) carry_s = before + inc;
        __syncthreads();
    }
    const uint32_t total = carry_s;
    if (tid == 0) {
        scal[5] = total;
        scal[6] = total > leak_cap ? 1u : 0u;
    }
    if (total > leak_cap) return;
    // 2. S_j: wave 0 walks the leaks in order, their positions staged 1024 at a time
    uint32_t S[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) S[w] = 64u * w + lane;
    if (wv == 0)
#pragma unroll
        for (int w = 0; w < NW; w++) snap[64u * w + lane] = (uint16_t)S[w];
    for (uint32_t j0 = 0; j0 < total; j0 += 1024) {
        __syncthreads();
        if (j0 + tid < total) lpos[tid] = pos[lklist[j0 + tid]];
        __syncthreads();
        if (wv != 0) continue;
        const uint32_t jn = total - j0 < 1024u ? total - j0 : 1024u;
        for (uint32_t j = 0; j < jn; j++) {
            const uint32_t x = lpos[j];
            if (x < cap) {   // (past the sentinel: an overflowed replay, which k_dc_fix reports)
                const uint32_t topv = (uint32_t)__builtin_amdgcn_readlane((int)S[NW - 1], 62);   // position W - 2
                uint32_t nx[NW];
#pragma unroll
                for (int w = 0; w < NW; w++) {
                    uint32_t v = (uint32_t)__shfl_down((int)S[w], 1, 64);
                    const uint32_t cr = (w + 1 < NW) ? (uint32_t)__builtin_amdgcn_readfirstlane((int)S[w + 1 < NW ? w + 1 : w]) : 0u;
                    if (lane == 63) v = cr;
                    nx[w] = v;
                }
#pragma unroll
                for (int w = 0; w < NW; w++) {
                    const uint32_t p = 64u * w + lane;
                    if (p == W - 2u) S[w] = topv + 1u;
                    else if (p >= x && p < W - 2u) S[w] = nx[w];
                }
            }
#pragma unroll
            for (int w = 0; w < NW; w++)
                snap[(uint64_t)(j0 + j + 1) * W + 64u * w + lane] = (uint16_t)(S[w] < 0xFFFFu ? S[w] : 0xFFFFu);
        }
    }
}

// the slot of every event: S_{leaks before k}[position of k]; per block
// {max_lane, highest allocated slot (0xFFFF: overflow), highest allocated
// position}
template <int NW>
__global__ void __launch_bounds__(DC_FIX_T) k_dc_fix(uint64_t nev_cap, const uint32_t *__restrict__ nev_dev,
                                                     const uint32_t *__restrict__ gate, const uint4 *__restrict__ ev,
                                                     const unsigned long long *__restrict__ lkmask,
                                                     const uint32_t *__restrict__ bpre, const uint16_t *__restrict__ pos,
                                                     const uint16_t *__restrict__ snap, uint16_t *__restrict__ slot,
                                                     uint32_t *__restrict__ stats, const uint32_t *__restrict__ scal) {
    constexpr uint32_t W = 64u * NW, cap = W - 1u;
    __shared__ uint32_t red[3][DC_FIX_T / 64];
    if (gate && *gate) return;
    const uint64_t nev = nev_dev ? (uint64_t)*nev_dev : nev_cap;
    const uint64_t k = (uint64_t)blockIdx.x * DC_FIX_T + threadIdx.x;
    const bool snap_ok = scal[6] == 0;
    uint32_t ml = 0, ms = 0, mp = 0;
    if (k < nev) {
        const uint32_t x = pos[k];
        const uint32_t f = ev[k].x;
        const unsigned long long m = lkmask[k >> 6];
        const uint32_t e = bpre[k >> 6] + (uint32_t)__builtin_popcountll(m & ((1ull << (k & 63)) - 1ull));
        uint32_t s = 0xFFFFu;
        if (x < cap && snap_ok) s = snap[(uint64_t)e * W + x];
        if (s >= 0xFFFFu) ms = 0xFFFFu;   // overflow (a position past the width, or a slot past u16)
        else {
            if (f & F_O) ml = s;
            if (f & F_A) { ms = s; mp = x; }
        }
        slot[k] = (uint16_t)s;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t a = (uint32_t)__shfl_xor((int)ml, d, 64), b = (uint32_t)__shfl_xor((int)ms, d, 64),
                       q = (uint32_t)__shfl_xor((int)mp, d, 64);
        ml = a > ml ? a : ml;
        ms = b > ms ? b : ms;
        mp = q > mp ? q : mp;
    }
    const uint32_t wv = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { red[0][wv] = ml; red[1][wv] = ms; red[2][wv] = mp; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t q = 1; q < DC_FIX_T / 64; q++) {
            ml = red[0][q] > ml ? red[0][q] : ml;
            ms = red[1][q] > ms ? red[1][q] : ms;
            mp = red[2][q] > mp ? red[2][q] : mp;
        }
        stats[3 * blockIdx.x] = ml;
        stats[3 * blockIdx.x + 1] = ms;
        stats[3 * blockIdx.x + 2] = mp;
    }
}

__global__ void k_dc_init(uint32_t *changed, uint32_t nflags) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nflags) changed[i] = i == 0 ? 1u : 0u;
}

template <int NW>
void launch_iter(hipStream_t s, const DcArgs &a, uint64_t nch, bool first) {
    if (first) hipLaunchKernelGGL((k_dc_iter<NW, true>), dim3((uint32_t)nch), dim3(64), 0, s, a);
    else hipLaunchKernelGGL((k_dc_iter<NW, false>), dim3((uint32_t)nch), dim3(64), 0, s, a);
}

}  // namespace

uint32_t wg_dc_words(uint32_t positions) { return positions < 64 ? 1u : positions < 128 ? 2u : positions < 256 ? 4u : 0u; }

// iterations R.it + 1 .. R.it + n (the first of a run is the warm-started one)
hipError_t wg_dc_iterate(hipStream_t s, ReplayRun &R, uint32_t n) {
    R.nch = (R.nev + R.chunk - 1) / R.chunk;
    if (R.dc_pos && R.sp_prev == R.dc_slot) R.sp_prev = R.dc_pos;   // (more iterations after a finish)
    for (uint32_t q = 0; q < n && R.it < R.max_iters; q++) {
        R.it++;
        DcArgs a{R.ev, R.death, R.nev, R.nev_dev, R.gate, R.chunk, R.warm, R.it, R.flags,
                 R.dc_dvec[R.it & 1], R.dc_dvec[(R.it + 1) & 1], R.sp_prev, R.sp_next, R.dc_lkmask};
        if (R.nch) {
            if (R.nw <= 1) launch_iter<1>(s, a, R.nch, R.it == 1);
            else if (R.nw <= 2) launch_iter<2>(s, a, R.nch, R.it == 1);
            else launch_iter<4>(s, a, R.nch, R.it == 1);
        }
        std::swap(R.sp_prev, R.sp_next);   // sp_prev: the last written positions
    }
    return hipGetLastError();
}

hipError_t wg_dc_init(hipStream_t s, ReplayRun &R, bool flags) {
    R.it = 0;
    R.sp_prev = R.slots_a;
    R.sp_next = R.slots_b;
    R.dc_pos = nullptr;
    if (!flags) return hipSuccess;
    const uint32_t nf = R.max_iters + 2;
    hipLaunchKernelGGL(k_dc_init, dim3((nf + 255) / 256), dim3(256), 0, s, R.flags, nf);
    return hipGetLastError();
}

// the slots of the positions in R.sp_prev: R.dc_slot, with the per-block stats
// the finish kernels reduce (R.dc_pos = the positions)
hipError_t wg_dc_finish(hipStream_t s, ReplayRun &R) {
    R.dc_pos = R.sp_prev;
    const uint64_t nb = (R.nev + DC_FIX_T - 1) / DC_FIX_T;
    R.dc_blocks = nb;
#define WG_DC_FIN(NW)                                                                                                     \
    do {                                                                                                                  \
        hipLaunchKernelGGL(k_dc_snap<NW>, dim3(1), dim3(1024), 0, s, R.nev, R.nev_dev, R.gate,                            \
                           (const unsigned long long *)R.dc_lkmask, (const uint16_t *)R.dc_pos, R.dc_bpre, R.dc_lklist,   \
                           R.dc_snap, R.dc_leak_cap, R.scal);                                                             \
        if (nb)                                                                                                           \
            hipLaunchKernelGGL(k_dc_fix<NW>, dim3((uint32_t)nb), dim3(DC_FIX_T), 0, s, R.nev, R.nev_dev, R.gate, R.ev,    \
                               (const unsigned long long *)R.dc_lkmask, (const uint32_t *)R.dc_bpre,                      \
                               (const uint16_t *)R.dc_pos, (const uint16_t *)R.dc_snap, R.dc_slot, R.stats,               \
                               (const uint32_t *)R.scal);                                                                 \
    } while (0)
    if (R.nw <= 1) WG_DC_FIN(1);
    else if (R.nw <= 2) WG_DC_FIN(2);
    else WG_DC_FIN(4);
#undef WG_DC_FIN
    R.sp_prev = R.dc_slot;   // what the lane kernels read as the slot of an event
    return hipGetLastError();
}

uint64_t wg_dc_fix_blocks(uint64_t nev) { return (nev + DC_FIX_T - 1) / DC_FIX_T; }
