// wg_lanes_replay.hip — the sequential core of the event-compressed lane
// assignment (wg_lanes_fast.hip): replay of the slot-occupancy events
// (SURVEY.md §7 hard part 1: "speculate-and-verify ... fixed-point iteration
// on shard entry states").
//
// The greedy's state between events is a 64-bit occupancy mask plus the
// slots of the chains still alive.  The event stream is cut into chunks of
// CH events (multiple of 64), one wave per chunk, all chunks replayed in
// parallel:
//   iteration i, chunk c:  entry occupancy = exit occupancy of chunk c-1
//                          from iteration i-1; slots of tokens born in
//                          earlier chunks read from iteration i-1's slots;
//                          writes its own event slots + exit occupancy and
//                          flags any difference from iteration i-1.
// An iteration that changes nothing is a fixed point: every chunk's output
// is its replay from its predecessors' outputs, which by induction from
// chunk 0 (exact entry: empty) IS the sequential result.  Chunk c is exact
// after at most c+1 iterations; in practice the state forgets a wrong guess
// within a few dozen events, so 2-4 iterations suffice.  The driver launches
// iterations in groups; an iteration whose predecessor changed nothing exits
// at once.
//
// Inside a chunk one wave replays 64 events per batch.  Token slots are
// resolved in parallel (previous batch by lane permute, older events from
// HBM one batch ahead); MIN / FREE events whose tokens are known have a
// fixed effect on the occupancy (clear the non-surviving token bits), folded
// with a segmented AND-scan across lanes; allocations (lowest free slot =
// ctz(~occ), :414-423), tokens born in the same batch and merges with more
// than two waiters are replayed in order by the scalar unit.  max_lane is
// the highest occupied slot after each occupying allocation (:462-471).
#include <utility>

#include "wg_internal.h"

#ifdef WG_REPLAY_PROFILE
// per iteration: [0] chunks run, [1] batches, [2] batches without scalar events,
// [3] scalar special events, [4] of which merges with > 2 waiters, [5] cycles
// per chunk (summed), [6] cycles in the scalar loop, [7] cycles in merges > 2
__device__ unsigned long long g_rp[64][8];
#define RP_ADD(i, v) atomicAdd(&g_rp[A.iter & 63][i], (unsigned long long)(v))
#endif

namespace {

enum : uint32_t { F_A = 1u, F_O = 2u, F_C = 4u, F_M = 8u, F_IN0 = 1u << 14, F_IN1 = 1u << 22 };
#ifndef WG_JMAX
#define WG_JMAX 6
#endif
constexpr int JMAX = WG_JMAX;   // speculative passes per batch before the scalar replay takes over
#ifndef WG_JMIN_ADV
#define WG_JMIN_ADV 4
#endif
constexpr int JMIN_ADV = WG_JMIN_ADV;   // lanes a pass must resolve beyond the previous one to go on

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}
__device__ __forceinline__ uint64_t rl64(uint64_t v, uint32_t lane) {
    return ((uint64_t)rl((uint32_t)(v >> 32), lane) << 32) | rl((uint32_t)v, lane);
}
// wave-uniform values loaded by every lane (global / LDS loads return VGPRs):
// moved to SGPRs so the scalar replay's occupancy stays in SGPRs (SALU chains
// instead of VALU + readlane hazards)
__device__ __forceinline__ uint32_t ufl(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t ufl64(uint64_t v) {
    return ((uint64_t)ufl((uint32_t)(v >> 32)) << 32) | ufl((uint32_t)v);
}
__device__ __forceinline__ uint64_t shfl_up64(uint64_t v, int d) {
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64);
    const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

struct ReplayArgs {
    uint64_t nev;
    uint32_t chunk;             // events per chunk (multiple of 64)
    uint32_t iter;              // iteration index (>= 1)
    const uint4 *ev;            // records, padded with >= 256 zero records
    const uint32_t *aux;        // token lists of merges with more than two waiters
    const uint16_t *slot_prev;  // iteration i-1
    uint16_t *slot_next;        // iteration i
    const unsigned long long *occ_prev;  // exit occupancy per chunk (NW words each), iteration i-1
    unsigned long long *occ_next;
    uint32_t *chunk_stats;      // per chunk: max_lane, max_slot
    uint32_t *changed;          // [iter] = 1 if iteration iter changed anything
    const uint32_t *nev_dev;    // speculative build: the event count in device memory (nev = its upper bound)
    const uint32_t *gate;       // speculative build: nonzero = the list is not well formed, replay nothing
    uint32_t warm;              // iteration 1: start this many events before the chunk (multiple of 64)
};

// The occupancy of up to 64*NW - 1 slots (active_lanes, commit_graph.rs:414-423
// grows without bound; the last bit is the overflow sentinel) as NW 64-bit
// words.  Words are only ever indexed by compile-time constants (unrolled
// loops with a compare), so the mask stays in registers.  NW = 1 is the
// common case and compiles to the single-word code.
template <int NW>
struct Occ {
    uint64_t w[NW];
    __device__ __forceinline__ static Occ fill(uint64_t v) {
        Occ m;
#pragma unroll
        for (int k = 0; k < NW; k++) m.w[k] = v;
        return m;
    }
    __device__ __forceinline__ static Occ bit(uint32_t s) {
        s &= 64u * NW - 1u;
        Occ m;
#pragma unroll
        for (int k = 0; k < NW; k++) m.w[k] = ((s >> 6) == (uint32_t)k) ? 1ull << (s & 63u) : 0ull;
        return m;
    }
    __device__ __forceinline__ Occ operator&(const Occ &o) const {
        Occ m;
#pragma unroll
        for (int k = 0; k < NW; k++) m.w[k] = w[k] & o.w[k];
        return m;
    }
    __device__ __forceinline__ Occ operator|(const Occ &o) const {
        Occ m;
#pragma unroll
        for (int k = 0; k < NW; k++) m.w[k] = w[k] | o.w[k];
        return m;
    }
    __device__ __forceinline__ Occ operator~() const {
        Occ m;
#pragma unroll
        for (int k = 0; k < NW; k++) m.w[k] = ~w[k];
        return m;
    }
    __device__ __forceinline__ bool any() const {
        uint64_t a = 0;
#pragma unroll
        for (int k = 0; k < NW; k++) a |= w[k];
        return a != 0;
    }
    __device__ __forceinline__ bool operator!=(const Occ &o) const {
        uint64_t a = 0;
#pragma unroll
        for (int k = 0; k < NW; k++) a |= w[k] ^ o.w[k];
        return a != 0;
    }
    // lowest_free_lane (:414-423): the lowest clear bit; the sentinel (last
    // bit) is never reported free, so a full table reports 64*NW - 1
    __device__ __forceinline__ uint32_t lowest_free() const {
        uint32_t r = 64u * NW - 1u;
#pragma unroll
        for (int k = NW - 1; k >= 0; k--) {
            const uint64_t f = ~w[k] | (k == NW - 1 ? 1ull << 63 : 0ull);
            if (f) r = 64u * k + (uint32_t)__builtin_ctzll(f);
        }
        return r;
    }
    // highest set bit, 0 for an empty mask
    __device__ __forceinline__ uint32_t highest() const {
        uint32_t r = 0;
#pragma unroll
        for (int k = 0; k < NW; k++)
            if (w[k]) r = 64u * k + 63u - (uint32_t)__builtin_clzll(w[k]);
        return r;
    }
    __device__ __forceinline__ Occ shfl_up(int d) const {
        Occ m;
#pragma unroll
        for (int k = 0; k < NW; k++) m.w[k] = shfl_up64(w[k], d);
        return m;
    }
    __device__ __forceinline__ Occ readlane(uint32_t lane) const {
        Occ m;
#pragma unroll
        for (int k = 0; k < NW; k++) m.w[k] = rl64(w[k], lane);
        return m;
    }
    __device__ __forceinline__ Occ xor_or_reduce() const {   // OR over the wave
        Occ m = *this;
        for (int d = 32; d >= 1; d >>= 1)
#pragma unroll
            for (int k = 0; k < NW; k++)
                m.w[k] |= ((uint64_t)(uint32_t)__shfl_xor((int)(m.w[k] >> 32), d, 64) << 32) |
                          (uint32_t)__shfl_xor((int)(uint32_t)m.w[k], d, 64);
        return m;
    }
    __device__ __forceinline__ static Occ load_uniform(const unsigned long long *p) {
        Occ m;
#pragma unroll
        for (int k = 0; k < NW; k++) m.w[k] = ufl64(p[k]);
        return m;
    }
};

// The chunk's own slots of this iteration, mirrored in LDS: a batch reads the
// slots of tokens born in the chunk's earlier batches right after the wave
// stored them, which through global memory costs a full round trip per batch.
constexpr uint32_t LSLOT_MAX = 4096;   // chunks up to this many events (WG_OPT_REPLAY_CHUNK)

template <int NW>
__global__ void __launch_bounds__(64) k_lf_replay(ReplayArgs A) {
    using M = Occ<NW>;
    __shared__ uint16_t lslot[LSLOT_MAX];
    const uint32_t lid = threadIdx.x & 63;
    if (A.changed[A.iter - 1] == 0) return;          // previous iteration was a fixed point
    if (A.gate && *A.gate) return;
    const uint64_t nev = A.nev_dev ? (uint64_t)*A.nev_dev : A.nev;
    const uint64_t c = blockIdx.x;
    const uint64_t e0 = c * A.chunk;
    if (e0 >= nev) return;
    const uint64_t e1 = (e0 + A.chunk < nev) ? e0 + A.chunk : nev;
    // Iteration 1 (no earlier iteration to take an entry state from) may start
    // `warm` events before the chunk from an empty table: the replay forgets a
    // wrong start within a few dozen events, so the chunk's own events — and
    // the next iteration's guesses — are mostly right already.  Warm-up slots
    // live in LDS only; nothing before e0 is written or counted.
    uint64_t ew = e0;
    if (A.iter == 1 && A.warm && e1 - e0 < LSLOT_MAX) {
        uint64_t w = A.warm;
        if (w > LSLOT_MAX - (e1 - e0)) w = (LSLOT_MAX - (e1 - e0)) & ~63ull;
        ew = e0 > w ? e0 - w : 0;
    }
    const bool lds = e1 - ew <= LSLOT_MAX;
#ifdef WG_REPLAY_PROFILE
    const unsigned long long rp_t0 = clock64();
    unsigned long long rp_batches = 0, rp_fast = 0, rp_sev = 0, rp_fm = 0, rp_cs = 0, rp_cfm = 0;
#endif
    // slot of a token born in this chunk before the current batch (this iteration)
    auto own = [&](uint64_t t) -> uint32_t { return lds ? (uint32_t)lslot[t - ew] : (uint32_t)A.slot_next[t]; };
    M occ = (c == 0 || ew < e0) ? M::fill(0ull) : M::load_uniform(A.occ_prev + (c - 1) * NW);
    M occ_or = M::fill(0ull), alloc_or = M::fill(0ull);   // OR of the occupancy after each occupying allocation / of allocated slots
    bool diff = false;
    uint32_t prev_v = 0;
    const uint4 *ev = A.ev;
    uint4 rec = ev[ew + lid];
    uint4 rec1 = ev[ew + 64 + lid];
    uint32_t q0_v = 0, q1_v = 0;
    // the previous iteration's slot of every event: the guess of the batch's
    // speculative replay and the reference of the change check
    uint32_t gp_v = (ew + lid >= e0 && ew + lid < e1) ? A.slot_prev[ew + lid] : 0u;
    M occ_or_v = M::fill(0ull), alloc_or_v = M::fill(0ull);   // per-lane parts of max_lane / max_s
    // old tokens of the first batch: all born before ew -> iteration i-1
    if ((rec.x & F_C) && (uint64_t)rec.y < ew) q0_v = A.slot_prev[rec.y];
    if ((rec.x & F_C) && (uint64_t)rec.z < ew) q1_v = A.slot_prev[rec.z];
    for (uint64_t base = ew; base < e1; base += 64) {
        const bool counted = base >= e0;   // (warm-up batches: no slots written, no max_lane)
        const uint32_t f_v = (base + lid < e1) ? rec.x : 0u;   // lanes past the chunk: no-op
        const uint32_t t0_v = rec.y, t1_v = rec.z, row_v = rec.w;
        const uint4 rec2 = ev[base + 128 + lid];
        const uint32_t gp_next = (base + 64 + lid >= e0 && base + 64 + lid < e1) ? A.slot_prev[base + 64 + lid] : 0u;
        // old tokens of the next batch (born before `base`): earlier chunks from
        // iteration i-1, this chunk's earlier batches from this iteration
        uint32_t n0_v = 0, n1_v = 0;
        if ((rec1.x & F_C) && (uint64_t)rec1.y < base)
            n0_v = (uint64_t)rec1.y < ew ? A.slot_prev[rec1.y] : own(rec1.y);
        if ((rec1.x & F_C) && (uint64_t)rec1.z < base)
            n1_v = (uint64_t)rec1.z < ew ? A.slot_prev[rec1.z] : own(rec1.z);
        // ---- parallel part: this lane's event ----------------------------------------
        const bool have_prev = base > ew;    // previous batch of this chunk is in prev_v
        const uint64_t pbase = base - 64;
        const uint32_t g0 = (uint32_t)__shfl((int)prev_v, (int)(t0_v & 63u), 64);
        const uint32_t g1 = (uint32_t)__shfl((int)prev_v, (int)(t1_v & 63u), 64);
        const uint32_t s0 = (have_prev && (uint64_t)t0_v >= pbase) ? g0 : q0_v;
        const uint32_t s1 = (have_prev && (uint64_t)t1_v >= pbase) ? g1 : q1_v;
        const bool isC = f_v & F_C;
        const bool special = (f_v & F_A) || (f_v & (F_IN0 | F_IN1 | F_M)) != 0;
        const uint32_t smin = s0 < s1 ? s0 : s1;
        M tokbits = M::bit(s0) | M::bit(s1);
        if (f_v & F_O) tokbits = tokbits & ~M::bit(smin);   // MIN keep: the minimum stays occupied
        const M amask = (isC && !special) ? ~tokbits : M::fill(~0ull);
        uint32_t cur_v = (isC && !special) ? smin : 0u;
        // segmented inclusive AND-scan: a segment starts right after each special lane
        M q = amask;
        uint32_t st = (lid == 0 || __shfl_up((int)special, 1, 64)) ? 1u : 0u;
        for (int d = 1; d < 64; d <<= 1) {
            const M qo = q.shfl_up(d);
            const uint32_t so = (uint32_t)__shfl_up((int)st, d, 64);
            if (lid >= (uint32_t)d && !st) { q = q & qo; st |= so; }
        }
        const uint64_t sm = __ballot(special);
        uint64_t smask = sm;
        // ---- speculative replay of the whole batch --------------------------------------
        // Every event is a map occ -> (occ & Am) | Om of the occupancy; given a
        // guess of every special event's slot, one ordered scan of the maps gives
        // the occupancy before each event and from it each event's slot
        // (allocation: lowest free slot; merge: the minimum waiter).  Iterating
        // guess <- result is exact at a fixed point (lane 0 is exact from the
        // entry occupancy, lane i once lanes < i are), and lanes before the first
        // mismatch are exact at any time, so the scalar replay below only takes
        // over from there.  The guess is the previous iteration's slot, which is
        // already right for every chunk whose entry did not change.
        // Iteration 1 has no previous slots (the guesses are the zero fill):
        // its batches go to the scalar replay directly.  Passes that stop
        // resolving lanes (fewer than JMIN_ADV more exact lanes than the
        // previous pass: the guesses are wrong throughout, as in the first
        // iterations after a chunk's entry changed) hand over to the scalar
        // replay early instead of spending all JMAX passes.
        if (sm && A.iter > 1 && !__any((f_v & F_M) != 0)) {
            const bool isA = (f_v & F_A) != 0, occupy = (f_v & F_O) != 0;
            const bool clrS = isC && special && !isA;
            const uint32_t src0 = (f_v >> 8) & 63u, src1 = (f_v >> 16) & 63u;
            uint32_t g = special ? gp_v : cur_v;
            M ob = occ, oa = occ;
            uint64_t mism = ~0ull;
            uint32_t lim_prev = 0;
            for (int it = 0; it < JMAX && mism; it++) {
                if (it > 0) {   // progress of the last pass: lanes [0, lim) are exact
                    const uint32_t lim_now = (uint32_t)__builtin_ctzll(mism);
                    if (lim_now < lim_prev + (uint32_t)JMIN_ADV) break;
                    lim_prev = lim_now;
                }
                const uint32_t ga = (uint32_t)__shfl((int)g, (int)src0, 64);
                const uint32_t gb = (uint32_t)__shfl((int)g, (int)src1, 64);
                const uint32_t a = (f_v & F_IN0) ? ga : s0, b = (f_v & F_IN1) ? gb : s1;
                const uint32_t m = a < b ? a : b;
                M Am = amask, Om = M::fill(0ull);
                if (isA) { Am = M::fill(~0ull); Om = occupy ? M::bit(g) : M::fill(0ull); }
                else if (clrS) { Am = ~(M::bit(a) | M::bit(b)); Om = occupy ? M::bit(m) : M::fill(0ull); }
                for (int d = 1; d < 64; d <<= 1) {   // inclusive scan of the maps, in event order
                    const M Ap = Am.shfl_up(d), Op = Om.shfl_up(d);
                    if (lid >= (uint32_t)d) { Om = (Op & Am) | Om; Am = Ap & Am; }
                }
                oa = (occ & Am) | Om;
                ob = oa.shfl_up(1);
                if (lid == 0) ob = occ;
                const uint32_t ng = isA ? ob.lowest_free() : (clrS ? m : cur_v);
                mism = __ballot(ng != g);   // lanes before the first mismatch kept their (exact) slot and oa
                g = ng;
            }
            // lanes [0, lim) are exact (and lane lim's slot, from an exact occupancy)
            const uint32_t lim = mism ? (uint32_t)__builtin_ctzll(mism) : 64u;
            if (lid < lim) {
                if (isA && occupy) occ_or_v = occ_or_v | oa;
                if (isA) alloc_or_v = alloc_or_v | M::bit(g);
            }
            if (!mism) {
                cur_v = g;
                occ = oa.readlane(63);
                smask = 0;                                   // the scan already covered every event
            } else {
                cur_v = (lid <= lim) ? g : cur_v;
                occ = ob.readlane(lim);                       // exact occupancy before event lim
                smask = sm & (~0ull << lim);
                const M bit = M::bit(rl(g, lim));
                const uint32_t fl = rl(f_v, lim);
                if (fl & F_A) {                              // event lim itself is exact: apply it
                    alloc_or = alloc_or | bit;
                    if (fl & F_O) { occ = occ | bit; occ_or = occ_or | occ; }
                } else {
                    const uint32_t pk = rl(s0, lim), pk1 = rl(s1, lim);
                    const uint32_t a = (fl & F_IN0) ? rl(cur_v, (fl >> 8) & 63u) : pk;
                    const uint32_t b = (fl & F_IN1) ? rl(cur_v, (fl >> 16) & 63u) : pk1;
                    occ = occ & ~(M::bit(a) | M::bit(b));
                    if (fl & F_O) occ = occ | bit;
                }
                smask &= smask - 1;                          // continue after event lim
            }
        }
        // ---- sequential part: special events (from the first unresolved one) --------
#ifdef WG_REPLAY_PROFILE
        rp_batches++;
        if (!smask) rp_fast++;
        const unsigned long long rp_s0 = clock64();
#endif
        while (smask) {
#ifdef WG_REPLAY_PROFILE
            rp_sev++;
#endif
            const uint32_t k = (uint32_t)__builtin_ctzll(smask);
            smask &= smask - 1;
            occ = occ & q.readlane(k);                          // the folded run before event k
            const uint32_t f = rl(f_v, k);
            uint32_t s;
            if (f & F_A) {
                s = occ.lowest_free();
                if (counted) alloc_or = alloc_or | M::bit(s);
                if (f & F_O) {
                    occ = occ | M::bit(s);
                    if (counted) occ_or = occ_or | occ;
                }
            } else {
                // tokens born in this batch, or more than two waiters
                uint32_t a = rl(s0, k), b = rl(s1, k);
                if (f & F_IN0) a = rl(cur_v, (f >> 8) & 63u);
                if (f & F_IN1) b = rl(cur_v, (f >> 16) & 63u);
                M clr = M::bit(a) | M::bit(b);
                uint32_t m = a < b ? a : b;
                if (f & F_M) {
#ifdef WG_REPLAY_PROFILE
                    rp_fm++;
                    const unsigned long long rp_m0 = clock64();
#endif
                    const uint32_t off = rl(row_v, k);      // record.w = aux offset: {count, tokens...}
                    const uint32_t cnt = ufl(A.aux[off]);
                    for (uint32_t x = 0; x < cnt; x++) {
                        const uint32_t t = ufl(A.aux[off + 1 + x]);
                        uint32_t ts;
                        if (t >= base) ts = rl(cur_v, (uint32_t)(t - base));
                        else if (have_prev && t >= pbase) ts = rl(prev_v, (uint32_t)(t - pbase));
                        else ts = ufl(t < ew ? A.slot_prev[t] : own(t));
                        clr = clr | M::bit(ts);
                        m = ts < m ? ts : m;
                    }
#ifdef WG_REPLAY_PROFILE
                    rp_cfm += clock64() - rp_m0;
#endif
                }
                occ = occ & ~clr;
                if (f & F_O) occ = occ | M::bit(m);
                s = m;
            }
            cur_v = (lid == k) ? s : cur_v;
        }
#ifdef WG_REPLAY_PROFILE
        rp_cs += clock64() - rp_s0;
#endif
        // the run after the last special event
        if (!(sm >> 63)) occ = occ & q.readlane(63);
        if (base + lid < e1) {
            const uint16_t nv = (uint16_t)cur_v;
            if (counted) {
                diff |= gp_v != nv;
                A.slot_next[base + lid] = nv;
            }
            if (lds) lslot[base - ew + lid] = nv;
        }
        gp_v = gp_next;
        // same-wave vector memory ops to one address complete in order; only keep
        // the compiler from moving the next batch's token loads above the store
        asm volatile("" ::: "memory");
        prev_v = cur_v;
        rec = rec1;
        rec1 = rec2;
        q0_v = n0_v;
        q1_v = n1_v;
    }
    occ_or = occ_or | occ_or_v.xor_or_reduce();
    alloc_or = alloc_or | alloc_or_v.xor_or_reduce();
    bool occ_changed = false;
    if (lid < (uint32_t)NW) {
        uint64_t w = 0;
#pragma unroll
        for (int k = 0; k < NW; k++)
            if ((uint32_t)k == lid) w = occ.w[k];
        A.occ_next[c * NW + lid] = w;
        occ_changed = w != A.occ_prev[c * NW + lid];
    }
    if (lid == 0) {
        A.chunk_stats[2 * c] = occ_or.highest();          // max_lane
        A.chunk_stats[2 * c + 1] = alloc_or.highest();    // max slot
    }
    // a warm-started first iteration is not the replay from iteration 0's
    // outputs, so it can never be the fixed point: it always counts as a change
    if (__any(diff) || occ_changed || ew < e0) A.changed[A.iter] = 1u;
#ifdef WG_REPLAY_PROFILE
    if (lid == 0) {
        RP_ADD(0, 1); RP_ADD(1, rp_batches); RP_ADD(2, rp_fast); RP_ADD(3, rp_sev); RP_ADD(4, rp_fm);
        RP_ADD(5, clock64() - rp_t0); RP_ADD(6, rp_cs); RP_ADD(7, rp_cfm);
    }
#endif
}

__global__ void k_lf_replay_init(uint64_t nchunks, unsigned long long *occ_prev, uint32_t *changed, uint32_t nflags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nchunks) occ_prev[i] = 0ull;    // initial guess (any guess is sound); nchunks counts words
    if (i < nflags) changed[i] = (i == 0) ? 1u : 0u;
}

// final: max_lane / slots / overflow over all chunks (nev_dev: chunks past the
// device event count hold nothing), by the first wave of the block
// scal[3]: the first of iterations 1..iters that changed nothing (0: none) —
// the iterations the next build launches before its first check
__device__ void replay_finish(uint64_t nchunks, const uint32_t *__restrict__ stats, uint32_t *__restrict__ scal,
                              const uint32_t *__restrict__ flags, uint32_t iters, uint32_t slot_cap,
                              const uint32_t *__restrict__ nev_dev, uint32_t chunk, bool dc) {
    const uint32_t lid = threadIdx.x;   // < 64
    uint32_t fp = ~0u;
    for (uint32_t i = 1 + lid; i <= iters; i += 64)
        if (flags[i] == 0 && i < fp) fp = i;
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t o = (uint32_t)__shfl_down((int)fp, d, 64);
        fp = o < fp ? o : fp;
    }
    if (lid == 0) scal[3] = fp == ~0u ? 0u : fp;
    if (nev_dev) {
        const uint64_t nd = ((uint64_t)*nev_dev + chunk - 1) / chunk;
        nchunks = nd < nchunks ? nd : nchunks;
    }
    // (the compacted replay, wg_lanes_dchunk.hip: three words per record, the
    // third the highest allocated position; an overflow reads 0xFFFF)
    const uint32_t st = dc ? 3u : 2u;
    uint32_t ml = 0, ms = 0, mp = 0;
    for (uint64_t c = lid; c < nchunks; c += 64) {
        ml = stats[st * c] > ml ? stats[st * c] : ml;
        ms = stats[st * c + 1] > ms ? stats[st * c + 1] : ms;
        if (dc) mp = stats[st * c + 2] > mp ? stats[st * c + 2] : mp;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const uint32_t a = (uint32_t)__shfl_down((int)ml, d, 64), b = (uint32_t)__shfl_down((int)ms, d, 64),
                       q = (uint32_t)__shfl_down((int)mp, d, 64);
        ml = a > ml ? a : ml;
        ms = b > ms ? b : ms;
        mp = q > mp ? q : mp;
    }
    if (lid == 0) {
        scal[0] = ml;
        scal[1] = ms + 1;
        scal[2] = ms >= (dc ? 0xFFFFu : slot_cap) ? 1u : 0u;   // the sentinel slot was handed out: the occupancy overflowed
        if (dc) scal[4] = mp + 1;
    }
}

__global__ void __launch_bounds__(64) k_lf_replay_finish(uint64_t nchunks, const uint32_t *__restrict__ stats,
                                                        uint32_t *__restrict__ scal, const uint32_t *__restrict__ flags,
                                                        uint32_t iters, uint32_t slot_cap, bool dc) {
    replay_finish(nchunks, stats, scal, flags, iters, slot_cap, nullptr, 1u, dc);
}

// speculative fast path: the scalars (first wave of block 0), then per row the
// slot of its chain's event = its lane (layouts.get(id), :278-283: ids are
// distinct here, so the row is its own canonical row) and its colour
__global__ void __launch_bounds__(256) k_lf_finish_lanes(uint64_t nchunks, const uint32_t *__restrict__ stats,
                                                        uint32_t *__restrict__ scal, const uint32_t *__restrict__ rflags,
                                                        uint32_t iters, uint32_t slot_cap, const uint32_t *__restrict__ nev_dev,
                                                        uint32_t chunk, uint64_t nl, const uint32_t *__restrict__ sp,
                                                        const uint16_t *__restrict__ slot_of, uint32_t *__restrict__ lane,
                                                        uint32_t *__restrict__ lane_out, uint8_t *__restrict__ color_out,
                                                        const uint8_t *__restrict__ flags, const uint32_t *__restrict__ gate,
                                                        bool dc) {
    if (*gate) return;   // not well formed: the exact stages redo the lanes
    if (blockIdx.x == 0 && threadIdx.x < 64) replay_finish(nchunks, stats, scal, rflags, iters, slot_cap, nev_dev, chunk, dc);
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nl) return;
    const uint32_t l = slot_of[sp[j] & ~WG_TOK_EV];
    lane[j] = l;
    lane_out[j] = l;
    color_out[j] = (flags[j] & WG_FLAG_ORPHAN) ? (uint8_t)WG_COLOR_ORPHAN : (uint8_t)(l % 6u);
}

}  // namespace

// one iteration at the run's occupancy width (R.nw words: up to 64 R.nw - 1 slots)
static void launch_replay(const ReplayRun &R, const ReplayArgs &a, hipStream_t s) {
    // iteration 1 restarts every chunk from an empty table: the serial step
    // (wg_lanes_serial.hip) does that at 8 instructions per event against
    // the scalar loop's ~320 cycles (r03: 97 of wide16's 156 us of replay)
    if (a.iter == 1 && R.death && R.nw <= 1 && R.chunk < 0xFFFFFFFFu) {
        (void)wg_replay_first(s, R, a.slot_next, a.occ_next);
        return;
    }
    if (R.nw <= 1) hipLaunchKernelGGL(k_lf_replay<1>, dim3(R.nch), dim3(64), 0, s, a);
    else if (R.nw <= 4) hipLaunchKernelGGL(k_lf_replay<4>, dim3(R.nch), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(k_lf_replay<16>, dim3(R.nch), dim3(64), 0, s, a);
}

// Replay driver.  wg_replay_start initialises and launches `blind` iterations
// without looking at the device (a fixed point found early makes the rest
// exit at once); the caller reads flags[it - 1] / flags[it] together with
// its own scalars and calls wg_replay_resume only when neither iteration was
// a fixed point.  Chunk c is exact after c + 1 iterations, so nch + 1
// iterations always reach the fixed point.
hipError_t wg_replay_start(wg_ctx *c, hipStream_t s, ReplayRun &R, uint32_t blind) {
    R.nch = (R.nev + R.chunk - 1) / R.chunk;
    R.it = 0;
    R.sp_prev = R.slots_a;
    R.sp_next = R.slots_b;
    R.op = R.occ_a;
    R.on = R.occ_b;
    if (R.max_iters > R.nch + 1) R.max_iters = (uint32_t)(R.nch + 1);
    if (R.nev == 0) {
        hipLaunchKernelGGL(k_lf_replay_finish, dim3(1), dim3(64), 0, s, (uint64_t)0, R.stats, R.scal, (const uint32_t *)R.flags, 0u,
                           64u * R.nw - 1u, false);
        return hipGetLastError();
    }
    const uint64_t ninit = R.nch > R.max_iters + 1 ? R.nch : R.max_iters + 1;
    const uint64_t ninit_w = ninit > R.nch * R.nw ? ninit : R.nch * R.nw;
    hipLaunchKernelGGL(k_lf_replay_init, dim3((ninit_w + 255) / 256), dim3(256), 0, s, R.nch * R.nw, R.occ_a, R.flags,
                       R.max_iters + 1);
    hipError_t e = hipMemsetAsync(R.slots_a, 0, R.nev * sizeof(uint16_t), s);
    if (e != hipSuccess) return e;
    if (blind > R.max_iters) blind = R.max_iters;
    for (uint32_t k = 0; k < blind; k++) {
        R.it++;
        ReplayArgs a{R.nev, R.chunk, R.it, R.ev, R.aux, R.sp_prev, R.sp_next, R.op, R.on, R.stats, R.flags, nullptr, nullptr,
                     R.warm};
        launch_replay(R, a, s);
        // after a fixed point later iterations do nothing; the converged slots are
        // in both buffers, so either pointer is final
        std::swap(R.sp_prev, R.sp_next);
        std::swap(R.op, R.on);
    }
    hipLaunchKernelGGL(k_lf_replay_finish, dim3(1), dim3(64), 0, s, R.nch, R.stats, R.scal, (const uint32_t *)R.flags, R.it,
                       64u * R.nw - 1u, false);
    return hipGetLastError();
}

// Speculative build (no host read of the event count): R.nev is an upper
// bound (the grid), R.nev_dev the count.  The initial state (zero occupancy
// guesses, the flag words, the slots' zero guess, the padding records) is
// written by the event kernel; then `blind` iterations; the scalars are
// reduced by the lanes kernel.  The caller checks convergence (flags[it - 1],
// flags[it]) with its end-of-build validation.
WgReplayInit wg_replay_prepare_spec(ReplayRun &R, uint32_t &blind) {
    R.nch = (R.nev + R.chunk - 1) / R.chunk;
    R.it = 0;
    R.sp_prev = R.slots_a;
    R.sp_next = R.slots_b;
    R.op = R.occ_a;
    R.on = R.occ_b;
    if (R.max_iters > R.nch + 1) R.max_iters = (uint32_t)(R.nch + 1);
    if (blind > R.max_iters) blind = R.max_iters;
    WgReplayInit I;
    I.occ = R.occ_a;
    I.occ_words = R.nch * R.nw;
    I.changed = R.flags;
    I.nflags = R.max_iters + 1;
    I.slots16 = reinterpret_cast<uint4 *>(R.slots_a);
    I.nslots16 = (R.nev * sizeof(uint16_t) + 15) / 16;
    I.nev_dev = R.nev_dev;
    uint64_t t = I.occ_words > I.nflags ? I.occ_words : I.nflags;
    if (t < I.nslots16) t = I.nslots16;
    I.total = t < 256 ? 256 : t;
    return I;
}

hipError_t wg_replay_iterate_spec(hipStream_t s, ReplayRun &R, uint32_t blind) {
    for (uint32_t k = 0; k < blind; k++) {
        R.it++;
        ReplayArgs a{R.nev, R.chunk, R.it, R.ev, R.aux, R.sp_prev, R.sp_next, R.op, R.on, R.stats, R.flags, R.nev_dev,
                     R.gate, R.warm};
        launch_replay(R, a, s);
        std::swap(R.sp_prev, R.sp_next);
        std::swap(R.op, R.on);
    }
    return hipGetLastError();
}

hipError_t wg_replay_finish_lanes(hipStream_t s, const ReplayRun &R, uint64_t nl, const uint32_t *sp, uint32_t *lane,
                                  uint32_t *lane_out, uint8_t *color_out, const uint8_t *flags) {
    const uint64_t g = nl ? (nl + 255) / 256 : 1;
    // the slot a run reports when its occupancy overflowed: the sentinel of its
    // width (the serial pass's 3- and 8-word forms: 191 / 511, not 255 / 1023)
    const uint32_t cap = (R.nw == 4 && R.ser_w3) ? 191u : (R.nw == 16 && R.ser_w8) ? 511u : 64u * R.nw - 1u;
    hipLaunchKernelGGL(k_lf_finish_lanes, dim3((uint32_t)g), dim3(256), 0, s, R.dc ? R.dc_blocks : R.nch, (const uint32_t *)R.stats,
                       R.scal, (const uint32_t *)R.flags, R.it, cap, R.nev_dev, R.dc ? WG_DC_FIX_T : R.chunk, nl, sp,
                       (const uint16_t *)R.sp_prev, lane, lane_out, color_out, flags, R.gate, R.dc);
    return hipGetLastError();
}

// Continue with polls (every 3rd iteration, then every 6th) until a fixed
// point or max_iters; *converged tells which.  A replay at a short chunk that
// is still moving at R.switch_it stops there (R.switched: the caller replays
// at WG_REPLAY_CHUNK_LONG from the start, so its iteration count is the long
// chunk's own and the next builds' blind count follows it).
hipError_t wg_replay_resume(wg_ctx *c, hipStream_t s, ReplayRun &R, bool *converged) {
    *converged = R.nev == 0;
    uint32_t next_poll = R.it + 3;
    if (R.switch_it && R.chunk < WG_REPLAY_CHUNK_LONG && next_poll > R.switch_it) next_poll = R.switch_it > R.it ? R.switch_it : R.it + 1;
    if (R.serial_it && R.chunk >= WG_REPLAY_CHUNK_LONG && next_poll > R.serial_it) next_poll = R.serial_it > R.it ? R.serial_it : R.it + 1;
    while (!*converged && R.it < R.max_iters) {
        R.it++;
        ReplayArgs a{R.nev, R.chunk, R.it, R.ev, R.aux, R.sp_prev, R.sp_next, R.op, R.on, R.stats, R.flags, nullptr, nullptr,
                     R.warm};
        launch_replay(R, a, s);
        std::swap(R.sp_prev, R.sp_next);
        std::swap(R.op, R.on);
        if (R.it == next_poll || R.it == R.max_iters) {
            next_poll = R.it + 6;
            uint64_t fl[2] = {1, 1};
            if (wg_fetch(c, {{R.flags + R.it - 1, false}, {R.flags + R.it, false}}, fl) != WG_OK) return hipErrorUnknown;
            *converged = fl[0] == 0 || fl[1] == 0;
            if (!*converged && R.switch_it && R.it >= R.switch_it && R.chunk < WG_REPLAY_CHUNK_LONG) {
                R.switched = true;
                return hipSuccess;
            }
            if (!*converged && R.serial_it && R.it >= R.serial_it && R.chunk >= WG_REPLAY_CHUNK_LONG) {
                R.to_serial = true;
                return hipSuccess;
            }
        }
    }
    if (R.nev)
        hipLaunchKernelGGL(k_lf_replay_finish, dim3(1), dim3(64), 0, s, R.nch, R.stats, R.scal, (const uint32_t *)R.flags, R.it,
                           64u * R.nw - 1u, false);
    return hipGetLastError();
}

#ifdef WG_REPLAY_PROFILE
// profiling builds only (-DWG_REPLAY_PROFILE): copy (and with reset, clear) the per-iteration counters
extern "C" int wg_debug_replay_profile(unsigned long long *out, int reset) {
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rp), sizeof(g_rp)) != hipSuccess) return WG_E_HIP;
    if (reset) {
        static unsigned long long zero[64][8];
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_rp), zero, sizeof(zero)) != hipSuccess) return WG_E_HIP;
    }
    return WG_OK;
}
#endif

// the scalars of a compacted replay (wg_lanes_dchunk.hip) after wg_dc_finish
hipError_t wg_dc_scalars(hipStream_t s, const ReplayRun &R) {
    hipLaunchKernelGGL(k_lf_replay_finish, dim3(1), dim3(64), 0, s, R.dc_blocks, R.stats, R.scal, (const uint32_t *)R.flags, R.it,
                       0xFFFFu, true);
    return hipGetLastError();
}
