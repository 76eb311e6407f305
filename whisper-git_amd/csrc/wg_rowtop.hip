// wg_rowtop.hip — row heights and the sequential-f32 row_top_y prefix
// (SURVEY.md §8a A6-A7).
//
// Heights: compute_row_heights (commit_graph.rs:486-507) maps each time gap
// through an f64 log to round(28 + 28 * (f32)ratio).  The map is monotone in
// the integer gap, so the host tabulates the 28 exact gap thresholds once
// (same libm log, same f32 rounding) and the device counts thresholds
// passed: bit-exact by construction, no transcendental on the GPU.
//
// row_top_y: `acc += h + band` in f32, strictly sequential (:329-335,
// :374-381).  Two regimes keep it parallel and still bit-exact:
//   * exact regime — while every step is an integer and the running sum stays
//     <= 2^24, every f32 add is exact: row_top is the plain integer prefix.
//   * rounding regime — within one binade [2^k, 2^k+1) (ulp u) the rounding
//     of acc + s depends on acc only through the parity of acc/u
//     (ties-to-even), so each row is a 2-state transducer {parity -> (ulps
//     added, new parity)}; transducers compose associatively.
// Kernels (chunks of 1024 rows):
//   rt_sum     f64 chunk sums, "all steps integral" and validity flags
//   rt_prefix  exact f64 prefix of chunk sums; marks the exact-regime chunks
//              and guesses every other chunk's binade
//   rt_tables  per non-exact chunk, 4 candidate binades: composed transducer
//   rt_walk    one wave, from the first non-exact chunk: composes 64 chunk
//              transducers per step (ordered shuffle scan) from the exact
//              running f32 value; a chunk in which acc crosses a binade is
//              replayed by the wave, 16 rows per lane, one transducer scan
//              per crossing (replay_chunk)
//   rt_rows    per chunk: exact prefix, or block scan of row transducers from
//              the chunk's exact start
// Negative or non-finite steps make the walk replay every row one by one
// (exact, slow; flagged in wg_geometry_summary.scan_path).
#include <cmath>

#include "wg_internal.h"

namespace {

constexpr int RT_T = 256;                 // threads per chunk block
constexpr int RT_Q = WG_RT_CHUNK / RT_T;  // rows per thread (4)
constexpr double TWO24 = 16777216.0;

enum : uint32_t { MODE_TABLE = 0, MODE_REPLAYED = 1, MODE_EXACT = 2 };

struct RtChunk {
    double   sum;     // f64 sum of steps in the chunk (exact for integral steps)
    double   prefix;  // f64 exclusive prefix (exact in the exact regime, else a guess)
    int32_t  kguess;  // binade of prefix
    uint32_t mode;    // MODE_*
    float    start;   // exact f32 acc at chunk start (MODE_TABLE / MODE_EXACT)
    int32_t  kstart;  // binade of start (MODE_TABLE)
    uint32_t integral;// every step of the chunk is an integer < 2^24
    uint32_t bad;     // a negative or non-finite step (the walk replays every row)
};

// 2-state transducer: parity p -> (d[p] ulps, o[p]); bit2 of f = valid
struct Td {
    uint32_t d0, d1, f;   // f: bit0 = o0, bit1 = o1, bit2 = valid
};
__device__ __forceinline__ Td td_identity() { return Td{0u, 0u, 0x2u | 0x4u}; }
__device__ __forceinline__ Td td_invalid() { return Td{0u, 0u, 0x2u}; }
// apply A then B
__device__ __forceinline__ Td td_compose(const Td &A, const Td &B) {
    const uint32_t a0 = A.f & 1u, a1 = (A.f >> 1) & 1u;
    Td r;
    r.d0 = A.d0 + (a0 ? B.d1 : B.d0);
    r.d1 = A.d1 + (a1 ? B.d1 : B.d0);
    const uint32_t o0 = (B.f >> a0) & 1u, o1 = (B.f >> a1) & 1u;
    r.f = o0 | (o1 << 1) | (A.f & B.f & 4u);
    return r;
}
// ordered inclusive scan of the lanes' transducers: lane i gets T_0 o ... o T_i
__device__ __forceinline__ Td td_scan(const Td &t) {
    return wg_wave_scan(t, td_identity(), [](const Td &a, const Td &b) { return td_compose(a, b); });
}

// The step at binade k: acc = 2^k + p*u represents every acc of parity p.
__device__ __forceinline__ Td row_td(float s, int k) {
    if (k < -100 || k > 126) return td_invalid();
    // x / u == x * 2^(23-k) exactly: every quotient below is an integer < 2^24
    const float base = ldexpf(1.0f, k), u = ldexpf(1.0f, k - 23), iu = ldexpf(1.0f, 23 - k), top = ldexpf(1.0f, k + 1);
    Td t;
    t.f = 4u;
    {
        const float a = base, r = a + s;
        if (!(r < top)) return td_invalid();
        t.d0 = (uint32_t)((r - a) * iu);
        t.f |= ((uint32_t)((r - base) * iu)) & 1u;
    }
    {
        const float a = base + u, r = a + s;
        if (!(r < top)) return td_invalid();
        t.d1 = (uint32_t)((r - a) * iu);
        t.f |= (((uint32_t)((r - base) * iu)) & 1u) << 1;
    }
    return t;
}

__device__ __forceinline__ float step_of(const float *__restrict__ h, const float *__restrict__ band, uint64_t i) {
    return band ? h[i] + band[i] : h[i] + 0.0f;   // `h + band` (:379); build() adds 0
}

__device__ __forceinline__ int binade_of(float a) { return ilogbf(a); }
// parity of a / 2^(k-23) for a in binade k (the quotient is an integer < 2^24)
__device__ __forceinline__ uint32_t parity_at(float a, int k) { return ((uint32_t)(a * ldexpf(1.0f, 23 - k))) & 1u; }

// ---------------------------------------------------------------------------
// heights
// ---------------------------------------------------------------------------
struct Thresh { uint32_t t[28]; };

// rows [0, m) of an n-row list (the last row of the LIST gets ROW_HEIGHT)
__global__ void k_heights(uint64_t m, uint64_t n, const int64_t *__restrict__ time, Thresh th, float *__restrict__ h) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    float out = WG_ROW_HEIGHT;
    if (i + 1 < n) {
        const uint64_t d = (uint64_t)time[i] - (uint64_t)time[i + 1];   // wrapping i64 sub
        uint64_t ad = ((int64_t)d < 0) ? (0ull - d) : d;                // unsigned_abs
        if (ad > 2592000ull) ad = 2592000ull;                             // .min(TIME_MAX_DELTA)
        uint32_t hh = 28;
#pragma unroll
        for (int k = 0; k < 28; k++) hh += (uint32_t)(ad >= (uint64_t)th.t[k]);
        out = (float)hh;
    }
    h[i] = out;
}

// ---------------------------------------------------------------------------
// row_top scan
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(RT_T) k_rt_sum(uint64_t n, const float *__restrict__ h, const float *__restrict__ band,
                                                 RtChunk *__restrict__ ch) {
    const uint64_t c = blockIdx.x;
    const uint64_t r0 = c * WG_RT_CHUNK + (uint64_t)threadIdx.x * RT_Q;
    double sum = 0.0;
    bool bad = false, frac = false;
#pragma unroll
    for (int q = 0; q < RT_Q; q++) {
        const uint64_t i = r0 + q;
        if (i < n) {
            const float s = step_of(h, band, i);
            bad |= !(s >= 0.0f) || !isfinite(s);
            frac |= !(s == truncf(s) && s < 16777216.0f);
            sum += (double)s;
        }
    }
    __shared__ double ws[RT_T / 64];
    __shared__ uint32_t wf[RT_T / 64];
    for (int d = 32; d >= 1; d >>= 1) sum += __shfl_down(sum, d, 64);
    const bool anyfrac = __any(frac), anybad = __any(bad);
    if ((threadIdx.x & 63) == 0) {
        ws[threadIdx.x >> 6] = sum;
        wf[threadIdx.x >> 6] = (anyfrac ? 1u : 0u) | (anybad ? 2u : 0u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        uint32_t fr = 0;
        for (int w = 0; w < RT_T / 64; w++) { t += ws[w]; fr |= wf[w]; }
        ch[c].sum = t;
        ch[c].integral = (fr & 1u) ? 0u : 1u;
        ch[c].bad = (fr >> 1) & 1u;
    }
}

// exact f64 prefix over chunks; exact-regime marking; binade guesses
// a0: the accumulator before row 0 (a suffix recomputed from an unchanged
// row_top value, wg_rowtop_run's r_from), null = 0
__global__ void __launch_bounds__(1024) k_rt_prefix(uint64_t nch, RtChunk *__restrict__ ch, uint32_t *__restrict__ flags,
                                                    const float *__restrict__ a0) {
    __shared__ double ws[16];
    __shared__ uint32_t wn[16];
    __shared__ double carry;
    __shared__ uint32_t carry_int;   // all chunks so far integral
    __shared__ uint32_t n_exact;     // the exact regime is a prefix of the chunks: its length
    // the flag words (no fill before the pass): [0] a negative / non-finite
    // step anywhere, [1] replayed chunks and [2] all-serial (the walk), [3] the
    // exact-regime length (below)
    uint32_t anybad = 0;
    for (uint64_t c = threadIdx.x; c < nch; c += 1024) anybad |= ch[c].bad;
    anybad = __syncthreads_or((int)anybad) ? 1u : 0u;
    if (threadIdx.x == 0) {
        flags[0] = anybad;
        flags[1] = 0u;
        flags[2] = 0u;
        // an exact start: a finite integer within 2^24 (row_top there is the exact sum)
        const float A0 = a0 ? *a0 : 0.0f;
        carry = (double)A0;
        carry_int = (A0 >= 0.0f && A0 <= 16777216.0f && A0 == truncf(A0)) ? 1u : 0u;
        n_exact = 0u;
    }
    __syncthreads();
    for (uint64_t base = 0; base < nch; base += 1024) {
        const uint64_t c = base + threadIdx.x;
        const double v = c < nch ? ch[c].sum : 0.0;
        const uint32_t nonint = (c < nch && !ch[c].integral) ? 1u : 0u;
        const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
        // chunk sums of integral steps are integers: the f64 prefix is exact in any order
        const double inc = wg_wave_scan(v, 0.0, [](double a, double b) { return a + b; });
        const uint32_t ninc = wg_wave_scan(nonint, 0u, [](uint32_t a, uint32_t b) { return a + b; });   // inclusive count of non-integral chunks
        if (lane == 63) { ws[w] = inc; wn[w] = ninc; }
        __syncthreads();
        double wb = 0.0, tot = 0.0;
        uint32_t nb = 0, ntot = 0;
        for (int k = 0; k < 16; k++) {
            if (k < w) { wb += ws[k]; nb += wn[k]; }
            tot += ws[k];
            ntot += wn[k];
        }
        const double pre = carry + wb + inc - v;
        const uint32_t nonint_incl = nb + ninc;   // non-integral chunks in [base, c]
        // exact regime: every chunk up to c integral and the sum after c <= 2^24
        const bool exact = c < nch && carry_int && nonint_incl == 0 && pre + v <= TWO24 && !anybad;
        if (c < nch) {
            ch[c].prefix = pre;
            ch[c].kguess = pre > 0.0 ? ilogb(pre) : -1000;
            ch[c].mode = exact ? MODE_EXACT : MODE_REPLAYED;
            ch[c].start = (float)pre;
        }
        const int nx = __syncthreads_count(exact);
        if (threadIdx.x == 0) { carry += tot; if (ntot) carry_int = 0u; n_exact += (uint32_t)nx; }
        __syncthreads();
    }
    if (threadIdx.x == 0) flags[3] = n_exact;   // the walk starts after the exact regime
}

__global__ void __launch_bounds__(RT_T) k_rt_tables(uint64_t n, const float *__restrict__ h, const float *__restrict__ band,
                                                    const RtChunk *__restrict__ ch, uint4 *__restrict__ tables) {
    const uint64_t c = blockIdx.x;
    if (ch[c].mode == MODE_EXACT) return;
    const uint64_t r0 = c * WG_RT_CHUNK + (uint64_t)threadIdx.x * RT_Q;
    float s[RT_Q];
#pragma unroll
    for (int q = 0; q < RT_Q; q++) s[q] = (r0 + q < n) ? step_of(h, band, r0 + q) : -1.0f;
    __shared__ Td wt[RT_T / 64];
    const int kg = ch[c].kguess;
    for (int b = 0; b < WG_RT_NBIN; b++) {
        const int k = kg - 1 + b;
        Td t = td_identity();
#pragma unroll
        for (int q = 0; q < RT_Q; q++)
            if (r0 + q < n) t = td_compose(t, row_td(s[q], k));
        t = td_scan(t);   // lane 63: the wave's rows composed in order
        if ((threadIdx.x & 63) == 63) wt[threadIdx.x >> 6] = t;
        __syncthreads();
        if (threadIdx.x == 0) {
            Td a = wt[0];
            for (int w = 1; w < RT_T / 64; w++) a = td_compose(a, wt[w]);
            tables[c * WG_RT_NBIN + b] = make_uint4(a.d0, a.d1, a.f, 0u);
        }
        __syncthreads();
    }
}

// ---- super-chunks: 64 chunks (64K rows) composed per candidate binade ----------------
constexpr int RT_SUP = 64;
struct SupState { float start; int32_t k; uint32_t mode; uint32_t pad; };   // mode 1: walked at super level

__device__ __forceinline__ Td td_reduce64(Td t) {   // ordered: lane 63 gets T_0 o ... o T_63
    return td_scan(t);
}

__global__ void __launch_bounds__(64) k_rt_super(uint64_t nch, const RtChunk *__restrict__ ch, const uint4 *__restrict__ tables,
                                                 uint4 *__restrict__ stab, int32_t *__restrict__ skbase,
                                                 SupState *__restrict__ sup) {
    const uint64_t S = blockIdx.x, c0 = S * RT_SUP, cc = c0 + (threadIdx.x & 63);
    const bool full = c0 + RT_SUP <= nch;
    double sm = full ? ch[cc].sum : 0.0;
    for (int d = 32; d >= 1; d >>= 1) sm += __shfl_down(sm, d, 64);
    sm = __shfl(sm, 0, 64);
    const int k0 = ch[c0 < nch ? c0 : 0].kguess - 1;
    for (int j = 0; j < WG_RT_NBIN; j++) {
        const int k = k0 + j;
        Td t = td_invalid();
        if (full && ch[cc].mode != MODE_EXACT) {
            const int b = k - ch[cc].kguess + 1;
            if (b >= 0 && b < WG_RT_NBIN) { const uint4 q = tables[cc * WG_RT_NBIN + b]; t = Td{q.x, q.y, q.z}; }
        }
        t = td_reduce64(t);
        // ulp counts stay far below 2^32 only where the ulp is >= 2 (k >= 24) and the sum is bounded
        const bool fits = full && k >= 24 && k < 120 && sm < ldexp(1.0, k - 23) * 2147483648.0;
        if ((threadIdx.x & 63) == 63) stab[S * WG_RT_NBIN + j] = fits ? make_uint4(t.d0, t.d1, t.f, 0u) : make_uint4(0u, 0u, 2u, 0u);
    }
    if ((threadIdx.x & 63) == 0) {
        skbase[S] = k0;
        sup[S] = SupState{0.0f, 0, 0u, 0u};   // (the walk marks the super-chunks it consumes whole)
    }
}

// Replay rows [r0, r1) from acc one by one (negative / non-finite steps).
__device__ float serial_rows(uint64_t r0, uint64_t r1, float acc, const float *__restrict__ h,
                             const float *__restrict__ band, float *__restrict__ row_top) {
    const int lid = threadIdx.x & 63;
    for (uint64_t base = r0; base < r1; base += 64) {
        const uint64_t i = base + lid;
        const float sv = i < r1 ? step_of(h, band, i) : 0.0f;
        float mine = 0.0f;
        const int cnt = (int)((r1 - base) < 64 ? (r1 - base) : 64);
        for (int j = 0; j < cnt; j++) {
            const float sj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, sv), j));
            if (lid == j) mine = acc;
            acc = acc + sj;
        }
        if (i < r1) row_top[i] = mine;
    }
    return acc;
}

// Replay rows [r0, r1) from acc (steps finite, >= 0) 64 rows at a time: one
// ordered transducer scan per binade the running value passes through.
__device__ float replay_rows(uint64_t r0, uint64_t r1, float acc, const float *__restrict__ h,
                             const float *__restrict__ band, float *__restrict__ row_top) {
    const uint32_t lid = threadIdx.x & 63;
    for (uint64_t base = r0; base < r1; base += 64) {
        const uint64_t i = base + lid;
        const uint32_t cnt = (uint32_t)((r1 - base) < 64 ? (r1 - base) : 64);
        const float sv = lid < cnt ? step_of(h, band, i) : 0.0f;
        float mine = 0.0f;
        uint32_t j = 0;   // first row of the piece not yet placed (uniform)
        while (j < cnt) {
            if (!(acc >= 1.0e-30f)) {   // acc == 0 (or tiny): one exact step
                const float sj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, sv), (int)j));
                if (lid == j) mine = acc;
                acc = acc + sj;
                j++;
                continue;
            }
            const int k = binade_of(acc);
            const float u = ldexpf(1.0f, k - 23);
            const double top = ldexp(1.0, k + 1);
            const uint32_t p = parity_at(acc, k);
            const Td t = td_scan((lid >= j && lid < cnt) ? row_td(sv, k) : td_identity());
            const uint32_t D = p ? t.d1 : t.d0;   // ulps added through this lane's row
            const bool ok = (t.f & 4u) && (double)acc + (double)D * (double)u < top;
            const uint64_t okm = __ballot(ok || lid < j) | (cnt < 64 ? (~0ull << cnt) : 0ull);
            const uint32_t f = okm == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~okm);   // first row crossing the binade
            const uint32_t Dprev = wg_wave_shr1(D, 0u);
            if (lid >= j && lid < f) mine = acc + (float)(lid == j ? 0u : Dprev) * u;
            if (f > j) acc = acc + (float)wg_lane(D, f - 1) * u;
            j = f;
            if (j < cnt) {   // the crossing row itself: one ordinary f32 add
                const float sj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, sv), (int)j));
                if (lid == j) mine = acc;
                acc = acc + sj;
                j++;
            }
        }
        if (lid < cnt) row_top[i] = mine;
    }
    return acc;
}

// Replay one chunk's rows [r0, r1) (at most 64 * 16) from acc > 0: lane L
// holds rows 16L..16L+15.  Per pass, the lanes' 16-row transducers at the
// binade of acc are scanned; every lane before the first one whose rows reach
// the next binade is placed in parallel, that lane's 16 rows are added one
// by one (plain f32 adds, the reference's own operation), and the next pass
// starts after it.  A chunk with b binade crossings takes b + 1 passes.
constexpr int RP_Q = 16;
static_assert(WG_RT_CHUNK <= 64 * RP_Q, "a chunk is replayed by one wave");
__device__ float replay_chunk(uint64_t r0, uint64_t r1, float acc, const float *__restrict__ h,
                              const float *__restrict__ band, float *__restrict__ row_top) {
    const uint32_t lid = threadIdx.x & 63;
    const uint32_t cnt = (uint32_t)(r1 - r0);
    float sv[RP_Q], mine[RP_Q];
#pragma unroll
    for (int q = 0; q < RP_Q; q++) {
        const uint32_t j = lid * RP_Q + q;
        sv[q] = j < cnt ? step_of(h, band, r0 + j) : 0.0f;
        mine[q] = 0.0f;
    }
    uint32_t j0 = 0;   // first row not yet placed (uniform, a multiple of RP_Q)
    while (j0 < cnt) {
        if (!(acc >= 1.0e-30f)) {   // zero / tiny: the row-by-row replay takes over
#pragma unroll
            for (int q = 0; q < RP_Q; q++)
                if (lid * RP_Q + q < j0) row_top[r0 + lid * RP_Q + q] = mine[q];
            return replay_rows(r0 + j0, r1, acc, h, band, row_top);
        }
        const int k = binade_of(acc);
        const float u = ldexpf(1.0f, k - 23);
        const double top = ldexp(1.0, k + 1);
        const uint32_t p = parity_at(acc, k);
        Td t = td_identity();
#pragma unroll
        for (int q = 0; q < RP_Q; q++) {
            const uint32_t j = lid * RP_Q + q;
            if (j >= j0 && j < cnt) t = td_compose(t, row_td(sv[q], k));
        }
        const Td inc = td_scan(t);
        const Td ex = wg_wave_shr1(inc, td_identity());
        const uint32_t Dinc = p ? inc.d1 : inc.d0;
        const bool ok = (inc.f & 4u) && (double)acc + (double)Dinc * (double)u < top;
        const uint64_t okm = __ballot(ok);
        const uint32_t f = okm == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~okm);
        if (lid < f) {
            uint32_t D = p ? ex.d1 : ex.d0;
            uint32_t par = p ? ((ex.f >> 1) & 1u) : (ex.f & 1u);
#pragma unroll
            for (int q = 0; q < RP_Q; q++) {
                const uint32_t j = lid * RP_Q + q;
                if (j >= j0 && j < cnt) {
                    mine[q] = acc + (float)D * u;
                    const Td r = row_td(sv[q], k);
                    D += par ? r.d1 : r.d0;
                    par = (r.f >> par) & 1u;
                }
            }
        }
        if (f == 64u) {
            acc = acc + (float)wg_lane(Dinc, 63) * u;
            break;
        }
        float a = acc + (float)(f == 0u ? 0u : wg_lane(Dinc, f - 1)) * u;
#pragma unroll
        for (int q = 0; q < RP_Q; q++) {
            const uint32_t j = f * RP_Q + q;
            if (j >= j0 && j < cnt) {
                const float sj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, sv[q]), (int)f));
                if (lid == f) mine[q] = a;
                a = a + sj;
            }
        }
        acc = a;
        j0 = (f + 1u) * RP_Q;
    }
#pragma unroll
    for (int q = 0; q < RP_Q; q++)
        if (lid * RP_Q + q < cnt) row_top[r0 + lid * RP_Q + q] = mine[q];
    return acc;
}

// table b of a chunk's (or super-chunk's) WG_RT_NBIN binade tables, invalid
// outside them; all of them are loaded, so the loads do not wait for b
__device__ __forceinline__ Td pick_table(const uint4 *__restrict__ tab, int b) {
    uint4 q[WG_RT_NBIN];
#pragma unroll
    for (int j = 0; j < WG_RT_NBIN; j++) q[j] = tab[j];
    uint4 r = make_uint4(0u, 0u, 2u, 0u);   // td_invalid()
#pragma unroll
    for (int j = 0; j < WG_RT_NBIN; j++)
        if (b == j) r = q[j];
    return Td{r.x, r.y, r.z};
}

__global__ void __launch_bounds__(64) k_rt_walk(uint64_t n, uint64_t nch, const float *__restrict__ h,
                                                const float *__restrict__ band, RtChunk *__restrict__ ch,
                                                const uint4 *__restrict__ tables, uint32_t *__restrict__ flags,
                                                float *__restrict__ row_top, uint64_t nsup, const uint4 *__restrict__ stab,
                                                const int32_t *__restrict__ skbase, SupState *__restrict__ sup,
                                                const float *__restrict__ a0) {
    const int lid = threadIdx.x & 63;
    const bool all_serial = flags[0] != 0;
    // skip the exact-regime prefix (its chunks are independent prefix sums;
    // k_rt_prefix counted them)
    uint64_t c = 0;
    if (!all_serial) {
        c = flags[3];
        if (c > nch) c = nch;
    }
    float A = c == 0 ? (a0 ? *a0 : 0.0f) : (float)(ch[c - 1].prefix + ch[c - 1].sum);   // exact (<= 2^24, integral)
    uint64_t replayed = 0;
    while (c < nch) {
        bool do_replay = all_serial || !(A > 0.0f) || !isfinite(A);
        if (!do_replay && (c % RT_SUP) == 0 && c / RT_SUP < nsup) {
            // super level: up to 64 super-chunks (4M rows) per step
            const int k = binade_of(A);
            const float u = ldexpf(1.0f, k - 23);
            const double top = ldexp(1.0, k + 1);
            const uint32_t p = parity_at(A, k);
            const uint64_t ss = c / RT_SUP + lid;
            // the base and all WG_RT_NBIN tables in one load round; the binade picks after
            Td t = td_invalid();
            if (ss < nsup) t = pick_table(stab + ss * WG_RT_NBIN, k - skbase[ss]);
            t = td_scan(t);
            const uint32_t D = p ? t.d1 : t.d0;
            const bool ok = (t.f & 4u) && ss < nsup && (double)A + (double)D * (double)u < top;
            const uint64_t okm = __ballot(ok);
            const int f = okm == ~0ull ? 64 : (int)__builtin_ctzll(~okm);
            const uint32_t Dprev = wg_wave_shr1(D, 0u);
            if (lid < f) sup[ss] = SupState{A + (float)(lid == 0 ? 0u : Dprev) * u, k, 1u, 0u};
            if (f > 0) {
                A = A + (float)wg_lane(D, (uint32_t)f - 1) * u;
                c += (uint64_t)f * RT_SUP;
                continue;
            }
        }
        if (!do_replay) {
            const int k = binade_of(A);
            const float u = ldexpf(1.0f, k - 23);
            const double top = ldexp(1.0, k + 1);
            const uint32_t p = parity_at(A, k);
            const uint64_t cc = c + lid;
            Td t = td_invalid();
            if (cc < nch) t = pick_table(tables + cc * WG_RT_NBIN, k - ch[cc].kguess + 1);
            t = td_scan(t);   // ordered inclusive scan: P_j = T_c o ... o T_{c+j}
            const uint32_t D = p ? t.d1 : t.d0;
            const bool ok = (t.f & 4u) && cc < nch && cc / RT_SUP == c / RT_SUP &&   // stop at the super boundary
                            (double)A + (double)D * (double)u < top;
            const uint64_t okm = __ballot(ok);
            const int f = okm == ~0ull ? 64 : (int)__builtin_ctzll(~okm);   // leading run of valid lanes
            const uint32_t Dprev = wg_wave_shr1(D, 0u);
            if (lid < f) {
                const uint32_t dp = lid == 0 ? 0u : Dprev;
                ch[cc].start = A + (float)dp * u;
                ch[cc].kstart = k;
                ch[cc].mode = MODE_TABLE;
            }
            if (f > 0) {
                const uint32_t Dl = wg_lane(D, (uint32_t)f - 1);
                A = A + (float)Dl * u;
                c += f;
            }
            // stopped before a chunk inside the super-chunk: that chunk crosses a binade
            do_replay = f < 64 && c < nch && !(f > 0 && (c % RT_SUP) == 0);
        }
        if (do_replay && c < nch) {
            const uint64_t r0 = c * WG_RT_CHUNK, r1 = (r0 + WG_RT_CHUNK < n) ? r0 + WG_RT_CHUNK : n;
            A = all_serial ? serial_rows(r0, r1, A, h, band, row_top)
                           : (A >= 1.0e-30f ? replay_chunk(r0, r1, A, h, band, row_top) : replay_rows(r0, r1, A, h, band, row_top));
            if (lid == 0) ch[c].mode = MODE_REPLAYED;
            c++;
            replayed++;
        }
    }
    if (lid == 0) {
        row_top[n] = A;
        flags[1] = (uint32_t)replayed;
        flags[2] = all_serial ? 1u : 0u;
    }
}

// A chunk inside a super-chunk the walk consumed whole: its start from the
// super-chunk's start and the scan of its chunks' tables up to it
__device__ __forceinline__ void super_start(const SupState &st, uint64_t S, uint64_t c, const RtChunk *__restrict__ ch,
                                            const uint4 *__restrict__ tables, float *start, int *kstart) {
    __shared__ float s_start;
    if (threadIdx.x < 64) {
        const int lid = threadIdx.x & 63;
        const uint64_t cc = S * RT_SUP + lid;
        const float u = ldexpf(1.0f, st.k - 23);
        const uint32_t p0 = parity_at(st.start, st.k);
        const int b = st.k - ch[cc].kguess + 1;
        const uint4 q = tables[cc * WG_RT_NBIN + b];   // valid: the super table was composed from these
        const Td t = td_scan(Td{q.x, q.y, q.z});
        const Td ex = wg_wave_shr1(t, td_identity());
        const uint32_t D = p0 ? ex.d1 : ex.d0;
        if ((uint64_t)lid == c - S * RT_SUP) s_start = st.start + (float)D * u;
    }
    __syncthreads();
    *start = s_start;
    *kstart = st.k;
}

__global__ void __launch_bounds__(RT_T) k_rt_rows(uint64_t n, uint64_t c_lo, const float *__restrict__ h,
                                                  const float *__restrict__ band, const RtChunk *__restrict__ ch,
                                                  float *__restrict__ row_top, uint64_t nsup,
                                                  const SupState *__restrict__ sup, const uint4 *__restrict__ tables) {
    const uint64_t c = c_lo + blockIdx.x;
    uint32_t mode = ch[c].mode;
    float A = ch[c].start;
    int kst = ch[c].kstart;
    if (mode == MODE_REPLAYED) {
        const uint64_t S = c / RT_SUP;
        if (S >= nsup || sup[S].mode != 1u) return;   // replayed by the walk
        super_start(sup[S], S, c, ch, tables, &A, &kst);
        mode = MODE_TABLE;
    }
    const int lid = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t r0 = c * WG_RT_CHUNK + (uint64_t)threadIdx.x * RT_Q;
    if (mode == MODE_EXACT) {
        // every partial sum is an integer <= 2^24: the f32 scan is exact
        float s[RT_Q], t = 0.0f;
#pragma unroll
        for (int q = 0; q < RT_Q; q++) { s[q] = (r0 + q < n) ? step_of(h, band, r0 + q) : 0.0f; t += s[q]; }
        const float inc = wg_wave_scan(t, 0.0f, [](float a, float b) { return a + b; });   // exact integers
        __shared__ float wsum[RT_T / 64];
        if (lid == 63) wsum[w] = inc;
        __syncthreads();
        float run = A + (inc - t);
        for (int k2 = 0; k2 < w; k2++) run += wsum[k2];
        // every partial value is an exact integer, so the association order is irrelevant
#pragma unroll
        for (int q = 0; q < RT_Q; q++) {
            if (r0 + q < n) row_top[r0 + q] = run;
            run += s[q];
        }
        return;   // row_top[n] is written by the walk
    }
    const int k = kst;
    const float u = ldexpf(1.0f, k - 23);
    const uint32_t p0 = parity_at(A, k);
    Td tr[RT_Q];
    Td t = td_identity();
#pragma unroll
    for (int q = 0; q < RT_Q; q++) {
        tr[q] = (r0 + q < n) ? row_td(step_of(h, band, r0 + q), k) : td_identity();
        t = td_compose(t, tr[q]);
    }
    // ordered block exclusive scan
    const Td inc = td_scan(t);
    __shared__ Td wt[RT_T / 64];
    if (lid == 63) wt[w] = inc;
    Td ex = wg_wave_shr1(inc, td_identity());
    __syncthreads();
    Td wp = td_identity();
    for (int k2 = 0; k2 < w; k2++) wp = td_compose(wp, wt[k2]);
    ex = td_compose(wp, ex);
    uint32_t D = p0 ? ex.d1 : ex.d0;
    uint32_t p = p0 ? ((ex.f >> 1) & 1u) : (ex.f & 1u);
#pragma unroll
    for (int q = 0; q < RT_Q; q++) {
        if (r0 + q < n) {
            row_top[r0 + q] = A + (float)D * u;
            D += p ? tr[q].d1 : tr[q].d0;
            p = (tr[q].f >> p) & 1u;
        }
    }
}

}  // namespace

// Host: exact gap thresholds of compute_row_heights (:486-507).
static float height_of_gap(uint64_t d) {
    const double log_max = std::log(1.0 + WG_TIME_MAX_DELTA / WG_TIME_BASE_SECONDS);
    double delta = (double)d;
    double clamped = delta < WG_TIME_MAX_DELTA ? delta : WG_TIME_MAX_DELTA;
    double ratio = std::log(1.0 + clamped / WG_TIME_BASE_SECONDS) / log_max;
    volatile float r32 = (float)ratio;
    volatile float prod = WG_MAX_EXTRA_HEIGHT * r32;
    volatile float h = WG_ROW_HEIGHT + prod;
    return std::round((float)h);
}

void wg_init_height_thresholds(uint32_t *th) {
    for (int k = 0; k < 28; k++) {
        const float target = 29.0f + (float)k;
        uint64_t lo = 0, hi = 2592001;   // first gap with height >= target, in [lo, hi]
        while (lo < hi) {
            uint64_t mid = (lo + hi) / 2;
            if (height_of_gap(mid) >= target) hi = mid; else lo = mid + 1;
        }
        th[k] = (uint32_t)lo;   // 2592001 = never reached
    }
}

extern "C" void wg_debug_height_thresholds(uint32_t *out28) { wg_init_height_thresholds(out28); }

int wg_heights_run(wg_ctx *c, uint64_t m, uint64_t n, float *out, const int64_t *time) {
    if (m == 0) return WG_OK;
    if (!time) time = c->d_time;
    Thresh th;
    for (int k = 0; k < 28; k++) th.t[k] = c->h_thresh[k];
    wg_stage_begin(c, "heights");
    hipLaunchKernelGGL(k_heights, dim3((m + 255) / 256), dim3(256), 0, c->stream, m, n, time, th, out);
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}

int wg_stage_heights(wg_ctx *c) {
    if (const int rc = wg_side_join(c)) return rc;
    c->n_list = c->n;
    WG_ALLOC(c, c->heights, c->n * 4 + 4);
    return wg_heights_run(c, c->n, c->n, c->heights.as<float>());
}

// row_top[0..n] of n rows with heights h (+ band, may be null).  Rows below
// row_lo are only walked through (a row shard needs row_top of its own rows;
// entries below row_lo are left unspecified).
int wg_rowtop_run(wg_ctx *c, uint64_t n, const float *h, const float *d_band, float *row_top, uint64_t row_lo,
                  uint64_t r_from) {
    // Rows below r_from kept their steps: row_top up to r_from is unchanged, so
    // the scan restarts at the chunk boundary below it from the row_top value
    // already there (the sequential sum carries nothing else).
    const float *a0 = nullptr;
    if (r_from > 0 && r_from <= n) {
        const uint64_t cs = r_from / WG_RT_CHUNK * WG_RT_CHUNK;
        if (cs > 0) {
            h += cs;
            if (d_band) d_band += cs;
            row_top += cs;
            a0 = row_top;
            n -= cs;
            row_lo = row_lo > cs ? row_lo - cs : 0;
        }
    }
    const uint64_t nch = (n + WG_RT_CHUNK - 1) / WG_RT_CHUNK;
    WG_ALLOC(c, c->rt_chunk, (nch + 1) * sizeof(RtChunk));
    WG_ALLOC(c, c->rt_tables, (nch + 1) * WG_RT_NBIN * sizeof(uint4));
    WG_ALLOC(c, c->rt_flags, 64);
    wg_stage_begin(c, "row_top");
    if (n == 0) {
        WG_HIP(c, hipMemsetAsync(c->rt_flags.p, 0, 64, c->stream));
        if (!a0) WG_HIP(c, hipMemsetAsync(row_top, 0, 4, c->stream));
        wg_stage_end(c);
        return WG_OK;
    }
    RtChunk *ch = c->rt_chunk.as<RtChunk>();
    uint32_t *fl = c->rt_flags.as<uint32_t>();
    hipLaunchKernelGGL(k_rt_sum, dim3(nch), dim3(RT_T), 0, c->stream, n, h, d_band, ch);
    hipLaunchKernelGGL(k_rt_prefix, dim3(1), dim3(1024), 0, c->stream, nch, ch, fl, a0);
    hipLaunchKernelGGL(k_rt_tables, dim3(nch), dim3(RT_T), 0, c->stream, n, h, d_band, (const RtChunk *)ch,
                       c->rt_tables.as<uint4>());
    const uint64_t nsup = nch / RT_SUP;   // full super-chunks only
    WG_ALLOC(c, c->rt_sup, nsup * (WG_RT_NBIN * 16 + 4 + sizeof(SupState)) + 64);
    uint4 *stab = c->rt_sup.as<uint4>();
    int32_t *skb = reinterpret_cast<int32_t *>(stab + nsup * WG_RT_NBIN);
    SupState *sup = reinterpret_cast<SupState *>(c->rt_sup.as<uint8_t>() + ((nsup * (WG_RT_NBIN * 16 + 4) + 15) / 16) * 16);
    if (nsup)
        hipLaunchKernelGGL(k_rt_super, dim3(nsup), dim3(64), 0, c->stream, nch, (const RtChunk *)ch,
                           c->rt_tables.as<const uint4>(), stab, skb, sup);
    hipLaunchKernelGGL(k_rt_walk, dim3(1), dim3(64), 0, c->stream, n, nch, h, d_band, ch,
                       c->rt_tables.as<const uint4>(), fl, row_top, nsup, (const uint4 *)stab, (const int32_t *)skb, sup, a0);
    const uint64_t c_lo = (row_lo < n ? row_lo : n) / WG_RT_CHUNK;
    if (c_lo < nch)
        hipLaunchKernelGGL(k_rt_rows, dim3(nch - c_lo), dim3(RT_T), 0, c->stream, n, c_lo, h, d_band, (const RtChunk *)ch,
                           row_top, nsup, (const SupState *)sup, c->rt_tables.as<const uint4>());
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}

int wg_stage_rowtop(wg_ctx *c, const float *d_band, uint64_t r_from) {
    if (const int rc = wg_side_join(c)) return rc;   // the side stream's row_top shares the scan buffers
    WG_ALLOC(c, c->g_row_top, (c->n + 1) * 4);
    return wg_rowtop_run(c, c->n, c->geom_heights(), d_band, c->g_row_top.as<float>(), 0, r_from);
}
