// wg_geom.hip — edge -> per-row geometry.
//
// Reference: RowGeometry init (commit_graph.rs:337-343, :383-394),
// decompose_edge_into_rows (:525-608) and Cubic (:614-695).  Each row's four
// lists are filled in edge order (child_row asc, then parent order), which
// graph_cell paints as z-order (:827-866); the engine reproduces that order
// exactly:
//   bottom_half  row r = same-lane edges of child r, in parent order
//   top_half     row r = same-lane edges into parent r, sorted by edge id
//   full         row r = same-lane edges with c < r < p, edge order
//   curves       row r = cross-lane edges with c <= r <= p whose strip is
//                non-empty (:577), edge order
// Counts come from difference arrays + scans; `full` and `curves` are
// ordered by a chunked sweep: one wave owns 64 rows and carries the ordered
// list of edges alive across its first row (registered per chunk, then
// rank-sorted), appends edges as their child rows are reached and compacts
// out edges that ended.  The per-segment Bezier clipping (two 40-step
// bisections + two de Casteljau splits) then runs one thread per segment.
//
// Bit-exact f32: built with -ffp-contract=off and the exact operation order
// of Cubic::y_at (:623-629), split's lerp (:657) and `dy * 0.4` (:557-562).
#include <algorithm>
#include <cstring>

#include "wg_internal.h"

namespace {

constexpr int T = 256;
constexpr uint32_t RF_ZERO = 1u, RF_CHILD = 2u, RF_PARENT = 4u;

// Capacity guard of a speculative geometry pass (the lists sized by the last
// pass's capacities, the totals only known on the device): a kernel that
// writes a list whose scanned total exceeds its capacity writes nothing and
// raises the overflow word; the end-of-build validation redoes the pass.
// Exact passes pass cap = ~0u.
struct Cap {
    const uint32_t *total;   // the list's scanned total (device)
    uint32_t cap;
    // a frame pass on a build not validated yet (WG_OPT_DEFER_VALIDATION): the
    // build pass's error words (sweep error [0], capacity overflow [8]); set,
    // its lists are incomplete and nothing may read them
    const uint32_t *gate;
};
// A kernel's guards read with every load issued before any is waited on: an
// absent pointer reads the overflow word instead of branching round its load
// (a load waited on alone at a kernel's start queues behind the CU's other
// loads; chained, the guards cost one round trip each).
template <int K>
struct CapVals {
    uint32_t gate, total[K];
};
template <int K>
__device__ __forceinline__ CapVals<K> cap_read(const Cap (&cs)[K], const uint32_t *ovf) {
    typedef const __attribute__((address_space(1))) uint32_t gword;   // global loads, not flat
    uint32_t g0[K], g8[K], t[K];
    for (int k = 0; k < K; k++) {   // every load first
        const bool hg = cs[k].gate != nullptr, ht = cs[k].total != nullptr;
        g0[k] = *(const gword *)(hg ? cs[k].gate : ovf);
        g8[k] = *(const gword *)(hg ? cs[k].gate + 8 : ovf);
        t[k] = *(const gword *)(ht ? cs[k].total : ovf);
    }
    CapVals<K> v;
    v.gate = 0;
    for (int k = 0; k < K; k++) {
        v.gate |= cs[k].gate ? g0[k] | g8[k] : 0u;
        v.total[k] = cs[k].total ? t[k] : 0u;
    }
    return v;
}
// (one state word from every load before any branch, so none is sunk past one)
template <int K>
__device__ __forceinline__ bool cap_over(const CapVals<K> &v, const Cap (&cs)[K], uint32_t *ovf) {
    uint32_t o = 0;
    for (int k = 0; k < K; k++) o |= (uint32_t)(cs[k].cap != ~0u) & (uint32_t)(v.total[k] > cs[k].cap);
    const uint32_t state = (v.gate ? 2u : 0u) | o;
    if (state == 0) return false;
    if (state == 1 && threadIdx.x == 0) atomicOr(ovf, 1u);
    return true;
}
template <int K>
__device__ __forceinline__ bool over_all(const Cap (&cs)[K], uint32_t *ovf) {
    return cap_over(cap_read(cs, ovf), cs, ovf);
}
__device__ __forceinline__ bool over(Cap a, uint32_t *ovf) {
    const Cap cs[1] = {a};
    return over_all(cs, ovf);
}

__device__ __forceinline__ uint32_t pack_vert(uint32_t lane, uint32_t kind, uint32_t color) {
    return (lane & 0xFFFFFFu) | (kind << 24) | (color << 28);
}

// RowGeometry {height, node_y} + per-row strip flags
// rows [lo, n) (lo > 0: a frame whose bands equal the last frame's below lo)
// zws / nz4 (full geometry pass): the stage's zero-initialised workspace,
// cleared here (grid-stride, 16-byte stores) instead of by a separate fill —
// the counting kernels that accumulate into it run after this one
__global__ void k_row_basic(uint64_t n, const float *__restrict__ h, const float *__restrict__ band,
                            const float *__restrict__ row_top, float *__restrict__ height, float *__restrict__ node_y,
                            uint8_t *__restrict__ rowflags, uint64_t lo = 0, uint4 *__restrict__ zws = nullptr,
                            uint64_t nz4 = 0, float *__restrict__ band_keep = nullptr,
                            const uint8_t *__restrict__ flags_ref = nullptr, uint32_t *__restrict__ diff = nullptr) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t i = tid; i < nz4; i += (uint64_t)gridDim.x * blockDim.x) zws[i] = make_uint4(0u, 0u, 0u, 0u);
    uint64_t r = lo + tid;
    if (r >= n) return;
    float ht, ny;
    if (band) {
        const float b = band[r];
        if (band_keep) band_keep[r] = b;   // the bands of this geometry (compared by the next frame)
        ht = roundf(h[r] + b);        // (h + band).round()  (:389)
        ny = roundf(b + WG_NODE_Y);   // (band + NODE_Y).round() (:390)
    } else {
        ht = h[r];                    // build(): height = h, node_y = NODE_Y (:339-341)
        ny = WG_NODE_Y;
    }
    height[r] = ht;
    node_y[r] = ny;
    const float top = row_top[r], bot = row_top[r + 1];
    const float node_abs = top + ny;          // child_y / parent_y of edges at this row (:554-555)
    uint8_t f = 0;
    if (bot - top < 1e-4f) f |= RF_ZERO;        // intermediate strip (:577)
    if (bot - node_abs < 1e-4f) f |= RF_CHILD;  // strip [child_y, row_bot]
    if (node_abs - top < 1e-4f) f |= RF_PARENT; // strip [row_top, parent_y]
    rowflags[r] = f;
    if (diff && flags_ref[r] != f) atomicOr(diff, 1u);   // the flags the curve lists were filtered with differ
}

// The full pass's first kernel, one thread per row:
//   * the row's edges (:301-320; when the layout stage left them to this pass:
//     prow != null) or their records (edges in place);
//   * RowGeometry {height, node_y} and the strip flags (k_row_basic);
//   * the child side of the per-row list counts (difference arrays for the
//     spans) and the sweep's carry-in counts per 64-row chunk (carry_diff):
//     edges are in child order, so these are plain stores, one carry count
//     per wave (its 64 rows share a chunk); the parent side follows per edge
//     with atomics (k_edge_counts, :526-528: child_row >= parent_row adds
//     nothing);
//   * the zeros the later atomics and fills start from (cntT, top_fill,
//     carry_fill, the flag words, the all-zero flag row) — every other count
//     array is written here in full.
struct EdgeRowsArgs {
    const uint32_t *edge_off;
    const uint32_t *poff;      // null: edges in place
    const int32_t *prow;
    const uint32_t *lane_out;
    const uint8_t *color_out;
    wg_edge *edges;
    const float *h, *band, *row_top;
    float *height, *node_y, *band_keep;
    uint8_t *rowflags, *zflags;
    uint8_t *flags_kept;       // the flags the curve lists are filtered with (rowflags_lists)
    uint32_t *cntB, *diffF, *diffC, *cntCend, *cntPend, *carry_diff, *cntT, *top_fill, *carry_fill, *misc;
};
// FUSED (r06): the workspace was zeroed beforehand (wg_geom_prezero, on the
// side stream beside the hash join), so the parent side of the counts
// (k_edge_counts) is added here too, per edge, and the child side goes in by
// atomics as well (a row's entries also collect other rows' parent-side
// adds): one launch and one pass over the edges fewer.
template <bool FUSED>
__global__ void __launch_bounds__(256) k_edges_rows(uint64_t n, EdgeRowsArgs A) {
    static_assert(WG_SWEEP_CH == 64, "a wave's rows are one sweep chunk");
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t cd = 0;
    // (FUSED) the parent side of the carry counts for the next four chunks,
    // 16 bits each: edges ending in one chunk all decrement one word, ~20-30
    // same-address atomics per chunk on the Linux shape (r06, as k_top_carry)
    uint64_t cdp = 0;
    if (r < n) {
        uint32_t b = 0, f = 0, cc = 0, ce = 0;
        const bool small = (A.prow ? A.poff[r + 1] - A.poff[r] : A.edge_off[r + 1] - A.edge_off[r]) < 0xFFFFu;
        // (plain accumulation, no by-reference closure: that put the counters in scratch)
#define WG_EDGE_COUNT(c_, p_, same_)                                                                 \
    do {                                                                                             \
        const uint32_t c = (c_), p = (p_);                                                           \
        if (c < p) {                                                                                 \
            const uint32_t k0_ = c / WG_SWEEP_CH + 1, k1_ = p / WG_SWEEP_CH;                          \
            cd += k0_ <= k1_;                                                                        \
            if (same_) { b++; f += c + 1 < p; }                                                      \
            else { cc += c + 1 < p; ce++; }   /* (the swept lists' flag row is all zero: no child-end filter) */ \
            if (FUSED) {   /* k_edge_counts' parent side (:526-528) */                               \
                if (k0_ <= k1_) {   /* near chunks: counted here, one atomic per wave and chunk below */ \
                    const uint32_t d_ = k1_ - c / WG_SWEEP_CH - 1u;                                   \
                    if (d_ < 4u && small) cdp += 1ull << (16u * d_);                                  \
                    else atomicAdd(&A.carry_diff[k1_ + 1], 0xFFFFFFFFu);                              \
                }                                                                                    \
                if (same_) {                                                                         \
                    atomicAdd(&A.cntT[p], 1u);                                                       \
                    if (c + 1 < p) atomicAdd(&A.diffF[p], 0xFFFFFFFFu);                              \
                } else {                                                                             \
                    if (c + 1 < p) atomicAdd(&A.diffC[p], 0xFFFFFFFFu);                              \
                    atomicAdd(&A.cntCend[p], 1u);                                                    \
                    atomicAdd(&A.cntPend[p], 1u);                                                    \
                }                                                                                    \
            }                                                                                        \
        }                                                                                            \
    } while (0)
        if (A.prow) {
            uint32_t o = A.edge_off[r];
            const uint32_t cl = A.lane_out[r], col = A.color_out[r];
            for (uint32_t k = A.poff[r]; k < A.poff[r + 1]; k++) {
                const int32_t p = A.prow[k];
                if (p < 0) continue;
                wg_edge e;
                e.child_row = (uint32_t)r;
                e.child_lane = cl;
                e.parent_row = (uint32_t)p;
                e.parent_lane = A.lane_out[p];
                e.color = col;
                A.edges[o] = e;
                o++;
                WG_EDGE_COUNT(e.child_row, e.parent_row, e.child_lane == e.parent_lane);
            }
        } else {
            for (uint32_t k = A.edge_off[r]; k < A.edge_off[r + 1]; k++) {
                const wg_edge e = A.edges[k];
                WG_EDGE_COUNT(e.child_row, e.parent_row, e.child_lane == e.parent_lane);
            }
        }
#undef WG_EDGE_COUNT
        A.cntB[r] = b;
        if (FUSED) {   // (zeroed; other rows' parent sides add into these entries)
            if (f) atomicAdd(&A.diffF[r + 1], f);
            if (cc) atomicAdd(&A.diffC[r + 1], cc);
            if (ce) atomicAdd(&A.cntCend[r], ce);
        } else {
            A.diffF[r + 1] = f;
            A.diffC[r + 1] = cc;
            A.cntCend[r] = ce;
            A.cntPend[r] = 0u;
            A.cntT[r] = 0u;
            A.top_fill[r] = 0u;
            A.zflags[r] = 0;
        }
        // RowGeometry (k_row_basic)
        float ht, ny;
        if (A.band) {
            const float bd = A.band[r];
            if (A.band_keep) A.band_keep[r] = bd;
            ht = roundf(A.h[r] + bd);        // (h + band).round()  (:389)
            ny = roundf(bd + WG_NODE_Y);     // (band + NODE_Y).round() (:390)
        } else {
            ht = A.h[r];                     // build(): height = h, node_y = NODE_Y (:339-341)
            ny = WG_NODE_Y;
        }
        A.height[r] = ht;
        A.node_y[r] = ny;
        const float top = A.row_top[r], bot = A.row_top[r + 1];
        const float node_abs = top + ny;
        uint8_t fl = 0;
        if (bot - top < 1e-4f) fl |= RF_ZERO;
        if (bot - node_abs < 1e-4f) fl |= RF_CHILD;
        if (node_abs - top < 1e-4f) fl |= RF_PARENT;
        A.rowflags[r] = fl;
        A.flags_kept[r] = fl;
    }
    if (!FUSED) {
        if (r == 0) { A.diffF[0] = 0u; A.diffC[0] = 0u; A.carry_diff[0] = 0u; }
        if (r < 64) A.misc[r] = 0u;
    }
    if (FUSED) {
        struct C5 { uint32_t v[5]; };
        C5 x{{cd, (uint32_t)cdp & 0xFFFFu, (uint32_t)(cdp >> 16) & 0xFFFFu, (uint32_t)(cdp >> 32) & 0xFFFFu,
              (uint32_t)(cdp >> 48)}};
        const C5 zero{{0u, 0u, 0u, 0u, 0u}};
        x = wg_wave_scan(x, zero, [](C5 a, const C5 &y) {
#pragma unroll
            for (int i = 0; i < 5; i++) a.v[i] += y.v[i];
            return a;
        });
        if ((threadIdx.x & 63) == 63 && r - 63 < n) {
            const uint64_t q = r / WG_SWEEP_CH;
            if (x.v[0]) atomicAdd(&A.carry_diff[q + 1], x.v[0]);
#pragma unroll
            for (int d = 1; d <= 4; d++)
                if (x.v[d]) atomicAdd(&A.carry_diff[q + d + 1], 0u - x.v[d]);
        }
        return;
    }
    const uint32_t tot = wg_wave_scan(cd, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    if ((threadIdx.x & 63) == 63 && r - 63 < n) {
        {
            A.carry_diff[r / WG_SWEEP_CH + 1] = tot;
            A.carry_fill[r / WG_SWEEP_CH] = 0u;
        }
    }
}

__global__ void k_edge_counts(uint64_t ne, const wg_edge *__restrict__ edges, const uint8_t *__restrict__ rowflags,
                              uint32_t *cntT, uint32_t *diffF, uint32_t *diffC, uint32_t *cntCend,
                              uint32_t *cntPend, uint32_t *carry_diff, const uint32_t *__restrict__ ne_dev) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= ne || (ne_dev && k >= *ne_dev)) return;
    const wg_edge e = edges[k];
    const uint32_t c = e.child_row, p = e.parent_row;
    if (c >= p) return;                                   // (:526-528)
    const uint32_t k0 = c / WG_SWEEP_CH + 1, k1 = p / WG_SWEEP_CH;
    if (k0 <= k1) atomicAdd(&carry_diff[k1 + 1], 0xFFFFFFFFu);
    if (e.child_lane == e.parent_lane) {
        atomicAdd(&cntT[p], 1u);
        if (c + 1 < p) atomicAdd(&diffF[p], 0xFFFFFFFFu);
    } else {
        if (c + 1 < p) atomicAdd(&diffC[p], 0xFFFFFFFFu);
        if (!(rowflags[p] & RF_PARENT)) atomicAdd(&cntCend[p], 1u);
        atomicAdd(&cntPend[p], 1u);   // (the parent-end share, for the filtered count)
    }
}

constexpr int GO_T = 256, GO_Q = 8;
constexpr uint64_t GO_TILE = (uint64_t)GO_T * GO_Q;

// 8 consecutive words at a 32-byte aligned address
__device__ __forceinline__ void ld8(const uint32_t *p, uint32_t (&v)[8]) {
    const uint4 a = reinterpret_cast<const uint4 *>(p)[0], b = reinterpret_cast<const uint4 *>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8(uint32_t *p, const uint32_t (&v)[8]) {
    reinterpret_cast<uint4 *>(p)[0] = make_uint4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<uint4 *>(p)[1] = make_uint4(v[4], v[5], v[6], v[7]);
}

// Tile sums (GO_TILE entries) of the three difference arrays the offsets
// kernel scans: the full-vertical and curve spans per row (n + 1 entries) and
// the sweep's carry-in counts per 64-row chunk (nch + 1 entries; tiles past
// its end sum to 0)
__global__ void __launch_bounds__(GO_T) k_tile_sums3(const uint32_t *__restrict__ F, const uint32_t *__restrict__ C,
                                                    const uint32_t *__restrict__ D, uint64_t n1, uint64_t nd1,
                                                    uint32_t *__restrict__ tsF, uint32_t *__restrict__ tsC,
                                                    uint32_t *__restrict__ tsD) {
    __shared__ uint32_t ws[GO_T / 64];
    const int a = blockIdx.y;
    const uint32_t *in = a == 0 ? F : (a == 1 ? C : D);
    const uint64_t len = a == 2 ? nd1 : n1;
    const uint64_t base = (uint64_t)blockIdx.x * GO_TILE + (uint64_t)threadIdx.x * GO_Q;
    uint32_t v[GO_Q];
    if (base + GO_Q <= len) ld8(in + base, v);
    else
#pragma unroll
        for (int k = 0; k < GO_Q; k++) v[k] = base + k < len ? in[base + k] : 0u;
    uint32_t t = 0;
#pragma unroll
    for (int k = 0; k < GO_Q; k++) t += v[k];
    t = wg_wave_scan(t, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < GO_T / 64; w++) tot += ws[w];
        (a == 0 ? tsF : (a == 1 ? tsC : tsD))[blockIdx.x] = tot;
    }
}

// ordered exclusive block scan (GO_T threads) of two values at once (defined below)
__device__ __forceinline__ uint2 go_block_excl(uint2 v, uint2 &tot);

// The sweep's carry-in counts of chunks [base, base + 8) from the chunk
// difference array D (nch + 1 entries, the tile's exclusive offset pre): the
// count of chunk k is the exclusive scan of D at k + 1; written over D[k]
// (each thread reads its entries before it writes them), with their 256-entry
// sums for the carry offsets' scan (wg_scan_bs_u32)
__device__ __forceinline__ void carry_counts(uint32_t *D, uint64_t nch, uint64_t base, uint32_t pre, uint32_t *bsD,
                                             uint64_t nbsD) {
    uint32_t v[GO_Q];
    if (base + GO_Q <= nch + 1) ld8(D + base, v);
    else
#pragma unroll
        for (int k = 0; k < GO_Q; k++) v[k] = base + k <= nch ? D[base + k] : 0u;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < GO_Q; k++) s += v[k];
    uint2 tot;
    uint32_t run = go_block_excl(make_uint2(s, 0u), tot).x + pre;
    uint32_t ex[GO_Q + 1];
#pragma unroll
    for (int k = 0; k < GO_Q; k++) { ex[k] = run; run += v[k]; }
    ex[GO_Q] = run;   // the next entry's exclusive value
    uint32_t cnt[GO_Q], t = 0;
#pragma unroll
    for (int k = 0; k < GO_Q; k++) {
        cnt[k] = base + k < nch ? ex[k + 1] : 0u;
        t += cnt[k];
    }
    if (base + GO_Q <= nch) st8(D + base, cnt);
    else
#pragma unroll
        for (int k = 0; k < GO_Q; k++)
            if (base + k < nch) D[base + k] = cnt[k];
#pragma unroll
    for (int d = 16; d >= 1; d >>= 1) t += (uint32_t)__shfl_xor((int)t, d, 64);
    const uint64_t sub = base / WG_BS_THREADS;
    if ((threadIdx.x & 31) == 0 && sub < nbsD) bsD[sub] = t;
}

// ordered exclusive block scan (GO_T threads) of two values at once
__device__ __forceinline__ uint2 go_block_excl(uint2 v, uint2 &tot) {
    __shared__ uint2 ws[GO_T / 64];
    const uint32_t a = wg_wave_scan(v.x, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    const uint32_t b = wg_wave_scan(v.y, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 63) ws[w] = make_uint2(a, b);
    __syncthreads();
    uint2 base = make_uint2(0u, 0u), t = make_uint2(0u, 0u);
#pragma unroll
    for (int k = 0; k < GO_T / 64; k++) {
        const uint2 q = ws[k];
        if (k < w) { base.x += q.x; base.y += q.y; }
        t.x += q.x; t.y += q.y;
    }
    __syncthreads();
    tot = t;
    return make_uint2(base.x + a - v.x, base.y + b - v.y);
}

// One launch after the tile sums of the two difference arrays (scanned
// over n + 1 entries, in place): the per-row span counts, the per-row list
// totals nV = nF + nT + nB (-> vert_off), nC (-> scurve_off, the superset:
// the flag row is all zero) and nK (-> curve_off, the superset filtered by
// the pass's strip flags, :577: a row's crossing, child-end and parent-end
// segments each dropped as a group by its flag) and their 256-row sums for
// the offsets' scan (wg_scan_bs_u32).
__global__ void __launch_bounds__(GO_T) k_geom_offsets(uint64_t n, uint32_t *F, uint32_t *C, const uint32_t *__restrict__ tsF,
                                                      const uint32_t *__restrict__ tsC, const uint32_t *__restrict__ cntT,
                                                      const uint32_t *__restrict__ cntB, const uint32_t *__restrict__ cntCend,
                                                      uint32_t *__restrict__ nV, uint32_t *__restrict__ nC,
                                                      uint32_t *__restrict__ bsV, uint32_t *__restrict__ bsC, uint64_t nbs,
                                                      uint32_t *D, const uint32_t *__restrict__ tsD, uint64_t nch,
                                                      uint32_t *__restrict__ bsD, uint64_t nbsD,
                                                      const uint32_t *__restrict__ cntPend,
                                                      const uint8_t *__restrict__ rowflags, uint32_t *__restrict__ nK,
                                                      uint32_t *__restrict__ bsK) {
    uint2 pre = make_uint2(0u, 0u), ptot;
    uint2 preD = make_uint2(0u, 0u), ptotD;
    for (uint64_t b = threadIdx.x; b < blockIdx.x; b += GO_T) { pre.x += tsF[b]; pre.y += tsC[b]; preD.x += tsD[b]; }
    (void)go_block_excl(pre, ptot);
    (void)go_block_excl(preD, ptotD);
    carry_counts(D, nch, (uint64_t)blockIdx.x * GO_TILE + (uint64_t)threadIdx.x * GO_Q, ptotD.x, bsD, nbsD);
    const uint64_t base = (uint64_t)blockIdx.x * GO_TILE + (uint64_t)threadIdx.x * GO_Q;
    uint32_t vF[GO_Q], vC[GO_Q], vT[GO_Q], vB[GO_Q], vE[GO_Q], vP[GO_Q], vR[GO_Q];
    const bool full = base + GO_Q <= n;   // every item a row (and within the n + 1 entries): 16-byte accesses
    if (full) {
        ld8(F + base, vF); ld8(C + base, vC); ld8(cntT + base, vT); ld8(cntB + base, vB); ld8(cntCend + base, vE);
        ld8(cntPend + base, vP);
        const uint2 f8 = *reinterpret_cast<const uint2 *>(rowflags + base);
#pragma unroll
        for (int k = 0; k < 4; k++) { vR[k] = (f8.x >> (8 * k)) & 0xFFu; vR[k + 4] = (f8.y >> (8 * k)) & 0xFFu; }
    } else {
#pragma unroll
        for (int k = 0; k < GO_Q; k++) {
            const bool in = base + k <= n;   // n + 1 entries
            vF[k] = in ? F[base + k] : 0u;
            vC[k] = in ? C[base + k] : 0u;
            const bool row = base + k < n;
            vT[k] = row ? cntT[base + k] : 0u;
            vB[k] = row ? cntB[base + k] : 0u;
            vE[k] = row ? cntCend[base + k] : 0u;
            vP[k] = row ? cntPend[base + k] : 0u;
            vR[k] = row ? rowflags[base + k] : 0u;
        }
    }
    uint2 sum = make_uint2(0u, 0u);
#pragma unroll
    for (int k = 0; k < GO_Q; k++) {
        sum.x += vF[k];
        sum.y += vC[k];
    }
    uint2 tot;
    uint2 run = go_block_excl(sum, tot);
    run.x += ptot.x;
    run.y += ptot.y;
    uint32_t tV = 0, tC = 0, tK = 0;
    uint32_t oF[GO_Q], oC[GO_Q], oV[GO_Q], oN[GO_Q], oK[GO_Q];
#pragma unroll
    for (int k = 0; k < GO_Q; k++) {
        oF[k] = run.x;
        oC[k] = run.y;
        run.x += vF[k];
        run.y += vC[k];
        // run = the exclusive value at row + 1: the edges alive across the row
        oV[k] = run.x + vT[k] + vB[k];
        oN[k] = run.y + vE[k];
        // kept: crossing (c < r < p) unless RF_ZERO, child-end (r == c) unless
        // RF_CHILD, parent-end (r == p) unless RF_PARENT (curve_kept)
        const uint32_t f = vR[k];
        oK[k] = ((f & RF_ZERO) ? 0u : run.y) + ((f & RF_CHILD) ? 0u : vE[k] - vP[k]) + ((f & RF_PARENT) ? 0u : vP[k]);
        if (base + k < n) { tV += oV[k]; tC += oN[k]; tK += oK[k]; }
    }
    if (full) {
        st8(F + base, oF); st8(C + base, oC); st8(nV + base, oV); st8(nC + base, oN); st8(nK + base, oK);
    } else {
#pragma unroll
        for (int k = 0; k < GO_Q; k++) {
            const uint64_t i = base + k;
            if (i <= n) { F[i] = oF[k]; C[i] = oC[k]; }
            if (i < n) { nV[i] = oV[k]; nC[i] = oN[k]; nK[i] = oK[k]; }
        }
    }
    // 256-row sums: 32 threads x 8 rows
#pragma unroll
    for (int d = 16; d >= 1; d >>= 1) {
        tV += (uint32_t)__shfl_xor((int)tV, d, 64);
        tC += (uint32_t)__shfl_xor((int)tC, d, 64);
        tK += (uint32_t)__shfl_xor((int)tK, d, 64);
    }
    const uint64_t sub = (uint64_t)blockIdx.x * (GO_TILE / WG_BS_THREADS) + threadIdx.x / 32;
    if ((threadIdx.x & 31) == 0 && sub < nbs) { bsV[sub] = tV; bsC[sub] = tC; bsK[sub] = tK; }
}

// one pass over the edges: same-lane edges' ids into their parent row's
// top-half slots (sorted and packed by the sweep wave, top_finish_row), and every edge into
// the carry-in list of each 64-row chunk it is alive across (sorted by
// k_carry_sort)
// The (edge, chunk) registrations of a wave's 64 edges are dealt to its
// lanes in turn: an edge alive across thousands of chunks (a long-lived
// branch of a wide list) no longer loops alone while its wave waits
// (linuxwide: 344 us with one lane per edge)
__global__ void __launch_bounds__(256) k_top_carry(uint64_t ne, const wg_edge *__restrict__ edges,
                            const uint32_t *__restrict__ vert_off,
                            const uint32_t *__restrict__ scanF, uint32_t *top_fill, uint32_t *vert,
                            const uint32_t *__restrict__ carry_off, uint32_t *carry_fill, uint32_t *carry,
                            const uint32_t *__restrict__ ne_dev, Cap vc, Cap cc, uint32_t *ovf) {
    __shared__ uint32_t s_pre[256 / 64][64], s_k0[256 / 64][64];
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lid = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const Cap gs[2] = {vc, cc};
    if (over_all(gs, ovf)) return;   // (uniform)
    const bool valid = k < ne && !(ne_dev && k >= *ne_dev);
    wg_edge e{};
    if (valid) e = edges[k];
    const bool live = valid && e.child_row < e.parent_row;
    const uint32_t k0 = e.child_row / WG_SWEEP_CH + 1, k1 = e.parent_row / WG_SWEEP_CH;
    const uint32_t span = (live && k1 >= k0) ? k1 - k0 + 1 : 0u;
    const uint32_t inc = wg_wave_scan(span, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    s_pre[wv][lid] = inc - span;
    s_k0[wv][lid] = k0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t kbase = k - lid;
    // the top-half slot first: its atomic in flight beside the registrations'
    const bool top = live && e.child_lane == e.parent_lane;
    const uint32_t p = e.parent_row;
    uint32_t tpos = 0;
    if (top) tpos = atomicAdd(&top_fill[p], 1u);
    for (uint32_t base = 0; base < tot; base += 64) {   // (uniform)
        const uint32_t t = base + lid;
        const bool act = t < tot;
        // the edge: the last lane whose exclusive start is <= t (lanes with
        // no registration share the next lane's start and come before it)
        uint32_t l = 0, q = 0;
        if (act) {
#pragma unroll
            for (uint32_t step = 32; step; step >>= 1)
                if (s_pre[wv][l + step] <= t) l += step;
            q = s_k0[wv][l] + (t - s_pre[wv][l]);
        }
        // r06: the batch's registrations into one chunk share one atomic (a
        // wave's edges start within ~64 rows, so a batch meets a few chunks;
        // one atomic per registration queued ~27 same-address adds per chunk
        // on the Linux shape), all of the batch's atomics in flight at once
        uint64_t pend = __ballot(act);
        uint32_t mine = 0, leader = 0, rank = 0;
        while (pend) {   // (uniform: one round per distinct chunk)
            const uint32_t lead = (uint32_t)__builtin_ctzll(pend);
            const uint32_t qq = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)lead);
            const bool in = act && q == qq;
            const uint64_t m = __ballot(in);
            if (lid == lead) mine = atomicAdd(&carry_fill[qq], (uint32_t)__builtin_popcountll(m));
            if (in) {
                leader = lead;
                rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            }
            pend &= ~m;
        }
        const uint32_t pos = (uint32_t)__shfl((int)mine, (int)leader, 64) + rank;
        if (act) carry[carry_off[q] + pos] = (uint32_t)(kbase + l);
    }
    if (!top) return;
    vert[vert_off[p] + scanF[p + 1] + tpos] = (uint32_t)k;   // edge id, packed below
}

// ---- carry-in registration for the sweep -------------------------------------
// rank sort of each chunk's carry list (one wave per chunk; lists are short)
__global__ void __launch_bounds__(64) k_carry_sort(uint64_t nch, const uint32_t *__restrict__ carry_off,
                                                    const uint32_t *__restrict__ carry, uint32_t *__restrict__ sorted,
                                                    Cap cc, uint32_t *ovf) {
    const uint64_t q = blockIdx.x;
    if (over(cc, ovf) || q >= nch) return;
    const uint32_t a = carry_off[q], b = carry_off[q + 1], len = b - a;
    for (uint32_t i = threadIdx.x; i < len; i += 64) {
        const uint32_t x = carry[a + i];
        uint32_t rank = 0;
        for (uint32_t j = 0; j < len; j++) rank += carry[a + j] < x;
        sorted[a + rank] = x;
    }
}

// ---- the sweep ---------------------------------------------------------------------
constexpr int SW_WAVES = 4;
constexpr int SW_CAP = 1024;  // edges alive across one row (per wave of the LDS sweep)
constexpr int SW_CAP_BLOCK = SW_WAVES * SW_CAP;   // ... a chunk past that: one wave with the block's whole pool
constexpr int SW_NE = 192;    // edges starting inside the 64-row chunk, staged in LDS
constexpr int SW_LDS_BLOCKS = 512;

__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Fallback sweep for chunks with more edges than the register sweep holds:
// active list in LDS (cap entries), appended / compacted row by row.  False
// when more than cap edges are alive across a row: the chunk's entries
// written so far sit at their final offsets, and the sweep with a larger
// list rewrites all of them.
__device__ bool sweep_chunk_lds(uint32_t cap, uint64_t q, uint64_t n, const wg_edge *__restrict__ edges,
        const uint32_t *__restrict__ edge_off, const uint32_t *__restrict__ carry_off,
        const uint32_t *__restrict__ carry_sorted, const uint8_t *__restrict__ rowflags,
        const uint32_t *__restrict__ vert_off, const uint32_t *__restrict__ curve_off,
        uint32_t *__restrict__ vert, uint32_t *__restrict__ curve_ref, uint32_t *__restrict__ curve_row,
        const uint32_t *__restrict__ kept_off, uint32_t *__restrict__ kept_ref, uint32_t *__restrict__ kept_row,
        uint32_t *__restrict__ err, uint32_t *E, uint32_t *C, uint32_t *P, uint32_t *I, uint32_t *NC, uint32_t *NP,
        uint32_t *NI, bool super) {
    const uint32_t lid = threadIdx.x & 63;
    const uint64_t R0 = q * WG_SWEEP_CH, R1 = (R0 + WG_SWEEP_CH < n) ? R0 + WG_SWEEP_CH : n;
    const uint32_t nr = (uint32_t)(R1 - R0);
    // per-row scalars of the chunk, one row per lane
    const uint64_t rr = R0 + lid;
    const uint32_t eoff_v = lid < nr ? edge_off[rr] : 0u;
    const uint32_t rf_v = lid < nr ? rowflags[rr] : 0u;
    const uint32_t voff_v = (!super && lid < nr) ? vert_off[rr] : 0u;
    const uint32_t coff_v = (super && lid < nr) ? curve_off[rr] : 0u;
    const uint32_t koff_v = (!super && lid < nr) ? kept_off[rr] : 0u;
    const uint32_t E1 = edge_off[R1];
    const uint32_t E0 = (uint32_t)__builtin_amdgcn_readlane((int)eoff_v, 0);
    const bool staged = E1 - E0 <= (uint32_t)SW_NE;
    // carry-in edges (alive across R0), sorted by edge id
    uint32_t cnt = 0;
    {
        const uint32_t a = carry_off[q], b = carry_off[q + 1];
        if (b - a > cap) return false;
        for (uint32_t i = lid; i < b - a; i += 64) {
            const uint32_t k = carry_sorted[a + i];
            const wg_edge e = edges[k];
            E[i] = k; C[i] = e.child_row; P[i] = e.parent_row;
            I[i] = (e.child_lane & 0xFFFFFFu) | (e.color << 24) | ((e.child_lane == e.parent_lane) ? 0x10000000u : 0u);
        }
        cnt = b - a;
    }
    // the chunk's own edges, staged once (coalesced)
    if (staged) {
        for (uint32_t i = lid; i < E1 - E0; i += 64) {
            const wg_edge e = edges[E0 + i];
            NC[i] = e.child_row; NP[i] = e.parent_row;
            NI[i] = (e.child_lane & 0xFFFFFFu) | (e.color << 24) | ((e.child_lane == e.parent_lane) ? 0x10000000u : 0u);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t j = 0; j < nr; j++) {
        const uint64_t r = R0 + j;
        // append edges whose child is row r (edge order)
        const uint32_t e0 = (uint32_t)__builtin_amdgcn_readlane((int)eoff_v, (int)j);
        const uint32_t e1 = (j + 1 < nr) ? (uint32_t)__builtin_amdgcn_readlane((int)eoff_v, (int)(j + 1)) : E1;
        for (uint32_t base = e0; base < e1; base += 64) {
            const uint32_t k = base + lid;
            bool take = false;
            uint32_t c = 0, p = 0, info = 0;
            if (k < e1) {
                if (staged) { c = NC[k - E0]; p = NP[k - E0]; info = NI[k - E0]; }
                else {
                    const wg_edge e = edges[k];
                    c = e.child_row; p = e.parent_row;
                    info = (e.child_lane & 0xFFFFFFu) | (e.color << 24) | ((e.child_lane == e.parent_lane) ? 0x10000000u : 0u);
                }
                take = c < p;
            }
            const uint64_t m = __ballot(take);
            if (cnt + __builtin_popcountll(m) > cap) return false;
            if (take) {
                const uint32_t pos = cnt + mbcnt(m);
                E[pos] = k; C[pos] = c; P[pos] = p; I[pos] = info;
            }
            cnt += __builtin_popcountll(m);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const uint32_t rf = (uint32_t)__builtin_amdgcn_readlane((int)rf_v, (int)j);
        uint32_t fbase = (uint32_t)__builtin_amdgcn_readlane((int)voff_v, (int)j);
        uint32_t cbase = (uint32_t)__builtin_amdgcn_readlane((int)coff_v, (int)j);
        uint32_t kbase = (uint32_t)__builtin_amdgcn_readlane((int)koff_v, (int)j);
        uint32_t kept = 0;
        for (uint32_t base = 0; base < cnt; base += 64) {
            const uint32_t idx = base + lid;
            const bool act = idx < cnt;
            uint32_t eid = 0, c = 0, p = 0, info = 0;
            if (act) { eid = E[idx]; c = C[idx]; p = P[idx]; info = I[idx]; }
            __builtin_amdgcn_wave_barrier();
            const bool same = (info & 0x10000000u) != 0;
            const bool full = !super && act && same && c < r && r < p;
            const bool skip = (r == c) ? (rf & RF_CHILD) : (r == p) ? (rf & RF_PARENT) : (rf & RF_ZERO);
            const bool seg = act && !same && c <= r && r <= p;
            const bool curv = super && seg;           // the superset (no strip flag)
            const bool kcur = !super && seg && !skip; // this pass's filtered list
            const bool keep = act && p > r;
            const uint64_t mf = __ballot(full), mc = __ballot(curv), mk = __ballot(keep), mq = __ballot(kcur);
            if (full) vert[fbase + mbcnt(mf)] = pack_vert(info & 0xFFFFFFu, WG_VERT_FULL, (info >> 24) & 0xFu);
            if (curv) { const uint32_t o = cbase + mbcnt(mc); curve_ref[o] = eid; curve_row[o] = (uint32_t)r; }
            if (kcur) { const uint32_t o = kbase + mbcnt(mq); kept_ref[o] = eid; kept_row[o] = (uint32_t)r; }
            if (keep) {
                const uint32_t o = kept + mbcnt(mk);
                E[o] = eid; C[o] = c; P[o] = p; I[o] = info;
            }
            fbase += __builtin_popcountll(mf);
            cbase += __builtin_popcountll(mc);
            kbase += __builtin_popcountll(mq);
            kept += __builtin_popcountll(mk);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        cnt = kept;
    }
    return true;
}

__global__ void __launch_bounds__(64 * SW_WAVES) k_sweep_lds(uint64_t n, const uint32_t *__restrict__ list,
        const uint32_t *__restrict__ list_n, const wg_edge *__restrict__ edges,
        const uint32_t *__restrict__ edge_off, const uint32_t *__restrict__ carry_off,
        const uint32_t *__restrict__ carry_sorted, const uint8_t *__restrict__ rowflags,
        const uint32_t *__restrict__ vert_off, const uint32_t *__restrict__ curve_off,
        uint32_t *__restrict__ vert, uint32_t *__restrict__ curve_ref, uint32_t *__restrict__ curve_row,
        const uint32_t *__restrict__ kept_off, uint32_t *__restrict__ kept_ref, uint32_t *__restrict__ kept_row,
        uint32_t *__restrict__ err, Cap vc, Cap sc, uint32_t *ovf, bool super, const uint32_t *__restrict__ run_if,
        const uint32_t *__restrict__ done) {
    if (super && (*run_if == 0 || *done != 0)) return;   // (uniform over the grid)
    const Cap gs[2] = {vc, sc};
    if (over_all(gs, ovf)) return;
    __shared__ uint32_t s_eid[SW_CAP_BLOCK];
    __shared__ uint32_t s_c[SW_CAP_BLOCK];
    __shared__ uint32_t s_p[SW_CAP_BLOCK];
    __shared__ uint32_t s_info[SW_CAP_BLOCK];
    __shared__ uint32_t n_c[SW_WAVES][SW_NE];
    __shared__ uint32_t n_p[SW_WAVES][SW_NE];
    __shared__ uint32_t n_info[SW_WAVES][SW_NE];
    __shared__ uint32_t wide[64], n_wide;   // this block's chunks past one wave's list
    const int w = threadIdx.x >> 6;
    if (threadIdx.x == 0) n_wide = 0;
    __syncthreads();
    const uint32_t cnt = *list_n;
    for (uint32_t i = blockIdx.x * SW_WAVES + w; i < cnt; i += gridDim.x * SW_WAVES) {
        const uint32_t o = (uint32_t)w * SW_CAP;
        const bool ok = sweep_chunk_lds(SW_CAP, list[i], n, edges, edge_off, carry_off, carry_sorted, rowflags, vert_off,
                                        curve_off, vert, curve_ref, curve_row, kept_off, kept_ref, kept_row, err,
                                        s_eid + o, s_c + o, s_p + o,
                                        s_info + o, n_c[w], n_p[w], n_info[w], super);
        if (!ok && (threadIdx.x & 63) == 0) {
            const uint32_t at = atomicAdd(&n_wide, 1u);
            if (at < 64u) wide[at] = list[i];
            else atomicOr(&err[0], 1u);
        }
    }
    __syncthreads();
    // the wide chunks: wave 0 with every wave's list (a few rows of a list
    // with more than a thousand lanes; more than SW_CAP_BLOCK alive: error)
    const uint32_t nw = n_wide < 64u ? n_wide : 64u;
    if (w == 0)
        for (uint32_t j = 0; j < nw; j++)
            if (!sweep_chunk_lds(SW_CAP_BLOCK, wide[j], n, edges, edge_off, carry_off, carry_sorted, rowflags, vert_off,
                                 curve_off, vert, curve_ref, curve_row, kept_off, kept_ref, kept_row, err, s_eid, s_c,
                                 s_p, s_info, n_c[0], n_p[0],
                                 n_info[0], super) &&
                (threadIdx.x & 63) == 0)
                atomicOr(&err[0], 1u);
}

// The sweep: one wave per 64-row chunk.  A chunk's edge set is fixed — the
// edges alive across its first row (carry-in, edge order) followed by the
// edges whose child row lies in the chunk (edge order) — so it is held in
// registers (slot s of lane l = set entry 64 s + l) and every row's ordered
// full / curve lists are ballots over "alive at this row": no LDS, no
// per-row compaction.  Chunks with more than 64 * SW_SLOTS edges go to the
// LDS sweep above.
constexpr int SW_SLOTS = 8;

// The chunk's carry-in list (registration order) ranked into edge order:
// edge ids are distinct, so rank = the number of smaller ids.  The list is
// staged once in the wave's LDS (padded with ~0, which no id exceeds) and
// ranked from there, four ids per broadcast read — a rank loop over HBM
// waits one load latency per id (a 160-lane list: 80 waits per lane).
constexpr uint32_t SW_STAGE = 64u * SW_SLOTS;   // ids staged per wave
__device__ __forceinline__ void carry_rank(const uint32_t *__restrict__ carry, uint32_t len, uint32_t *stage,
                                           uint32_t *out) {
    const uint32_t lid = threadIdx.x & 63;
    if (len > SW_STAGE) {   // (the LDS-sweep chunks only: ranked from HBM)
        for (uint32_t i = lid; i < len; i += 64) {
            const uint32_t x = carry[i];
            uint32_t rank = 0;
            for (uint32_t j = 0; j < len; j++) rank += carry[j] < x;
            out[rank] = x;
        }
        return;
    }
    for (uint32_t i = lid; i < ((len + 3) & ~3u); i += 64) stage[i] = i < len ? carry[i] : ~0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint4 *s4 = reinterpret_cast<const uint4 *>(stage);
    for (uint32_t i = lid; i < len; i += 64) {
        const uint32_t x = stage[i];
        uint32_t rank = 0;
        for (uint32_t j = 0; j < (len + 3) / 4; j++) {
            const uint4 v = s4[j];
            rank += (v.x < x) + (v.y < x) + (v.z < x) + (v.w < x);
        }
        out[rank] = x;
    }
}

// SUPER = false (a full pass): the full verticals and this pass's curve lists
// filtered by the rows' strip flags; true (a frame pass whose flags differ
// from the full pass's, run_if != 0, once per layout: done): the flag-free
// curve superset the frame filter takes (k_curve_keep / k_curve_compact)
// per row (one lane each, before the sweep's row loop): the top-half entries
// (edge ids placed by k_top_carry) sorted by edge id and packed, then the
// bottom halves (same-lane edges of child r, in parent order) after them.
// r06: the row's offsets come with the sweep's prologue; its ids (up to
// TF_REG in registers; more are sorted in memory) and its own edges load in
// one round, the top edges' gather in the next.
constexpr int TF_REG = 4;
__device__ __forceinline__ void top_finish_row(uint32_t *__restrict__ vert, const wg_edge *__restrict__ edges, uint32_t tpos,
                                               uint32_t nt, uint32_t ea, uint32_t eb) {
    uint32_t tk[TF_REG];
    wg_edge be[TF_REG];
#pragma unroll
    for (int i = 0; i < TF_REG; i++) {
        tk[i] = ~0u;
        if ((uint32_t)i < nt) tk[i] = vert[tpos + i];
        be[i] = wg_edge{1u, 0u, 0u, 1u, 0u};   // (not live)
        if (ea + (uint32_t)i < eb) be[i] = edges[ea + i];
    }
    uint32_t *v = vert + tpos;
    if (nt <= (uint32_t)TF_REG) {
        // sorting network (ids distinct; the padding ~0 sorts last)
#define WG_TF_CX(i, j)                                                  \
        if (tk[j] < tk[i]) { const uint32_t t_ = tk[i]; tk[i] = tk[j]; tk[j] = t_; }
        WG_TF_CX(0, 1) WG_TF_CX(2, 3) WG_TF_CX(0, 2) WG_TF_CX(1, 3) WG_TF_CX(1, 2)
#undef WG_TF_CX
        wg_edge te[TF_REG];
#pragma unroll
        for (int i = 0; i < TF_REG; i++)
            if ((uint32_t)i < nt) te[i] = edges[tk[i]];
#pragma unroll
        for (int i = 0; i < TF_REG; i++)
            if ((uint32_t)i < nt) v[i] = pack_vert(te[i].child_lane, WG_VERT_TOP, te[i].color);
    } else {   // (in-degree past TF_REG: insertion sort by edge id in memory)
        for (uint32_t i = 1; i < nt; i++) {
            const uint32_t x = v[i];
            uint32_t j = i;
            while (j > 0 && v[j - 1] > x) { v[j] = v[j - 1]; j--; }
            v[j] = x;
        }
        for (uint32_t i = 0; i < nt; i++) {
            const wg_edge e = edges[v[i]];
            v[i] = pack_vert(e.child_lane, WG_VERT_TOP, e.color);
        }
    }
    uint32_t o = nt;
#pragma unroll
    for (int i = 0; i < TF_REG; i++) {
        const wg_edge e = be[i];
        if (e.child_row < e.parent_row && e.child_lane == e.parent_lane) v[o++] = pack_vert(e.child_lane, WG_VERT_BOTTOM, e.color);
    }
    for (uint32_t k = ea + TF_REG; k < eb; k++) {   // (rows with more parents)
        const wg_edge e = edges[k];
        if (e.child_row < e.parent_row && e.child_lane == e.parent_lane) v[o++] = pack_vert(e.child_lane, WG_VERT_BOTTOM, e.color);
    }
}

template <bool SUPER>
__global__ void __launch_bounds__(64 * SW_WAVES) k_sweep(uint64_t n, uint64_t q0, uint64_t q1, const wg_edge *__restrict__ edges,
        const uint32_t *__restrict__ edge_off, const uint32_t *__restrict__ carry_off,
        const uint32_t *__restrict__ carry, uint32_t *__restrict__ carry_sorted, const uint8_t *__restrict__ rowflags,
        const uint32_t *__restrict__ vert_off, const uint32_t *__restrict__ curve_off,
        uint32_t *__restrict__ vert, uint32_t *__restrict__ curve_ref, uint32_t *__restrict__ curve_row,
        const uint32_t *__restrict__ kept_off, uint32_t *__restrict__ kept_ref, uint32_t *__restrict__ kept_row,
        uint32_t *__restrict__ big, uint32_t *__restrict__ big_n, uint32_t reg_cap, Cap vc, Cap sc, Cap cc, uint32_t *ovf,
        const uint32_t *__restrict__ run_if, const uint32_t *__restrict__ done, const uint32_t *__restrict__ scanF,
        const uint32_t *__restrict__ cntT, uint32_t lds_off) {
    __shared__ uint32_t s_car[SW_WAVES][64 * SW_SLOTS];
    __shared__ __attribute__((aligned(16))) uint32_t s_stage[SW_WAVES][SW_STAGE];
    const uint32_t lid = threadIdx.x & 63;
    const uint64_t q = q0 + (uint64_t)blockIdx.x * SW_WAVES + (threadIdx.x >> 6);   // chunks [q0, q1)
    // Every load that depends on nothing else is issued before any is waited
    // on (r06): the guards, the chunk's carry and edge ranges and the per-row
    // scalars (a tail wave past q1 reads chunk q1 - 1's and returns below).
    const uint64_t qc = q < q1 ? q : q1 - 1;
    const uint64_t R0 = qc * WG_SWEEP_CH, R1 = (R0 + WG_SWEEP_CH < n) ? R0 + WG_SWEEP_CH : n;
    const uint32_t nr = (uint32_t)(R1 - R0);
    const uint64_t rr = R0 + lid;
    const bool inr = lid < nr;
    const uint32_t a = carry_off[qc], a1 = carry_off[qc + 1];
    const uint32_t E0 = edge_off[R0], E1 = edge_off[R1];
    const uint32_t voff_v = (!SUPER && inr) ? vert_off[rr] : 0u;
    const uint32_t coff_v = (SUPER && inr) ? curve_off[rr] : 0u;
    const uint32_t koff_v = (!SUPER && inr) ? kept_off[rr] : 0u;
    const uint32_t rf_v = (!SUPER && inr) ? rowflags[rr] : 0u;
    const uint32_t nf_v = (!SUPER && inr) ? scanF[rr + 1] : 0u;   // the row's full verticals (its tops follow them)
    const uint32_t nt_v = (!SUPER && inr) ? cntT[rr] : 0u;        // ... and its top halves (the bottoms follow)
    const uint32_t ea_v = (!SUPER && inr) ? edge_off[rr] : 0u, eb_v = (!SUPER && inr) ? edge_off[rr + 1] : 0u;
    const Cap gs[3] = {vc, sc, cc};
    const CapVals<3> gv = cap_read(gs, ovf);
    if (SUPER) {
        const uint32_t ri = *run_if, dn = *done;
        if ((ri == 0) | (dn != 0)) return;
    }
    if (cap_over(gv, gs, ovf) || q >= q1) return;
    if (!SUPER && inr) top_finish_row(vert, edges, voff_v + nf_v, nt_v, ea_v, eb_v);
    const uint32_t ncar = a1 - a;
    const uint32_t total = ncar + (E1 - E0);
    if (total > reg_cap || total > 64u * SW_SLOTS) {   // the LDS sweep (k_sweep_lds) reads the ranked list from HBM
        if (lds_off) {   // (not launched: the pass is redone exactly)
            if (lid == 0) atomicOr(ovf, 1u);
            return;
        }
        carry_rank(carry + a, ncar, s_stage[threadIdx.x >> 6], carry_sorted + a);
        if (lid == 0) big[atomicAdd(big_n, 1u)] = (uint32_t)q;
        return;
    }
    const uint32_t nslots = (total + 63) / 64;
    uint32_t *sorted = s_car[threadIdx.x >> 6];
    carry_rank(carry + a, ncar, s_stage[threadIdx.x >> 6], sorted);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // per slot: the edge id, the packed full-vertical entry, two row windows
    // as (first row, length - 1) for an unsigned compare — full verticals on
    // rows c < r < p of same-lane edges, curve segments on rows c <= r <= p of
    // cross-lane edges; an empty window has first row ~0.  A full pass writes the curve list filtered by
    // the row's strip flags (every segment of a row without flags); the
    // flag-free superset is swept only for a frame pass whose flags differ
    // (SUPER).
    uint32_t ek[SW_SLOTS], fb[SW_SLOTS], fl[SW_SLOTS], cb[SW_SLOTS], cl[SW_SLOTS], pv[SW_SLOTS];
#pragma unroll
    for (int sl = 0; sl < SW_SLOTS; sl++) {
        const uint32_t idx = 64u * sl + lid;
        ek[sl] = 0; fb[sl] = ~0u; fl[sl] = 0; cb[sl] = ~0u; cl[sl] = 0; pv[sl] = 0;
        if ((uint32_t)sl < nslots && idx < total) {
            const uint32_t k = idx < ncar ? sorted[idx] : E0 + (idx - ncar);
            const wg_edge e = edges[k];
            ek[sl] = k;
            const uint32_t c = e.child_row, p = e.parent_row;
            if (c < p) {
                if (e.child_lane == e.parent_lane) {
                    if (c + 1 < p) { fb[sl] = c + 1; fl[sl] = p - c - 2; }
                    pv[sl] = pack_vert(e.child_lane & 0xFFFFFFu, WG_VERT_FULL, e.color & 0xFu);
                } else {
                    cb[sl] = c;
                    cl[sl] = p - c;
                }
            }
        }
    }
    for (uint32_t j = 0; j < nr; j++) {
        const uint32_t r = (uint32_t)(R0 + j);
        uint32_t fbase = (uint32_t)__builtin_amdgcn_readlane((int)voff_v, (int)j);
        uint32_t cbase = (uint32_t)__builtin_amdgcn_readlane((int)coff_v, (int)j);
        uint32_t kbase = (uint32_t)__builtin_amdgcn_readlane((int)koff_v, (int)j);
        const uint32_t rf = (uint32_t)__builtin_amdgcn_readlane((int)rf_v, (int)j);
#pragma unroll
        for (int sl = 0; sl < SW_SLOTS; sl++) {
            if ((uint32_t)sl >= nslots) break;
            if (!SUPER) {
                const bool full = r - fb[sl] <= fl[sl];
                const uint64_t mf = __ballot(full);
                if (mf) {
                    if (full) vert[fbase + mbcnt(mf)] = pv[sl];
                    fbase += __builtin_popcountll(mf);
                }
            }
            const bool curv = r - cb[sl] <= cl[sl];
            const uint64_t mc = __ballot(curv);
            if (SUPER && mc) {
                if (curv) { const uint32_t o = cbase + mbcnt(mc); curve_ref[o] = ek[sl]; curve_row[o] = r; }
                cbase += __builtin_popcountll(mc);
            }
            if (!SUPER && mc) {
                uint64_t mk = mc;
                if (rf) {   // (uniform) curve_kept: r == c -> RF_CHILD, r == p -> RF_PARENT, else RF_ZERO
                    const uint32_t d = r - cb[sl];
                    const uint32_t skip = d == 0 ? (rf & RF_CHILD) : (d == cl[sl] ? (rf & RF_PARENT) : (rf & RF_ZERO));
                    mk = __ballot(curv && !skip);
                }
                if ((mk >> lid) & 1ull) { const uint32_t o = kbase + mbcnt(mk); kept_ref[o] = ek[sl]; kept_row[o] = r; }
                kbase += __builtin_popcountll(mk);
            }
        }
    }
}

// ---- Cubic (:614-695), exact f32 operation order ---------------------------------
struct Pt { float x, y; };
struct Cubic { Pt p0, p1, p2, p3; };

__device__ __forceinline__ float y_at(const Cubic &c, float t) {   // :623-629
    const float s = 1.0f - t;
    return s * s * s * c.p0.y + 3.0f * s * s * t * c.p1.y + 3.0f * s * t * t * c.p2.y + t * t * t * c.p3.y;
}
__device__ __forceinline__ float t_at_y(const Cubic &c, float target) {   // :635-654
    if (target <= c.p0.y) return 0.0f;
    if (target >= c.p3.y) return 1.0f;
    float lo = 0.0f, hi = 1.0f;
    for (int i = 0; i < 40; i++) {
        const float mid = (lo + hi) * 0.5f;
        // Once the midpoint rounds to an end point every later step either
        // keeps (lo, hi) or collapses it onto mid, and the result
        // (lo + hi) * 0.5 is mid either way (doubling and halving are exact):
        // stopping here is bit-identical to the 40 steps (~24 for t near 0.5).
        if (mid == lo || mid == hi) return mid;
        const float y = y_at(c, mid);
        if (y < target) lo = mid; else hi = mid;
    }
    return (lo + hi) * 0.5f;
}
__device__ __forceinline__ Pt lerp(Pt a, Pt b, float t) { return Pt{a.x + (b.x - a.x) * t, a.y + (b.y - a.y) * t}; }
__device__ __forceinline__ void split(const Cubic &c, float t, Cubic *left, Cubic *right) {   // :656-678
    const Pt q01 = lerp(c.p0, c.p1, t), q12 = lerp(c.p1, c.p2, t), q23 = lerp(c.p2, c.p3, t);
    const Pt r012 = lerp(q01, q12, t), r123 = lerp(q12, q23, t);
    const Pt s = lerp(r012, r123, t);
    if (left) *left = Cubic{c.p0, q01, r012, s};
    if (right) *right = Cubic{s, r123, q23, c.p3};
}
__device__ __forceinline__ float clamp_rs(float x, float lo, float hi) {
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
__device__ __forceinline__ Cubic subcurve(const Cubic &c, float a, float b) {   // :683-694
    if (a <= 0.0f && b >= 1.0f) return c;
    Cubic right, left;
    split(c, clamp_rs(a, 0.0f, 1.0f), nullptr, &right);
    if (b >= 1.0f) return right;
    const float new_t = clamp_rs((b - a) / (1.0f - a), 0.0f, 1.0f);
    split(right, new_t, &left, nullptr);
    return left;
}

// pmin > 0: records of edges whose parent row is below pmin are left as they
// are (a frame whose bands and row_top are unchanged above row pmin)
// refilt (the frame pass): nonzero = the curve lists were refiltered by this
// pass, so every record moved and pmin does not apply
// A segment's cubic (:552-562): child_y / parent_y from row_top + node_y, or
// per edge (edge_y: row-sharded geometry, endpoints may lie in other shards)
__device__ __forceinline__ Cubic edge_cubic(const wg_edge &e, uint32_t ref, const float *__restrict__ row_top,
                                            const float *__restrict__ node_y, const float2 *__restrict__ edge_y,
                                            float *child_y, float *parent_y) {
    if (edge_y) {
        const float2 ey = edge_y[ref];
        *child_y = ey.x;
        *parent_y = ey.y;
    } else {
        *child_y = row_top[e.child_row] + node_y[e.child_row];     // :554
        *parent_y = row_top[e.parent_row] + node_y[e.parent_row];  // :555
    }
    const float dy = *parent_y - *child_y;
    Cubic cv;
    cv.p0 = Pt{(float)e.child_lane, *child_y};
    cv.p1 = Pt{(float)e.child_lane, *child_y + dy * 0.4f};
    cv.p2 = Pt{(float)e.parent_lane, *parent_y - dy * 0.4f};
    cv.p3 = Pt{(float)e.parent_lane, *parent_y};
    return cv;
}

// Curve clipping in two launches.  The strip bottom of an edge's segment in
// row r (row_top[r + 1], r below the parent row) is the strip top of the same
// edge's segment in row r + 1, so its t_at_y is the same value: k_curves_tb
// bisects every segment's bottom once (t_b), k_curves takes each segment's
// top from the same edge's record in the row above (a short search of that
// row's edge-ordered list; a record filtered out there — an empty strip — is
// bisected here instead): one bisection per segment instead of two.
// pmin > 0: records of edges whose parent row is below pmin are left as they
// are (a frame whose bands and row_top are unchanged above row pmin)
// refilt (the frame pass): nonzero = the curve lists were refiltered by this
// pass (every record moved: all are recomputed)
// records [*lo (0 when null), *hi): the counts live on the device; grid-stride
// (a row slice's grid is sized by a guess)
__global__ void k_curves_tb(const uint32_t *__restrict__ lo, const uint32_t *__restrict__ hi,
                            const uint32_t *__restrict__ curve_ref,
                            const uint32_t *__restrict__ curve_row, const wg_edge *__restrict__ edges,
                            const float *__restrict__ row_top, const float *__restrict__ node_y,
                            const float2 *__restrict__ edge_y, float *__restrict__ tb, uint32_t pmin, Cap sc,
                            uint32_t *ovf, const uint32_t *__restrict__ refilt) {
    if (over(sc, ovf)) return;
    if (refilt && *refilt) pmin = 0;
    const uint32_t k1 = *hi;
    for (uint64_t k = (lo ? *lo : 0u) + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < k1;
         k += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t ref = curve_ref[k];
        const wg_edge e = edges[ref];
        if (e.parent_row < pmin) continue;
        const uint32_t row = curve_row[k];
        if (row == e.parent_row) continue;       // t_b = 1 (:589-593)
        float child_y, parent_y;
        const Cubic cv = edge_cubic(e, ref, row_top, node_y, edge_y, &child_y, &parent_y);
        tb[k] = t_at_y(cv, row_top[row + 1]);    // strip_bot = row bottom (:574-578)
    }
}

// row_lo: the first row of the slice; the row above it belongs to another
// slice (its t_b may not be computed yet): bisected here
__global__ void k_curves(const uint32_t *__restrict__ lo, const uint32_t *__restrict__ hi, uint32_t row_lo,
                         const uint32_t *__restrict__ curve_ref,
                         const uint32_t *__restrict__ curve_row, const uint32_t *__restrict__ curve_off,
                         const wg_edge *__restrict__ edges, const float *__restrict__ row_top,
                         const float *__restrict__ node_y, const float2 *__restrict__ edge_y,
                         const float *__restrict__ tb, wg_curve *__restrict__ out, uint8_t *__restrict__ out_color,
                         uint32_t pmin, Cap sc, uint32_t *ovf, const uint32_t *__restrict__ refilt) {
    if (over(sc, ovf)) return;
    if (refilt && *refilt) pmin = 0;
    const uint32_t k1 = *hi;
    for (uint64_t k = (lo ? *lo : 0u) + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < k1;
         k += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t ref = curve_ref[k];
    const wg_edge e = edges[ref];
    if (e.parent_row < pmin) continue;
    const uint32_t row = curve_row[k];
    float child_y, parent_y;
    const Cubic cv = edge_cubic(e, ref, row_top, node_y, edge_y, &child_y, &parent_y);
    const float rtop = row_top[row];
    const float strip_top = (row == e.child_row) ? child_y : rtop;
    float t_a = 0.0f;
    if (row != e.child_row && row == row_lo) {
        t_a = t_at_y(cv, strip_top);   // (the same value the row above's record holds as its t_b)
    } else if (row != e.child_row) {
        // the same edge's record in row - 1 holds t_at_y(row_top[row]) as its t_b
        // (lower bound by bisection: the list is in edge order; a wide row
        // holds hundreds of records)
        uint32_t j = curve_off[row - 1], a1 = curve_off[row], hi = a1;
        while (j < hi) {
            const uint32_t mid = j + (hi - j) / 2;
            if (curve_ref[mid] < ref) j = mid + 1; else hi = mid;
        }
        t_a = (j < a1 && curve_ref[j] == ref) ? tb[j] : t_at_y(cv, strip_top);
    }
    const float t_b = (row == e.parent_row) ? 1.0f : tb[k];
    const Cubic s = subcurve(cv, t_a, t_b);
    float4 *o = reinterpret_cast<float4 *>(out + k);
    o[0] = make_float4(s.p0.x, s.p0.y - rtop, s.p1.x, s.p1.y - rtop);
    o[1] = make_float4(s.p2.x, s.p2.y - rtop, s.p3.x, s.p3.y - rtop);
    out_color[k] = (uint8_t)e.color;
    }
}

inline uint32_t blocks(uint64_t n) { return (uint32_t)((n + T - 1) / T); }

// Curve lists are swept once per layout as a superset (every cross-lane
// segment c <= r <= p, strip flags ignored) and filtered per geometry pass by
// the row's own flags (:577): r == c needs a child strip, r == p a parent
// strip, c < r < p a non-zero-height row.  The full pass's sweep writes its
// own filtered lists beside the superset (counts from k_geom_offsets); the
// frame pass refilters the superset here.
__device__ __forceinline__ bool curve_kept(uint32_t r, const wg_edge &e, uint32_t f) {
    const uint32_t skip = (r == e.child_row) ? (f & RF_CHILD) : (r == e.parent_row) ? (f & RF_PARENT) : (f & RF_ZERO);
    return skip == 0;
}

// cond (the frame pass): only when *cond (the row flags changed); otherwise
// the current offsets' per-row counts, so the scan that follows reproduces them
// (+ the block's sum of the counts for the offsets' scan, wg_scan_bs_u32)
__global__ void __launch_bounds__(WG_BS_THREADS) k_curve_keep(uint64_t n, const uint32_t *__restrict__ soff,
                                                             const uint32_t *__restrict__ sref,
                                                             const wg_edge *__restrict__ edges,
                                                             const uint8_t *__restrict__ rowflags, uint32_t *__restrict__ cnt,
                                                             const uint32_t *__restrict__ cond,
                                                             const uint32_t *__restrict__ cur_off, Cap sc, uint32_t *ovf,
                                                             uint8_t *__restrict__ flags_kept, uint32_t *__restrict__ bsum,
                                                             uint32_t *__restrict__ super_done) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // (the superset this refilter reads stands for the layout's later frames)
    if (super_done && cond && *cond && r == 0) *super_done = 1u;
    uint32_t k = 0;
    if (!over(sc, ovf) && r < n) {
        const uint32_t f = rowflags[r];
        flags_kept[r] = (uint8_t)f;   // the flags the curve lists are filtered with (equal when cond is 0)
        if (cond && !*cond) {
            k = cur_off[r + 1] - cur_off[r];
        } else {
            const uint32_t a = soff[r], b = soff[r + 1];
            k = b - a;
            if (f) {
                k = 0;
                for (uint32_t j = a; j < b; j++) k += curve_kept((uint32_t)r, edges[sref[j]], f) ? 1u : 0u;
            }
        }
        cnt[r] = k;
    }
    wg_bsum_store(k, bsum);
}

__global__ void k_curve_compact(uint64_t n, const uint32_t *__restrict__ soff, const uint32_t *__restrict__ sref,
                                const wg_edge *__restrict__ edges, const uint8_t *__restrict__ rowflags,
                                const uint32_t *__restrict__ coff, uint32_t *__restrict__ ref, uint32_t *__restrict__ row,
                                const uint32_t *__restrict__ cond, Cap sc, uint32_t *ovf) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (over(sc, ovf) || r >= n) return;
    if (cond && !*cond) return;   // the lists stand
    const uint32_t a = soff[r], b = soff[r + 1], f = rowflags[r];
    uint32_t o = coff[r];
    for (uint32_t j = a; j < b; j++) {
        const uint32_t k = sref[j];
        if (f && !curve_kept((uint32_t)r, edges[k], f)) continue;
        ref[o] = k;
        row[o] = (uint32_t)r;
        o++;
    }
}

}  // namespace

// filter the curve superset by a frame pass's row flags -> curve_off / curve_ref / curve_row.
// cond (on the device): refilter only if the flags changed —
// otherwise the same offsets are rescanned and the lists stand, no host read.
static Cap no_cap() { return Cap{nullptr, ~0u, nullptr}; }
static int filter_curves(wg_ctx *c, uint64_t n, hipStream_t s, const uint32_t *cond, Cap sc, uint32_t *ovf) {
    uint32_t *coff = c->curve_off.as<uint32_t>();
    WG_ALLOC(c, c->curve_cnt, (n + 2) * 4);
    WG_ALLOC(c, c->rowflags_lists, n + 4);
    uint32_t *cnt = c->curve_cnt.as<uint32_t>();
    // (the geometry pass's other tile sums are consumed by now: the same words)
    WG_ALLOC(c, c->bsum, (wg_bs_blocks(n) + 64) * 4);
    static_assert(T == WG_BS_THREADS, "k_curve_keep is a wg_scan_bs_u32 producer");
    hipLaunchKernelGGL(k_curve_keep, dim3(blocks(n)), dim3(T), 0, s, n, c->scurve_off.as<const uint32_t>(),
                       c->scurve_ref.as<const uint32_t>(), c->edges.as<const wg_edge>(), c->rowflags.as<const uint8_t>(),
                       cnt, cond, (const uint32_t *)coff, sc, ovf, c->rowflags_lists.as<uint8_t>(), c->bsum.as<uint32_t>(),
                       c->geom_err ? c->geom_err + 5 : nullptr);
    {
        WgScanBs S;
        S.na = 1;
        S.in[0] = cnt;
        S.out[0] = coff;
        S.bsum[0] = c->bsum.as<const uint32_t>();
        WG_HIP(c, wg_scan_bs_u32(S, n, c->scan_tmp.p, s));
    }
    hipLaunchKernelGGL(k_curve_compact, dim3(blocks(n)), dim3(T), 0, s, n, c->scurve_off.as<const uint32_t>(),
                       c->scurve_ref.as<const uint32_t>(), c->edges.as<const wg_edge>(), c->rowflags.as<const uint8_t>(),
                       (const uint32_t *)coff, c->curve_ref.as<uint32_t>(), c->curve_row.as<uint32_t>(), cond, sc, ovf);
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

// curve records of rows [r0, r1) (their range read on the device); grid: an
// upper bound of the records, or a guess (the kernels stride)
static void launch_curves(wg_ctx *c, uint64_t r0, uint64_t r1, uint64_t grid_recs, hipStream_t s, uint32_t pmin, Cap sc,
                          uint32_t *ovf, const uint32_t *refilt) {
    if (!grid_recs || r1 <= r0) return;
    const uint32_t *lo = r0 ? c->curve_off.as<const uint32_t>() + r0 : nullptr;
    hipLaunchKernelGGL(k_curves_tb, dim3(blocks(grid_recs)), dim3(T), 0, s, lo, c->curve_off.as<const uint32_t>() + r1,
                       c->curve_ref.as<const uint32_t>(), c->curve_row.as<const uint32_t>(), c->edges.as<const wg_edge>(),
                       c->g_row_top.as<const float>(), c->g_node_y.as<const float>(),
                       reinterpret_cast<const float2 *>(c->edge_y), c->curve_tb.as<float>(), pmin, sc, ovf, refilt);
    hipLaunchKernelGGL(k_curves, dim3(blocks(grid_recs)), dim3(T), 0, s, lo, c->curve_off.as<const uint32_t>() + r1,
                       (uint32_t)r0, c->curve_ref.as<const uint32_t>(), c->curve_row.as<const uint32_t>(), c->curve_off.as<const uint32_t>(),
                       c->edges.as<const wg_edge>(), c->g_row_top.as<const float>(), c->g_node_y.as<const float>(),
                       reinterpret_cast<const float2 *>(c->edge_y), c->curve_tb.as<const float>(), c->curve.as<wg_curve>(),
                       c->curve_color.as<uint8_t>(), pmin, sc, ovf, refilt);
}

// the lazily read summary of the last pass (total height, scan path, curve count)
int wg_geom_summary_sync(wg_ctx *c) {
    if (!c->geom_sum_stale) return WG_OK;
    uint64_t v[3] = {0, 0, 0};
    const int rc = wg_fetch(c, {{c->geom_sum_at[0], false}, {c->geom_sum_at[1], false}, {c->geom_sum_at[2], false}}, v);
    if (rc != WG_OK) return rc;
    const uint32_t tbits = (uint32_t)v[0];
    std::memcpy(&c->total_height, &tbits, 4);
    c->scan_path = v[1] ? 1u : 0u;
    c->n_curve = v[2];
    c->geom_sum_stale = false;
    return WG_OK;
}

// speculative full pass: its validation words (WG_GEOM_SPEC_ITEMS) and their check
int wg_geom_spec_items(wg_ctx *c, WgFetch *it) {
    const uint64_t n = c->n;
    const uint32_t *err = c->geom_err;
    it[0] = WgFetch{err + 8, false};                                   // capacity overflow
    it[1] = WgFetch{err, false};                                       // > SW_CAP edges alive across a row
    it[2] = WgFetch{c->vert_off.as<uint32_t>() + n, false};
    it[3] = WgFetch{c->scurve_off.as<uint32_t>() + n, false};
    it[4] = WgFetch{c->carry_off.as<uint32_t>() + (n + WG_SWEEP_CH - 1) / WG_SWEEP_CH, false};
    it[5] = WgFetch{c->g_row_top.as<uint32_t>() + n, false};
    it[6] = WgFetch{c->rt_flags.as<uint32_t>() + 2, false};
    it[7] = WgFetch{c->curve_off.as<uint32_t>() + n, false};
    return WG_GEOM_SPEC_ITEMS;
}

// true = the speculative pass fit its capacities (the lists are exact)
bool wg_geom_spec_check(wg_ctx *c, const uint64_t *v) {
    if (v[0] || v[1]) return false;   // overflow: the exact pass sizes and redoes; too many edges: it fails
    c->n_vert = v[2];
    c->lists_nsuper = v[3];
    const uint32_t tbits = (uint32_t)v[5];
    std::memcpy(&c->total_height, &tbits, 4);
    c->scan_path = v[6] ? 1u : 0u;
    c->n_curve = v[7];
    c->geom_sum_stale = false;
    c->lists_gen = c->layout_gen;
    c->lists_n = c->n;
    c->lists_ne = c->n_edges;
    return true;
}

int wg_geom_lists(wg_ctx *c, uint64_t r0, uint64_t r1, int slice, hipStream_t s) {
    const wg_ctx::ListsDef &L = c->glist;
    const uint64_t n = L.n;
    if (r1 > n || r0 >= r1 || (r0 % WG_SWEEP_CH) || (r1 != n && (r1 % WG_SWEEP_CH)))
        return wg_fail(c, WG_E_INVALID, "list slice [%llu,%llu) of %llu rows", (unsigned long long)r0, (unsigned long long)r1,
                       (unsigned long long)n);
    const wg_edge *E = c->edges.as<const wg_edge>();
    const uint32_t *edge_off = c->edge_cnt.as<const uint32_t>();
    const uint32_t *voff = c->vert_off.as<const uint32_t>(), *soff = c->scurve_off.as<const uint32_t>();
    const uint32_t *koff = c->curve_off.as<const uint32_t>(), *carry_off = c->carry_off.as<const uint32_t>();
    const Cap vc{L.vtot, L.vcap, nullptr}, sc{L.stot, L.scap, nullptr}, cc{L.ctot, L.ccap, nullptr};
    uint32_t *err = L.err, *ovf = err + 8;
    uint32_t *vert = c->vert.as<uint32_t>();
    // chunks too wide for the register sweep: listed per slice (counts in
    // err[1] / err[4]) and swept through LDS
    const uint64_t q0 = r0 / WG_SWEEP_CH, q1 = (r1 + WG_SWEEP_CH - 1) / WG_SWEEP_CH;
    uint32_t *big = c->sweep_big.as<uint32_t>() + q0, *big_n = err + (slice ? 4 : 1);
    uint32_t *carry_sorted = c->carry_sorted.as<uint32_t>();
    hipLaunchKernelGGL(k_sweep<false>, dim3((uint32_t)((q1 - q0 + SW_WAVES - 1) / SW_WAVES)), dim3(64 * SW_WAVES), 0, s, n,
                       q0, q1, E, edge_off, carry_off, (const uint32_t *)c->carry.as<uint32_t>(), carry_sorted,
                       c->rowflags.as<const uint8_t>(), voff, soff, vert, c->scurve_ref.as<uint32_t>(),
                       c->scurve_row.as<uint32_t>(), koff, c->curve_ref.as<uint32_t>(), c->curve_row.as<uint32_t>(), big,
                       big_n, c->sweep_reg_cap < 64u * SW_SLOTS ? c->sweep_reg_cap : 64u * SW_SLOTS, vc, sc, cc, ovf,
                       (const uint32_t *)nullptr, (const uint32_t *)nullptr, L.cntF, L.cntT, L.lds_off ? 1u : 0u);
    // (one wave per wide chunk, ~73 KB of LDS per block: two blocks per CU,
    // the whole chip for lists whose every chunk is wide; sized by the last
    // pass's count of wide chunks; 64 blocks for a list that had none, as
    // many as before r04: a block lists at most 64 chunks past one wave's
    // pool for its whole-block pass)
    const uint64_t lds_want = 64 + (uint64_t)c->sweep_wide_last / SW_WAVES;
    const uint64_t lds_grid = std::min<uint64_t>(std::min<uint64_t>(SW_LDS_BLOCKS, lds_want),
                                                 (q1 - q0 + SW_WAVES - 1) / SW_WAVES);
    if (!L.lds_off) hipLaunchKernelGGL(k_sweep_lds, dim3((uint32_t)lds_grid), dim3(64 * SW_WAVES), 0, s, n, (const uint32_t *)big,
                       (const uint32_t *)big_n, E, edge_off, carry_off, (const uint32_t *)carry_sorted,
                       c->rowflags.as<const uint8_t>(), voff, soff, vert, c->scurve_ref.as<uint32_t>(),
                       c->scurve_row.as<uint32_t>(), koff, c->curve_ref.as<uint32_t>(), c->curve_row.as<uint32_t>(), err,
                       vc, sc, ovf, false, (const uint32_t *)nullptr, (const uint32_t *)nullptr);
    // the records of the slice's rows: a grid for its share of the records
    // (+ a quarter), the kernels stride over the rest
    uint64_t grid_recs = L.n_super_grid;
    if (r1 - r0 < n) grid_recs = std::min<uint64_t>(L.n_super_grid, L.n_super_grid * (r1 - r0) / n * 5 / 4 + 64 * T);
    launch_curves(c, r0, r1, grid_recs, s, 0u, sc, ovf, nullptr);
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

// The flag-free curve superset of the last full pass's layout, for a frame
// pass whose row flags differ from the full pass's (run_if: its flag-change
// word, on the device): swept once per layout (done: the full pass's error
// word 5, raised by the first refilter); a frame pass whose flags equal the
// full pass's keeps the full pass's lists and skips both kernels.
static void launch_superset(wg_ctx *c, uint64_t n, hipStream_t s, const uint32_t *run_if, Cap g, uint32_t *ovf) {
    if (!n || !c->geom_err) return;
    const uint64_t nch = (n + WG_SWEEP_CH - 1) / WG_SWEEP_CH;
    uint32_t *err = c->geom_err;
    const wg_edge *E = c->edges.as<const wg_edge>();
    const uint32_t *edge_off = c->edge_cnt.as<const uint32_t>(), *carry_off = c->carry_off.as<const uint32_t>();
    const uint32_t *soff = c->scurve_off.as<const uint32_t>();
    uint32_t *big = c->sweep_big.as<uint32_t>(), *big_n = err + 6;
    hipLaunchKernelGGL(k_sweep<true>, dim3((uint32_t)((nch + SW_WAVES - 1) / SW_WAVES)), dim3(64 * SW_WAVES), 0, s, n,
                       (uint64_t)0, nch, E, edge_off, carry_off, (const uint32_t *)c->carry.as<uint32_t>(),
                       c->carry_sorted.as<uint32_t>(), (const uint8_t *)nullptr, (const uint32_t *)nullptr, soff,
                       (uint32_t *)nullptr, c->scurve_ref.as<uint32_t>(), c->scurve_row.as<uint32_t>(),
                       (const uint32_t *)nullptr, (uint32_t *)nullptr, (uint32_t *)nullptr, big, big_n,
                       c->sweep_reg_cap < 64u * SW_SLOTS ? c->sweep_reg_cap : 64u * SW_SLOTS, g, g, g, ovf, run_if,
                       (const uint32_t *)(err + 5), (const uint32_t *)nullptr, (const uint32_t *)nullptr, 0u);
    const uint64_t lds_grid = std::min<uint64_t>(std::min<uint64_t>(SW_LDS_BLOCKS, 64 + (uint64_t)c->sweep_wide_last / SW_WAVES),
                                                 (nch + SW_WAVES - 1) / SW_WAVES);
    hipLaunchKernelGGL(k_sweep_lds, dim3((uint32_t)lds_grid), dim3(64 * SW_WAVES), 0, s, n, (const uint32_t *)big,
                       (const uint32_t *)big_n, E, edge_off, carry_off, (const uint32_t *)c->carry_sorted.as<uint32_t>(),
                       c->rowflags.as<const uint8_t>(), (const uint32_t *)nullptr, soff, (uint32_t *)nullptr,
                       c->scurve_ref.as<uint32_t>(), c->scurve_row.as<uint32_t>(), (const uint32_t *)nullptr,
                       (uint32_t *)nullptr, (uint32_t *)nullptr, err, g, g, ovf, true, run_if, (const uint32_t *)(err + 5));
}

int wg_geom_lists_flush(wg_ctx *c) {
    if (!c->glist.deferred) return WG_OK;
    c->glist.deferred = false;
    return wg_geom_lists(c, 0, c->glist.n, 0, c->stream);
}

// The full pass's zero-initialised workspace (per-row counts and difference
// arrays, top fill, carry counts and fill, sweep flags, the all-zero flag row)
// for n rows, in 32-bit words
static uint64_t geom_zero_words(uint64_t n) {
    const uint64_t nch = (n + WG_SWEEP_CH - 1) / WG_SWEEP_CH;
    const uint64_t rowa = (n + 2 + 63) & ~63ull, cha = (nch + 2 + 63) & ~63ull;
    return (7 * rowa + 2 * cha + 64 + rowa / 4 + 3) & ~3ull;   // cleared in 16-byte units
}

// r06: the workspace of the next full pass over n rows, zeroed on the current
// stream (the build's side stream, beside the hash join and the lanes; the
// geometry stage joins it first), so the pass counts both edge ends in one
// kernel (k_edges_rows<true>)
int wg_geom_prezero(wg_ctx *c, uint64_t n) {
    c->geom_zero_n = ~0ull;
    if (!n) return WG_OK;
    const uint64_t zw = geom_zero_words(n);
    WG_ALLOC(c, c->geom_zero, zw * 4);
    WG_HIP(c, hipMemsetAsync(c->geom_zero.p, 0, zw * 4, c->stream));
    c->geom_zero_n = n;
    return WG_OK;
}

int wg_stage_geometry(wg_ctx *c, const float *d_band) {
    if (const int rc = wg_geom_lists_flush(c)) return rc;   // (a deferred pass's lists, before anything reuses them)
    if (const int rc = wg_side_join(c)) return rc;
    const uint64_t n = c->n, ne = c->n_edges;
    hipStream_t s = c->stream;
    WG_ALLOC(c, c->g_height, n * 4 + 4);
    WG_ALLOC(c, c->g_node_y, n * 4 + 4);
    WG_ALLOC(c, c->rowflags, n + 4);
    WG_ALLOC(c, c->vert_off, (n + 2) * 4);
    WG_ALLOC(c, c->curve_off, (n + 2) * 4);
    WG_ALLOC(c, c->scurve_off, (n + 2) * 4);
    { const int _sr = wg_scan_reserve(c, n + 2); if (_sr != WG_OK) return _sr; }
    const float *h = c->geom_heights();
    const float *rt = c->g_row_top.as<const float>();
    if (n && c->lists_gen == c->layout_gen && c->lists_n == n && c->lists_ne == ne) {
        // same layout: the lists stand; only the curve filter can change with the flags
        // a frame whose bands equal the last frame's below row r0 (wg_row_geometry):
        // rows below r0 keep height / node_y / flags, and curve records of edges
        // that end above r0 keep their geometry (row_top up to r0 is unchanged).
        // No host read: whether the flags changed decides on the device (the
        // refilter and the curve range); the summary is read when asked for.
        const uint64_t r0 = c->geom_r0 < n ? c->geom_r0 : 0;
        c->geom_r0 = 0;
        // two sets of flag words used in turn: this pass's row kernel raises the
        // change flag in one and clears the other for the next pass
        if (c->geom_diff.cap < 128) {
            WG_ALLOC(c, c->geom_diff, 128);
            WG_HIP(c, hipMemsetAsync(c->geom_diff.p, 0, 128, s));
        }
        const int par = c->geom_diff_par;
        c->geom_diff_par ^= 1;
        wg_stage_begin(c, "geom_reuse");
        uint32_t *diff = c->geom_diff.as<uint32_t>() + 16 * par;
        hipLaunchKernelGGL(k_row_basic, dim3(blocks(n - r0)), dim3(T), 0, s, n, h, d_band, rt, c->g_height.as<float>(),
                           c->g_node_y.as<float>(), c->rowflags.as<uint8_t>(), r0,
                           reinterpret_cast<uint4 *>(c->geom_diff.as<uint32_t>() + 16 * (par ^ 1)), (uint64_t)4,
                           c->band_keep, c->rowflags_lists.as<const uint8_t>(), diff);
        // (a build awaiting its validation whose lists did not fit: no reads of them)
        const Cap bg = Cap{nullptr, ~0u, c->pend.build ? c->geom_err : nullptr};
        launch_superset(c, n, s, diff, bg, diff + 8);
        int rc = filter_curves(c, n, s, diff, bg, diff + 8);
        if (rc != WG_OK) return rc;
        wg_stage_end(c);
        wg_stage_begin(c, "geom_curves");
        // re-filtered lists move every record: all of them are recomputed then
        launch_curves(c, 0, n, c->lists_nsuper, s, (uint32_t)r0, bg, diff + 8, diff);
        WG_HIP(c, hipGetLastError());
        wg_stage_end(c);
        c->geom_sum_at[0] = rt + n;
        c->geom_sum_at[1] = c->rt_flags.as<uint32_t>() + 2;
        c->geom_sum_at[2] = c->curve_off.as<uint32_t>() + n;
        c->geom_sum_stale = true;
        return WG_OK;
    }
    const bool spec = c->spec;
    c->lists_gen = ~0ull;
    c->n_vert = c->n_curve = 0;
    c->geom_sum_stale = false;
    if (n == 0) {
        WG_HIP(c, hipMemsetAsync(c->vert_off.p, 0, 4, s));
        WG_HIP(c, hipMemsetAsync(c->curve_off.p, 0, 4, s));
        c->lists_nsuper = 0;
        return WG_OK;
    }
    const wg_edge *E = c->edges.as<const wg_edge>();
    const uint32_t *edge_off = c->edge_cnt.as<const uint32_t>();
    // speculative build: the edge count is on the device (ne is its upper bound)
    const uint32_t *ne_dev = spec ? edge_off + n : nullptr;
    // every array that starts at zero lives in one workspace, cleared by the
    // pass's first kernel.  The last region is an all-zero flag row: the lists
    // are swept as a superset.
    const uint64_t nch = (n + WG_SWEEP_CH - 1) / WG_SWEEP_CH;
    const uint64_t rowa = (n + 2 + 63) & ~63ull, cha = (nch + 2 + 63) & ~63ull;
    const uint64_t zwords = geom_zero_words(n);
    // zeroed beforehand for this pass (wg_geom_prezero): the fused count kernel
    const bool prezero = c->geom_zero_n == n && c->geom_zero.cap >= zwords * 4;
    c->geom_zero_n = ~0ull;
    WG_ALLOC(c, c->geom_zero, zwords * 4);
    WG_ALLOC(c, c->rowflags_lists, n + 4);
    uint32_t *cntF = c->geom_zero.as<uint32_t>(), *cntT = cntF + rowa, *cntB = cntT + rowa;
    uint32_t *cntC = cntB + rowa, *cntCend = cntC + rowa, *cntPend = cntCend + rowa, *top_fill = cntPend + rowa;
    uint32_t *carry_cnt = top_fill + rowa, *carry_fill = carry_cnt + cha, *sweep_err = carry_fill + cha;
    uint32_t *ovf = sweep_err + 8;   // capacity overflow of a speculative pass
    c->geom_err = sweep_err;
    const uint8_t *zflags = reinterpret_cast<const uint8_t *>(sweep_err + 64);
    uint32_t *voff = c->vert_off.as<uint32_t>(), *soff = c->scurve_off.as<uint32_t>();
    uint32_t *koff = c->curve_off.as<uint32_t>();

    wg_stage_begin(c, "geom_counts");
    {
        EdgeRowsArgs A{};
        A.edge_off = edge_off;
        if (c->edges_pending) {   // the layout stage left the edge list to this kernel
            A.poff = c->d_poff;
            A.prow = c->prow.as<const int32_t>();
            A.lane_out = c->lane_out.as<const uint32_t>();
            A.color_out = c->color_out.as<const uint8_t>();
        }
        A.edges = c->edges.as<wg_edge>();
        A.h = h; A.band = d_band; A.row_top = rt;
        A.height = c->g_height.as<float>(); A.node_y = c->g_node_y.as<float>(); A.band_keep = c->band_keep;
        A.rowflags = c->rowflags.as<uint8_t>(); A.zflags = const_cast<uint8_t *>(zflags);
        A.flags_kept = c->rowflags_lists.as<uint8_t>();
        A.cntB = cntB; A.diffF = cntF; A.diffC = cntC; A.cntCend = cntCend; A.cntPend = cntPend; A.carry_diff = carry_cnt;
        A.cntT = cntT; A.top_fill = top_fill; A.carry_fill = carry_fill; A.misc = sweep_err;
        if (prezero) hipLaunchKernelGGL(k_edges_rows<true>, dim3(blocks(n)), dim3(256), 0, s, n, A);
        else hipLaunchKernelGGL(k_edges_rows<false>, dim3(blocks(n)), dim3(256), 0, s, n, A);
        c->edges_pending = false;
    }
    if (ne && !prezero)
        hipLaunchKernelGGL(k_edge_counts, dim3(blocks(ne)), dim3(T), 0, s, ne, E, zflags, cntT, cntF, cntC, cntCend,
                           cntPend, carry_cnt, ne_dev);
    // carry-in offsets: the exclusive scan of the chunk difference counts, then
    // of the per-chunk counts it holds one entry later
    WG_ALLOC(c, c->carry_off, (nch + 2) * 4);
    uint32_t *carry_off = c->carry_off.as<uint32_t>();

    // offsets: tile sums of the three difference arrays; one kernel for their
    // scans, the per-row list totals and the per-chunk carry counts (+ their
    // 256-entry sums); one launch for the three offset arrays
    const uint64_t nbs = wg_bs_blocks(n), nbsD = wg_bs_blocks(nch), nt2 = (n + 1 + GO_TILE - 1) / GO_TILE;
    WG_ALLOC(c, c->bsum, (3 * nbs + nbsD + 3 * nt2 + 512) * 4);
    uint32_t *bsV = c->bsum.as<uint32_t>(), *bsC = bsV + nbs, *bsK = bsC + nbs, *bsD = bsK + nbs;
    uint32_t *tsF = bsD + nbsD + 64, *tsC = tsF + nt2 + 64, *tsD = tsC + nt2 + 64;
    hipLaunchKernelGGL(k_tile_sums3, dim3((uint32_t)nt2, 3), dim3(GO_T), 0, s, (const uint32_t *)cntF, (const uint32_t *)cntC,
                       (const uint32_t *)carry_cnt, n + 1, nch + 1, tsF, tsC, tsD);
    hipLaunchKernelGGL(k_geom_offsets, dim3((uint32_t)nt2), dim3(GO_T), 0, s, n, cntF, cntC, (const uint32_t *)tsF,
                       (const uint32_t *)tsC, (const uint32_t *)cntT, (const uint32_t *)cntB, (const uint32_t *)cntCend,
                       voff, soff, bsV, bsC, nbs, carry_cnt, (const uint32_t *)tsD, nch, bsD, nbsD,
                       (const uint32_t *)cntPend, c->rowflags.as<const uint8_t>(), koff, bsK);
    {
        WgScanBs S;
        S.na = 4;
        S.in[0] = voff; S.out[0] = voff; S.bsum[0] = bsV;
        S.in[1] = soff; S.out[1] = soff; S.bsum[1] = bsC;
        S.in[2] = carry_cnt; S.out[2] = carry_off; S.bsum[2] = bsD; S.len[2] = nch;
        S.in[3] = koff; S.out[3] = koff; S.bsum[3] = bsK;
        WG_HIP(c, wg_scan_bs_u32(S, n, c->scan_tmp.p, s));
    }
    // list capacities: exact from the totals, or (speculative build) the
    // buffers as the last pass left them, checked on the device
    Cap vc = no_cap(), sc = no_cap(), cc = no_cap();
    uint64_t n_super_grid = 0;
    if (!spec) {
        uint64_t tot[3] = {0, 0, 0};
        const int rc = wg_fetch(c, {{voff + n, false}, {soff + n, false}, {carry_off + nch, false}}, tot);
        if (rc != WG_OK) return rc;
        c->n_vert = tot[0];
        const uint64_t n_super = tot[1];
        const uint64_t ncarry = tot[2];
        WG_ALLOC(c, c->vert, c->n_vert * 4 + 16);
        WG_ALLOC(c, c->scurve_ref, n_super * 4 + 16);
        WG_ALLOC(c, c->scurve_row, n_super * 4 + 16);
        WG_ALLOC(c, c->curve, n_super * sizeof(wg_curve) + 64);
        WG_ALLOC(c, c->curve_color, n_super + 16);
        WG_ALLOC(c, c->curve_ref, n_super * 4 + 16);
        WG_ALLOC(c, c->curve_row, n_super * 4 + 16);
        WG_ALLOC(c, c->curve_tb, n_super * 4 + 16);
        WG_ALLOC(c, c->carry, ncarry * 4 + 16);
        WG_ALLOC(c, c->carry_sorted, ncarry * 4 + 16);
        n_super_grid = n_super;
    } else {
        auto cap_of = [](const DevBuf &b, size_t elem) -> uint64_t { return b.cap / elem; };
        const uint64_t vcap = cap_of(c->vert, 4);
        uint64_t scap = cap_of(c->scurve_ref, 4);
        scap = std::min(scap, cap_of(c->scurve_row, 4));
        scap = std::min(scap, cap_of(c->curve, sizeof(wg_curve)));
        scap = std::min(scap, cap_of(c->curve_color, 1));
        scap = std::min(scap, cap_of(c->curve_ref, 4));
        scap = std::min(scap, cap_of(c->curve_row, 4));
        scap = std::min(scap, cap_of(c->curve_tb, 4));
        const uint64_t ccap = std::min(cap_of(c->carry, 4), cap_of(c->carry_sorted, 4));
        auto u32 = [](uint64_t v) { return (uint32_t)std::min<uint64_t>(v, 0xFFFFFFFEull); };
        vc = Cap{voff + n, u32(vcap), nullptr};
        sc = Cap{soff + n, u32(scap), nullptr};
        cc = Cap{carry_off + nch, u32(ccap), nullptr};
        n_super_grid = scap;
        c->spec_nsuper_grid = scap;
    }
    wg_stage_end(c);

    wg_stage_begin(c, "geom_lists");
    if (ne)
        hipLaunchKernelGGL(k_top_carry, dim3(blocks(ne)), dim3(T), 0, s, ne, E, voff, cntF, top_fill, c->vert.as<uint32_t>(),
                           (const uint32_t *)carry_off, carry_fill, c->carry.as<uint32_t>(), ne_dev, vc, cc, ovf);
    WG_ALLOC(c, c->sweep_big, nch * 4 + 16);
    wg_ctx::ListsDef &L = c->glist;
    L = wg_ctx::ListsDef{};
    L.n = n;
    L.n_super_grid = n_super_grid;
    L.cntF = cntF;
    L.cntT = cntT;
    L.vtot = vc.total; L.vcap = vc.cap;
    L.stot = sc.total; L.scap = sc.cap;
    L.ctot = cc.total; L.ccap = cc.cap;
    L.err = sweep_err;
    // a speculative pass validated with the emission's read: the lists are
    // left to the emission (row-sliced under its first tiles).  Below ~256K
    // rows the list kernels sit at the launch floor: slicing would only add
    // five launches.
    if (spec && c->defer_validation && c->slice_on && !c->sh.on && n >= c->slice_min_rows) {
        L.deferred = true;
        WG_HIP(c, hipGetLastError());
        wg_stage_end(c);
        return WG_OK;
    }
    // r06: a speculative pass skips the LDS sweep's launch (~5 us at its
    // floor on the critical path) when the last exact pass had no wide chunk
    L.lds_off = spec && !c->sh.on && c->sweep_wide_last == 0;
    if (const int rc = wg_geom_lists(c, 0, n, 0, s)) return rc;
    wg_stage_end(c);
    if (spec) return WG_OK;   // validated at the end of the build (wg_geom_spec_items / wg_geom_spec_check)
    uint64_t fin[5] = {0, 0, 0, 0, 0};
    {
        const int rc = wg_fetch(c, {{sweep_err, false}, {rt + n, false}, {c->rt_flags.as<uint32_t>() + 2, false},
                                    {c->curve_off.as<uint32_t>() + n, false}, {sweep_err + 1, false}}, fin);
        if (rc != WG_OK) return rc;
    }
    c->sweep_wide_last = (uint32_t)fin[4];
    if (fin[0]) return wg_fail(c, WG_E_UNSUPPORTED, "more than %d edges alive across one row", SW_CAP_BLOCK);
    c->n_curve = fin[3];
    c->lists_nsuper = n_super_grid;
    c->lists_gen = c->layout_gen;
    c->lists_n = n;
    c->lists_ne = ne;
    const uint32_t tbits = (uint32_t)fin[1];
    std::memcpy(&c->total_height, &tbits, 4);
    c->scan_path = fin[2] ? 1u : 0u;
    return WG_OK;
}
