// wg_vertex.hip — graph_cell path emission tessellated to SplineVertex
// buffers (frozen spec WG-TESS-1).
//
// Reference: graph_cell (commit_graph.rs:803-908) builds, per row, the
// z-ordered paths full/top/bottom verticals -> curve segments -> node disk ->
// selected ring, with lane_center_x (:786-790) and the curve x mapping
// (:846-850).  The legacy CPU tessellator that turned such paths into
// SplineVertex triangle lists (docs/render_engine.md:148-170) is absent
// from the snapshot; WG-TESS-1 freezes it: vertical -> 6 vertices, curve
// segment -> 16 strip quads = 96 vertices, node -> 24-triangle fan = 72
// vertices, ring -> 24 quads = 144 vertices.
//
// HBM-write-bound: 24 B per vertex out, a few bytes of geometry in.  A
// workgroup owns a fixed tile of 1024 vertices (24 KiB out):
//   1. one round of independent global loads, all addressed from a per-tile
//      record (k_vtx_prep): the rows overlapping the tile, its vertical
//      entries (one contiguous range of vert[]) and its curve segments (one
//      contiguous range of curve[]); pair -> row by a prefix-max of row starts
//      (every primitive has an even vertex count, so vertex PAIRS never
//      straddle a row or a primitive);
//   2. the <= 24 curve segments overlapping the tile are tessellated once,
//      all lanes together (17 strip points each: Bezier point, tangent,
//      normal with one sqrt and two divisions), into LDS — the per-vertex
//      work that remains is cheap and barely diverges across primitive kinds;
//   3. each thread emits one pair (48 B) per round into a per-wave LDS
//      stage; the wave then writes its 64 pairs as three fully contiguous
//      1 KiB store instructions.
#include "wg_internal.h"
#include "wgraph_tess.h"

namespace {

#ifndef WG_VTX_THREADS
#define WG_VTX_THREADS 256
#endif
// Vertices per workgroup tile: 1024 (24 KiB out) by default; 2048 for lists
// whose geometry outgrows the Infinity Cache (each tile's load round then
// waits on HBM under the saturated write stream, and a larger tile amortises
// it: DESIGN.md §3 "one load round per tile"; WG_OPT_VTX_TILE).
// (tile sweep on wide16 1M: 1024 0.98 ms, 1536 1.01, 2048 1.05, 512 1.07)
constexpr int VT = WG_VTX_THREADS;
template <int TILE>
struct TileGeo {
    static constexpr int PAIRS = TILE / 2;
    static constexpr int ROUNDS = PAIRS / VT;
    static constexpr int MAXR = TILE / WG_VTX_PER_NODE + 3;         // rows overlapping a tile
    static constexpr int MAXC = TILE / WG_VTX_PER_CURVE + 3;        // curve segments overlapping a tile
    static constexpr int MAXV = TILE / WG_VTX_PER_VERTICAL + 2;     // vertical entries overlapping a tile
    static_assert(PAIRS % VT == 0, "a tile is a whole number of rounds of one pair per thread");
    static_assert(MAXR <= 64, "rows of a tile are loaded by one wave");
};
typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int NPTS = WG_TESS_CURVE_SEGMENTS + 1;          // 17 strip points per segment

__constant__ float c_cos[25] = WG_UNIT_CIRCLE_COS_INIT;
__constant__ float c_sin[25] = WG_UNIT_CIRCLE_SIN_INIT;

// Vertex offset of row j of [rb, re) in closed form: a row's vertex count is
// 6 per vertical entry, 96 per curve segment, 72 for the node and 144 more on
// the selected row, and vert_off / curve_off are prefix sums already — no
// count pass and no scan.
__device__ __forceinline__ uint64_t vtx_at(uint64_t rb, uint64_t j, int64_t sel, const uint32_t *__restrict__ voff,
                                           const uint32_t *__restrict__ coff, uint32_t v0, uint32_t c0) {
    const uint64_t r = rb + j;
    uint64_t v = (uint64_t)WG_VTX_PER_VERTICAL * (voff[r] - v0) + (uint64_t)WG_VTX_PER_CURVE * (coff[r] - c0) +
                 (uint64_t)WG_VTX_PER_NODE * j;
    if (sel >= 0 && (uint64_t)sel >= rb && (uint64_t)sel < r) v += WG_VTX_PER_RING;
    return v;
}

// vtx_off[0..rows] and the per-tile records, written by the row whose vertex
// range contains the tile start: {first row, first vertical entry A, first
// curve K0, straddle bits}.  A tile's verticals are vert[A(t) .. A(t+1) +
// sV(t+1)) and its curves curve[K0(t) .. K0(t+1) + sC(t+1)), because every
// row's entries are contiguous and rows are consecutive; a sentinel record
// closes the range.  tcap: tile records the buffer holds (the launch may
// precede the host's knowledge of the total; a list that does not fit writes
// no records).
// gate: a build awaiting its validation (WG_OPT_DEFER_VALIDATION) whose
// geometry lists did not fit (its error words [0] / [8]): nothing is read or
// written (the validation redoes the build and this emission)
// ff (fused): the vertex total and the pending words are read out to the host
// by the thread of row `rows` right after it wrote the total — no k_fetch
// launch and no event between this kernel and the tiles (r05: the event cost
// ~12 us on the step's critical path)
template <int TILE>
__global__ void k_vtx_prep(uint64_t rb, uint64_t rows, int64_t sel, const uint32_t *__restrict__ voff,
                           const uint32_t *__restrict__ coff, uint64_t *__restrict__ vtx_off, uint64_t tcap,
                           uint4 *__restrict__ info, const uint32_t *__restrict__ gate, WgFusedFetch ff) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j > rows) return;
    // r06: every load in one round before the first wait (the gate's branch
    // held the offsets' loads behind it: two dependent round trips).  Row
    // j + 1 <= rows + 1 is inside vert_off / curve_off (n + 2 entries).
    typedef const __attribute__((address_space(1))) uint32_t gword;   // global loads, not flat
    const uint64_t r = rb + j;
    const uint32_t g0 = gate ? *(gword *)gate : 0u, g8 = gate ? *(gword *)(gate + 8) : 0u;
    const uint32_t v0 = voff[rb], c0 = coff[rb], vo = voff[r], v1 = voff[r + 1], co = coff[r], c1 = coff[r + 1];
    const uint32_t vn = voff[rb + rows], cn = coff[rb + rows];
    asm volatile("" ::"v"(g0), "v"(g8), "v"(v0), "v"(c0), "v"(vo), "v"(v1), "v"(co), "v"(c1), "v"(vn), "v"(cn));
    if (g0 | g8) {   // (the host still gets the words: they say the build did not hold)
        if (j == rows && ff.seq_word) wg_fused_fetch_store(ff);
        return;
    }
    // vtx_at's closed form on the loaded words
    auto at = [&](uint64_t jj, uint32_t vv, uint32_t cc) -> uint64_t {
        uint64_t v = (uint64_t)WG_VTX_PER_VERTICAL * (vv - v0) + (uint64_t)WG_VTX_PER_CURVE * (cc - c0) +
                     (uint64_t)WG_VTX_PER_NODE * jj;
        if (sel >= 0 && (uint64_t)sel >= rb && (uint64_t)sel < rb + jj) v += WG_VTX_PER_RING;
        return v;
    };
    const uint64_t s = at(j, vo, co);
    vtx_off[j] = s;
    if (j == rows) {
        if (ff.seq_word) wg_fused_fetch_store(ff);
        return;
    }
    const uint64_t e = at(j + 1, v1, c1);
    const uint64_t ntiles = (at(rows, vn, cn) + TILE - 1) / TILE;
    if (ntiles + 1 > tcap) return;
    const uint32_t nv = v1 - vo, nc = c1 - co;
    const uint64_t cv = s + (uint64_t)WG_VTX_PER_VERTICAL * nv;
    for (uint64_t t = (s + TILE - 1) / TILE; t * TILE < e; t++) {
        const uint64_t vt = t * TILE;
        uint32_t A, K0, fl = 0;
        if (vt < cv) {
            const uint64_t d = vt - s;
            A = vo + (uint32_t)(d / WG_VTX_PER_VERTICAL);
            fl |= (d % WG_VTX_PER_VERTICAL) ? 1u : 0u;
            K0 = co;
        } else {
            A = vo + nv;
            const uint64_t d = vt - cv;
            if (d < (uint64_t)WG_VTX_PER_CURVE * nc) {
                K0 = co + (uint32_t)(d / WG_VTX_PER_CURVE);
                fl |= (d % WG_VTX_PER_CURVE) ? 2u : 0u;
            } else {
                K0 = co + nc;
            }
        }
        info[t] = make_uint4((uint32_t)j, A, K0, fl);
    }
    if (j == rows - 1) info[ntiles] = make_uint4((uint32_t)rows, v1, c1, 0u);
}

struct RowInfo {
    uint64_t vstart;
    uint32_t voff, nv, coff, nc;
    float    h, ny, cx;
    uint32_t ncol;
    uint32_t dim;   // 0, or 8 for a row dimmed by the search (palette entries 8..15)
};

__device__ __forceinline__ float lane_x(uint32_t lane, uint32_t vis) {   // lane_center_x (:786-790)
    const uint32_t visual = lane < vis - 1 ? lane : vis - 1;
    return (float)visual * WG_LANE_W + WG_LANE_W * 0.5f;
}
__device__ __forceinline__ float clamp_rs(float x, float lo, float hi) {
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}

template <int TILE>
__global__ void __launch_bounds__(VT) k_vtx_tile(uint64_t rb, uint64_t re, uint64_t vcap, uint32_t vis,
        const uint64_t *__restrict__ vtx_off, const uint32_t *__restrict__ voff, const uint32_t *__restrict__ vert,
        const uint32_t *__restrict__ coff, const wg_curve *__restrict__ curve, const uint8_t *__restrict__ curve_color,
        const float *__restrict__ height, const float *__restrict__ node_y, const uint32_t *__restrict__ lane_out,
        const uint8_t *__restrict__ color_out, const float4 *__restrict__ palette,
        const uint4 *__restrict__ tinfo, const uint8_t *__restrict__ match, int64_t mlo, int64_t mhi,
        float4 *__restrict__ out, uint64_t ntl, const uint32_t *__restrict__ max_lane_dev,
        const uint32_t *__restrict__ gate, int part, uint64_t split_row, uint64_t p1) {
    using G = TileGeo<TILE>;
    constexpr int PAIRS = G::PAIRS, ROUNDS = G::ROUNDS, MAXR = G::MAXR, MAXC = G::MAXC, MAXV = G::MAXV;
    __shared__ RowInfo rows[MAXR];
    __shared__ __attribute__((aligned(4))) uint8_t pair_row[PAIRS];   // row (within the tile) of every vertex pair
    __shared__ float4 pts[MAXC * NPTS];            // (L.x, L.y, R.x, R.y) per strip point
    __shared__ uint32_t curve_col[MAXC];
    __shared__ uint32_t vents[MAXV];               // the tile's vertical entries
    __shared__ __attribute__((aligned(16))) float4 stage[VT / 64][64 * 3];
    __shared__ uint32_t wmax[VT / 64];
    __shared__ float4 pal[2 * WG_PALETTE_SIZE];    // palette, then the same at WG_DIM_ALPHA
    __shared__ float2 circ[3][WG_TESS_NODE_SEGMENTS + 2];   // r*(cos, sin) for node, ring inner, ring outer radius
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (gate && (gate[0] | gate[8])) return;   // (see k_vtx_prep)
    // the grid may be sized by the buffer's capacity (ntl tiles): workgroups
    // past the total's tiles exit, and a total beyond the capacity writes
    // nothing (the host relaunches)
    const uint64_t total = vtx_off[re - rb];
    const uint64_t nt = (total + TILE - 1) / TILE;
    if (total > vcap || nt > ntl) return;   // the tile records would not fit either
    // XCD-aware tile order: workgroups are dealt to the 8 XCDs round-robin, so
    // workgroup b runs on XCD b % 8; that XCD writes one contiguous eighth of the
    // buffer (per tiles) instead of every 8th tile.  Store-only kernels of this
    // shape: 5.6 -> 6.1-6.3 TB/s (profiles/microbench/store_sweep.hip).  The
    // split follows the device's total, so the working workgroups are the
    // first 8 * per of the grid, on all eight XCDs, whatever the capacity.
    // part 1 / 2 (a row-sliced emission): the tiles before / from tile t1,
    // the first tile that may hold a vertex of row split_row or later (its
    // lists are the second slice's, built while part 1 runs); t1 is capped
    // by part 1's grid p1
    uint64_t lo = 0, hi = nt;
    if (part) {
        uint64_t t1 = vtx_off[split_row] / TILE;
        t1 = t1 < p1 ? t1 : p1;
        if (part == 1) hi = t1; else lo = t1;
    }
    const uint64_t per = (hi - lo + 7) / 8;
    const uint64_t tile = lo + (uint64_t)(blockIdx.x % 8u) * per + blockIdx.x / 8u;
    if (blockIdx.x / 8u >= per || tile >= hi) return;
    const uint64_t v0 = tile * TILE;
    const uint4 ti = tinfo[tile], tn = tinfo[tile + 1];   // everything below hangs on these
    const uint64_t v1 = (v0 + TILE < total) ? v0 + TILE : total;
    const uint64_t nrows = re - rb;
    if (max_lane_dev) {   // a build not validated yet (WG_OPT_DEFER_VALIDATION): graph_width (:353-354) from its max_lane
        const uint32_t ml = *max_lane_dev;
        vis = ml + 1 < (uint32_t)WG_LANE_COUNT_VISUAL ? ml + 1 : (uint32_t)WG_LANE_COUNT_VISUAL;
        if (vis < 1) vis = 1;   // (a build that will not validate: any value, the emission is redone)
    }
    const float visf = (float)(vis - 1);
    const uint64_t first = ti.x;
    const uint32_t A = ti.y, K0 = ti.z;
    uint32_t nV = tn.y + (tn.w & 1u) - A, nC = tn.z + ((tn.w >> 1) & 1u) - K0;
    nV = nV < (uint32_t)MAXV ? nV : (uint32_t)MAXV;   // bounds hold by construction; never overrun LDS
    nC = nC < (uint32_t)MAXC ? nC : (uint32_t)MAXC;
    // ---- 1. one round of independent global loads: rows, verticals, curves ---------
    // Every load of the tile is issued before any is used (wave 0 the rows, the
    // other waves first the vertical entries, every thread its curve strip
    // points' records): once the geometry no longer sits in the Infinity Cache
    // each round trip costs microseconds under the saturated write stream, and
    // rows -> verticals -> curves one after the other in wave 0 took the
    // Linux-shaped list's emission from 2.3 to 3.3 ms.
    // only the rows overlapping the tile, [first, first row of the next tile]:
    // loading a fixed 64-row window made every XCD's L2 fetch nearly every
    // row (tiles are dealt round-robin to the 8 XCDs) — 0.3 GB of HBM reads
    // per 1M-row launch
    const uint64_t jr = first + lane;
    const uint32_t span = tn.x >= first ? (uint32_t)(tn.x - first) : 0u;
    const bool rowok = wid == 0 && jr < nrows && lane <= span && lane < (uint32_t)MAXR;
    // the row's words as loaded: no arithmetic on them until every load is out
    uint64_t r_vstart = 0;
    uint32_t r_v0 = 0, r_v1 = 0, r_c0 = 0, r_c1 = 0, r_lane = 0, r_col = 0, r_m = 1;
    float r_h = 0.0f, r_ny = 0.0f;
    if (rowok) {
        const uint64_t r = rb + jr;
        r_vstart = vtx_off[jr];
        r_v0 = voff[r];
        r_v1 = voff[r + 1];
        r_c0 = coff[r];
        r_c1 = coff[r + 1];
        r_h = height[r];
        r_ny = node_y[r];
        r_lane = lane_out[r];
        r_col = color_out[r];
        // search dimming (history_view, commit_graph.rs:1467, 1482): rows of the
        // match range whose flag is 0 take the dimmed palette
        if (match && (int64_t)r >= mlo && (int64_t)r < mhi) r_m = match[(int64_t)r - mlo];
    }
    constexpr int VPT = (MAXV + VT - 1) / VT, CPT = (MAXC * NPTS + VT - 1) / VT;
    const uint32_t vi0 = (tid + VT - 64) % VT;   // vertical entries: waves 1.. first (wave 0 loads the rows)
    uint32_t vv[VPT];
#pragma unroll
    for (int q = 0; q < VPT; q++) {
        const uint32_t i = vi0 + q * VT;
        vv[q] = i < nV ? vert[A + i] : 0u;
    }
    float4 ca[CPT], cb[CPT];
    uint32_t ccol[CPT];
#pragma unroll
    for (int q = 0; q < CPT; q++) {
        const uint32_t task = tid + q * VT, k = K0 + task / NPTS;
        ca[q] = cb[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        ccol[q] = 0;
        if (task < nC * NPTS) {
            ca[q] = reinterpret_cast<const float4 *>(curve + k)[0];
            cb[q] = reinterpret_cast<const float4 *>(curve + k)[1];
            if (task % NPTS == 0) ccol[q] = curve_color[k];
        }
    }
    float4 palv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (tid < 2 * WG_PALETTE_SIZE) palv = palette[tid];
    const uint32_t cw = tid / (WG_TESS_NODE_SEGMENTS + 1), cq = tid % (WG_TESS_NODE_SEGMENTS + 1);
    float cc = 0.0f, cs = 0.0f;
    if (tid < 3 * (WG_TESS_NODE_SEGMENTS + 1)) { cc = c_cos[cq]; cs = c_sin[cq]; }
    if (tid < 3 * (WG_TESS_NODE_SEGMENTS + 1)) {
        const float r = cw == 0 ? WG_NODE_RADIUS
                      : cw == 1 ? WG_NODE_RADIUS - WG_SELECTED_RING_WIDTH * 0.5f
                                : WG_NODE_RADIUS + WG_SELECTED_RING_WIDTH * 0.5f;
        circ[cw][cq] = make_float2(r * cc, r * cs);
    }
    if (tid < 2 * WG_PALETTE_SIZE) pal[tid] = palv;
    RowInfo ri;
    ri.vstart = r_vstart;
    ri.voff = r_v0;
    ri.nv = r_v1 - r_v0;
    ri.coff = r_c0;
    ri.nc = r_c1 - r_c0;
    ri.h = r_h;
    ri.ny = r_ny;
    ri.cx = lane_x(r_lane, vis);
    ri.ncol = r_col;
    ri.dim = r_m ? 0u : 8u;
    if (wid == 0) {
        // wave 0 alone clears pair_row and then marks the row starts: LDS ops of
        // one wave complete in order, so no other wave can clear a mark after it
        // was written (the clear used to be spread over all waves, unordered
        // against wave 0's marks before the barrier)
        for (uint32_t i = lane; i < PAIRS / 4; i += 64) reinterpret_cast<uint32_t *>(pair_row)[i] = 0u;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (rowok && ri.vstart < v1) {
            rows[lane] = ri;
            const uint32_t sp = ri.vstart > v0 ? (uint32_t)((ri.vstart - v0) >> 1) : 0u;
            pair_row[sp] = lane;   // distinct rows start at distinct pairs (>= 36 pairs per row)
        }
    }
#pragma unroll
    for (int q = 0; q < VPT; q++) {
        const uint32_t i = vi0 + q * VT;
        if (i < nV) vents[i] = vv[q];
    }
    {
        // the <= MAXC curve segments overlapping the tile, tessellated once
        const float hw = WG_LINE_WIDTH * 0.5f;
#pragma unroll
        for (int q = 0; q < CPT; q++) {
            const uint32_t task = tid + q * VT;
            if (task >= nC * NPTS) break;
            const uint32_t slot = task / NPTS, jj = task % NPTS;
            float X[4] = {ca[q].x, ca[q].z, cb[q].x, cb[q].z}, Y[4] = {ca[q].y, ca[q].w, cb[q].y, cb[q].w};
#pragma unroll
            for (int i = 0; i < 4; i++) X[i] = clamp_rs(X[i], 0.0f, visf) * WG_LANE_W + WG_LANE_W * 0.5f;  // to_x (:847-850)
            const float t = (float)jj * WG_TESS_DT;
            const float s = 1.0f - t;
            const float px = s * s * s * X[0] + 3.0f * s * s * t * X[1] + 3.0f * s * t * t * X[2] + t * t * t * X[3];
            const float py = s * s * s * Y[0] + 3.0f * s * s * t * Y[1] + 3.0f * s * t * t * Y[2] + t * t * t * Y[3];
            const float dx = 3.0f * s * s * (X[1] - X[0]) + 6.0f * s * t * (X[2] - X[1]) + 3.0f * t * t * (X[3] - X[2]);
            const float dy = 3.0f * s * s * (Y[1] - Y[0]) + 6.0f * s * t * (Y[2] - Y[1]) + 3.0f * t * t * (Y[3] - Y[2]);
            const float len = sqrtf(dx * dx + dy * dy);
            float nx, ny;
            if (len > 0.0f) { nx = -dy / len; ny = dx / len; } else { nx = 1.0f; ny = 0.0f; }
            pts[task] = make_float4(px + hw * nx, py + hw * ny, px - hw * nx, py - hw * ny);
            if (jj == 0) curve_col[slot] = ccol[q];
        }
    }
    __syncthreads();
    // ---- 2. prefix-max over pair_row: each thread owns ROUNDS consecutive pairs ----------
    {
        uint32_t loc[ROUNDS], m = 0;
#pragma unroll
        for (int q = 0; q < ROUNDS; q++) { const uint32_t x = pair_row[tid * ROUNDS + q]; m = x > m ? x : m; loc[q] = m; }
        uint32_t inc = m;
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = (uint32_t)__shfl_up((int)inc, d, 64);
            if (lane >= (uint32_t)d) inc = o > inc ? o : inc;
        }
        if (lane == 63) wmax[wid] = inc;
        uint32_t ex = (uint32_t)__shfl_up((int)inc, 1, 64);
        if (lane == 0) ex = 0;
        __syncthreads();
        for (uint32_t w = 0; w < wid; w++) ex = wmax[w] > ex ? wmax[w] : ex;
#pragma unroll
        for (int q = 0; q < ROUNDS; q++) pair_row[tid * ROUNDS + q] = loc[q] > ex ? loc[q] : ex;
    }
    __syncthreads();
    // ---- 3. emit pairs; per-wave LDS transpose -> contiguous stores --------------------------
    const float hw = WG_LINE_WIDTH * 0.5f;
    const uint32_t npairs = (uint32_t)((v1 - v0) >> 1);
    float4 *st = stage[wid];
#pragma unroll 1
    for (int q = 0; q < ROUNDS; q++) {
        const uint32_t wbase = q * VT + wid * 64;          // this wave's first pair in the round
        if (wbase >= npairs) break;
        const uint32_t p = wbase + lane;
        if (p < npairs) {
            const RowInfo &ri = rows[pair_row[p]];
            uint32_t l = (uint32_t)(v0 + 2ull * p - ri.vstart);   // even
            float xa, ya, xb, yb;
            uint32_t col;
            if (l < 6u * ri.nv) {
                const uint32_t e = vents[ri.voff + l / 6u - A];
                const uint32_t corner = l % 6u;   // 0, 2, 4
                const float xc = lane_x(WG_VERT_LANE(e), vis);
                const uint32_t kind = WG_VERT_KIND(e);
                const float y0 = kind == WG_VERT_BOTTOM ? ri.ny : 0.0f;
                const float y1 = kind == WG_VERT_TOP ? ri.ny : ri.h;
                const float xl = xc - hw, xr = xc + hw;
                // (xl,y0) (xr,y0) | (xl,y1) (xr,y0) | (xr,y1) (xl,y1)
                xa = corner == 4 ? xr : xl;
                ya = corner == 0 ? y0 : y1;
                xb = corner == 4 ? xl : xr;
                yb = corner == 4 ? y1 : y0;
                col = WG_VERT_COLOR(e);
            } else if ((l -= 6u * ri.nv) < 96u * ri.nc) {
                const uint32_t slot = ri.coff + l / 96u - K0, m = l % 96u;
                const uint32_t seg = m / 6u, corner = m % 6u;   // 0, 2, 4
                // L_j R_j | L_j+1 R_j | R_j+1 L_j+1
                const float4 pa = pts[slot * NPTS + seg + (corner == 0 ? 0u : 1u)];
                const float4 pb = pts[slot * NPTS + seg + (corner == 4 ? 1u : 0u)];
                if (corner == 4) { xa = pa.z; ya = pa.w; xb = pb.x; yb = pb.y; }
                else             { xa = pa.x; ya = pa.y; xb = pb.z; yb = pb.w; }
                col = curve_col[slot];
            } else if ((l -= 96u * ri.nc) < (uint32_t)WG_VTX_PER_NODE) {
                // fan triangle t: (C, Q_t, Q_t+1); vertices l and l+1 may sit in two triangles
                const uint32_t ta = l / 3u, ca = l % 3u, tb = (l + 1) / 3u, cb = (l + 1) % 3u;
                const float2 oa = circ[0][ca == 0 ? 0u : ta + ca - 1u], ob = circ[0][cb == 0 ? 0u : tb + cb - 1u];   // r*cos, r*sin
                const float xa_ = ri.cx + oa.x, ya_ = ri.ny + oa.y, xb_ = ri.cx + ob.x, yb_ = ri.ny + ob.y;
                xa = ca == 0 ? ri.cx : xa_;
                ya = ca == 0 ? ri.ny : ya_;
                xb = cb == 0 ? ri.cx : xb_;
                yb = cb == 0 ? ri.ny : yb_;
                col = ri.ncol;
            } else {
                l -= WG_VTX_PER_NODE;
                const uint32_t qd = l / 6u, corner = l % 6u;   // 0, 2, 4
                // o_q i_q | o_q+1 i_q | i_q+1 o_q+1   (circ[1] inner radius, circ[2] outer)
                const uint32_t ia = corner == 0 ? qd : qd + 1u, ib = corner == 4 ? qd + 1u : qd;
                const float2 oa = circ[corner == 4 ? 1 : 2][ia], ob = circ[corner == 4 ? 2 : 1][ib];
                xa = ri.cx + oa.x; ya = ri.ny + oa.y;
                xb = ri.cx + ob.x; yb = ri.ny + ob.y;
                col = WG_COLOR_FOREGROUND;
            }
            const float4 c4 = pal[(col & 7u) | ri.dim];
            st[lane * 3 + 0] = make_float4(xa, ya, c4.x, c4.y);
            st[lane * 3 + 1] = make_float4(c4.z, c4.w, xb, yb);
            st[lane * 3 + 2] = c4;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the wave's pairs [wbase, wbase + cnt) are 3 * cnt contiguous float4 in the output
        const uint32_t cnt = (npairs - wbase) < 64u ? (npairs - wbase) : 64u;
        float4 *dst = out + (v0 / 2 + wbase) * 3;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            const uint32_t i = k * 64 + lane;
            // streaming (non-temporal) stores: the buffer is not re-read by this pass
            if (i < cnt * 3) {
#ifdef WG_PLAIN_STORES
                reinterpret_cast<v4f *>(dst)[i] = reinterpret_cast<const v4f *>(st)[i];
#else
                __builtin_nontemporal_store(reinterpret_cast<const v4f *>(st)[i], reinterpret_cast<v4f *>(dst) + i);
#endif
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// order-sensitive checksum (same definition as oracle/wg_oracle.c)
__global__ void k_checksum(const uint32_t *__restrict__ w, uint64_t nwords, unsigned long long *acc) {
    unsigned long long s = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t x = ((uint64_t)w[i] << 32) ^ (i * 0x9E3779B97F4A7C15ull);
        x ^= x >> 33; x *= 0xFF51AFD7ED558CCDull; x ^= x >> 33; x *= 0xC4CEB9FE1A85EC53ull; x ^= x >> 33;
        s += x;
    }
    for (int d = 32; d >= 1; d >>= 1) s += __shfl_down(s, d, 64);
    if ((threadIdx.x & 63) == 0) atomicAdd(acc, s);
}

}  // namespace

int wg_stage_vertices(wg_ctx *c, uint64_t rb, uint64_t re, int64_t sel) {
    const uint64_t rows = re - rb;
    hipStream_t s = c->stream;
    // the tile size: WG_OPT_VTX_TILE, or (auto) from the last emission's
    // vertex count: past 4e8 (its geometry past the Infinity Cache) 2048, past
    // 1.6e9 4096, else 1024 (r05 A/B, profiles/r05/r05c_vtx_tile.jsonl:
    // linuxwide 1M 13.93 / 12.81 / 12.65 ms/step at 1024 / 2048 / 4096,
    // wide16 3M 4.28 / 4.19 / 4.33, wide16 1M 1.479 / 1.498, C4 3.881 / 3.896)
    uint32_t TILE = c->vtx_tile_opt;
    if (!TILE) {
        const uint64_t last = c->vtx_tiles_last * c->vtx_tile_last;
        TILE = last > 4 * wg_ctx::WG_VTX_BIG_VERTICES ? 4096u : last > wg_ctx::WG_VTX_BIG_VERTICES ? 2048u : 1024u;
    }
    if (TILE != c->vtx_tile_last) {   // (tile indices of the last emission do not carry over)
        c->vtx_tiles_last = c->vtx_tiles_last * c->vtx_tile_last / TILE;
        c->vtx_t1_last = 0;
        c->vtx_tile_last = TILE;
    }
    WG_ALLOC(c, c->vtx_off, (rows + 2) * 8);
    { const int _sr = wg_scan_reserve(c, rows + 2); if (_sr != WG_OK) return _sr; }
    c->vrow_begin = rb;
    c->vrow_end = re;
    c->selected = sel;
    c->n_vtx = 0;
    if (rows == 0) {
        WG_HIP(c, hipMemsetAsync(c->vtx_off.p, 0, 8, s));
        return WG_OK;
    }
    wg_stage_begin(c, "vtx_counts");
    uint64_t *off = c->vtx_off.as<uint64_t>();
    const uint32_t *gate = c->pend.build ? c->geom_err : nullptr;   // a build awaiting its validation
    auto prep = [&](uint64_t tcap, const WgFusedFetch &ff) {   // vtx_off + tile records (none when tcap is too small)
#define WG_PREP_LAUNCH(TL)                                                                                       \
        hipLaunchKernelGGL(k_vtx_prep<TL>, dim3((rows + 1 + 255) / 256), dim3(256), 0, s, rb, rows, sel,          \
                           c->vert_off.as<const uint32_t>(), c->curve_off.as<const uint32_t>(), off, tcap,       \
                           c->tile_first.as<uint4>(), gate, ff)
        if (TILE == 4096) WG_PREP_LAUNCH(4096);
        else if (TILE == 2048) WG_PREP_LAUNCH(2048);
        else WG_PREP_LAUNCH(1024);
#undef WG_PREP_LAUNCH
    };
    const WgFusedFetch no_fetch{};
    const uint64_t vcap = c->vtx.cap > 64 ? (c->vtx.cap - 64) / sizeof(wg_vertex) : 0;
    const uint64_t tcap = c->tile_first.cap / sizeof(uint4);
    const bool early = vcap > 0 && tcap > 1;
    // a full pass's deferred lists (wg_geom_lists): row-sliced under the
    // emission of the whole list, else run whole here
    const bool sliced = c->glist.deferred && early && rb == 0 && rows == c->glist.n;
    if (!sliced)
        if (const int rc = wg_geom_lists_flush(c)) return rc;
    float q = roundf(c->graph_width / WG_LANE_W);
    uint32_t vis = q <= 0.0f ? 0u : (uint32_t)q;
    if (vis < 1) vis = 1;
    // The total is read back without stalling the stream: the tiles are
    // launched right away into the buffers as they are (steady-state frames
    // fit the last frame's capacity; the kernels exit past the total and
    // write nothing when it does not fit), and relaunched only if needed.
    // a build awaiting its validation (WG_OPT_DEFER_VALIDATION): its words ride on this read
    WgFetch fi[4 + WG_PENDING_ITEMS];
    fi[0] = WgFetch{off + rows, true};
    const int npend = c->pend.build ? c->pend.k : 0;
    for (int i = 0; i < npend; i++) fi[1 + i] = c->pend.it[i];
    // the split row h (a chunk boundary, about slice_frac of the rows): its
    // vertex offset rides on the read (part 1's grid for the next frame)
    uint64_t h = 0;
    if (sliced) {
        h = (uint64_t)((double)rows * c->slice_frac) / WG_SWEEP_CH * WG_SWEEP_CH;
        const uint64_t hmax = (rows - 1) / WG_SWEEP_CH * WG_SWEEP_CH;
        h = h < WG_SWEEP_CH ? WG_SWEEP_CH : (h > hmax ? hmax : h);
        fi[1 + npend] = WgFetch{off + h, true};
        fi[2 + npend] = WgFetch{c->glist.err + 1, false};   // the slices' wide chunks
        fi[3 + npend] = WgFetch{c->glist.err + 4, false};
    }
    const int nfi = 1 + npend + (sliced ? 3 : 0);
    bool fused_read = false;
    if (sliced) {
        prep(early ? tcap : 0, no_fetch);   // (the read is launched below, with the tiles)
    } else if (early && c->fused_read) {
        // the read folded into the prep kernel (r05): its last thread writes the
        // total and the pending words to the host right after computing the
        // total, so the tiles start right after the prep — no k_fetch launch,
        // no system-scope release and no event record between them (r04 read on
        // the side stream behind an event record: a ~12 us gap before the tiles)
        WgFusedFetch ff;
        if (const int rc = wg_fetch_fused_begin(c, nfi, fi, &ff)) return rc;
        prep(tcap, ff);
        fused_read = true;
    } else {
        prep(early ? tcap : 0, no_fetch);
        if (const int rc = wg_fetch_begin_n(c, nfi, fi)) return rc;
    }
    // (a pending single-GPU build, or a sharded one whose replay is unchecked:
    // graph_width from the device's lane scalars)
    const uint32_t *ml_dev =
        npend && (!c->pend.shard || c->sh.replay_pending) ? c->lane_scalars.as<const uint32_t>() : nullptr;
    // search-match flags of global rows [match_rb, match_re) -> context rows [mlo, mhi)
    const uint8_t *match = c->match_on ? c->match_flags.as<const uint8_t>() : nullptr;
    const int64_t mlo = (int64_t)c->match_rb - (int64_t)c->sh.s + (int64_t)c->sh.row_base;
    const int64_t mhi = mlo + (int64_t)(c->match_re - c->match_rb);
    // part 0: every tile; 1 / 2: the tiles before / from the split (see
    // k_vtx_tile); ntl: the tile bound of the fit check, the same for both parts
    // mark: the launch is the "vtx_emit" stage (the sliced emission marks its
    // two parts together: from part 1's start to the side's join)
    auto launch_on = [&](hipStream_t st, uint64_t vcap, uint64_t grid, uint64_t ntl, int part, uint64_t p1, bool mark) {
        if (mark) {
            wg_stage_end(c);
            wg_stage_begin(c, "vtx_emit");
        }
        // (grid rounded up to whole XCD rounds: k_vtx_tile's tile order)
#define WG_VTX_LAUNCH(TL)                                                                                                     \
        hipLaunchKernelGGL(k_vtx_tile<TL>, dim3((uint32_t)((grid + 7) / 8 * 8)), dim3(VT), 0, st, rb, re, vcap, vis,          \
                           (const uint64_t *)off, c->vert_off.as<const uint32_t>(), c->vert.as<const uint32_t>(),             \
                           c->curve_off.as<const uint32_t>(), c->curve.as<const wg_curve>(), c->curve_color.as<const uint8_t>(),\
                           c->g_height.as<const float>(), c->g_node_y.as<const float>(), c->lane_out.as<const uint32_t>(),    \
                           c->color_out.as<const uint8_t>(), c->palette.as<const float4>(), c->tile_first.as<const uint4>(),  \
                           match, mlo, mhi, c->vtx.as<float4>(), ntl, ml_dev, gate, part, h, p1)
        if (TILE == 4096) WG_VTX_LAUNCH(4096);
        else if (TILE == 2048) WG_VTX_LAUNCH(2048);
        else WG_VTX_LAUNCH(1024);
#undef WG_VTX_LAUNCH
        if (mark) wg_stage_end(c);
    };
    auto launch = [&](uint64_t vcap, uint64_t grid, uint64_t ntl, int part, uint64_t p1) {
        launch_on(s, vcap, grid, ntl, part, p1, true);
    };
    // the early grid: the buffers' capacity, bounded by twice the last
    // emission's tiles (a context whose lists shrank would otherwise launch
    // its largest list's grid every frame); a list that outgrows it is
    // launched again whole below
    uint64_t early_grid = std::min((vcap + TILE - 1) / TILE, tcap - 1);
    if (c->vtx_tiles_last) early_grid = std::min(early_grid, 2 * c->vtx_tiles_last + 64);
    // part 1's grid: the last sliced frame's split tile (a guess the first
    // time); part 2 covers the rest of the early grid, checked below
    uint64_t g1 = 0, g2 = 0;
    if (sliced) {
        // main: rows [0, h)'s lists, then their tiles (part 1); the side
        // stream, after those lists: rows [h, n)'s lists beside part 1, the
        // read (the validation words include both slices' flags), the other
        // tiles (part 2); main then waits for the side (every later call and
        // the next build are ordered after part 2)
        c->glist.deferred = false;
        c->sliced_emits++;
        g1 = c->vtx_t1_last ? c->vtx_t1_last : (uint64_t)((double)early_grid * c->slice_frac);
        g1 = (std::min(g1, early_grid) + 7) / 8 * 8;
        g2 = early_grid > g1 ? early_grid - g1 + 64 : 64;
        if (const int rc = wg_geom_lists(c, 0, h, 0, s)) return rc;
        if (const int rc = wg_side_fork(c)) return rc;
        int rc = wg_geom_lists(c, h, rows, 1, c->stream);
        if (rc == WG_OK) rc = wg_fetch_begin_n(c, nfi, fi);
        if (rc == WG_OK) launch_on(c->stream, vcap, g2, early_grid, 2, g1, false);
        wg_side_done(c);
        if (rc) return rc;
        wg_stage_end(c);
        wg_stage_begin(c, "vtx_emit");
        launch_on(s, vcap, g1, early_grid, 1, g1, false);
        if ((rc = wg_side_join(c)) != WG_OK) return rc;
        wg_stage_end(c);
    } else if (early) {
        launch(vcap, early_grid, early_grid, 0, 0);
    }
    if (fused_read && !c->sh.on && c->side) {
        // the next build's empty table, on the side stream (ordered after the
        // previous builds' use of it by this build's fork); r06: a build with
        // its table on the side stream has cleared it there already, beside
        // its lanes (wg_side_build_begin), and this finds it clean
        if (const int rc = wg_hash_clear_next(c, c->side)) return rc;
    }
    uint64_t fv[4 + WG_PENDING_ITEMS] = {0};
    if (const int rc = wg_fetch_end(c, fv)) return rc;
    if (npend) {   // validate the build; one that did not hold is redone here, with this frame and emission
        bool redone = false;
        if (const int rc = wg_validate_pending(c, fv + 1, &redone)) return rc;
        if (redone) return WG_OK;
    }
    const uint64_t total = fv[0];
    c->n_vtx = total;
    const uint64_t ntiles = (total + TILE - 1) / TILE;
    c->vtx_tiles_last = ntiles;
    if (!early || total > vcap || ntiles + 1 > tcap || ntiles > early_grid) {   // did not fit: size the buffers and launch again
        if (early) wg_stage_begin(c, "vtx_counts");
        if (const int rc = wg_alloc_placed(c, c->vtx, total * sizeof(wg_vertex) + 64, true)) return rc;
        WG_ALLOC(c, c->tile_first, (ntiles + 1) * sizeof(uint4));
        prep(ntiles + 1, no_fetch);
        launch(total, ntiles, ntiles, 0, 0);
    } else if (sliced) {
        const uint64_t t1 = fv[1 + npend] / TILE;
        c->vtx_t1_last = t1;
        c->sweep_wide_last = (uint32_t)(fv[2 + npend] + fv[3 + npend]);
        const uint64_t need2 = ntiles - std::min(t1, g1);
        if (need2 > (g2 + 7) / 8 * 8) launch(vcap, need2, early_grid, 2, g1);   // part 2 short of tiles: again, whole
    }
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

// ---------------------------------------------------------------------------
// Output buffer placement (WG_OPT_VTX_PLACE): the vertex buffer (the glyph
// quads' buffer measured no gain, r06bd: 1.253 against 1.248 ms).  The emission's store rate is a
// property of the physical pages behind the vertex buffer: one 5.75 GB buffer
// takes 0.81-0.83 ms or 0.92-0.94 ms per wide16 1M emission (7.0 or 6.1 TB/s),
// fixed for the buffer's lifetime and changed only by reallocating it with
// the same inputs (profiles/r06/r06ax_*; not clocks or power: r06at_*).  A buffer
// of 1 GiB or more is therefore chosen from up to vtx_place candidates, each timed
// with the emission's own store pattern (non-temporal 16-byte stores in 24 KiB
// tiles taken grid-stride, one pass; r06bk-bm: fast candidates 0.90-0.96 ms,
// slow 1.09-1.18 for 6.1 GB — twice the separation of a first probe that gave
// each workgroup one contiguous block), and the fastest is kept, the
// others freed (r06ay: the probe's best of 4 picked buffers emitting in
// 0.819-0.855 ms where plain allocations in the same process took 0.82-0.94;
// the first large allocation of a process landed on the slow pages on 5 of 6
// boxes, r06at-bb).  The probe ranks candidates within a process only: its
// absolute rate differs from box to box.  Once per growth of the buffer (1/16
// headroom; ~5 ms for 4 x 6 GB on the first emission), never per frame.
// ---------------------------------------------------------------------------
#define WG_PLACE_MIN_BYTES (1ull << 30)

// 24 KiB tiles (the emission's tile of 1024 vertices), taken grid-stride by
// the workgroups, 16-byte non-temporal stores
constexpr uint32_t PROBE_TILE4 = 1536;
__global__ void __launch_bounds__(256) k_store_probe(v4f *__restrict__ out, uint64_t n4) {
    const v4f z = {0.f, 0.f, 0.f, 0.f};
    const uint64_t ntile = (n4 + PROBE_TILE4 - 1) / PROBE_TILE4;
    for (uint64_t t = blockIdx.x; t < ntile; t += gridDim.x) {
        const uint64_t b = t * PROBE_TILE4, e = b + PROBE_TILE4 < n4 ? b + PROBE_TILE4 : n4;
        for (uint64_t i = b + threadIdx.x; i < e; i += 256) __builtin_nontemporal_store(z, out + i);
    }
}

static int vtx_probe_ms(wg_ctx *c, void *p, size_t bytes, float *ms) {
    hipEvent_t e0, e1;
    WG_HIP(c, hipEventCreate(&e0));
    WG_HIP(c, hipEventCreate(&e1));
    const uint64_t n4 = bytes / sizeof(v4f);
    *ms = 1e30f;
    int rc = WG_OK;
    for (int rep = 0; rep < 1 && rc == WG_OK; rep++) {   // one pass (r06ba: 3 passes cost the first emission 14 ms for 4 candidates)
        float t = 0.f;
        hipError_t e = hipEventRecord(e0, c->stream);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_store_probe, dim3(4096), dim3(256), 0, c->stream, reinterpret_cast<v4f *>(p), n4);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipEventRecord(e1, c->stream);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        if (e == hipSuccess) e = hipEventElapsedTime(&t, e0, e1);
        if (e != hipSuccess) rc = wg_fail(c, WG_E_HIP, "vertex placement probe: %s", hipGetErrorString(e));
        else if (t < *ms) *ms = t;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return rc;
}

int wg_alloc_placed(wg_ctx *c, DevBuf &buf, size_t bytes, bool record) {
    const uint32_t k_max = std::min<uint32_t>(c->vtx_place, 8);
    if (bytes <= buf.cap && buf.p) return WG_OK;
    if (record) c->vtx_place_n = 0;
    if (k_max <= 1 || bytes < WG_PLACE_MIN_BYTES) {
        WG_ALLOC(c, buf, bytes);
        return WG_OK;
    }
    WG_HIP(c, hipStreamSynchronize(c->stream));
    buf.release();
    DevBuf cand[8];
    float best = 1e30f;
    int ib = -1, rc = WG_OK;
    for (uint32_t k = 0; k < k_max && rc == WG_OK; k++) {
        if (k) {   // another candidate only with room for it beside the ones held
            size_t fr = 0, tot = 0;
            if (hipMemGetInfo(&fr, &tot) != hipSuccess || fr < bytes + bytes / 16 + (4ull << 30)) break;
        }
        if (cand[k].ensure(bytes) != hipSuccess) { (void)hipGetLastError(); break; }
        float ms = 0.f;
        rc = vtx_probe_ms(c, cand[k].p, cand[k].cap, &ms);
        if (rc == WG_OK) {
            if (record) {
                c->vtx_place_ms[k] = ms;
                c->vtx_place_n = k + 1;
            }
            if (ms < best) { best = ms; ib = (int)k; }
        }
    }
    for (int k = 0; k < 8; k++) if (k != ib) cand[k].release();
    if (rc != WG_OK) { if (ib >= 0) cand[ib].release(); return rc; }
    if (ib < 0) { WG_ALLOC(c, buf, bytes); return WG_OK; }
    buf.p = cand[ib].p;
    buf.cap = cand[ib].cap;
    if (record) c->vtx_place_pick = (uint32_t)ib;
    return WG_OK;
}

int wg_words_checksum(wg_ctx *c, const uint32_t *w, uint64_t nw, uint64_t *out) {
    WG_ALLOC(c, c->chk, 64);
    WG_HIP(c, hipMemsetAsync(c->chk.p, 0, 8, c->stream));
    if (nw) {
        uint64_t b = (nw + 255) / 256;
        if (b > 4096) b = 4096;
        hipLaunchKernelGGL(k_checksum, dim3(b), dim3(256), 0, c->stream, w, nw, c->chk.as<unsigned long long>());
        WG_HIP(c, hipGetLastError());
    }
    return wg_fetch(c, {{c->chk.p, true}}, out);
}

int wg_vertex_checksum_run(wg_ctx *c, uint64_t *out) {
    return wg_words_checksum(c, c->vtx.as<const uint32_t>(), c->n_vtx * 6, out);
}
