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
// HBM-write-bound.  The output is cut into fixed tiles of 1536 vertices
// (36 KiB) so every workgroup writes the same number of bytes: the
// workgroup locates the rows overlapping its tile, each thread computes
// whole vertices into an LDS staging tile, and the tile leaves as
// contiguous 16-byte stores (one 1 KiB wave-instruction per 64 lanes).
#include "wg_internal.h"
#include "wgraph_tess.h"

namespace {

constexpr int VT = 256;
constexpr int TILE = WG_VTX_TILE;
constexpr int MAXR = TILE / WG_VTX_PER_NODE + 3;

__constant__ float c_cos[25] = WG_UNIT_CIRCLE_COS_INIT;
__constant__ float c_sin[25] = WG_UNIT_CIRCLE_SIN_INIT;

__global__ void k_vtx_counts(uint64_t rb, uint64_t re, int64_t sel, const uint32_t *__restrict__ voff,
                             const uint32_t *__restrict__ coff, uint64_t *__restrict__ cnt) {
    uint64_t r = rb + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= re) return;
    uint64_t v = (uint64_t)WG_VTX_PER_VERTICAL * (voff[r + 1] - voff[r]) +
                 (uint64_t)WG_VTX_PER_CURVE * (coff[r + 1] - coff[r]) + WG_VTX_PER_NODE;
    if (sel >= 0 && (uint64_t)sel == r) v += WG_VTX_PER_RING;
    cnt[r - rb] = v;
}

struct RowInfo {
    uint64_t vstart;
    uint32_t voff, nv, coff, nc;
    float    h, ny, cx;
    uint32_t ncol, sel;
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

__global__ void __launch_bounds__(VT) k_vtx_tiles(uint64_t rb, uint64_t re, uint64_t total, int64_t sel, uint32_t vis,
        const uint64_t *__restrict__ vtx_off, const uint32_t *__restrict__ voff, const uint32_t *__restrict__ vert,
        const uint32_t *__restrict__ coff, const wg_curve *__restrict__ curve, const uint8_t *__restrict__ curve_color,
        const float *__restrict__ height, const float *__restrict__ node_y, const uint32_t *__restrict__ lane_out,
        const uint8_t *__restrict__ color_out, const float4 *__restrict__ palette, float *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float stage[TILE * 6];
    __shared__ RowInfo rows[MAXR];
    __shared__ uint32_t s_first, s_nrows;
    __shared__ float4 pal[WG_PALETTE_SIZE];
    const uint64_t v0 = (uint64_t)blockIdx.x * TILE;
    const uint64_t v1 = (v0 + TILE < total) ? v0 + TILE : total;
    const uint64_t nrows = re - rb;
    if (threadIdx.x < WG_PALETTE_SIZE) pal[threadIdx.x] = palette[threadIdx.x];
    if (threadIdx.x == 0) {
        // last row with vtx_off[row] <= v0
        uint64_t lo = 0, hi = nrows - 1;
        while (lo < hi) {
            uint64_t mid = (lo + hi + 1) / 2;
            if (vtx_off[mid] <= v0) lo = mid; else hi = mid - 1;
        }
        s_first = (uint32_t)lo;
        s_nrows = 0;
    }
    __syncthreads();
    const uint64_t first = s_first;
    if (threadIdx.x < MAXR) {
        const uint64_t j = first + threadIdx.x;
        if (j < nrows && vtx_off[j] < v1) {
            const uint64_t r = rb + j;
            RowInfo ri;
            ri.vstart = vtx_off[j];
            ri.voff = voff[r];
            ri.nv = voff[r + 1] - ri.voff;
            ri.coff = coff[r];
            ri.nc = coff[r + 1] - ri.coff;
            ri.h = height[r];
            ri.ny = node_y[r];
            ri.cx = lane_x(lane_out[r], vis);
            ri.ncol = color_out[r];
            ri.sel = (sel >= 0 && (uint64_t)sel == r) ? 1u : 0u;
            rows[threadIdx.x] = ri;
            atomicMax(&s_nrows, threadIdx.x + 1);
        }
    }
    __syncthreads();
    const uint32_t nr = s_nrows;
    const float hw = WG_LINE_WIDTH * 0.5f;
    const float visf = (float)(vis - 1);
    for (uint64_t v = v0 + threadIdx.x; v < v1; v += VT) {
        uint32_t j = 0;
        while (j + 1 < nr && rows[j + 1].vstart <= v) j++;
        const RowInfo &ri = rows[j];
        uint32_t l = (uint32_t)(v - ri.vstart);
        float x, y;
        uint32_t col;
        if (l < 6u * ri.nv) {
            const uint32_t e = vert[ri.voff + l / 6u];
            const uint32_t corner = l % 6u;
            const float xc = lane_x(WG_VERT_LANE(e), vis);
            const uint32_t kind = WG_VERT_KIND(e);
            const float y0 = kind == WG_VERT_BOTTOM ? ri.ny : 0.0f;
            const float y1 = kind == WG_VERT_TOP ? ri.ny : ri.h;
            // (xl,y0) (xr,y0) (xl,y1) (xr,y0) (xr,y1) (xl,y1)
            const bool right = corner == 1 || corner == 3 || corner == 4;
            const bool low = corner == 2 || corner == 4 || corner == 5;
            x = right ? xc + hw : xc - hw;
            y = low ? y1 : y0;
            col = WG_VERT_COLOR(e);
        } else if ((l -= 6u * ri.nv) < 96u * ri.nc) {
            const uint32_t k = ri.coff + l / 96u, m = l % 96u;
            const uint32_t seg = m / 6u, corner = m % 6u;
            // corners: L_j R_j L_j+1 R_j R_j+1 L_j+1
            const uint32_t jj = seg + ((corner == 2 || corner == 4 || corner == 5) ? 1u : 0u);
            const bool rside = corner == 1 || corner == 3 || corner == 4;
            const float4 a = reinterpret_cast<const float4 *>(curve + k)[0];
            const float4 b = reinterpret_cast<const float4 *>(curve + k)[1];
            float X[4] = {a.x, a.z, b.x, b.z}, Y[4] = {a.y, a.w, b.y, b.w};
#pragma unroll
            for (int q = 0; q < 4; q++) X[q] = clamp_rs(X[q], 0.0f, visf) * WG_LANE_W + WG_LANE_W * 0.5f;   // to_x (:847-850)
            const float t = (float)jj * WG_TESS_DT;
            const float s = 1.0f - t;
            const float px = s * s * s * X[0] + 3.0f * s * s * t * X[1] + 3.0f * s * t * t * X[2] + t * t * t * X[3];
            const float py = s * s * s * Y[0] + 3.0f * s * s * t * Y[1] + 3.0f * s * t * t * Y[2] + t * t * t * Y[3];
            const float dx = 3.0f * s * s * (X[1] - X[0]) + 6.0f * s * t * (X[2] - X[1]) + 3.0f * t * t * (X[3] - X[2]);
            const float dy = 3.0f * s * s * (Y[1] - Y[0]) + 6.0f * s * t * (Y[2] - Y[1]) + 3.0f * t * t * (Y[3] - Y[2]);
            const float len = sqrtf(dx * dx + dy * dy);
            float nx, ny;
            if (len > 0.0f) { nx = -dy / len; ny = dx / len; } else { nx = 1.0f; ny = 0.0f; }
            if (rside) { x = px - hw * nx; y = py - hw * ny; }
            else       { x = px + hw * nx; y = py + hw * ny; }
            col = curve_color[k];
        } else if ((l -= 96u * ri.nc) < (uint32_t)WG_VTX_PER_NODE) {
            const uint32_t tri = l / 3u, corner = l % 3u;
            const float r = WG_NODE_RADIUS;
            if (corner == 0) { x = ri.cx; y = ri.ny; }
            else {
                const uint32_t q = tri + corner - 1u;
                x = ri.cx + r * c_cos[q];
                y = ri.ny + r * c_sin[q];
            }
            col = ri.ncol;
        } else {
            l -= WG_VTX_PER_NODE;
            const uint32_t q = l / 6u, corner = l % 6u;
            const float ri_ = WG_NODE_RADIUS - WG_SELECTED_RING_WIDTH * 0.5f;
            const float ro = WG_NODE_RADIUS + WG_SELECTED_RING_WIDTH * 0.5f;
            // o0 i0 o1 i0 i1 o1
            const bool inner = corner == 1 || corner == 3 || corner == 4;
            const uint32_t qq = q + ((corner == 2 || corner == 4 || corner == 5) ? 1u : 0u);
            const float rad = inner ? ri_ : ro;
            x = ri.cx + rad * c_cos[qq];
            y = ri.ny + rad * c_sin[qq];
            col = WG_COLOR_FOREGROUND;
        }
        const float4 c4 = pal[col & 7u];
        float *o = stage + (v - v0) * 6;
        o[0] = x; o[1] = y; o[2] = c4.x; o[3] = c4.y; o[4] = c4.z; o[5] = c4.w;
    }
    __syncthreads();
    // contiguous write-out: tile start is 16-byte aligned (TILE * 24 = 36864)
    const uint64_t nfl = (v1 - v0) * 6;
    const uint64_t n4 = nfl / 4;
    float4 *dst = reinterpret_cast<float4 *>(out + v0 * 6);
    const float4 *src = reinterpret_cast<const float4 *>(stage);
    for (uint64_t i = threadIdx.x; i < n4; i += VT) dst[i] = src[i];
    if (threadIdx.x == 0 && (nfl & 3)) {
        float2 *d2 = reinterpret_cast<float2 *>(out + v0 * 6 + n4 * 4);
        *d2 = make_float2(stage[n4 * 4], stage[n4 * 4 + 1]);
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
    WG_ALLOC(c, c->vtx_off, (rows + 2) * 8);
    WG_ALLOC(c, c->scan_tmp, wg_scan_tmp_bytes(rows + 2));
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
    hipLaunchKernelGGL(k_vtx_counts, dim3((rows + 255) / 256), dim3(256), 0, s, rb, re, sel,
                       c->vert_off.as<const uint32_t>(), c->curve_off.as<const uint32_t>(), off);
    WG_HIP(c, wg_exclusive_scan_u64(off, off, rows, c->scan_tmp.p, s));
    uint64_t total = 0;
    WG_HIP(c, hipMemcpyAsync(&total, off + rows, 8, hipMemcpyDeviceToHost, s));
    WG_HIP(c, hipStreamSynchronize(s));
    wg_stage_end(c);
    c->n_vtx = total;
    WG_ALLOC(c, c->vtx, total * sizeof(wg_vertex) + 64);
    float q = roundf(c->graph_width / WG_LANE_W);
    uint32_t vis = q <= 0.0f ? 0u : (uint32_t)q;
    if (vis < 1) vis = 1;
    const uint64_t ntiles = (total + TILE - 1) / TILE;
    wg_stage_begin(c, "vtx_emit");
    hipLaunchKernelGGL(k_vtx_tiles, dim3(ntiles), dim3(VT), 0, s, rb, re, total, sel, vis, (const uint64_t *)off,
                       c->vert_off.as<const uint32_t>(), c->vert.as<const uint32_t>(), c->curve_off.as<const uint32_t>(),
                       c->curve.as<const wg_curve>(), c->curve_color.as<const uint8_t>(), c->g_height.as<const float>(),
                       c->g_node_y.as<const float>(), c->lane_out.as<const uint32_t>(), c->color_out.as<const uint8_t>(),
                       c->palette.as<const float4>(), c->vtx.as<float>());
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}

int wg_vertex_checksum_run(wg_ctx *c, uint64_t *out) {
    WG_ALLOC(c, c->chk, 64);
    WG_HIP(c, hipMemsetAsync(c->chk.p, 0, 8, c->stream));
    const uint64_t nw = c->n_vtx * 6;
    if (nw) {
        uint64_t b = (nw + 255) / 256;
        if (b > 4096) b = 4096;
        hipLaunchKernelGGL(k_checksum, dim3(b), dim3(256), 0, c->stream, c->vtx.as<const uint32_t>(), nw,
                           c->chk.as<unsigned long long>());
        WG_HIP(c, hipGetLastError());
    }
    uint64_t v = 0;
    WG_HIP(c, hipMemcpyAsync(&v, c->chk.p, 8, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    *out = v;
    return WG_OK;
}
