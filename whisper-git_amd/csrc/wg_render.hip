// wg_render.hip — the consumer adapter: the emitted
// SplineVertex / TextVertex buffers rasterised into an RGBA8 image, and a PNG
// writer, closing the loop with the reference's headless screenshot mode
// (screenshot_mode.rs:101-141: build, prepare, render into an offscreen
// image cleared to the theme colour, capture, save PNG).  The reference's
// rasteriser is aetna-vulkano's Vulkan pipeline (absent third-party code), so
// the engine freezes its own rules, WG-RAST-1:
//   * rows in order; per row its graph triangles (vertex buffer order), then
//     its glyph quads (two triangles each); painter's order, "over" blending
//     dst = src * a + dst * (1 - a) in f32 onto an opaque clear colour;
//   * screen position X = (x + dx) * scale, Y = (y + Yr) * scale with
//     Yr = (row_top[r] - row_top[top_row]) + origin_y (dx = graph_x for graph
//     vertices, 0 for glyphs);
//   * one sample at the pixel centre, considered when inside the triangle's
//     closed f32 bounding box; edge functions E(a, b, p) = (b.x - a.x) *
//     (p.y - a.y) - (b.y - a.y) * (p.x - a.x); zero-area triangles skipped,
//     negative ones re-oriented; a pixel is covered when every edge has E > 0
//     or E == 0 and owns the edge (b.y < a.y, or b.y == a.y and b.x > a.x);
//   * graph triangles: flat colour of their first vertex; glyph triangles:
//     barycentric UV ((w0 u0 + w1 u1) + w2 u2) / area, bilinear SDF sample
//     d (texel centres, clamped), alpha = a * clamp((d - 0.5) * k + 0.5, 0, 1)
//     with k = 2 * spread * (text_px / em_px) * scale;
//   * output byte = floor(clamp(v, 0, 1) * 255 + 0.5), alpha 255.
//
// GPU: one 256-thread workgroup per 16x16 tile, one pixel per thread.  Rows
// are y-ordered, so a tile finds the rows that can touch it by binary search
// over row_top widened by the largest overshoot of any row's triangles past
// its own strip (one reduction pass); their triangles are staged in LDS 256
// at a time and every pixel walks them in order, keeping its colour in
// registers.
#include "wg_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace {

constexpr int TS = 16;            // tile side
constexpr int RT = TS * TS;       // threads per tile = pixels
constexpr int CH = RT;            // triangles staged per round

struct RenderArgs {
    uint32_t W, H;
    float scale, graph_x, origin_y;
    float bg[3];
    uint64_t top_ctx;             // context row of top_row
    const float *row_top;         // context rows
    // graph layer: rows [g_rb, g_re) (context), vertex offsets relative to g_rb
    uint64_t g_rb, g_re;
    const uint64_t *g_off;
    const float4 *g_vtx;          // wg_vertex pairs as float4 triples
    // text layer
    uint64_t t_rb, t_re;
    const uint64_t *t_off;        // quad offsets relative to t_rb
    const float4 *t_vtx;          // wg_text_vertex = 2 float4
    const uint8_t *sdf;
    uint32_t aw, ah;
    float k;
    const float *margin;          // [0]: largest overshoot (row-local px), [1] != 0: row_top not monotonic
};

__device__ __forceinline__ float edge(float ax, float ay, float bx, float by, float px, float py) {
    return (bx - ax) * (py - ay) - (by - ay) * (px - ax);
}
__device__ __forceinline__ bool owns(float ax, float ay, float bx, float by) {
    return by < ay || (by == ay && bx > ax);
}

// rows [lo, hi) (context) of the active layers: the largest extent of any
// row's vertices outside [0, height] (row-local), and whether row_top fails to
// be non-decreasing over them (then tiles walk every row)
__global__ void k_row_overshoot(RenderArgs A, uint64_t lo, uint64_t hi, const float *__restrict__ height,
                                float *__restrict__ margin) {
    const uint64_t r = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= hi) return;
    float m = 0.0f;
    const float h = height[r];
    if (A.g_vtx && r >= A.g_rb && r < A.g_re) {
        const float *v = reinterpret_cast<const float *>(A.g_vtx);
        for (uint64_t i = A.g_off[r - A.g_rb]; i < A.g_off[r - A.g_rb + 1]; i++) {
            const float y = v[i * 6 + 1];
            m = fmaxf(m, fmaxf(-y, y - h));
        }
    }
    if (A.t_vtx && r >= A.t_rb && r < A.t_re) {
        const float *v = reinterpret_cast<const float *>(A.t_vtx);
        for (uint64_t i = A.t_off[r - A.t_rb] * 6; i < A.t_off[r - A.t_rb + 1] * 6; i++) {
            const float y = v[i * 8 + 1];
            m = fmaxf(m, fmaxf(-y, y - h));
        }
    }
    if (m > 0.0f) atomicMax(reinterpret_cast<unsigned int *>(margin), __float_as_uint(m));   // non-negative floats order as ints
    if (!(A.row_top[r + 1] >= A.row_top[r])) reinterpret_cast<unsigned int *>(margin)[1] = 1u;
}

struct Tri {
    float x[3], y[3];
    float area;
    float r, g, b, a;
    float u[3], v[3];
    float minx, maxx, miny, maxy;
    uint32_t text;
};

__global__ __launch_bounds__(RT) void k_raster(RenderArgs A, uint8_t *__restrict__ out) {
    __shared__ Tri tri[CH];
    __shared__ uint64_t s_rows[2];
    const uint32_t tx0 = blockIdx.x * TS, ty0 = blockIdx.y * TS;
    const uint32_t px = tx0 + (threadIdx.x % TS), py = ty0 + (threadIdx.x / TS);
    const float cx = (float)px + 0.5f, cy = (float)py + 0.5f;
    float cr = A.bg[0], cg = A.bg[1], cb = A.bg[2];
    // rows whose strip, widened by the margin, meets the tile's y span (content px)
    uint64_t lo2 = ~0ull, hi = 0;   // rows of the active layers
    if (A.g_vtx) { lo2 = A.g_rb; hi = A.g_re; }
    if (A.t_vtx) { lo2 = A.t_rb < lo2 ? A.t_rb : lo2; hi = A.t_re > hi ? A.t_re : hi; }
    if (lo2 > hi) lo2 = hi;
    if (threadIdx.x == 0) {
        // the same f32 expression as the triangles' row offset Yr
        auto yl = [&](uint64_t r) { return (A.row_top[r] - A.row_top[A.top_ctx]) + A.origin_y; };
        // slack: 1 px plus a few f32 ulps of the row_top magnitudes involved
        const float mag = fmaxf(fmaxf(fabsf(A.row_top[lo2]), fabsf(A.row_top[hi])), fabsf(A.row_top[A.top_ctx])) +
                          fabsf(A.origin_y);
        const float m = A.margin[0] + 1.0f + mag * 1.0e-6f;
        const float ya = (float)ty0 / A.scale - m, yb = (float)(ty0 + TS) / A.scale + m;
        uint64_t a = lo2, c = hi;
        if (!__float_as_uint(A.margin[1])) {   // row_top is non-decreasing: binary searches
            uint64_t b = hi;   // first row whose strip bottom reaches ya
            while (a < b) { const uint64_t mid = (a + b) >> 1; if (yl(mid + 1) < ya) a = mid + 1; else b = mid; }
            c = a;
            uint64_t d = hi;   // first row whose strip top is below yb
            while (c < d) { const uint64_t mid = (c + d) >> 1; if (yl(mid) <= yb) c = mid + 1; else d = mid; }
        }
        s_rows[0] = a;
        s_rows[1] = c;
    }
    __syncthreads();
    const uint64_t r0 = s_rows[0], r1 = s_rows[1];
    for (uint64_t r = r0; r < r1; r++) {
        const float Yr = (A.row_top[r] - A.row_top[A.top_ctx]) + A.origin_y;
        for (int layer = 0; layer < 2; layer++) {
            uint64_t t0 = 0, t1 = 0;
            if (layer == 0 && A.g_vtx && r >= A.g_rb && r < A.g_re) {
                t0 = A.g_off[r - A.g_rb] / 3; t1 = A.g_off[r - A.g_rb + 1] / 3;
            } else if (layer == 1 && A.t_vtx && r >= A.t_rb && r < A.t_re) {
                t0 = A.t_off[r - A.t_rb] * 2; t1 = A.t_off[r - A.t_rb + 1] * 2;
            }
            for (uint64_t c0 = t0; c0 < t1; c0 += CH) {
                const uint64_t n = (t1 - c0) < (uint64_t)CH ? (t1 - c0) : (uint64_t)CH;
                __syncthreads();   // the previous round's readers are done
                if (threadIdx.x < n) {
                    Tri T;
                    const uint64_t t = c0 + threadIdx.x;
                    T.text = layer;
                    for (int k = 0; k < 3; k++) {
                        float x, y;
                        if (layer == 0) {
                            const float *v = reinterpret_cast<const float *>(A.g_vtx) + (t * 3 + k) * 6;
                            x = (v[0] + A.graph_x) * A.scale;
                            y = (v[1] + Yr) * A.scale;
                            if (k == 0) { T.r = v[2]; T.g = v[3]; T.b = v[4]; T.a = v[5]; }
                            T.u[k] = T.v[k] = 0.0f;
                        } else {
                            const float *v = reinterpret_cast<const float *>(A.t_vtx) + (t * 3 + k) * 8;
                            x = v[0] * A.scale;
                            y = (v[1] + Yr) * A.scale;
                            T.u[k] = v[2];
                            T.v[k] = v[3];
                            if (k == 0) { T.r = v[4]; T.g = v[5]; T.b = v[6]; T.a = v[7]; }
                        }
                        T.x[k] = x;
                        T.y[k] = y;
                    }
                    T.area = edge(T.x[0], T.y[0], T.x[1], T.y[1], T.x[2], T.y[2]);
                    if (T.area < 0.0f) {   // re-orient: swap vertices 1 and 2
                        float s;
                        s = T.x[1]; T.x[1] = T.x[2]; T.x[2] = s;
                        s = T.y[1]; T.y[1] = T.y[2]; T.y[2] = s;
                        s = T.u[1]; T.u[1] = T.u[2]; T.u[2] = s;
                        s = T.v[1]; T.v[1] = T.v[2]; T.v[2] = s;
                        T.area = -T.area;
                    }
                    T.minx = fminf(fminf(T.x[0], T.x[1]), T.x[2]);
                    T.maxx = fmaxf(fmaxf(T.x[0], T.x[1]), T.x[2]);
                    T.miny = fminf(fminf(T.y[0], T.y[1]), T.y[2]);
                    T.maxy = fmaxf(fmaxf(T.y[0], T.y[1]), T.y[2]);
                    tri[threadIdx.x] = T;
                }
                __syncthreads();
                if (px < A.W && py < A.H) {
                    for (uint32_t i = 0; i < n; i++) {
                        const Tri &T = tri[i];
                        if (!(T.area > 0.0f)) continue;
                        if (!(cx >= T.minx && cx <= T.maxx && cy >= T.miny && cy <= T.maxy)) continue;
                        const float w0 = edge(T.x[1], T.y[1], T.x[2], T.y[2], cx, cy);
                        const float w1 = edge(T.x[2], T.y[2], T.x[0], T.y[0], cx, cy);
                        const float w2 = edge(T.x[0], T.y[0], T.x[1], T.y[1], cx, cy);
                        const bool in0 = w0 > 0.0f || (w0 == 0.0f && owns(T.x[1], T.y[1], T.x[2], T.y[2]));
                        const bool in1 = w1 > 0.0f || (w1 == 0.0f && owns(T.x[2], T.y[2], T.x[0], T.y[0]));
                        const bool in2 = w2 > 0.0f || (w2 == 0.0f && owns(T.x[0], T.y[0], T.x[1], T.y[1]));
                        if (!(in0 && in1 && in2)) continue;
                        float sa = T.a;
                        if (T.text) {
                            const float u = ((w0 * T.u[0] + w1 * T.u[1]) + w2 * T.u[2]) / T.area;
                            const float v = ((w0 * T.v[0] + w1 * T.v[1]) + w2 * T.v[2]) / T.area;
                            const float fx = u * (float)A.aw - 0.5f, fy = v * (float)A.ah - 0.5f;
                            const float x0f = floorf(fx), y0f = floorf(fy);
                            const float ax = fx - x0f, ay = fy - y0f;
                            const int ix = (int)x0f, iy = (int)y0f;
                            const int xa = min(max(ix, 0), (int)A.aw - 1), xb = min(max(ix + 1, 0), (int)A.aw - 1);
                            const int ya = min(max(iy, 0), (int)A.ah - 1), yb = min(max(iy + 1, 0), (int)A.ah - 1);
                            const float inv = 1.0f / 255.0f;
                            const float s00 = (float)A.sdf[ya * A.aw + xa] * inv, s10 = (float)A.sdf[ya * A.aw + xb] * inv;
                            const float s01 = (float)A.sdf[yb * A.aw + xa] * inv, s11 = (float)A.sdf[yb * A.aw + xb] * inv;
                            const float top = s00 + (s10 - s00) * ax, bot = s01 + (s11 - s01) * ax;
                            const float d = top + (bot - top) * ay;
                            float al = (d - 0.5f) * A.k + 0.5f;
                            al = al < 0.0f ? 0.0f : (al > 1.0f ? 1.0f : al);
                            sa = sa * al;
                        }
                        const float ia = 1.0f - sa;
                        cr = T.r * sa + cr * ia;
                        cg = T.g * sa + cg * ia;
                        cb = T.b * sa + cb * ia;
                    }
                }
            }
        }
    }
    if (px < A.W && py < A.H) {
        auto q = [](float v) { v = v < 0.0f ? 0.0f : (v > 1.0f ? 1.0f : v); return (uint8_t)floorf(v * 255.0f + 0.5f); };
        uchar4 o = make_uchar4(q(cr), q(cg), q(cb), 255);
        reinterpret_cast<uchar4 *>(out)[(uint64_t)py * A.W + px] = o;
    }
}

// ---- PNG (stored deflate blocks; no compression library) ---------------------------
uint32_t crc_table[256];
bool crc_ready = false;
void crc_init() {
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_table[n] = c;
    }
    crc_ready = true;
}
uint32_t crc_update(uint32_t crc, const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) crc = crc_table[(crc ^ p[i]) & 0xFF] ^ (crc >> 8);
    return crc;
}
void put32(std::vector<uint8_t> &v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16)); v.push_back((uint8_t)(x >> 8)); v.push_back((uint8_t)x);
}
void chunk(std::vector<uint8_t> &out, const char *type, const std::vector<uint8_t> &data) {
    put32(out, (uint32_t)data.size());
    const size_t at = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    const uint32_t crc = crc_update(0xFFFFFFFFu, out.data() + at, data.size() + 4) ^ 0xFFFFFFFFu;
    put32(out, crc);
}

}  // namespace

extern "C" {

int wg_render(wg_ctx *c, const wg_render_params *p, uint8_t *rgba, int32_t out_residency) {
    if (!c || !p || !rgba) return WG_E_INVALID;
    WG_SETTLE(c);
    if (out_residency != WG_HOST && out_residency != WG_DEVICE) return wg_fail(c, WG_E_INVALID, "bad residency");
    if (!p->width || !p->height || p->width > 16384 || p->height > 16384)
        return wg_fail(c, WG_E_INVALID, "image %ux%u outside 1..16384", p->width, p->height);
    if (!(p->scale > 0.0f)) return wg_fail(c, WG_E_INVALID, "scale must be positive");
    if (!c->have_geom) return wg_fail(c, WG_E_STATE, "no geometry");
    const bool g = p->layers & WG_RENDER_GRAPH, t = p->layers & WG_RENDER_TEXT;
    if (g && !c->have_vtx) return wg_fail(c, WG_E_STATE, "no vertices emitted");
    if (t && !c->have_text) return wg_fail(c, WG_E_STATE, "no glyphs emitted");
    const ShardState &S = c->sh;
    if (p->top_row < S.s || p->top_row > S.e) return wg_fail(c, WG_E_INVALID, "top_row outside the built rows");
    (void)hipSetDevice(c->device);
    hipStream_t s = c->stream;
    const uint64_t b = S.row_base;   // global row -> context row: r - s + b
    RenderArgs A{};
    A.W = p->width;
    A.H = p->height;
    A.scale = p->scale;
    A.graph_x = p->graph_x;
    A.origin_y = p->origin_y;
    for (int i = 0; i < 3; i++) A.bg[i] = p->clear[i];
    A.top_ctx = p->top_row - S.s + b;
    A.row_top = c->g_row_top.as<const float>();
    if (g) {
        A.g_rb = c->vrow_begin - S.s + b;
        A.g_re = c->vrow_end - S.s + b;
        A.g_off = c->vtx_off.as<const uint64_t>();
        A.g_vtx = c->vtx.as<const float4>();
    }
    if (t) {
        const FontSlot &F = c->fonts[c->text_slot];
        A.t_rb = c->text_rb - S.s + b;
        A.t_re = c->text_re - S.s + b;
        A.t_off = c->text_off.as<const uint64_t>();
        A.t_vtx = c->text_vtx.as<const float4>();
        A.sdf = F.sdf.as<const uint8_t>();
        A.aw = F.W;
        A.ah = F.H;
        A.k = 2.0f * (float)F.spread * c->text_scale * p->scale;
    }
    if (!g && !t) { A.g_rb = A.g_re = A.t_rb = A.t_re = A.top_ctx; }
    WG_ALLOC(c, c->render_small, 64);
    WG_HIP(c, hipMemsetAsync(c->render_small.p, 0, 8, s));
    A.margin = c->render_small.as<const float>();
    const uint64_t npx = (uint64_t)p->width * p->height;
    uint8_t *dst = rgba;
    if (out_residency == WG_HOST) {
        WG_ALLOC(c, c->render_img, npx * 4);
        dst = c->render_img.as<uint8_t>();
    }
    wg_stage_begin(c, "render");
    uint64_t lo = ~0ull, hi = 0;   // rows of the active layers (context)
    if (g) { lo = A.g_rb; hi = A.g_re; }
    if (t) { lo = std::min(lo, A.t_rb); hi = std::max(hi, A.t_re); }
    if (hi > lo) {
        RenderArgs B = A;
        if (!g) B.g_vtx = nullptr;
        hipLaunchKernelGGL(k_row_overshoot, dim3((uint32_t)((hi - lo + 255) / 256)), dim3(256), 0, s, B, lo, hi,
                           c->g_height.as<const float>(), c->render_small.as<float>());
    }
    if (!g) A.g_vtx = nullptr;
    hipLaunchKernelGGL(k_raster, dim3((p->width + TS - 1) / TS, (p->height + TS - 1) / TS), dim3(RT), 0, s, A, dst);
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    if (out_residency == WG_HOST) WG_HIP(c, hipMemcpyAsync(rgba, dst, npx * 4, hipMemcpyDeviceToHost, s));
    WG_HIP(c, hipStreamSynchronize(s));
    return WG_OK;
}

int wg_write_png(const char *path, const uint8_t *rgba, uint32_t width, uint32_t height) {
    if (!path || !rgba || !width || !height) return WG_E_INVALID;
    if (!crc_ready) crc_init();
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::vector<uint8_t> ihdr;
    put32(ihdr, width);
    put32(ihdr, height);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});   // 8-bit RGBA, deflate, no filter method extras, no interlace
    chunk(png, "IHDR", ihdr);
    // zlib stream of stored blocks over the scanlines (filter byte 0 each)
    const size_t line = (size_t)width * 4 + 1, raw_n = line * height;
    std::vector<uint8_t> z = {0x78, 0x01};
    uint32_t a1 = 1, a2 = 0;   // Adler-32
    size_t done = 0;
    std::vector<uint8_t> raw(raw_n);
    for (uint32_t y = 0; y < height; y++) {
        raw[y * line] = 0;
        std::memcpy(&raw[y * line + 1], rgba + (size_t)y * width * 4, (size_t)width * 4);
    }
    while (done < raw_n || raw_n == 0) {
        const size_t n = std::min<size_t>(65535, raw_n - done);
        const bool last = done + n == raw_n;
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)(n & 0xFF)); z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)(~n & 0xFF)); z.push_back((uint8_t)((~n >> 8) & 0xFF));
        z.insert(z.end(), raw.begin() + done, raw.begin() + done + n);
        for (size_t i = done; i < done + n; i++) { a1 = (a1 + raw[i]) % 65521u; a2 = (a2 + a1) % 65521u; }
        done += n;
        if (last) break;
    }
    put32(z, (a2 << 16) | a1);
    chunk(png, "IDAT", z);
    chunk(png, "IEND", {});
    FILE *f = std::fopen(path, "wb");
    if (!f) return WG_E_INVALID;
    const size_t w = std::fwrite(png.data(), 1, png.size(), f);
    std::fclose(f);
    return w == png.size() ? WG_OK : WG_E_INVALID;
}

}  // extern "C"
