// wg_font.hip — SDF font atlas (frozen spec WG-SDF-1 in
// DESIGN.md §5b).
//
// The reference's legacy text path (docs/render_engine.md:105-131: Roboto
// Regular/Bold, ASCII 32-126 rasterised by fontdue at 2x oversampling, a
// custom EDT turning coverage into an R8 SDF atlas with per-glyph advance,
// bearing and UV) is absent from the snapshot, and fontdue is not vendored,
// so the engine freezes its own pipeline:
//   host     TrueType parse (head/hhea/maxp/cmap fmt 4/hmtx/loca/glyf incl.
//            offset composites), quadratic contours flattened into 8 lines
//            each, scaled to atlas pixels, glyph cells shelf-packed
//   k_font_coverage   one workgroup per (glyph, 8-row band), the band's edges
//            compacted into LDS: every cell pixel counts which of its 4x4
//            sample points lie inside the outline (non-zero winding) ->
//            coverage 0..16; inside = coverage >= 8
//   k_edt_cols        pass 1, one lane per column of a 64 x 64 tile staged in
//                     LDS with R rows above and below: one sweep down, one up
//            outward: squared vertical distance to the nearest pixel of the
//            other class
//   k_edt_rows        pass 2, one workgroup per row staged in LDS: squared
//            distance = min over q of g(q) + (x-q)^2, scanned outward with an
//            early exit; exact for distances <= R = 4 * spread, "far" beyond
//            (the SDF saturates at `spread`)
//            -> SDF byte: 127.5 - (d_out - d_in) * 127.5 / spread, clamped
// All arithmetic is integer or exact f32 (dyadic sample offsets, correctly
// rounded division/sqrt), so the oracle (oracle/font_oracle.py, fontTools +
// numpy) reproduces every byte; its EDT is pinned against scipy's exact EDT.
#include <cmath>
#include <cstring>
#include <vector>

#include "wg_internal.h"

namespace {

constexpr int QUAD_STEPS = 8;          // lines per quadratic segment
constexpr int COV_T = 256;

struct GlyphDesc {          // per glyph, device
    uint32_t edge_off, n_edges;
    int32_t bx0, by1;       // bitmap box: left x, top y (y up), atlas pixels
    uint32_t cw, ch;        // cell size (bitmap + 2 * spread)
    uint32_t ax, ay;        // cell origin in the atlas
};

// ---- pass 0: coverage -----------------------------------------------------------
// grid = (glyph, band of BAND cell rows): the band's edges are compacted into
// LDS first (winding sums are integer, so their order does not matter), then
// every pixel of the band tests only those.
constexpr int BAND = 8;
constexpr int BAND_EDGES = 1024;

__global__ void __launch_bounds__(COV_T) k_font_coverage(const GlyphDesc *__restrict__ gd, const float4 *__restrict__ edges,
                                                         uint32_t spread, uint32_t W, uint8_t *__restrict__ cov) {
    __shared__ float4 se[BAND_EDGES];
    __shared__ uint32_t s_n;
    const GlyphDesc g = gd[blockIdx.x];
    const uint32_t cj0 = blockIdx.y * BAND;
    if (cj0 >= g.ch) return;
    const uint32_t cj1 = cj0 + BAND < g.ch ? cj0 + BAND : g.ch;
    // sample rows of the band lie in (ybot, ytop)
    const float ytop = (float)(g.by1 - ((int32_t)cj0 - (int32_t)spread));
    const float ybot = (float)(g.by1 - ((int32_t)cj1 - (int32_t)spread));
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const float4 *E = edges + g.edge_off;
    for (uint32_t i = threadIdx.x; i < g.n_edges; i += COV_T) {
        const float4 e = E[i];
        const float ylo = e.y < e.w ? e.y : e.w, yhi = e.y < e.w ? e.w : e.y;
        if (yhi > ybot && ylo < ytop) {
            const uint32_t k = atomicAdd(&s_n, 1u);
            if (k < (uint32_t)BAND_EDGES) se[k] = e;
        }
    }
    __syncthreads();
    const uint32_t ne = s_n;
    const float4 *B = se;
    if (ne > (uint32_t)BAND_EDGES) { B = E; }   // too many for LDS: test every edge of the glyph
    const uint32_t nb = ne > (uint32_t)BAND_EDGES ? g.n_edges : ne;
    const float off[4] = {0.125f, 0.375f, 0.625f, 0.875f};
    const uint32_t npx = g.cw * (cj1 - cj0);
    for (uint32_t p = threadIdx.x; p < npx; p += COV_T) {
        const uint32_t ci = p % g.cw, cj = cj0 + p / g.cw;
        const int32_t i = (int32_t)ci - (int32_t)spread, j = (int32_t)cj - (int32_t)spread;
        const float px = (float)(g.bx0 + i), py = (float)(g.by1 - j);
        int wind[16];
#pragma unroll
        for (int q = 0; q < 16; q++) wind[q] = 0;
        for (uint32_t k = 0; k < nb; k++) {
            const float4 e = B[k];   // (x0, y0, x1, y1), y up
            const bool up = e.y < e.w;
            const float ylo = up ? e.y : e.w, yhi = up ? e.w : e.y;
            if (py - 0.125f < ylo || py - 0.875f >= yhi) continue;   // no sample row of this pixel in [ylo, yhi)
#pragma unroll
            for (int sy = 0; sy < 4; sy++) {
                const float y = py - off[sy];
                if (!(ylo <= y && y < yhi)) continue;
                const float t = (y - e.y) / (e.w - e.y);
                const float xi = e.x + t * (e.z - e.x);
#pragma unroll
                for (int sx = 0; sx < 4; sx++) {
                    const float x = px + off[sx];
                    if (xi > x) wind[sy * 4 + sx] += up ? 1 : -1;
                }
            }
        }
        uint32_t k = 0;
#pragma unroll
        for (int q = 0; q < 16; q++) k += wind[q] != 0;
        cov[(uint64_t)(g.ay + cj) * W + g.ax + ci] = (uint8_t)k;
    }
}

// ---- pass 1: columns ---------------------------------------------------------------
// gin[y][x]  = (vertical distance from an inside pixel to the nearest outside pixel)^2
// gout[y][x] = (vertical distance from an outside pixel to the nearest inside pixel)^2
// 0 on the pixel's own class; capped at (R + 1)^2.  One thread per pixel
// scanning its column outward (coalesced across x), exit at the first hit.
// One wave per 64 x 64 pixel tile: the tile's columns plus R rows above and
// below are staged in LDS (1 = inside, 0 = outside, 2 = past the atlas),
// then each lane sweeps its column down and up once, keeping the last row
// of either class seen: a pixel's nearest pixel of the other class above
// (below) is the last (next) row of that class, so d = min of the two
// distances, capped at R + 1 — the same value as scanning k = 1..R.
constexpr uint32_t EC_TX = 64, EC_TY = 64, EC_RMAX = 240;   // R = 4 * spread, spread <= 60
__global__ void __launch_bounds__(64) k_edt_cols(const uint8_t *__restrict__ cov, uint32_t W, uint32_t H, uint32_t R,
                                                uint16_t *__restrict__ gin, uint16_t *__restrict__ gout) {
    __shared__ __attribute__((aligned(16))) uint8_t t[(EC_TY + 2 * EC_RMAX) * EC_TX];
    __shared__ uint16_t dup[EC_TY * EC_TX];
    const uint32_t x0 = blockIdx.x * EC_TX, y0 = blockIdx.y * EC_TY;
    const uint32_t rows = EC_TY + 2 * R;
    const uint32_t c = threadIdx.x, x = x0 + c;
    if ((W & 15u) == 0 && x0 + EC_TX <= W) {
        // 16-byte loads, 16 rows per wave instruction, all of them in flight
        const uint32_t q = c & 3u, rsub = c >> 2;   // 4 lanes per 64-byte row, 16 rows per round
        for (uint32_t lr0 = 0; lr0 < rows; lr0 += 16) {
            const uint32_t lr = lr0 + rsub;
            const int64_t y = (int64_t)y0 + (int64_t)lr - (int64_t)R;
            uint4 v = make_uint4(0x02020202u, 0x02020202u, 0x02020202u, 0x02020202u);
            if (lr < rows && y >= 0 && y < (int64_t)H) {
                const uint4 w = *reinterpret_cast<const uint4 *>(cov + (uint64_t)y * W + x0 + 16 * q);
                auto cls = [](uint32_t b) {   // byte-wise (b >= 8) ? 1 : 0
                    uint32_t r = 0;
#pragma unroll
                    for (int k = 0; k < 4; k++) r |= (((b >> (8 * k)) & 0xFFu) >= 8u ? 1u : 0u) << (8 * k);
                    return r;
                };
                v = make_uint4(cls(w.x), cls(w.y), cls(w.z), cls(w.w));
            }
            if (lr < rows) *reinterpret_cast<uint4 *>(t + lr * EC_TX + 16 * q) = v;
        }
        __syncthreads();   // (rows were staged by other lanes)
    } else {
        for (uint32_t lr = 0; lr < rows; lr++) {
            const int64_t y = (int64_t)y0 + (int64_t)lr - (int64_t)R;
            t[lr * EC_TX + c] = (y < 0 || y >= (int64_t)H || x >= W) ? 2u : (cov[(uint64_t)y * W + x] >= 8 ? 1u : 0u);
        }
    }
    // (below, each lane reads only its own column)
    const int32_t far = (int32_t)R + 1;
    int32_t last[2] = {-1000000, -1000000};   // staged row of the last pixel of class 0 / 1 above
    for (uint32_t lr = 0; lr < R + EC_TY; lr++) {
        const uint32_t v = t[lr * EC_TX + c];
        if (lr >= R) {
            const int32_t du = (v < 2u) ? (int32_t)lr - last[v ^ 1u] : far;
            dup[(lr - R) * EC_TX + c] = (uint16_t)(du < far ? du : far);
        }
        if (v < 2u) last[v] = (int32_t)lr;
    }
    int32_t next[2] = {1000000, 1000000};     // ... and below
    for (int32_t lr = (int32_t)rows - 1; lr >= (int32_t)R; lr--) {
        const uint32_t v = t[lr * EC_TX + c];
        if (lr < (int32_t)(R + EC_TY)) {
            const uint32_t ly = (uint32_t)lr - R, y = y0 + ly;
            if (x < W && y < H) {
                const int32_t dd = next[v ^ 1u] - lr;
                int32_t d = dup[ly * EC_TX + c];
                d = dd < d ? dd : d;
                const uint64_t o = (uint64_t)y * W + x;
                gin[o] = (uint16_t)(v ? d * d : 0);
                gout[o] = (uint16_t)(v ? 0 : d * d);
            }
        }
        if (v < 2u) next[v] = lr;
    }
}

// ---- pass 2: rows -> squared distances and the SDF byte -------------------------------
constexpr int ROW_T = 256;
constexpr int ROW_MAX = 4096;

__device__ __forceinline__ uint32_t row_min(const uint16_t *g, int32_t x, int32_t W, uint32_t R) {
    const uint32_t cap = (R + 1) * (R + 1);
    uint32_t best = g[x];
    for (uint32_t o = 1; o <= R && o * o < best; o++) {
        const uint32_t oo = o * o;
        if (x - (int32_t)o >= 0) { const uint32_t v = g[x - o] + oo; best = v < best ? v : best; }
        if (x + (int32_t)o < W) { const uint32_t v = g[x + o] + oo; best = v < best ? v : best; }
    }
    return best < cap ? best : cap;
}

__global__ void __launch_bounds__(ROW_T) k_edt_rows(const uint16_t *__restrict__ gin, const uint16_t *__restrict__ gout,
                                                    uint32_t W, uint32_t R, float spread, uint16_t *__restrict__ d2in,
                                                    uint16_t *__restrict__ d2out, uint8_t *__restrict__ sdf) {
    __shared__ uint16_t si[ROW_MAX], so[ROW_MAX];
    const uint64_t y = blockIdx.x;
    for (uint32_t x = threadIdx.x; x < W; x += ROW_T) {
        si[x] = gin[y * W + x];
        so[x] = gout[y * W + x];
    }
    __syncthreads();
    const float k = 127.5f / spread;
    for (uint32_t x = threadIdx.x; x < W; x += ROW_T) {
        const uint32_t a = row_min(si, (int32_t)x, (int32_t)W, R), b = row_min(so, (int32_t)x, (int32_t)W, R);
        if (d2in) d2in[y * W + x] = (uint16_t)a;
        if (d2out) d2out[y * W + x] = (uint16_t)b;
        const float signed_d = sqrtf((float)b) - sqrtf((float)a);   // > 0 outside
        float v = 127.5f - signed_d * k;
        v = v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v);
        sdf[y * W + x] = (uint8_t)floorf(v + 0.5f);
    }
}

// ---- TrueType (host) ---------------------------------------------------------------------
struct Reader {
    const uint8_t *p;
    uint64_t n;
    bool ok = true;
    uint32_t u8(uint64_t o) { if (o + 1 > n) { ok = false; return 0; } return p[o]; }
    uint32_t u16(uint64_t o) { if (o + 2 > n) { ok = false; return 0; } return (uint32_t)p[o] << 8 | p[o + 1]; }
    int32_t i16(uint64_t o) { return (int16_t)u16(o); }
    uint32_t u32(uint64_t o) { if (o + 4 > n) { ok = false; return 0; } return (uint32_t)p[o] << 24 | (uint32_t)p[o + 1] << 16 | (uint32_t)p[o + 2] << 8 | p[o + 3]; }
};

struct Font {
    Reader r;
    uint64_t head = 0, hhea = 0, maxp = 0, cmap = 0, hmtx = 0, loca = 0, glyf = 0;
    uint64_t loca_len = 0, glyf_len = 0;
    uint32_t upem = 0, nglyphs = 0, nhm = 0;
    int32_t loca_fmt = 0, ascent = 0, descent = 0, line_gap = 0;
    uint64_t cmap4 = 0;

    bool open(const uint8_t *p, uint64_t n) {
        r = Reader{p, n};
        const uint32_t nt = r.u16(4);
        for (uint32_t i = 0; i < nt; i++) {
            const uint64_t rec = 12 + 16ull * i;
            const uint32_t tag = r.u32(rec), off = r.u32(rec + 8), len = r.u32(rec + 12);
            if ((uint64_t)off + len > n) return false;
            switch (tag) {
            case 0x68656164: head = off; break;                 // head
            case 0x68686561: hhea = off; break;                 // hhea
            case 0x6D617870: maxp = off; break;                 // maxp
            case 0x636D6170: cmap = off; break;                 // cmap
            case 0x686D7478: hmtx = off; break;                 // hmtx
            case 0x6C6F6361: loca = off; loca_len = len; break; // loca
            case 0x676C7966: glyf = off; glyf_len = len; break; // glyf
            default: break;
            }
        }
        if (!head || !hhea || !maxp || !cmap || !hmtx || !loca || !glyf) return false;
        upem = r.u16(head + 18);
        loca_fmt = r.i16(head + 50);
        nglyphs = r.u16(maxp + 4);
        ascent = r.i16(hhea + 4);
        descent = r.i16(hhea + 6);
        line_gap = r.i16(hhea + 8);
        nhm = r.u16(hhea + 34);
        const uint32_t ns = r.u16(cmap + 2);
        for (uint32_t i = 0; i < ns && !cmap4; i++) {
            const uint32_t pid = r.u16(cmap + 4 + 8 * i), eid = r.u16(cmap + 6 + 8 * i), off = r.u32(cmap + 8 + 8 * i);
            if (((pid == 3 && eid == 1) || pid == 0) && r.u16(cmap + off) == 4) cmap4 = cmap + off;
        }
        return r.ok && upem && cmap4 && nhm;
    }
    uint32_t glyph_index(uint32_t c) {
        const uint32_t segx2 = r.u16(cmap4 + 6);
        const uint64_t ends = cmap4 + 14, starts = ends + segx2 + 2, deltas = starts + segx2, ranges = deltas + segx2;
        for (uint32_t s = 0; s < segx2 / 2; s++) {
            if (r.u16(ends + 2 * s) < c) continue;
            const uint32_t st = r.u16(starts + 2 * s);
            if (st > c) return 0;
            const uint32_t delta = r.u16(deltas + 2 * s), ro = r.u16(ranges + 2 * s);
            if (ro == 0) return (c + delta) & 0xFFFF;
            const uint32_t g = r.u16(ranges + 2 * s + ro + 2 * (c - st));
            return g ? (g + delta) & 0xFFFF : 0;
        }
        return 0;
    }
    uint32_t advance(uint32_t g) { return r.u16(hmtx + 4ull * (g < nhm ? g : nhm - 1)); }
    bool glyph_range(uint32_t g, uint64_t *off, uint64_t *len) {
        if (g >= nglyphs) return false;
        uint64_t a, b;
        if (loca_fmt == 0) { a = 2ull * r.u16(loca + 2ull * g); b = 2ull * r.u16(loca + 2ull * g + 2); }
        else { a = r.u32(loca + 4ull * g); b = r.u32(loca + 4ull * g + 4); }
        if (b < a || b > glyf_len) return false;
        *off = glyf + a;
        *len = b - a;
        return true;
    }

    struct Pt { float x, y; bool on; };
    // contours of glyph g (font units), composites resolved with integer offsets
    bool outline(uint32_t g, std::vector<std::vector<Pt>> &cs, int depth = 0) {
        uint64_t o, len;
        if (!glyph_range(g, &o, &len)) return false;
        if (len == 0) return true;
        const int32_t nc = r.i16(o);
        if (nc >= 0) {
            std::vector<uint32_t> endp(nc);
            for (int32_t i = 0; i < nc; i++) endp[i] = r.u16(o + 10 + 2ull * i);
            const uint32_t np = nc ? endp[nc - 1] + 1 : 0;
            uint64_t q = o + 10 + 2ull * nc;
            q += 2 + r.u16(q);   // instructions
            std::vector<uint8_t> fl(np);
            for (uint32_t i = 0; i < np;) {
                const uint8_t f = (uint8_t)r.u8(q++);
                fl[i++] = f;
                if (f & 8) { uint32_t rep = r.u8(q++); while (rep-- && i < np) fl[i++] = f; }
            }
            std::vector<int32_t> xs(np), ys(np);
            int32_t v = 0;
            for (uint32_t i = 0; i < np; i++) {
                const uint8_t f = fl[i];
                if (f & 2) { const int32_t d = (int32_t)r.u8(q++); v += (f & 16) ? d : -d; }
                else if (!(f & 16)) { v += r.i16(q); q += 2; }
                xs[i] = v;
            }
            v = 0;
            for (uint32_t i = 0; i < np; i++) {
                const uint8_t f = fl[i];
                if (f & 4) { const int32_t d = (int32_t)r.u8(q++); v += (f & 32) ? d : -d; }
                else if (!(f & 32)) { v += r.i16(q); q += 2; }
                ys[i] = v;
            }
            uint32_t a = 0;
            for (int32_t cI = 0; cI < nc; cI++) {
                std::vector<Pt> c;
                for (uint32_t i = a; i <= endp[cI] && i < np; i++) c.push_back(Pt{(float)xs[i], (float)ys[i], (fl[i] & 1) != 0});
                a = endp[cI] + 1;
                if (!c.empty()) cs.push_back(c);
            }
            return r.ok;
        }
        if (depth > 4) return false;
        uint64_t q = o + 10;
        for (;;) {
            const uint32_t f = r.u16(q), gi = r.u16(q + 2);
            q += 4;
            int32_t dx, dy;
            if (f & 1) { dx = r.i16(q); dy = r.i16(q + 2); q += 4; }
            else { dx = (int8_t)r.u8(q); dy = (int8_t)r.u8(q + 1); q += 2; }
            if (!(f & 2)) return false;                          // point-matched components: unsupported
            if (f & (0x8 | 0x40 | 0x80)) return false;           // scaled components: unsupported
            std::vector<std::vector<Pt>> sub;
            if (!outline(gi, sub, depth + 1)) return false;
            for (auto &c : sub) {
                for (auto &p : c) { p.x += (float)dx; p.y += (float)dy; }
                cs.push_back(c);
            }
            if (!(f & 0x20)) break;
        }
        return r.ok;
    }
};

// contour -> lines (WG-SDF-1): on/off points, implied midpoints, quadratics in 8 steps
void flatten(const std::vector<Font::Pt> &c, float scale, std::vector<float4> &out) {
    const size_t n = c.size();
    if (n < 2) return;
    size_t s = 0;
    while (s < n && !c[s].on) s++;
    Font::Pt start;
    if (s == n) start = Font::Pt{(c[0].x + c[1].x) * 0.5f, (c[0].y + c[1].y) * 0.5f, true};   // all off-curve
    else start = c[s];
    std::vector<float2> pts;   // flattened, font units
    pts.push_back(make_float2(start.x, start.y));
    Font::Pt cur = start;
    bool have_ctrl = false;
    Font::Pt ctrl{};
    auto quad = [&](Font::Pt p0, Font::Pt cc, Font::Pt p1) {
        for (int k = 1; k <= QUAD_STEPS; k++) {
            const float t = (float)k * (1.0f / QUAD_STEPS);
            const float mt = 1.0f - t;
            const float a = mt * mt, b = 2.0f * mt * t, d = t * t;
            pts.push_back(make_float2(a * p0.x + b * cc.x + d * p1.x, a * p0.y + b * cc.y + d * p1.y));
        }
    };
    const size_t first = (s == n) ? 1 : s + 1;
    for (size_t m = 0; m < n; m++) {
        const Font::Pt p = c[(first + m) % n];
        if (s != n && (first + m) % n == s) {   // back at the start point: close below
            break;
        }
        if (p.on) {
            if (have_ctrl) { quad(cur, ctrl, p); have_ctrl = false; }
            else pts.push_back(make_float2(p.x, p.y));
            cur = p;
        } else {
            if (have_ctrl) {
                const Font::Pt mid{(ctrl.x + p.x) * 0.5f, (ctrl.y + p.y) * 0.5f, true};
                quad(cur, ctrl, mid);
                cur = mid;
            }
            ctrl = p;
            have_ctrl = true;
        }
    }
    if (have_ctrl) quad(cur, ctrl, start);
    else pts.push_back(make_float2(start.x, start.y));
    for (size_t i = 0; i + 1 < pts.size(); i++) {
        const float x0 = pts[i].x * scale, y0 = pts[i].y * scale, x1 = pts[i + 1].x * scale, y1 = pts[i + 1].y * scale;
        if (y0 == y1) continue;    // horizontal lines never cross a sample row
        out.push_back(make_float4(x0, y0, x1, y1));
    }
}

}  // namespace

// 64-bit hash of the font's bytes (word-wise multiply-xorshift), for the rebuild check
static uint64_t font_bytes_hash(const uint8_t *p, uint64_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ n;
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, p + i, 8);
        h = (h ^ w) * 0xFF51AFD7ED558CCDull;
        h ^= h >> 32;
    }
    for (; i < n; i++) h = (h ^ p[i]) * 0x100000001B3ull;
    return h ^ (h >> 29);
}

// coverage then the two EDT passes over the slot's uploaded outlines
static int font_atlas_run(wg_ctx *c, FontSlot &S) {
    hipStream_t s = c->stream;
    const uint32_t W = S.W, H = S.H, spread = S.spread;
    const uint64_t npx = (uint64_t)W * H;
    wg_stage_begin(c, "font_atlas");
    wg_stage_begin(c, "font_coverage");
    WG_HIP(c, hipMemsetAsync(S.cov.p, 0, npx, s));
    if (S.n_gd)
        hipLaunchKernelGGL(k_font_coverage, dim3(S.n_gd, (S.max_ch + BAND - 1) / BAND), dim3(COV_T), 0, s,
                           S.gdesc.as<const GlyphDesc>(), S.edges.as<const float4>(), spread, W, S.cov.as<uint8_t>());
    wg_stage_end(c);
    wg_stage_begin(c, "font_edt");
    hipLaunchKernelGGL(k_edt_cols, dim3((W + EC_TX - 1) / EC_TX, (H + EC_TY - 1) / EC_TY), dim3(EC_TX), 0, s,
                       S.cov.as<const uint8_t>(), W, H, S.R,
                       S.gin.as<uint16_t>(), S.gout.as<uint16_t>());
    hipLaunchKernelGGL(k_edt_rows, dim3(H), dim3(ROW_T), 0, s, S.gin.as<const uint16_t>(), S.gout.as<const uint16_t>(), W,
                       S.R, (float)spread, S.d2in.as<uint16_t>(), S.d2out.as<uint16_t>(), S.sdf.as<uint8_t>());
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    wg_stage_end(c);
    WG_HIP(c, hipStreamSynchronize(s));
    S.built = true;
    return WG_OK;
}

extern "C" {

int wg_font_atlas_build(wg_ctx *c, int slot, const uint8_t *ttf, uint64_t len, const wg_atlas_params *prm) {
    if (!c || !ttf || !prm || slot < 0 || slot >= WG_FONT_SLOTS) return WG_E_INVALID;
    const uint32_t W = prm->width, H = prm->height, spread = prm->spread;
    if (W == 0 || H == 0 || W > ROW_MAX || spread == 0 || spread > 60 || !(prm->em_px > 0.0f) ||
        prm->first_char > prm->last_char || prm->last_char > 0xFFFF)
        return wg_fail(c, WG_E_INVALID, "bad atlas parameters");
    (void)hipSetDevice(c->device);
    FontSlot &S = c->fonts[slot];
    S.built = false;
    const uint64_t key = font_bytes_hash(ttf, len);
    if (S.have_key && S.key_len == len && S.key_hash == key && !std::memcmp(&S.key_prm, prm, sizeof(*prm)) &&
        S.key_bytes.size() == len && !std::memcmp(S.key_bytes.data(), ttf, len))
        return font_atlas_run(c, S);   // the same font at the same parameters: the device inputs stand
    S.have_key = false;
    Font f;
    if (!f.open(ttf, len)) return wg_fail(c, WG_E_INVALID, "not a TrueType font with cmap format 4");
    const float scale = prm->em_px / (float)f.upem;
    std::vector<float4> edges;
    std::vector<GlyphDesc> gd;
    S.glyphs.clear();
    uint32_t cx = 0, cy = 0, row_h = 0;
    for (uint32_t ch = prm->first_char; ch <= prm->last_char; ch++) {
        const uint32_t g = f.glyph_index(ch);
        wg_glyph m{};
        m.codepoint = ch;
        m.advance = (float)f.advance(g) * scale;
        std::vector<std::vector<Font::Pt>> cs;
        if (!f.outline(g, cs)) return wg_fail(c, WG_E_UNSUPPORTED, "glyph %u (U+%04X) outline not supported", g, ch);
        uint64_t go, gl;
        f.glyph_range(g, &go, &gl);
        if (gl > 0 && !cs.empty()) {
            const float xmin = (float)f.r.i16(go + 2), ymin = (float)f.r.i16(go + 4);
            const float xmax = (float)f.r.i16(go + 6), ymax = (float)f.r.i16(go + 8);
            const int32_t bx0 = (int32_t)floorf(xmin * scale), bx1 = (int32_t)ceilf(xmax * scale);
            const int32_t by0 = (int32_t)floorf(ymin * scale), by1 = (int32_t)ceilf(ymax * scale);
            m.bearing_x = bx0;
            m.bearing_top = by1;
            m.w = (uint32_t)(bx1 - bx0);
            m.h = (uint32_t)(by1 - by0);
            const uint32_t cw = m.w + 2 * spread, chh = m.h + 2 * spread;
            if (cx + cw > W) { cx = 0; cy += row_h; row_h = 0; }
            if (cw > W || cy + chh > H) return wg_fail(c, WG_E_UNSUPPORTED, "atlas %ux%u too small at em %.1f px", W, H, prm->em_px);
            m.atlas_x = cx;
            m.atlas_y = cy;
            GlyphDesc d;
            d.edge_off = (uint32_t)edges.size();
            for (auto &cc : cs) flatten(cc, scale, edges);
            d.n_edges = (uint32_t)edges.size() - d.edge_off;
            d.bx0 = bx0;
            d.by1 = by1;
            d.cw = cw;
            d.ch = chh;
            d.ax = cx;
            d.ay = cy;
            gd.push_back(d);
            cx += cw;
            row_h = chh > row_h ? chh : row_h;
        }
        S.glyphs.push_back(m);
    }
    S.W = W;
    S.H = H;
    S.spread = spread;
    S.em_px = prm->em_px;
    S.R = 4 * spread;
    S.ascent = (float)f.ascent * scale;
    S.descent = (float)f.descent * scale;
    S.line_gap = (float)f.line_gap * scale;
    S.n_edges = edges.size();
    S.first_char = prm->first_char;
    hipStream_t s = c->stream;
    const uint64_t npx = (uint64_t)W * H;
    WG_ALLOC(c, S.edges, edges.size() * sizeof(float4) + 16);
    WG_ALLOC(c, S.gdesc, gd.size() * sizeof(GlyphDesc) + 16);
    WG_ALLOC(c, S.cov, npx);
    WG_ALLOC(c, S.sdf, npx);
    WG_ALLOC(c, S.gin, npx * 2);
    WG_ALLOC(c, S.gout, npx * 2);
    WG_ALLOC(c, S.d2in, npx * 2);
    WG_ALLOC(c, S.d2out, npx * 2);
    WG_ALLOC(c, S.gtab, S.glyphs.size() * sizeof(wg_glyph) + 16);
    if (!edges.empty()) WG_HIP(c, hipMemcpyAsync(S.edges.p, edges.data(), edges.size() * sizeof(float4), hipMemcpyHostToDevice, s));
    if (!gd.empty()) WG_HIP(c, hipMemcpyAsync(S.gdesc.p, gd.data(), gd.size() * sizeof(GlyphDesc), hipMemcpyHostToDevice, s));
    WG_HIP(c, hipMemcpyAsync(S.gtab.p, S.glyphs.data(), S.glyphs.size() * sizeof(wg_glyph), hipMemcpyHostToDevice, s));
    S.n_gd = (uint32_t)gd.size();
    S.max_ch = 0;
    for (const GlyphDesc &d : gd) S.max_ch = d.ch > S.max_ch ? d.ch : S.max_ch;
    const int rc = font_atlas_run(c, S);
    if (rc == WG_OK) {
        S.have_key = true;
        S.key_len = len;
        S.key_hash = key;
        S.key_prm = *prm;
        S.key_bytes.assign(ttf, ttf + len);
    }
    return rc;
}

int wg_font_atlas_info(wg_ctx *c, int slot, wg_atlas_info *out) {
    if (!c || !out || slot < 0 || slot >= WG_FONT_SLOTS) return WG_E_INVALID;
    const FontSlot &S = c->fonts[slot];
    if (!S.built) return wg_fail(c, WG_E_STATE, "font slot %d not built", slot);
    out->width = S.W;
    out->height = S.H;
    out->spread = S.spread;
    out->n_glyphs = (uint32_t)S.glyphs.size();
    out->n_edges = (uint32_t)S.n_edges;
    out->far_d2 = (S.R + 1) * (S.R + 1);
    out->em_px = S.em_px;
    out->ascent = S.ascent;
    out->descent = S.descent;
    out->line_gap = S.line_gap;
    out->first_char = S.first_char;
    return WG_OK;
}

int wg_copy_font_atlas(wg_ctx *c, int slot, uint8_t *sdf, uint8_t *coverage, uint16_t *d2_in, uint16_t *d2_out,
                       wg_glyph *glyphs) {
    if (!c || slot < 0 || slot >= WG_FONT_SLOTS) return WG_E_INVALID;
    FontSlot &S = c->fonts[slot];
    if (!S.built) return wg_fail(c, WG_E_STATE, "font slot %d not built", slot);
    const uint64_t npx = (uint64_t)S.W * S.H;
    hipStream_t s = c->stream;
    if (sdf) WG_HIP(c, hipMemcpyAsync(sdf, S.sdf.p, npx, hipMemcpyDeviceToHost, s));
    if (coverage) WG_HIP(c, hipMemcpyAsync(coverage, S.cov.p, npx, hipMemcpyDeviceToHost, s));
    if (d2_in) WG_HIP(c, hipMemcpyAsync(d2_in, S.d2in.p, npx * 2, hipMemcpyDeviceToHost, s));
    if (d2_out) WG_HIP(c, hipMemcpyAsync(d2_out, S.d2out.p, npx * 2, hipMemcpyDeviceToHost, s));
    WG_HIP(c, hipStreamSynchronize(s));
    if (glyphs) std::memcpy(glyphs, S.glyphs.data(), S.glyphs.size() * sizeof(wg_glyph));
    return WG_OK;
}

}  // extern "C"
