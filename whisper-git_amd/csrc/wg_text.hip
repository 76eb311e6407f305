// wg_text.hip — per-row SDF glyph quads (frozen spec
// WG-TEXT-1 in DESIGN.md §5c).
//
// The reference lays a commit row out as short SHA (mono, muted), avatar,
// summary ("(no summary)" when empty, ellipsised) and, right-aligned, the
// relative time (commit_graph.rs:1002-1130; short_id = first 7 hex digits of
// the id, git/mod.rs:300; format_relative_time, git/mod.rs:34-49, which reads
// the clock — the engine takes `now` as an input).  The legacy TextRenderer
// turned each character into one textured quad of 6 TextVertex
// {position, tex_coord, color} (docs/render_engine.md:113-131), absent from
// the snapshot.  WG-TEXT-1 freezes that layout on top of the WG-SDF-1 atlas.
//
// Two kernels:
//   k_text_rows    one lane per row: builds the three runs (hex digits,
//                  summary bytes, relative-time text), advances the pen
//                  sequentially in f32 (the order a CPU layout loop uses),
//                  clips the summary at summary_max_x and writes one 16-byte
//                  record per visible glyph {pen x, baseline, glyph, run},
//                  staged per wave and flushed as per-row runs.  VALU-issue
//                  bound (one character per lane per iteration, lanes idle
//                  past their row's end), not memory bound.
//   k_text_quads   one thread per glyph record: 6 TextVertex (192 B) staged
//                  per wave in LDS and written as contiguous 1 KiB stores
// Rows are counted first (same walk, counts only) so every record has a
// fixed slot.
#include "wg_internal.h"

namespace {

constexpr int T = 256;
inline uint32_t blocks(uint64_t n) { return (uint32_t)((n + T - 1) / T); }

struct TextArgs {
    uint64_t rb, re;                 // rows
    const uint8_t *oid;
    const int64_t *time;
    const uint8_t *flags;
    const uint8_t *sum;              // summary bytes
    const uint64_t *sum_off;         // [N + 1] (global rows)
    const float *node_y;             // row arrays of the current geometry (context indexing)
    uint64_t row_base;               // context index of global row `rb` minus rb
    const wg_glyph *glyphs;
    uint32_t first_char, n_glyphs;
    float scale;                     // text_px / em_px
    float sha_x, summary_x, summary_max_x, time_right_x, baseline_dy;
    int64_t now;
    const uint8_t *match;            // search-match flags of global rows [mrb, mre), or null (no dimming)
    uint64_t mrb, mre;
};

// format_relative_time (git/mod.rs:34-49) into buf, returns the length
__device__ __forceinline__ uint32_t relative_time(int64_t now, int64_t t, char *buf) {
    int64_t d = now - t;
    if (d < 0) d = 0;
    if (d < 60) {
        const char *s = "just now";
        for (int i = 0; i < 8; i++) buf[i] = s[i];
        return 8;
    }
    int64_t v;
    const char *unit;
    uint32_t ul;
    if (d < 4294967296ll) {   // same quotients in 32-bit arithmetic
        const uint32_t d32 = (uint32_t)d;
        if (d32 < 3600u) { v = d32 / 60u; unit = "m"; ul = 1; }
        else if (d32 < 86400u) { v = d32 / 3600u; unit = "h"; ul = 1; }
        else if (d32 < 604800u) { v = d32 / 86400u; unit = "d"; ul = 1; }
        else if (d32 < 2592000u) { v = d32 / 604800u; unit = "w"; ul = 1; }
        else if (d32 < 31536000u) { v = d32 / 2592000u; unit = "mo"; ul = 2; }
        else { v = d32 / 31536000u; unit = "y"; ul = 1; }
    } else if (d < 3600) { v = d / 60; unit = "m"; ul = 1; }
    else if (d < 86400) { v = d / 3600; unit = "h"; ul = 1; }
    else if (d < 604800) { v = d / 86400; unit = "d"; ul = 1; }
    else if (d < 2592000) { v = d / 604800; unit = "w"; ul = 1; }
    else if (d < 31536000) { v = d / 2592000; unit = "mo"; ul = 2; }
    else { v = d / 31536000; unit = "y"; ul = 1; }
    char tmp[20];
    uint32_t n = 0;
    if (v < 4294967296ll) {   // 32-bit digits (the common case)
        uint32_t v32 = (uint32_t)v;
        do { tmp[n++] = (char)('0' + v32 % 10u); v32 /= 10u; } while (v32);
    } else {
        do { tmp[n++] = (char)('0' + v % 10); v /= 10; } while (v);
    }
    uint32_t len = 0;
    while (n) buf[len++] = tmp[--n];
    for (uint32_t i = 0; i < ul; i++) buf[len++] = unit[i];
    return len;
}

__device__ __forceinline__ uint32_t glyph_of(const TextArgs &A, uint32_t ch) {
    uint32_t g = ch - A.first_char;
    if (ch < A.first_char || g >= A.n_glyphs) g = '?' - A.first_char;   // outside the atlas: '?'
    return g;
}

// The pen walk is sequential in f32 per row, so a lane owns a row; the 64
// rows of a wave advance in lock step, one character per iteration (a run
// switch takes one iteration), which keeps the loop wave-uniform:
//   * byte -> {glyph, visible, advance * scale} from a 256-entry LDS table
//     (every byte maps through glyph_of; the product is the same f32 value the
//     per-glyph multiply gives);
//   * the short SHA and the relative-time text sit in LDS per lane;
//   * records go to a per-wave LDS stage (pen + glyph/run, 8 B; the baseline is
//     per row), one slot per lane per iteration, and every RT_R iterations the
//     wave flushes them: a lane's pending records are contiguous in the
//     output, so RT_R lanes write one row's (<= RT_R * 16 B) run per store instruction
//     instead of 64 scattered 16-B stores.
constexpr int RT_R = 8;                    // iterations between flushes (record slots per lane)
constexpr int RT_STR = 24;                 // per lane: SHA at [0, 7), time text at [8, 8 + 14]

template <bool WRITE>
__global__ void __launch_bounds__(T) k_text_rows(TextArgs A, uint64_t *__restrict__ cnt, const uint64_t *__restrict__ off,
                                                 uint4 *__restrict__ rec) {
    __shared__ float s_adv[256];
    __shared__ uint32_t s_gl[256];                          // glyph | visible << 31
    __shared__ uint8_t s_str[T / 64][RT_STR][64];           // [wave][char][lane]
    __shared__ uint2 s_rec[WRITE ? T / 64 : 1][WRITE ? RT_R : 1][64];   // {pen, glyph | run << 24}
    __shared__ uint64_t s_base[WRITE ? T / 64 : 1][64];
    __shared__ uint32_t s_pend[WRITE ? T / 64 : 1][64];
    __shared__ float s_y[WRITE ? T / 64 : 1][64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    {
        const uint32_t g = glyph_of(A, tid);
        const wg_glyph gl = A.glyphs[g];
        s_adv[tid] = gl.advance * A.scale;
        s_gl[tid] = g | (gl.w ? 0x80000000u : 0u);
    }
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + tid;
    const uint64_t r = A.rb + j;
    const bool live = r < A.re;
    float base = 0.0f, tx = 0.0f;
    uint32_t nsha = 0, nt = 0, nsum = 0, d = 0;
    const uint8_t *sum = nullptr;
    bool nosum = false;
    uint8_t(*str)[64] = s_str[w];
    if (live) {
        base = A.node_y[A.row_base + r] + A.baseline_dy;
        if (!(A.flags[r] & WG_FLAG_SYNTHETIC)) {
            const char *hex = "0123456789abcdef";
            for (int i = 0; i < 7; i++) {
                const uint8_t b = A.oid[r * 20 + i / 2];
                str[i][lane] = (uint8_t)hex[(i & 1) ? (b & 15) : (b >> 4)];
            }
            nsha = 7;
        }
        if (A.sum) {
            const uint64_t so = A.sum_off[r];
            nsum = (uint32_t)(A.sum_off[r + 1] - so);
            sum = A.sum + so;
        }
        if (nsum == 0) { nosum = true; nsum = 12; }
        char tb[16];
        nt = relative_time(A.now, A.time[r], tb);
        for (uint32_t i = 0; i < nt; i++) str[8 + i][lane] = (uint8_t)tb[i];
        // search dimming (commit_graph.rs:1467, 1482): colours 3..5 = the run colours at WG_DIM_ALPHA
        d = (A.match && r >= A.mrb && r < A.mre && !A.match[r - A.mrb]) ? 3u : 0u;
    }
    if (WRITE) s_y[w][lane] = base;
    __syncthreads();   // glyph table, strings
    if (live) {
        float wdt = 0.0f;   // run_width: f32 sum of advances in order
        for (uint32_t i = 0; i < nt; i++) wdt = wdt + s_adv[str[8 + i][lane]];
        tx = A.time_right_x - wdt;
    }
    const uint8_t *none = reinterpret_cast<const uint8_t *>("(no summary)");
    uint32_t n = 0, flushed = 0, it = 0;
    const uint64_t obase = WRITE && live ? off[j] : 0ull;
    // the wave writes the records staged so far: a lane's pending records are
    // contiguous in the output (8 lanes per row and store instruction)
    auto flush = [&]() {
        s_base[w][lane] = obase + flushed;
        s_pend[w][lane] = n - flushed;
        flushed = n;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t q = lane % RT_R;
#pragma unroll
        for (int t = 0; t < RT_R; t++) {
            const uint32_t row = t * (64 / RT_R) + lane / RT_R;
            if (q < s_pend[w][row]) {
                const uint2 v = s_rec[w][q][row];
                rec[s_base[w][row] + q] = make_uint4(v.x, __float_as_uint(s_y[w][row]), v.y & 0xFFFFFFu, v.y >> 24);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // one glyph of run `run` at pen: returns false when the run is clipped
    auto glyph = [&](uint32_t ch, float &pen, float max_x, uint32_t run) -> bool {
        const float next = pen + s_adv[ch];
        if (next > max_x) return false;   // clipped (summary column)
        const uint32_t gv = s_gl[ch];
        if (gv >> 31) {
            if (WRITE) s_rec[w][n - flushed][lane] = make_uint2(__float_as_uint(pen), (gv & 0xFFFFFFu) | ((run + d) << 24));
            n++;
        }
        pen = next;
        return true;
    };
    // the three runs one after the other, each a wave-uniform loop (one
    // character per lane per iteration; every RT_R iterations a flush)
    {   // short SHA: 7 characters (none on synthetic rows)
        float pen = A.sha_x;
        bool on = true;   // (a run also stops where the pen passes 3e38, as in the reference walk)
#pragma unroll 1
        for (uint32_t i = 0; i < 7; i++) {
            if (on && i < nsha) on = glyph(str[i][lane], pen, 3.0e38f, 0u);
            if (WRITE && ++it % RT_R == 0) flush();
        }
    }
    {   // summary, clipped at summary_max_x
        float pen = A.summary_x;
        bool on = live;
#pragma unroll 1
        for (uint32_t i = 0; __any(on && i < nsum); i++) {
            if (on && i < nsum) on = glyph(nosum ? none[i] : sum[i], pen, A.summary_max_x, 1u);
            if (WRITE && ++it % RT_R == 0) flush();
        }
    }
    {   // relative time, right-aligned at time_right_x
        float pen = tx;
        bool on = true;
#pragma unroll 1
        for (uint32_t i = 0; __any(on && i < nt); i++) {
            if (on && i < nt) on = glyph(str[8 + i][lane], pen, 3.0e38f, 2u);
            if (WRITE && ++it % RT_R == 0) flush();
        }
    }
    if (WRITE) flush();
    if (!WRITE && live) cnt[j] = n;
}

struct QuadArgs {
    uint64_t nq;
    const uint4 *rec;
    const wg_glyph *glyphs;
    float scale, spread, inv_w, inv_h;
    float4 color[6];                 // run colours, then the same at WG_DIM_ALPHA
    uint64_t nblk, per_xcd;          // blocks of QT quads; blocks per XCD (XCD-aware order)
};

#ifndef WG_QUAD_THREADS
#define WG_QUAD_THREADS 256
#endif
constexpr int QT = WG_QUAD_THREADS;

__global__ void __launch_bounds__(QT) k_text_quads(QuadArgs A, float4 *__restrict__ out) {
    __shared__ __attribute__((aligned(16))) float4 stage[QT / 64][64 * 12];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // XCD-aware order (as k_vtx_tile): workgroup b runs on XCD b % 8, which
    // writes one contiguous eighth of the buffer
    const uint64_t blk = (uint64_t)(blockIdx.x % 8u) * A.per_xcd + blockIdx.x / 8u;
    if (blk >= A.nblk) return;
    const uint64_t q0 = blk * QT + w * 64;   // this wave's first quad
    if (q0 >= A.nq) return;
    const uint64_t q = q0 + lane;
    float4 *st = stage[w];
    if (q < A.nq) {
        const uint4 r = A.rec[q];
        const float pen = __uint_as_float(r.x), base = __uint_as_float(r.y);
        const wg_glyph g = A.glyphs[r.z];
        const float4 c = A.color[r.w];
        const float cw = (float)(g.w + 2u * (uint32_t)A.spread), ch = (float)(g.h + 2u * (uint32_t)A.spread);
        const float x0 = pen + ((float)g.bearing_x - A.spread) * A.scale;
        const float y0 = base - ((float)g.bearing_top + A.spread) * A.scale;
        const float x1 = x0 + cw * A.scale, y1 = y0 + ch * A.scale;
        const float u0 = (float)g.atlas_x * A.inv_w, v0 = (float)g.atlas_y * A.inv_h;
        const float u1 = ((float)g.atlas_x + cw) * A.inv_w, v1 = ((float)g.atlas_y + ch) * A.inv_h;
        // (x0,y0) (x1,y0) (x0,y1) | (x1,y0) (x1,y1) (x0,y1); TextVertex = {x, y, u, v, r, g, b, a}
        const float px[6] = {x0, x1, x0, x1, x1, x0}, py[6] = {y0, y0, y1, y0, y1, y1};
        const float pu[6] = {u0, u1, u0, u1, u1, u0}, pv[6] = {v0, v0, v1, v0, v1, v1};
#pragma unroll
        for (int k = 0; k < 6; k++) {
            st[lane * 12 + 2 * k] = make_float4(px[k], py[k], pu[k], pv[k]);
            st[lane * 12 + 2 * k + 1] = c;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint64_t cnt = (A.nq - q0) < 64 ? (A.nq - q0) : 64;
    float4 *dst = out + q0 * 12;
#pragma unroll
    for (int k = 0; k < 12; k++) {
        const uint32_t i = k * 64 + lane;
        typedef float v4f __attribute__((ext_vector_type(4)));
        if (i < cnt * 12) {
#ifdef WG_PLAIN_STORES
            reinterpret_cast<v4f *>(dst)[i] = reinterpret_cast<const v4f *>(st)[i];
#else
            __builtin_nontemporal_store(reinterpret_cast<const v4f *>(st)[i], reinterpret_cast<v4f *>(dst) + i);
#endif
        }
    }
}

}  // namespace

extern "C" {

int wg_emit_glyphs(wg_ctx *c, uint64_t rb, uint64_t re, const uint8_t *summary, const uint64_t *summary_off,
                   int32_t residency, const wg_text_params *p) {
    if (!c || !p) return WG_E_INVALID;
    WG_SETTLE(c);
    if (p->slot < 0 || p->slot >= WG_FONT_SLOTS || !c->fonts[p->slot].built)
        return wg_fail(c, WG_E_STATE, "font atlas slot %d not built", p->slot);
    if (!c->have_geom) return wg_fail(c, WG_E_STATE, "no geometry");
    const ShardState &S = c->sh;
    if (rb > re || rb < S.s || re > S.e) return wg_fail(c, WG_E_INVALID, "row range outside the built rows");
    if (!(p->text_px > 0.0f)) return wg_fail(c, WG_E_INVALID, "text_px must be positive");
    (void)hipSetDevice(c->device);
    hipStream_t s = c->stream;
    FontSlot &F = c->fonts[p->slot];
    c->have_text = false;
    const uint64_t rows = re - rb, N = S.N;
    const uint8_t *d_sum = nullptr;
    const uint64_t *d_off = nullptr;
    if (summary_off) {
        if (residency == WG_HOST) {
            const uint64_t bytes = summary_off[N] - summary_off[0];
            WG_ALLOC(c, c->text_sum, bytes + 16);
            WG_ALLOC(c, c->text_sum_off, (N + 1) * 8);
            if (bytes) WG_HIP(c, hipMemcpyAsync(c->text_sum.p, summary + summary_off[0], bytes, hipMemcpyHostToDevice, s));
            // offsets relative to the copied bytes
            std::vector<uint64_t> rel(N + 1);
            for (uint64_t i = 0; i <= N; i++) rel[i] = summary_off[i] - summary_off[0];
            WG_HIP(c, hipMemcpyAsync(c->text_sum_off.p, rel.data(), (N + 1) * 8, hipMemcpyHostToDevice, s));
            WG_HIP(c, hipStreamSynchronize(s));
            d_sum = c->text_sum.as<uint8_t>();
            d_off = c->text_sum_off.as<uint64_t>();
        } else if (residency == WG_DEVICE) {
            d_sum = summary;
            d_off = summary_off;
        } else {
            return wg_fail(c, WG_E_INVALID, "bad residency %d", residency);
        }
    }
    TextArgs A;
    A.rb = rb;
    A.re = re;
    A.oid = c->d_oid;
    A.time = c->d_time;
    A.flags = c->d_flags;
    A.sum = d_sum;
    A.sum_off = d_off;
    A.node_y = c->g_node_y.as<const float>();
    A.row_base = S.row_base - S.s;          // context index = global row + row_base - s
    A.glyphs = F.gtab.as<const wg_glyph>();
    A.first_char = F.first_char;
    A.n_glyphs = (uint32_t)F.glyphs.size();
    A.scale = p->text_px / F.em_px;
    A.sha_x = p->sha_x;
    A.summary_x = p->summary_x;
    A.summary_max_x = p->summary_max_x;
    A.time_right_x = p->time_right_x;
    A.baseline_dy = p->baseline_dy;
    A.now = p->now;
    A.match = c->match_on ? c->match_flags.as<const uint8_t>() : nullptr;
    A.mrb = c->match_rb;
    A.mre = c->match_re;
    if ('?' < F.first_char || '?' - F.first_char >= F.glyphs.size())
        return wg_fail(c, WG_E_UNSUPPORTED, "atlas lacks '?' (the substitute glyph)");
    WG_ALLOC(c, c->text_off, (rows + 2) * 8);
    { const int _sr = wg_scan_reserve(c, rows + 2); if (_sr != WG_OK) return _sr; }
    c->text_rb = rb;
    c->text_re = re;
    c->text_slot = p->slot;
    c->text_scale = A.scale;
    c->n_quads = 0;
    wg_stage_begin(c, "text_rows");
    uint64_t nq = 0;
    if (rows) {
        hipLaunchKernelGGL(k_text_rows<false>, dim3(blocks(rows)), dim3(T), 0, s, A, c->text_off.as<uint64_t>(),
                           (const uint64_t *)nullptr, (uint4 *)nullptr);
        WG_HIP(c, wg_exclusive_scan_u64(c->text_off.as<uint64_t>(), c->text_off.as<uint64_t>(), rows, c->scan_tmp.p, s));
        const int frc = wg_fetch(c, {{c->text_off.as<uint64_t>() + rows, true}}, &nq);
        if (frc != WG_OK) return frc;
        WG_ALLOC(c, c->text_rec, nq * 16 + 16);
        hipLaunchKernelGGL(k_text_rows<true>, dim3(blocks(rows)), dim3(T), 0, s, A, (uint64_t *)nullptr,
                           (const uint64_t *)c->text_off.as<uint64_t>(), c->text_rec.as<uint4>());
    } else {
        WG_HIP(c, hipMemsetAsync(c->text_off.p, 0, 8, s));
    }
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    c->n_quads = nq;
    WG_ALLOC(c, c->text_vtx, nq * 6 * sizeof(wg_text_vertex) + 64);   // (placement measured no gain here: r06bd)
    wg_stage_begin(c, "text_quads");
    if (nq) {
        QuadArgs Q;
        Q.nq = nq;
        Q.rec = c->text_rec.as<const uint4>();
        Q.glyphs = F.gtab.as<const wg_glyph>();
        Q.scale = A.scale;
        Q.spread = (float)F.spread;
        Q.inv_w = 1.0f / (float)F.W;
        Q.inv_h = 1.0f / (float)F.H;
        for (int k = 0; k < 3; k++) {
            const float *col = k == 0 ? p->color_sha : (k == 1 ? p->color_summary : p->color_time);
            Q.color[k] = make_float4(col[0], col[1], col[2], col[3]);
            Q.color[k + 3] = make_float4(col[0], col[1], col[2], col[3] * WG_DIM_ALPHA);
        }
        Q.nblk = (nq + QT - 1) / QT;
        Q.per_xcd = (Q.nblk + 7) / 8;
        hipLaunchKernelGGL(k_text_quads, dim3((uint32_t)(Q.per_xcd * 8)), dim3(QT), 0, s, Q, c->text_vtx.as<float4>());
        WG_HIP(c, hipGetLastError());
    }
    wg_stage_end(c);
    c->have_text = true;
    return WG_OK;
}

int wg_glyph_summary_get(wg_ctx *c, wg_glyph_summary *out) {
    if (!c || !out) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_text) return wg_fail(c, WG_E_STATE, "no glyphs emitted");
    out->row_begin = c->text_rb;
    out->row_end = c->text_re;
    out->n_quads = c->n_quads;
    out->n_vertices = c->n_quads * 6;
    uint64_t chk = 0;
    int rc = wg_words_checksum(c, c->text_vtx.as<const uint32_t>(), c->n_quads * 6 * 8, &chk);
    if (rc != WG_OK) return rc;
    out->checksum = chk;
    return WG_OK;
}

int wg_copy_glyph_vertices(wg_ctx *c, uint64_t first, uint64_t count, wg_text_vertex *dst) {
    if (!c || (!dst && count)) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_text) return wg_fail(c, WG_E_STATE, "no glyphs emitted");
    const uint64_t nv = c->n_quads * 6;
    if (first > nv || count > nv - first) return wg_fail(c, WG_E_INVALID, "vertex range out of bounds");
    if (count)
        WG_HIP(c, hipMemcpyAsync(dst, c->text_vtx.as<wg_text_vertex>() + first, count * sizeof(wg_text_vertex),
                                 hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

int wg_copy_glyph_offsets(wg_ctx *c, uint64_t *dst) {
    if (!c || !dst) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_text) return wg_fail(c, WG_E_STATE, "no glyphs emitted");
    WG_HIP(c, hipMemcpyAsync(dst, c->text_off.p, (c->text_re - c->text_rb + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

}  // extern "C"
