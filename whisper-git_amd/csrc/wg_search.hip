// wg_search.hip — search-match flags.
//
// Reference: history_view (commit_graph.rs:1320-1332) lowers the search query
// once (`search_query.to_lowercase()`, :1326) and computes, per commit,
// commit_matches_query (:1509-1523):
//     summary.to_lowercase().contains(q) || author.to_lowercase().contains(q)
//  || short_id.to_lowercase().contains(q) || id.to_string().to_lowercase().starts_with(q)
// with short_id = the first 7 hex digits of the id (git/mod.rs:300), empty
// for synthetic rows (git/mod.rs:360, 404); an empty query matches every row
// (:1323-1324).  Non-matching rows are drawn at opacity 0.3 (:1467, 1482):
// wg_emit_vertices / wg_emit_glyphs scale their alpha by WG_DIM_ALPHA.
//
// Per-row byte work (~the text bytes + 20 B of id per row).  A lane owns a
// row: its summary and then its author bytes are copied into the lane's
// column of a lane-major LDS block (batched aligned loads; the wave then reads
// consecutive words at every step), and the lane lowers them as a byte
// stream (ASCII inline; other code points through the Unicode tables in LDS,
// the two-byte range by a direct delta table, Final_Sigma by a scan of the
// neighbouring code points in the column) into the matcher: a 64-bit shift
// register for queries of <= 8 lowered bytes, else Knuth-Morris-Pratt with
// the query and failure table in LDS.  VALU-bound: a wave runs its longest
// row, and a lane at a non-ASCII code point holds the others for the whole
// decode / lower / encode path (measured: ~0.37 ms per 1M rows with ASCII
// summaries and the name pool's non-ASCII authors, ~0.6 ms with 15%
// non-ASCII summary words, whatever the byte path: flat or LDS reads, KMP or
// shift register).  Rows longer than 128 bytes, or queries longer than the
// LDS copy, take the generic stream from HBM.
#include "wg_internal.h"
#include "wg_unicase.h"

#include <cstring>

namespace {

constexpr int MT = 256;                 // rows per workgroup
constexpr int QLDS = 2048;              // query bytes held in LDS

__constant__ uint32_t c_lower[WG_LOWER_N][3] = WG_LOWER_TABLE_INIT;
__constant__ uint32_t c_cased[WG_CASED_N][2] = WG_CASED_TABLE_INIT;
__constant__ uint32_t c_ign[WG_IGNORABLE_N][2] = WG_IGNORABLE_TABLE_INIT;
const uint32_t h_lower[WG_LOWER_N][3] = WG_LOWER_TABLE_INIT;
const uint32_t h_cased[WG_CASED_N][2] = WG_CASED_TABLE_INIT;
const uint32_t h_ign[WG_IGNORABLE_N][2] = WG_IGNORABLE_TABLE_INIT;

struct MatchArgs {
    uint64_t rb, re;                       // global rows
    const uint8_t *sum, *auth;             // text bytes (NULL: field empty)
    const uint64_t *sum_off, *auth_off;    // [N+1] global (or rebased host copies)
    const uint8_t *oid, *flags;
    const uint8_t *q;                      // lowered query [m]
    const int16_t *lut2;                   // [WG_LUT2_N] simple lowercase deltas of U+0080..U+07FF
    const uint16_t *fail;                  // KMP failure table [m]
    uint32_t m;
    uint8_t *out;                          // [re - rb]
    unsigned long long *count;
};

// Rows of a wave are transposed into LDS lane-major: word j of lane k's row
// at col[j * 64 + k].  A per-lane walk over its own row then reads
// consecutive words across the wave at every step — the byte-offset layout
// put the 64 lanes' reads at effectively random banks (about 5-way
// conflicts on every read).  Rows longer than TT_W words go through the
// stream from HBM.
constexpr uint32_t TT_W = 32;             // words (128 bytes) of a row held in LDS

// a row's bytes in its lane-major LDS column
struct LdsCol {
    const uint32_t *col;
    __device__ uint8_t operator[](uint32_t i) const { return (uint8_t)(col[(i >> 2) * 64] >> (8u * (i & 3u))); }
};

// the lowered bytes of the non-ASCII unit at g[i] (row g[0, n) in the column), as wg_lower_stream
__device__ __forceinline__ uint32_t lower_unit(const WgCaseTables &T, const LdsCol &g, uint32_t i, uint32_t n,
                                               uint32_t *len, uint8_t *buf) {
    const uint32_t cp = wg_utf8_decode(g, i, n, len);
    if (cp & 0x80000000u) { buf[0] = (uint8_t)cp; return 1; }
    if (cp == 0x130) { buf[0] = 'i'; buf[1] = 0xCC; buf[2] = 0x87; return 3; }   // SpecialCasing
    if (cp == 0x3A3) return wg_utf8_encode(wg_final_sigma(T, g, i, n) ? 0x3C2u : 0x3C3u, buf);
    return wg_utf8_encode(wg_lower_simple(T, cp), buf);
}

// row's lowered stream against the query: the last <= 8 bytes in a 64-bit
// shift register (m <= 8), or KMP with q / fail in LDS
template <bool SHORT>
__device__ __forceinline__ bool match_row(const WgCaseTables &T, const uint32_t *col, uint32_t n,
                                          uint64_t qv, uint64_t qmask, const uint8_t *q, const uint16_t *fail, uint32_t m) {
    uint64_t win = 0;
    uint32_t fed = 0, k = 0, widx = 0xFFFFFFFFu, w = 0;
    auto feed = [&](uint32_t c) -> bool {
        if (SHORT) {
            win = (win << 8) | c;
            fed++;
            return fed >= m && (win & qmask) == qv;
        }
        while (k && q[k] != c) k = fail[k];
        if (q[k] == c) k++;
        return k == m;
    };
    for (uint32_t i = 0; i < n;) {
        if ((i >> 2) != widx) { widx = i >> 2; w = col[widx * 64]; }
        const uint32_t b0 = (w >> (8u * (i & 3u))) & 0xFFu;
        if (b0 < 0x80u) {
            if (feed((b0 - 'A' < 26u) ? b0 + 32 : b0)) return true;
            i++;
            continue;
        }
        uint32_t len;
        uint8_t buf[4];
        const uint32_t nb = lower_unit(T, LdsCol{col}, i, n, &len, buf);
        for (uint32_t j = 0; j < nb; j++)
            if (feed(buf[j])) return true;
        i += len;
    }
    return false;
}

__global__ __launch_bounds__(MT) void k_match(MatchArgs A) {
    __shared__ uint32_t s_tt[MT / 64][TT_W * 64];
    __shared__ uint8_t s_q[QLDS];
    __shared__ uint16_t s_fail[QLDS];
    // the case tables (6.5 KiB) and the two-byte range's deltas in LDS
    __shared__ uint32_t s_lower[WG_LOWER_N][3];
    __shared__ uint32_t s_cased[WG_CASED_N][2];
    __shared__ uint32_t s_ign[WG_IGNORABLE_N][2];
    __shared__ int16_t s_lut2[WG_LUT2_N];
    for (uint32_t i = threadIdx.x; i < WG_LOWER_N * 3; i += MT) (&s_lower[0][0])[i] = (&c_lower[0][0])[i];
    for (uint32_t i = threadIdx.x; i < WG_CASED_N * 2; i += MT) (&s_cased[0][0])[i] = (&c_cased[0][0])[i];
    for (uint32_t i = threadIdx.x; i < WG_IGNORABLE_N * 2; i += MT) (&s_ign[0][0])[i] = (&c_ign[0][0])[i];
    for (uint32_t i = threadIdx.x; i < WG_LUT2_N / 2; i += MT)
        reinterpret_cast<uint32_t *>(s_lut2)[i] = reinterpret_cast<const uint32_t *>(A.lut2)[i];
    const WgCaseTables T{s_lower, s_cased, s_ign, s_lut2};
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t r = A.rb + (uint64_t)blockIdx.x * MT + threadIdx.x;
    const bool live = r < A.re;
    const uint32_t m = A.m;
    const bool qlds = m <= (uint32_t)QLDS;
    if (qlds)
        for (uint32_t i = threadIdx.x; i < m; i += MT) { s_q[i] = A.q[i]; s_fail[i] = A.fail[i]; }
    uint64_t qv = 0, qmask = 0;   // short queries: the query's bytes as the shift register holds them
    if (m <= 8)
        for (uint32_t i = 0; i < m; i++) { qv = (qv << 8) | A.q[i]; qmask = (qmask << 8) | 0xFFu; }
    __syncthreads();   // tables and query
    WgKmp km{qlds ? s_q : A.q, qlds ? s_fail : A.fail, m, 0};
    bool hit = false;
    uint32_t *col = &s_tt[wv][lane];
    // summary, then author
    for (int f = 0; f < 2; f++) {
        const uint8_t *text = f ? A.auth : A.sum;
        const uint64_t *off = f ? A.auth_off : A.sum_off;
        if (!off) continue;
        const uint64_t s = live ? off[r] : 0, n = live ? off[r + 1] - s : 0;
        const uint8_t *g = text + s;
        const bool lds = n <= TT_W * 4 && qlds;
        if (lds && !hit) {
            // this lane's row into its LDS column: 4-byte windows from aligned words
            // (a second word only when the window reaches into it: no read past the row)
            // (only aligned words holding a byte of the row are read; the loads of
            // a batch are all issued before the first is waited for)
            const uintptr_t base = reinterpret_cast<uintptr_t>(g);
            const uint32_t sh = (uint32_t)(base & 3u);
            const uint32_t *aw = reinterpret_cast<const uint32_t *>(base - sh);
            const uint32_t nw = (uint32_t)((n + 3) >> 2), naw = (uint32_t)((n + sh + 3) >> 2);
            for (uint32_t j0 = 0; j0 < nw; j0 += 8) {
                uint32_t x[9];
#pragma unroll
                for (int u = 0; u < 9; u++) x[u] = (j0 + u < naw) ? aw[j0 + u] : 0u;
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (j0 + u < nw) col[(j0 + u) * 64] = __builtin_amdgcn_alignbyte(x[u + 1], x[u], sh);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (live && !hit && n) {
            if (lds) {
                hit = m <= 8 ? match_row<true>(T, col, (uint32_t)n, qv, qmask, s_q, s_fail, m)
                             : match_row<false>(T, col, (uint32_t)n, qv, qmask, s_q, s_fail, m);
            } else {
                km.k = 0;
                hit = wg_lower_stream(T, g, (uint32_t)n, km);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the column is rewritten by the next field
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (live && !hit && m <= 40) {
        // id hex (lowercase already): short_id contains q (non-synthetic rows), id starts with q
        uint8_t hex[40];
        const uint8_t *id = A.oid + r * 20;
        for (int i = 0; i < 20; i++) {
            const uint32_t b = id[i], hi = b >> 4, lo = b & 15;
            hex[2 * i] = (uint8_t)(hi < 10 ? '0' + hi : 'a' + hi - 10);
            hex[2 * i + 1] = (uint8_t)(lo < 10 ? '0' + lo : 'a' + lo - 10);
        }
        const uint8_t *q = km.q;
        bool pre = true;
        for (uint32_t i = 0; i < m; i++) pre &= hex[i] == q[i];
        hit = pre;
        if (!hit && m <= 7 && !(A.flags[r] & WG_FLAG_SYNTHETIC)) {
            km.k = 0;
            for (int i = 0; i < 7 && !hit; i++) hit = km(hex[i]);
        }
    }
    if (live) A.out[r - A.rb] = hit ? 1 : 0;
    const int cnt = __syncthreads_count(live && hit);
    if (threadIdx.x == 0 && cnt) atomicAdd(A.count, (unsigned long long)cnt);
}

inline uint32_t mblocks(uint64_t n) { return (uint32_t)((n + MT - 1) / MT); }

}  // namespace

// Rust `str::to_lowercase` of a byte string on the host (same tables as the device)
std::vector<uint8_t> wg_lower_host(const uint8_t *p, uint64_t n) {
    const WgCaseTables T{h_lower, h_cased, h_ign};
    std::vector<uint8_t> out;
    out.reserve(n + 8);
    auto sink = [&out](uint8_t b) { out.push_back(b); return false; };
    wg_lower_stream(T, p, (uint32_t)n, sink);
    return out;
}

extern "C" {

int wg_match_rows(wg_ctx *c, const uint8_t *query, uint64_t query_len, uint64_t rb, uint64_t re, const wg_row_text *text,
                  uint64_t *match_count) {
    if (!c || (query_len && !query)) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_layout) return wg_fail(c, WG_E_STATE, "no layout built");
    const ShardState &S = c->sh;
    const uint64_t N = S.N;
    if (rb > re || re > N) return wg_fail(c, WG_E_INVALID, "row range outside the list");
    if (query_len >= 0xFFFF0000ull) return wg_fail(c, WG_E_UNSUPPORTED, "query longer than 4 GiB");
    (void)hipSetDevice(c->device);
    hipStream_t s = c->stream;
    const uint64_t rows = re - rb;
    c->match_on = false;
    c->match_rb = rb;
    c->match_re = re;
    WG_ALLOC(c, c->match_flags, rows + 16);
    // q = search_query.to_lowercase() (:1326); an empty query matches every row (:1323-1324)
    const std::vector<uint8_t> q = wg_lower_host(query, query_len);
    if (q.size() > 65535) return wg_fail(c, WG_E_UNSUPPORTED, "lowered query longer than 65535 bytes");
    if (q.empty()) {
        if (rows) WG_HIP(c, hipMemsetAsync(c->match_flags.p, 1, rows, s));
        c->match_count = rows;
        if (match_count) *match_count = rows;
        WG_HIP(c, hipStreamSynchronize(s));
        return WG_OK;
    }
    const uint32_t m = (uint32_t)q.size();
    std::vector<uint16_t> fail(m, 0);
    for (uint32_t i = 1, j = 0; i + 1 < m; i++) {   // fail[i + 1]: longest proper border of q[0, i]
        while (j && q[i] != q[j]) j = fail[j];
        if (q[i] == q[j]) j++;
        fail[i + 1] = (uint16_t)j;
    }
    const uint8_t *d_txt[2] = {nullptr, nullptr};
    const uint64_t *d_off[2] = {nullptr, nullptr};
    if (text) {
        const uint8_t *tb[2] = {text->summary, text->author};
        const uint64_t *to[2] = {text->summary_off, text->author_off};
        for (int f = 0; f < 2; f++) {
            if (!to[f]) continue;
            if (text->residency == WG_HOST) {
                // rows [rb, re) only: bytes [off[rb], off[re]) and offsets rebased to them
                const uint64_t b0 = to[f][rb], bytes = to[f][re] - b0;
                DevBuf &tx = c->match_txt[f], &ox = c->match_off[f];
                WG_ALLOC(c, tx, bytes + 16);
                WG_ALLOC(c, ox, (rows + 1) * 8);
                if (bytes) WG_HIP(c, hipMemcpyAsync(tx.p, tb[f] + b0, bytes, hipMemcpyHostToDevice, s));
                std::vector<uint64_t> &rel = c->match_rel[f];
                rel.resize(rows + 1);
                for (uint64_t i = 0; i <= rows; i++) rel[i] = to[f][rb + i] - b0;
                WG_HIP(c, hipMemcpyAsync(ox.p, rel.data(), (rows + 1) * 8, hipMemcpyHostToDevice, s));
                d_txt[f] = tx.as<uint8_t>();
                d_off[f] = ox.as<uint64_t>() - rb;   // indexed by global row
            } else if (text->residency == WG_DEVICE) {
                d_txt[f] = tb[f];
                d_off[f] = to[f];
            } else {
                return wg_fail(c, WG_E_INVALID, "bad residency %d", text->residency);
            }
        }
    }
    if (!c->match_lut2.p) {   // once per context: the two-byte range's deltas, from the host tables
        const WgCaseTables HT{h_lower, h_cased, h_ign};
        std::vector<int16_t> lut(WG_LUT2_N);
        for (uint32_t cp = 0x80; cp < 0x800; cp++) lut[cp - 0x80] = (int16_t)((int32_t)wg_lower_simple(HT, cp) - (int32_t)cp);
        WG_ALLOC(c, c->match_lut2, WG_LUT2_N * 2 + 16);
        WG_HIP(c, hipMemcpyAsync(c->match_lut2.p, lut.data(), WG_LUT2_N * 2, hipMemcpyHostToDevice, s));
        WG_HIP(c, hipStreamSynchronize(s));
    }
    WG_ALLOC(c, c->match_q, 16 + m * 3 + 16);
    std::vector<uint8_t> &qh = c->match_qhost;
    qh.assign(16 + (size_t)m * 3, 0);
    std::memcpy(qh.data() + 16, fail.data(), (size_t)m * 2);
    std::memcpy(qh.data() + 16 + (size_t)m * 2, q.data(), m);
    WG_HIP(c, hipMemsetAsync(c->match_q.p, 0, 8, s));
    WG_HIP(c, hipMemcpyAsync(c->match_q.as<uint8_t>() + 16, qh.data() + 16, (size_t)m * 3, hipMemcpyHostToDevice, s));
    MatchArgs A;
    A.rb = rb;
    A.re = re;
    A.sum = d_txt[0];
    A.auth = d_txt[1];
    A.sum_off = d_off[0];
    A.auth_off = d_off[1];
    A.oid = c->d_oid;
    A.flags = c->d_flags;
    A.fail = reinterpret_cast<const uint16_t *>(c->match_q.as<uint8_t>() + 16);
    A.q = c->match_q.as<uint8_t>() + 16 + (size_t)m * 2;
    A.m = m;
    A.lut2 = c->match_lut2.as<const int16_t>();
    A.out = c->match_flags.as<uint8_t>();
    A.count = c->match_q.as<unsigned long long>();
    wg_stage_begin(c, "match");
    if (rows) hipLaunchKernelGGL(k_match, dim3(mblocks(rows)), dim3(MT), 0, s, A);
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    uint64_t cnt = 0;
    const int frc = wg_fetch(c, {{c->match_q.p, true}}, &cnt);   // also orders the host copies above
    if (frc != WG_OK) return frc;
    c->match_count = cnt;
    c->match_on = true;
    if (match_count) *match_count = cnt;
    return WG_OK;
}

int wg_copy_match_flags(wg_ctx *c, uint8_t *dst) {
    if (!c) return WG_E_INVALID;
    WG_SETTLE(c);
    const uint64_t rows = c->match_re - c->match_rb;
    if (!c->match_flags.p) return wg_fail(c, WG_E_STATE, "no match flags computed");
    if (rows && !dst) return WG_E_INVALID;
    (void)hipSetDevice(c->device);
    if (rows) WG_HIP(c, hipMemcpyAsync(dst, c->match_flags.p, rows, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

int wg_lower_utf8(const uint8_t *src, uint64_t n, uint8_t *dst, uint64_t cap, uint64_t *out_len) {
    if ((n && !src) || !out_len) return WG_E_INVALID;
    if (n >= 0xFFFF0000ull) return WG_E_UNSUPPORTED;
    const std::vector<uint8_t> v = wg_lower_host(src, n);
    *out_len = v.size();
    if (dst && cap) std::memcpy(dst, v.data(), v.size() < cap ? v.size() : cap);
    return WG_OK;
}

}  // extern "C"
