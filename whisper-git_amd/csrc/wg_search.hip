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
// HBM-bound byte work (≈ the text bytes + 20 B of id per row).  A workgroup
// owns 256 consecutive rows; their summary bytes (one contiguous range of
// the CSR) and then their author bytes are staged in LDS with coalesced
// 4-byte loads, and each thread lowers its row's fields as a byte stream
// (ASCII inline, other code points through the Unicode tables, Final_Sigma
// by a scan of the neighbouring code points) into a Knuth-Morris-Pratt matcher of the lowered
// query (query and failure table in LDS).
#include "wg_internal.h"
#include "wg_unicase.h"

#include <cstring>

namespace {

constexpr int MT = 256;                 // rows per workgroup
constexpr int STAGE_WORDS = 6144;       // 24 KiB of staged text per field
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
    const uint16_t *fail;                  // KMP failure table [m]
    uint32_t m;
    uint8_t *out;                          // [re - rb]
    unsigned long long *count;
};

// stage bytes [b0, b1) of text into LDS words; false if they do not fit
__device__ bool stage_field(const uint8_t *text, uint64_t b0, uint64_t b1, uint32_t *s_words, uint32_t &shift) {
    const uint64_t a0 = b0 & ~3ull;
    const uint64_t nw = (b1 - a0 + 3) >> 2;
    shift = (uint32_t)(b0 - a0);
    if (nw > (uint64_t)STAGE_WORDS) return false;
    // aligned 4-byte loads: every word holds at least one byte of [b0, b1), so
    // no load leaves the page of a byte the caller owns
    const uint32_t *w = reinterpret_cast<const uint32_t *>(text + a0);
    for (uint64_t i = threadIdx.x; i < nw; i += MT) s_words[i] = w[i];
    return true;
}

__global__ __launch_bounds__(MT) void k_match(MatchArgs A) {
    __shared__ uint32_t s_txt[STAGE_WORDS];
    __shared__ uint8_t s_q[QLDS];
    __shared__ uint16_t s_fail[QLDS];
    // the case tables (6.5 KiB) in LDS: the binary searches of non-ASCII code
    // points are chains of dependent loads, ~5x shorter from LDS than through
    // the constant/L2 path
    __shared__ uint32_t s_lower[WG_LOWER_N][3];
    __shared__ uint32_t s_cased[WG_CASED_N][2];
    __shared__ uint32_t s_ign[WG_IGNORABLE_N][2];
    for (uint32_t i = threadIdx.x; i < WG_LOWER_N * 3; i += MT) (&s_lower[0][0])[i] = (&c_lower[0][0])[i];
    for (uint32_t i = threadIdx.x; i < WG_CASED_N * 2; i += MT) (&s_cased[0][0])[i] = (&c_cased[0][0])[i];
    for (uint32_t i = threadIdx.x; i < WG_IGNORABLE_N * 2; i += MT) (&s_ign[0][0])[i] = (&c_ign[0][0])[i];
    const WgCaseTables T{s_lower, s_cased, s_ign};
    const uint64_t r0 = A.rb + (uint64_t)blockIdx.x * MT;
    const uint64_t r1 = r0 + MT < A.re ? r0 + MT : A.re;
    const uint64_t r = r0 + threadIdx.x;
    const bool live = r < r1;
    const bool qlds = A.m <= (uint32_t)QLDS;
    if (qlds)
        for (uint32_t i = threadIdx.x; i < A.m; i += MT) { s_q[i] = A.q[i]; s_fail[i] = A.fail[i]; }
    __syncthreads();   // tables and query
    WgKmp km{qlds ? s_q : A.q, qlds ? s_fail : A.fail, A.m, 0};
    bool hit = false;
    // summary, then author: stage the workgroup's byte range, match from LDS
    for (int f = 0; f < 2; f++) {
        const uint8_t *text = f ? A.auth : A.sum;
        const uint64_t *off = f ? A.auth_off : A.sum_off;
        if (!off) continue;
        const uint64_t b0 = off[r0], b1 = off[r1];
        __syncthreads();   // the previous field's readers are done with s_txt
        uint32_t shift = 0;
        const bool staged = b1 > b0 && stage_field(text, b0, b1, s_txt, shift);
        __syncthreads();
        if (live && !hit) {
            const uint64_t s = off[r], n = off[r + 1] - s;
            const uint8_t *p = staged ? reinterpret_cast<const uint8_t *>(s_txt) + shift + (s - b0) : text + s;
            km.k = 0;
            if (n) hit = wg_lower_stream(T, p, (uint32_t)n, km);
        }
    }
    if (live && !hit && A.m <= 40) {
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
        for (uint32_t i = 0; i < A.m; i++) pre &= hex[i] == q[i];
        hit = pre;
        if (!hit && A.m <= 7 && !(A.flags[r] & WG_FLAG_SYNTHETIC)) {
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
