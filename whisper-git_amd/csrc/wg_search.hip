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
// Per-row byte work (~the text bytes + 20 B of id per row).  A workgroup
// owns 256 rows and stages both their fields into one LDS image when they fit
// (else one field per pass), with every lane busy in each phase
// (LDS-resident, barrier-separated):
//  1. stage: each field's bytes of the 256 rows (one contiguous range) into
//     LDS by coalesced word loads, ASCII lowered on the way in (SWAR), the
//     lead bytes of non-ASCII code points listed (wave-aggregated appends;
//     the 0xCE leads from the top of the same list);
//  2. Final_Sigma for the listed 0xCE leads that are U+03A3, over the
//     original bytes (ASCII lowering keeps case classes);
//  3. the listed code points lowered IN PLACE by the thread holding the list
//     entry (one flat table load per code point).  A "special" — U+0130 and
//     the simple mappings whose UTF-8 length differs (U+1E9E, U+212A, ...) —
//     cannot be lowered in place: it is marked (0xFF, its index, 0xFE...:
//     bytes the lowered query does not hold) and, if its lowered bytes share
//     one with the query, listed for a local walk;
//  4. every byte position holding the query's first byte is tested against
//     the query's first 8 lowered bytes (a 64-bit window from three LDS words;
//     the rest of a longer query on a window hit); the row (binary search
//     over the rows' LDS offsets) must hold the whole window.  A window over
//     a mark never matches, and windows off the specials are exact;
//  5. the windows over each listed special: the lowered stream from 3 (m - 1)
//     buffer bytes before it to as many after, marks expanded, through a
//     shift-register matcher.
// Fallbacks, all exact: a query holding 0xFE / 0xFF / bytes < 32 or a field
// holding raw 0xFE / 0xFF (no marks: the rows with specials are walked whole,
// decoding), queries over 16 bytes (rows with relevant specials walked whole,
// KMP), more code points than the lists hold or a field over the LDS buffer
// (the row's own thread streams it from HBM through wg_lower_stream).  Last,
// per row, the id's hex digits (short id contains q / id starts with q),
// only for queries that are all hex digits.
#include "wg_internal.h"
#include "wg_unicase.h"

#include <algorithm>
#include <cstring>

namespace {

constexpr int MT = 256;                 // rows per workgroup
#define WG_MATCH_STRIPES 8              // match-count words (one per 64-byte line)
#define WG_FILT_LEADS 6                 // lead bytes the lead-filtered variant lists (0xCE apart)

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
    const uint32_t *flat;                  // [WG_FLAT_N] per BMP code point, then [WG_SPECIAL_N] specials' lowered bytes
    const uint16_t *fail;                  // KMP failure table [m]
    uint32_t m;
    uint32_t qhex;                         // the query can match the id's hex (m <= 40, all of [0-9a-f])
    uint32_t marks;                        // the query holds no 0xFE / 0xFF byte: specials can be marked in place
    uint32_t spec_rel;                     // bit i: special i's lowered bytes share a byte with the query
    // the lead-filtered variants (k_match<..., MODE 1 / 2>, see the lowering
    // pass): the lead bytes it lists — up to WG_FILT_LEADS, 0xCE apart (flt_ce)
    uint32_t flt_n, flt_ce;
    uint8_t flt_lead[8];
    // the query's first <= 8 bytes little-endian (as an LDS window holds them) and its mask; its last
    // <= 16 big-endian in two words with their masks (as the walks' shift registers hold them; m <= 16).
    // Host-computed: byte loads at the kernel's start wait behind the CU's staging loads.
    uint64_t qv, qmask, qlo, qhi, mlo, mhi;
    uint8_t *out;                          // [re - rb]
    unsigned long long *count;
};

constexpr uint32_t MCAP = 22528;           // bytes of a workgroup's staged fields held in LDS
constexpr uint32_t MCAPW = MCAP / 4;
constexpr uint32_t LCAP = 2560;            // listed lead bytes of a pass (the 0xCE leads from the top down, the others from the bottom up)
constexpr uint32_t SPCAP = 128;            // ... specials walked locally
// per-row flags (s_rf): matched, and per field the walk it needs
constexpr uint32_t RF_HIT = 1u;
__device__ __forceinline__ uint32_t rf_mark(int f) { return 2u << (3 * f); }     // a marked special: walk, fast hits stand
__device__ __forceinline__ uint32_t rf_decode(int f) { return 4u << (3 * f); }   // an unmarked special: decoding walk, fast hits void
__device__ __forceinline__ uint32_t rf_hbm(int f) { return 8u << (3 * f); }      // field over the buffer: stream from HBM

// bytes in LDS
struct LdsBytes {
    const uint8_t *b;
    __device__ uint8_t operator[](uint32_t i) const { return b[i]; }
};

// the four bytes of w with 'A'..'Z' lowered (bytes >= 0x80 unchanged)
__device__ __forceinline__ uint32_t ascii_lower4(uint32_t w) {
    const uint32_t h = w & 0x7F7F7F7Fu;
    const uint32_t ge_a = h + 0x3F3F3F3Fu;     // bit 7 set: byte >= 'A'
    const uint32_t gt_z = h + 0x25252525u;     // bit 7 set: byte > 'Z'
    const uint32_t up = ge_a & ~gt_z & ~w & 0x80808080u;
    return w | (up >> 2);
}

// bit 7 of each byte of w that equals b
__device__ __forceinline__ uint32_t eq_bytes(uint32_t w, uint32_t b) {
    const uint32_t x = w ^ (b * 0x01010101u);
    return ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x) & 0x80808080u;
}

// the lead-filtered variant's leads to list: bit 7 of each byte of w that is
// one of the n lead bytes (MatchArgs::flt_lead).  MODE 1 (an ASCII query):
// the leads are a subset of {0xC4, 0xE2} (U+0130 and U+212A, the only code
// points whose lowering holds an ASCII byte), selected by bits 0 / 1 of n.
template <int MODE>
__device__ __forceinline__ uint32_t filt_lead_bytes(uint32_t w, const uint8_t (&lb)[8], uint32_t n) {
    if (MODE == 1) return ((n & 1u) ? eq_bytes(w, 0xC4u) : 0u) | ((n & 2u) ? eq_bytes(w, 0xE2u) : 0u);
    uint32_t m = 0;
#pragma unroll
    for (int i = 0; i < WG_FILT_LEADS; i++)
        if ((uint32_t)i < n) m |= eq_bytes(w, lb[i]);
    return m;
}

// the largest r < nr with rel[r] <= p (p >= rel[0]): the row holding byte p
__device__ __forceinline__ uint32_t row_of(const uint32_t *rel, uint32_t nr, uint32_t p) {
    uint32_t lo = 0, hi = nr;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (rel[mid] <= p) lo = mid;
        else hi = mid;
    }
    return lo;
}

// word k of a field's staged range: bytes [bias, span) of the LDS image hold
// gp[0, span - bias); aligned words inside by one load, the edge words by bytes
__device__ __forceinline__ uint32_t stage_word(const uint8_t *gp, uint32_t bias, uint32_t span, uint32_t k) {
    if (4 * k >= bias && 4 * k + 4 <= span)
        return reinterpret_cast<const uint32_t *>(gp - bias)[k];   // (plain loads: 1-2% ahead of non-temporal, r05v)
    uint32_t v = 0;
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t pos = 4 * k + j;
        if (pos >= bias && pos < span) v |= (uint32_t)gp[pos - bias] << (8 * j);
    }
    return v;
}

__device__ __forceinline__ uint32_t hex_char(uint32_t v) { return v < 10 ? '0' + v : 'a' + v - 10; }

// the last <= 16 lowered bytes in two 64-bit shift registers against the query (m <= 16)
struct FeedShift {
    uint64_t lo, hi, qlo, qhi, mlo, mhi;
    uint32_t fed, m;
    __device__ bool operator()(uint32_t c) {
        hi = (hi << 8) | (lo >> 56);
        lo = (lo << 8) | c;
        fed++;
        return fed >= m && (lo & mlo) == qlo && (hi & mhi) == qhi;
    }
};

// A row of the LDS buffer after the in-place pass: every code point lowered
// (U+03A3 resolved) except the specials, whose lowering changes the UTF-8
// length.  A special is either marked — its bytes rewritten as 0xFF, its
// index, 0xFE... (bytes the lowered query does not hold, and that no raw
// byte of the workgroup's field is) — or left as it was.  The row's lowered
// stream: bytes as they stand, a mark expanded to its special's lowered
// bytes, and with DECODE a raw special lowered again (simple lowercase is
// idempotent on its image, checked over every code point of the tables, so
// re-lowering a lowered code point is a no-op; only then is decoding needed).
// Without marks (the query or the field holds 0xFE / 0xFF) those bytes are
// the text's own.
// the matcher the walks feed: the last <= 16 bytes in shift registers
// (m <= 16), else KMP over the query in HBM
struct WalkFeed {
    FeedShift sh;
    WgKmp km;
    bool kmp;
    __device__ bool operator()(uint32_t c) { return kmp ? km((uint8_t)c) : sh(c); }
};

// the local walk over a marked special (m <= 16): the buffer's bytes as they
// stand, each mark expanded to its special's lowered bytes
__device__ __forceinline__ bool walk_marked(const uint8_t *sb, uint32_t a, uint32_t b, const uint32_t *special,
                                            FeedShift f) {
    for (uint32_t p = a; p < b; p++) {
        const uint32_t c = sb[p];
        if (c < 0xFEu) {
            if (f(c)) return true;
        } else if (c == 0xFFu) {
            const uint32_t x = special[sb[p + 1]];
            for (uint32_t i = 0; i < (x >> 24); i++)
                if (f((x >> (8 * i)) & 0xFFu)) return true;
            p++;
        }
    }
    return false;
}

__device__ bool walk_row(const WgCaseTables &T, const uint32_t *buf, uint32_t rs, uint32_t re, const uint32_t *special,
                         bool marks, bool decode, WalkFeed feed) {
    const uint8_t *sb = reinterpret_cast<const uint8_t *>(buf);
    uint32_t skip = 0;   // bytes still to skip: a mark's index byte, the rest of a decoded code point
    for (uint32_t k = rs >> 2; 4 * k < re; k++) {
        const uint32_t w = buf[k];
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t p = 4 * k + j;
            if (p < rs || p >= re) continue;
            if (skip) { skip--; continue; }
            const uint32_t b = (w >> (8 * j)) & 0xFFu;
            if (b < 0x80u || (!decode && b < 0xFEu)) {
                if (feed(b)) return true;
                continue;
            }
            if (marks && b == 0xFEu) continue;
            if (marks && b == 0xFFu) {
                const uint32_t x = special[sb[p + 1]];
                for (uint32_t i = 0; i < (x >> 24); i++)
                    if (feed((x >> (8 * i)) & 0xFFu)) return true;
                skip = 1;
                continue;
            }
            uint32_t len;   // decode: a raw code point lowered again
            const uint32_t cp = wg_utf8_decode(LdsBytes{sb + rs}, p - rs, re - rs, &len);
            uint32_t o, no;
            if (cp & 0x80000000u) { o = cp & 0xFFu; no = 1; }
            else if (cp == 0x130u) { o = 'i' | 0xCCu << 8 | 0x87u << 16; no = 3; }
            else {
                uint8_t e[4];
                no = wg_utf8_encode(wg_lower_simple(T, cp), e);
                o = (uint32_t)e[0] | (uint32_t)e[1] << 8 | (uint32_t)e[2] << 16 | (uint32_t)e[3] << 24;
            }
            for (uint32_t i = 0; i < no; i++)
                if (feed((o >> (8 * i)) & 0xFFu)) return true;
            skip = len - 1;
        }
    }
    return false;
}

// NT threads per workgroup (256 or 512) over its MT rows; SB words per thread
// per staging batch.  r06: 512 threads give every LDS-bound phase (lowering,
// Final_Sigma, the first-byte windows, the walks' list) twice the lanes, and
// a CU twice the waves to hide each phase's round trips with (the workgroup's
// LDS is unchanged, so the same workgroups fit per CU)
// MODE 0: every lead listed; 2: the lead-filtered variant (a query whose
// matches can hold the lowering of code points under a few lead bytes only;
// MatchArgs::flt_*); 1: the same for an ASCII query, its leads fixed.  Each a
// variant of its own so the other queries' code is what it was.
template <int NT, int SB, int WPS, int MODE>
__global__ __launch_bounds__(NT, WPS) void k_match(MatchArgs A) {
    __shared__ uint32_t s_buf[MCAPW + 4];
    __shared__ uint32_t s_rel[2][MT + 1];     // per region of the staged image: its rows' byte offsets in it
    __shared__ uint16_t s_lead[LCAP];         // LDS positions of the staged lead bytes (>= 0xC0): others at [0, n), 0xCE
                                              // (U+0380..U+03BF; bit 15: a final U+03A3) at [LCAP - nce, LCAP)
    uint16_t *const s_ce = s_lead + LCAP;     // (s_ce[-1 - i]: the i-th 0xCE lead)
    __shared__ uint32_t s_rf[MT];             // per row: RF_HIT, rf_mark / rf_decode / rf_hbm per field
    __shared__ uint16_t s_wrow[2 * MT];       // rows to walk whole: row | region << 8
    __shared__ uint16_t s_spos[SPCAP];        // marked specials the query could overlap: walked locally
    __shared__ uint32_t s_special[WG_SPECIAL_N];
    __shared__ uint32_t s_cnt[8];             // per pass (4 words each, so a pass never clears counts a slower wave of the previous pass still reads): leads | 0xCE leads << 16, rows to walk, flags (1: a row starts with a continuation byte, 2: a raw 0xFE / 0xFF byte), specials listed
    uint8_t *const sb = reinterpret_cast<uint8_t *>(s_buf);
    const WgCaseTables T{c_lower, c_cased, c_ign, A.flat};
    const uint32_t *special = s_special;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t spv = tid < WG_SPECIAL_N ? A.flat[WG_FLAT_N + tid] : 0u;   // to LDS after the staging loads
    const uint64_t r0 = A.rb + (uint64_t)blockIdx.x * MT;
    const uint32_t nr = (uint32_t)((A.re - r0) < MT ? (A.re - r0) : MT);
    const uint32_t m = A.m;
    const uint64_t qv = A.qv, qmask = A.qmask;
    const uint32_t q0 = (uint32_t)(qv & 0xFFu);
    const FeedShift sh{0, 0, A.qlo, A.qhi, A.mlo, A.mhi, 0, m};
    const WalkFeed wf{sh, WgKmp{A.q, A.fail, m, 0}, m > 16};
    const uint32_t flt_n = A.flt_n;
    uint8_t flt_lead[8];
#pragma unroll
    for (int i = 0; i < 8; i++) flt_lead[i] = A.flt_lead[i];
    if (tid < MT) s_rf[tid] = 0;
    if (tid < 8) s_cnt[tid] = 0;
    // both fields' row offsets and ranges up front (one round trip)
    uint64_t orow[2] = {0, 0}, gsf[2] = {0, 0}, gef[2] = {0, 0};
    for (int f = 0; f < 2; f++) {
        const uint64_t *off = f ? A.auth_off : A.sum_off;
        if (!off) continue;
        gsf[f] = off[r0];
        gef[f] = off[r0 + nr];
        if (tid < nr) orow[f] = off[r0 + tid];
    }
    // The fields' images in LDS: both in one pass when they fit together
    // (summary words, one zero word, author words), else one pass each; a
    // field past the buffer takes the stream from HBM.  Each staged field is
    // a region of the pass.
    uint32_t fspan[2] = {0, 0};
    bool fst[2] = {false, false};
    for (int f = 0; f < 2; f++) {
        if (!(f ? A.auth_off : A.sum_off)) continue;
        const uint8_t *gp = (f ? A.auth : A.sum) + gsf[f];
        const uint64_t span = gef[f] - gsf[f] + (reinterpret_cast<uintptr_t>(gp) & 3u);
        if (span > MCAP) {
            if (tid < nr) s_rf[tid] |= rf_hbm(f);   // (each thread its own row; read after a barrier)
            continue;
        }
        fspan[f] = (uint32_t)span;
        fst[f] = true;
    }
    const bool both = fst[0] && fst[1] && ((fspan[0] + 3) >> 2) + 1 + ((fspan[1] + 3) >> 2) <= MCAPW;
    const int npass = both ? 1 : (int)fst[0] + (int)fst[1];
    for (int pass = 0; pass < npass; pass++) {
        // the pass's regions (uniform): field, text, bias, image span, first word
        const uint32_t ng = both ? 2u : 1u;
        int fg[2];
        fg[0] = both ? 0 : (pass == 0 ? (fst[0] ? 0 : 1) : 1);
        fg[1] = 1;
        const uint8_t *gpg[2];
        uint32_t biasg[2], spang[2], nwg[2], baseg[2];
        for (uint32_t g = 0; g < 2; g++) {
            const int f = fg[g];
            gpg[g] = (f ? A.auth : A.sum) + gsf[f];
            biasg[g] = (uint32_t)(reinterpret_cast<uintptr_t>(gpg[g]) & 3u);
            spang[g] = fspan[f];
            nwg[g] = (spang[g] + 3) >> 2;
        }
        baseg[0] = 0;
        baseg[1] = nwg[0] + 1;
        const uint32_t tw = ng == 2 ? baseg[1] + nwg[1] : nwg[0];   // words of the image
        const uint32_t pb1 = ng == 2 ? 4 * baseg[1] : 0xFFFFFFFFu;   // first byte of region 1
        uint32_t lo[2], hi[2];
        for (uint32_t g = 0; g < 2; g++) {
            lo[g] = 4 * baseg[g] + biasg[g];
            hi[g] = 4 * baseg[g] + spang[g];
        }
        auto reg = [&](uint32_t p) -> uint32_t { return p >= pb1 ? 1u : 0u; };
        uint32_t *const pc = s_cnt + 4 * pass;   // zeroed before the loop
        __syncthreads();   // the previous pass's readers are done with the buffer
        // stage: aligned words inside each field's range by word loads, the edge
        // words by bytes; ASCII lowered on the way in (SWAR; case classes
        // unchanged, so Final_Sigma below still sees the original's), lead bytes
        // listed (wave-aggregated: one LDS atomic per wave and batch)
        {
            uint32_t raw_ff = 0;
            for (uint32_t k0 = tid - lane; k0 < tw; k0 += SB * NT) {   // wave-uniform trip count
                uint32_t v[SB], cnt = 0;
#pragma unroll
                for (int u = 0; u < SB; u++) {
                    const uint32_t k = k0 + lane + u * NT;
                    const uint32_t g = (ng == 2 && k >= baseg[1]) ? 1u : 0u;
                    const uint32_t kk = k - baseg[g];
                    v[u] = 0;
                    if (k < tw && kk < nwg[g]) v[u] = stage_word(gpg[g], biasg[g], spang[g], kk);
                }
#pragma unroll
                for (int u = 0; u < SB; u++) {
                    const uint32_t k = k0 + lane + u * NT;
                    const uint32_t w = v[u];
                    if (k < tw) s_buf[k] = ascii_lower4(w);
                    // bytes >= 0xC0; an ASCII query lists only the leads it needs (see the lowering pass)
                    const uint32_t ce = (MODE == 0 || (MODE == 2 && A.flt_ce)) ? eq_bytes(w, 0xCEu) : 0u;   // (a subset of the leads)
                    const uint32_t lead = MODE ? filt_lead_bytes<MODE>(w, flt_lead, flt_n) | ce : w & (w << 1) & 0x80808080u;
                    cnt += (uint32_t)__builtin_popcount(lead & ~ce) + ((uint32_t)__builtin_popcount(ce) << 16);
                    raw_ff |= w & (w << 1) & (w << 2) & (w << 3) & (w << 4) & (w << 5) & (w << 6) & 0x80808080u;   // 0xFE / 0xFF
                }
                if (__ballot(cnt != 0)) {
                    uint32_t incl = cnt;
                    for (uint32_t d = 1; d < 64; d <<= 1) {
                        const uint32_t t = __shfl_up(incl, d, 64);
                        if (lane >= d) incl += t;
                    }
                    uint32_t base = 0;
                    if (lane == 63) base = atomicAdd(&pc[0], incl);
                    base = __shfl(base, 63, 64);
                    uint32_t il = (base & 0xFFFFu) + ((incl - cnt) & 0xFFFFu), ic = (base >> 16) + ((incl - cnt) >> 16);
#pragma unroll
                    for (int u = 0; u < SB; u++) {
                        const uint32_t w = v[u], k = k0 + lane + u * NT;
                        const uint32_t ce = (MODE == 0 || (MODE == 2 && A.flt_ce)) ? eq_bytes(w, 0xCEu) : 0u;   // (a subset of the leads)
                        const uint32_t lead = MODE ? filt_lead_bytes<MODE>(w, flt_lead, flt_n) | ce : w & (w << 1) & 0x80808080u;
                        if (!lead) continue;
                        for (uint32_t j = 0; j < 4; j++) {
                            if (!((lead >> (8 * j)) & 0x80u)) continue;
                            if ((ce >> (8 * j)) & 0x80u) {
                                if (ic < LCAP) s_ce[-1 - (int)ic] = (uint16_t)(4 * k + j);
                                ic++;
                            } else {
                                if (il < LCAP) s_lead[il] = (uint16_t)(4 * k + j);
                                il++;
                            }
                        }
                    }
                }
            }
            if (tid < 4) s_buf[tw + tid] = 0;
            if (pass == 0 && tid < WG_SPECIAL_N) s_special[tid] = spv;
            for (uint32_t g = 0; g < ng; g++) {
                if (tid < nr) s_rel[g][tid] = 4 * baseg[g] + (uint32_t)(orow[fg[g]] - gsf[fg[g]]) + biasg[g];
                if (tid == 0) s_rel[g][nr] = hi[g];
            }
            if (raw_ff) atomicOr(&pc[2], 2u);
        }
        __syncthreads();
        const uint32_t nlead = pc[0] & 0xFFFFu, nce = pc[0] >> 16;
        if (nlead + nce > LCAP) {   // uniform: more code points than the lists hold: the stream from HBM
            for (uint32_t g = 0; g < ng; g++)
                if (tid < nr) atomicOr(&s_rf[tid], rf_hbm(fg[g]));
            continue;
        }
        for (uint32_t g = 0; g < ng; g++)
            if (tid < nr && s_rel[g][tid] < s_rel[g][tid + 1] && (sb[s_rel[g][tid]] & 0xC0u) == 0x80u) atomicOr(&pc[2], 1u);
        // Final_Sigma of the U+03A3s, over the original non-ASCII bytes (nothing non-ASCII written yet)
        // (none listed when the lead-filtered variant leaves 0xCE out)
        for (uint32_t i = tid; i < nce; i += NT) {
            const uint32_t p = s_ce[-1 - (int)i];
            const uint32_t *rel = s_rel[reg(p)];
            const uint32_t r = row_of(rel, nr, p), rs = rel[r], n = rel[r + 1] - rs;
            const LdsBytes g{sb + rs};
            uint32_t len;
            if (wg_utf8_decode(g, p - rs, n, &len) == 0x3A3u && wg_final_sigma(T, g, p - rs, n))
                s_ce[-1 - (int)i] = (uint16_t)(p | 0x8000u);
        }
        __syncthreads();
        // lower the listed code points in place (a lead's thread writes its whole
        // sequence).  Decoded against the end of their region unless a row starts
        // with a continuation byte (then against their row).  A special is marked
        // and its row set to walk — unless its lowered bytes share none with the
        // query: then no match can overlap it; where marks are off it is left
        // as it was and its row walked by decoding, fast hits void.
        // The lead-filtered variant (r06) lists only the leads of code points
        // whose lowering a match can hold (the host's relevance test, at
        // wg_match_rows): every other code point stays as it is, bytes that no
        // window or walk of the query can match lowered or not — no decode, no
        // table load, and the lists overflow far less often.
        const uint32_t fl = pc[2];
        const bool exact = (fl & 1u) != 0, marks = A.marks && !(fl & 2u);
        for (uint32_t i = tid; i < nlead + nce; i += NT) {
            const uint32_t e = i < nlead ? s_lead[i] : s_ce[-1 - (int)(i - nlead)];
            const uint32_t p = e & 0x7FFFu, g = reg(p);
            const uint32_t *rel = s_rel[g];
            uint32_t rs = 0, n = hi[g];
            if (exact) {
                const uint32_t r = row_of(rel, nr, p);
                rs = rel[r];
                n = rel[r + 1] - rs;
            }
            uint32_t len;
            const uint32_t cp = wg_utf8_decode(LdsBytes{sb + rs}, p - rs, n, &len);
            if (cp & 0x80000000u) continue;   // stands for itself
            uint32_t lc;
            if (cp < WG_FLAT_N) {
                const uint32_t x = A.flat[cp];
                if (x & WG_FLAT_LENCHG) {   // includes U+0130 -> "i̇"
                    const uint32_t idx = (x >> WG_FLAT_SPECIAL_SHIFT) & 31u;
                    if (marks) {
                        sb[p] = 0xFF;
                        sb[p + 1] = (uint8_t)idx;
                        for (uint32_t j = 2; j < len; j++) sb[p + j] = 0xFE;
                        if ((A.spec_rel >> idx) & 1u) {   // walked locally (windows over it), or the row whole
                            const uint32_t si = m <= 16 ? atomicAdd(&pc[3], 1u) : SPCAP;
                            if (si < SPCAP) s_spos[si] = (uint16_t)p;
                            else atomicOr(&s_rf[row_of(rel, nr, p)], rf_mark(fg[g]));
                        }
                    } else {   // raw bytes stay: no window of the row can be trusted
                        atomicOr(&s_rf[row_of(rel, nr, p)], rf_decode(fg[g]));
                    }
                    continue;
                }
                lc = x & 0xFFFFu;
            } else {
                lc = wg_lower_simple(T, cp);
                if (lc < 0x10000u) {   // none in the tables; walked by decoding if it ever is
                    atomicOr(&s_rf[row_of(rel, nr, p)], rf_decode(fg[g]));
                    continue;
                }
            }
            if (cp == 0x3A3u) lc = (e & 0x8000u) ? 0x3C2u : 0x3C3u;
            if (lc == cp) continue;
            uint8_t o[4];
            wg_utf8_encode(lc, o);
            for (uint32_t j = 0; j < len; j++) sb[p + j] = o[j];
        }
        __syncthreads();
        for (uint32_t g = 0; g < ng; g++)
            if (tid < nr && (s_rf[tid] & (rf_mark(fg[g]) | rf_decode(fg[g]))))
                s_wrow[atomicAdd(&pc[1], 1u)] = (uint16_t)(tid | g << 8);
        // every byte position holding the query's first byte against its first 8 bytes
        for (uint32_t k = tid + (lo[0] >> 2); k < tw; k += NT) {
            const uint32_t w0 = s_buf[k];
            uint32_t cand = eq_bytes(w0, q0);
            if (!cand) continue;
            const uint32_t w1 = s_buf[k + 1], w2 = s_buf[k + 2];
            while (cand) {
                const uint32_t j = (uint32_t)__builtin_ctz(cand) >> 3;
                cand &= cand - 1;
                const uint64_t x = (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, j) |
                                   ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, j) << 32);
                const uint32_t p = 4 * k + j, g = reg(p);
                if ((x & qmask) != qv || p < lo[g] || p + m > hi[g]) continue;
                const uint32_t *rel = s_rel[g];
                const uint32_t r = row_of(rel, nr, p);
                if (p + m > rel[r + 1] || (s_rf[r] & rf_decode(fg[g]))) continue;
                bool ok = true;
                for (uint32_t i = 8; i < m && ok; i++) ok = sb[p + i] == A.q[i];
                if (ok) atomicOr(&s_rf[r], RF_HIT);
            }
        }
        __syncthreads();
        // rows with a special the query could overlap, compacted: the row's lowered stream from LDS
        // ... and the windows over each listed special: the lowered stream from
        // 3 (m - 1) bytes before it to as many after (each 3 bytes of the buffer
        // hold at least one lowered byte), entered at a byte outside a mark
        const uint32_t nwalk = pc[1], nsp = pc[3] < SPCAP ? pc[3] : SPCAP;
        for (uint32_t i = tid; i < nwalk + nsp; i += NT) {
            uint32_t row, a, b;
            bool dec = false;
            if (i >= nwalk) {
                const uint32_t p = s_spos[i - nwalk];
                const uint32_t *rel = s_rel[reg(p)];
                row = row_of(rel, nr, p);
                const uint32_t rs = rel[row], re = rel[row + 1], back = 3 * (m - 1);
                a = p - rs > back ? p - back : rs;
                while (a < p && (sb[a] == 0xFEu || (a > rs && sb[a - 1] == 0xFFu))) a++;
                b = re - p > 3 + back ? p + 3 + back : re;
            } else {
                const uint32_t e = s_wrow[i], g = e >> 8;
                row = e & 0xFFu;
                a = s_rel[g][row];
                b = s_rel[g][row + 1];
                dec = (s_rf[row] & rf_decode(fg[g])) != 0;
            }
            if (s_rf[row] & RF_HIT) continue;
            const bool h = i >= nwalk ? walk_marked(sb, a, b, special, sh) : walk_row(T, s_buf, a, b, special, marks, dec, wf);
            if (h) atomicOr(&s_rf[row], RF_HIT);
        }
    }
    __syncthreads();
    const bool live = tid < nr;
    const uint64_t r = r0 + tid;
    bool hit = live && (s_rf[tid] & RF_HIT);
    for (int f = 0; f < 2 && live && !hit; f++) {   // fields over the LDS buffer: the stream from HBM
        const uint8_t *text = f ? A.auth : A.sum;
        const uint64_t *off = f ? A.auth_off : A.sum_off;
        if (!off || !(s_rf[tid] & rf_hbm(f))) continue;
        const uint64_t s = off[r];
        WgKmp km{A.q, A.fail, m, 0};
        hit = wg_lower_stream(T, text + s, (uint32_t)(off[r + 1] - s), km);
    }
    if (live && !hit && A.qhex) {
        // the id's hex (lowercase): id starts with q, or short_id (7 digits, non-synthetic rows) contains q
        const uint8_t *id = A.oid + r * 20;
        const uint32_t w0 = (reinterpret_cast<uintptr_t>(A.oid) & 3u)
                                ? (uint32_t)id[0] | (uint32_t)id[1] << 8 | (uint32_t)id[2] << 16 | (uint32_t)id[3] << 24
                                : *reinterpret_cast<const uint32_t *>(id);
        uint64_t hex8 = 0;
        for (int i = 0; i < 4; i++) {
            const uint32_t b = (w0 >> (8 * i)) & 0xFFu;
            hex8 |= (uint64_t)hex_char(b >> 4) << (16 * i);
            hex8 |= (uint64_t)hex_char(b & 15u) << (16 * i + 8);
        }
        hit = (hex8 & qmask) == qv;
        for (uint32_t i = 8; i < m && hit; i++) {
            const uint32_t b = A.oid[r * 20 + i / 2];
            hit = hex_char((i & 1) ? (b & 15u) : (b >> 4)) == A.q[i];
        }
        if (!hit && m <= 7 && !(A.flags[r] & WG_FLAG_SYNTHETIC))
            for (uint32_t s = 1; s + m <= 7 && !hit; s++) hit = ((hex8 >> (8 * s)) & qmask) == qv;
    }
    if (live) A.out[r - A.rb] = hit ? 1 : 0;
    const int cnt = __syncthreads_count(live && hit);
    if (tid == 0 && cnt) atomicAdd(A.count + 8 * (blockIdx.x % WG_MATCH_STRIPES), (unsigned long long)cnt);
}

inline uint32_t mblocks(uint64_t n) { return (uint32_t)((n + MT - 1) / MT); }

}  // namespace

// The search kernel's table: per BMP code point its simple lowercase, Cased,
// Case_Ignorable, and whether lowering changes its UTF-8 length (the
// "specials": U+0130 -> "i̇" and the simple mappings across a UTF-8 length,
// each with its index); then per special its lowered bytes | length << 24.
static std::vector<uint32_t> wg_build_flat_table() {
    const WgCaseTables HT{h_lower, h_cased, h_ign};
    std::vector<uint32_t> t(WG_FLAT_N + WG_SPECIAL_N, 0);
    uint32_t ns = 0;
    auto entry = [&](uint32_t cp) {
        const uint32_t lc = wg_lower_simple(HT, cp);
        uint8_t b0[4], b1[4];
        const uint32_t n0 = wg_utf8_encode(cp, b0), n1 = wg_utf8_encode(lc, b1);
        uint32_t e = (lc & 0xFFFFu) | (wg_is_cased(HT, cp) ? WG_FLAT_CASED : 0u) | (wg_is_ignorable(HT, cp) ? WG_FLAT_IGN : 0u);
        if ((cp == 0x130u || lc >= WG_FLAT_N || n0 != n1) && ns < WG_SPECIAL_N) {   // 25 in the tables
            const uint32_t x = cp == 0x130u ? ('i' | 0xCCu << 8 | 0x87u << 16 | 3u << 24)
                                            : ((uint32_t)b1[0] | (n1 > 1 ? (uint32_t)b1[1] << 8 : 0u) |
                                               (n1 > 2 ? (uint32_t)b1[2] << 16 : 0u) | n1 << 24);
            t[WG_FLAT_N + ns] = x;
            e |= WG_FLAT_LENCHG | ns << WG_FLAT_SPECIAL_SHIFT;
            ns++;
        }
        t[cp] = e;
    };
    entry(0x130u);   // special 0
    for (uint32_t cp = 0; cp < WG_FLAT_N; cp++)
        if (cp != 0x130u) entry(cp);
    return t;
}

// built once per process (a function-local static: thread-safe initialisation)
const std::vector<uint32_t> &wg_match_flat_table() {
    static const std::vector<uint32_t> table = wg_build_flat_table();
    return table;
}

// The inverse of the simple lowercase mapping, {lowercase, code point} sorted,
// without the specials (their relevance is MatchArgs::spec_rel's exact test),
// and the specials' own code points by index.  Built once per process.
namespace {
struct LowerInverse {
    std::vector<std::pair<uint32_t, uint32_t>> pairs;
    uint32_t special_cp[WG_SPECIAL_N] = {};
};
const LowerInverse &lower_inverse() {
    static const LowerInverse inv = [] {
        LowerInverse v;
        const WgCaseTables HT{h_lower, h_cased, h_ign};
        const std::vector<uint32_t> &flat = wg_match_flat_table();
        for (uint32_t cp = 0x80; cp < 0x110000u; cp++) {
            if (cp >= 0xD800 && cp < 0xE000) continue;
            if (cp < WG_FLAT_N && (flat[cp] & WG_FLAT_LENCHG)) {
                v.special_cp[(flat[cp] >> WG_FLAT_SPECIAL_SHIFT) & 31u] = cp;
                continue;
            }
            const uint32_t lc = wg_lower_simple(HT, cp);
            if (lc != cp) v.pairs.emplace_back(lc, cp);
        }
        std::sort(v.pairs.begin(), v.pairs.end());
        return v;
    }();
    return inv;
}
}  // namespace

// The lead-filtered variant (r06).  A match holds the lowered text's bytes
// at the query's code points (for a well-formed query a window can only match
// at code point boundaries, every byte of the query being a lead or a
// continuation of one), so only code points whose lowering is one of the
// query's code points need lowering — those under a few lead bytes — plus
// U+03A3 when the query holds sigma (Final_Sigma decides between its two
// forms) and the specials spec_rel found relevant.  Any other code point, left
// as it is, holds bytes no window of the query can match, and so does its
// lowering.  Sets A.flt_*; flt_n = ~0 when the query is not well-formed UTF-8
// or needs more than WG_FILT_LEADS lead bytes besides 0xCE (the full variant).
static void match_lead_filter(const std::vector<uint8_t> &q, MatchArgs &A) {
    A.flt_n = 0xFFFFFFFFu;
    A.flt_ce = 0;
    for (uint8_t &b : A.flt_lead) b = 0;
    const LowerInverse &inv = lower_inverse();
    bool lead[256] = {};
    const uint32_t m = (uint32_t)q.size();
    for (uint32_t i = 0; i < m;) {
        uint32_t len;
        const uint32_t cp = wg_utf8_decode(q.data(), i, m, &len);
        if (cp & 0x80000000u) return;   // not well formed: the full variant
        i += len;
        auto it = std::lower_bound(inv.pairs.begin(), inv.pairs.end(), std::make_pair(cp, 0u));
        for (; it != inv.pairs.end() && it->first == cp; ++it) {
            uint8_t e[4];
            wg_utf8_encode(it->second, e);
            lead[e[0]] = true;
        }
        if (cp == 0x3C2u || cp == 0x3C3u) lead[0xCE] = true;   // U+03A3 (Final_Sigma)
    }
    for (uint32_t i = 0; i < WG_SPECIAL_N; i++)
        if (((A.spec_rel >> i) & 1u) && inv.special_cp[i]) {
            uint8_t e[4];
            wg_utf8_encode(inv.special_cp[i], e);
            lead[e[0]] = true;
        }
    uint32_t n = 0;
    for (uint32_t b = 0x80; b < 0x100; b++) {
        if (!lead[b] || b == 0xCE) continue;
        if (n == WG_FILT_LEADS) return;   // too many: the full variant
        A.flt_lead[n++] = (uint8_t)b;
    }
    A.flt_n = n;
    A.flt_ce = lead[0xCE] ? 1u : 0u;
}

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
    if (!c->match_flat.p) {   // once per context: the BMP's lowercase and case classes, and the specials
        const std::vector<uint32_t> &flat = wg_match_flat_table();
        WG_ALLOC(c, c->match_flat, flat.size() * 4 + 16);
        WG_HIP(c, hipMemcpyAsync(c->match_flat.p, flat.data(), flat.size() * 4, hipMemcpyHostToDevice, s));
        WG_HIP(c, hipStreamSynchronize(s));
    }
    // {the match count in WG_MATCH_STRIPES words, one per 64-byte line} + fail
    // u16[m] + q u8[m]: a workgroup adds its count to stripe blockIdx % 8 (r06:
    // ~4k same-address adds on one word queued behind the kernel's end)
    constexpr size_t QH = 64 * WG_MATCH_STRIPES;
    WG_ALLOC(c, c->match_q, QH + m * 3 + 16);
    std::vector<uint8_t> &qh = c->match_qhost;
    qh.assign(QH + (size_t)m * 3, 0);
    std::memcpy(qh.data() + QH, fail.data(), (size_t)m * 2);
    std::memcpy(qh.data() + QH + (size_t)m * 2, q.data(), m);
    WG_HIP(c, hipMemsetAsync(c->match_q.p, 0, QH, s));
    WG_HIP(c, hipMemcpyAsync(c->match_q.as<uint8_t>() + QH, qh.data() + QH, (size_t)m * 3, hipMemcpyHostToDevice, s));
    MatchArgs A;
    A.rb = rb;
    A.re = re;
    A.sum = d_txt[0];
    A.auth = d_txt[1];
    A.sum_off = d_off[0];
    A.auth_off = d_off[1];
    A.oid = c->d_oid;
    A.flags = c->d_flags;
    A.fail = reinterpret_cast<const uint16_t *>(c->match_q.as<uint8_t>() + QH);
    A.q = c->match_q.as<uint8_t>() + QH + (size_t)m * 2;
    A.m = m;
    A.qhex = m <= 40;
    A.marks = 1;
    for (uint8_t b : q) {
        A.qhex &= (b - '0' < 10u) || (b - 'a' < 6u);
        A.marks &= b < 0xFE && b >= WG_SPECIAL_N;   // a mark's bytes never in the query
    }
    A.qv = 0;
    A.qmask = m < 8 ? (1ull << (8 * m)) - 1 : ~0ull;
    for (uint32_t i = 0; i < m && i < 8; i++) A.qv |= (uint64_t)q[i] << (8 * i);
    A.qlo = A.qhi = A.mlo = A.mhi = 0;
    for (uint32_t i = 0; i < m && m <= 16; i++) {
        if (i + 8 < m) { A.qhi = (A.qhi << 8) | q[i]; A.mhi = (A.mhi << 8) | 0xFFu; }
        else { A.qlo = (A.qlo << 8) | q[i]; A.mlo = (A.mlo << 8) | 0xFFu; }
    }
    // A special can take part in a match only if its lowered bytes L and the
    // query agree wherever they overlap at some shift (L inside q, q inside L,
    // or one's prefix the other's suffix): a match holds L contiguously.  r06:
    // this exact test replaced "shares a byte" — "fix" no longer walks every
    // U+0130 (L = "i" U+0307 overlaps "fix" at no shift).
    A.spec_rel = 0;
    {
        const std::vector<uint32_t> &flat = wg_match_flat_table();
        for (uint32_t i = 0; i < WG_SPECIAL_N; i++) {
            const uint32_t x = flat[WG_FLAT_N + i], l = x >> 24;
            bool rel = false;
            for (int64_t d = -(int64_t)l + 1; d < (int64_t)m && !rel; d++) {   // L starts at q[d]
                bool ok = true;
                for (uint32_t j = 0; j < l && ok; j++) {
                    const int64_t qi = d + (int64_t)j;
                    if (qi >= 0 && qi < (int64_t)m) ok = q[(size_t)qi] == ((x >> (8 * j)) & 0xFFu);
                }
                rel = ok;
            }
            if (rel) A.spec_rel |= 1u << i;
        }
    }
    match_lead_filter(q, A);
    // the variant: 1 an ASCII query (its leads a subset of {C4, E2}: flt_n
    // becomes the selection bits), 2 other filtered queries, 0 the rest
    int mode = A.flt_n == 0xFFFFFFFFu ? 0 : 2;
    if (mode == 2 && !A.flt_ce) {
        uint32_t sel = 0;
        bool only = true;
        for (uint32_t i = 0; i < A.flt_n; i++) {
            if (A.flt_lead[i] == 0xC4u) sel |= 1u;
            else if (A.flt_lead[i] == 0xE2u) sel |= 2u;
            else only = false;
        }
        bool ascii = true;
        for (uint8_t b : q) ascii &= b < 0x80;
        if (only && ascii) {
            mode = 1;
            A.flt_n = sel;
        }
    }
    if (mode == 0) A.flt_n = 0;
    A.flat = c->match_flat.as<const uint32_t>();
    A.out = c->match_flags.as<uint8_t>();
    A.count = c->match_q.as<unsigned long long>();
    wg_stage_begin(c, "match");
    if (rows) {
        // (WPS: waves per SIMD the registers must allow — 8: four 512-thread
        // workgroups per CU, as many as their LDS allows)
#define WG_MATCH_LAUNCH(NT_, SB_, WPS_)                                                                  \
        do {                                                                                             \
            if (mode == 1) hipLaunchKernelGGL((k_match<NT_, SB_, WPS_, 1>), dim3(mblocks(rows)), dim3(NT_), 0, s, A);  \
            else if (mode == 2) hipLaunchKernelGGL((k_match<NT_, SB_, WPS_, 2>), dim3(mblocks(rows)), dim3(NT_), 0, s, A); \
            else hipLaunchKernelGGL((k_match<NT_, SB_, WPS_, 0>), dim3(mblocks(rows)), dim3(NT_), 0, s, A);            \
        } while (0)
        if (c->match_threads == 512) WG_MATCH_LAUNCH(512, 4, 8);
        else if (c->match_threads == 513) WG_MATCH_LAUNCH(512, 4, 6);
        else WG_MATCH_LAUNCH(256, 8, 1);
#undef WG_MATCH_LAUNCH
    }
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    uint64_t stripes[WG_MATCH_STRIPES] = {0};
    WgFetch fi[WG_MATCH_STRIPES];
    for (int k = 0; k < WG_MATCH_STRIPES; k++) fi[k] = WgFetch{c->match_q.as<uint8_t>() + 64 * k, true};
    const int frc = wg_fetch_n(c, WG_MATCH_STRIPES, fi, stripes);   // also orders the host copies above
    if (frc != WG_OK) return frc;
    uint64_t cnt = 0;
    for (uint64_t v : stripes) cnt += v;
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
