// wg_unicase.h — `str::to_lowercase` as a byte stream, host and device.
//
// The reference lowers the search query (commit_graph.rs:1326) and every
// searched field (:1510-1521) with Rust's `str::to_lowercase`: the Unicode
// default lowercase mapping = the simple per-code-point mapping, the
// unconditional SpecialCasing entry U+0130 -> U+0069 U+0307, and U+03A3
// -> U+03C2 in the Final_Sigma context (preceded by a Cased code point with
// only Case_Ignorable ones between, and not followed by Case_Ignorable* then
// Cased), else U+03C3.  Tables: wg_case_tables.h (generated, Unicode
// WG_UNICODE_VERSION).
//
// Input bytes are decoded as UTF-8; a byte that does not start a well-formed
// sequence (overlong, surrogate, > U+10FFFF, truncated) stands for itself:
// it is copied through and is neither Cased nor Case_Ignorable (Rust strings
// are always well formed, so this only defines the engine on other input;
// it equals Python's `surrogateescape` round trip).
#pragma once

#include <cstdint>

#include "wg_case_tables.h"

#if defined(__HIPCC__)
#define WG_HD __host__ __device__
#else
#define WG_HD
#endif

struct WgCaseTables {
    const uint32_t (*lower)[3];   // WG_LOWER_N    {lo, hi, delta<<2 | step}
    const uint32_t (*cased)[2];   // WG_CASED_N    {lo, hi}
    const uint32_t (*ign)[2];     // WG_IGNORABLE_N
    // optional: per BMP code point, its simple lowercase | Cased << 16 |
    // Case_Ignorable << 17 | lowering changes its UTF-8 length << 18 (one
    // load instead of the range searches; built from the tables above)
    const uint32_t *flat = nullptr;
};
#define WG_FLAT_N 0x10000u
#define WG_FLAT_CASED (1u << 16)
#define WG_FLAT_IGN (1u << 17)
#define WG_FLAT_LENCHG (1u << 18)
#define WG_FLAT_SPECIAL_SHIFT 19   // bits 19-23: a length-changing code point's index among the specials
#define WG_SPECIAL_N 32u

// UTF-8 decode at p[i] (i < n).  Returns the code point and its length, or
// 0x80000000 | byte with length 1 for a byte that starts no well-formed sequence.
// P: any byte source with p[i] (a pointer, or a strided LDS column)
template <class P>
WG_HD inline uint32_t wg_utf8_decode(const P &p, uint32_t i, uint32_t n, uint32_t *len) {
    const uint32_t b0 = (uint8_t)p[i];
    *len = 1;
    if (b0 < 0x80) return b0;
    uint32_t need, cp, lo = 0x80, hi = 0xBF;
    if (b0 >= 0xC2 && b0 <= 0xDF) { need = 1; cp = b0 & 0x1F; }
    else if (b0 >= 0xE0 && b0 <= 0xEF) {
        need = 2; cp = b0 & 0x0F;
        if (b0 == 0xE0) lo = 0xA0;          // overlong
        if (b0 == 0xED) hi = 0x9F;          // surrogates
    } else if (b0 >= 0xF0 && b0 <= 0xF4) {
        need = 3; cp = b0 & 0x07;
        if (b0 == 0xF0) lo = 0x90;          // overlong
        if (b0 == 0xF4) hi = 0x8F;          // > U+10FFFF
    } else {
        return 0x80000000u | b0;
    }
    if (i + need >= n) return 0x80000000u | b0;   // truncated
    for (uint32_t k = 1; k <= need; k++) {
        const uint32_t b = (uint8_t)p[i + k];
        if (b < (k == 1 ? lo : 0x80u) || b > (k == 1 ? hi : 0xBFu)) return 0x80000000u | b0;
        cp = (cp << 6) | (b & 0x3F);
    }
    *len = need + 1;
    return cp;
}

WG_HD inline uint32_t wg_utf8_encode(uint32_t cp, uint8_t *o) {
    if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
    if (cp < 0x800) { o[0] = (uint8_t)(0xC0 | (cp >> 6)); o[1] = (uint8_t)(0x80 | (cp & 0x3F)); return 2; }
    if (cp < 0x10000) {
        o[0] = (uint8_t)(0xE0 | (cp >> 12)); o[1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F));
        o[2] = (uint8_t)(0x80 | (cp & 0x3F));
        return 3;
    }
    o[0] = (uint8_t)(0xF0 | (cp >> 18)); o[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
    o[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F)); o[3] = (uint8_t)(0x80 | (cp & 0x3F));
    return 4;
}

// last range with lo <= cp, or -1
template <int W>
WG_HD inline int wg_range_find(const uint32_t (*tab)[W], int n, uint32_t cp) {
    int lo = 0, hi = n - 1, r = -1;
    while (lo <= hi) {
        const int mid = (lo + hi) >> 1;
        if (tab[mid][0] <= cp) { r = mid; lo = mid + 1; }
        else hi = mid - 1;
    }
    return r;
}

WG_HD inline uint32_t wg_lower_simple(const WgCaseTables &T, uint32_t cp) {
    if (cp < 0x80) return (cp - 'A' < 26u) ? cp + 32 : cp;
    if (T.flat && cp < WG_FLAT_N) return T.flat[cp] & 0xFFFFu;
    const int r = wg_range_find<3>(T.lower, WG_LOWER_N, cp);
    if (r < 0 || cp > T.lower[r][1]) return cp;
    const uint32_t step = T.lower[r][2] & 3u;
    if ((cp - T.lower[r][0]) % step) return cp;
    return (uint32_t)((int32_t)cp + ((int32_t)T.lower[r][2] >> 2));
}

WG_HD inline bool wg_in_ranges(const uint32_t (*tab)[2], int n, uint32_t cp) {
    const int r = wg_range_find<2>(tab, n, cp);
    return r >= 0 && cp <= tab[r][1];
}
WG_HD inline bool wg_is_cased(const WgCaseTables &T, uint32_t cp) {
    if (cp & 0x80000000u) return false;
    if (cp < 0x80) return (cp | 32u) - 'a' < 26u;
    if (T.flat && cp < WG_FLAT_N) return (T.flat[cp] & WG_FLAT_CASED) != 0;
    return wg_in_ranges(T.cased, WG_CASED_N, cp);
}
WG_HD inline bool wg_is_ignorable(const WgCaseTables &T, uint32_t cp) {
    if (cp & 0x80000000u) return false;
    if (cp < 0x80) return cp == '\'' || cp == '.' || cp == ':' || cp == '^' || cp == '`';
    if (T.flat && cp < WG_FLAT_N) return (T.flat[cp] & WG_FLAT_IGN) != 0;
    return wg_in_ranges(T.ign, WG_IGNORABLE_N, cp);
}

// the code point that ends at byte i > 0 (a code point boundary) and its start
template <class P>
WG_HD inline uint32_t wg_utf8_prev(const P &p, uint32_t i, uint32_t n, uint32_t *start) {
    uint32_t j = i - 1;
    while (j > 0 && i - j < 4 && ((uint8_t)p[j] & 0xC0) == 0x80) j--;
    uint32_t len;
    const uint32_t cp = wg_utf8_decode(p, j, n, &len);
    if (!(cp & 0x80000000u) && j + len == i) { *start = j; return cp; }
    *start = i - 1;   // byte i-1 is not the end of a well-formed sequence: it stands alone
    return 0x80000000u | (uint8_t)p[i - 1];
}

// Final_Sigma for the U+03A3 at byte i (length 2) of p[0, n)
template <class P>
WG_HD inline bool wg_final_sigma(const WgCaseTables &T, const P &p, uint32_t i, uint32_t n) {
    // before: the last non-ignorable code point in [0, i) is cased
    bool before = false;
    for (uint32_t j = i; j > 0;) {
        const uint32_t cp = wg_utf8_prev(p, j, n, &j);
        if (!wg_is_ignorable(T, cp)) { before = wg_is_cased(T, cp); break; }
    }
    if (!before) return false;
    for (uint32_t j = i + 2, len; j < n; j += len) {
        const uint32_t cp = wg_utf8_decode(p, j, n, &len);
        if (!wg_is_ignorable(T, cp)) return !wg_is_cased(T, cp);
    }
    return true;
}

// Feed the lowercase UTF-8 bytes of p[0, n) to sink(byte) -> bool (true = stop).
// Returns true when the sink stopped the stream.
template <class Sink>
WG_HD inline bool wg_lower_stream(const WgCaseTables &T, const uint8_t *p, uint32_t n, Sink &sink) {
    uint8_t buf[6];
    for (uint32_t i = 0, len; i < n; i += len) {
        const uint32_t b0 = p[i];
        if (b0 < 0x80) {   // ASCII fast path
            len = 1;
            if (sink((uint8_t)((b0 - 'A' < 26u) ? b0 + 32 : b0))) return true;
            continue;
        }
        const uint32_t cp = wg_utf8_decode(p, i, n, &len);
        uint32_t k;
        if (cp & 0x80000000u) {
            buf[0] = (uint8_t)cp;
            k = 1;
        } else if (cp == 0x130) {          // SpecialCasing: i + COMBINING DOT ABOVE
            buf[0] = 'i'; buf[1] = 0xCC; buf[2] = 0x87;
            k = 3;
        } else if (cp == 0x3A3) {          // Final_Sigma
            k = wg_utf8_encode(wg_final_sigma(T, p, i, n) ? 0x3C2u : 0x3C3u, buf);
        } else {
            k = wg_utf8_encode(wg_lower_simple(T, cp), buf);
        }
        for (uint32_t j = 0; j < k; j++)
            if (sink(buf[j])) return true;
    }
    return false;
}

// Knuth-Morris-Pratt matcher over a byte stream: q[0, m) with fail[k] = the
// longest proper border of q[0, k) (fail[0] unused).  m >= 1.
struct WgKmp {
    const uint8_t *q;
    const uint16_t *fail;
    uint32_t m, k;
    WG_HD bool operator()(uint8_t b) {
        while (k && q[k] != b) k = fail[k];
        if (q[k] == b) k++;
        return k == m;
    }
};
