// wg_lanes_refs.h — the lane fast path's per-row reference pass
// (wg_lanes_fast.hip k_lf_refs), shared with the hash join's per-row probe
// (wg_hash.hip k_probe_rows), which runs it right after resolving the row's
// parents on a single-GPU build.
#pragma once
#include "wg_internal.h"

namespace {

constexpr uint64_t REF_NONE = ~0ull;

__device__ __forceinline__ unsigned long long ref_key(uint64_t row, uint32_t kidx) {
    return ((unsigned long long)row << 16) | kidx;
}

// is parent ref k of a row (refs from pa) the first occurrence of that parent in the row's in-list refs?
__device__ __forceinline__ bool first_in_row(const int32_t *__restrict__ prow, uint32_t pa, uint32_t k, int32_t p) {
    for (uint32_t q = pa; q < k; q++)
        if (prow[q] == p) return false;
    return true;
}

// Row gi's references: the first (row, parent index) reference to every
// in-range target (atomicMin), first-parent child counts, and leaky
// references (a target at this row or earlier) into lfirst.  Returns true
// when the row makes the list "not well formed" for the fast path.
__device__ __forceinline__ bool lf_refs_row(const LfRange &R, uint64_t gi, unsigned long long *first_ref, uint32_t *fpc) {
    bool bad = R.canon && R.canon[gi] != (uint32_t)gi;
    const uint32_t pa = R.poff[gi], pb = R.poff[gi + 1];
    for (uint32_t k = pa; k < pb; k++) {
        const int32_t p = R.prow[k];
        if (p < 0) continue;
        if (k - pa > 0xFFFFu) { bad = true; continue; }
        if ((uint64_t)p <= gi) {                     // leaky: target at this row or earlier
            if (!R.lfirst) { bad = true; continue; }
            if ((uint64_t)p < R.s) continue;         // in an earlier shard: a crossing entry (LfRange::isfb)
            if (first_in_row(R.prow, pa, k, p)) atomicMin(&R.lfirst[p - R.s], ref_key(gi, k - pa));
            continue;
        }
        if ((uint64_t)p >= R.e) continue;            // beyond the shard: crossing entry
        if (!first_in_row(R.prow, pa, k, p)) continue;
        atomicMin(&first_ref[p - R.s], ref_key(gi, k - pa));
        if (k == pa) atomicAdd(&fpc[p - R.s], 1u);
    }
    return bad;
}

// the lane stage's initial state (what k_lf_clear writes), row i of n
struct LfClear {
    unsigned long long *first_ref = nullptr, *lfirst = nullptr;
    uint32_t *fpc = nullptr, *ch_fill = nullptr, *flags = nullptr, *scal = nullptr;
};
__device__ __forceinline__ void lf_clear_at(const LfClear &L, uint64_t n, uint64_t i) {
    if (i < n) L.first_ref[i] = REF_NONE;
    if (L.lfirst && i < n) L.lfirst[i] = REF_NONE;
    if (i < n + 2) { L.fpc[i] = 0u; L.ch_fill[i] = 0u; }
    if (i < 16) L.flags[i] = 0u;
    if (L.scal && i < 16) L.scal[i] = 0u;
}

}  // namespace
