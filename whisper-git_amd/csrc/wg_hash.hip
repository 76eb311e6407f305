// wg_hash.hip — oid -> row hash join on the GPU.
//
// Replaces `commit_set: HashMap<Oid, ()>` and `row_by_oid: HashMap<Oid, usize>`
// (commit_graph.rs:272-274; looked up at :306-311, :441, :448).  One
// open-addressing table in HBM, 8-byte entries {fingerprint:32 | row:32}.
// `collect()` lets the LAST occurrence of a duplicate id win (:273-274),
// reproduced with atomicMax on entries of the same key (same fingerprint,
// full 20-byte compare).  Outputs:
//   canon[i]  = last row whose id equals row i's id
//   prow[k]   = canonical row of parent reference k, or -1 if not in the list
#include "wg_internal.h"
#include "wg_hashfn.h"
#include "wg_lanes_refs.h"

namespace {

// Insert in two passes.  Place: every row writes its entry to its home slot
// with a plain 8-byte store (one of the rows sharing a home slot wins, an
// aligned 8-byte store is never torn).  Settle: a row whose home slot does not
// hold its entry probes on from there with compare-and-swap, as a one-pass
// insert would.  Memory-side atomics are the insert's cost (~20 G requests/s
// chip-wide): on a table at load <= 0.5 most rows own their home slot, so
// only the rest (~20-30%) pay a CAS, and they pay it without a plain read
// before it.  Linear probing stays valid: every slot between a key's home and
// its slot is occupied, because the place pass filled the home slots first.
//
// Two tables alternate between builds: the place pass also empties the other
// one (and its duplicate word) for the next build, so no fill launch precedes
// the join.
// (lf.first_ref set: the lane stage's initial state too, LfClear)
__global__ void k_hash_place(const uint8_t *__restrict__ oid, uint64_t n, unsigned long long *table, uint64_t mask,
                             unsigned long long *next_table, uint64_t next_words, LfClear lf) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t w = i; w < next_words; w += (uint64_t)gridDim.x * blockDim.x) next_table[w] = HEMPTY;
    if (lf.first_ref)
        for (uint64_t w = i; w < n + 16; w += (uint64_t)gridDim.x * blockDim.x) lf_clear_at(lf, n, w);
    if (i >= n) return;
    const Key k = load_key(oid + i * 20);
    table[key_hash(k) & mask] = ((unsigned long long)key_fp(k) << 32) | (uint32_t)i;
}

__global__ void k_hash_settle(const uint8_t *__restrict__ oid, uint64_t n, unsigned long long *table, uint64_t mask,
                              uint32_t *dup) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const Key k = load_key(oid + i * 20);
    const uint32_t fp = key_fp(k);
    const unsigned long long mine = ((unsigned long long)fp << 32) | (uint32_t)i;
    uint64_t h = key_hash(k) & mask;
    unsigned long long cur = table[h];
    if (cur == mine) return;   // owns its home slot
    for (uint64_t probes = 0; probes <= mask; probes++) {
        if (cur == HEMPTY) {
            const unsigned long long prev = atomicCAS(&table[h], HEMPTY, mine);
            if (prev == HEMPTY) return;
            cur = prev;
        }
        if ((uint32_t)(cur >> 32) == fp && key_eq(k, oid + (uint64_t)(uint32_t)cur * 20)) {
            atomicMax(&table[h], mine);    // same key: the last row wins (:273-274)
            atomicAnd(dup, 0u);            // the word after the table starts all ones
            return;
        }
        h = (h + 1) & mask;
        cur = table[h];
    }
}

// One thread per row: canon[i] (the row itself when no insert met its own
// key: ids all distinct), prow of the row's parent references (-1: not in
// the list, :306-311) and the row's edge count (parents found, lane-
// independent, so the edge offsets are ready before the lanes are) with the
// block's sum of it for the offsets' scan (wg_scan_bs_u32).  first_ref set:
// then the lane fast path's reference pass of the row (lf_refs_row, the
// k_lf_refs of a single-GPU build) on the parents just resolved.
__global__ void __launch_bounds__(WG_BS_THREADS) k_probe_rows(const uint8_t *__restrict__ oid, uint64_t n,
                                                             const uint32_t *__restrict__ poff, const uint8_t *__restrict__ poid,
                                                             const unsigned long long *__restrict__ table, uint64_t mask,
                                                             const uint32_t *__restrict__ dup, uint32_t *__restrict__ canon,
                                                             int32_t *__restrict__ prow, uint32_t *__restrict__ edge_cnt,
                                                             uint32_t *__restrict__ bsum, LfRange R,
                                                             unsigned long long *first_ref, uint32_t *fpc, uint32_t *viol) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t cnt = 0;
    if (i < n) {
        if (*dup == 0xFFFFFFFFu) canon[i] = (uint32_t)i;
        else {
            const int64_t r = hash_find(load_key(oid + i * 20), oid, table, mask);
            canon[i] = r < 0 ? (uint32_t)i : (uint32_t)r;
        }
        const uint32_t pa = poff[i], pb = poff[i + 1];
        for (uint32_t k = pa; k < pb; k++) {
            const int32_t p = (int32_t)hash_find(load_key(poid + (uint64_t)k * 20), oid, table, mask);
            prow[k] = p;
            cnt += p >= 0;
        }
        edge_cnt[i] = cnt;
        if (first_ref && lf_refs_row(R, i, first_ref, fpc)) atomicOr(viol, 1u);
    }
    wg_bsum_store(cnt, bsum);
}

}  // namespace

int wg_stage_hash_join(wg_ctx *c) {
    const uint64_t n = c->n, e = c->e_refs;
    uint64_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    c->hcap = cap;
    const uint64_t words = cap + 1;   // the table, then the duplicate flag word (all ones = none)
    const int t = c->htab_cur, o = t ^ 1;
    for (int k : {t, o}) {
        if (c->htab[k].cap < words * 8 + 64) c->htab_clean[k] = 0;   // (re)allocated below: not known empty
        WG_ALLOC(c, c->htab[k], words * 8 + 64);
    }
    WG_ALLOC(c, c->canon, n * 4 + 4);
    WG_ALLOC(c, c->prow, e * 4 + 4);
    WG_ALLOC(c, c->edge_cnt, (n + 1) * 4);
    WG_ALLOC(c, c->bsum, 3 * (wg_bs_blocks(n) + 64) * 4);
    { const int _sr = wg_scan_reserve(c, n + 1); if (_sr != WG_OK) return _sr; }
    wg_stage_begin(c, "hash_join");
    unsigned long long *table = c->htab[t].as<unsigned long long>();
    if (c->htab_clean[t] < words) WG_HIP(c, hipMemsetAsync(table, 0xFF, words * 8, c->stream));
    uint32_t *dup = reinterpret_cast<uint32_t *>(table + cap);
    const int T = WG_BS_THREADS;
    const uint32_t g = (uint32_t)((n + T - 1) / T);
    c->lf_refs_done = false;
    if (n) {
        // the lane fast path's clear and reference pass ride on these kernels
        // (wg_lf_refs skips its own: lf_refs_done)
        LfClear L;
        LfRange R;
        const bool lanes = !c->force_general_lanes;
        if (lanes) {
            WG_ALLOC(c, c->lf[LF_FIRST], n * 8 + 8);
            WG_ALLOC(c, c->lf[LF_LFIRST], n * 8 + 8);
            WG_ALLOC(c, c->lf[LF_FPC], (n + 2) * 4);
            WG_ALLOC(c, c->lf[LF_CHFILL], (n + 2) * 4);
            WG_ALLOC(c, c->lf[LF_FLAGS], 64);
            WG_ALLOC(c, c->lane_scalars, 64);
            L.first_ref = c->lf[LF_FIRST].as<unsigned long long>();
            L.lfirst = c->lf[LF_LFIRST].as<unsigned long long>();
            L.fpc = c->lf[LF_FPC].as<uint32_t>();
            L.ch_fill = c->lf[LF_CHFILL].as<uint32_t>();
            L.flags = c->lf[LF_FLAGS].as<uint32_t>();
            L.scal = c->lane_scalars.as<uint32_t>();
            R.s = 0;
            R.nl = n;
            R.e = n;
            R.poff = c->d_poff;
            R.prow = c->prow.as<const int32_t>();
            R.canon = c->canon.as<const uint32_t>();
            R.lfirst = L.lfirst;
        }
        hipLaunchKernelGGL(k_hash_place, dim3(g), dim3(T), 0, c->stream, c->d_oid, n, table, cap - 1,
                           c->htab[o].as<unsigned long long>(), words, L);
        c->htab_clean[o] = words;
        hipLaunchKernelGGL(k_hash_settle, dim3(g), dim3(T), 0, c->stream, c->d_oid, n, table, cap - 1, dup);
        hipLaunchKernelGGL(k_probe_rows, dim3(g), dim3(T), 0, c->stream, c->d_oid, n, c->d_poff, c->d_poid,
                           (const unsigned long long *)table, cap - 1, (const uint32_t *)dup, c->canon.as<uint32_t>(),
                           c->prow.as<int32_t>(), c->edge_cnt.as<uint32_t>(), c->bsum.as<uint32_t>(), R, L.first_ref,
                           L.fpc, L.flags);
        c->lf_refs_done = lanes;
        WgScanBs S;
        S.na = 1;
        S.in[0] = c->edge_cnt.as<const uint32_t>();
        S.out[0] = c->edge_cnt.as<uint32_t>();
        S.bsum[0] = c->bsum.as<const uint32_t>();
        WG_HIP(c, wg_scan_bs_u32(S, n, c->scan_tmp.p, c->stream));
        // read by wg_stage_edges after the lane stage's own synchronisation (a
        // speculative build reads it with its end-of-build validation)
        if (!c->spec)
            if (const int rc = wg_fetch_defer(c, {{c->edge_cnt.as<uint32_t>() + n, false}})) return rc;
    } else {
        WG_HIP(c, hipMemsetAsync(c->edge_cnt.p, 0, 4, c->stream));
    }
    c->htab_clean[t] = 0;
    c->htab_cur = o;
    c->htab_last = table;
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}
