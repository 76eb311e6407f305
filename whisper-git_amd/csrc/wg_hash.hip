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

// Parents sit a few rows below their children in a history listing (86% of
// the wide16 list's references within 16 rows, 99.9% within 64).  With every
// id distinct the row holding an id is THE row for it, so the reference pass
// runs in three kernels around the table build (which runs on the side
// stream meanwhile):
//   k_probe_near    one block per 256 rows: each reference looks for its id
//                   among the next PROBE_WIN rows' ids (staged in LDS with a
//                   fingerprint table); a miss (farther, earlier, or not in
//                   the list) is marked PROW_MISS; the first (row, index)
//                   reference and first-parent child count of every target of
//                   the block (LfRange first_ref / fpc) from the hits of the
//                   rows that can reach it, LDS atomics, one plain store per
//                   target (which is also the lane stage's clear)
//   k_probe_fix     after the table: the misses through the table (two
//                   dependent random reads each), their share of the lane
//                   pass with global atomics (as lf_refs_row), canon, the
//                   edge counts and their block sums.  Duplicate ids: the
//                   table decides every reference (the last row wins) and the
//                   list is flagged for the general lane walk.
constexpr int PROBE_WIN = 64;
constexpr int32_t PROW_MISS = -2;
constexpr int T = WG_BS_THREADS;

// k_probe_near: block b owns rows [b, b + 256) and targets [b, b + 256).
// The ids of rows [b - 63, b + 320] go to LDS with a small open-addressing
// table over their fingerprints; every row of [b - 64, b + 256) resolves its
// references against it (a hit must lie within PROBE_WIN rows below the
// child: the rows that can reach a target of this block), the block's own
// rows write prow / their hit count / the miss flag, and the hits into the
// block's targets feed the first-reference and first-parent-child counts
// with LDS atomics (rows [b - 64, b) are resolved again for that: 25% more
// lookups instead of a second kernel over prow).  A reference is first in
// its row when no earlier reference of the row has the same id.
constexpr int NR_LO = PROBE_WIN - 1;                 // rows staged below b
constexpr int NR = NR_LO + T + PROBE_WIN + 1;        // rows b - 63 .. b + 320
constexpr int NH = 1024;                             // LDS table slots (>= 2.5 x NR)
__device__ __forceinline__ uint32_t near_slot(uint32_t fp) { return (fp * 0x9E3779B1u) >> 22; }

// (fused join, r05) place: the table's place pass rides on the staging of
// the block's own rows — their ids are loaded anyway — and the next build's
// table is emptied here unless a long list's emission does it
struct NearPlace {
    unsigned long long *table = nullptr;   // null: the table is built elsewhere (side stream)
    uint64_t mask = 0;
    unsigned long long *next_table = nullptr;
    uint64_t next_words = 0;
};

__global__ void __launch_bounds__(T) k_probe_near(const uint8_t *__restrict__ oid, uint64_t n,
                                                  const uint32_t *__restrict__ poff, const uint8_t *__restrict__ poid,
                                                  int32_t *__restrict__ prow, uint32_t *__restrict__ edge_cnt,
                                                  uint8_t *__restrict__ rowmiss, LfClear L, NearPlace P) {
    __shared__ uint32_t wkey[NR * 5];
    __shared__ uint32_t htab[NH];                    // staged row index + 1, 0 empty
    __shared__ unsigned long long fr[T];
    __shared__ uint32_t fc[T];
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x;
    const int64_t r0 = (int64_t)b - NR_LO;           // staged row 0
    for (int t = threadIdx.x; t < NH; t += T) htab[t] = 0u;
    fr[threadIdx.x] = REF_NONE;
    fc[threadIdx.x] = 0u;
    __syncthreads();
    for (uint64_t w = (uint64_t)blockIdx.x * T + threadIdx.x; w < P.next_words; w += (uint64_t)gridDim.x * T)
        P.next_table[w] = HEMPTY;
    for (int t = threadIdx.x; t < NR; t += T) {
        const int64_t r = r0 + t;
        if (r < 0 || (uint64_t)r >= n) continue;
        const Key k = load_key(oid + (uint64_t)r * 20);
#pragma unroll
        for (int w = 0; w < 5; w++) wkey[t * 5 + w] = k.w[w];
        uint32_t h = near_slot(key_fp(k));
        while (atomicCAS(&htab[h], 0u, (uint32_t)t + 1u) != 0u) h = (h + 1u) & (NH - 1u);
        if (P.table && (uint64_t)r >= b && (uint64_t)r < b + T)   // the place pass for the block's own rows
            P.table[key_hash(k) & P.mask] = ((unsigned long long)key_fp(k) << 32) | (uint32_t)r;
    }
    __syncthreads();
    for (int t = threadIdx.x; t < T + PROBE_WIN; t += T) {
        const int64_t is = (int64_t)b - PROBE_WIN + t;
        if (is < 0 || (uint64_t)is >= n) continue;
        const uint64_t i = (uint64_t)is;
        const bool own = i >= b;
        const uint32_t pa = poff[i], pb = poff[i + 1];
        uint32_t cnt = 0;
        bool miss = false;
        for (uint32_t k = pa; k < pb; k++) {
            int32_t p = PROW_MISS;
            Key key{};
            if (k - pa < 64u) {
                key = load_key(poid + (uint64_t)k * 20);
                uint32_t h = near_slot(key_fp(key));
                for (uint32_t e = htab[h]; e != 0u; h = (h + 1u) & (NH - 1u), e = htab[h]) {
                    const uint32_t *q = wkey + (e - 1u) * 5;
                    if (q[0] == key.w[0] && q[1] == key.w[1] && q[2] == key.w[2] && q[3] == key.w[3] && q[4] == key.w[4]) {
                        const int64_t r = r0 + (int64_t)(e - 1u);
                        if (r > (int64_t)i && r <= (int64_t)i + PROBE_WIN) p = (int32_t)r;
                        break;
                    }
                }
            }
            if (own) {
                prow[k] = p;
                cnt += p >= 0;
                miss |= p < 0;
            }
            // the lane pass's counts for hits into this block's targets
            if (L.first_ref && p >= 0 && (uint64_t)p >= b && (uint64_t)p < b + T) {
                bool first = true;
                for (uint32_t q = pa; q < k && first; q++) first = !key_eq(key, poid + (uint64_t)q * 20);
                if (first) {
                    atomicMin(&fr[(uint64_t)p - b], ref_key(i, k - pa));
                    if (k == pa) atomicAdd(&fc[(uint64_t)p - b], 1u);
                }
            }
        }
        if (own) {
            edge_cnt[i] = cnt;
            rowmiss[i] = miss ? 1 : 0;
        }
    }
    __syncthreads();
    if (!L.first_ref) return;
    const uint64_t r = b + threadIdx.x;
    if (r < n) {
        L.first_ref[r] = fr[threadIdx.x];
        L.lfirst[r] = REF_NONE;
    }
    if (r < n + 2) {
        L.fpc[r] = r < n ? fc[threadIdx.x] : 0u;
        L.ch_fill[r] = 0u;
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x < 2 && n + threadIdx.x >= b + T) {
        L.fpc[n + threadIdx.x] = 0u;   // (the last block covers n, n + 1 unless n is a multiple of 256)
        L.ch_fill[n + threadIdx.x] = 0u;
    }
    if (blockIdx.x == 0 && threadIdx.x < 16) {
        L.flags[threadIdx.x] = 0u;
        if (L.scal) L.scal[threadIdx.x] = 0u;
    }
}

__global__ void __launch_bounds__(WG_BS_THREADS) k_probe_fix(const uint8_t *__restrict__ oid, uint64_t n,
                                                            const uint32_t *__restrict__ poff, const uint8_t *__restrict__ poid,
                                                            const unsigned long long *__restrict__ table, uint64_t mask,
                                                            const uint32_t *__restrict__ dup, uint32_t *__restrict__ canon,
                                                            int32_t *__restrict__ prow, uint32_t *__restrict__ edge_cnt,
                                                            const uint8_t *__restrict__ rowmiss, uint32_t *__restrict__ bsum,
                                                            LfClear L) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t cnt = 0;
    if (i < n) {
        // every first load before the first wait (the common row needs only these)
        const uint32_t pa = poff[i], pb = poff[i + 1], ec = edge_cnt[i], rm = rowmiss[i];
        asm volatile("" ::"v"(ec), "v"(rm));   // (held here: not sunk past the branch into a second round trip)
        if (*dup != 0xFFFFFFFFu) {
            // duplicate ids (:273-274 last write wins): the table decides every
            // reference; such a list takes the general lane walk
            const int64_t r = hash_find(load_key(oid + i * 20), oid, table, mask);
            canon[i] = r < 0 ? (uint32_t)i : (uint32_t)r;
            for (uint32_t k = pa; k < pb; k++) {
                const int32_t p = (int32_t)hash_find(load_key(poid + (uint64_t)k * 20), oid, table, mask);
                prow[k] = p;
                cnt += p >= 0;
            }
            if (L.flags && canon[i] != (uint32_t)i) atomicOr(&L.flags[0], 1u);
        } else {
            canon[i] = (uint32_t)i;
            cnt = ec;
            if (L.flags && pb - pa > 0x10000u) atomicOr(&L.flags[0], 1u);   // (lf_refs_row's bound)
            if (rm) {
                uint64_t mm = 0;   // the row's misses among its first 64 references
                for (uint32_t k = pa; k < pb; k++) {
                    if (prow[k] != PROW_MISS) continue;
                    const int32_t p = (int32_t)hash_find(load_key(poid + (uint64_t)k * 20), oid, table, mask);
                    prow[k] = p;
                    cnt += p >= 0;
                    if (k - pa < 64u) mm |= 1ull << (k - pa);
                }
                // their share of the lane pass (lf_refs_row on these references)
                if (L.first_ref)
                    for (uint32_t k = pa; k < pb; k++) {
                        if (k - pa < 64u && !(mm >> (k - pa) & 1ull)) continue;
                        const int32_t p = prow[k];
                        if (p < 0 || k - pa > 0xFFFFu || !first_in_row(prow, pa, k, p)) continue;
                        if ((uint64_t)p <= i) atomicMin(&L.lfirst[p], ref_key(i, k - pa));   // leaky
                        else {
                            atomicMin(&L.first_ref[p], ref_key(i, k - pa));
                            if (k == pa) atomicAdd(&L.fpc[p], 1u);
                        }
                    }
            }
        }
        edge_cnt[i] = cnt;
    }
    wg_bsum_store(cnt, bsum);
}

}  // namespace

// The table's buffers for this build: two tables used in turn (the next
// build's emptied by this build's place pass, or by a long list's emission
// beside its tiles when `later`); the current one is emptied first if it is
// not known empty.
static int hash_table_prepare(wg_ctx *c, unsigned long long **table, unsigned long long **next, uint64_t *words, bool *later) {
    const uint64_t n = c->n;
    // load <= 0.25 (r06; was 0.5): a quarter as many rows lose their home slot
    // to the place pass, and the settle pass's compare-and-swap chains are
    // what gates the near probe's fix-up (8 bytes per slot: 32 MB at 1M rows)
    uint64_t cap = 1024;
    while (cap < 4 * n) cap <<= 1;
    c->hcap = cap;
    *words = cap + 1;   // the table, then the duplicate flag word (all ones = none)
    const int t = c->htab_cur, o = t ^ 1;
    for (int k : {t, o}) {
        if (c->htab[k].cap < *words * 8 + 64) c->htab_clean[k] = 0;   // (re)allocated below: not known empty
        WG_ALLOC(c, c->htab[k], *words * 8 + 64);
    }
    *table = c->htab[t].as<unsigned long long>();
    *next = c->htab[o].as<unsigned long long>();
    // a clear of this table queued on the side stream by the last emission
    // (wg_hash_clear_next) completes before anything here fills it
    if (const int rc = wg_side_join(c)) return rc;
    if (c->htab_clean[t] < *words) WG_HIP(c, hipMemsetAsync(*table, 0xFF, *words * 8, c->stream));
    // the next build's table is emptied by this build, unless a long list's
    // emission will (wg_hash_clear_next, beside its tiles: 8 bytes per slot
    // off the build's critical path)
    *later = c->defer_validation && !c->sh.on && n >= c->slice_min_rows;
    if (!*later) c->htab_clean[o] = *words;
    c->htab_clean[t] = 0;
    c->htab_cur = o;
    c->htab_last = *table;
    c->hash_table = *table;
    return WG_OK;
}

// The table build (place + settle): on the side stream when the build
// forks one (wg_side_build_begin: it overlaps the window probe), else inline
int wg_hash_table_launch(wg_ctx *c) {
    const uint64_t n = c->n;
    unsigned long long *table = nullptr, *next = nullptr;
    uint64_t words = 0;
    bool later = false;
    if (const int rc = hash_table_prepare(c, &table, &next, &words, &later)) return rc;
    uint32_t *dup = reinterpret_cast<uint32_t *>(table + c->hcap);
    if (n) {
        const uint32_t g = (uint32_t)((n + T - 1) / T);
        hipLaunchKernelGGL(k_hash_place, dim3(g), dim3(T), 0, c->stream, c->d_oid, n, table, c->hcap - 1, next,
                           later ? 0ull : words, LfClear{});
        hipLaunchKernelGGL(k_hash_settle, dim3(g), dim3(T), 0, c->stream, c->d_oid, n, table, c->hcap - 1, dup);
    }
    c->hash_built = true;
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

// the next build's table (and its duplicate word) emptied on stream s, if
// the last build left it to the emission
int wg_hash_clear_next(wg_ctx *c, hipStream_t s) {
    const int o = c->htab_cur;
    const uint64_t words = c->hcap + 1;
    if (!c->hcap || c->htab_clean[o] >= words || c->htab[o].cap < words * 8) return WG_OK;
    WG_HIP(c, hipMemsetAsync(c->htab[o].p, 0xFF, words * 8, s));
    c->htab_clean[o] = words;
    if (s == c->side && c->stream != c->side) {
        // the main stream waits for the clear before the next build fills the
        // table (wg_side_join at the next fork or in hash_table_prepare)
        WG_HIP(c, hipEventRecord(c->ev_join, s));
        c->side_pending = true;
    }
    return WG_OK;
}

int wg_stage_hash_join(wg_ctx *c) {
    const uint64_t n = c->n, e = c->e_refs;
    WG_ALLOC(c, c->canon, n * 4 + 4);
    WG_ALLOC(c, c->prow, e * 4 + 4);
    WG_ALLOC(c, c->edge_cnt, (n + 1) * 4);
    WG_ALLOC(c, c->rowmiss, n + 4);
    // block sums: the edge counts' at [3 (nbs + 64), 4 (nbs + 64)), apart from
    // the lane stage's three arrays (its scan may take this one along)
    const uint64_t nbs = wg_bs_blocks(n);
    WG_ALLOC(c, c->bsum, 4 * (nbs + 64) * 4);
    uint32_t *ebs = c->bsum.as<uint32_t>() + 3 * (nbs + 64);
    c->edge_scan_pending = false;
    { const int _sr = wg_scan_reserve(c, n + 1); if (_sr != WG_OK) return _sr; }
    wg_stage_begin(c, "hash_join");
    // the table: built on the side stream already (joined below), or here —
    // fused (c->join_fused, r05): its place pass inside the window probe, the
    // settle pass between the probe and the fix-up, all on this stream
    const bool side = c->hash_built && c->hash_on_side;
    NearPlace P;
    bool fused = false;
    if (!c->hash_built) {
        if (c->join_fused && n) {
            unsigned long long *next = nullptr;
            uint64_t words = 0;
            bool later = false;
            if (const int rc = hash_table_prepare(c, &P.table, &next, &words, &later)) return rc;
            P.mask = c->hcap - 1;
            P.next_table = next;
            P.next_words = later ? 0ull : words;
            fused = true;
        } else if (const int rc = wg_hash_table_launch(c)) {
            return rc;
        }
    }
    c->hash_built = false;
    c->hash_on_side = false;
    const uint64_t cap = c->hcap;
    unsigned long long *table = c->hash_table;
    const uint32_t *dup = reinterpret_cast<const uint32_t *>(table + cap);
    const uint32_t g = (uint32_t)((n + T - 1) / T);
    c->lf_refs_done = false;
    if (n) {
        // the lane fast path's clear and reference pass ride on these kernels
        // (wg_lf_refs skips its own: lf_refs_done)
        LfClear L;
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
        }
        hipLaunchKernelGGL(k_probe_near, dim3(g), dim3(T), 0, c->stream, c->d_oid, n, c->d_poff, c->d_poid,
                           c->prow.as<int32_t>(), c->edge_cnt.as<uint32_t>(), c->rowmiss.as<uint8_t>(), L, P);
        if (fused)
            hipLaunchKernelGGL(k_hash_settle, dim3(g), dim3(T), 0, c->stream, c->d_oid, n, table, cap - 1,
                               reinterpret_cast<uint32_t *>(table + cap));
        if (side) WG_HIP(c, hipStreamWaitEvent(c->stream, c->ev_hash, 0));
        hipLaunchKernelGGL(k_probe_fix, dim3(g), dim3(T), 0, c->stream, c->d_oid, n, c->d_poff, c->d_poid,
                           (const unsigned long long *)table, cap - 1, dup, c->canon.as<uint32_t>(), c->prow.as<int32_t>(),
                           c->edge_cnt.as<uint32_t>(), (const uint8_t *)c->rowmiss.as<uint8_t>(), ebs, L);
        c->lf_refs_done = lanes;
        if (c->spec && lanes) {
            // r06: a speculative build's lane stage runs its offsets scan next
            // (wg_lf_refs, no kernel between): this scan joins that launch
            c->edge_scan_pending = true;
        } else {
            WgScanBs S;
            S.na = 1;
            S.in[0] = c->edge_cnt.as<const uint32_t>();
            S.out[0] = c->edge_cnt.as<uint32_t>();
            S.bsum[0] = ebs;
            WG_HIP(c, wg_scan_bs_u32(S, n, c->scan_tmp.p, c->stream));
        }
        // read by wg_stage_edges after the lane stage's own synchronisation (a
        // speculative build reads it with its end-of-build validation)
        if (!c->spec)
            if (const int rc = wg_fetch_defer(c, {{c->edge_cnt.as<uint32_t>() + n, false}})) return rc;
    } else {
        if (side) WG_HIP(c, hipStreamWaitEvent(c->stream, c->ev_hash, 0));
        WG_HIP(c, hipMemsetAsync(c->edge_cnt.p, 0, 4, c->stream));
    }
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}
