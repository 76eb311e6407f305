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
__global__ void k_hash_place(const uint8_t *__restrict__ oid, uint64_t n, unsigned long long *table, uint64_t mask) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
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

// ids all distinct (no insert met its own key): every row is canonical and
// the second probe pass is skipped
__global__ void k_canon(const uint8_t *__restrict__ oid, uint64_t n, const unsigned long long *__restrict__ table,
                        uint64_t mask, const uint32_t *__restrict__ dup, uint32_t *__restrict__ canon) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (*dup == 0xFFFFFFFFu) { canon[i] = (uint32_t)i; return; }
    int64_t r = hash_find(load_key(oid + i * 20), oid, table, mask);
    canon[i] = r < 0 ? (uint32_t)i : (uint32_t)r;
}

__global__ void k_probe_parents(const uint8_t *__restrict__ poid, uint64_t e, const uint8_t *__restrict__ oid,
                                const unsigned long long *__restrict__ table, uint64_t mask, int32_t *__restrict__ prow) {
    uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= e) return;
    prow[k] = (int32_t)hash_find(load_key(poid + k * 20), oid, table, mask);
}

// edges per row = parents found in the list (:306-311); lane-independent, so
// the edge offsets and the total are ready before the lanes are
__global__ void k_edge_cnt(uint64_t n, const uint32_t *__restrict__ poff, const int32_t *__restrict__ prow,
                           uint32_t *__restrict__ edge_cnt) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t cnt = 0;
    for (uint32_t k = poff[i]; k < poff[i + 1]; k++) cnt += prow[k] >= 0;
    edge_cnt[i] = cnt;
}

}  // namespace

int wg_stage_hash_join(wg_ctx *c) {
    const uint64_t n = c->n, e = c->e_refs;
    uint64_t cap = 1024;
    while (cap < 2 * n) cap <<= 1;
    c->hcap = cap;
    WG_ALLOC(c, c->hash, cap * 8 + 64);
    WG_ALLOC(c, c->canon, n * 4 + 4);
    WG_ALLOC(c, c->prow, e * 4 + 4);
    wg_stage_begin(c, "hash_join");
    // one fill: the table (empty = all ones) and, after it, the duplicate flag (all ones = none)
    WG_HIP(c, hipMemsetAsync(c->hash.p, 0xFF, cap * 8 + 4, c->stream));
    uint32_t *dup = reinterpret_cast<uint32_t *>(c->hash.as<unsigned long long>() + cap);
    const int T = 256;
    if (n) {
        hipLaunchKernelGGL(k_hash_place, dim3((n + T - 1) / T), dim3(T), 0, c->stream, c->d_oid, n,
                           c->hash.as<unsigned long long>(), cap - 1);
        hipLaunchKernelGGL(k_hash_settle, dim3((n + T - 1) / T), dim3(T), 0, c->stream, c->d_oid, n,
                           c->hash.as<unsigned long long>(), cap - 1, dup);
        hipLaunchKernelGGL(k_canon, dim3((n + T - 1) / T), dim3(T), 0, c->stream, c->d_oid, n,
                           c->hash.as<const unsigned long long>(), cap - 1, dup,
                           c->canon.as<uint32_t>());
    }
    if (e)
        hipLaunchKernelGGL(k_probe_parents, dim3((e + T - 1) / T), dim3(T), 0, c->stream, c->d_poid, e, c->d_oid,
                           c->hash.as<const unsigned long long>(), cap - 1, c->prow.as<int32_t>());
    WG_ALLOC(c, c->edge_cnt, (n + 1) * 4);
    { const int _sr = wg_scan_reserve(c, n + 1); if (_sr != WG_OK) return _sr; }
    if (n) {
        hipLaunchKernelGGL(k_edge_cnt, dim3((n + T - 1) / T), dim3(T), 0, c->stream, n, c->d_poff,
                           c->prow.as<const int32_t>(), c->edge_cnt.as<uint32_t>());
        WG_HIP(c, wg_exclusive_scan_u32(c->edge_cnt.as<uint32_t>(), c->edge_cnt.as<uint32_t>(), n, c->scan_tmp.p, c->stream));
        // read by wg_stage_edges after the lane stage's own synchronisation (a
        // speculative build reads it with its end-of-build validation)
        if (!c->spec)
            if (const int rc = wg_fetch_defer(c, {{c->edge_cnt.as<uint32_t>() + n, false}})) return rc;
    }
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}
