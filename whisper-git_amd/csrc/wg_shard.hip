// wg_shard.hip — row-sharded GraphLayout::build and row_geometry_with_bands
// (SURVEY.md §8e): one process per GPU, rank r owns the contiguous rows
// [s, e) of a commit list every rank holds in HBM, and the ranks meet at a
// few all-gather points (RCCL over xGMI through the caller's
// torch.distributed group; the engine only packs and unpacks messages).
//
// The greedy lane walk (commit_graph.rs:276-295, 401-471) is sequential over
// the whole list, but its state only changes at lane events (wg_lanes_fast.hip),
// and the references that cross a shard boundary are few (one per chain alive
// at the boundary plus the long merges).  The exchanges:
//   X1  well-formedness flags + the parent references this shard could not
//       resolve locally (child row, parent index, id)
//   X2  the rows the owning shards found for them: every rank derives the
//       same table of crossing entries (references to rows beyond the
//       child's shard), so every shard knows every waiter created before it
//   X3  event counts, per crossing entry the token of its chain (shard-local
//       event or an earlier crossing entry), and the shard's event records
//       with shard-local tokens: every rank resolves the tokens to global
//       event ids, rewrites the records in place, replays the global event
//       stream (latency-bound, ~the same cost at 8M rows as at 1M) and reads
//       its own rows' lanes from it
//       X3 also carries, per crossing entry, the row token of its child row
//       (from the child's shard) and of its parent row (from the parent's), so
//       after the replay every rank reads the far endpoints' lanes itself.
// Geometry then runs unchanged on a local problem with no exchange: the
// shard's rows between a zero-height head row (child of every edge coming from
// earlier shards) and a zero-height tail row (parent of every edge leaving
// it), with the true endpoint y of every edge supplied per edge.  row_top
// (sequential f32, :329-335 / :374-381) is computed for every row of the list
// on every rank (side stream), so a far endpoint's y is local too, and a later
// frame's geometry (new bands) takes no exchange at all.
//
// Parents at earlier rows (clock skew, orphans re-sorted by time,
// git/mod.rs:767-772) stay on this path as the single-GPU replay keeps them:
// leaky references (:441-446) whose "first" decision (LfRange::lfirst, and
// for a target in an earlier shard k_lf_xfirst with the target shard's
// WG_XF_LLEAKY bit from X2) is the same on every rank.
// Lists with duplicate ids, more than 1023 lane slots or a replay without
// fixed point fall back, on every rank alike, to the single-GPU build over the
// whole list.
#include <cstring>
#include <vector>

#include "wg_internal.h"
#include "wg_hashfn.h"

namespace {

constexpr int T = 256;
constexpr uint32_t XT_PENDING = 0xFFFFFFFEu;
inline uint32_t blocks(uint64_t n) { return (uint32_t)((n + T - 1) / T); }

// ---- X1 / X2: parent resolution ------------------------------------------------
// Local table of the shard's own rows, in the two passes of wg_hash.hip
// (place: plain store to the home slot; settle: the rows that lost their home
// slot probe on with compare-and-swap)
__global__ void k_sh_place(const uint8_t *__restrict__ oid, uint64_t s, uint64_t nl, unsigned long long *table,
                           uint64_t mask) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    const uint64_t gi = s + i;
    const Key k = load_key(oid + gi * 20);
    table[key_hash(k) & mask] = ((unsigned long long)key_fp(k) << 32) | (uint32_t)gi;
}

__global__ void k_sh_settle(const uint8_t *__restrict__ oid, uint64_t s, uint64_t nl, unsigned long long *table,
                            uint64_t mask) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    const uint64_t gi = s + i;
    const Key k = load_key(oid + gi * 20);
    const unsigned long long mine = ((unsigned long long)key_fp(k) << 32) | (uint32_t)gi;
    uint64_t h = key_hash(k) & mask;
    unsigned long long cur = table[h];
    if (cur == mine) return;
    for (uint64_t probes = 0; probes <= mask; probes++) {
        if (cur == HEMPTY) {
            const unsigned long long prev = atomicCAS(&table[h], HEMPTY, mine);
            if (prev == HEMPTY) return;
            cur = prev;
        }
        if ((uint32_t)(cur >> 32) == key_fp(k) && key_eq(k, oid + (uint64_t)(uint32_t)cur * 20)) {
            atomicMax(&table[h], mine);
            return;
        }
        h = (h + 1) & mask;
        cur = table[h];
    }
}

// every id whose partition (hash) is this rank: any id seen twice?  Same two
// passes over the partition table; a settling row that meets its own key flags
// it.  The place pass, which streams all N ids, also lists the partition's
// rows {home slot, fingerprint, row}, compacted per block into the block's own
// segment of the list (DUP_R * T entries, count in bcnt[block]: no shared
// counter), so the settle pass touches those ~N/world entries instead of
// rereading and rehashing every id.
constexpr int DUP_R = 8;   // rows per thread of the place pass
inline uint32_t dup_blocks(uint64_t n) { return (uint32_t)((n + (uint64_t)T * DUP_R - 1) / ((uint64_t)T * DUP_R)); }

__global__ void __launch_bounds__(T) k_sh_dup_place(const uint8_t *__restrict__ oid, uint64_t n, uint32_t world,
                                                    uint32_t rank, unsigned long long *table, uint64_t mask,
                                                    uint4 *__restrict__ list, uint32_t *__restrict__ bcnt) {
    __shared__ uint32_t wcnt[T / 64];
    const int lid = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint4 *seg = list + (uint64_t)blockIdx.x * (T * DUP_R);
    uint32_t run = 0;   // entries of the block so far (uniform)
    for (int r = 0; r < DUP_R; r++) {
        const uint64_t i = ((uint64_t)blockIdx.x * DUP_R + r) * T + threadIdx.x;
        bool act = false;
        uint64_t hk = 0;
        uint32_t fp = 0;
        if (i < n) {
            const Key k = load_key(oid + i * 20);
            hk = key_hash(k);
            fp = key_fp(k);
            act = (uint32_t)((hk >> 40) % world) == rank;
        }
        if (act) table[hk & mask] = ((unsigned long long)fp << 32) | (uint32_t)i;
        const uint64_t m = __ballot(act);
        if (lid == 0) wcnt[wv] = (uint32_t)__popcll(m);
        __syncthreads();
        uint32_t before = 0, total = 0;
#pragma unroll
        for (int w = 0; w < T / 64; w++) {
            const uint32_t cw = wcnt[w];
            before += w < wv ? cw : 0u;
            total += cw;
        }
        if (act) seg[run + before + __popcll(m & ((1ull << lid) - 1ull))] = make_uint4((uint32_t)(hk & mask), fp, (uint32_t)i, 0u);
        run += total;
        __syncthreads();
    }
    if (threadIdx.x == 0) bcnt[blockIdx.x] = run;
}

__global__ void __launch_bounds__(T) k_sh_dup_settle(const uint8_t *__restrict__ oid, unsigned long long *table,
                                                     uint64_t mask, const uint4 *__restrict__ list,
                                                     const uint32_t *__restrict__ bcnt, uint32_t *flags) {
    const uint4 *seg = list + (uint64_t)blockIdx.x * (T * DUP_R);
    const uint32_t cnt = bcnt[blockIdx.x];
    for (uint32_t j = threadIdx.x; j < cnt; j += T) {
        const uint4 en = seg[j];
        const unsigned long long mine = ((unsigned long long)en.y << 32) | en.z;
        uint64_t h = en.x;
        unsigned long long cur = table[h];
        if (cur == mine) continue;
        for (uint64_t probes = 0; probes <= mask; probes++) {
            if (cur == HEMPTY) {
                const unsigned long long prev = atomicCAS(&table[h], HEMPTY, mine);
                if (prev == HEMPTY) break;
                cur = prev;
            }
            if ((uint32_t)(cur >> 32) == en.y &&
                key_eq(load_key(oid + (uint64_t)en.z * 20), oid + (uint64_t)(uint32_t)cur * 20)) {
                atomicOr(&flags[1], 1u);
                break;
            }
            h = (h + 1) & mask;
            cur = table[h];
        }
    }
}

// own references against the local table, one thread per reference
// (E0 = parent_off[s], E1 = parent_off[e]: read here rather than by the host)
__global__ void k_sh_probe(uint64_t s, uint64_t e, const uint32_t *__restrict__ poff, const uint8_t *__restrict__ poid,
                           const uint8_t *__restrict__ oid, const unsigned long long *__restrict__ table,
                           uint64_t mask, int32_t *__restrict__ prow_l) {
    const uint64_t E0 = poff[s], E1 = poff[e];
    for (uint64_t k = E0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < E1; k += (uint64_t)gridDim.x * blockDim.x)
        prow_l[k - E0] = (int32_t)hash_find(load_key(poid + k * 20), oid, table, mask);
}

// per own row: count of the unresolved references; more than 2^16 parents
// flags a violation.  A parent at this row or an earlier own row is leaky: its
// row is marked in lk (its shard answers X2 with WG_XF_LLEAKY for it)
__global__ void k_sh_ucnt(uint64_t s, uint64_t nl, const uint32_t *__restrict__ poff, const int32_t *__restrict__ prow_l,
                          uint32_t *__restrict__ ucnt, uint32_t *flags, uint8_t *__restrict__ lk) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    const uint64_t E0 = poff[s];
    const uint64_t gi = s + i;
    const uint32_t pa = poff[gi], pb = poff[gi + 1];
    uint32_t nu = 0;
    bool bad = pb - pa > 0x10000u;
    for (uint32_t k = pa; k < pb; k++) {
        const int32_t r = prow_l[k - E0];
        if (r < 0) nu++;
        else if ((uint64_t)r <= gi) lk[(uint64_t)r - s] = 1;
    }
    ucnt[i] = nu;
    if (bad) atomicOr(&flags[0], 1u);
}

// unresolved reference record: {child row, parent index, id[5], 0} (32 bytes), row order
__global__ void k_sh_pack_unres(uint64_t s, uint64_t nl, const uint32_t *__restrict__ poff, const uint8_t *__restrict__ poid,
                                const int32_t *__restrict__ prow_l, const uint32_t *__restrict__ uoff,
                                uint32_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nl) return;
    const uint64_t E0 = poff[s];
    const uint64_t gi = s + i;
    const uint32_t pa = poff[gi], pb = poff[gi + 1];
    uint32_t o = uoff[i];
    for (uint32_t k = pa; k < pb; k++) {
        if (prow_l[k - E0] >= 0) continue;
        uint32_t *r = out + (uint64_t)o * 8;
        const uint32_t *src = reinterpret_cast<const uint32_t *>(poid + (uint64_t)k * 20);
        r[0] = (uint32_t)gi;
        r[1] = k - pa;
#pragma unroll
        for (int w = 0; w < 5; w++) r[2 + w] = src[w];
        r[7] = 0;
        o++;
    }
}

struct Sections {            // per-rank sections of a gathered buffer
    const uint8_t *base;
    uint64_t stride;
    uint32_t world;
    uint64_t off[17];        // prefix of entry counts, off[world] = total
};

__device__ __forceinline__ uint32_t section_of(const Sections &S, uint64_t g) {
    uint32_t r = 0;
    while (r + 1 < S.world && S.off[r + 1] <= g) r++;
    return r;
}

// found row (bit 30: an own row at or after it references it: a leaky reference)
constexpr int32_t SH_FOUND_LLEAKY = 0x40000000;
__global__ void k_sh_probe_gathered(uint64_t L, const uint32_t *__restrict__ rec, const uint8_t *__restrict__ oid,
                                    const unsigned long long *__restrict__ table, uint64_t mask, uint64_t s,
                                    const uint8_t *__restrict__ lk, int32_t *__restrict__ found) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= L) return;
    int32_t r = (int32_t)hash_find(load_key(reinterpret_cast<const uint8_t *>(rec + g * 8 + 2)), oid, table, mask);
    if (r >= 0 && lk[(uint64_t)r - s]) r |= SH_FOUND_LLEAKY;
    found[g] = r;
}

// row of every unresolved reference of every rank: the shard that owns the id found it
__global__ void k_sh_combine(Sections F, uint64_t L, const uint32_t *__restrict__ rec, int32_t *__restrict__ row,
                             uint32_t *__restrict__ xflag, uint32_t *flags) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= L) return;
    int32_t best = -1;
    for (uint32_t r = 0; r < F.world; r++) {
        const int32_t v = reinterpret_cast<const int32_t *>(F.base + r * F.stride)[g];
        best = v > best ? v : best;
    }
    row[g] = best;   // (ids are distinct when the build goes on: one rank found it)
    xflag[g] = best >= 0 ? 1u : 0u;
    (void)flags;
}

// crossing entries (every rank's resolved-elsewhere references, rank-major, row order)
__global__ void k_sh_xbuild(uint64_t L, const uint32_t *__restrict__ rec, const int32_t *__restrict__ row,
                            const uint32_t *__restrict__ xpos, uint64_t own_lo, uint64_t own_hi,
                            const uint32_t *__restrict__ poff, uint64_t E0, WgXEnt *__restrict__ xall,
                            int32_t *__restrict__ prow_l, uint32_t *__restrict__ refx) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= L || row[g] < 0) return;
    const uint32_t c = rec[g * 8], kidx = rec[g * 8 + 1];
    bool first = true;   // no earlier reference of the same row resolves to the same parent
    for (uint64_t h = g; h > 0 && rec[(h - 1) * 8] == c; h--)
        if (row[h - 1] == row[g]) first = false;
    const uint32_t x = xpos[g];
    const int32_t p = row[g] & ~SH_FOUND_LLEAKY;
    WgXEnt en;
    en.c = c;
    en.p = (uint32_t)p;
    en.kf = kidx | (first ? WG_XF_FIRST_IN_ROW : 0u) | ((row[g] & SH_FOUND_LLEAKY) ? WG_XF_LLEAKY : 0u);
    en.pad = 0;
    xall[x] = en;
    if (g >= own_lo && g < own_hi) {
        const uint64_t k = (uint64_t)poff[c] + kidx;
        prow_l[k - E0] = p;
        refx[k - E0] = x - xpos[own_lo];
    }
}

// ---- X3: chain tokens of crossing entries -> global event ids ---------------------------
// entries of rank r are [xoff[r], xoff[r+1]); a token names either an event of
// the entry's own rank or an entry of an earlier rank (depth < world)
__global__ void k_sh_resolve(uint64_t nx, uint32_t world, const uint64_t *__restrict__ xoff,
                             const uint64_t *__restrict__ evoff, const uint32_t *__restrict__ tok, uint32_t *xt) {
    for (uint64_t x = threadIdx.x; x < nx; x += blockDim.x) xt[x] = XT_PENDING;
    __syncthreads();
    for (uint32_t round = 0; round <= world; round++) {
        for (uint64_t x = threadIdx.x; x < nx; x += blockDim.x) {
            if (xt[x] != XT_PENDING) continue;
            const uint32_t v = tok[x];
            if (v == WG_TOK_NONE) { xt[x] = WG_TOK_NONE; continue; }
            if (v & WG_TOK_EV) {
                uint32_t r = 0;
                while (r + 1 < world && xoff[r + 1] <= x) r++;
                xt[x] = WG_TOK_EV | ((v & ~WG_TOK_EV) + (uint32_t)evoff[r]);
            } else {
                const uint32_t y = xt[v & ~WG_TOK_X];
                if (y != XT_PENDING) xt[x] = y;
            }
        }
        __syncthreads();
    }
}

// ---- crossing-edge endpoints (no exchange) ------------------------------------------------
__device__ __forceinline__ float node_y_of(const float *__restrict__ band, uint64_t row) {
    return band ? roundf(band[row] + WG_NODE_Y) : WG_NODE_Y;   // (:390) / build default (:341)
}

// the global tokens of every entry's child row and parent row (X3: the child's
// shard sent the first, the parent's shard the second; NONE elsewhere)
struct EndToks {
    const uint8_t *base;
    uint64_t stride, tok_a;   // rank r's ctok region at base + r stride + 16 + tok_a, its ptok region tok_a later
    uint32_t world;
};
__device__ __forceinline__ uint32_t sh_globalize(uint32_t v, uint64_t ev_base, const uint32_t *__restrict__ xt) {
    if (v == WG_TOK_NONE) return v;
    if (v & WG_TOK_EV) return WG_TOK_EV | ((v & ~WG_TOK_EV) + (uint32_t)ev_base);
    if (v & WG_TOK_X) return xt[v & ~WG_TOK_X];
    return v;
}
__global__ void k_sh_etok(EndToks E, uint64_t nx, const uint64_t *__restrict__ xoff, const uint64_t *__restrict__ evoff,
                          const uint32_t *__restrict__ xt, uint32_t *__restrict__ etok) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= nx) return;
    uint32_t r = 0;
    while (r + 1 < E.world && xoff[r + 1] <= x) r++;
    const uint8_t *reg = E.base + r * E.stride + 16 + E.tok_a;
    const uint32_t ct = sh_globalize(reinterpret_cast<const uint32_t *>(reg)[x - xoff[r]], evoff[r], xt);
    uint32_t pt = WG_TOK_NONE;
    for (uint32_t q = 0; q < E.world; q++) {
        const uint32_t v = reinterpret_cast<const uint32_t *>(E.base + q * E.stride + 16 + 2 * E.tok_a)[x];
        if (v != WG_TOK_NONE) pt = sh_globalize(v, evoff[q], xt);
    }
    etok[2 * x] = ct;
    etok[2 * x + 1] = pt;
}

// after the replay: the lanes of both endpoints of every entry
__global__ void k_sh_end_lanes(uint64_t n2, const uint32_t *__restrict__ etok, const uint16_t *__restrict__ slot_of,
                               uint32_t *__restrict__ elane) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n2) return;
    const uint32_t t = etok[i];
    elane[i] = t == WG_TOK_NONE ? 0u : (uint32_t)slot_of[t & ~WG_TOK_EV];
}

// per entry: child record {entry, lane, colour, y}, parent record {entry, lane, y, 0}
__global__ void k_sh_ends(uint64_t nx, const WgXEnt *__restrict__ xall, const uint32_t *__restrict__ elane,
                          const uint8_t *__restrict__ flags, const float *__restrict__ rt_g, const float *__restrict__ band,
                          uint4 *__restrict__ xchild, uint4 *__restrict__ xpar) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= nx) return;
    const WgXEnt en = xall[x];
    const uint32_t lc = elane[2 * x], lp = elane[2 * x + 1];
    const uint32_t col = (flags[en.c] & WG_FLAG_ORPHAN) ? (uint32_t)WG_COLOR_ORPHAN : lc % 6u;
    xchild[x] = make_uint4((uint32_t)x, lc, col, __float_as_uint(rt_g[en.c] + node_y_of(band, en.c)));
    xpar[x] = make_uint4((uint32_t)x, lp, __float_as_uint(rt_g[en.p] + node_y_of(band, en.p)), 0u);
}

// the local problem's rows: head (0), own rows (1..nl), tail (nl+1)
__global__ void k_sh_local_rows(uint64_t s, uint64_t nl, const float *__restrict__ h_g, const float *__restrict__ band_g,
                                const float *__restrict__ rt_g, float *__restrict__ h_l, float *__restrict__ band_l,
                                float *__restrict__ rt_l) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r > nl + 2) return;
    // row_top: head and first own row share rt_g[s]; tail and end share rt_g[e]
    const uint64_t g = r == 0 ? s : (r <= nl ? s + r - 1 : s + nl);
    rt_l[r] = rt_g[g];
    if (r < nl + 2) {
        const bool own = r >= 1 && r <= nl;
        h_l[r] = own ? h_g[s + r - 1] : 0.0f;
        if (band_l) band_l[r] = own ? band_g[s + r - 1] : 0.0f;
    }
}

__global__ void k_sh_in_flags(uint64_t s, const WgXEnt *__restrict__ xall, uint64_t xin_end, uint32_t *__restrict__ f) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= xin_end) return;
    f[x] = xall[x].p >= s ? 1u : 0u;
}

__global__ void k_sh_own_counts(uint64_t s, uint64_t nl, const uint32_t *__restrict__ poff, const int32_t *__restrict__ prow,
                                const uint32_t *__restrict__ in_scan, uint64_t xin_end, uint32_t *__restrict__ cnt) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nl + 2) return;
    uint32_t v = 0;
    if (r == 0) v = in_scan[xin_end];
    else if (r <= nl) {
        const uint64_t gi = s + r - 1;
        for (uint32_t k = poff[gi]; k < poff[gi + 1]; k++) v += prow[k] >= 0;
    }
    cnt[r] = v;
}

struct LocalEdgeArgs {
    uint64_t s, nl, e, xin_end, xown_begin;
    const WgXEnt *xall;
    const uint32_t *poff;
    const int32_t *prow;        // by global ref index
    const uint32_t *refx;       // by global ref index: own crossing entry (section-local)
    const uint32_t *in_scan;    // position of incoming entries
    const uint32_t *edge_off;   // local edge CSR
    const uint32_t *lane_l;
    const uint8_t *color_l;
    const float *rt_g, *band;
    const uint4 *xchild, *xpar;
    wg_edge *edges;             // local
    float2 *edge_y;
    wg_edge *own_g;             // own edges, global numbering
    uint32_t y_only;            // same layout as the last pass: the edges stand, only edge_y changes
};

__device__ __forceinline__ void far_parent(const LocalEdgeArgs &A, uint64_t p, uint64_t x, uint32_t *pl, uint32_t *plane,
                                           float *py) {
    if (p < A.s) {   // an earlier shard's row (a leaky reference): the head row, skipped by the decomposition (:526-528)
        *pl = 0;
        *plane = A.xpar[x].y;
        *py = 0.0f;
    } else if (p < A.e) {
        *pl = (uint32_t)(p - A.s + 1);
        *plane = A.lane_l[p - A.s + 1];
        *py = A.rt_g[p] + node_y_of(A.band, p);
    } else {
        *pl = (uint32_t)(A.nl + 1);
        *plane = A.xpar[x].y;
        *py = __uint_as_float(A.xpar[x].z);
    }
}

__global__ void k_sh_edges_in(LocalEdgeArgs A) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= A.xin_end) return;
    const WgXEnt en = A.xall[x];
    if (en.p < A.s) return;
    const uint32_t o = A.in_scan[x];
    uint32_t pl, plane;
    float py;
    far_parent(A, en.p, x, &pl, &plane, &py);
    A.edge_y[o] = make_float2(__uint_as_float(A.xchild[x].w), py);   // the child's shard sent its y
    if (A.y_only) return;
    wg_edge ed;
    ed.child_row = 0;
    ed.child_lane = A.xchild[x].y;
    ed.parent_row = pl;
    ed.parent_lane = plane;
    ed.color = A.xchild[x].z;
    A.edges[o] = ed;
}

__global__ void k_sh_edges_own(LocalEdgeArgs A) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.nl) return;
    const uint64_t gi = A.s + i;
    uint32_t o = A.edge_off[i + 1];
    const uint32_t n_in = A.edge_off[1];
    const uint32_t cl = A.lane_l[i + 1], col = A.color_l[i + 1];
    const float cy = A.rt_g[gi] + node_y_of(A.band, gi);
    for (uint32_t k = A.poff[gi]; k < A.poff[gi + 1]; k++) {
        const int32_t p = A.prow[k];
        if (p < 0) continue;
        uint32_t pl, plane;
        float py;
        far_parent(A, (uint64_t)p, ((uint64_t)p >= A.e || (uint64_t)p < A.s) ? A.xown_begin + A.refx[k] : 0, &pl, &plane,
                   &py);
        A.edge_y[o] = make_float2(cy, py);
        if (A.y_only) { o++; continue; }
        wg_edge ed;
        ed.child_row = (uint32_t)(i + 1);
        ed.child_lane = cl;
        ed.parent_row = pl;
        ed.parent_lane = plane;
        ed.color = col;
        A.edges[o] = ed;
        ed.child_row = (uint32_t)gi;
        ed.parent_row = (uint32_t)p;
        A.own_g[o - n_in] = ed;
        o++;
    }
}

// X1 header from the device: {violation | duplicate, unresolved references,
// E0 = parent_off[s], E1 = parent_off[e]} and the message length
__global__ void k_sh_x1_head(uint4 *__restrict__ dst, unsigned long long *__restrict__ len, const uint32_t *__restrict__ flags,
                             const uint32_t *__restrict__ ucnt_off, uint64_t nl, const uint32_t *__restrict__ poff,
                             uint64_t s, uint64_t e) {
    const uint32_t nu = ucnt_off[nl];
    *dst = make_uint4(flags[0] | flags[1], nu, poff[s], poff[e]);
    *len = 16ull + (unsigned long long)nu * 32ull;
}
// X3's header and length from the lane prelude's device words: {events,
// merge words, not well formed} (no records when not well formed)
// (+ the rank's own crossing entries [*xb, *xe) and the crossing table's
// earlier-row flag, both known only on the device at X2)
// Counts past the message's capacity (ev_cap records, aux_cap merge words)
// mark the list not well formed before the event kernel runs: it writes
// nothing (gated on flags[0]) and every rank falls back at X3.
__global__ void k_sh_x3_head(uint4 *__restrict__ dst, unsigned long long *__restrict__ len, uint32_t *__restrict__ flags,
                             const uint32_t *__restrict__ nev, const uint32_t *__restrict__ naux, uint64_t tok_b,
                             const uint32_t *__restrict__ early, const uint32_t *__restrict__ xb, const uint32_t *__restrict__ xe,
                             uint32_t spec_bit, uint64_t ev_cap, uint64_t aux_cap) {
    if ((uint64_t)nev[0] > ev_cap || (uint64_t)naux[0] > aux_cap) flags[0] |= 4u;
    const uint32_t viol = (flags[0] ? 1u : 0u) | (early[0] ? 2u : 0u), ne = nev[0], na = naux[0];
    *dst = make_uint4(ne, na, viol | spec_bit, xe[0] - xb[0]);
    *len = 16ull + tok_b + (viol ? 0ull : (unsigned long long)ne * 16ull + (unsigned long long)na * 4ull);
}
// transport slot of a message whose length is on the device: header, then the
// payload when it fits (its first 16 bytes zero otherwise); 16-byte moves
__global__ void __launch_bounds__(256) k_sh_pack_dev(uint4 *__restrict__ slot, uint64_t cap, const uint4 *__restrict__ msg,
                                                     const unsigned long long *__restrict__ len) {
    const uint64_t b = *len;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, ts = (uint64_t)gridDim.x * blockDim.x;
    if (t == 0) slot[0] = make_uint4((uint32_t)b, (uint32_t)(b >> 32), 0u, 0u);
    if (b > cap) {
        if (t == 0) slot[1] = make_uint4(0u, 0u, 0u, 0u);
        return;
    }
    for (uint64_t i = t; i < (b + 15) / 16; i += ts) slot[1 + i] = msg[i];
    if (b == 0 && t == 0) slot[1] = make_uint4(0u, 0u, 0u, 0u);
}
// transport slot: 16-byte length header, then the payload's first 16 bytes zeroed (overwritten by the payload copy)
__global__ void k_sh_slot_head(uint4 *__restrict__ dst, uint4 v) {
    dst[0] = v;
    dst[1] = make_uint4(0u, 0u, 0u, 0u);
}

__global__ void k_sh_lane_out(uint64_t s, uint64_t nl, const uint32_t *__restrict__ lane_asg, const uint8_t *__restrict__ flags,
                              uint32_t *__restrict__ lane_l, uint8_t *__restrict__ color_l) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nl + 2) return;
    if (r == 0 || r > nl) { lane_l[r] = 0; color_l[r] = 0; return; }
    const uint32_t l = lane_asg[r - 1];
    lane_l[r] = l;
    color_l[r] = (flags[s + r - 1] & WG_FLAG_ORPHAN) ? (uint8_t)WG_COLOR_ORPHAN : (uint8_t)(l % 6u);
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
// exchange points: X1 unresolved references, X2 their rows, X3 chain tokens,
// endpoint row tokens and event records (geometry passes take none)
enum { SH_IDLE = 0, SH_X1, SH_X2, SH_X3 };

static int sh_send(wg_ctx *c, uint64_t bytes, wg_shard_msg *out) {
    WG_ALLOC(c, c->sh.msg, bytes + 64);
    c->sh.msg_bytes = bytes;
    c->sh.msg_dev = false;
    out->send = c->sh.msg.p;
    out->bytes = bytes;
    out->done = 0;
    out->step = c->sh.step;
    return WG_OK;
}
// a message whose length the producing kernels write to msg_len: `cap_bytes`
// bounds it (the buffer's size); the host learns the length from the heads
static int sh_send_dev(wg_ctx *c, uint64_t cap_bytes, wg_shard_msg *out) {
    WG_ALLOC(c, c->sh.msg, cap_bytes + 64);
    WG_ALLOC(c, c->sh.msg_len, 16);
    c->sh.msg_bytes = cap_bytes;
    c->sh.msg_dev = true;
    out->send = c->sh.msg.p;
    out->bytes = WG_SHARD_BYTES_ON_DEVICE;
    out->done = 0;
    out->step = c->sh.step;
    return WG_OK;
}
static void sh_done(wg_ctx *c, wg_shard_msg *out) {
    c->sh.step = SH_IDLE;
    c->sh.build_band = nullptr;   // (build_frame's bands are the caller's: not kept past the call)
    if (!out) return;             // (a deferred check settling after the call)
    out->send = nullptr;
    out->bytes = 0;
    out->done = 1;
    out->step = 0;
}

static Sections make_sections(const void *gathered, uint64_t stride, int world, const std::vector<uint64_t> &cnt) {
    Sections S;
    S.base = reinterpret_cast<const uint8_t *>(gathered);
    S.stride = stride;
    S.world = (uint32_t)world;
    S.off[0] = 0;
    for (int r = 0; r < world; r++) S.off[r + 1] = S.off[r] + cnt[r];
    return S;
}

// per-rank 16-byte headers of a gathered buffer (from the caller's host copy when given)
static int read_headers(wg_ctx *c, const void *gathered, uint64_t stride, std::vector<uint32_t> &hdr) {
    const int W = c->sh.world;
    hdr.assign((size_t)W * 4, 0);
    if (c->sh.heads) {
        for (int r = 0; r < W; r++)
            for (int k = 0; k < 4; k++) hdr[4 * r + k] = c->sh.heads[4 * r + k];
        return WG_OK;
    }
    WgFetch it[64];
    for (int r = 0; r < W; r++)
        for (int k = 0; k < 4; k++) it[4 * r + k] = WgFetch{(const uint8_t *)gathered + r * stride + 4 * k, false};
    uint64_t v[64];
    const int rc = wg_fetch_n(c, 4 * W, it, v);
    if (rc != WG_OK) return rc;
    for (int r = 0; r < W; r++)
        for (int k = 0; k < 4; k++) hdr[4 * r + k] = (uint32_t)v[4 * r + k];
    return WG_OK;
}

// a rank's message must hold what its header announces (a mismatch would turn into reads past its slot)
static int check_len(wg_ctx *c, int r, uint64_t need, const char *what) {
    if (need > c->sh.sizes[r])
        return wg_fail(c, WG_E_INVALID, "%s: rank %d announces %llu bytes, sent %llu", what, r, (unsigned long long)need,
                       (unsigned long long)c->sh.sizes[r]);
    return WG_OK;
}

static LfRange sh_range(wg_ctx *c) {
    ShardState &S = c->sh;
    LfRange R;
    R.s = S.s;
    R.nl = S.e - S.s;
    R.e = S.e;
    R.poff = c->d_poff;
    R.prow = S.prow.as<const int32_t>() - S.E0;
    R.canon = nullptr;
    R.xall = S.xall.as<const WgXEnt>();
    R.xin_end = S.xoff[S.rank];
    R.xown_begin = S.xoff[S.rank];
    R.xown_end = S.xoff[S.rank + 1];
    R.isfb = S.isfb.as<uint8_t>() - S.E0;
    R.xsec = S.xsec.as<uint32_t>() - S.E0;
    return R;
}

static void sh_graph_width(wg_ctx *c) {
    const uint32_t vis = c->max_lane + 1 < (uint32_t)WG_LANE_COUNT_VISUAL ? c->max_lane + 1 : (uint32_t)WG_LANE_COUNT_VISUAL;
    const float gw = (float)vis * WG_LANE_W;
    c->graph_width = gw > WG_LANE_W ? gw : WG_LANE_W;
}

// lanes of the local rows (+ the two boundary rows) from the replay's lane assignment
static void sh_lane_out(wg_ctx *c) {
    ShardState &S = c->sh;
    const uint64_t nl = S.e - S.s, nloc = nl + 2;
    hipLaunchKernelGGL(k_sh_lane_out, dim3(blocks(nloc)), dim3(T), 0, c->stream, S.s, nl, c->lane_asg.as<const uint32_t>(),
                       c->d_flags, c->lane_out.as<uint32_t>(), c->color_out.as<uint8_t>());
}

// whole-list build on every rank (inputs that the sharded path does not take)
static int sh_fallback(wg_ctx *c, wg_shard_msg *out) {
    ShardState &S = c->sh;
    S.replicated = true;
    S.replay_pending = false;
    c->n = S.N;
    c->e_refs = S.Etot;
    c->edge_y = nullptr;
    int rc;
    if ((rc = wg_stage_hash_join(c)) != WG_OK) return rc;
    if ((rc = wg_stage_lanes(c, false)) != WG_OK) return rc;
    if ((rc = wg_stage_edges(c, false)) != WG_OK) return rc;
    if ((rc = wg_stage_heights(c)) != WG_OK) return rc;
    c->have_layout = true;
    c->layout_gen++;
    c->alt_heights_on = false;   // (a new built list: its own heights)
    if ((rc = wg_stage_rowtop(c, nullptr)) != WG_OK) return rc;
    if ((rc = wg_stage_geometry(c, nullptr)) != WG_OK) return rc;
    c->have_geom = true;
    S.row_base = S.s;
    if (S.build_band && (rc = wg_row_geometry(c, S.build_band, WG_DEVICE)) != WG_OK) return rc;   // (build_frame)
    sh_done(c, out);
    return WG_OK;
}

// the speculative X3 replay's words, checked with the local geometry's
// validation read: {flags[it - 1], flags[it], max_lane, slots, overflow, first
// iteration that changed nothing, and for the compacted replay the positions
// + 1, the leaks, more leaks than its snapshots hold}
constexpr int SH_REPLAY_ITEMS = 9;
static int sh_replay_items(wg_ctx *c, WgFetch *it) {
    const ShardState &S = c->sh;
    it[0] = WgFetch{S.rp_it ? S.rp_flags + S.rp_it - 1 : S.rp_flags, false};
    it[1] = WgFetch{S.rp_flags + S.rp_it, false};
    for (int k = 0; k < 7; k++) it[2 + k] = WgFetch{S.rp_scal + k, false};
    return SH_REPLAY_ITEMS;
}

static int sh_local_geometry(wg_ctx *c, const float *band_g, wg_shard_msg *out, bool allow_spec);

// the lanes of both endpoints of every crossing entry, from the replay that just ran
static void sh_end_lanes(wg_ctx *c) {
    ShardState &S = c->sh;
    const uint64_t n2 = 2 * S.xoff[S.world];
    if (n2)
        hipLaunchKernelGGL(k_sh_end_lanes, dim3(blocks(n2)), dim3(T), 0, c->stream, n2, S.etok.as<const uint32_t>(),
                           c->lf_slot_of, S.elane.as<uint32_t>());
}

// the exact replay of the gathered global events (its lanes, the endpoints' lanes)
static int sh_replay_exact(wg_ctx *c, bool *ok) {
    ShardState &S = c->sh;
    c->replay_death = S.death.as<const uint32_t>();
    const int rc = wg_lf_replay_lanes(c, sh_range(c), c->n_events, c->lf[LF_EVREC].as<const uint4>(),
                                      c->lf[LF_AUX].as<const uint32_t>(), c->lane_asg.as<uint32_t>(), ok);
    c->replay_death = nullptr;
    if (rc != WG_OK || !*ok) return rc;
    c->lane_path = 0;
    sh_graph_width(c);
    sh_lane_out(c);
    sh_end_lanes(c);
    return WG_OK;
}

// A speculative replay's words: past its blind iterations or its width -> the
// exact replay (*redo); else they are committed
static int sh_replay_check(wg_ctx *c, const uint64_t *w, bool *redo, bool *fallback) {
    ShardState &S = c->sh;
    *redo = *fallback = false;
    S.replay_pending = false;
    const bool conv = S.rp_it == 0 || w[0] == 0 || w[1] == 0;
    if (conv && !w[4] && !(S.rp_dc && w[8])) {
        ReplayRun run;
        run.it = S.rp_it;
        run.chunk = S.rp_chunk;
        run.dc = S.rp_dc;
        run.nw = S.rp_nw;
        run.warm = S.rp_warm;
        wg_lf_replay_spec_commit(c, run, (uint32_t)w[2], (uint32_t)w[3], (uint32_t)w[5], (uint32_t)w[6], (uint32_t)w[7]);
        sh_graph_width(c);
        return WG_OK;
    }
    *redo = true;
    c->spec_redo_lanes++;
    bool ok = false;
    const int rc = sh_replay_exact(c, &ok);
    if (rc == WG_OK && !ok) *fallback = true;
    return rc;
}

// The local geometry problem, with no exchange: the far endpoints' lanes from
// the replay (etok -> elane), their y from the whole list's row_top; the
// shard's rows between a head and a tail row; the unchanged geometry stages.
static int sh_local_geometry(wg_ctx *c, const float *band_g, wg_shard_msg *out, bool allow_spec) {
    ShardState &S = c->sh;
    const uint64_t s = S.s, e = S.e, nl = e - s, nloc = nl + 2, nx = S.xoff[S.world];
    hipStream_t st = c->stream;
    int rc = wg_side_join(c);
    if (rc != WG_OK) return rc;
    // the build's first pass takes the row_top the build began on the side
    // stream (its bands: none, or build_frame's); any later pass rescans
    if (!(S.rt_fresh && band_g == S.rt_band)) {
        WG_ALLOC(c, S.rt_g, (S.N + 1) * 4);
        if ((rc = wg_rowtop_run(c, S.N, S.h_g.as<const float>(), band_g, S.rt_g.as<float>(), 0)) != WG_OK) return rc;
    }
    S.rt_fresh = false;
    S.band_g = band_g;
    WG_ALLOC(c, S.xchild, nx * 16 + 16);
    WG_ALLOC(c, S.xpar, nx * 16 + 16);
    if (nx)
        hipLaunchKernelGGL(k_sh_ends, dim3(blocks(nx)), dim3(T), 0, st, nx, S.xall.as<const WgXEnt>(),
                           S.elane.as<const uint32_t>(), c->d_flags, S.rt_g.as<const float>(), band_g, S.xchild.as<uint4>(),
                           S.xpar.as<uint4>());
    // local rows
    WG_ALLOC(c, c->heights, nloc * 4 + 4);
    WG_ALLOC(c, c->g_row_top, (nloc + 1) * 4);
    if (band_g) WG_ALLOC(c, c->band, nloc * 4 + 4);
    hipLaunchKernelGGL(k_sh_local_rows, dim3(blocks(nloc + 1)), dim3(T), 0, st, s, nl, S.h_g.as<const float>(), band_g,
                       S.rt_g.as<const float>(), c->heights.as<float>(), band_g ? c->band.as<float>() : nullptr,
                       c->g_row_top.as<float>());
    // local edges: incoming (earlier shards, edge order) then own.  A later pass
    // on the same layout keeps them and rewrites only their endpoint y.
    const uint64_t xin = S.xoff[S.rank];
    const int32_t *prow = S.prow.as<const int32_t>() - S.E0;
    const bool same_layout = S.local_gen == c->layout_gen;
    // The first pass on a layout (the build's default geometry) runs
    // speculatively once an earlier pass sized the buffers: local edges sized
    // by their bounds (incoming <= the earlier shards' crossing entries, own <=
    // the shard's references), the geometry lists by capacity, one read at
    // the end (wg_layout_build's scheme).  A speculative
    // replay (X3) is checked with the same read.
    const bool spec = allow_spec && !same_layout && S.geom_spec_ready;
    if (S.replay_pending && !spec) {   // (nothing to ride on: its words now)
        WgFetch it[SH_REPLAY_ITEMS];
        uint64_t w[SH_REPLAY_ITEMS] = {0};
        sh_replay_items(c, it);
        if ((rc = wg_fetch_n(c, SH_REPLAY_ITEMS, it, w)) != WG_OK) return rc;
        bool redo = false, fb = false;
        if ((rc = sh_replay_check(c, w, &redo, &fb)) != WG_OK) return rc;
        if (fb) return sh_fallback(c, out);
        if (redo) return sh_local_geometry(c, band_g, out, false);
    }
    if (!same_layout) {
        WG_ALLOC(c, S.in_scan, (xin + 2) * 4);
        WG_ALLOC(c, c->edge_cnt, (nloc + 2) * 4);
        { const int _sr = wg_scan_reserve(c, nloc + xin + 2); if (_sr != WG_OK) return _sr; }
        WG_HIP(c, hipMemsetAsync(S.in_scan.p, 0, 8, st));
        if (xin) hipLaunchKernelGGL(k_sh_in_flags, dim3(blocks(xin)), dim3(T), 0, st, s, S.xall.as<const WgXEnt>(), xin,
                                    S.in_scan.as<uint32_t>());
        WG_HIP(c, wg_exclusive_scan_u32(S.in_scan.as<uint32_t>(), S.in_scan.as<uint32_t>(), xin, c->scan_tmp.p, st));
        hipLaunchKernelGGL(k_sh_own_counts, dim3(blocks(nloc)), dim3(T), 0, st, s, nl, c->d_poff, prow,
                           S.in_scan.as<const uint32_t>(), xin, c->edge_cnt.as<uint32_t>());
        WG_HIP(c, wg_exclusive_scan_u32(c->edge_cnt.as<uint32_t>(), c->edge_cnt.as<uint32_t>(), nloc, c->scan_tmp.p, st));
        if (spec) {
            S.local_ne = xin + (S.E1 - S.E0);   // upper bounds until the validation read
            S.local_nin = xin;
            WG_ALLOC(c, c->edges, S.local_ne * sizeof(wg_edge) + 16);
            WG_ALLOC(c, S.edge_y, S.local_ne * 8 + 16);
            WG_ALLOC(c, S.own_edges, (S.E1 - S.E0) * sizeof(wg_edge) + 16);
        } else {
            uint64_t tot[2] = {0, 0};
            if ((rc = wg_fetch(c, {{c->edge_cnt.as<uint32_t>() + nloc, false}, {c->edge_cnt.as<uint32_t>() + 1, false}},
                               tot)) != WG_OK)
                return rc;
            S.local_ne = tot[0];
            S.local_nin = tot[1];
            WG_ALLOC(c, c->edges, S.local_ne * sizeof(wg_edge) + 16);
            WG_ALLOC(c, S.edge_y, S.local_ne * 8 + 16);
            WG_ALLOC(c, S.own_edges, (S.local_ne - S.local_nin) * sizeof(wg_edge) + 16);
        }
    }
    const uint64_t ne = S.local_ne, n_in = S.local_nin;
    LocalEdgeArgs A;
    A.s = s; A.nl = nl; A.e = e; A.xin_end = xin; A.xown_begin = S.xoff[S.rank];
    A.xall = S.xall.as<const WgXEnt>();
    A.poff = c->d_poff;
    A.prow = prow;
    A.refx = S.refx.as<const uint32_t>() - S.E0;
    A.in_scan = S.in_scan.as<const uint32_t>();
    A.edge_off = c->edge_cnt.as<const uint32_t>();
    A.lane_l = c->lane_out.as<const uint32_t>();
    A.color_l = c->color_out.as<const uint8_t>();
    A.rt_g = S.rt_g.as<const float>();
    A.band = band_g;
    A.xchild = S.xchild.as<const uint4>();
    A.xpar = S.xpar.as<const uint4>();
    A.edges = c->edges.as<wg_edge>();
    A.edge_y = S.edge_y.as<float2>();
    A.own_g = S.own_edges.as<wg_edge>();
    A.y_only = same_layout ? 1u : 0u;
    if (xin) hipLaunchKernelGGL(k_sh_edges_in, dim3(blocks(xin)), dim3(T), 0, st, A);
    if (nl) hipLaunchKernelGGL(k_sh_edges_own, dim3(blocks(nl)), dim3(T), 0, st, A);
    WG_HIP(c, hipGetLastError());
    c->n = nloc;
    c->n_edges = ne;
    c->edge_y = S.edge_y.as<const float>();
    S.n_own_edges = ne - n_in;
    S.local_gen = c->layout_gen;
    const float *band_l = band_g ? c->band.as<const float>() : nullptr;
    S.geom_banded = band_g != nullptr;
    c->spec = spec;
    rc = wg_stage_geometry(c, band_l);
    c->spec = false;
    if (rc != WG_OK) return rc;
    if (spec) {
        WgFetch it[WG_GEOM_SPEC_ITEMS + 2 + SH_REPLAY_ITEMS];
        int k = wg_geom_spec_items(c, it);
        it[k++] = WgFetch{c->edge_cnt.as<uint32_t>() + nloc, false};
        it[k++] = WgFetch{c->edge_cnt.as<uint32_t>() + 1, false};
        if (S.replay_pending) k += sh_replay_items(c, it + k);
        static_assert(WG_GEOM_SPEC_ITEMS + 2 + SH_REPLAY_ITEMS <= WG_PENDING_ITEMS, "shard geometry words exceed a pending build's");
        if (c->defer_validation) {
            // no host read: the words ride on the emission's vertex-total read
            // (the emission is gated on the pass's overflow words, as after a
            // deferred single-GPU build; graph_width from the device while the
            // replay is unchecked); any host query settles them first
            PendingBuild &P = c->pend;
            P = PendingBuild{};
            P.build = true;
            P.shard = true;
            P.k = k;
            for (int i = 0; i < k; i++) P.it[i] = it[i];
            c->have_geom = true;
            if (out) sh_done(c, out);
            return WG_OK;
        }
        uint64_t v[WG_GEOM_SPEC_ITEMS + 2 + SH_REPLAY_ITEMS] = {0};
        if ((rc = wg_fetch_n(c, k, it, v)) != WG_OK) return rc;
        bool redo = false;
        if ((rc = wg_shard_geom_validate(c, v, &redo)) != WG_OK) return rc;
        if (c->sh.replicated) { if (out) sh_done(c, out); return WG_OK; }   // (the replay fell back)
    }
    S.geom_spec_ready = c->lists_gen == c->layout_gen;
    c->have_geom = true;
    if (out) sh_done(c, out);
    return WG_OK;
}

// the speculative local geometry pass's words (WG_GEOM_SPEC_ITEMS, then the
// local edge count and the incoming edges' count): the counts, and past a
// capacity the exact pass (the local edges are in place)
int wg_shard_geom_validate(wg_ctx *c, const uint64_t *v, bool *redo) {
    ShardState &S = c->sh;
    *redo = false;
    if (S.replay_pending) {   // the speculative replay first: new lanes redo the local geometry exactly
        bool rr = false, fb = false;
        int rc = sh_replay_check(c, v + WG_GEOM_SPEC_ITEMS + 2, &rr, &fb);
        if (rc != WG_OK) return rc;
        if (fb) {
            *redo = true;
            return sh_fallback(c, nullptr);
        }
        if (rr) {
            *redo = true;
            c->spec_redo_geom++;
            c->lists_gen = ~0ull;
            S.local_gen = ~0ull;
            S.rt_fresh = true;   // (row_top does not depend on the lanes)
            S.rt_band = S.band_g;
            return sh_local_geometry(c, S.band_g, nullptr, false);
        }
    }
    S.local_ne = v[WG_GEOM_SPEC_ITEMS];
    S.local_nin = v[WG_GEOM_SPEC_ITEMS + 1];
    c->n_edges = S.local_ne;
    S.n_own_edges = S.local_ne - S.local_nin;
    if (!wg_geom_spec_check(c, v)) {
        *redo = true;
        c->spec_redo_geom++;
        c->lists_gen = ~0ull;
        const int rc = wg_stage_geometry(c, S.geom_banded ? c->band.as<const float>() : nullptr);
        if (rc != WG_OK) return rc;
    }
    S.geom_spec_ready = c->lists_gen == c->layout_gen;
    return WG_OK;
}

extern "C" {

static int shard_build_impl(wg_ctx *c, const wg_commits *in, int world, int rank, uint64_t row_begin, uint64_t row_end,
                            const float *band, int32_t band_res, wg_shard_msg *out);

int wg_shard_build_begin(wg_ctx *c, const wg_commits *in, int world, int rank, uint64_t row_begin, uint64_t row_end,
                         wg_shard_msg *out) {
    if (!c || !in || !out) return WG_E_INVALID;
    WG_SETTLE(c);
    return shard_build_impl(c, in, world, rank, row_begin, row_end, nullptr, WG_DEVICE, out);
}

int wg_shard_build_frame_begin(wg_ctx *c, const wg_commits *in, int world, int rank, uint64_t row_begin, uint64_t row_end,
                               const float *band, int32_t band_res, wg_shard_msg *out) {
    if (!c || !in || !out || !band) return WG_E_INVALID;
    WG_SETTLE(c);
    if (band_res != WG_HOST && band_res != WG_DEVICE) return wg_fail(c, WG_E_INVALID, "bad residency %d", band_res);
    return shard_build_impl(c, in, world, rank, row_begin, row_end, band, band_res, out);
}

static int shard_build_impl(wg_ctx *c, const wg_commits *in, int world, int rank, uint64_t row_begin, uint64_t row_end,
                            const float *band, int32_t band_res, wg_shard_msg *out) {
    c->lf_refs_done = false;   // (only a single-GPU hash join does the lane references)
    c->build_banded = false;
    if (world < 1 || world > 16 || rank < 0 || rank >= world) return wg_fail(c, WG_E_INVALID, "bad world/rank %d/%d", world, rank);
    if (in->residency != WG_DEVICE) return wg_fail(c, WG_E_INVALID, "sharded builds take device-resident commits");
    const uint64_t N = in->n_commits;
    if (row_begin > row_end || row_end > N) return wg_fail(c, WG_E_INVALID, "row range outside the list");
    (void)hipSetDevice(c->device);
    ShardState &S = c->sh;
    S.on = true;
    S.replicated = false;
    S.world = world;
    S.rank = rank;
    S.N = N;
    S.s = row_begin;
    S.e = row_end;
    S.Etot = in->n_parents;
    S.row_base = 1;
    c->have_layout = c->have_geom = c->have_vtx = c->have_text = false;
    c->lists_gen = ~0ull;
    c->edge_y = nullptr;
    c->d_oid = in->oid;
    c->match_on = false;   // match flags belong to the previous commit list
    c->d_time = in->time;
    c->d_poff = in->parent_off;
    c->d_poid = in->parent_oid;
    if (in->flags) c->d_flags = in->flags;
    else {
        WG_ALLOC(c, c->in_flags, N + 4);
        WG_HIP(c, hipMemsetAsync(c->in_flags.p, 0, N + 4, c->stream));
        c->d_flags = c->in_flags.as<uint8_t>();
    }
    c->n = N;
    c->e_refs = S.Etot;
    c->replay_shape(N);   // (the whole list's length: every rank makes the same replay choices)
    hipStream_t st = c->stream;
    S.rt_fresh = false;
    S.build_band = nullptr;
    S.replay_pending = false;
    if (band && N) {   // build_frame: the bands, on the device (a host band copied before the side fork)
        if (band_res == WG_HOST) {
            WG_ALLOC(c, S.band_host, N * 4 + 4);
            WG_HIP(c, hipMemcpyAsync(S.band_host.p, band, N * 4, hipMemcpyHostToDevice, st));
            S.build_band = S.band_host.as<const float>();
        } else {
            S.build_band = band;
        }
    }
    if (world == 1) {
        uint64_t eo[2] = {0, 0};
        if (N) {
            const int frc = wg_fetch(c, {{c->d_poff + row_begin, false}, {c->d_poff + row_end, false}}, eo);
            if (frc != WG_OK) return frc;
        }
        S.E0 = eo[0];
        S.E1 = eo[1];
        c->e_refs_own = S.E1 - S.E0;
        return sh_fallback(c, out);
    }
    // The shard's reference range [E0, E1) = parent_off[s], parent_off[e] is
    // read with this segment's closing read: reading it first would wait for
    // the previous step's emission and leave the GPU idle while this
    // segment's kernels are queued.  Until then the own references' rows are
    // sized by the list's reference count and indexed from parent_off[s] on
    // the device.
    const uint64_t nl = row_end - row_begin, El = S.Etot;
    // heights and row_top of every row of the list (zero bands, or
    // build_frame's): side stream, overlapping the exchanges; the crossing
    // edges' far endpoints read their y from it
    c->n_list = N;
    WG_ALLOC(c, S.h_g, N * 4 + 4);
    WG_ALLOC(c, S.rt_g, (N + 1) * 4);
    int rc = wg_side_zero_rowtop(c, N, S.h_g.as<float>(), S.rt_g.as<float>(), 0, S.build_band);
    if (rc != WG_OK) return rc;
    S.rt_fresh = true;
    S.rt_band = S.build_band;
    // ---- local table, probes, global duplicate scan -------------------------------------
    // (load <= 0.25, as the single-GPU table since r06: fewer rows lose their
    // home slot to the place passes, shorter compare-and-swap chains in settle)
    uint64_t cap = 1024;
    while (cap < 4 * nl) cap <<= 1;
    uint64_t pcap = 1024;
    while (pcap < 4 * (N / world + 1) + 1024) pcap <<= 1;
    WG_ALLOC(c, c->hash, cap * 8);
    WG_ALLOC(c, S.ptable, pcap * 8);
    WG_ALLOC(c, S.dlist, (uint64_t)dup_blocks(N) * (T * DUP_R * 16 + 4) + 16);
    WG_ALLOC(c, S.prow, El * 4 + 4);
    WG_ALLOC(c, S.xcnt, (nl + 2) * 4);
    WG_ALLOC(c, S.lk, nl + 16);
    WG_ALLOC(c, S.flags, 64);
    { const int _sr = wg_scan_reserve(c, nl + 2); if (_sr != WG_OK) return _sr; }
    wg_stage_begin(c, "hash_join");
    WG_HIP(c, hipMemsetAsync(c->hash.p, 0xFF, cap * 8, st));
    WG_HIP(c, hipMemsetAsync(S.ptable.p, 0xFF, pcap * 8, st));
    WG_HIP(c, hipMemsetAsync(S.flags.p, 0, 64, st));
    WG_HIP(c, hipMemsetAsync(S.lk.p, 0, nl + 16, st));
    if (nl) hipLaunchKernelGGL(k_sh_place, dim3(blocks(nl)), dim3(T), 0, st, c->d_oid, row_begin, nl,
                               c->hash.as<unsigned long long>(), cap - 1);
    const uint32_t nbd = dup_blocks(N);
    uint32_t *bcnt = reinterpret_cast<uint32_t *>(S.dlist.as<uint4>() + (uint64_t)nbd * T * DUP_R);
    if (N) hipLaunchKernelGGL(k_sh_dup_place, dim3(nbd), dim3(T), 0, st, c->d_oid, N, (uint32_t)world, (uint32_t)rank,
                              S.ptable.as<unsigned long long>(), pcap - 1, S.dlist.as<uint4>(), bcnt);
    if (nl) hipLaunchKernelGGL(k_sh_settle, dim3(blocks(nl)), dim3(T), 0, st, c->d_oid, row_begin, nl,
                               c->hash.as<unsigned long long>(), cap - 1);
    if (N) hipLaunchKernelGGL(k_sh_dup_settle, dim3(nbd), dim3(T), 0, st, c->d_oid, S.ptable.as<unsigned long long>(),
                              pcap - 1, S.dlist.as<const uint4>(), (const uint32_t *)bcnt, S.flags.as<uint32_t>());
    if (nl) {
        hipLaunchKernelGGL(k_sh_probe, dim3(blocks(nl + nl / 2)), dim3(T), 0, st, row_begin, row_end, c->d_poff, c->d_poid,
                           c->d_oid, c->hash.as<const unsigned long long>(), cap - 1, S.prow.as<int32_t>());
        hipLaunchKernelGGL(k_sh_ucnt, dim3(blocks(nl)), dim3(T), 0, st, row_begin, nl, c->d_poff,
                           S.prow.as<const int32_t>(), S.xcnt.as<uint32_t>(), S.flags.as<uint32_t>(), S.lk.as<uint8_t>());
    }
    WG_HIP(c, wg_exclusive_scan_u32(S.xcnt.as<uint32_t>(), S.xcnt.as<uint32_t>(), nl, c->scan_tmp.p, st));
    c->hcap = cap;
    S.step = SH_X1;
    // X1: {violation | duplicate, n, E0, E1} + one 32-byte record per unresolved
    // reference, row order.  Nothing is read back here: the header and the
    // length are written on the device, bounded by the list's references, and
    // this rank learns its own counts from the gathered heads (X1 exchange).
    rc = sh_send_dev(c, 16 + El * 32, out);
    if (rc != WG_OK) return rc;
    hipLaunchKernelGGL(k_sh_x1_head, dim3(1), dim3(1), 0, st, S.msg.as<uint4>(), S.msg_len.as<unsigned long long>(),
                       (const uint32_t *)S.flags.as<uint32_t>(), (const uint32_t *)S.xcnt.as<uint32_t>(), nl, c->d_poff,
                       row_begin, row_end);
    if (nl) hipLaunchKernelGGL(k_sh_pack_unres, dim3(blocks(nl)), dim3(T), 0, st, row_begin, nl, c->d_poff, c->d_poid,
                               S.prow.as<const int32_t>(), S.xcnt.as<const uint32_t>(),
                               reinterpret_cast<uint32_t *>(S.msg.as<uint8_t>() + 16));
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}

int wg_shard_msg_bytes(wg_ctx *c, uint64_t *out) {
    if (!c || !out) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->sh.msg_dev) { *out = c->sh.msg_bytes; return WG_OK; }
    (void)hipSetDevice(c->device);
    uint64_t b = 0;
    if (const int rc = wg_fetch(c, {{c->sh.msg_len.p, true}}, &b)) return rc;
    if (b > c->sh.msg_bytes) return wg_fail(c, WG_E_INVALID, "message length %llu beyond its buffer", (unsigned long long)b);
    *out = b;
    return WG_OK;
}

int wg_shard_copy_msg(wg_ctx *c, void *dst) {
    if (!c) return WG_E_INVALID;
    WG_SETTLE(c);
    uint64_t b = 0;
    if (const int rc = wg_shard_msg_bytes(c, &b)) return rc;
    if (!dst && b) return WG_E_INVALID;
    if (b) WG_HIP(c, hipMemcpyAsync(dst, c->sh.msg.p, b, hipMemcpyDefault, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

int wg_shard_pack_slot(wg_ctx *c, void *slot, uint64_t cap) {
    // k_sh_slot_head writes 32 bytes (slot header + the first 16 message bytes, zero when the message is
    // longer than the slot) and the receivers read 16-byte vectors: cap is a multiple of 16, >= 16
    if (!c || !slot || (reinterpret_cast<uintptr_t>(slot) & 15u) || cap < 16 || (cap & 15u)) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->sh.on || c->sh.step == SH_IDLE) return wg_fail(c, WG_E_STATE, "no sharded call in progress");
    (void)hipSetDevice(c->device);
    if (c->sh.msg_dev) {   // length on the device: one kernel writes the header and copies what fits
        const uint64_t nvec = std::min(cap, c->sh.msg_bytes + 15) / 16 + 1;
        const uint64_t g = std::max<uint64_t>(1, std::min<uint64_t>((nvec + 255) / 256, 1024));
        hipLaunchKernelGGL(k_sh_pack_dev, dim3((uint32_t)g), dim3(256), 0, c->stream, static_cast<uint4 *>(slot), cap,
                           c->sh.msg.as<const uint4>(), c->sh.msg_len.as<const unsigned long long>());
        WG_HIP(c, hipGetLastError());
        return WG_OK;
    }
    const uint64_t b = c->sh.msg_bytes;
    hipLaunchKernelGGL(k_sh_slot_head, dim3(1), dim3(1), 0, c->stream, static_cast<uint4 *>(slot),
                       make_uint4((uint32_t)b, (uint32_t)(b >> 32), 0u, 0u));
    if (b && b <= cap)
        WG_HIP(c, hipMemcpyAsync(static_cast<uint8_t *>(slot) + 16, c->sh.msg.p, b, hipMemcpyDeviceToDevice, c->stream));
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

int wg_shard_slot_heads(wg_ctx *c, const void *gathered, uint64_t stride, int world, uint64_t *out) {
    // every slot is read up to byte 32 (length header + the message's 16-byte header): slots of
    // wg_shard_pack_slot, stride = cap + 16 with cap a multiple of 16, >= 16
    if (!c || !gathered || !out || world < 1 || 3 * world > 64 || (reinterpret_cast<uintptr_t>(gathered) & 15u) ||
        stride < 32 || (stride & 15u))
        return WG_E_INVALID;
    WG_SETTLE(c);
    (void)hipSetDevice(c->device);
    WgFetch it[64];
    const uint8_t *g = static_cast<const uint8_t *>(gathered);
    for (int r = 0; r < world; r++) {
        it[3 * r] = WgFetch{g + r * stride, true};            // slot length
        it[3 * r + 1] = WgFetch{g + r * stride + 16, true};   // the message's 16-byte header
        it[3 * r + 2] = WgFetch{g + r * stride + 24, true};
    }
    return wg_fetch_n(c, 3 * world, it, out);
}

int wg_shard_exchange(wg_ctx *c, const void *gathered, uint64_t stride, const uint64_t *sizes, const uint32_t *heads,
                      wg_shard_msg *out) {
    if (!c || !out || !sizes) return WG_E_INVALID;
    WG_SETTLE(c);
    ShardState &S = c->sh;
    S.heads = heads;   // valid for this call only
    S.sizes = sizes;
    struct ClearHeads { ShardState &S; ~ClearHeads() { S.heads = nullptr; S.sizes = nullptr; } } clear_heads{S};
    const int W = S.world;
    if (!S.on || S.step == SH_IDLE) return wg_fail(c, WG_E_STATE, "no sharded call in progress");
    for (int r = 0; r < W; r++)
        if (sizes[r] > stride) return wg_fail(c, WG_E_INVALID, "message %d longer than the stride", r);
    if (!gathered && stride) return wg_fail(c, WG_E_INVALID, "null gathered buffer");
    (void)hipSetDevice(c->device);
    hipStream_t st = c->stream;
    const uint64_t s = S.s, e = S.e, nl = e - s, El = S.E1 - S.E0;
    int rc;
    switch (S.step) {
    case SH_X1: {   // everyone's unresolved references -> rows this shard owns
        std::vector<uint32_t> hdr;
        if ((rc = read_headers(c, gathered, stride, hdr)) != WG_OK) return rc;
        // this rank's own reference range and unresolved count came back in its header
        S.E0 = hdr[4 * S.rank + 2];
        S.E1 = hdr[4 * S.rank + 3];
        S.n_unres = hdr[4 * S.rank + 1];
        if (S.E1 < S.E0 || S.E1 > S.Etot)
            return wg_fail(c, WG_E_INVALID, "X1 header of rank %d: references [%llu, %llu) of %llu (%u %u %u %u / %u %u %u %u)",
                           S.rank, (unsigned long long)S.E0, (unsigned long long)S.E1, (unsigned long long)S.Etot,
                           hdr[0], hdr[1], hdr[2], hdr[3], hdr[4], hdr[5], hdr[6], hdr[7]);
        c->e_refs_own = S.E1 - S.E0;
        S.uoffs.assign(W + 1, 0);
        bool bad = false;
        for (int r = 0; r < W; r++) {
            bad |= hdr[4 * r] != 0;
            S.uoffs[r + 1] = S.uoffs[r] + hdr[4 * r + 1];
            if (!bad && (rc = check_len(c, r, 16 + (uint64_t)hdr[4 * r + 1] * 32, "X1 unresolved references")) != WG_OK)
                return rc;
        }
        if (bad) return sh_fallback(c, out);
        const uint64_t L = S.uoffs[W];
        WG_ALLOC(c, S.unres, L * 32 + 32);      // every rank's records, compacted (one launch)
        {
            WgCopies cp;
            for (int r = 0; r < W; r++)
                cp.add(S.unres.as<uint8_t>() + S.uoffs[r] * 32, (const uint8_t *)gathered + r * stride + 16,
                       (uint64_t)hdr[4 * r + 1] * 32);
            if ((rc = wg_copy_batch(c, cp, st)) != WG_OK) return rc;
        }
        S.step = SH_X2;
        if ((rc = sh_send(c, L * 4, out)) != WG_OK) return rc;
        if (L) hipLaunchKernelGGL(k_sh_probe_gathered, dim3(blocks(L)), dim3(T), 0, st, L, S.unres.as<const uint32_t>(),
                                  c->d_oid, c->hash.as<const unsigned long long>(), c->hcap - 1, S.s,
                                  (const uint8_t *)S.lk.as<uint8_t>(), S.msg.as<int32_t>());
        WG_HIP(c, hipGetLastError());
        return WG_OK;
    }
    case SH_X2: {   // rows of every unresolved reference -> crossing table; lanes up to the chain tokens
        const uint64_t L = S.uoffs[W];
        for (int r = 0; r < W; r++)
            if ((rc = check_len(c, r, L * 4, "X2 rows")) != WG_OK) return rc;
        std::vector<uint64_t> dummy(W, 0);
        Sections SF = make_sections(gathered, stride, W, dummy);
        WG_ALLOC(c, S.xt, L * 4 + 16);         // row per record
        WG_ALLOC(c, S.xtok, (L + 2) * 4);      // crossing flag -> position
        WG_ALLOC(c, S.refx, El * 4 + 4);
        { const int _sr = wg_scan_reserve(c, L + 2); if (_sr != WG_OK) return _sr; }
        WG_HIP(c, hipMemsetAsync(S.xtok.p, 0, 8, st));
        if (L) hipLaunchKernelGGL(k_sh_combine, dim3(blocks(L)), dim3(T), 0, st, SF, L, S.unres.as<const uint32_t>(),
                                  S.xt.as<int32_t>(), S.xtok.as<uint32_t>(), S.flags.as<uint32_t>() + 4);
        WG_HIP(c, wg_exclusive_scan_u32(S.xtok.as<uint32_t>(), S.xtok.as<uint32_t>(), L, c->scan_tmp.p, st));
        // No host read: the crossing table is sized by the L records, the
        // rank's own entries [xtok[uoffs[rank]], xtok[uoffs[rank + 1]]) stay on
        // the device (LfRange::xb_dev), and their count and the earlier-row
        // flag travel in X3's header (every rank learns xoff from the heads
        // and falls back at X3 on the flag)
        WG_ALLOC(c, S.xall, L * sizeof(WgXEnt) + 16);
        if (L) hipLaunchKernelGGL(k_sh_xbuild, dim3(blocks(L)), dim3(T), 0, st, L, S.unres.as<const uint32_t>(),
                                  S.xt.as<const int32_t>(), S.xtok.as<const uint32_t>(), S.uoffs[S.rank], S.uoffs[S.rank + 1],
                                  c->d_poff, S.E0, S.xall.as<WgXEnt>(), S.prow.as<int32_t>(), S.refx.as<uint32_t>());
        WG_ALLOC(c, S.isfb, El + 16);
        WG_ALLOC(c, S.xsec, El * 4 + 16);
        WG_HIP(c, hipMemsetAsync(S.isfb.p, 0, El + 16, st));
        WG_ALLOC(c, c->lane_scalars, 64);
        WG_HIP(c, hipMemsetAsync(c->lane_scalars.p, 0, 64, st));
        S.xoff.assign(W + 1, 0);   // known from X3's heads
        LfRange R = sh_range(c);
        R.xin_end = L;          // bounds; the kernels read the device values
        R.xown_begin = 0;
        R.xown_end = L;
        R.xb_dev = S.xtok.as<const uint32_t>() + S.uoffs[S.rank];
        R.xe_dev = S.xtok.as<const uint32_t>() + S.uoffs[S.rank + 1];
        WG_ALLOC(c, c->lf[LF_LFIRST], nl * 8 + 8);
        R.lfirst = c->lf[LF_LFIRST].as<unsigned long long>();   // parents at earlier own rows (leaky)
        wg_stage_begin(c, "lanes");
        // The message (header, tokens, then the event records and merge-token
        // lists) is bounded by the rows' references (a row makes at most
        // max(1, parents) events) and by the L records (tokens; every
        // reference arriving from an earlier shard is one of them and adds a
        // waiter to a merge here, so the merge lists hold at most
        // 2 (n + E + L) + 16 words — ADVICE r03: without L a high fan-in
        // root in a small last shard overran the message), and its header and
        // length are written on the device, as X1's are; every rank learns the
        // counts from the gathered heads.  Not well formed (or past those
        // bounds: k_sh_x3_head): no records, every rank falls back at X3.
        if ((rc = wg_lf_refs(c, R, false)) != WG_OK) return rc;
        if ((rc = wg_lf_chain(c, R)) != WG_OK) return rc;
        wg_stage_end(c);
        // token regions (each L words, 16-byte aligned, the same on every rank):
        // own entries' chain tokens, own entries' child row tokens, parent row
        // tokens by global entry; then the records
        const uint64_t tok_a = (L * 4 + 15) & ~15ull, tok_b = 3 * tok_a;
        const uint64_t ev_cap = nl + El, aux_cap = 2 * (nl + El + L) + 16;
        S.step = SH_X3;
        if ((rc = sh_send_dev(c, 16 + tok_b + ev_cap * 16 + aux_cap * 4, out)) != WG_OK) return rc;
        hipLaunchKernelGGL(k_sh_x3_head, dim3(1), dim3(1), 0, st, S.msg.as<uint4>(), S.msg_len.as<unsigned long long>(),
                           c->lf[LF_FLAGS].as<uint32_t>(), c->lf[LF_EVOFF].as<const uint32_t>() + nl,
                           c->lf[LF_AUXOFF].as<const uint32_t>() + nl, tok_b, S.flags.as<const uint32_t>() + 4, R.xb_dev,
                           R.xe_dev, (S.geom_spec_ready && c->spec_replay_shard) ? 4u : 0u, ev_cap, aux_cap);
        uint8_t *m = S.msg.as<uint8_t>() + 16;
        if ((rc = wg_lf_export_tokens(c, R, reinterpret_cast<uint32_t *>(m))) != WG_OK) return rc;
        if ((rc = wg_lf_export_ends(c, R, reinterpret_cast<uint32_t *>(m + tok_a), reinterpret_cast<uint32_t *>(m + 2 * tok_a),
                                    S.xtok.as<const uint32_t>() + L, L)) != WG_OK)
            return rc;
        // the event records travel in the same message, with shard-local tokens
        if ((rc = wg_lf_events_local(c, R, reinterpret_cast<uint4 *>(m + tok_b), nullptr)) != WG_OK) return rc;
        return WG_OK;
    }
    case SH_X3: {   // global event ids; replay the global event stream; lanes of own rows; default geometry
        std::vector<uint32_t> hdr;
        if ((rc = read_headers(c, gathered, stride, hdr)) != WG_OK) return rc;
        S.evoff.assign(W + 1, 0);
        S.auxoff.assign(W + 1, 0);
        S.xoff.assign(W + 1, 0);
        bool bad = false, spec_all = true;
        const uint64_t L = S.uoffs[W], tok_a = (L * 4 + 15) & ~15ull, tok_b = 3 * tok_a;
        for (int r = 0; r < W; r++) {
            S.evoff[r + 1] = S.evoff[r] + hdr[4 * r];
            S.auxoff[r + 1] = S.auxoff[r] + hdr[4 * r + 1];
            S.xoff[r + 1] = S.xoff[r] + hdr[4 * r + 3];   // own crossing entries (X2 left them on the device)
            bad |= (hdr[4 * r + 2] & 3u) != 0;            // not well formed
            spec_all &= (hdr[4 * r + 2] & 4u) != 0;       // every rank may replay speculatively
        }
        if (S.xoff[W] > L)
            return wg_fail(c, WG_E_INVALID, "X3 headers: %llu crossing entries of %llu records",
                           (unsigned long long)S.xoff[W], (unsigned long long)L);
        if (bad || S.evoff[W] >= (1ull << 30)) return sh_fallback(c, out);
        const uint64_t nx = S.xoff[W];
        for (int r = 0; r < W; r++) {
            if ((rc = check_len(c, r, 16 + tok_b + (uint64_t)hdr[4 * r] * 16 + (uint64_t)hdr[4 * r + 1] * 4,
                                "X3 tokens and event records")) != WG_OK)
                return rc;
        }
        WG_ALLOC(c, S.xtok, nx * 4 + 16);
        WG_ALLOC(c, S.xt, nx * 4 + 16);
        // every rank's crossing tokens, event records and aux words (after its
        // tokens, 16-byte aligned: rank r's events at evoff[r], aux words at
        // auxoff[r]) and the three offset tables: one launch
        const uint64_t nev = S.evoff[W], naux = S.auxoff[W];
        DevBuf &evrec = c->lf[LF_EVREC], &aux = c->lf[LF_AUX];
        WG_ALLOC(c, evrec, (nev + 256) * 16);
        WG_ALLOC(c, aux, naux * 4 + 4);
        WG_ALLOC(c, S.dev_small, 96 * 8);
        WG_HIP(c, hipMemsetAsync(evrec.as<uint4>() + nev, 0, 256 * 16, st));
        {
            WgCopies cp;
            for (int r = 0; r < W; r++) {
                const uint64_t n = S.xoff[r + 1] - S.xoff[r];
                const uint64_t ne_r = S.evoff[r + 1] - S.evoff[r], na_r = S.auxoff[r + 1] - S.auxoff[r];
                const uint8_t *src = (const uint8_t *)gathered + r * stride + 16;
                cp.add(S.xtok.as<uint32_t>() + S.xoff[r], src, n * 4);
                cp.add(evrec.as<uint4>() + S.evoff[r], src + tok_b, ne_r * 16);
                cp.add(aux.as<uint32_t>() + S.auxoff[r], src + tok_b + ne_r * 16, na_r * 4);
            }
            cp.words(S.dev_small.as<uint64_t>(), 0, S.xoff.data(), (uint32_t)W + 1);
            cp.words(S.dev_small.as<uint64_t>(), 20, S.evoff.data(), (uint32_t)W + 1);
            cp.words(S.dev_small.as<uint64_t>(), 40, S.auxoff.data(), (uint32_t)W + 1);
            if ((rc = wg_copy_batch(c, cp, st)) != WG_OK) return rc;
        }
        if (nx) hipLaunchKernelGGL(k_sh_resolve, dim3(1), dim3(1024), 0, st, nx, (uint32_t)W, S.dev_small.as<const uint64_t>(),
                                   S.dev_small.as<const uint64_t>() + 20, S.xtok.as<const uint32_t>(), S.xt.as<uint32_t>());
        LfRange R = sh_range(c);
        if ((rc = wg_lf_events_finish(c, R, (uint32_t)S.evoff[S.rank], S.xt.as<const uint32_t>(), nx, nev, (uint32_t)W,
                                      S.dev_small.as<const uint64_t>() + 20, S.dev_small.as<const uint64_t>() + 40,
                                      evrec.as<uint4>(), aux.as<uint32_t>())) != WG_OK)
            return rc;
        c->n_events = nev;
        // the endpoints' row tokens (global), and every token's consumption time
        WG_ALLOC(c, S.etok, nx * 8 + 16);
        WG_ALLOC(c, S.elane, nx * 8 + 16);
        if (nx) {
            EndToks E{(const uint8_t *)gathered, stride, tok_a, (uint32_t)W};
            hipLaunchKernelGGL(k_sh_etok, dim3(blocks(nx)), dim3(T), 0, st, E, nx, S.dev_small.as<const uint64_t>(),
                               S.dev_small.as<const uint64_t>() + 20, S.xt.as<const uint32_t>(), S.etok.as<uint32_t>());
        }
        WG_ALLOC(c, S.death, (nev + 256) * 4);
        if ((rc = wg_lf_death_from_records(c, nev, evrec.as<const uint4>(), aux.as<const uint32_t>(), S.death.as<uint32_t>())) !=
            WG_OK)
            return rc;
        WG_ALLOC(c, c->lane_asg, nl * 4 + 4);
        const uint64_t nloc = nl + 2;
        WG_ALLOC(c, c->lane_out, nloc * 4 + 4);
        WG_ALLOC(c, c->color_out, nloc + 4);
        S.replay_pending = false;
        if (nev && spec_all) {
            // after a sharded build sized every rank's context (a decision all
            // ranks take alike, from the X3 heads): the blind iterations with
            // no host read, the words checked with the local geometry's
            ReplayRun run;
            c->replay_death = S.death.as<const uint32_t>();
            rc = wg_lf_replay_lanes_spec(c, R, nev, evrec.as<const uint4>(), aux.as<const uint32_t>(),
                                         c->lane_asg.as<uint32_t>(), run);
            c->replay_death = nullptr;
            if (rc != WG_OK) return rc;
            S.replay_pending = true;
            c->spec_replays_shard++;
            S.rp_it = run.it;
            S.rp_chunk = run.chunk;
            S.rp_flags = run.flags;
            S.rp_scal = run.scal;
            S.rp_dc = run.dc;
            S.rp_nw = run.nw;
            S.rp_warm = run.warm;
            sh_lane_out(c);
            sh_end_lanes(c);
        } else {
            bool ok = false;
            if ((rc = sh_replay_exact(c, &ok)) != WG_OK) return rc;
            if (!ok) return sh_fallback(c, out);        // no fixed point / > 1023 slots: same decision on every rank
        }
        c->have_layout = true;
        c->layout_gen++;
        c->alt_heights_on = false;   // (a new built list: its own heights)
        return sh_local_geometry(c, S.build_band, out, true);   // the default geometry, or build_frame's
    }
    default:
        return wg_fail(c, WG_E_STATE, "bad shard step %d", S.step);
    }
}

int wg_shard_geometry_begin(wg_ctx *c, const float *band, int32_t residency, wg_shard_msg *out) {
    if (!c || !out) return WG_E_INVALID;
    WG_SETTLE(c);
    ShardState &S = c->sh;
    if (!S.on || !c->have_layout) return wg_fail(c, WG_E_STATE, "no sharded layout built");
    if (S.step != SH_IDLE) return wg_fail(c, WG_E_STATE, "a sharded call is in progress");
    (void)hipSetDevice(c->device);
    c->have_vtx = c->have_text = false;
    const float *d_band = nullptr;
    if (band) {
        if (residency == WG_HOST) {
            WG_ALLOC(c, S.band_host, S.N * 4 + 4);
            if (S.N) WG_HIP(c, hipMemcpyAsync(S.band_host.p, band, S.N * 4, hipMemcpyHostToDevice, c->stream));
            d_band = S.band_host.as<float>();
        } else if (residency == WG_DEVICE) {
            d_band = band;
        } else {
            return wg_fail(c, WG_E_INVALID, "bad residency %d", residency);
        }
    }
    if (S.replicated) {
        c->have_geom = false;
        int rc = wg_row_geometry(c, d_band, WG_DEVICE);
        if (rc != WG_OK) return rc;
        sh_done(c, out);
        return WG_OK;
    }
    c->have_geom = false;
    return sh_local_geometry(c, d_band, out, true);
}

}  // extern "C"
