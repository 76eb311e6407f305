// wg_lanes_fast.hip — event-compressed lane assignment (SURVEY.md §7 hard
// part 1), bit-identical to GraphLayout::build's greedy (commit_graph.rs:
// 276-295, 401-471) on well-formed commit lists.
//
// Well-formed = every id distinct (checked in parallel; duplicate ids take
// the general walk in wg_lanes.hip).  Then the sequential state has a static
// description:
//   * a slot waiting for commit j is set only by a child of j (rows < j) and
//     stays until row j, so the waiters of j are: one slot per first-parent
//     child, plus one slot if the FIRST in-list reference to j (row, parent
//     index order) is a secondary parent (:447-459 allocates only then);
//   * w(j) = #waiters.  w = 1: j inherits its single waiter's slot (no state
//     change).  w = 0: lowest free slot (ALLOC).  w >= 2: lowest waiter slot,
//     the others freed (MIN, :287-291).  First parent outside the list: the
//     slot is freed (FREE) or never occupied (probe ALLOC).  First
//     references through a secondary parent: SECALLOC (:454-458).
//   * a parent p at an earlier row (or the row itself: clock skew, orphans
//     re-sorted by time, git/mod.rs:767-772; self parents) is "leaky": its
//     row is processed, so nothing ever frees a slot set to wait for it
//     (:287-291 only runs at p's own row).  A leaky first parent keeps the
//     row's slot occupied for good (the row's chain never ends); a leaky
//     secondary parent allocates (SECALLOC, never consumed) unless an
//     earlier leaky reference — from a row in [p, i), or an earlier parent
//     of the same row — already holds a slot for p (:450-452).  So a leaky
//     reference is "first" by the minimum (row, parent index) among the
//     leaky references to p (LfRange::lfirst), apart from p's own waiters.
// Only those events touch the slot-occupancy state, and they are a few
// percent of rows.  The pipeline:
//   refs     first reference + first-parent child count per row (atomics)
//   rows     w(j), event and merge-token counts -> scans -> event ids
//   chain    every row's "source" token via pointer jumping along w = 1
//            first-parent chains (log2 N rounds)
//   events   16-byte event records in row order; merges with more than two
//            waiters list all their tokens in an aux array
//   replay   the event stream cut into chunks replayed in parallel and
//            iterated to a fixed point (wg_lanes_replay.hip): 64-bit
//            occupancy mask, lowest-free = ctz(~occ)
//   lanes    lane[j] = slot of source(j)   (parallel gather)
// max_lane = max over occupying allocations of the highest occupied slot
// (update_peak, :462-471, can only rise when a slot is taken).
//
// Every phase works on a row range [s, e) (LfRange): a single-GPU build is
// the whole list; a row-sharded build (wg_shard.hip) runs the same phases on
// its shard, with the references that cross shard boundaries supplied as
// crossing entries.  A waiter created before s is a crossing token (WG_TOK_X)
// until the other shards report which event started its chain.
#include "wg_internal.h"
#include "wg_lanes_refs.h"

namespace {

constexpr int T = 256;
constexpr uint32_t TAGS = WG_TOK_EV | WG_TOK_X;

// event record flags (uint4.x): A = takes the lowest free slot, O = occupies
// its slot afterwards, C = clears its token slots (MIN / FREE), M = more than
// two waiters (all tokens listed in aux at record.w); IN0/IN1 = token 0/1
// lives in the event's own 64-event batch at local index bits 8..13 / 16..21.
enum : uint32_t { F_A = 1u, F_O = 2u, F_C = 4u, F_M = 8u, F_IN0 = 1u << 14, F_IN1 = 1u << 22 };

__device__ __forceinline__ uint32_t token_bits(uint64_t e, uint32_t t0, uint32_t t1) {
    uint32_t b = ((t0 & 63u) << 8) | ((t1 & 63u) << 16);
    if ((t0 >> 6) == (e >> 6)) b |= F_IN0;
    if ((t1 >> 6) == (e >> 6)) b |= F_IN1;
    return b;
}

inline uint32_t blocks(uint64_t n) { return (uint32_t)((n + T - 1) / T); }

// crossing-entry bounds, from the device when the range carries them (LfRange::xb_dev)
__device__ __forceinline__ uint64_t lf_xin_end(const LfRange &R) { return R.xb_dev ? (uint64_t)*R.xb_dev : R.xin_end; }
__device__ __forceinline__ uint64_t lf_xown_begin(const LfRange &R) { return R.xb_dev ? (uint64_t)*R.xb_dev : R.xown_begin; }
__device__ __forceinline__ uint64_t lf_xown_end(const LfRange &R) { return R.xe_dev ? (uint64_t)*R.xe_dev : R.xown_end; }

// is ref k (row gi, index kidx, target p) the first in-list reference to p?
__device__ __forceinline__ bool is_first_ref(const LfRange &R, const unsigned long long *__restrict__ first_ref,
                                             uint64_t gi, uint32_t k, uint32_t kidx, uint64_t p) {
    if (p <= gi) {   // leaky; without lfirst k_lf_refs flagged the list and nothing here is used
        if (p < R.s) return R.isfb[k] != 0;   // target in an earlier shard: k_lf_xfirst decided
        return R.lfirst && R.lfirst[p - R.s] == ref_key(gi, kidx);
    }
    if (p >= R.e) return R.isfb[k] != 0;
    return first_ref[p - R.s] == ref_key(gi, kidx);
}

__global__ void k_lf_refs(LfRange R, unsigned long long *first_ref, uint32_t *fpc, uint32_t *viol) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R.nl) return;
    if (lf_refs_row(R, R.s + i, first_ref, fpc)) atomicOr(viol, 1u);
}

// references from earlier shards into this one
__global__ void k_lf_xin(LfRange R, unsigned long long *first_ref, uint32_t *fpc) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= lf_xin_end(R)) return;
    const WgXEnt en = R.xall[x];
    if (!(en.kf & WG_XF_FIRST_IN_ROW) || en.p < R.s || en.p >= R.e) return;
    const uint32_t kidx = en.kf & 0xFFFFu;
    atomicMin(&first_ref[en.p - R.s], ref_key(en.c, kidx));
    if (kidx == 0) atomicAdd(&fpc[en.p - R.s], 1u);
}

// own references beyond the shard: first reference to their target?  A
// reference to an earlier shard's row is leaky (:441-446): first among the
// leaky references to that row, i.e. its own shard holds none (WG_XF_LLEAKY:
// every row of that shard precedes this one) and no crossing entry of a row
// between them, or an earlier one of this row, refers to it
__global__ void k_lf_xfirst(LfRange R) {
    const uint64_t xe = lf_xown_end(R);
    const uint64_t x = lf_xown_begin(R) + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= xe) return;
    const WgXEnt en = R.xall[x];
    const uint32_t kidx = en.kf & 0xFFFFu;
    const uint32_t k = R.poff[en.c] + kidx;
    if (!(en.kf & WG_XF_FIRST_IN_ROW)) { R.isfb[k] = 0; return; }
    const bool leaky = en.p <= en.c;
    const unsigned long long key = ref_key(en.c, kidx);
    bool first = !(leaky && (en.kf & WG_XF_LLEAKY));
    for (uint64_t y = 0; y < xe && first; y++) {
        const WgXEnt o = R.xall[y];
        // For a leaky entry only earlier leaky references count: forward
        // references to the same row (from rows c' < p, which sort before it)
        // are consumed at row p (:287-291) and hold nothing afterwards.  For a
        // forward entry no leaky reference can sort before it.
        if (o.p == en.p && (o.kf & WG_XF_FIRST_IN_ROW) && ref_key(o.c, o.kf & 0xFFFFu) < key && (!leaky || o.p <= o.c))
            first = false;
    }
    R.isfb[k] = first ? 1 : 0;
}

// per row: w, first-parent-in-list, event count, merge-token count; the
// block sums of the event / merge-token / first-parent-child counts feed one
// scan launch for ev_off, aux_off and ch_off (wg_scan_bs_u32)
__global__ void __launch_bounds__(WG_BS_THREADS) k_lf_rows(LfRange R, const unsigned long long *__restrict__ first_ref,
                                                          const uint32_t *__restrict__ fpc, uint32_t *__restrict__ winfo,
                                                          uint32_t *__restrict__ ev_cnt, uint32_t *__restrict__ aux_cnt,
                                                          uint32_t *__restrict__ bsum, uint32_t nbs) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t ne = 0, na_aux = 0, nfp = 0;
    if (j < R.nl) {
        const uint64_t gj = R.s + j;
        const unsigned long long fr = first_ref[j];
        const uint32_t sec_first = (fr != REF_NONE && (fr & 0xFFFFu) != 0) ? 1u : 0u;
        nfp = fpc[j];
        const uint32_t w = nfp + sec_first;
        const uint32_t pa = R.poff[gj], pb = R.poff[gj + 1];
        const bool fp_in = pb > pa && R.prow[pa] >= 0;
        uint32_t nc = 0;
        for (uint32_t k = pa + 1; k < pb; k++) {
            const int32_t p = R.prow[k];
            if (p >= 0 && is_first_ref(R, first_ref, gj, k, k - pa, (uint64_t)p)) nc++;
        }
        const uint32_t na = (w != 1) ? 1u : 0u;
        const uint32_t nb = (w == 1 && !fp_in) ? 1u : 0u;
        winfo[j] = (w < 0x3FFFFFFFu ? w : 0x3FFFFFFFu) | (fp_in ? 0x40000000u : 0u) | (sec_first ? 0x80000000u : 0u);
        ne = na + nb + nc;
        na_aux = w > 2 ? w + 1 : 0u;
        ev_cnt[j] = ne;
        aux_cnt[j] = na_aux;
    }
    wg_bsum_store(ne, bsum);
    wg_bsum_store(na_aux, bsum + nbs);
    wg_bsum_store(nfp, bsum + 2 * nbs);
}

// per row: the SECALLOC event of every first reference through a secondary
// parent, and the row into its first parent's list of first-parent children
__global__ void k_lf_secev_children(LfRange R, const unsigned long long *__restrict__ first_ref,
                                    const uint32_t *__restrict__ winfo, const uint32_t *__restrict__ ev_off,
                                    uint32_t *__restrict__ secev, const uint32_t *__restrict__ ch_off, uint32_t *ch_fill,
                                    uint32_t *ch, uint32_t *__restrict__ death) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= R.nl) return;
    const uint64_t gj = R.s + j;
    // the consumption time of the row's events: none yet (k_lf_events writes the consumers')
    if (death)
        for (uint32_t e = ev_off[j]; e < ev_off[j + 1]; e++) death[e] = 0xFFFFFFFFu;
    const uint32_t wi = winfo[j], w = wi & 0x3FFFFFFFu;
    const bool fp_in = wi & 0x40000000u;
    uint32_t e = ev_off[j] + ((w != 1) ? 1u : 0u) + ((w == 1 && !fp_in) ? 1u : 0u);
    const uint32_t pa = R.poff[gj], pb = R.poff[gj + 1];
    for (uint32_t k = pa + 1; k < pb; k++) {
        const int32_t p = R.prow[k];
        if (p < 0 || !is_first_ref(R, first_ref, gj, k, k - pa, (uint64_t)p)) continue;
        if ((uint64_t)p <= gj) {}                    // leaky: nothing waits for this slot
        else if ((uint64_t)p < R.e) secev[p - R.s] = WG_TOK_EV | e;
        else R.xsec[k] = WG_TOK_EV | e;
        e++;
    }
    if (pa == pb) return;
    const int32_t p = R.prow[pa];
    if (p < 0 || (uint64_t)p >= R.e || (uint64_t)p <= gj) return;   // beyond the range / leaky
    const uint64_t pl = (uint64_t)p - R.s;
    // (bounded on any input: this kernel is queued before the host knows the
    // list is well formed, and with duplicate ids the first-parent counts the
    // lists were sized by and the parent rows differ — the general walk
    // replaces these results then)
    const uint32_t at = atomicAdd(&ch_fill[pl], 1u);
    if (at < ch_off[pl + 1] - ch_off[pl]) ch[ch_off[pl] + at] = (uint32_t)j;
}

// first references into this shard through a secondary parent of an earlier shard
__global__ void k_lf_xin_secev(LfRange R, const unsigned long long *__restrict__ first_ref, uint32_t *__restrict__ secev) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= lf_xin_end(R)) return;
    const WgXEnt en = R.xall[x];
    const uint32_t kidx = en.kf & 0xFFFFu;
    if (!(en.kf & WG_XF_FIRST_IN_ROW) || kidx == 0 || en.p < R.s || en.p >= R.e) return;
    if (first_ref[en.p - R.s] == ref_key(en.c, kidx)) secev[en.p - R.s] = WG_TOK_X | (uint32_t)x;
}

__global__ void k_lf_xin_children(LfRange R, const uint32_t *__restrict__ ch_off, uint32_t *ch_fill, uint32_t *ch) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= lf_xin_end(R)) return;
    const WgXEnt en = R.xall[x];
    if ((en.kf & 0xFFFFu) != 0 || en.p < R.s || en.p >= R.e) return;
    const uint64_t pl = en.p - R.s;
    const uint32_t at = atomicAdd(&ch_fill[pl], 1u);
    if (at < ch_off[pl + 1] - ch_off[pl]) ch[ch_off[pl] + at] = WG_TOK_X | (uint32_t)x;
}

// the chain source pointer of row j before jumping
__device__ __forceinline__ uint32_t sp_init(uint64_t j, const uint32_t *__restrict__ winfo, const uint32_t *__restrict__ ev_off,
                                            const uint32_t *__restrict__ ch_off, const uint32_t *__restrict__ ch,
                                            const uint32_t *__restrict__ secev) {
    const uint32_t wi = winfo[j], w = wi & 0x3FFFFFFFu;
    if (w != 1) return WG_TOK_EV | ev_off[j];              // own ALLOC / MIN event
    if (wi & 0x80000000u) return secev[j];                 // waiter = secondary allocation
    return ch[ch_off[j]];                                  // waiter = the only first-parent child
}

// Chain sources: sp[j] is a token (tagged) or the row whose token row j
// inherits, always an earlier row.  Resolution in two phases:
//   k_lf_jump_tile  pointer jumping inside tiles of JT_ROWS rows in LDS:
//                   afterwards every pointer leaves its tile (or is a token);
//   k_lf_jump4      each pass follows up to 4 links, so P becomes P^4: every
//                   link crosses a tile, and ceil(log4(tiles)) passes finish.
constexpr int JT_THREADS = 1024, JT_ROWS = 4096;   // (16384: one jump4 pass fewer, the tile pass 18 -> 50 us)

__global__ void __launch_bounds__(JT_THREADS) k_lf_jump_tile(uint64_t nl, uint32_t *__restrict__ sp,
                                                              const uint32_t *__restrict__ winfo, const uint32_t *__restrict__ ev_off,
                                                              const uint32_t *__restrict__ ch_off, const uint32_t *__restrict__ ch,
                                                              const uint32_t *__restrict__ secev) {
    __shared__ uint32_t L[JT_ROWS];
    const uint64_t t0 = (uint64_t)blockIdx.x * JT_ROWS;
    const uint32_t nt = (uint32_t)((nl - t0) < (uint64_t)JT_ROWS ? (nl - t0) : (uint64_t)JT_ROWS);
    for (uint32_t i = threadIdx.x; i < nt; i += JT_THREADS) L[i] = sp_init(t0 + i, winfo, ev_off, ch_off, ch, secev);
    __syncthreads();
    // in place: a stored value is always a later link of the same chain, so a
    // racing read only skips further; stop once no pointer stays in the tile.
    // Pointers lead to earlier rows on the inputs this path accepts, so 13
    // rounds always suffice; the bound keeps any other input finite.
    for (int round = 0; round < 32; round++) {
        int moved = 0;
        for (uint32_t i = threadIdx.x; i < nt; i += JT_THREADS) {
            const uint32_t v = L[i];
            if (!(v & TAGS) && (uint64_t)v >= t0 && (uint64_t)v < t0 + nt && v - t0 != i) {   // inside the tile
                L[i] = L[v - t0];
                moved = 1;
            }
        }
        if (!__syncthreads_or(moved)) break;
    }
    for (uint32_t i = threadIdx.x; i < nt; i += JT_THREADS) sp[t0 + i] = L[i];
}

__global__ void k_lf_jump4(uint64_t nl, const uint32_t *__restrict__ in, uint32_t *__restrict__ out) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nl) return;
    uint32_t v = in[j];
#pragma unroll
    for (int h = 0; h < 4; h++) {
        if ((v & TAGS) || (uint64_t)v >= nl) break;   // (a pointer past the rows: only on inputs the path rejects)
        v = in[v];
    }
    out[j] = v;
}

// token of every own crossing entry: the chain of its child row (first
// parent) or its SECALLOC event (first reference through a secondary parent)
__global__ void k_lf_export(LfRange R, const uint32_t *__restrict__ sp, uint32_t *__restrict__ tok) {
    const uint64_t xb = lf_xown_begin(R);
    const uint64_t x = xb + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= lf_xown_end(R)) return;
    const WgXEnt en = R.xall[x];
    const uint32_t kidx = en.kf & 0xFFFFu;
    uint32_t t = WG_TOK_NONE;
    if (kidx == 0) t = sp[en.c - R.s];
    else if ((en.kf & WG_XF_FIRST_IN_ROW) && R.isfb[R.poff[en.c] + kidx]) t = R.xsec[R.poff[en.c] + kidx];
    tok[x - xb] = t;
}

// X3 (no X6): the row token of every own entry's child row, and of the parent
// row of every entry (of any shard) whose parent is in this one — after the
// replay every rank reads the far endpoints' lanes from them
__global__ void k_lf_export_ends(LfRange R, const uint32_t *__restrict__ sp, uint32_t *__restrict__ ctok,
                                 uint32_t *__restrict__ ptok, const uint32_t *__restrict__ xtot, uint64_t xcap) {
    const uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= xcap) return;
    const uint64_t nx = *xtot, xb = lf_xown_begin(R), xe = lf_xown_end(R);
    uint32_t pt = WG_TOK_NONE;
    if (x < nx) {
        const WgXEnt en = R.xall[x];
        if (en.p >= R.s && en.p < R.e) pt = sp[en.p - R.s];
        if (x >= xb && x < xe) ctok[x - xb] = sp[en.c - R.s];
    }
    ptok[x] = pt;
}

__device__ __forceinline__ uint32_t globalize(uint32_t v, uint32_t ev_base, const uint32_t *__restrict__ xt) {
    if (v & WG_TOK_EV) return WG_TOK_EV | ((v & ~WG_TOK_EV) + ev_base);
    if (v & WG_TOK_X) return xt[v & ~WG_TOK_X];
    return v;
}

__global__ void k_lf_globalize(uint64_t nl, uint32_t ev_base, const uint32_t *__restrict__ xt, uint32_t *sp,
                               uint32_t *secev, const uint32_t *__restrict__ winfo) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nl) return;
    sp[j] = globalize(sp[j], ev_base, xt);
    if (winfo[j] & 0x80000000u) secev[j] = globalize(secev[j], ev_base, xt);
}

// LOCAL (sharded build, before the crossing tokens are known): tokens stay
// tagged (EV = shard-local event, X = crossing-table entry), the flags carry
// no token bits and aux offsets are shard-local; k_lf_events_finish turns the
// gathered records into exactly what the global form would have written.
template <bool LOCAL>
__global__ void k_lf_events(LfRange R, uint32_t ev_base, uint32_t aux_base, const uint32_t *__restrict__ xt,
                            const unsigned long long *__restrict__ first_ref, const uint32_t *__restrict__ winfo,
                            const uint32_t *__restrict__ ev_off, const uint32_t *__restrict__ aux_off,
                            const uint32_t *__restrict__ ch_off, const uint32_t *__restrict__ ch,
                            const uint32_t *__restrict__ secev, const uint32_t *__restrict__ sp,
                            uint4 *__restrict__ ev, uint32_t *__restrict__ aux, const uint32_t *__restrict__ gate = nullptr,
                            WgReplayInit RI = WgReplayInit{}, const uint32_t *__restrict__ aux_after = nullptr,
                            uint32_t *__restrict__ death = nullptr) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // (a message whose merge-token lists follow its records: the event count is on the device)
    if (aux_after) aux = reinterpret_cast<uint32_t *>(ev + *aux_after);
    // speculative build: the replay's initial state (wg_replay_prepare_spec)
    for (uint64_t i = j; i < RI.total; i += (uint64_t)gridDim.x * blockDim.x) {
        if (i < RI.occ_words) RI.occ[i] = 0ull;
        if (i < RI.nflags) RI.changed[i] = (i == 0) ? 1u : 0u;
        if (i < RI.nslots16) RI.slots16[i] = make_uint4(0u, 0u, 0u, 0u);
        if (RI.nev_dev && i < 256) ev[*RI.nev_dev + i] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (j >= R.nl) return;
    const uint64_t gj = R.s + j;
    // the row's first loads issued with the gate's, waited on once
    const uint32_t wi = winfo[j], w = wi & 0x3FFFFFFFu;
    uint32_t e = ev_off[j];                  // shard-local event index; global id = ev_base + e
    const uint32_t pa = R.poff[gj], pb = R.poff[gj + 1];
    asm volatile("" ::"v"(wi), "v"(e), "v"(pa), "v"(pb));   // (held here: not sunk past the gate's branch)
    if (gate && *gate) return;   // speculative build: not well formed (the general walk takes over)
    const bool fp_in = wi & 0x40000000u, sec_first = wi & 0x80000000u;
    if (w == 0) {
        ev[e] = make_uint4(fp_in ? (F_A | F_O) : F_A, 0u, 0u, (uint32_t)gj);
        e++;
    } else if (w >= 2) {
        // tokens: sources of the first-parent children, plus the secondary allocation
        uint32_t t[2] = {0u, 0u};
        uint32_t nt = 0;
        uint32_t *list = (w > 2) ? aux + aux_off[j] : nullptr;
        if (list) list[0] = w;
        for (uint32_t k = ch_off[j]; k < ch_off[j + 1]; k++) {
            const uint32_t v = ch[k];
            const uint32_t tk = LOCAL ? ((v & WG_TOK_X) ? v : sp[v])
                                      : ((v & WG_TOK_X) ? xt[v & ~WG_TOK_X] : sp[v]) & ~WG_TOK_EV;
            if (nt < 2) t[nt] = tk;
            if (list) list[1 + nt] = tk;
            nt++;
        }
        if (sec_first) {
            const uint32_t tk = LOCAL ? secev[j] : secev[j] & ~WG_TOK_EV;
            if (nt < 2) t[nt] = tk;
            if (list) list[1 + nt] = tk;
            nt++;
        }
        const uint32_t f = F_C | (fp_in ? F_O : 0u) | ((w > 2) ? F_M : 0u);
        ev[e] = make_uint4(f | (LOCAL ? 0u : token_bits(ev_base + e, t[0], t[1])), t[0], t[1],
                           (w > 2) ? aux_base + aux_off[j] : (uint32_t)gj);
        if (death) {   // (single GPU: tokens are event ids) this event consumes every waiter's token
            const uint32_t dn = ev_off[R.nl];   // (a token past the events is never written through)
            if (list) {
                for (uint32_t q = 1; q <= w; q++)
                    if (list[q] < dn) death[list[q]] = e + 1u;
            } else {
                if (t[0] < dn) death[t[0]] = e + 1u;
                if (t[1] < dn) death[t[1]] = e + 1u;
            }
        }
        e++;
    } else if (!fp_in) {
        const uint32_t t0 = LOCAL ? sp[j] : sp[j] & ~WG_TOK_EV;
        ev[e] = make_uint4(F_C | (LOCAL ? 0u : token_bits(ev_base + e, t0, t0)), t0, t0, (uint32_t)gj);
        if (death && t0 < ev_off[R.nl]) death[t0] = e + 1u;
        e++;
    }
    for (uint32_t k = pa + 1; k < pb; k++) {
        const int32_t p = R.prow[k];
        if (p >= 0 && is_first_ref(R, first_ref, gj, k, k - pa, (uint64_t)p)) {
            ev[e] = make_uint4(F_A | F_O, 0u, 0u, (uint32_t)gj);
            e++;
        }
    }
}

// consumption times from global records (the sharded build's gathered
// stream; a single-GPU build writes them in k_lf_events): tokens never
// consumed keep 0xFFFFFFFF.  A token past the events (a crossing entry that
// resolved to no token, WG_TOK_NONE) is not written through.
__global__ void k_lf_death_fill(uint64_t nev, uint32_t *__restrict__ death) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < nev) death[k] = 0xFFFFFFFFu;
}
__global__ void k_lf_death_scatter(uint64_t nev, const uint4 *__restrict__ ev, const uint32_t *__restrict__ aux,
                                   uint32_t *__restrict__ death) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nev) return;
    const uint4 r = ev[k];
    if (!(r.x & F_C)) return;
    const uint32_t t = (uint32_t)k + 1u;
    if (r.x & F_M) {
        const uint32_t n = aux[r.w];
        for (uint32_t q = 0; q < n; q++) {
            const uint32_t tk = aux[r.w + 1 + q];
            if (tk < nev) death[tk] = t;
        }
    } else {
        if (r.y < nev) death[r.y] = t;
        if (r.z < nev) death[r.z] = t;
    }
}

__global__ void k_lf_lanes(uint64_t nl, const uint32_t *__restrict__ sp, const uint16_t *__restrict__ slot_of,
                           uint32_t *__restrict__ lane, const uint32_t *__restrict__ gate = nullptr) {
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nl) return;
    if (gate && *gate) return;
    lane[j] = slot_of[sp[j] & ~WG_TOK_EV];
}

// the lane stage's initial state in one launch (instead of four fills):
// first references "none", per-row counters and the chain fill counters 0,
// the flag words 0
__global__ void k_lf_clear(uint64_t n, LfClear L) {
    lf_clear_at(L, n, (uint64_t)blockIdx.x * blockDim.x + threadIdx.x);   // (+ the lane scalars: max_lane, slots, ...)
}

// gathered shard-local records (k_lf_events<true> of every rank, rank r's at
// evoff[r] / auxoff[r]) -> global form: tokens through globalize with the
// owning rank's base, token bits at the global index, aux offsets rebased.
// Allocation records carry no tokens and are already final.
__global__ void k_lf_events_finish(uint64_t nev, uint32_t world, const uint64_t *__restrict__ evoff,
                                   const uint64_t *__restrict__ auxoff, const uint32_t *__restrict__ xt, uint64_t nx,
                                   uint4 *__restrict__ ev, uint32_t *__restrict__ aux) {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nev) return;
    uint4 r = ev[g];
    if (!(r.x & F_C)) return;
    uint32_t k = 0;
    while (k + 1 < world && evoff[k + 1] <= g) k++;
    const uint32_t base = (uint32_t)evoff[k];
    auto glob = [&](uint32_t v) -> uint32_t {
        if (!(v & WG_TOK_EV) && (v & WG_TOK_X) && (v & ~WG_TOK_X) >= nx) return v;   // not a crossing entry
        return globalize(v, base, xt) & ~WG_TOK_EV;
    };
    r.y = glob(r.y);
    r.z = glob(r.z);
    r.x |= token_bits(g, r.y, r.z);
    if (r.x & F_M) {
        r.w += (uint32_t)auxoff[k];
        uint32_t *list = aux + r.w;
        const uint32_t n = list[0];
        for (uint32_t q = 1; q <= n; q++) list[q] = glob(list[q]);
    }
    ev[g] = r;
}

}  // namespace


static const uint32_t *lf_sp(wg_ctx *c) { return c->lf_sp_b ? c->lf[LF_SPB].as<const uint32_t>() : c->lf[LF_SPA].as<const uint32_t>(); }

int wg_lf_refs(wg_ctx *c, const LfRange &R, bool read_back, uint32_t *scal) {
    const uint64_t n = R.nl;
    hipStream_t s = c->stream;
    DevBuf &first_ref = c->lf[LF_FIRST], &fpc = c->lf[LF_FPC], &winfo = c->lf[LF_WINFO], &ev_off = c->lf[LF_EVOFF];
    DevBuf &flags = c->lf[LF_FLAGS], &aux_off = c->lf[LF_AUXOFF], &ch_off = c->lf[LF_CHOFF];
    WG_ALLOC(c, first_ref, n * 8 + 8);
    WG_ALLOC(c, fpc, (n + 2) * 4);
    WG_ALLOC(c, winfo, n * 4 + 4);
    WG_ALLOC(c, ev_off, (n + 2) * 4);
    WG_ALLOC(c, aux_off, (n + 2) * 4);
    WG_ALLOC(c, ch_off, (n + 2) * 4);
    WG_ALLOC(c, flags, 64);
    DevBuf &ch_fill = c->lf[LF_CHFILL];
    WG_ALLOC(c, ch_fill, (n + 2) * 4);
    const uint64_t nbs = wg_bs_blocks(n);
    WG_ALLOC(c, c->bsum, 4 * (nbs + 64) * 4);   // (the edge counts' block sums at [3 (nbs + 64), ...), wg_stage_hash_join)
    { const int _sr = wg_scan_reserve(c, n + 2); if (_sr != WG_OK) return _sr; }
    wg_stage_begin(c, "lf_refs");
    if (c->lf_refs_done) {   // cleared by the hash join's place pass, references taken by its per-row probe
        c->lf_refs_done = false;
    } else {
        LfClear L;
        L.first_ref = first_ref.as<unsigned long long>();
        L.lfirst = R.lfirst;
        L.fpc = fpc.as<uint32_t>();
        L.ch_fill = ch_fill.as<uint32_t>();
        L.flags = flags.as<uint32_t>();
        L.scal = scal;
        hipLaunchKernelGGL(k_lf_clear, dim3(blocks(n + 16)), dim3(T), 0, s, n, L);
        if (n) hipLaunchKernelGGL(k_lf_refs, dim3(blocks(n)), dim3(T), 0, s, R, first_ref.as<unsigned long long>(),
                                  fpc.as<uint32_t>(), flags.as<uint32_t>());
    }
    if (R.xin_end)
        hipLaunchKernelGGL(k_lf_xin, dim3(blocks(R.xin_end)), dim3(T), 0, s, R, first_ref.as<unsigned long long>(),
                           fpc.as<uint32_t>());
    if (R.xown_end > R.xown_begin)
        hipLaunchKernelGGL(k_lf_xfirst, dim3(blocks(R.xown_end - R.xown_begin)), dim3(T), 0, s, R);
    // event / merge-token / child counts and their block sums, then one scan
    // launch: ev_off, aux_off (in place) and ch_off (the first-parent children
    // lists, from fpc)
    uint32_t *bs = c->bsum.as<uint32_t>();
    if (n) hipLaunchKernelGGL(k_lf_rows, dim3(blocks(n)), dim3(T), 0, s, R, first_ref.as<const unsigned long long>(),
                              fpc.as<const uint32_t>(), winfo.as<uint32_t>(), ev_off.as<uint32_t>(), aux_off.as<uint32_t>(),
                              bs, (uint32_t)nbs);
    WgScanBs S;
    S.na = 3;
    S.in[0] = ev_off.as<const uint32_t>(); S.out[0] = ev_off.as<uint32_t>(); S.bsum[0] = bs;
    S.in[1] = aux_off.as<const uint32_t>(); S.out[1] = aux_off.as<uint32_t>(); S.bsum[1] = bs + nbs;
    S.in[2] = fpc.as<const uint32_t>(); S.out[2] = ch_off.as<uint32_t>(); S.bsum[2] = bs + 2 * nbs;
    if (c->edge_scan_pending) {   // the hash join's edge-count scan, in the same launch (speculative build)
        c->edge_scan_pending = false;
        S.na = 4;
        S.in[3] = c->edge_cnt.as<const uint32_t>(); S.out[3] = c->edge_cnt.as<uint32_t>(); S.bsum[3] = bs + 3 * (nbs + 64);
    }
    WG_HIP(c, wg_scan_bs_u32(S, n, c->scan_tmp.p, s));
    // read back while the chain phase runs (wg_lf_refs_end); a speculative
    // build reads the same words with its end-of-build validation instead
    const int rc = read_back ? wg_fetch_begin(c, {{flags.p, false}, {ev_off.as<uint32_t>() + n, false},
                                                  {aux_off.as<uint32_t>() + n, false}})
                             : WG_OK;
    wg_stage_end(c);
    return rc;
}

int wg_lf_refs_end(wg_ctx *c, uint32_t *viol, uint64_t *nev, uint64_t *naux) {
    uint64_t hdr[3] = {0, 0, 0};
    if (const int rc = wg_fetch_end(c, hdr)) return rc;
    *viol = (uint32_t)hdr[0];
    *nev = hdr[1];
    *naux = hdr[2];
    return WG_OK;
}

int wg_lf_chain(wg_ctx *c, const LfRange &R) {
    const uint64_t n = R.nl;
    hipStream_t s = c->stream;
    DevBuf &first_ref = c->lf[LF_FIRST], &winfo = c->lf[LF_WINFO], &ev_off = c->lf[LF_EVOFF];
    DevBuf &secev = c->lf[LF_SECEV], &ch_off = c->lf[LF_CHOFF], &ch_fill = c->lf[LF_CHFILL], &ch = c->lf[LF_CH];
    DevBuf &spA = c->lf[LF_SPA], &spB = c->lf[LF_SPB];
    // children: own rows' first parents in range + earlier shards' first parents
    const uint64_t nref = c->e_refs_own + R.xin_end;
    WG_ALLOC(c, secev, n * 4 + 4);
    WG_ALLOC(c, ch_off, (n + 2) * 4);
    WG_ALLOC(c, ch_fill, (n + 2) * 4);
    WG_ALLOC(c, ch, nref * 4 + 4);
    WG_ALLOC(c, spA, n * 4 + 4);
    WG_ALLOC(c, spB, n * 4 + 4);
    wg_stage_begin(c, "lf_chain");
    // ch_fill was cleared with the stage's other state (k_lf_clear), ch_off
    // scanned with the event offsets (wg_lf_refs)
    // single-GPU builds (no crossing entries): the events' consumption times for
    // the replay's first iteration (wg_replay_first), set by k_lf_events
    uint32_t *death = nullptr;
    if (!R.xall) {
        const uint64_t nev_cap = n + c->e_refs_own;   // a row makes at most max(1, parents) events
        WG_ALLOC(c, c->lf[LF_DEATH], (nev_cap + 256) * 4);
        death = c->lf[LF_DEATH].as<uint32_t>();
    }
    c->lf_death = death;
    if (n) hipLaunchKernelGGL(k_lf_secev_children, dim3(blocks(n)), dim3(T), 0, s, R, first_ref.as<const unsigned long long>(),
                              winfo.as<const uint32_t>(), ev_off.as<const uint32_t>(), secev.as<uint32_t>(),
                              ch_off.as<const uint32_t>(), ch_fill.as<uint32_t>(), ch.as<uint32_t>(), death);
    if (R.xin_end)
        hipLaunchKernelGGL(k_lf_xin_secev, dim3(blocks(R.xin_end)), dim3(T), 0, s, R,
                           first_ref.as<const unsigned long long>(), secev.as<uint32_t>());
    if (R.xin_end)
        hipLaunchKernelGGL(k_lf_xin_children, dim3(blocks(R.xin_end)), dim3(T), 0, s, R, ch_off.as<const uint32_t>(),
                           ch_fill.as<uint32_t>(), ch.as<uint32_t>());
    // chain resolution: tiles in LDS, then passes of 4 links over the tile crossings
    const uint64_t ntiles = (n + JT_ROWS - 1) / JT_ROWS;
    if (n) hipLaunchKernelGGL(k_lf_jump_tile, dim3(ntiles), dim3(JT_THREADS), 0, s, n, spA.as<uint32_t>(),
                              winfo.as<const uint32_t>(), ev_off.as<const uint32_t>(), ch_off.as<const uint32_t>(),
                              ch.as<const uint32_t>(), secev.as<const uint32_t>());
    int rounds = 0;
    for (uint64_t reach = 1; reach < ntiles; reach *= 4) rounds++;
    DevBuf *in = &spA, *out = &spB;
    for (int r = 0; r < rounds; r++) {
        hipLaunchKernelGGL(k_lf_jump4, dim3(blocks(n)), dim3(T), 0, s, n, in->as<const uint32_t>(), out->as<uint32_t>());
        DevBuf *t = in; in = out; out = t;
    }
    c->lf_sp_b = (in == &spB);
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}

int wg_lf_export_tokens(wg_ctx *c, const LfRange &R, uint32_t *tok) {
    const uint64_t nx = R.xown_end - R.xown_begin;
    if (nx) hipLaunchKernelGGL(k_lf_export, dim3(blocks(nx)), dim3(T), 0, c->stream, R, lf_sp(c), tok);
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

int wg_lf_export_ends(wg_ctx *c, const LfRange &R, uint32_t *ctok, uint32_t *ptok, const uint32_t *xtot, uint64_t xcap) {
    if (xcap) hipLaunchKernelGGL(k_lf_export_ends, dim3(blocks(xcap)), dim3(T), 0, c->stream, R, lf_sp(c), ctok, ptok, xtot, xcap);
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

int wg_lf_death_from_records(wg_ctx *c, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *death) {
    if (!nev) return WG_OK;
    hipLaunchKernelGGL(k_lf_death_fill, dim3(blocks(nev)), dim3(T), 0, c->stream, nev, death);
    hipLaunchKernelGGL(k_lf_death_scatter, dim3(blocks(nev)), dim3(T), 0, c->stream, nev, ev, aux, death);
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

int wg_lf_events(wg_ctx *c, const LfRange &R, uint32_t ev_base, const uint32_t *xt, uint4 *ev_out, uint32_t *aux_out,
                 uint32_t aux_base) {
    const uint64_t n = R.nl;
    if (!n) return WG_OK;
    hipStream_t s = c->stream;
    uint32_t *sp = const_cast<uint32_t *>(lf_sp(c));
    wg_stage_begin(c, "lf_events");
    if (ev_base || xt)
        hipLaunchKernelGGL(k_lf_globalize, dim3(blocks(n)), dim3(T), 0, s, n, ev_base, xt, sp, c->lf[LF_SECEV].as<uint32_t>(),
                           c->lf[LF_WINFO].as<const uint32_t>());
    hipLaunchKernelGGL(k_lf_events<false>, dim3(blocks(n)), dim3(T), 0, s, R, ev_base, aux_base, xt,
                       c->lf[LF_FIRST].as<const unsigned long long>(), c->lf[LF_WINFO].as<const uint32_t>(),
                       c->lf[LF_EVOFF].as<const uint32_t>(), c->lf[LF_AUXOFF].as<const uint32_t>(),
                       c->lf[LF_CHOFF].as<const uint32_t>(), c->lf[LF_CH].as<const uint32_t>(),
                       c->lf[LF_SECEV].as<const uint32_t>(), (const uint32_t *)sp, ev_out, aux_out, nullptr, WgReplayInit{},
                       nullptr, (ev_base == 0 && !xt) ? c->lf_death : nullptr);
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}

int wg_lf_events_local(wg_ctx *c, const LfRange &R, uint4 *ev_out, uint32_t *aux_out) {
    const uint64_t n = R.nl;
    if (!n) return WG_OK;
    wg_stage_begin(c, "lf_events");
    // aux_out == nullptr: the merge-token lists right after the records, at the
    // device event count; nothing is written when the list is not well formed
    const bool after = aux_out == nullptr;
    hipLaunchKernelGGL(k_lf_events<true>, dim3(blocks(n)), dim3(T), 0, c->stream, R, 0u, 0u, (const uint32_t *)nullptr,
                       c->lf[LF_FIRST].as<const unsigned long long>(), c->lf[LF_WINFO].as<const uint32_t>(),
                       c->lf[LF_EVOFF].as<const uint32_t>(), c->lf[LF_AUXOFF].as<const uint32_t>(),
                       c->lf[LF_CHOFF].as<const uint32_t>(), c->lf[LF_CH].as<const uint32_t>(),
                       c->lf[LF_SECEV].as<const uint32_t>(), lf_sp(c), ev_out, aux_out,
                       after ? c->lf[LF_FLAGS].as<const uint32_t>() : (const uint32_t *)nullptr, WgReplayInit{},
                       after ? c->lf[LF_EVOFF].as<const uint32_t>() + n : (const uint32_t *)nullptr);
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}

int wg_lf_events_finish(wg_ctx *c, const LfRange &R, uint32_t ev_base, const uint32_t *xt, uint64_t nx, uint64_t nev,
                        uint32_t world, const uint64_t *d_evoff, const uint64_t *d_auxoff, uint4 *ev, uint32_t *aux) {
    hipStream_t s = c->stream;
    wg_stage_begin(c, "lf_events");
    if (R.nl)
        hipLaunchKernelGGL(k_lf_globalize, dim3(blocks(R.nl)), dim3(T), 0, s, R.nl, ev_base, xt,
                           const_cast<uint32_t *>(lf_sp(c)), c->lf[LF_SECEV].as<uint32_t>(),
                           c->lf[LF_WINFO].as<const uint32_t>());
    if (nev)
        hipLaunchKernelGGL(k_lf_events_finish, dim3(blocks(nev)), dim3(T), 0, s, nev, world, d_evoff, d_auxoff, xt, nx,
                           ev, aux);
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}

// Replays nev global events (records padded with 256 zero records) to the
// fixed point and assigns the lanes of the range; c->max_lane / n_slots.
// The replay's convergence check rides on the lane-scalar read: steady-state
// builds launch exactly the iterations they need with one host sync.
static int replay_lanes_at(wg_ctx *c, const LfRange &R, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *lane,
                           uint32_t nw, bool *ok, bool *overflow, bool narrow = true, bool *was_narrow = nullptr);

static int replay_lanes_dc(wg_ctx *c, const LfRange &R, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *lane,
                           bool *ok, bool *to_serial);

int wg_lf_replay_lanes(wg_ctx *c, const LfRange &R, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *lane,
                       bool *ok) {
    *ok = false;
    // the compacted replay (it needs the consumption times); past its width,
    // its leak snapshots or the serial pass's cost it hands over to the serial pass
    if (c->use_dc() && c->replay_death) {
        bool to_serial = false;
        const int rc = replay_lanes_dc(c, R, nev, ev, aux, lane, ok, &to_serial);
        if (rc != WG_OK || *ok) return rc;
        c->replay_serial = true;   // (auto and mode 3: the serial pass from here on, until it expires)
        c->serial_builds = 0;
    }
    // the occupancy width of the last build first; a replay that overflowed
    // it is redone wider (63 -> 255 -> 1023 slots; 4095 on the serial
    // workgroup); a serial pass in a narrower form (3 of 4 words: 191 slots,
    // 8 of 16: 511) that overflowed is redone at its full width first
    bool narrow = true;
    for (uint32_t nw = c->replay_nw;;) {
        bool overflow = false, was_narrow = false;
        const int rc = replay_lanes_at(c, R, nev, ev, aux, lane, nw, ok, &overflow, narrow, &was_narrow);
        if (rc != WG_OK || !overflow || (nw >= 64 && !was_narrow)) return rc;
        if (was_narrow) { narrow = false; continue; }
        nw = nw < 4 ? 4u : (nw < 16 ? 16u : 64u);
    }
}

// the form code of a serial pass at nw words (wg_debug_counters [12])
static uint32_t serial_form(const ReplayRun &run) {
    if (run.nw <= 1) return 201;
    if (run.nw <= 4) return run.ser_w3 ? 203 : 204;
    if (run.nw <= 16) return run.ser_w8 ? 208 : 216;
    return 264;
}

// The compacted replay's run and buffers (wg_lanes_dchunk.hip) for nev events
// (a bound when the run's nev_dev is set) at nw words of positions.
static int dc_setup(wg_ctx *c, ReplayRun &run, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t nw) {
    run = ReplayRun{};
    run.dc = true;
    run.nev = nev;
    run.nw = nw;
    run.chunk = nev >= WG_REPLAY_WIDE_EVENTS ? 2 * WG_REPLAY_CHUNK_SHORT : WG_REPLAY_CHUNK_SHORT;
    run.warm = c->dc_warm;
    const uint64_t nch = (nev + run.chunk - 1) / run.chunk + 1;
    run.max_iters = (uint32_t)nch + 1;   // always enough to reach the fixed point
    const uint64_t nb = nev / 64 + 2, W = 64ull * nw;
    DevBuf *b = c->lf;
    WG_ALLOC(c, b[LF_SLOT], (nev + 64) * sizeof(uint16_t));
    WG_ALLOC(c, b[LF_SLOTB], (nev + 64) * sizeof(uint16_t));
    WG_ALLOC(c, b[LF_DCVEC], 2 * nch * W * 4);
    WG_ALLOC(c, b[LF_DCMASK], nb * 8);
    WG_ALLOC(c, b[LF_DCPRE], nb * 4);
    WG_ALLOC(c, b[LF_DCLIST], (uint64_t)WG_DC_LEAK_CAP * 4);
    WG_ALLOC(c, b[LF_DCSNAP], ((uint64_t)WG_DC_LEAK_CAP + 1) * W * 2);
    WG_ALLOC(c, b[LF_DCSLOT], (nev + 64) * sizeof(uint16_t));
    WG_ALLOC(c, b[LF_STATS], (nev / WG_DC_FIX_T + 2) * 12);
    WG_ALLOC(c, b[LF_RFLAGS], (run.max_iters + 2) * 4);
    run.ev = ev;
    run.aux = aux;
    run.slots_a = b[LF_SLOT].as<uint16_t>();
    run.slots_b = b[LF_SLOTB].as<uint16_t>();
    run.dc_dvec[0] = b[LF_DCVEC].as<uint32_t>();
    run.dc_dvec[1] = b[LF_DCVEC].as<uint32_t>() + nch * W;
    run.dc_lkmask = b[LF_DCMASK].as<unsigned long long>();
    run.dc_bpre = b[LF_DCPRE].as<uint32_t>();
    run.dc_lklist = b[LF_DCLIST].as<uint32_t>();
    run.dc_snap = b[LF_DCSNAP].as<uint16_t>();
    run.dc_leak_cap = WG_DC_LEAK_CAP;
    run.dc_slot = b[LF_DCSLOT].as<uint16_t>();
    run.stats = b[LF_STATS].as<uint32_t>();
    run.flags = b[LF_RFLAGS].as<uint32_t>();
    run.scal = c->lane_scalars.as<uint32_t>();
    run.death = c->replay_death;
    return WG_OK;
}

// a compacted replay's outcome: the context's scalars and next choices
// (w: max_lane, slots, positions + 1, leaks, first iteration that changed nothing)
static void dc_commit(wg_ctx *c, const ReplayRun &run, uint64_t nev, uint32_t max_lane, uint32_t n_slots, uint32_t positions,
                      uint32_t leaks, uint32_t first_still) {
    c->max_lane = max_lane;
    c->n_slots = n_slots;
    c->replay_nw = wg_ctx::nw_for_slots(n_slots);
    c->replay_iters = run.it;
    const uint32_t w = wg_dc_words(positions);
    c->dc_nw = w ? w : 4u;
    c->last_leaks = leaks;
    c->last_dc_warm = run.warm;
    c->last_form = 300u + run.nw;
    c->last_serial = false;
    c->dc_adapt(first_still, nev, run.nw, run.warm, run.chunk, c->replay_nw);
    c->lane_path = 0;
    // (auto) a list shape with no leaks may suit the chunked replay after all:
    // it is tried again after WG_SERIAL_RETRY such builds (a skewed list's
    // choice does not hold later lists of the same length)
    if (c->replay_mode == 0 && c->replay_dc) {
        c->dc_plain_builds = leaks ? 0u : c->dc_plain_builds + 1u;
        if (c->dc_plain_builds >= wg_ctx::WG_SERIAL_RETRY) {
            c->replay_dc = false;
            c->dc_plain_builds = 0;
            c->replay_blind = 4;
        }
    }
}

// The exact compacted replay: c->dc_blind iterations, then polls; positions
// past the width are redone wider (1 -> 2 -> 4 words).  *to_serial: more
// leaks than the snapshots hold, more than 4 words, or (auto) iterations past
// what the serial pass costs.
static int replay_lanes_dc(wg_ctx *c, const LfRange &R, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *lane,
                           bool *ok, bool *to_serial) {
    hipStream_t s = c->stream;
    *ok = *to_serial = false;
    uint32_t nw = c->dc_nw ? c->dc_nw : 1u;
    for (;;) {
        ReplayRun run;
        int rc = dc_setup(c, run, nev, ev, aux, nw);
        if (rc != WG_OK) return rc;
        // (auto) the iterations after the first that cost what the serial pass does
        const double first = wg_ctx::dc_cost_us(nw, run.warm, run.chunk, 1);
        const double rest = wg_ctx::serial_cost_us(nev, c->replay_nw) - first;
        const uint32_t budget = 2u + (rest > 0 ? (uint32_t)(rest / wg_ctx::dc_iter_us(nw, run.chunk)) : 0u);
        wg_stage_begin(c, "lf_loop");
        WG_HIP(c, wg_dc_init(s, run, true));
        WG_HIP(c, wg_dc_iterate(s, run, c->dc_blind < 2 ? 2u : c->dc_blind));
        const uint32_t *ls = c->lane_scalars.as<const uint32_t>();
        uint64_t w[9] = {0, 0, 0, 0, 0, 0, 0, 1, 1};
        bool conv = false;
        for (;;) {
            WG_HIP(c, wg_dc_finish(s, run));
            WG_HIP(c, wg_dc_scalars(s, run));
            rc = wg_fetch(c, {{ls, false}, {ls + 1, false}, {ls + 2, false}, {ls + 3, false}, {ls + 4, false}, {ls + 5, false},
                              {ls + 6, false}, {run.flags + run.it - 1, false}, {run.flags + run.it, false}}, w);
            if (rc != WG_OK) { wg_stage_end(c); return rc; }
            conv = nev == 0 || w[7] == 0 || w[8] == 0;
            if (conv || run.it >= run.max_iters) break;
            if (c->replay_mode == 0 && run.it >= budget) break;
            WG_HIP(c, wg_dc_iterate(s, run, 4));
        }
        wg_stage_end(c);
        if (!conv || w[6]) { *to_serial = true; return WG_OK; }   // (auto budget spent / more leaks than the snapshots hold)
        if (w[2]) {                                                // positions past the width: wider
            if (nw >= 4) { *to_serial = true; return WG_OK; }
            nw = nw < 2 ? 2u : 4u;
            continue;
        }
        if (R.nl) hipLaunchKernelGGL(k_lf_lanes, dim3(blocks(R.nl)), dim3(T), 0, s, R.nl, lf_sp(c), run.sp_prev, lane);
        WG_HIP(c, hipGetLastError());
        c->lf_slot_of = run.sp_prev;
        dc_commit(c, run, nev, (uint32_t)w[0], (uint32_t)w[1], (uint32_t)w[4], (uint32_t)w[5], (uint32_t)w[3]);
        *ok = true;
        return WG_OK;
    }
}

// the run's buffers and geometry at occupancy width nw (exact and speculative sharded replays)
static int replay_setup(wg_ctx *c, ReplayRun &run, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t nw,
                        bool narrow = true) {
    run.nev = nev;
    run.nw = nw;
    // (the serial pass's cost is its words: 8 instead of 16 when the last
    // list of this context held at most 448 slots, 3 instead of 4 at most
    // 170; a list past 511 / 191 overflows and the caller redoes it at the
    // full width)
    const uint32_t hint = c->slots_hint();
    run.ser_w8 = narrow && nw == 16 && hint > 0 && hint <= 448;
    run.ser_w3 = narrow && nw == 4 && hint > 0 && hint <= 170;
    c->replay_geometry(&run.chunk, &run.warm);
    const uint64_t nch = (nev + run.chunk - 1) / run.chunk + 1;
    run.max_iters = (uint32_t)nch + 1;   // always enough to reach the fixed point
    DevBuf &slot_a = c->lf[LF_SLOT], &slot_b = c->lf[LF_SLOTB], &occ = c->lf[LF_OCC], &stats = c->lf[LF_STATS];
    DevBuf &rflags = c->lf[LF_RFLAGS];
    WG_ALLOC(c, slot_a, (nev + 64) * sizeof(uint16_t));
    WG_ALLOC(c, slot_b, (nev + 64) * sizeof(uint16_t));
    WG_ALLOC(c, occ, (nch * 16 + 16) * nw);
    WG_ALLOC(c, stats, nch * 8 + 8);
    WG_ALLOC(c, rflags, (run.max_iters + 2) * 4);
    run.ev = ev;
    run.aux = aux;
    run.slots_a = slot_a.as<uint16_t>();
    run.slots_b = slot_b.as<uint16_t>();
    run.occ_a = occ.as<unsigned long long>();
    run.occ_b = occ.as<unsigned long long>() + nch * nw;
    run.stats = stats.as<uint32_t>();
    run.flags = rflags.as<uint32_t>();
    run.scal = c->lane_scalars.as<uint32_t>();
    run.death = c->replay_death;
    return WG_OK;
}

// Speculative form (the sharded build's X3 step, wg_shard.hip): the blind
// iterations and the lanes of the range with no host read.  The convergence
// and width words (run.flags[it - 1], run.flags[it], the lane scalars) travel
// in the X6 header (k_sh_x6_head); a replay that was no fixed point is redone
// by wg_lf_replay_lanes then, and wg_lf_replay_spec_commit applies the words.
int wg_lf_replay_lanes_spec(wg_ctx *c, const LfRange &R, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *lane,
                            ReplayRun &run) {
    run = ReplayRun{};
    hipStream_t s = c->stream;
    if (c->use_dc() && c->replay_death) {   // the compacted replay: blind iterations, then its slots and scalars
        int rc = dc_setup(c, run, nev, ev, aux, c->dc_nw ? c->dc_nw : 1u);
        if (rc != WG_OK) return rc;
        wg_stage_begin(c, "lf_loop");
        WG_HIP(c, wg_dc_init(s, run, true));
        WG_HIP(c, wg_dc_iterate(s, run, c->dc_blind < 2 ? 2u : c->dc_blind));
        WG_HIP(c, wg_dc_finish(s, run));
        WG_HIP(c, wg_dc_scalars(s, run));
        if (R.nl) hipLaunchKernelGGL(k_lf_lanes, dim3(blocks(R.nl)), dim3(T), 0, s, R.nl, lf_sp(c), run.sp_prev, lane);
        c->lf_slot_of = run.sp_prev;
        c->last_serial = false;
        WG_HIP(c, hipGetLastError());
        wg_stage_end(c);
        return WG_OK;
    }
    int rc = replay_setup(c, run, nev, ev, aux, c->replay_nw);
    if (rc != WG_OK) return rc;
    wg_stage_begin(c, "lf_loop");
    if (c->use_serial() || run.nw > 16) {   // (past 1023 slots only the serial workgroup replays)
        DevBuf &rec = c->lf[LF_SERREC];
        WG_ALLOC(c, rec, wg_replay_serial_rec_bytes(nev));
        WG_HIP(c, wg_replay_serial(s, run, rec.as<uint4>()));
        c->last_serial = true;
        c->last_form = serial_form(run);
        c->serial_done();
    } else {
        WG_HIP(c, wg_replay_start(c, s, run, c->replay_blind < 2 ? 2u : c->replay_blind));
        c->last_serial = false;
        c->last_form = 100u + run.nw;
    }
    if (R.nl) hipLaunchKernelGGL(k_lf_lanes, dim3(blocks(R.nl)), dim3(T), 0, s, R.nl, lf_sp(c), run.sp_prev, lane);
    c->lf_slot_of = run.sp_prev;
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}

void wg_lf_replay_spec_commit(wg_ctx *c, const ReplayRun &run, uint32_t max_lane, uint32_t n_slots, uint32_t first_still,
                              uint32_t positions, uint32_t leaks) {
    if (run.dc) {
        dc_commit(c, run, c->n_events, max_lane, n_slots, positions, leaks, first_still);
        return;
    }
    c->max_lane = max_lane;
    c->n_slots = n_slots;
    c->replay_nw = wg_ctx::nw_for_slots(n_slots);
    c->replay_iters = run.it;
    c->replay_adapt(first_still, run.chunk);
    c->lane_path = 0;
}

static int replay_lanes_at(wg_ctx *c, const LfRange &R, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *lane,
                           uint32_t nw, bool *ok, bool *overflow, bool narrow, bool *was_narrow) {
    hipStream_t s = c->stream;
    *ok = false;
    *overflow = false;
    ReplayRun run;
    int src = replay_setup(c, run, nev, ev, aux, nw, narrow);
    if (src != WG_OK) return src;
    if (was_narrow) *was_narrow = c->use_serial() && (run.ser_w3 || run.ser_w8);
    if (c->use_serial() || nw > 16) {   // one exact pass: the scalars come with it (past 1023 slots: the only one)
        DevBuf &rec = c->lf[LF_SERREC];
        WG_ALLOC(c, rec, wg_replay_serial_rec_bytes(nev));
        wg_stage_begin(c, "lf_loop");
        WG_HIP(c, wg_replay_serial(s, run, rec.as<uint4>()));
        c->last_serial = true;
        c->last_form = serial_form(run);
        if (R.nl) hipLaunchKernelGGL(k_lf_lanes, dim3(blocks(R.nl)), dim3(T), 0, s, R.nl, lf_sp(c), run.sp_prev, lane);
        c->lf_slot_of = run.sp_prev;
        WG_HIP(c, hipGetLastError());
        const uint32_t *ls = c->lane_scalars.as<const uint32_t>();
        uint64_t sc[3] = {0, 0, 0};
        const int rc = wg_fetch(c, {{ls, false}, {ls + 1, false}, {ls + 2, false}}, sc);
        wg_stage_end(c);
        if (rc != WG_OK) return rc;
        c->replay_iters = 1;
        if (sc[2]) { *overflow = true; return WG_OK; }   // more than 64 nw - 1 slots: the caller widens
        c->max_lane = (uint32_t)sc[0];
        c->n_slots = (uint32_t)sc[1];
        c->replay_nw = wg_ctx::nw_for_slots(c->n_slots);
        c->serial_done();
        *ok = true;
        return WG_OK;
    }
    if (run.chunk < WG_REPLAY_CHUNK_LONG && c->replay_auto) run.switch_it = WG_REPLAY_SWITCH_IT;
    // auto: a replay at the long chunk still moving once its iterations cost
    // what the serial pass would stops there and replays serially
    if (c->replay_mode == 0)
        run.serial_it = 1u + (uint32_t)(wg_ctx::serial_cost_us(nev, nw) / wg_ctx::WG_CHUNKED_ITER_US);
    wg_stage_begin(c, "lf_loop");
    c->last_serial = false;
    c->last_form = 100u + nw;
    WG_HIP(c, wg_replay_start(c, s, run, c->replay_blind));
    const uint32_t blind = run.it;
    const uint32_t *ls = c->lane_scalars.as<const uint32_t>();
    uint64_t sc[6] = {0, 0, 0, 1, 1, 0};
    bool conv = nev == 0;
    for (int pass = 0; pass < 2; pass++) {
        if (R.nl) hipLaunchKernelGGL(k_lf_lanes, dim3(blocks(R.nl)), dim3(T), 0, s, R.nl, lf_sp(c), run.sp_prev, lane);
        c->lf_slot_of = run.sp_prev;
        WG_HIP(c, hipGetLastError());
        if (nev && !conv) {
            int rc = wg_fetch(c, {{ls, false}, {ls + 1, false}, {ls + 2, false}, {run.flags + run.it - 1, false},
                                  {run.flags + run.it, false}, {ls + 3, false}}, sc);
            if (rc != WG_OK) return rc;
            conv = sc[3] == 0 || sc[4] == 0;
        } else {
            int rc = wg_fetch(c, {{ls, false}, {ls + 1, false}, {ls + 2, false}}, sc);
            if (rc == WG_OK && nev) rc = wg_fetch(c, {{ls + 3, false}}, sc + 5);   // (the resumed replay's first no-change iteration)
            if (rc != WG_OK) return rc;
        }
        if (conv) break;
        WG_HIP(c, wg_replay_resume(c, s, run, &conv));   // not there yet: iterate with polls
        if (!conv) break;
    }
    wg_stage_end(c);
    if (run.switched) {   // still moving at the short chunk: this list shape takes the compacted replay (auto) or the long chunk
        c->replay_blind = 4;
        if (c->replay_mode == 0 && c->replay_death) {
            c->replay_dc = true;
            return wg_lf_replay_lanes(c, R, nev, ev, aux, lane, ok);
        }
        c->replay_long = true;
        return replay_lanes_at(c, R, nev, ev, aux, lane, nw, ok, overflow);
    }
    if (run.to_serial) {  // still moving at the long chunk: this list shape replays serially
        c->replay_serial = true;
        return replay_lanes_at(c, R, nev, ev, aux, lane, nw, ok, overflow);
    }
    c->replay_iters = run.it;
    // next build: the iterations this one needed — up to the first iteration
    // that changed nothing (k_lf_replay_finish) — at once if more, halving the
    // excess if fewer (a list that needed many must not hold later ones for long)
    if (sc[5] >= 1) c->replay_adapt((uint32_t)sc[5], run.chunk);
    else if (run.it > blind) c->replay_blind = run.it;
    if (conv && sc[2]) *overflow = true;            // more than 64 nw - 1 slots: the caller widens
    if (!conv || sc[2]) return WG_OK;               // no fixed point / overflow
    c->max_lane = (uint32_t)sc[0];
    c->n_slots = (uint32_t)sc[1];
    c->replay_nw = wg_ctx::nw_for_slots(c->n_slots);
    *ok = true;
    return WG_OK;
}

// Speculative single-GPU lane build (no host read-back): event records sized
// by their upper bound n + E (each row makes at most max(1, parents)
// events; merge token lists hold at most 4/3 (n + E) words), the event count
// read by the kernels from the device, the replay run for the blind
// iteration count of the last build, and every kernel after the
// well-formedness check gated on its flag.  The validation words
// (wg_lanes_spec_check) are read with the end-of-build validation.
static int lanes_fast_spec(wg_ctx *c, const LfRange &R) {
    const uint64_t n = R.nl;
    int rc = wg_lf_refs(c, R, false, c->lane_scalars.as<uint32_t>());
    if (rc != WG_OK) return rc;
    if ((rc = wg_lf_chain(c, R)) != WG_OK) return rc;
    const uint64_t nev_cap = n + c->e_refs, naux_cap = 2 * (n + c->e_refs) + 16;
    const uint32_t *gate = c->lf[LF_FLAGS].as<const uint32_t>();
    const uint32_t *nev_dev = c->lf[LF_EVOFF].as<const uint32_t>() + n;
    DevBuf &evrec = c->lf[LF_EVREC], &aux = c->lf[LF_AUX];
    WG_ALLOC(c, evrec, (nev_cap + 256) * 16);
    WG_ALLOC(c, aux, naux_cap * 4);
    hipStream_t s = c->stream;
    ReplayRun &run = c->spec_run;
    uint32_t blind;
    WgReplayInit RI;
    if (c->use_dc()) {   // the compacted replay (the flag words cleared by the event kernel)
        int rc2 = dc_setup(c, run, nev_cap, evrec.as<const uint4>(), aux.as<const uint32_t>(), c->dc_nw ? c->dc_nw : 1u);
        if (rc2 != WG_OK) return rc2;
        run.nev_dev = nev_dev;
        run.gate = gate;
        run.death = c->lf_death;
        blind = c->dc_blind < 2 ? 2u : c->dc_blind;
        if (blind > run.max_iters) blind = run.max_iters;
        WG_HIP(c, wg_dc_init(s, run, false));
        RI.changed = run.flags;
        RI.nflags = run.max_iters + 2;
        RI.nev_dev = nev_dev;
        RI.total = RI.nflags > 256 ? RI.nflags : 256;
    } else {
        run = ReplayRun{};
        run.nev = nev_cap;
        run.nw = c->replay_nw;
        // (the serial pass's narrower forms, as replay_setup takes them)
        const uint32_t hint = c->slots_hint();   // (wg_stage_lanes cleared n_slots)
        run.ser_w8 = run.nw == 16 && hint > 0 && hint <= 448;
        run.ser_w3 = run.nw == 4 && hint > 0 && hint <= 170;
        c->replay_geometry(&run.chunk, &run.warm);
        const uint64_t nch = (nev_cap + run.chunk - 1) / run.chunk + 1;
        run.max_iters = (uint32_t)nch + 1;
        DevBuf &slot_a = c->lf[LF_SLOT], &slot_b = c->lf[LF_SLOTB], &occ = c->lf[LF_OCC], &stats = c->lf[LF_STATS];
        DevBuf &rflags = c->lf[LF_RFLAGS];
        WG_ALLOC(c, slot_a, (nev_cap + 64) * sizeof(uint16_t));
        WG_ALLOC(c, slot_b, (nev_cap + 64) * sizeof(uint16_t));
        WG_ALLOC(c, occ, (nch * 16 + 16) * run.nw);
        WG_ALLOC(c, stats, nch * 8 + 8);
        WG_ALLOC(c, rflags, (run.max_iters + 2) * 4);
        run.ev = evrec.as<const uint4>();
        run.aux = aux.as<const uint32_t>();
        run.slots_a = slot_a.as<uint16_t>();
        run.slots_b = slot_b.as<uint16_t>();
        run.occ_a = occ.as<unsigned long long>();
        run.occ_b = occ.as<unsigned long long>() + nch * run.nw;
        run.stats = stats.as<uint32_t>();
        run.flags = rflags.as<uint32_t>();
        run.scal = c->lane_scalars.as<uint32_t>();
        run.nev_dev = nev_dev;
        run.gate = gate;
        run.death = c->lf_death;
        blind = c->replay_blind < 2 ? 2u : c->replay_blind;
        RI = wg_replay_prepare_spec(run, blind);
    }
    wg_stage_begin(c, "lf_events");
    hipLaunchKernelGGL(k_lf_events<false>, dim3(blocks(n)), dim3(T), 0, s, R, 0u, 0u, (const uint32_t *)nullptr,
                       c->lf[LF_FIRST].as<const unsigned long long>(), c->lf[LF_WINFO].as<const uint32_t>(),
                       c->lf[LF_EVOFF].as<const uint32_t>(), c->lf[LF_AUXOFF].as<const uint32_t>(),
                       c->lf[LF_CHOFF].as<const uint32_t>(), c->lf[LF_CH].as<const uint32_t>(),
                       c->lf[LF_SECEV].as<const uint32_t>(), lf_sp(c), evrec.as<uint4>(), aux.as<uint32_t>(), gate, RI,
                       nullptr, c->lf_death);
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    wg_stage_begin(c, "lf_loop");
    if (run.dc) {
        WG_HIP(c, wg_dc_iterate(s, run, blind));
        WG_HIP(c, wg_dc_finish(s, run));
        c->last_serial = false;
    } else if (c->use_serial() || run.nw > 16) {   // exact in one pass (the run then reads as converged at iteration 1)
        DevBuf &rec = c->lf[LF_SERREC];
        WG_ALLOC(c, rec, wg_replay_serial_rec_bytes(nev_cap));
        WG_HIP(c, wg_replay_serial(s, run, rec.as<uint4>()));
        c->last_serial = true;
    } else {
        WG_HIP(c, wg_replay_iterate_spec(s, run, blind));
        c->last_serial = false;
    }
    // scalars + lanes + lane_out / colours in one launch (wg_stage_edges skips k_lane_out)
    WG_ALLOC(c, c->lane_out, n * 4 + 4);
    WG_ALLOC(c, c->color_out, n + 4);
    WG_HIP(c, wg_replay_finish_lanes(s, run, n, lf_sp(c), c->lane_asg.as<uint32_t>(), c->lane_out.as<uint32_t>(),
                                     c->color_out.as<uint8_t>(), c->d_flags));
    c->lane_out_fused = true;
    wg_stage_end(c);
    return WG_OK;
}

// The speculative lane build's validation words (WG_LANES_SPEC_ITEMS): {not
// well formed, events, aux words, max_lane, slots, past the occupancy width,
// changed at it - 1, changed at it, first iteration that changed nothing, and
// for the compacted replay its positions + 1, leaks, more leaks than its
// snapshots hold}.
int wg_lanes_spec_items(wg_ctx *c, WgFetch *it) {
    const uint64_t n = c->n;
    const uint32_t *ls = c->lane_scalars.as<const uint32_t>();
    const ReplayRun &run = c->spec_run;
    it[0] = WgFetch{c->lf[LF_FLAGS].p, false};
    it[1] = WgFetch{c->lf[LF_EVOFF].as<uint32_t>() + n, false};
    it[2] = WgFetch{c->lf[LF_AUXOFF].as<uint32_t>() + n, false};
    it[3] = WgFetch{ls, false};
    it[4] = WgFetch{ls + 1, false};
    it[5] = WgFetch{ls + 2, false};
    it[6] = WgFetch{run.flags + run.it - 1, false};
    it[7] = WgFetch{run.flags + run.it, false};
    it[8] = WgFetch{ls + 3, false};   // first iteration that changed nothing
    it[9] = WgFetch{ls + 4, false};
    it[10] = WgFetch{ls + 5, false};
    it[11] = WgFetch{ls + 6, false};
    return WG_LANES_SPEC_ITEMS;
}

// Validation of a speculative lane build from those words: true = the lanes
// are the greedy's (well formed, a fixed point, within the width); c->max_lane,
// n_slots, n_events, the replay's blind count are updated.
bool wg_lanes_spec_check(wg_ctx *c, const uint64_t *v) {
    const bool conv = v[6] == 0 || v[7] == 0;
    const ReplayRun &run = c->spec_run;
    if (v[0] || v[5] || !conv || (run.dc && v[11])) return false;   // (the exact stages redo the lanes)
    c->n_events = v[1];
    if (run.dc) {
        dc_commit(c, run, v[1], (uint32_t)v[3], (uint32_t)v[4], (uint32_t)v[9], (uint32_t)v[10], (uint32_t)v[8]);
        return true;
    }
    c->last_form = c->last_serial ? serial_form(run) : 100u + run.nw;
    if (c->last_serial) c->serial_done();
    c->max_lane = (uint32_t)v[3];
    c->n_slots = (uint32_t)v[4];
    c->replay_nw = wg_ctx::nw_for_slots(c->n_slots);
    c->replay_iters = c->spec_run.it;
    c->replay_adapt((uint32_t)v[8], c->spec_run.chunk);   // blind count and chunk length from the iterations it took
    c->lane_path = 0;
    return true;
}

// Single-GPU build.  Returns WG_OK with *used = false when the input needs
// the general walk.  spec: the speculative form (lanes_fast_spec), *used = true
// and the caller validates.
int wg_lanes_fast(wg_ctx *c, bool *used, bool spec) {
    *used = false;
    LfRange R;
    R.s = 0;
    R.nl = c->n;
    R.e = c->n;
    R.poff = c->d_poff;
    R.prow = c->prow.as<const int32_t>();
    R.canon = c->canon.as<const uint32_t>();
    WG_ALLOC(c, c->lf[LF_LFIRST], c->n * 8 + 8);
    R.lfirst = c->lf[LF_LFIRST].as<unsigned long long>();   // parents at earlier rows stay on this path
    c->e_refs_own = c->e_refs;
    c->replay_shape(c->n);
    if (spec) {
        const int rc = lanes_fast_spec(c, R);
        *used = rc == WG_OK;
        return rc;
    }
    uint32_t viol = 0;
    uint64_t nev = 0, naux = 0;
    int rc = wg_lf_refs(c, R, true, c->lane_scalars.as<uint32_t>());
    if (rc != WG_OK) return rc;
    rc = wg_lf_chain(c, R);                          // queued before the flags are back (bounded on any input)
    const int rc2 = wg_lf_refs_end(c, &viol, &nev, &naux);
    if (rc != WG_OK) return rc;
    if (rc2 != WG_OK) return rc2;
    if (viol) return WG_OK;                          // not well formed: general walk
    c->n_events = nev;
    DevBuf &evrec = c->lf[LF_EVREC], &aux = c->lf[LF_AUX];
    WG_ALLOC(c, evrec, (nev + 256) * 16);
    WG_ALLOC(c, aux, naux * 4 + 4);
    WG_HIP(c, hipMemsetAsync(evrec.as<uint4>() + nev, 0, 256 * 16, c->stream));   // no-op padding for the replay prefetch
    if ((rc = wg_lf_events(c, R, 0, nullptr, evrec.as<uint4>(), aux.as<uint32_t>(), 0)) != WG_OK) return rc;
    bool ok = false;
    c->replay_death = c->lf_death;   // (the whole list's events: the first iteration may use them)
    rc = wg_lf_replay_lanes(c, R, nev, evrec.as<const uint4>(), aux.as<const uint32_t>(), c->lane_asg.as<uint32_t>(), &ok);
    c->replay_death = nullptr;
    if (rc != WG_OK) return rc;
    if (!ok) return WG_OK;                           // no fixed point / more than 63 slots: general walk
    c->lane_path = 0;
    *used = true;
    return WG_OK;
}
