// wg_lanes_fast.hip — event-compressed lane assignment (SURVEY.md §7 hard
// part 1), bit-identical to GraphLayout::build's greedy (commit_graph.rs:
// 276-295, 401-471) on well-formed commit lists.
//
// Well-formed = every id distinct and every in-list parent at a larger row
// (checked in parallel; anything else — duplicate ids, clock-skewed parents,
// self parents — takes the general walk in wg_lanes.hip).  Then the
// sequential state has a static description:
//   * a slot waiting for commit j is set only by a child of j (rows < j) and
//     stays until row j, so the waiters of j are: one slot per first-parent
//     child, plus one slot if the FIRST in-list reference to j (row, parent
//     index order) is a secondary parent (:447-459 allocates only then);
//   * w(j) = #waiters.  w = 1: j inherits its single waiter's slot (no state
//     change).  w = 0: lowest free slot (ALLOC).  w >= 2: lowest waiter slot,
//     the others freed (MIN, :287-291).  First parent outside the list: the
//     slot is freed (FREE) or never occupied (probe ALLOC).  First
//     references through a secondary parent: SECALLOC (:454-458).
// Only those events touch the slot-occupancy state, and they are a few
// percent of rows.  The pipeline:
//   refs     first reference + first-parent child count per row (atomics)
//   rows     w(j), event counts -> scan -> event ids
//   chain    every row's "source" event via pointer jumping along w = 1
//            first-parent chains (log2 N rounds)
//   events   16-byte event records in row order
//   replay   the event stream cut into chunks replayed in parallel and
//            iterated to a fixed point (wg_lanes_replay.hip): 64-bit
//            occupancy mask, lowest-free = ctz(~occ)
//   lanes    lane[j] = slot of source(j)   (parallel gather)
// max_lane = max over occupying allocations of the highest occupied slot
// (update_peak, :462-471, can only rise when a slot is taken).
#include "wg_internal.h"

namespace {

constexpr int T = 256;
constexpr uint32_t EVF = 0x80000000u;   // "is an event id" tag in the chain pointers
constexpr uint64_t REF_NONE = ~0ull;

// event record flags (uint4.x): A = takes the lowest free slot, O = occupies
// its slot afterwards, C = clears its token slots (MIN / FREE), M = more than
// two waiters (tokens read from the child list); IN0/IN1 = token 0/1 lives in
// the event's own 64-event batch at local index bits 8..13 / 16..21.
enum : uint32_t { F_A = 1u, F_O = 2u, F_C = 4u, F_M = 8u, F_IN0 = 1u << 14, F_IN1 = 1u << 22 };
// replay word (per lane, built at batch start): bits 0..3 flags, 8..15 / 16..23 token slots
enum : uint32_t { X_IN0 = 1u << 4, X_IN1 = 1u << 5 };

__device__ __forceinline__ uint32_t token_bits(uint32_t e, uint32_t t0, uint32_t t1) {
    uint32_t b = ((t0 & 63u) << 8) | ((t1 & 63u) << 16);
    if ((t0 >> 6) == (e >> 6)) b |= F_IN0;
    if ((t1 >> 6) == (e >> 6)) b |= F_IN1;
    return b;
}

inline uint32_t blocks(uint64_t n) { return (uint32_t)((n + T - 1) / T); }

// is parent ref k of row i the first occurrence of that parent in the row's in-list refs?
__device__ __forceinline__ bool first_in_row(const int32_t *__restrict__ prow, uint32_t pa, uint32_t k, int32_t p) {
    for (uint32_t q = pa; q < k; q++)
        if (prow[q] == p) return false;
    return true;
}

__global__ void k_lf_refs(uint64_t n, const uint32_t *__restrict__ canon, const uint32_t *__restrict__ poff,
                          const int32_t *__restrict__ prow, unsigned long long *first_ref, uint32_t *fpc,
                          uint32_t *viol) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    bool bad = canon[i] != (uint32_t)i;
    const uint32_t pa = poff[i], pb = poff[i + 1];
    for (uint32_t k = pa; k < pb; k++) {
        const int32_t p = prow[k];
        if (p < 0) continue;
        if ((uint64_t)p <= i) { bad = true; continue; }
        if (k - pa > 0xFFFFu) { bad = true; continue; }
        if (!first_in_row(prow, pa, k, p)) continue;
        atomicMin(&first_ref[p], ((unsigned long long)i << 16) | (k - pa));
        if (k == pa) atomicAdd(&fpc[p], 1u);
    }
    if (bad) atomicOr(viol, 1u);
}

// per row: w, first-parent-in-list, event count
__global__ void k_lf_rows(uint64_t n, const uint32_t *__restrict__ poff, const int32_t *__restrict__ prow,
                          const unsigned long long *__restrict__ first_ref, const uint32_t *__restrict__ fpc,
                          uint32_t *__restrict__ winfo, uint32_t *__restrict__ ev_cnt) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const unsigned long long fr = first_ref[j];
    const uint32_t sec_first = (fr != REF_NONE && (fr & 0xFFFFu) != 0) ? 1u : 0u;
    const uint32_t w = fpc[j] + sec_first;
    const uint32_t pa = poff[j], pb = poff[j + 1];
    const bool fp_in = pb > pa && prow[pa] >= 0;
    uint32_t nc = 0;
    for (uint32_t k = pa + 1; k < pb; k++) {
        const int32_t p = prow[k];
        if (p >= 0 && first_ref[p] == (((unsigned long long)j << 16) | (k - pa))) nc++;
    }
    const uint32_t na = (w != 1) ? 1u : 0u;
    const uint32_t nb = (w == 1 && !fp_in) ? 1u : 0u;
    winfo[j] = (w < 0x3FFFFFFFu ? w : 0x3FFFFFFFu) | (fp_in ? 0x40000000u : 0u) | (sec_first ? 0x80000000u : 0u);
    ev_cnt[j] = na + nb + nc;
}

// SECALLOC event id of every parent whose first reference is secondary
__global__ void k_lf_secev(uint64_t n, const uint32_t *__restrict__ poff, const int32_t *__restrict__ prow,
                           const unsigned long long *__restrict__ first_ref, const uint32_t *__restrict__ winfo,
                           const uint32_t *__restrict__ ev_off, uint32_t *__restrict__ secev) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t wi = winfo[j], w = wi & 0x3FFFFFFFu;
    const bool fp_in = wi & 0x40000000u;
    uint32_t e = ev_off[j] + ((w != 1) ? 1u : 0u) + ((w == 1 && !fp_in) ? 1u : 0u);
    const uint32_t pa = poff[j], pb = poff[j + 1];
    for (uint32_t k = pa + 1; k < pb; k++) {
        const int32_t p = prow[k];
        if (p >= 0 && first_ref[p] == (((unsigned long long)j << 16) | (k - pa))) secev[p] = e++;
    }
}

__global__ void k_lf_children(uint64_t n, const uint32_t *__restrict__ poff, const int32_t *__restrict__ prow,
                              const uint32_t *__restrict__ ch_off, uint32_t *ch_fill, uint32_t *ch) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t pa = poff[i];
    if (pa == poff[i + 1]) return;
    const int32_t p = prow[pa];
    if (p < 0) return;
    ch[ch_off[p] + atomicAdd(&ch_fill[p], 1u)] = (uint32_t)i;
}

__global__ void k_lf_sp_init(uint64_t n, const uint32_t *__restrict__ winfo, const uint32_t *__restrict__ ev_off,
                             const uint32_t *__restrict__ ch_off, const uint32_t *__restrict__ ch,
                             const uint32_t *__restrict__ secev, uint32_t *__restrict__ sp) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t wi = winfo[j], w = wi & 0x3FFFFFFFu;
    if (w != 1) sp[j] = EVF | ev_off[j];                       // own ALLOC / MIN event
    else if (wi & 0x80000000u) sp[j] = EVF | secev[j];          // waiter = secondary allocation
    else sp[j] = ch[ch_off[j]];                                 // waiter = the only first-parent child
}

__global__ void k_lf_jump(uint64_t n, const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint32_t *changed) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t v = in[j];
    uint32_t o = v;
    if (!(v & EVF)) o = in[v];
    out[j] = o;
    if (!(o & EVF) && changed) *changed = 1u;
}

__global__ void k_lf_events(uint64_t n, const uint32_t *__restrict__ poff, const int32_t *__restrict__ prow,
                            const unsigned long long *__restrict__ first_ref, const uint32_t *__restrict__ winfo,
                            const uint32_t *__restrict__ ev_off, const uint32_t *__restrict__ ch_off,
                            const uint32_t *__restrict__ ch, const uint32_t *__restrict__ secev,
                            const uint32_t *__restrict__ sp, uint4 *__restrict__ ev) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint32_t wi = winfo[j], w = wi & 0x3FFFFFFFu;
    const bool fp_in = wi & 0x40000000u, sec_first = wi & 0x80000000u;
    uint32_t e = ev_off[j];
    if (w == 0) {
        ev[e] = make_uint4(fp_in ? (F_A | F_O) : F_A, 0u, 0u, (uint32_t)j);
        e++;
    } else if (w >= 2) {
        // tokens: sources of the first-parent children, plus the secondary allocation
        uint32_t t[2] = {0u, 0u};
        uint32_t nt = 0;
        for (uint32_t k = ch_off[j]; k < ch_off[j + 1] && nt < 2; k++) t[nt++] = sp[ch[k]] & ~EVF;
        if (sec_first && nt < 2) t[nt++] = secev[j];
        const uint32_t f = F_C | (fp_in ? F_O : 0u) | ((w > 2) ? F_M : 0u);
        ev[e] = make_uint4(f | token_bits(e, t[0], t[1]), t[0], t[1], (uint32_t)j);
        e++;
    } else if (!fp_in) {
        const uint32_t t0 = sp[j] & ~EVF;
        ev[e] = make_uint4(F_C | token_bits(e, t0, t0), t0, t0, (uint32_t)j);
        e++;
    }
    const uint32_t pa = poff[j], pb = poff[j + 1];
    for (uint32_t k = pa + 1; k < pb; k++) {
        const int32_t p = prow[k];
        if (p >= 0 && first_ref[p] == (((unsigned long long)j << 16) | (k - pa))) {
            ev[e] = make_uint4(F_A | F_O, 0u, 0u, (uint32_t)j);
            e++;
        }
    }
}

__global__ void k_lf_lanes(uint64_t n, const uint32_t *__restrict__ sp, const uint8_t *__restrict__ slot_of,
                           uint32_t *__restrict__ lane) {
    uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    lane[j] = slot_of[sp[j] & ~EVF];
}

}  // namespace

// Returns WG_OK with *used = false when the input needs the general walk.
int wg_lanes_fast(wg_ctx *c, bool *used) {
    *used = false;
    const uint64_t n = c->n, e = c->e_refs;
    hipStream_t s = c->stream;
    DevBuf &first_ref = c->lf[0], &fpc = c->lf[1], &winfo = c->lf[2], &ev_off = c->lf[3], &secev = c->lf[4];
    DevBuf &ch_off = c->lf[5], &ch_fill = c->lf[6], &ch = c->lf[7], &spA = c->lf[8], &spB = c->lf[9];
    DevBuf &evrec = c->lf[10], &slot_of = c->lf[11], &flags = c->lf[12];
    WG_ALLOC(c, first_ref, n * 8 + 8);
    WG_ALLOC(c, fpc, (n + 2) * 4);
    WG_ALLOC(c, winfo, n * 4 + 4);
    WG_ALLOC(c, ev_off, (n + 2) * 4);
    WG_ALLOC(c, secev, n * 4 + 4);
    WG_ALLOC(c, ch_off, (n + 2) * 4);
    WG_ALLOC(c, ch_fill, (n + 2) * 4);
    WG_ALLOC(c, ch, e * 4 + 4);
    WG_ALLOC(c, spA, n * 4 + 4);
    WG_ALLOC(c, spB, n * 4 + 4);
    WG_ALLOC(c, flags, 64);
    WG_ALLOC(c, c->scan_tmp, wg_scan_tmp_bytes(n + 2));
    const uint32_t *poff = c->d_poff;
    const int32_t *prow = c->prow.as<const int32_t>();

    wg_stage_begin(c, "lf_refs");
    WG_HIP(c, hipMemsetAsync(first_ref.p, 0xFF, n * 8, s));
    WG_HIP(c, hipMemsetAsync(fpc.p, 0, (n + 2) * 4, s));
    WG_HIP(c, hipMemsetAsync(ch_fill.p, 0, (n + 2) * 4, s));
    WG_HIP(c, hipMemsetAsync(flags.p, 0, 64, s));
    hipLaunchKernelGGL(k_lf_refs, dim3(blocks(n)), dim3(T), 0, s, n, c->canon.as<const uint32_t>(), poff, prow,
                       first_ref.as<unsigned long long>(), fpc.as<uint32_t>(), flags.as<uint32_t>());
    hipLaunchKernelGGL(k_lf_rows, dim3(blocks(n)), dim3(T), 0, s, n, poff, prow, first_ref.as<const unsigned long long>(),
                       fpc.as<const uint32_t>(), winfo.as<uint32_t>(), ev_off.as<uint32_t>());
    WG_HIP(c, wg_exclusive_scan_u32(ev_off.as<uint32_t>(), ev_off.as<uint32_t>(), n, c->scan_tmp.p, s));
    uint32_t hdr[2] = {0, 0};
    WG_HIP(c, hipMemcpyAsync(&hdr[0], flags.p, 4, hipMemcpyDeviceToHost, s));
    WG_HIP(c, hipMemcpyAsync(&hdr[1], ev_off.as<uint32_t>() + n, 4, hipMemcpyDeviceToHost, s));
    WG_HIP(c, hipStreamSynchronize(s));
    wg_stage_end(c);
    if (hdr[0]) return WG_OK;                       // not well formed: general walk
    const uint64_t nev = hdr[1];
    c->n_events = nev;
    WG_ALLOC(c, evrec, (nev + 256) * 16);
    WG_HIP(c, hipMemsetAsync(evrec.as<uint4>() + nev, 0, 256 * 16, s));   // no-op padding for the replay prefetch
    WG_ALLOC(c, slot_of, nev + 64);
    wg_stage_begin(c, "lf_chain");
    hipLaunchKernelGGL(k_lf_secev, dim3(blocks(n)), dim3(T), 0, s, n, poff, prow, first_ref.as<const unsigned long long>(),
                       winfo.as<const uint32_t>(), ev_off.as<const uint32_t>(), secev.as<uint32_t>());
    // first-parent children CSR
    WG_HIP(c, wg_exclusive_scan_u32(fpc.as<uint32_t>(), ch_off.as<uint32_t>(), n, c->scan_tmp.p, s));
    hipLaunchKernelGGL(k_lf_children, dim3(blocks(n)), dim3(T), 0, s, n, poff, prow, ch_off.as<const uint32_t>(),
                       ch_fill.as<uint32_t>(), ch.as<uint32_t>());
    hipLaunchKernelGGL(k_lf_sp_init, dim3(blocks(n)), dim3(T), 0, s, n, winfo.as<const uint32_t>(),
                       ev_off.as<const uint32_t>(), ch_off.as<const uint32_t>(), ch.as<const uint32_t>(),
                       secev.as<const uint32_t>(), spA.as<uint32_t>());
    // pointer jumping: after r rounds every pointer skips 2^r chain links
    int rounds = 1;
    while ((1ull << rounds) < n + 1) rounds++;
    DevBuf *in = &spA, *out = &spB;
    for (int r = 0; r < rounds; r++) {
        hipLaunchKernelGGL(k_lf_jump, dim3(blocks(n)), dim3(T), 0, s, n, in->as<const uint32_t>(), out->as<uint32_t>(),
                           (uint32_t *)nullptr);
        DevBuf *t = in; in = out; out = t;
    }
    const uint32_t *sp = in->as<const uint32_t>();
    wg_stage_end(c);
    wg_stage_begin(c, "lf_events");
    hipLaunchKernelGGL(k_lf_events, dim3(blocks(n)), dim3(T), 0, s, n, poff, prow, first_ref.as<const unsigned long long>(),
                       winfo.as<const uint32_t>(), ev_off.as<const uint32_t>(), ch_off.as<const uint32_t>(),
                       ch.as<const uint32_t>(), secev.as<const uint32_t>(), sp, evrec.as<uint4>());
    wg_stage_end(c);
    wg_stage_begin(c, "lf_loop");
    const uint32_t chunk = c->replay_chunk;
    const uint64_t nch = (nev + chunk - 1) / chunk + 1;
    const uint32_t max_iters = (uint32_t)nch + 1;   // always enough to reach the fixed point
    DevBuf &slot_b = c->lf[13], &occ = c->lf[14], &stats = c->lf[15], &rflags = c->lf[16];
    WG_ALLOC(c, slot_b, nev + 64);
    WG_ALLOC(c, occ, nch * 16 + 16);
    WG_ALLOC(c, stats, nch * 8 + 8);
    WG_ALLOC(c, rflags, (max_iters + 2) * 4);
    uint8_t *slots = nullptr;
    uint32_t iters = 0;
    WG_HIP(c, wg_lane_replay(s, nev, chunk, evrec.as<const uint4>(), ch_off.as<const uint32_t>(), ch.as<const uint32_t>(),
                             sp, secev.as<const uint32_t>(), winfo.as<const uint32_t>(), slot_of.as<uint8_t>(),
                             slot_b.as<uint8_t>(), occ.as<unsigned long long>(), occ.as<unsigned long long>() + nch,
                             stats.as<uint32_t>(), rflags.as<uint32_t>(), max_iters, c->lane_scalars.as<uint32_t>(),
                             &slots, &iters));
    c->replay_iters = iters;
    wg_stage_end(c);
    if (iters > max_iters) return WG_OK;            // no fixed point within budget: general walk
    hipLaunchKernelGGL(k_lf_lanes, dim3(blocks(n)), dim3(T), 0, s, n, sp, (const uint8_t *)slots,
                       c->lane_asg.as<uint32_t>());
    WG_HIP(c, hipGetLastError());
    uint32_t sc[4];
    WG_HIP(c, hipMemcpyAsync(sc, c->lane_scalars.p, 16, hipMemcpyDeviceToHost, s));
    WG_HIP(c, hipStreamSynchronize(s));
    if (sc[2]) return WG_OK;                        // more than 63 slots: general walk
    c->max_lane = sc[0];
    c->n_slots = sc[1];
    c->lane_path = 0;
    *used = true;
    return WG_OK;
}
