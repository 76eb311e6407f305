// wg_lanes.hip — lane assignment and the edge list.
//
// Reference: GraphLayout::build's commit loop (commit_graph.rs:276-295) with
// find_or_assign_lane (:401-412), lowest_free_lane (:414-423), the
// duplicate-waiter free (:287-291), update_lanes_for_parents (:425-460) and
// update_peak (:462-471); colours (:278-283); edge list (:301-320).
//
// The greedy is order dependent: lane INDICES are defined by a sequential
// walk over `active_lanes: Vec<Option<Oid>>`.  This file holds the general
// engine path, a single-wave walk with the slot table held in VGPRs (slot
// s = lane s%64 of register s/64), the commit stream prefetched 64 rows at a
// time and every per-row decision made with wave ballots.  Ids are replaced
// by canonical rows from the hash join, so `Some(oid) == Some(oid')` is an
// integer compare.  Every input the reference accepts is handled here
// exactly (duplicate ids, parents at earlier rows, self parents, repeated
// parents, octopus merges).
#include "wg_internal.h"

namespace {

constexpr int LANE_NCH_MAX = 16;   // up to 1024 slots in registers

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = threadIdx.x & 63;
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

template <int NCH>
struct Slots {
    uint32_t s[NCH];
    uint32_t len;   // active_lanes.len()  (wave-uniform)

    __device__ __forceinline__ void init() {
#pragma unroll
        for (int c = 0; c < NCH; c++) s[c] = WG_EMPTY;
        len = 0;
    }
    // lowest_free_lane (:414-423): lowest None among [0,len); else push.
    __device__ __forceinline__ uint32_t lowest_free(bool &overflow) {
        const uint32_t lid = threadIdx.x & 63;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if ((uint32_t)c * 64 >= len) break;
            uint64_t m = __ballot(s[c] == WG_EMPTY && c * 64 + lid < len);
            if (m) return c * 64 + (uint32_t)__builtin_ctzll(m);
        }
        uint32_t l = len;
        if (l >= (uint32_t)NCH * 64) { overflow = true; return 0; }
        len = l + 1;   // push(None)
        return l;
    }
    __device__ __forceinline__ void set(uint32_t idx, uint32_t v) {
        const uint32_t lid = threadIdx.x & 63;
#pragma unroll
        for (int c = 0; c < NCH; c++)
            if ((idx >> 6) == (uint32_t)c && lid == (idx & 63)) s[c] = v;
    }
    __device__ __forceinline__ bool contains(uint32_t key) {
        uint64_t any = 0;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if ((uint32_t)c * 64 >= len) break;
            any |= __ballot(s[c] == key);
        }
        return any != 0;
    }
    // highest Some index, or -1
    __device__ __forceinline__ int highest_some() {
        int hi = -1;
#pragma unroll
        for (int c = 0; c < NCH; c++) {
            if ((uint32_t)c * 64 >= len) break;
            uint64_t m = __ballot(s[c] != WG_EMPTY);
            if (m) hi = c * 64 + 63 - __builtin_clzll(m);
        }
        return hi;
    }
};

// General single-wave walk.  scal[0] = max_lane, scal[1] = n_slots, scal[2] = overflow
template <int NCH>
__global__ void __launch_bounds__(64) k_lanes_general(uint64_t n, const uint32_t *__restrict__ canon,
                                                     const uint32_t *__restrict__ poff,
                                                     const int32_t *__restrict__ prow,
                                                     uint32_t *__restrict__ lane_asg, uint32_t *__restrict__ scal) {
    const uint32_t lid = threadIdx.x & 63;
    Slots<NCH> S;
    S.init();
    int max_lane = 0;
    bool overflow = false;
    for (uint64_t base = 0; base < n && !overflow; base += 64) {
        const uint64_t i = base + lid;
        const bool valid = i < n;
        const uint32_t key_v = valid ? canon[i] : 0u;
        const uint32_t pa_v = valid ? poff[i] : 0u;
        const uint32_t pb_v = valid ? poff[i + 1] : 0u;
        const int32_t fp_v = (valid && pb_v > pa_v) ? prow[pa_v] : -1;
        const int32_t s1_v = (valid && pb_v > pa_v + 1) ? prow[pa_v + 1] : -1;
        uint32_t out_v = 0;
        const int cnt = (int)((n - base) < 64 ? (n - base) : 64);
        for (int j = 0; j < cnt; j++) {
            const uint32_t key = __builtin_amdgcn_readlane(key_v, j);
            const uint32_t pa = __builtin_amdgcn_readlane(pa_v, j);
            const uint32_t pb = __builtin_amdgcn_readlane(pb_v, j);
            const int32_t fpk = __builtin_amdgcn_readlane(fp_v, j);
            const int32_t s1 = __builtin_amdgcn_readlane(s1_v, j);
            // find_or_assign_lane (:401-412) + free duplicate waiters (:287-291)
            uint32_t lane = WG_EMPTY;
#pragma unroll
            for (int c = 0; c < NCH; c++) {
                if ((uint32_t)c * 64 >= S.len) break;
                const uint64_t m = __ballot(S.s[c] == key);
                if (m) {
                    if (lane == WG_EMPTY) lane = c * 64 + (uint32_t)__builtin_ctzll(m);
                    if (S.s[c] == key && c * 64 + lid != lane) S.s[c] = WG_EMPTY;
                }
            }
            if (lane == WG_EMPTY) lane = S.lowest_free(overflow);
            if (overflow) break;
            if (lid == (uint32_t)j) out_v = lane;
            // update_lanes_for_parents (:425-460)
            if (pb == pa) {
                S.set(lane, WG_EMPTY);
            } else {
                S.set(lane, fpk >= 0 ? (uint32_t)fpk : WG_EMPTY);
                for (uint32_t k = pa + 1; k < pb; k++) {
                    const int32_t q = (k == pa + 1) ? s1 : prow[k];
                    if (q < 0) continue;                       // !commit_set.contains_key
                    if (S.contains((uint32_t)q)) continue;     // active_lanes.contains
                    const uint32_t nl = S.lowest_free(overflow);
                    if (overflow) break;
                    S.set(nl, (uint32_t)q);
                }
                if (overflow) break;
            }
            // update_peak (:462-471)
            const int hi = S.highest_some();
            if (hi > max_lane) max_lane = hi;
        }
        if (valid) lane_asg[i] = out_v;
    }
    if (lid == 0) {
        scal[0] = (uint32_t)max_lane;
        scal[1] = S.len;
        scal[2] = overflow ? 1u : 0u;
    }
}

// layouts.get(id) per row + colour rule (:278-283, history_view :1363-1367)
__global__ void k_lane_out(uint64_t n, const uint32_t *__restrict__ canon, const uint32_t *__restrict__ lane_asg,
                           const uint8_t *__restrict__ flags, uint32_t *__restrict__ lane_out,
                           uint8_t *__restrict__ color_out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t ci = canon[i];
    const uint32_t l = lane_asg[ci];
    lane_out[i] = l;
    color_out[i] = (flags[ci] & WG_FLAG_ORPHAN) ? (uint8_t)WG_COLOR_ORPHAN : (uint8_t)(l % 6u);
}

template <int NCH>
hipError_t launch_general(wg_ctx *c) {
    hipLaunchKernelGGL((k_lanes_general<NCH>), dim3(1), dim3(64), 0, c->stream, c->n, c->canon.as<const uint32_t>(),
                       c->d_poff, c->prow.as<const int32_t>(), c->lane_asg.as<uint32_t>(), c->lane_scalars.as<uint32_t>());
    return hipGetLastError();
}

}  // namespace

// spec: the speculative build (wg_layout_build validates afterwards; the
// general walk is only taken from the exact form)
int wg_stage_lanes(wg_ctx *c, bool spec) {
    const uint64_t n = c->n;
    WG_ALLOC(c, c->lane_asg, n * 4 + 4);
    WG_ALLOC(c, c->lane_scalars, 64);
    c->max_lane = 0;
    if (c->n_slots) c->slots_last = c->n_slots;   // (the replay's narrow forms follow the last list's slots)
    c->n_slots = 0;
    c->lane_path = 1;
    c->graph_width = WG_LANE_W;   // max_lane 0 -> one visible lane (:353-354)
    c->lane_out_fused = false;
    if (n == 0) return WG_OK;
    wg_stage_begin(c, "lanes");
    if (!c->force_general_lanes) {   // (the fast path's first kernel clears the lane scalars)
        bool used = false;
        int rc = wg_lanes_fast(c, &used, spec);
        if (rc != WG_OK) return rc;
        if (spec) {   // max_lane / graph_width are set by the validation
            wg_stage_end(c);
            return WG_OK;
        }
        if (used) {
            wg_stage_end(c);
            uint32_t vis = c->max_lane + 1 < (uint32_t)WG_LANE_COUNT_VISUAL ? c->max_lane + 1 : (uint32_t)WG_LANE_COUNT_VISUAL;
            float gw = (float)vis * WG_LANE_W;
            c->graph_width = gw > WG_LANE_W ? gw : WG_LANE_W;
            return WG_OK;
        }
    }
    WG_HIP(c, hipMemsetAsync(c->lane_scalars.p, 0, 64, c->stream));
    WG_HIP(c, launch_general<1>(c));
    const uint32_t *ls = c->lane_scalars.as<const uint32_t>();
    uint64_t sc[3];
    int frc = wg_fetch(c, {{ls, false}, {ls + 1, false}, {ls + 2, false}}, sc);
    if (frc != WG_OK) return frc;
    if (sc[2]) {   // more than 64 slots: rerun with the wide slot table
        WG_HIP(c, launch_general<LANE_NCH_MAX>(c));
        frc = wg_fetch(c, {{ls, false}, {ls + 1, false}, {ls + 2, false}}, sc);
        if (frc != WG_OK) return frc;
        if (sc[2]) return wg_fail(c, WG_E_UNSUPPORTED, "lane table exceeds %d slots", LANE_NCH_MAX * 64);
    }
    wg_stage_end(c);
    c->max_lane = (uint32_t)sc[0];
    c->n_slots = (uint32_t)sc[1];
    uint32_t vis = c->max_lane + 1 < (uint32_t)WG_LANE_COUNT_VISUAL ? c->max_lane + 1 : (uint32_t)WG_LANE_COUNT_VISUAL;
    float gw = (float)vis * WG_LANE_W;                 // graph_width (:353-354)
    c->graph_width = gw > WG_LANE_W ? gw : WG_LANE_W;
    return WG_OK;
}

// ne_known >= 0: the edge count, already read.  spec: the edge count is not
// read back here; the buffer is sized by its upper
// bound (the parent references), c->n_edges holds that bound until the
// end-of-build validation and the geometry kernels read the count from
// edge_cnt[n] on the device
int wg_stage_edges(wg_ctx *c, bool spec, int64_t ne_known) {
    const uint64_t n = c->n;
    WG_ALLOC(c, c->lane_out, n * 4 + 4);
    WG_ALLOC(c, c->color_out, n + 4);
    c->n_edges = 0;
    if (n == 0) {
        WG_ALLOC(c, c->edge_cnt, 16);
        WG_HIP(c, hipMemsetAsync(c->edge_cnt.p, 0, 4, c->stream));
        return WG_OK;
    }
    wg_stage_begin(c, "edges");
    const int T = 256;
    if (!c->lane_out_fused)   // (the speculative fast path's lane kernel wrote them)
        hipLaunchKernelGGL(k_lane_out, dim3((n + T - 1) / T), dim3(T), 0, c->stream, n, c->canon.as<const uint32_t>(),
                           c->lane_asg.as<const uint32_t>(), c->d_flags, c->lane_out.as<uint32_t>(), c->color_out.as<uint8_t>());
    WG_HIP(c, hipGetLastError());
    // edge offsets: scanned after the hash join (wg_stage_hash_join); the
    // total was copied out then and the lane stage has synchronised since
    uint64_t ne = c->e_refs;
    if (ne_known >= 0) ne = (uint64_t)ne_known;   // read by the caller (a speculative build's validation)
    else if (!spec)
        if (const int rc = wg_fetch_deferred(c, &ne)) return rc;
    c->n_edges = ne;
    WG_ALLOC(c, c->edges, (uint64_t)ne * sizeof(wg_edge) + 16);
    // the records are written by the full geometry pass that follows every
    // layout build (wg_geom.hip k_edges_rows, with the pass's first counts)
    c->edges_pending = true;
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    return WG_OK;
}
