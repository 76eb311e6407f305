// wg_order.hip — the commit list's row order (input
// ingestion and the revwalk order contract).
//
// Reference:
//   commit_graph_with_orphans (git/mod.rs:761-775): the revwalk list
//     (TOPOLOGICAL | TIME, git/mod.rs:569-596) with the reflog orphans
//     appended is re-sorted by time, newest first, with a STABLE sort
//     (`sort_by_key(Reverse(time))`) — only when there are orphans;
//   insert_synthetics_sorted (git/mod.rs:234-242), called before every
//     GraphLayout::build (repo_tab.rs:607-611, 975-980): each synthetic row,
//     in order, is inserted before the first row whose time <= its time (or
//     appended), into the list that already holds the earlier ones.
// The result is a permutation perm[final row] = source row, sources numbered
// walk rows, then orphans, then synthetics.
//
// GPU: a stable LSD radix sort of (tmax - time) with the source index as
// payload (rocPRIM; keys narrowed to the bits the time range needs), one
// pass that finds every synthetic's first base row with time <= t
// (atomicMin per synthetic), the few synthetic-vs-synthetic decisions on the
// host, and one pass that scatters the base rows past the synthetics.
#include "wg_internal.h"

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>

namespace {

constexpr int OT = 256;
inline uint32_t oblocks(uint64_t n) { return (uint32_t)((n + OT - 1) / OT); }

// min / max of time over [0, n): scal[0] = min ^ sign, scal[1] = max ^ sign (order-preserving u64)
__global__ void k_time_range(const int64_t *__restrict__ t, uint64_t n, unsigned long long *scal) {
    unsigned long long lo = ~0ull, hi = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * OT + threadIdx.x; i < n; i += (uint64_t)gridDim.x * OT) {
        const unsigned long long u = (unsigned long long)t[i] ^ 0x8000000000000000ull;
        lo = u < lo ? u : lo;
        hi = u > hi ? u : hi;
    }
    for (int d = 32; d >= 1; d >>= 1) {
        const unsigned long long a = __shfl_down(lo, d, 64), b = __shfl_down(hi, d, 64);
        lo = a < lo ? a : lo;
        hi = b > hi ? b : hi;
    }
    // one atomic pair per workgroup: every wave's atomics on the same two
    // words serialise at the memory side
    __shared__ unsigned long long s_lo[OT / 64], s_hi[OT / 64];
    if ((threadIdx.x & 63) == 0) { s_lo[threadIdx.x >> 6] = lo; s_hi[threadIdx.x >> 6] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < OT / 64; w++) {
            lo = s_lo[w] < lo ? s_lo[w] : lo;
            hi = s_hi[w] > hi ? s_hi[w] : hi;
        }
        atomicMin(scal, lo);
        atomicMax(scal + 1, hi);
    }
}

// key = tmax - time (ascending key = descending time), payload = source row
__global__ void k_sort_keys(const int64_t *__restrict__ tw, uint64_t nw, const int64_t *__restrict__ to, uint64_t n,
                            const unsigned long long *__restrict__ scal, unsigned long long *__restrict__ key,
                            uint32_t *__restrict__ idx) {
    const uint64_t i = (uint64_t)blockIdx.x * OT + threadIdx.x;
    if (i >= n) return;
    const unsigned long long tmax = scal[1];
    const int64_t t = i < nw ? tw[i] : to[i - nw];
    key[i] = tmax - ((unsigned long long)t ^ 0x8000000000000000ull);
    idx[i] = (uint32_t)i;
}

// first base row (in sorted order) with time <= ts[j], for every synthetic j
__global__ void k_syn_first(const uint32_t *__restrict__ perm, uint64_t nb, const int64_t *__restrict__ tw, uint64_t nw,
                            const int64_t *__restrict__ to, const int64_t *__restrict__ ts, uint32_t ns,
                            unsigned int *__restrict__ first) {
    const uint64_t i = (uint64_t)blockIdx.x * OT + threadIdx.x;
    const bool live = i < nb;
    int64_t t = 0;
    if (live) {
        const uint32_t src = perm ? perm[i] : (uint32_t)i;
        t = src < nw ? tw[src] : to[src - nw];
    }
    // wave minimum first: one atomic per wave and synthetic (the per-row
    // atomics on ns words serialised at the memory side)
    for (uint32_t j = 0; j < ns; j++) {
        const bool q = live && t <= ts[j];
        if (!__any(q)) continue;
        uint32_t m = q ? (uint32_t)i : 0xFFFFFFFFu;
        for (int d = 32; d >= 1; d >>= 1) {
            const uint32_t o = (uint32_t)__shfl_down((int)m, d, 64);
            m = o < m ? o : m;
        }
        // early rows usually qualify: skip the atomic once a smaller row is in
        if ((threadIdx.x & 63) == 0 && m != 0xFFFFFFFFu &&
            m < __hip_atomic_load(first + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
            atomicMin(first + j, m);
    }
}

// final position of base row i: i + (synthetics anchored at base rows <= i)
__global__ void k_place(const uint32_t *__restrict__ perm, uint64_t nb, const uint32_t *__restrict__ anchor_sorted,
                        uint32_t ns, uint32_t *__restrict__ out) {
    const uint64_t i = (uint64_t)blockIdx.x * OT + threadIdx.x;
    if (i >= nb) return;
    uint32_t lo = 0, hi = ns;   // count of anchors <= i
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (anchor_sorted[mid] <= (uint32_t)i) lo = mid + 1;
        else hi = mid;
    }
    out[i + lo] = perm ? perm[i] : (uint32_t)i;
}

__global__ void k_put_syn(const uint32_t *__restrict__ pos_src, uint32_t ns, uint32_t *__restrict__ out) {
    const uint32_t j = blockIdx.x * OT + threadIdx.x;
    if (j < ns) out[pos_src[2 * j]] = pos_src[2 * j + 1];
}

}  // namespace

extern "C" {

int wg_order_rows(wg_ctx *c, const int64_t *walk_time, uint64_t n_walk, const int64_t *orphan_time, uint64_t n_orphans,
                  const int64_t *syn_time, uint64_t n_syn, int32_t residency, uint32_t *perm_out, int32_t out_residency) {
    if (!c) return WG_E_INVALID;
    WG_SETTLE(c);
    if ((n_walk && !walk_time) || (n_orphans && !orphan_time) || (n_syn && !syn_time)) return WG_E_INVALID;
    if (residency != WG_HOST && residency != WG_DEVICE) return wg_fail(c, WG_E_INVALID, "bad residency %d", residency);
    if (out_residency != WG_HOST && out_residency != WG_DEVICE)
        return wg_fail(c, WG_E_INVALID, "bad output residency %d", out_residency);
    const uint64_t nb = n_walk + n_orphans, ntot = nb + n_syn;
    if (ntot >= 0xFFFFFFF0ull) return wg_fail(c, WG_E_UNSUPPORTED, "%llu rows exceed 2^32-16", (unsigned long long)ntot);
    if (n_syn > 4096) return wg_fail(c, WG_E_UNSUPPORTED, "more than 4096 synthetic rows");
    (void)hipSetDevice(c->device);
    hipStream_t s = c->stream;
    DevBuf *B = c->ord;   // 0 times, 1 keys, 2 keys out, 3 idx, 4 idx out, 5 rocprim tmp, 6 small, 7 result
    const int64_t *tw = walk_time, *to = orphan_time, *ts = syn_time;
    if (residency == WG_HOST) {
        WG_ALLOC(c, B[0], (ntot + 1) * 8);
        int64_t *d = B[0].as<int64_t>();
        if (n_walk) WG_HIP(c, hipMemcpyAsync(d, walk_time, n_walk * 8, hipMemcpyHostToDevice, s));
        if (n_orphans) WG_HIP(c, hipMemcpyAsync(d + n_walk, orphan_time, n_orphans * 8, hipMemcpyHostToDevice, s));
        if (n_syn) WG_HIP(c, hipMemcpyAsync(d + nb, syn_time, n_syn * 8, hipMemcpyHostToDevice, s));
        tw = d;
        to = d + n_walk;
        ts = d + nb;
    }
    WG_ALLOC(c, B[6], 64 + 16 * n_syn + 16);   // scalars | first base row per synthetic | anchors + (pos, src)
    WG_ALLOC(c, B[7], ntot * 4 + 16);
    wg_stage_begin(c, "order");
    // 1. orphans present: stable sort of walk + orphans by time, newest first (:771-772)
    const uint32_t *perm = nullptr;
    if (n_orphans && nb > 1) {
        WG_ALLOC(c, B[1], nb * 8 + 16);
        WG_ALLOC(c, B[2], nb * 8 + 16);
        WG_ALLOC(c, B[3], nb * 4 + 16);
        WG_ALLOC(c, B[4], nb * 4 + 16);
        unsigned long long *scal = B[6].as<unsigned long long>();
        WG_HIP(c, hipMemsetAsync(scal, 0xFF, 8, s));   // min <- ~0
        WG_HIP(c, hipMemsetAsync(scal + 1, 0, 8, s));  // max <- 0
        const uint32_t g = std::min<uint32_t>(oblocks(nb), 512);
        hipLaunchKernelGGL(k_time_range, dim3(g), dim3(OT), 0, s, tw, n_walk, scal);
        if (n_orphans) hipLaunchKernelGGL(k_time_range, dim3(1), dim3(OT), 0, s, to, n_orphans, scal);
        hipLaunchKernelGGL(k_sort_keys, dim3(oblocks(nb)), dim3(OT), 0, s, tw, n_walk, to, nb, (const unsigned long long *)scal,
                           B[1].as<unsigned long long>(), B[3].as<uint32_t>());
        uint64_t mm[2] = {0, 0};
        if (const int rc = wg_fetch(c, {{scal, true}, {scal + 1, true}}, mm)) return rc;
        const uint64_t range = mm[1] - mm[0];
        const unsigned end_bit = range ? 64u - (unsigned)__builtin_clzll(range) : 1u;
        size_t tmp = 0;
        WG_HIP(c, rocprim::radix_sort_pairs(nullptr, tmp, B[1].as<const unsigned long long>(), B[2].as<unsigned long long>(),
                                            B[3].as<const uint32_t>(), B[4].as<uint32_t>(), (unsigned)nb, 0u, end_bit, s));
        WG_ALLOC(c, B[5], tmp + 16);
        WG_HIP(c, rocprim::radix_sort_pairs(B[5].p, tmp, B[1].as<const unsigned long long>(), B[2].as<unsigned long long>(),
                                            B[3].as<const uint32_t>(), B[4].as<uint32_t>(), (unsigned)nb, 0u, end_bit, s));
        perm = B[4].as<const uint32_t>();
    }
    uint32_t *out = B[7].as<uint32_t>();
    // 2. synthetics, one at a time (git/mod.rs:234-242)
    if (n_syn == 0) {
        if (perm) WG_HIP(c, hipMemcpyAsync(out, perm, nb * 4, hipMemcpyDeviceToDevice, s));
        else if (nb) hipLaunchKernelGGL(k_place, dim3(oblocks(nb)), dim3(OT), 0, s, perm, nb, (const uint32_t *)nullptr, 0u, out);
    } else {
        unsigned int *first = reinterpret_cast<unsigned int *>(B[6].as<uint8_t>() + 64);
        WG_HIP(c, hipMemsetAsync(first, 0xFF, n_syn * 4, s));
        if (nb) hipLaunchKernelGGL(k_syn_first, dim3(oblocks(nb)), dim3(OT), 0, s, perm, nb, tw, n_walk, to, ts,
                                   (uint32_t)n_syn, first);
        std::vector<uint32_t> fb(n_syn);
        std::vector<int64_t> st(n_syn);
        WG_HIP(c, hipMemcpyAsync(fb.data(), first, n_syn * 4, hipMemcpyDeviceToHost, s));
        WG_HIP(c, hipMemcpyAsync(st.data(), ts, n_syn * 8, residency == WG_HOST ? hipMemcpyDeviceToHost : hipMemcpyDefault, s));
        WG_HIP(c, hipStreamSynchronize(s));
        // Each synthetic sits before a base anchor (nb = the end); among those
        // of one anchor, list order is kept as a sequence.  Synthetic j goes
        // before the first row (base or earlier synthetic) with time <= t_j.
        std::vector<std::vector<uint32_t>> at;   // per distinct anchor: synthetics in list order
        std::vector<uint32_t> anchors;           // sorted distinct anchors
        for (uint32_t j = 0; j < n_syn; j++) {
            const uint32_t b = fb[j] == 0xFFFFFFFFu ? (uint32_t)nb : fb[j];
            // earliest qualifying element in list order: walk anchors ascending; within
            // an anchor its synthetics come before the base row itself
            uint32_t ai = 0;
            bool placed = false;
            for (; ai < anchors.size() && anchors[ai] <= b && !placed; ai++) {
                auto &v = at[ai];
                for (size_t k = 0; k < v.size(); k++)
                    if (st[v[k]] <= st[j]) { v.insert(v.begin() + k, j); placed = true; break; }
            }
            if (placed) continue;
            // first qualifying element is base row b (or the end)
            auto it = std::lower_bound(anchors.begin(), anchors.end(), b);
            const size_t pos = (size_t)(it - anchors.begin());
            if (it != anchors.end() && *it == b) at[pos].push_back(j);
            else { anchors.insert(it, b); at.insert(at.begin() + pos, std::vector<uint32_t>{j}); }
        }
        // final positions: synthetic k of anchor a sits at a + (synthetics of anchors < a) + k
        std::vector<uint32_t> anchor_list, pos_src;   // anchor per synthetic (sorted), (position, source) pairs
        uint32_t before = 0;
        for (size_t ai = 0; ai < anchors.size(); ai++) {
            for (size_t k = 0; k < at[ai].size(); k++) {
                anchor_list.push_back(anchors[ai]);
                pos_src.push_back(anchors[ai] + before + (uint32_t)k);
                pos_src.push_back((uint32_t)nb + at[ai][k]);
            }
            before += (uint32_t)at[ai].size();
        }
        uint32_t *danch = reinterpret_cast<uint32_t *>(B[6].as<uint8_t>() + 64 + 4 * n_syn);
        c->ord_host.assign(anchor_list.begin(), anchor_list.end());
        c->ord_host.insert(c->ord_host.end(), pos_src.begin(), pos_src.end());
        WG_HIP(c, hipMemcpyAsync(danch, c->ord_host.data(), c->ord_host.size() * 4, hipMemcpyHostToDevice, s));
        if (nb) hipLaunchKernelGGL(k_place, dim3(oblocks(nb)), dim3(OT), 0, s, perm, nb, (const uint32_t *)danch,
                                   (uint32_t)n_syn, out);
        hipLaunchKernelGGL(k_put_syn, dim3(oblocks(n_syn)), dim3(OT), 0, s, (const uint32_t *)(danch + n_syn),
                           (uint32_t)n_syn, out);
    }
    WG_HIP(c, hipGetLastError());
    wg_stage_end(c);
    c->ord_n = ntot;
    if (perm_out && ntot)
        WG_HIP(c, hipMemcpyAsync(perm_out, out, ntot * 4, out_residency == WG_HOST ? hipMemcpyDeviceToHost
                                                                                    : hipMemcpyDeviceToDevice, s));
    WG_HIP(c, hipStreamSynchronize(s));
    return WG_OK;
}

}  // extern "C"
