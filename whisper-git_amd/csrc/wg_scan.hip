// wg_scan.hip — exclusive prefix sums (CSR offsets of rows, edges, vertices).
//
// Reduce-then-scan over tiles of 2048 elements (256 threads x 8 items,
// wave64 shuffles + one LDS exchange per block); tile sums are scanned
// recursively.  Used for every CSR offset array of the engine.
#include "wg_internal.h"

namespace {

constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 8;
constexpr uint64_t SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

// The 8 items of a thread: two 16-byte loads / stores when in bounds and
// aligned (uniform: every thread's base is a multiple of 8 items), else one
// item at a time
template <class TI, class TO>
__device__ __forceinline__ void load8(const TI *in, uint64_t base, uint64_t n, TO (&v)[SCAN_ITEMS]) {
    if constexpr (sizeof(TI) == 4) {
        if (base + SCAN_ITEMS <= n && (reinterpret_cast<uintptr_t>(in) & 15) == 0) {
            const uint4 a = reinterpret_cast<const uint4 *>(in + base)[0], b = reinterpret_cast<const uint4 *>(in + base)[1];
            v[0] = (TO)a.x; v[1] = (TO)a.y; v[2] = (TO)a.z; v[3] = (TO)a.w;
            v[4] = (TO)b.x; v[5] = (TO)b.y; v[6] = (TO)b.z; v[7] = (TO)b.w;
            return;
        }
    }
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) v[k] = (base + k < n) ? (TO)in[base + k] : (TO)0;
}
template <class TO>
__device__ __forceinline__ void store8(TO *out, uint64_t base, uint64_t n, const TO (&v)[SCAN_ITEMS]) {
    if constexpr (sizeof(TO) == 4) {
        if (base + SCAN_ITEMS <= n && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
            reinterpret_cast<uint4 *>(out + base)[0] = make_uint4((uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]);
            reinterpret_cast<uint4 *>(out + base)[1] = make_uint4((uint32_t)v[4], (uint32_t)v[5], (uint32_t)v[6], (uint32_t)v[7]);
            return;
        }
    }
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++)
        if (base + k < n) out[base + k] = v[k];
}

template <class T>
__device__ __forceinline__ T wave_incl_scan(T v) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (lane >= d) v += o;
    }
    return v;
}

// returns the exclusive block prefix of v and the block total
template <class T>
__device__ __forceinline__ T block_excl_scan(T v, T &total) {
    __shared__ T wsum[SCAN_THREADS / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    T inc = wave_incl_scan(v);
    if (lane == 63) wsum[wid] = inc;
    __syncthreads();
    T base = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < SCAN_THREADS / 64; w++) {
        T s = wsum[w];
        if (w < wid) base += s;
        tot += s;
    }
    __syncthreads();
    total = tot;
    return base + inc - v;
}

template <class TI, class TO>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_reduce(const TI *__restrict__ in, TO *__restrict__ bsum, uint64_t n) {
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    TO v[SCAN_ITEMS];
    load8<TI, TO>(in, base, n, v);
    TO s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) s += v[k];
    TO tot;
    (void)block_excl_scan<TO>(s, tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

template <class TI, class TO>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_down(const TI *in, TO *out, const TO *__restrict__ boff, uint64_t n) {
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    TO v[SCAN_ITEMS];
    load8<TI, TO>(in, base, n, v);
    TO s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) s += v[k];
    TO tot;
    TO run = block_excl_scan<TO>(s, tot) + (boff ? boff[blockIdx.x] : (TO)0);
    TO o[SCAN_ITEMS];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        o[k] = run;
        run += v[k];
    }
    store8<TO>(out, base, n, o);
    // the thread holding the last element writes the grand total to out[n]
    if (n > 0 && base <= n - 1 && n - 1 < base + SCAN_ITEMS) out[n] = run;
    if (n == 0 && blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
}

// down-sweep whose block offset is the sum of the preceding tile sums,
// reduced by the block itself (tile count <= SCAN_TILE): no separate scan of
// the tile sums
template <class TI, class TO>
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_down2(const TI *in, TO *out, const TO *__restrict__ bsum, uint64_t n) {
    TO pre = 0;
    for (uint64_t b = threadIdx.x; b < blockIdx.x; b += SCAN_THREADS) pre += bsum[b];
    TO ptot;
    (void)block_excl_scan<TO>(pre, ptot);
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    TO v[SCAN_ITEMS];
    load8<TI, TO>(in, base, n, v);
    TO s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) s += v[k];
    TO tot;
    TO run = block_excl_scan<TO>(s, tot) + ptot;
    TO o[SCAN_ITEMS];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        o[k] = run;
        run += v[k];
    }
    store8<TO>(out, base, n, o);
    if (n > 0 && base <= n - 1 && n - 1 < base + SCAN_ITEMS) out[n] = run;
}

// two arrays of the same length in the same two launches (blockIdx.y picks the array)
struct Pair32 { const uint32_t *in[2]; uint32_t *out[2]; uint32_t *bsum[2]; };

__global__ void __launch_bounds__(SCAN_THREADS) k_scan2_reduce(Pair32 P, uint64_t n) {
    const uint32_t *in = P.in[blockIdx.y];
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    load8<uint32_t, uint32_t>(in, base, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) s += v[k];
    uint32_t tot;
    (void)block_excl_scan<uint32_t>(s, tot);
    if (threadIdx.x == 0) P.bsum[blockIdx.y][blockIdx.x] = tot;
}

__global__ void __launch_bounds__(SCAN_THREADS) k_scan2_down(Pair32 P, uint64_t n) {
    const uint32_t *in = P.in[blockIdx.y];
    uint32_t *out = P.out[blockIdx.y];
    const uint32_t *bsum = P.bsum[blockIdx.y];
    uint32_t pre = 0;
    for (uint64_t b = threadIdx.x; b < blockIdx.x; b += SCAN_THREADS) pre += bsum[b];
    uint32_t ptot;
    (void)block_excl_scan<uint32_t>(pre, ptot);
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    load8<uint32_t, uint32_t>(in, base, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) s += v[k];
    uint32_t tot;
    uint32_t run = block_excl_scan<uint32_t>(s, tot) + ptot;
    uint32_t o[SCAN_ITEMS];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        o[k] = run;
        run += v[k];
    }
    store8<uint32_t>(out, base, n, o);
    if (n > 0 && base <= n - 1 && n - 1 < base + SCAN_ITEMS) out[n] = run;
}

// down-sweep from producer tile sums (WgScanBs): a tile of SCAN_TILE elements
// holds BS_PER_TILE producer blocks; its offset is the sum of the producer
// sums before it — summed by the block itself (bpre null) or read from their
// scanned form bpre (many tiles)
constexpr uint64_t BS_PER_TILE = SCAN_TILE / WG_BS_THREADS;
static_assert(SCAN_TILE % WG_BS_THREADS == 0, "producer blocks tile the scan tiles");
struct ScanBsArgs {
    const uint32_t *in[4];
    uint32_t *out[4];
    const uint32_t *bsum[4];
    const uint32_t *bpre[4];   // exclusive scan of bsum, or null
    uint64_t n[4];
};
__global__ void __launch_bounds__(SCAN_THREADS) k_scan_bs_down(ScanBsArgs P) {
    const int a = blockIdx.y;
    const uint32_t *in = P.in[a];
    uint32_t *out = P.out[a];
    const uint64_t n = P.n[a];
    if ((uint64_t)blockIdx.x * SCAN_TILE > n) return;   // (a shorter array: its tiles end earlier)
    const uint64_t b0 = (uint64_t)blockIdx.x * BS_PER_TILE;
    uint32_t ptot;
    if (P.bpre[a]) {
        ptot = P.bpre[a][b0];
    } else {
        uint32_t pre = 0;
        for (uint64_t b = threadIdx.x; b < b0; b += SCAN_THREADS) pre += P.bsum[a][b];
        (void)block_excl_scan<uint32_t>(pre, ptot);
    }
    const uint64_t base = (uint64_t)blockIdx.x * SCAN_TILE + (uint64_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    load8<uint32_t, uint32_t>(in, base, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) s += v[k];
    uint32_t tot;
    uint32_t run = block_excl_scan<uint32_t>(s, tot) + ptot;
    uint32_t o[SCAN_ITEMS];
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        o[k] = run;
        run += v[k];
    }
    store8<uint32_t>(out, base, n, o);
    if (n > 0 && base <= n - 1 && n - 1 < base + SCAN_ITEMS) out[n] = run;
    if (n == 0 && blockIdx.x == 0 && threadIdx.x == 0) out[0] = 0;
}

uint64_t nblocks(uint64_t n) { return n == 0 ? 1 : (n + SCAN_TILE - 1) / SCAN_TILE; }

template <class TO>
size_t tmp_bytes_rec(uint64_t n) {
    uint64_t nb = nblocks(n);
    if (nb <= 1) return 0;
    return (nb + 1) * sizeof(TO) + 256 + tmp_bytes_rec<TO>(nb);
}

template <class TI, class TO>
hipError_t scan_rec(const TI *in, TO *out, uint64_t n, char *tmp, hipStream_t s) {
    uint64_t nb = nblocks(n);
    if (nb <= 1) {
        hipLaunchKernelGGL((k_scan_down<TI, TO>), dim3(1), dim3(SCAN_THREADS), 0, s, in, out, (const TO *)nullptr, n);
        return hipGetLastError();
    }
    TO *bsum = reinterpret_cast<TO *>(tmp);
    char *next = tmp + (((nb + 1) * sizeof(TO) + 255) & ~size_t(255));
    hipLaunchKernelGGL((k_scan_reduce<TI, TO>), dim3(nb), dim3(SCAN_THREADS), 0, s, in, bsum, n);
    if (nb <= SCAN_TILE) {   // two launches: tile sums, then tiles with self-reduced offsets
        hipLaunchKernelGGL((k_scan_down2<TI, TO>), dim3(nb), dim3(SCAN_THREADS), 0, s, in, out, (const TO *)bsum, n);
        return hipGetLastError();
    }
    hipError_t e = scan_rec<TO, TO>(bsum, bsum, nb, next, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_scan_down<TI, TO>), dim3(nb), dim3(SCAN_THREADS), 0, s, in, out, (const TO *)bsum, n);
    return hipGetLastError();
}

}  // namespace

size_t wg_scan_tmp_bytes(uint64_t n) {
    // + wg_scan_bs_u32's scanned producer sums (four arrays) and their recursion
    const uint64_t nbs = wg_bs_blocks(n);
    return tmp_bytes_rec<uint64_t>(n) + 4 * (((nbs + 1) * 4 + 255) & ~size_t(255)) + tmp_bytes_rec<uint64_t>(nbs) + 1024;
}

hipError_t wg_exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, void *tmp, hipStream_t s) {
    return scan_rec<uint32_t, uint32_t>(in, out, n, (char *)tmp, s);
}
hipError_t wg_exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, void *tmp, hipStream_t s) {
    return scan_rec<uint64_t, uint64_t>(in, out, n, (char *)tmp, s);
}

hipError_t wg_exclusive_scan2_u32(const uint32_t *in0, uint32_t *out0, const uint32_t *in1, uint32_t *out1, uint64_t n,
                                  void *tmp, hipStream_t s) {
    const uint64_t nb = nblocks(n);
    if (nb <= 1 || nb > SCAN_TILE) {   // one tile, or more tiles than one block reduces: one scan at a time
        hipError_t e = scan_rec<uint32_t, uint32_t>(in0, out0, n, (char *)tmp, s);
        return e != hipSuccess ? e : scan_rec<uint32_t, uint32_t>(in1, out1, n, (char *)tmp, s);
    }
    Pair32 P;
    P.in[0] = in0; P.in[1] = in1; P.out[0] = out0; P.out[1] = out1;
    P.bsum[0] = reinterpret_cast<uint32_t *>(tmp);
    P.bsum[1] = P.bsum[0] + ((nb + 63) & ~63ull);   // wg_scan_tmp_bytes holds (nb + 1) u64 >= 2 * (nb + 64) u32
    hipLaunchKernelGGL(k_scan2_reduce, dim3((uint32_t)nb, 2), dim3(SCAN_THREADS), 0, s, P, n);
    hipLaunchKernelGGL(k_scan2_down, dim3((uint32_t)nb, 2), dim3(SCAN_THREADS), 0, s, P, n);
    return hipGetLastError();
}

hipError_t wg_scan_bs_u32(const WgScanBs &S, uint64_t n, void *tmp, hipStream_t s) {
    if (S.na < 1 || S.na > 4) return hipErrorInvalidValue;
    ScanBsArgs P{};
    char *t = (char *)tmp;
    for (int a = 0; a < S.na; a++) {
        P.in[a] = S.in[a];
        P.out[a] = S.out[a];
        P.bsum[a] = S.bsum[a];
        P.bpre[a] = nullptr;
        P.n[a] = S.len[a] ? S.len[a] : n;
        const uint64_t nbs = wg_bs_blocks(P.n[a]);
        if (nbs > WG_BS_SELF) {   // many tiles: scan the producer sums first (one array of the tmp at a time)
            uint32_t *pre = reinterpret_cast<uint32_t *>(t);
            t += ((nbs + 1) * 4 + 255) & ~size_t(255);
            hipError_t e = scan_rec<uint32_t, uint32_t>(S.bsum[a], pre, nbs, t, s);
            if (e != hipSuccess) return e;
            P.bpre[a] = pre;
        }
    }
    if ((size_t)(t - (char *)tmp) + tmp_bytes_rec<uint64_t>(wg_bs_blocks(n)) > wg_scan_tmp_bytes(n))
        return hipErrorInvalidValue;   // (cannot happen: 4 (n/256 + 65) u32 + the recursion fit the reserve)
    hipLaunchKernelGGL(k_scan_bs_down, dim3((uint32_t)nblocks(n), (uint32_t)S.na), dim3(SCAN_THREADS), 0, s, P);
    return hipGetLastError();
}

hipError_t wg_tile_sums2_u32(const uint32_t *in0, const uint32_t *in1, uint64_t n, uint32_t *ts0, uint32_t *ts1,
                             hipStream_t s) {
    Pair32 P;
    P.in[0] = in0; P.in[1] = in1; P.out[0] = nullptr; P.out[1] = nullptr;
    P.bsum[0] = ts0; P.bsum[1] = ts1;
    hipLaunchKernelGGL(k_scan2_reduce, dim3((uint32_t)nblocks(n), 2), dim3(SCAN_THREADS), 0, s, P, n);
    return hipGetLastError();
}

int wg_scan_reserve(wg_ctx *c, uint64_t n) {
    WG_ALLOC(c, c->scan_tmp, wg_scan_tmp_bytes(n));
    return WG_OK;
}
