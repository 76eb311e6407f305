// wg_api.hip — C ABI entry points (include/wgraph.h) and stage orchestration.
//
// Each exported function names the GraphLayout item it replaces
// (/root/reference/src/commit_graph.rs).  No C++ exception crosses the ABI;
// every failure returns a negative status with a message in wg_last_error().
#include <atomic>
#include <chrono>
#include <thread>
#include <cstdarg>
#include <cstring>
#include <new>

#include "wg_internal.h"

int wg_fail(wg_ctx *c, int code, const char *fmt, ...) {
    if (c) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof(buf), fmt, ap);
        va_end(ap);
        c->err = buf;
    }
    return code;
}

// Stage timing events: a device-scope release (the default system-scope
// fence writes back and invalidates the caches between the kernels they
// bracket: ~10 us before and after the emission kernel in a timed step).
// WG_EVENT_SCOPE=system (diagnostic): HIP's default fence for these events
// and the side stream's, for same-box comparisons.
static bool wg_system_events() {
    static const bool sys = [] { const char *v = std::getenv("WG_EVENT_SCOPE"); return v && !std::strcmp(v, "system"); }();
    return sys;
}
unsigned wg_event_scope() { return wg_system_events() ? 0u : hipEventReleaseToDevice; }
static hipError_t wg_timing_event(hipEvent_t *e) {
    return hipEventCreateWithFlags(e, wg_system_events() ? hipEventDefault : hipEventReleaseToDevice);
}

// Stages nest: begin takes the next slot and pushes it, end closes the top.
void wg_stage_begin(wg_ctx *c, const char *name) {
    if (!c->timing) return;
    if (c->n_stages >= WG_STAGE_MAX || c->stage_depth >= 8 ||
        (c->timing_emit_only && std::strcmp(name, "vtx_emit") != 0)) {
        c->stage_stack[c->stage_depth++ & 7] = -1;
        return;
    }
    StageTimer &t = c->stages[c->n_stages];
    if (!t.a) { (void)wg_timing_event(&t.a); (void)wg_timing_event(&t.b); }
    t.name = name;
    (void)hipEventRecord(t.a, c->stream);
    c->stage_stack[c->stage_depth++] = c->n_stages++;
}
void wg_stage_end(wg_ctx *c) {
    if (!c->timing || c->stage_depth <= 0) return;
    const int idx = c->stage_stack[--c->stage_depth];
    if (idx >= 0) (void)hipEventRecord(c->stages[idx].b, c->stream);
}

namespace {
constexpr int FETCH_MAX = 64;
struct FetchArgs { const void *p[FETCH_MAX]; unsigned long long wide; uint32_t n; };
// the words, then (system-scope release) the launch's sequence number: the
// host sees the words once it sees the number, without a runtime wait
__global__ void k_fetch(FetchArgs a, unsigned long long *out, unsigned long long *seq_word, unsigned long long seq) {
    const uint32_t i = threadIdx.x;
    if (i < a.n) out[i] = ((a.wide >> i) & 1ull) ? *reinterpret_cast<const unsigned long long *>(a.p[i])
                                                 : (unsigned long long)*reinterpret_cast<const uint32_t *>(a.p[i]);
    __threadfence_system();
    __syncthreads();
    if (i == 0) __hip_atomic_store(seq_word, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// one piece per blockIdx.y; 16-byte moves when the piece allows them
__global__ void __launch_bounds__(256) k_copy_batch(WgCopyBatch B) {
    const uint32_t k = blockIdx.y;
    if (k == 0 && blockIdx.x == 0 && threadIdx.x < B.nwords) B.wdst[threadIdx.x] = B.words[threadIdx.x];
    if (k >= B.n) return;
    const uint8_t *src = static_cast<const uint8_t *>(B.src[k]);
    uint8_t *dst = static_cast<uint8_t *>(B.dst[k]);
    const uint64_t nb = B.bytes[k];
    const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, ts = (uint64_t)gridDim.x * blockDim.x;
    if (((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | nb) & 15u) == 0) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst);
        for (uint64_t i = t0; i < nb / 16; i += ts) d4[i] = s4[i];
    } else {
        const uint32_t *s1 = reinterpret_cast<const uint32_t *>(src);
        uint32_t *d1 = reinterpret_cast<uint32_t *>(dst);
        for (uint64_t i = t0; i < nb / 4; i += ts) d1[i] = s1[i];
    }
}
}  // namespace

int wg_copy_batch(wg_ctx *c, const WgCopies &cp, hipStream_t s) {
    if (cp.overflow) return wg_fail(c, WG_E_UNSUPPORTED, "copy batch overflow (more than %d pieces)", WG_BCOPY_MAX);
    const WgCopyBatch &B = cp.b;
    if (B.n == 0 && B.nwords == 0) return WG_OK;
    uint64_t mx = 0;
    for (uint32_t k = 0; k < B.n; k++) {
        if (((reinterpret_cast<uintptr_t>(B.src[k]) | reinterpret_cast<uintptr_t>(B.dst[k]) | B.bytes[k]) & 3u) != 0)
            return wg_fail(c, WG_E_INVALID, "copy batch piece %u not 4-byte aligned", k);
        mx = B.bytes[k] > mx ? B.bytes[k] : mx;
    }
    uint64_t gx = (mx + 4095) / 4096;
    gx = gx < 1 ? 1 : (gx > 512 ? 512 : gx);
    hipLaunchKernelGGL(k_copy_batch, dim3((uint32_t)gx, B.n ? B.n : 1u), dim3(256), 0, s, B);
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

int wg_side_fork(wg_ctx *c) {
    if (!c->side) {
        // (normal priority: at the highest, the hash table's kernels starved
        // the near probe beside them, 58 -> 81 us, r04f/r04g traces)
        WG_HIP(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
        // stream-to-stream order on one device: a device-scope release suffices
        WG_HIP(c, hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming | wg_event_scope()));
        WG_HIP(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming | wg_event_scope()));
        WG_HIP(c, hipEventCreateWithFlags(&c->ev_slice, hipEventDisableTiming | wg_event_scope()));
    }
    if (const int rc = wg_side_join(c)) return rc;
    WG_HIP(c, hipEventRecord(c->ev_fork, c->stream));
    WG_HIP(c, hipStreamWaitEvent(c->side, c->ev_fork, 0));
    c->side_main = c->stream;
    c->stream = c->side;
    return WG_OK;
}

void wg_side_done(wg_ctx *c) {
    if (c->stream != c->side || !c->side_main) return;
    const hipError_t e = hipEventRecord(c->ev_join, c->side);
    c->stream = c->side_main;
    c->side_main = nullptr;
    if (e == hipSuccess) c->side_pending = true;
    else (void)hipStreamSynchronize(c->side);   // no event: order by waiting
}

int wg_side_join(wg_ctx *c) {
    if (!c->side_pending) return WG_OK;
    c->side_pending = false;
    // already reached (the host ran behind the device, e.g. the next build
    // after an emission whose side read it waited for): no wait packet on
    // the main queue — a cross-queue wait costs ~10 us even when satisfied
    const hipError_t q = hipEventQuery(c->ev_join);
    if (q == hipSuccess) return WG_OK;
    if (q == hipErrorNotReady) (void)hipGetLastError();   // (a status, not a failure: not left as the last error)
    WG_HIP(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
    return WG_OK;
}

int wg_side_zero_rowtop(wg_ctx *c, uint64_t m, float *h, float *rt, uint64_t row_lo, const float *band,
                        const float *band_host, float *band_dev) {
    int rc = wg_side_fork(c);
    if (rc != WG_OK) return rc;
    if (band_host && m) {   // (build_frame's host band, copied on this stream)
        const hipError_t e = hipMemcpyAsync(band_dev, band_host, m * 4, hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) rc = wg_fail(c, WG_E_HIP, "band copy: %s", hipGetErrorString(e));
    }
    if (rc == WG_OK) rc = wg_heights_run(c, m, c->n_list, h);
    if (rc == WG_OK) rc = wg_rowtop_run(c, m, h, band, rt, row_lo);
    wg_side_done(c);
    return rc;
}

int wg_side_build_begin(wg_ctx *c, uint64_t m, float *h, float *rt, const float *band, const float *band_host,
                        float *band_dev) {
    int rc = wg_side_fork(c);
    if (rc != WG_OK) return rc;
    if (!c->ev_hash) {
        const hipError_t e = hipEventCreateWithFlags(&c->ev_hash, hipEventDisableTiming | wg_event_scope());
        if (e != hipSuccess) rc = wg_fail(c, WG_E_HIP, "event: %s", hipGetErrorString(e));
    }
    // (the fused join builds its table on the main stream, wg_stage_hash_join)
    if (rc == WG_OK && !c->join_fused) rc = wg_hash_table_launch(c);
    if (rc == WG_OK && !c->join_fused) {
        const hipError_t e = hipEventRecord(c->ev_hash, c->stream);
        if (e != hipSuccess) rc = wg_fail(c, WG_E_HIP, "event: %s", hipGetErrorString(e));
        c->hash_on_side = true;
    }
    if (rc == WG_OK && band_host && m) {   // (build_frame's host band, copied on this stream)
        const hipError_t e = hipMemcpyAsync(band_dev, band_host, m * 4, hipMemcpyHostToDevice, c->stream);
        if (e != hipSuccess) rc = wg_fail(c, WG_E_HIP, "band copy: %s", hipGetErrorString(e));
    }
    if (rc == WG_OK) rc = wg_heights_run(c, m, c->n_list, h);
    if (rc == WG_OK) rc = wg_rowtop_run(c, m, h, band, rt, 0);
    if (rc == WG_OK) rc = wg_geom_prezero(c, m);   // (the build's geometry pass joins this stream first)
    // r06: the next build's table (left to this list's emission by the place
    // pass, hash_table_prepare's `later`), emptied here instead, beside the
    // lane stage's latency-bound kernels — the emission saturates HBM and a
    // clear queued there ran beside the next build's geometry kernels
    if (rc == WG_OK && c->hash_on_side) rc = wg_hash_clear_next(c, c->stream);
    wg_side_done(c);
    if (rc != WG_OK) c->hash_built = c->hash_on_side = false;
    return rc;
}

int wg_fetch(wg_ctx *c, std::initializer_list<WgFetch> items, uint64_t *out) {
    return wg_fetch_n(c, (int)items.size(), items.begin(), out);
}

// mapped pinned words: [0, FETCH_MAX) for wg_fetch, [FETCH_MAX, 2 FETCH_MAX) for wg_fetch_begin,
// [2 FETCH_MAX, 3 FETCH_MAX) for wg_fetch_defer
static int fetch_launch(wg_ctx *c, int n, const WgFetch *items, uint64_t slot0) {
    if (n < 0 || n > FETCH_MAX) return wg_fail(c, WG_E_INVALID, "wg_fetch: too many items");
    if (!c->h_fetch) {
        WG_HIP(c, hipHostMalloc((void **)&c->h_fetch, (3 * FETCH_MAX + 8) * sizeof(uint64_t),
                                hipHostMallocMapped | hipHostMallocCoherent));
        WG_HIP(c, hipHostGetDevicePointer((void **)&c->d_fetch, c->h_fetch, 0));
        memset(c->h_fetch, 0, (3 * FETCH_MAX + 8) * sizeof(uint64_t));
    }
    FetchArgs a{};
    a.n = 0;
    for (int i = 0; i < n; i++) {
        a.p[a.n] = items[i].p;
        if (items[i].wide) a.wide |= 1ull << a.n;
        a.n++;
    }
    const int region = (int)(slot0 / FETCH_MAX);
    c->fetch_want[region] = ++c->fetch_seq;
    hipLaunchKernelGGL(k_fetch, dim3(1), dim3(64), 0, c->stream, a, (unsigned long long *)c->d_fetch + slot0,
                       (unsigned long long *)c->d_fetch + 3 * FETCH_MAX + region, (unsigned long long)c->fetch_seq);
    WG_HIP(c, hipGetLastError());
    return WG_OK;
}

static inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#elif defined(__aarch64__)
    asm volatile("yield");
#endif
}

// Wait for the region's sequence word (k_fetch stores it last, system-scope
// release): a few us after k_fetch ends, where a runtime wait costs tens of
// us of wake-up and bookkeeping.  Busy for the first 50 us only (a read
// queued behind a slow collective would otherwise hold a core), then
// polling with a yield between reads; false after 5 ms: the caller takes
// the runtime wait, which also reports a failed launch.
static bool fetch_spin(wg_ctx *c, int region) {
    volatile uint64_t *w = (volatile uint64_t *)c->h_fetch + 3 * FETCH_MAX + region;
    const uint64_t want = c->fetch_want[region];
    const auto t0 = std::chrono::steady_clock::now();
    bool busy = true;
    for (uint32_t i = 1;; i++) {
        if (*w == want) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return true;
        }
        if (busy) {
            cpu_relax();
            if ((i & 255u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(50)) busy = false;
        } else {
            std::this_thread::yield();
            if ((i & 15u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(5)) return false;
        }
    }
}

int wg_fetch_n(wg_ctx *c, int n, const WgFetch *items, uint64_t *out) {
    if (const int rc = fetch_launch(c, n, items, 0)) return rc;
    if (!fetch_spin(c, 0)) WG_HIP(c, hipStreamSynchronize(c->stream));
    for (int i = 0; i < n; i++) out[i] = ((volatile uint64_t *)c->h_fetch)[i];
    return WG_OK;
}

int wg_fetch_begin(wg_ctx *c, std::initializer_list<WgFetch> items) {
    return wg_fetch_begin_n(c, (int)items.size(), items.begin());
}

int wg_fetch_begin_n(wg_ctx *c, int n, const WgFetch *items) {
    if (c->fetch_pending) {   // left behind by a failed call: drop it
        (void)(c->fetch_fused ? hipStreamSynchronize(c->stream) : hipEventSynchronize(c->ev_fetch));
        c->fetch_pending = 0;
        c->fetch_fused = false;
    }
    if (const int rc = fetch_launch(c, n, items, FETCH_MAX)) return rc;
    // (a device-scope release: the words reach the host by k_fetch's own
    // system-scope stores; the event only backs the host's fallback wait)
    if (!c->ev_fetch) WG_HIP(c, hipEventCreateWithFlags(&c->ev_fetch, hipEventDisableTiming | wg_event_scope()));
    WG_HIP(c, hipEventRecord(c->ev_fetch, c->stream));
    c->fetch_pending = n;
    return WG_OK;
}

// ---------------------------------------------------------------------------
// Deferred validation of a speculative build (WG_OPT_DEFER_VALIDATION)
// ---------------------------------------------------------------------------
int wg_settle(wg_ctx *c) {
    if (const int rc = wg_geom_lists_flush(c)) return rc;   // (the words below include the lists' flags)
    if (!c->pend.build) return WG_OK;
    uint64_t v[WG_PENDING_ITEMS] = {0};
    if (const int rc = wg_fetch_n(c, c->pend.k, c->pend.it, v)) return rc;
    bool redone = false;
    return wg_validate_pending(c, v, &redone);
}

// The end-of-build check of wg_layout_build on words v (WG_PENDING_ITEMS);
// what did not hold is redone by the exact stages.  After a deferred build:
// the frame pass and the emission queued since are redone as well.
static int build_check(wg_ctx *c, const uint64_t *v, int kl, int k, bool *redo) {
    const uint64_t ne = v[k - 1];
    const bool lanes_ok = wg_lanes_spec_check(c, v);
    int rc;
    if (!lanes_ok) {   // the exact lane stage (fast path with its reads, or the general walk)
        if ((rc = wg_stage_lanes(c, false)) != WG_OK) return rc;
        if ((rc = wg_stage_edges(c, false, (int64_t)ne)) != WG_OK) return rc;
        c->layout_gen++;
        c->alt_heights_on = false;   // (a new built list: its own heights)
    } else {
        c->n_edges = ne;
        const uint32_t vis = c->max_lane + 1 < (uint32_t)WG_LANE_COUNT_VISUAL ? c->max_lane + 1 : (uint32_t)WG_LANE_COUNT_VISUAL;
        const float gw = (float)vis * WG_LANE_W;   // graph_width (:353-354)
        c->graph_width = gw > WG_LANE_W ? gw : WG_LANE_W;
    }
    c->spec_builds++;
    c->spec_redo_lanes += !lanes_ok;
    *redo = !lanes_ok || !wg_geom_spec_check(c, v + kl);
    if (*redo) {
        c->spec_redo_geom++;
        c->lists_gen = ~0ull;
        c->spec = false;
        // (the row_top again with the build's bands: a frame pass queued since
        // may have rescanned it with its own)
        const float *bb = c->build_banded ? c->band_prev.as<const float>() : nullptr;
        if ((rc = wg_stage_rowtop(c, bb)) != WG_OK) return rc;
        if ((rc = wg_stage_geometry(c, bb)) != WG_OK) return rc;
    }
    c->spec_ready = c->lists_gen == c->layout_gen;   // an exact or validated build: the buffers are sized
    c->have_geom = true;
    c->geom_key_gen = c->layout_gen;   // the geometry of (this layout, the build's bands)
    c->geom_key_band = c->build_banded;
    return WG_OK;
}

static int row_geometry_impl(wg_ctx *c, const float *band, int32_t residency);

int wg_validate_pending(wg_ctx *c, const uint64_t *v, bool *redone) {
    *redone = false;
    if (!c->pend.build) return WG_OK;
    const PendingBuild P = c->pend;
    c->pend = PendingBuild{};
    bool redo = false;
    int rc = P.shard ? wg_shard_geom_validate(c, v, &redo) : build_check(c, v, P.kl, P.k, &redo);
    if (rc != WG_OK || !redo) return rc;
    *redone = true;
    if (P.frame && (rc = row_geometry_impl(c, P.frame_band ? c->band_prev.as<const float>() : nullptr, WG_DEVICE)) != WG_OK)
        return rc;
    if (P.emit) {
        const ShardState &S = c->sh;
        const int64_t sel_l = (P.sel >= 0 && (uint64_t)P.sel >= S.s && (uint64_t)P.sel < S.e)
                                  ? (int64_t)((uint64_t)P.sel - S.s + S.row_base) : -1;
        if ((rc = wg_stage_vertices(c, P.rb - S.s + S.row_base, P.re - S.s + S.row_base, sel_l)) != WG_OK) return rc;
        c->have_vtx = true;
    }
    return WG_OK;
}

// Deferred read: the words are copied in stream order now and read by the
// host later (wg_fetch_deferred), typically after a synchronisation the
// stage needed anyway — a value the host needs only later costs no stall.
int wg_fetch_defer(wg_ctx *c, std::initializer_list<WgFetch> items) {
    if (const int rc = fetch_launch(c, (int)items.size(), items.begin(), 2 * FETCH_MAX)) return rc;
    if (!c->ev_defer) WG_HIP(c, hipEventCreateWithFlags(&c->ev_defer, hipEventDisableTiming | wg_event_scope()));
    WG_HIP(c, hipEventRecord(c->ev_defer, c->stream));
    c->defer_pending = (int)items.size();
    return WG_OK;
}

int wg_fetch_deferred(wg_ctx *c, uint64_t *out) {
    if (!c->defer_pending) return wg_fail(c, WG_E_STATE, "wg_fetch_deferred: nothing deferred");
    const int n = c->defer_pending;
    c->defer_pending = 0;
    if (!fetch_spin(c, 2)) WG_HIP(c, hipEventSynchronize(c->ev_defer));
    for (int i = 0; i < n; i++) out[i] = ((volatile uint64_t *)c->h_fetch)[2 * FETCH_MAX + i];
    return WG_OK;
}

int wg_fetch_fused_begin(wg_ctx *c, int n, const WgFetch *items, WgFusedFetch *f) {
    static_assert(WG_FETCH_MAX == FETCH_MAX, "fused fetch region size");
    if (n < 0 || n > FETCH_MAX) return wg_fail(c, WG_E_INVALID, "wg_fetch: too many items");
    if (c->fetch_pending) {   // left behind by a failed call: drop it
        (void)hipStreamSynchronize(c->stream);
        c->fetch_pending = 0;
    }
    if (!c->h_fetch) {
        WG_HIP(c, hipHostMalloc((void **)&c->h_fetch, (3 * FETCH_MAX + 8) * sizeof(uint64_t),
                                hipHostMallocMapped | hipHostMallocCoherent));
        WG_HIP(c, hipHostGetDevicePointer((void **)&c->d_fetch, c->h_fetch, 0));
        memset(c->h_fetch, 0, (3 * FETCH_MAX + 8) * sizeof(uint64_t));
    }
    *f = WgFusedFetch{};
    for (int i = 0; i < n; i++) {
        f->p[i] = items[i].p;
        if (items[i].wide) f->wide |= 1ull << i;
    }
    f->n = (uint32_t)n;
    f->out = (unsigned long long *)c->d_fetch + FETCH_MAX;
    f->seq_word = (unsigned long long *)c->d_fetch + 3 * FETCH_MAX + 1;
    f->seq = c->fetch_want[1] = ++c->fetch_seq;
    c->fetch_pending = n;
    c->fetch_fused = true;
    return WG_OK;
}

int wg_fetch_end(wg_ctx *c, uint64_t *out) {
    if (!c->fetch_pending) return wg_fail(c, WG_E_STATE, "wg_fetch_end: nothing pending");
    const int n = c->fetch_pending;
    c->fetch_pending = 0;
    const bool fused = c->fetch_fused;
    c->fetch_fused = false;
    if (!fetch_spin(c, 1)) WG_HIP(c, fused ? hipStreamSynchronize(c->stream) : hipEventSynchronize(c->ev_fetch));
    for (int i = 0; i < n; i++) out[i] = ((volatile uint64_t *)c->h_fetch)[FETCH_MAX + i];
    return WG_OK;
}

extern "C" {

int wg_abi_version(void) { return WGRAPH_ABI_VERSION; }

wg_ctx *wg_create(int device_ordinal) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return nullptr;
    int dev = device_ordinal;
    if (dev < 0 && hipGetDevice(&dev) != hipSuccess) return nullptr;
    if (dev >= ndev || hipSetDevice(dev) != hipSuccess) return nullptr;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return nullptr;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return nullptr;   // CDNA4 only
    wg_ctx *c = new (std::nothrow) wg_ctx();
    if (!c) return nullptr;
    c->device = dev;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { delete c; return nullptr; }
    c->own_stream = true;
    wg_init_height_thresholds(c->h_thresh);
    return c;
}

void wg_destroy(wg_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->side_main) c->stream = c->side_main;
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->side) (void)hipStreamSynchronize(c->side);
    DevBuf *bufs[] = {&c->in_oid, &c->in_time, &c->in_poff, &c->in_poid, &c->in_flags, &c->hash, &c->canon,
                      &c->prow, &c->lane_asg, &c->lane_out, &c->color_out, &c->lane_scalars, &c->edge_cnt,
                      &c->edges, &c->heights, &c->band, &c->g_height, &c->g_node_y, &c->g_row_top,
                      &c->rt_chunk, &c->rt_tables, &c->rt_sup, &c->rt_flags, &c->geom_zero,
                      &c->vert_off, &c->curve_off, &c->vert, &c->curve, &c->curve_color,
                      &c->curve_ref, &c->curve_row, &c->carry_off, &c->carry,
                      &c->scan_tmp, &c->scal, &c->rowflags, &c->rowflags_lists, &c->geom_diff, &c->scurve_off,
                      &c->scurve_ref, &c->scurve_row, &c->sweep_big, &c->vtx_off, &c->vtx, &c->palette, &c->chk,
                      &c->carry_sorted, &c->curve_tb, &c->curve_cnt, &c->tile_first, &c->hs_time, &c->hs_out, &c->htab[0], &c->htab[1], &c->bsum};
    for (DevBuf *b : bufs) b->release();
    for (DevBuf &b : c->lf) b.release();
    ShardState &S = c->sh;
    DevBuf *sb[] = {&S.msg, &S.ptable, &S.prow, &S.unres, &S.flags, &S.xcnt, &S.refx, &S.isfb, &S.xsec, &S.xall,
                    &S.xtok, &S.xt, &S.dev_small, &S.h_g, &S.rt_g, &S.band_host, &S.xchild, &S.xpar, &S.in_scan,
                    &S.edge_y, &S.own_edges};
    for (DevBuf *b : sb) b->release();
    DevBuf *tb[] = {&c->text_sum, &c->text_sum_off, &c->text_off, &c->text_rec, &c->text_vtx};
    for (DevBuf *b : tb) b->release();
    for (FontSlot &f : c->fonts) {
        DevBuf *fb[] = {&f.edges, &f.gdesc, &f.cov, &f.sdf, &f.gin, &f.gout, &f.d2in, &f.d2out, &f.gtab};
        for (DevBuf *b : fb) b->release();
    }
    c->tile_first.release();
    DevBuf *xb[] = {&c->band_prev, &c->geom_diff_first, &c->render_small, &c->render_img, &c->match_flags,
                    &c->match_q, &c->match_flat};
    for (DevBuf *b : xb) b->release();
    for (int f = 0; f < 2; f++) { c->match_txt[f].release(); c->match_off[f].release(); }
    for (DevBuf &b : c->ord) b.release();
    for (FontSlot &f : c->fonts) {
        DevBuf *fb[] = {&f.edges, &f.gdesc, &f.cov, &f.sdf, &f.gin, &f.gout, &f.d2in, &f.d2out, &f.gtab};
        for (DevBuf *b : fb) b->release();
    }
    for (int i = 0; i < WG_STAGE_MAX; i++) {
        if (c->stages[i].a) (void)hipEventDestroy(c->stages[i].a);
        if (c->stages[i].b) (void)hipEventDestroy(c->stages[i].b);
    }
    if (c->h_fetch) (void)hipHostFree(c->h_fetch);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
    if (c->ev_join) (void)hipEventDestroy(c->ev_join);
    if (c->ev_hash) (void)hipEventDestroy(c->ev_hash);
    if (c->ev_slice) (void)hipEventDestroy(c->ev_slice);
    if (c->ev_fetch) (void)hipEventDestroy(c->ev_fetch);
    if (c->ev_defer) (void)hipEventDestroy(c->ev_defer);
    delete c;
}

const char *wg_last_error(const wg_ctx *c) { return c ? c->err.c_str() : "null context"; }

int wg_set_stream(wg_ctx *c, void *s) {
    if (!c) return WG_E_INVALID;
    WG_SETTLE(c);
    (void)hipSetDevice(c->device);
    if (c->own_stream && c->stream) {
        WG_HIP(c, hipStreamSynchronize(c->stream));
        WG_HIP(c, hipStreamDestroy(c->stream));
    }
    if (s) { c->stream = (hipStream_t)s; c->own_stream = false; }
    else {
        WG_HIP(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
    }
    return WG_OK;
}

int wg_vertex_placement_get(wg_ctx *c, uint32_t *n_probed, uint32_t *kept, float *probe_ms) {
    if (!c) return WG_E_INVALID;
    if (n_probed) *n_probed = c->vtx_place_n;
    if (kept) *kept = c->vtx_place_pick;
    if (probe_ms) for (int k = 0; k < 8; k++) probe_ms[k] = c->vtx_place_ms[k];
    return WG_OK;
}

int wg_set_option(wg_ctx *c, int option, int64_t value) {
    if (!c) return WG_E_INVALID;
    switch (option) {
    case WG_OPT_LANE_PATH: c->force_general_lanes = value != 0; return WG_OK;
    case WG_OPT_REPLAY_CHUNK:
        if (value < 64 || value > (1 << 20) || (value & 63)) return wg_fail(c, WG_E_INVALID, "replay chunk must be a multiple of 64");
        c->replay_chunk = (uint32_t)value;
        c->replay_auto = false;
        return WG_OK;
    case WG_OPT_TIMING_EMIT_ONLY: c->timing_emit_only = value != 0; return WG_OK;
    case WG_OPT_REPLAY_WARMUP:
        if (value < 0 || value > 3584 || (value & 63)) return wg_fail(c, WG_E_INVALID, "replay warm-up must be a multiple of 64 in 0..3584");
        c->replay_warm = (uint32_t)value;
        c->replay_auto = false;
        return WG_OK;
    case WG_OPT_DEFER_VALIDATION:
        WG_SETTLE(c);
        c->defer_validation = value != 0;
        return WG_OK;
    case WG_OPT_SHARD_SPEC_REPLAY:
        c->spec_replay_shard = value != 0;
        return WG_OK;
    case WG_OPT_REPLAY_MODE:
        if (value < 0 || value > 3)
            return wg_fail(c, WG_E_INVALID, "replay mode must be 0 (auto), 1 (chunked), 2 (serial) or 3 (compacted)");
        c->replay_mode = (uint32_t)value;
        return WG_OK;
    case WG_OPT_SLICE_LISTS:
        if (value < 0 || value > 2) return wg_fail(c, WG_E_INVALID, "slice lists must be 0, 1 or 2");
        WG_SETTLE(c);
        c->slice_on = value != 0;
        c->slice_min_rows = value == 2 ? 4 * WG_SWEEP_CH : 1ull << 18;
        return WG_OK;
    case WG_OPT_MATCH_THREADS:
        if (value != 0 && value != 256 && value != 512 && value != 513)   // (513: 512 threads at 6 waves per SIMD, for A/B)
            return wg_fail(c, WG_E_INVALID, "match threads %lld", (long long)value);
        c->match_threads = value ? (uint32_t)value : 512u;
        return WG_OK;
    case WG_OPT_FUSED_READ:
        WG_SETTLE(c);
        c->fused_read = value != 0;
        return WG_OK;
    case WG_OPT_VTX_TILE:
        if (value != 0 && value != 1024 && value != 2048 && value != 4096)
            return wg_fail(c, WG_E_INVALID, "vertex tile must be 0, 1024, 2048 or 4096");
        c->vtx_tile_opt = (uint32_t)value;
        return WG_OK;
    case WG_OPT_JOIN_FUSED:
        c->join_fused = value != 0;
        return WG_OK;
    case WG_OPT_DC_WARMUP:
        if (value < 0 || value > (1 << 20) || (value & 63)) return wg_fail(c, WG_E_INVALID, "warm-up must be a multiple of 64 in 0..2^20");
        c->dc_warm_fixed = (uint32_t)value;
        c->dc_warm = value ? (uint32_t)value : wg_ctx::WG_DC_WARM0;
        return WG_OK;
    case WG_OPT_SWEEP_REG:
        if (value < 0 || value > 512) return wg_fail(c, WG_E_INVALID, "sweep register capacity must be 0..512");
        c->sweep_reg_cap = (uint32_t)value;
        return WG_OK;
    case WG_OPT_VTX_PLACE:
        if (value < 0 || value > 8) return wg_fail(c, WG_E_INVALID, "vertex placement candidates must be 0..8");
        WG_SETTLE(c);
        WG_HIP(c, hipStreamSynchronize(c->stream));
        c->vtx.release();   // placed afresh by the next emission
        c->have_vtx = false;
        c->vtx_place = value ? (uint32_t)value : 1u;   // (0: one allocation, as 1)
        return WG_OK;
    default: return wg_fail(c, WG_E_INVALID, "unknown option %d", option);
    }
}

int wg_synchronize(wg_ctx *c) {
    if (!c) return WG_E_INVALID;
    WG_SETTLE(c);
    if (wg_side_join(c) != WG_OK) return WG_E_HIP;
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

// ---------------------------------------------------------------------------
// GraphLayout::build (:265-355)
// ---------------------------------------------------------------------------
static int layout_build_impl(wg_ctx *c, const wg_commits *in, const float *fband, int32_t fres);

int wg_layout_build(wg_ctx *c, const wg_commits *in) {
    if (c) WG_SETTLE(c);
    if (!c || !in) return WG_E_INVALID;
    return layout_build_impl(c, in, nullptr, WG_DEVICE);
}

// GraphLayout::build followed by row_geometry_with_bands(band) (history_view's
// first frame after a refresh, commit_graph.rs:1419-1421).  build's own
// row_geometry (:322-346) is replaced by the frame's before anyone can read
// it, so the build's geometry pass takes the bands itself: the banded row_top
// on the side stream beside the hash join and lanes, and no second pass.
int wg_layout_build_frame(wg_ctx *c, const wg_commits *in, const float *band, int32_t residency) {
    if (c) WG_SETTLE(c);
    if (!c || !in || !band) return WG_E_INVALID;
    if (residency != WG_HOST && residency != WG_DEVICE) return wg_fail(c, WG_E_INVALID, "bad residency %d", residency);
    const int rc = layout_build_impl(c, in, band, residency);
    if (rc != WG_OK || c->build_banded) return rc;
    return row_geometry_impl(c, band, residency);   // (an empty list)
}

static int layout_build_impl(wg_ctx *c, const wg_commits *in, const float *fband, int32_t fres) {
    (void)hipSetDevice(c->device);
    c->have_layout = c->have_geom = c->have_vtx = c->have_text = false;
    c->lists_gen = ~0ull;
    c->sh.on = false;
    c->match_on = false;   // match flags belong to the previous commit list
    c->sh.step = 0;
    c->edge_y = nullptr;
    const uint64_t n = in->n_commits;
    if (n >= 0xFFFFFFF0ull) return wg_fail(c, WG_E_UNSUPPORTED, "n_commits %llu exceeds 2^32-16", (unsigned long long)n);
    if (n > 0 && (!in->oid || !in->time || !in->parent_off)) return wg_fail(c, WG_E_INVALID, "null input array");
    uint64_t e = 0;
    if (n > 0) {
        if (in->residency == WG_HOST) e = in->parent_off[n];
        else e = in->n_parents;
        if (e != in->n_parents) return wg_fail(c, WG_E_INVALID, "n_parents %llu != parent_off[N] %llu",
                                               (unsigned long long)in->n_parents, (unsigned long long)e);
        if (e > 0 && !in->parent_oid) return wg_fail(c, WG_E_INVALID, "null parent_oid");
    }
    c->n = n;
    c->e_refs = e;
    c->sh.N = n;
    c->sh.s = 0;
    c->sh.e = n;
    c->sh.row_base = 0;
    if (in->residency == WG_HOST) {
        wg_stage_begin(c, "h2d");
        WG_ALLOC(c, c->in_oid, n * 20 + 4);
        WG_ALLOC(c, c->in_time, n * 8 + 8);
        WG_ALLOC(c, c->in_poff, (n + 1) * 4);
        WG_ALLOC(c, c->in_poid, e * 20 + 4);
        WG_ALLOC(c, c->in_flags, n + 4);
        if (n) {
            WG_HIP(c, hipMemcpyAsync(c->in_oid.p, in->oid, n * 20, hipMemcpyHostToDevice, c->stream));
            WG_HIP(c, hipMemcpyAsync(c->in_time.p, in->time, n * 8, hipMemcpyHostToDevice, c->stream));
            if (in->flags) WG_HIP(c, hipMemcpyAsync(c->in_flags.p, in->flags, n, hipMemcpyHostToDevice, c->stream));
            else WG_HIP(c, hipMemsetAsync(c->in_flags.p, 0, n, c->stream));
        }
        WG_HIP(c, hipMemcpyAsync(c->in_poff.p, in->parent_off, (n + 1) * 4, hipMemcpyHostToDevice, c->stream));
        if (e) WG_HIP(c, hipMemcpyAsync(c->in_poid.p, in->parent_oid, e * 20, hipMemcpyHostToDevice, c->stream));
        c->d_oid = c->in_oid.as<uint8_t>();
        c->d_time = c->in_time.as<int64_t>();
        c->d_poff = c->in_poff.as<uint32_t>();
        c->d_poid = c->in_poid.as<uint8_t>();
        c->d_flags = c->in_flags.as<uint8_t>();
        wg_stage_end(c);
    } else if (in->residency == WG_DEVICE) {
        c->d_oid = in->oid;
        c->d_time = in->time;
        c->d_poff = in->parent_off;
        c->d_poid = in->parent_oid;
        if (in->flags) c->d_flags = in->flags;
        else {
            WG_ALLOC(c, c->in_flags, n + 4);
            WG_HIP(c, hipMemsetAsync(c->in_flags.p, 0, n + 4, c->stream));
            c->d_flags = c->in_flags.as<uint8_t>();
        }
    } else {
        return wg_fail(c, WG_E_INVALID, "bad residency %d", in->residency);
    }
    int rc;
    // heights and the zero-band row_top depend on the commit times only: they
    // run on the side stream while the hash join and the lanes run here
    c->n_list = n;
    WG_ALLOC(c, c->heights, n * 4 + 4);
    WG_ALLOC(c, c->g_row_top, (n + 1) * 4);
    // wg_layout_build_frame: the frame's bands instead (a host band is
    // copied on the side stream first)
    c->build_banded = fband && n;
    const float *db = nullptr;
    if (c->build_banded) {
        db = fband;
        if (fres == WG_HOST) {
            WG_ALLOC(c, c->band, n * 4 + 4);
            db = c->band.as<const float>();
        }
        WG_ALLOC(c, c->band_prev, n * 4 + 4);   // the bands kept for the next frame's compare
    }
    // the hash table's build goes first on the side stream: the window probe
    // of the parent references runs beside it (wg_stage_hash_join)
    c->hash_built = c->hash_on_side = false;
    if ((rc = wg_side_build_begin(c, n, c->heights.as<float>(), c->g_row_top.as<float>(), db,
                                  db && fres == WG_HOST ? fband : nullptr, c->band.as<float>())) != WG_OK)
        return rc;
    // Speculative build (once an exact build has sized this context's
    // buffers): no host read until the end — event records and edges sized by
    // upper bounds, the replay run for the last build's iteration count, the
    // geometry lists sized by the buffers in place, every count read by the
    // kernels from the device — then one read validating all of it.  What did
    // not hold (a list that is not well formed, a replay short of its fixed
    // point, a list past its capacity) is redone by the exact stages.
    struct SpecOff { wg_ctx *c; ~SpecOff() { c->spec = false; } } spec_off{c};
    c->spec = c->spec_ready && !c->force_general_lanes && n > 0;
    const bool spec = c->spec;
    if ((rc = wg_stage_hash_join(c)) != WG_OK) return rc;
    if ((rc = wg_stage_lanes(c, spec)) != WG_OK) return rc;
    if ((rc = wg_stage_edges(c, spec)) != WG_OK) return rc;
    c->have_layout = true;
    c->layout_gen++;
    c->alt_heights_on = false;   // (a new built list: its own heights)
    // self.row_geometry with the default node_y / zero bands (:322-346), or
    // the frame's (build_frame; its bands copied to band_prev as they are read)
    if ((rc = wg_side_join(c)) != WG_OK) return rc;
    {
        struct KeepOff { wg_ctx *c; ~KeepOff() { c->band_keep = nullptr; } } keep_off{c};
        c->band_keep = db ? c->band_prev.as<float>() : nullptr;
        if ((rc = wg_stage_geometry(c, db)) != WG_OK) return rc;
    }
    if (spec) {
        constexpr int K = WG_PENDING_ITEMS;
        static_assert(K + 1 <= FETCH_MAX, "validation words exceed one fetch");
        WgFetch it[K];
        const int kl = wg_lanes_spec_items(c, it);
        int k = kl + wg_geom_spec_items(c, it + kl);
        it[k++] = WgFetch{c->edge_cnt.as<uint32_t>() + n, false};
        c->spec = false;
        if (c->defer_validation) {
            // no host read: the words are read with the next emission's vertex
            // total (or by the next call that needs the layout on the host).
            // Until then the lists are taken as the build's (a frame pass on
            // this layout reuses them, grids sized by their capacities) and
            // the emission takes graph_width from the device.
            PendingBuild &P = c->pend;
            P = PendingBuild{};
            P.build = true;
            P.k = k;
            P.kl = kl;
            for (int i = 0; i < k; i++) P.it[i] = it[i];
            c->lists_gen = c->layout_gen;
            c->lists_n = n;
            c->lists_ne = c->n_edges;
            c->lists_nsuper = c->spec_nsuper_grid;
            c->geom_sum_stale = false;
            c->have_geom = true;
            c->geom_key_gen = c->layout_gen;
            c->geom_key_band = c->build_banded;
            return WG_OK;
        }
        uint64_t v[K] = {0};
        if ((rc = wg_fetch_n(c, k, it, v)) != WG_OK) return rc;
        bool redo = false;
        return build_check(c, v, kl, k, &redo);
    }
    c->spec_ready = c->lists_gen == c->layout_gen;   // an exact or validated build: the buffers are sized
    c->have_geom = true;
    c->geom_key_gen = c->layout_gen;   // the geometry of (this layout, the build's bands)
    c->geom_key_band = c->build_banded;
    return WG_OK;
}

int wg_layout_summary_get(wg_ctx *c, wg_layout_summary *out) {
    if (!c || !out) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_layout) return wg_fail(c, WG_E_STATE, "no layout built");
    const ShardState &S = c->sh;
    out->n_rows = S.e - S.s;
    out->row_begin = S.s;
    out->n_edges = c->n_edges;
    if (S.on && !S.replicated) out->n_edges = S.n_own_edges;
    else if (S.on) {
        uint32_t eo[2] = {0, 0};
        WG_HIP(c, hipMemcpyAsync(&eo[0], c->edge_cnt.as<uint32_t>() + S.s, 4, hipMemcpyDeviceToHost, c->stream));
        WG_HIP(c, hipMemcpyAsync(&eo[1], c->edge_cnt.as<uint32_t>() + S.e, 4, hipMemcpyDeviceToHost, c->stream));
        WG_HIP(c, hipStreamSynchronize(c->stream));
        out->n_edges = eo[1] - eo[0];
    }
    out->max_lane = c->max_lane;
    out->n_slots = c->n_slots;
    out->graph_width = c->graph_width;
    out->lane_path = c->lane_path;
    return WG_OK;
}

int wg_copy_lanes(wg_ctx *c, uint32_t *lane, uint8_t *color) {
    if (!c) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_layout) return wg_fail(c, WG_E_STATE, "no layout built");
    const uint64_t rows = c->sh.e - c->sh.s, b = c->sh.row_base;
    if (lane && rows)
        WG_HIP(c, hipMemcpyAsync(lane, c->lane_out.as<uint32_t>() + b, rows * 4, hipMemcpyDeviceToHost, c->stream));
    if (color && rows)
        WG_HIP(c, hipMemcpyAsync(color, c->color_out.as<uint8_t>() + b, rows, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

int wg_copy_edges(wg_ctx *c, wg_edge *edges) {
    if (!c || !edges) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_layout) return wg_fail(c, WG_E_STATE, "no layout built");
    const ShardState &S = c->sh;
    if (S.on && !S.replicated) {
        if (S.n_own_edges)
            WG_HIP(c, hipMemcpyAsync(edges, S.own_edges.p, S.n_own_edges * sizeof(wg_edge), hipMemcpyDeviceToHost, c->stream));
    } else if (S.on) {
        uint32_t eo[2] = {0, 0};
        WG_HIP(c, hipMemcpyAsync(&eo[0], c->edge_cnt.as<uint32_t>() + S.s, 4, hipMemcpyDeviceToHost, c->stream));
        WG_HIP(c, hipMemcpyAsync(&eo[1], c->edge_cnt.as<uint32_t>() + S.e, 4, hipMemcpyDeviceToHost, c->stream));
        WG_HIP(c, hipStreamSynchronize(c->stream));
        if (eo[1] > eo[0])
            WG_HIP(c, hipMemcpyAsync(edges, c->edges.as<wg_edge>() + eo[0], (eo[1] - eo[0]) * sizeof(wg_edge),
                                     hipMemcpyDeviceToHost, c->stream));
    } else if (c->n_edges) {
        WG_HIP(c, hipMemcpyAsync(edges, c->edges.p, c->n_edges * sizeof(wg_edge), hipMemcpyDeviceToHost, c->stream));
    }
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

int wg_copy_row_heights(wg_ctx *c, float *h) {
    if (!c || !h) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_layout) return wg_fail(c, WG_E_STATE, "no layout built");
    const uint64_t rows = c->sh.e - c->sh.s;
    if (rows) WG_HIP(c, hipMemcpyAsync(h, c->heights.as<float>() + c->sh.row_base, rows * 4, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

// compute_row_heights (:486-507) as the free function it is in the reference:
// heights of any time list, independent of the context's layout
int wg_compute_row_heights(wg_ctx *c, const int64_t *time, uint64_t n, int32_t residency, float *heights) {
    if (!c || (n && (!time || !heights))) return WG_E_INVALID;
    if (residency != WG_HOST && residency != WG_DEVICE) return wg_fail(c, WG_E_INVALID, "bad residency %d", residency);
    if (n == 0) return WG_OK;
    (void)hipSetDevice(c->device);
    const int64_t *d_time = time;
    float *d_out = heights;
    if (residency == WG_HOST) {
        WG_ALLOC(c, c->hs_time, n * 8);
        WG_ALLOC(c, c->hs_out, n * 4);
        WG_HIP(c, hipMemcpyAsync(c->hs_time.p, time, n * 8, hipMemcpyHostToDevice, c->stream));
        d_time = c->hs_time.as<const int64_t>();
        d_out = c->hs_out.as<float>();
    }
    int rc = wg_heights_run(c, n, n, d_out, d_time);
    if (rc != WG_OK) return rc;
    if (residency == WG_HOST) WG_HIP(c, hipMemcpyAsync(heights, d_out, n * 4, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

// ---------------------------------------------------------------------------
// row_geometry_with_bands (:367-399)
// ---------------------------------------------------------------------------
// first row whose band differs bitwise from the previous frame's (atomicMin)
__global__ void k_band_diff(const uint32_t *__restrict__ a, const uint32_t *__restrict__ b, uint64_t n,
                            unsigned long long *first) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        if (a[i] != b[i]) { atomicMin(first, (unsigned long long)i); return; }
}

// row_geometry_with_bands(&self, commits, band_heights) (:367-399) with its
// commits argument: heights from the passed list's times (compute_row_heights
// (commits), :372), the geometry from the built edges; the built list itself
// (same times) is the per-frame path of wg_row_geometry.  One row per built
// row: a list of another length is refused (WG_E_INVALID), never replaced by
// the built list.
int wg_row_geometry_list(wg_ctx *c, const wg_commits *cm, const float *band, int32_t band_residency) {
    if (!c || !cm) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_layout) return wg_fail(c, WG_E_STATE, "no layout built");
    if (c->sh.on && !c->sh.replicated) return wg_fail(c, WG_E_STATE, "sharded layout: use wg_shard_geometry_begin");
    if (cm->n_commits != c->n)
        return wg_fail(c, WG_E_INVALID, "row_geometry_with_bands: %llu commits for a layout built on %llu (one row per built row)",
                       (unsigned long long)cm->n_commits, (unsigned long long)c->n);
    const uint64_t n = c->n;
    if (n && !cm->time) return wg_fail(c, WG_E_INVALID, "row_geometry_with_bands: commits without times");
    (void)hipSetDevice(c->device);
    const int64_t *t = cm->time;
    if (n && cm->residency == WG_HOST) {
        WG_ALLOC(c, c->alt_time, n * 8 + 8);
        WG_HIP(c, hipMemcpyAsync(c->alt_time.p, cm->time, n * 8, hipMemcpyHostToDevice, c->stream));
        t = c->alt_time.as<const int64_t>();
    } else if (n && cm->residency != WG_DEVICE) {
        return wg_fail(c, WG_E_INVALID, "bad residency %d", cm->residency);
    }
    // The built list's times by pointer only when they are the engine's own
    // copy (a host-resident build).  Anything else — a copy, or the caller's
    // device buffer the build read, which may have been rewritten since — has
    // its heights recomputed as it stands and compared with the heights the
    // build computed (a snapshot the caller cannot touch): equal heights give
    // the same geometry, so the per-frame reuse stands.
    const bool own = c->d_time == c->in_time.as<const int64_t>();
    bool same = !n || (t == c->d_time && own);
    if (!same) {
        WG_ALLOC(c, c->alt_heights, n * 4 + 4);
        if (const int rc = wg_heights_run(c, n, n, c->alt_heights.as<float>(), t)) return rc;
        WG_ALLOC(c, c->geom_diff_first, 16);
        WG_HIP(c, hipMemsetAsync(c->geom_diff_first.p, 0xFF, 8, c->stream));
        const uint64_t g = std::min<uint64_t>((n + 255) / 256, 2048);
        hipLaunchKernelGGL(k_band_diff, dim3((uint32_t)g), dim3(256), 0, c->stream, c->alt_heights.as<const uint32_t>(),
                           c->heights.as<const uint32_t>(), n, c->geom_diff_first.as<unsigned long long>());
        uint64_t first = 0;
        if (const int frc = wg_fetch(c, {{c->geom_diff_first.p, true}}, &first)) return frc;
        same = first == ~0ull;
    }
    if (same) {
        if (c->alt_heights_on) { c->alt_heights_on = false; c->geom_key_gen = ~0ull; }
    } else {
        c->alt_heights_on = true;
        c->geom_key_gen = ~0ull;   // (no per-frame reuse across height sets)
    }
    return row_geometry_impl(c, band, band_residency);
}

int wg_row_geometry(wg_ctx *c, const float *band, int32_t residency) {
    if (!c) return WG_E_INVALID;
    if (c->alt_heights_on) {   // the built list again: its own heights
        WG_SETTLE(c);
        c->alt_heights_on = false;
        c->geom_key_gen = ~0ull;
    }
    if (c->pend.build) {   // a deferred build: this pass is redone with it if it does not hold
        c->pend.frame = true;
        c->pend.frame_band = band != nullptr;
        c->pend.emit = false;
    }
    return row_geometry_impl(c, band, residency);
}

static int row_geometry_impl(wg_ctx *c, const float *band, int32_t residency) {
    if (!c->have_layout) return wg_fail(c, WG_E_STATE, "no layout built");
    if (c->sh.on && !c->sh.replicated) return wg_fail(c, WG_E_STATE, "sharded layout: use wg_shard_geometry_begin");
    (void)hipSetDevice(c->device);
    const bool had_geom = c->have_geom;
    c->have_geom = c->have_vtx = c->have_text = false;
    const float *d_band = nullptr;
    if (band) {
        if (residency == WG_HOST) {
            WG_ALLOC(c, c->band, c->n * 4 + 4);
            if (c->n) WG_HIP(c, hipMemcpyAsync(c->band.p, band, c->n * 4, hipMemcpyHostToDevice, c->stream));
            d_band = c->band.as<float>();
        } else if (residency == WG_DEVICE) {
            d_band = band;
        } else {
            return wg_fail(c, WG_E_INVALID, "bad residency %d", residency);
        }
    }
    // Per-frame reuse (history_view recomputes
    // row_geometry_with_bands every frame, commit_graph.rs:1419-1421): the same
    // layout with bitwise the same bands as the geometry in place -> nothing to do.
    const bool same_layout = had_geom && c->geom_key_gen == c->layout_gen;
    c->geom_r0 = 0;   // whole pass unless the compare below finds equal leading bands
    if (same_layout && !band && !c->geom_key_band) { c->have_geom = true; return WG_OK; }
    if (same_layout && band && c->geom_key_band && c->n) {
        WG_ALLOC(c, c->geom_diff_first, 16);
        WG_HIP(c, hipMemsetAsync(c->geom_diff_first.p, 0xFF, 8, c->stream));
        const uint64_t g = std::min<uint64_t>((c->n + 255) / 256, 2048);
        hipLaunchKernelGGL(k_band_diff, dim3((uint32_t)g), dim3(256), 0, c->stream, reinterpret_cast<const uint32_t *>(d_band),
                           c->band_prev.as<const uint32_t>(), c->n, c->geom_diff_first.as<unsigned long long>());
        uint64_t first = 0;
        if (const int frc = wg_fetch(c, {{c->geom_diff_first.p, true}}, &first)) return frc;
        if (first == ~0ull) { c->have_geom = true; return WG_OK; }
        c->geom_r0 = first;   // rows below `first` keep their geometry
    }
    int rc;
    // the bands this geometry is made with, kept for the next frame's compare:
    // written by k_row_basic as it reads them (rows below r0 are equal already)
    if (band && c->n) {
        WG_ALLOC(c, c->band_prev, c->n * 4 + 4);
        c->band_keep = c->band_prev.as<float>();
    }
    struct KeepOff { wg_ctx *c; ~KeepOff() { c->band_keep = nullptr; } } keep_off{c};
    // bands equal below geom_r0: row_top is rescanned from there
    if ((rc = wg_stage_rowtop(c, d_band, c->geom_r0)) != WG_OK) return rc;
    if ((rc = wg_stage_geometry(c, d_band)) != WG_OK) return rc;
    c->have_geom = true;
    c->geom_key_gen = c->layout_gen;
    c->geom_key_band = band != nullptr;
    c->geom_r0 = 0;
    return WG_OK;
}

// the own rows' slice of the row arrays: [b, b + rows), CSR ranges from vert_off/curve_off[b]
static int own_geometry_range(wg_ctx *c, uint64_t *v0, uint64_t *v1, uint64_t *c0, uint64_t *c1) {
    const uint64_t b = c->sh.row_base, rows = c->sh.e - c->sh.s;
    uint32_t o[4] = {0, 0, 0, 0};
    WG_HIP(c, hipMemcpyAsync(&o[0], c->vert_off.as<uint32_t>() + b, 4, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipMemcpyAsync(&o[1], c->vert_off.as<uint32_t>() + b + rows, 4, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipMemcpyAsync(&o[2], c->curve_off.as<uint32_t>() + b, 4, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipMemcpyAsync(&o[3], c->curve_off.as<uint32_t>() + b + rows, 4, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    *v0 = o[0]; *v1 = o[1]; *c0 = o[2]; *c1 = o[3];
    return WG_OK;
}

int wg_geometry_summary_get(wg_ctx *c, wg_geometry_summary *out) {
    if (!c || !out) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_geom) return wg_fail(c, WG_E_STATE, "no geometry");
    if (const int rc = wg_geom_summary_sync(c)) return rc;
    out->n_rows = c->sh.e - c->sh.s;
    out->n_vert = c->n_vert;
    out->n_curve = c->n_curve;
    out->total_height = c->total_height;
    out->scan_path = c->scan_path;
    if (c->sh.on) {
        uint64_t v0, v1, c0, c1;
        int rc = own_geometry_range(c, &v0, &v1, &c0, &c1);
        if (rc != WG_OK) return rc;
        out->n_vert = v1 - v0;
        out->n_curve = c1 - c0;
        float t = 0.0f;   // row_top at the end of the shard
        WG_HIP(c, hipMemcpyAsync(&t, c->g_row_top.as<float>() + c->sh.row_base + (c->sh.e - c->sh.s), 4,
                                 hipMemcpyDeviceToHost, c->stream));
        WG_HIP(c, hipStreamSynchronize(c->stream));
        out->total_height = t;
    }
    return WG_OK;
}

int wg_copy_geometry(wg_ctx *c, const wg_geometry_host *d) {
    if (!c || !d) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_geom) return wg_fail(c, WG_E_STATE, "no geometry");
    if (const int rc = wg_geom_summary_sync(c)) return rc;
    const uint64_t n = c->sh.e - c->sh.s, b = c->sh.row_base;
    uint64_t v0 = 0, v1 = c->n_vert, c0 = 0, c1 = c->n_curve;
    if (c->sh.on) {
        int rc = own_geometry_range(c, &v0, &v1, &c0, &c1);
        if (rc != WG_OK) return rc;
    }
    hipStream_t s = c->stream;
    if (d->height && n) WG_HIP(c, hipMemcpyAsync(d->height, c->g_height.as<float>() + b, n * 4, hipMemcpyDeviceToHost, s));
    if (d->node_y && n) WG_HIP(c, hipMemcpyAsync(d->node_y, c->g_node_y.as<float>() + b, n * 4, hipMemcpyDeviceToHost, s));
    if (d->row_top) WG_HIP(c, hipMemcpyAsync(d->row_top, c->g_row_top.as<float>() + b, (n + 1) * 4, hipMemcpyDeviceToHost, s));
    if (d->vert_off) WG_HIP(c, hipMemcpyAsync(d->vert_off, c->vert_off.as<uint32_t>() + b, (n + 1) * 4, hipMemcpyDeviceToHost, s));
    if (d->curve_off) WG_HIP(c, hipMemcpyAsync(d->curve_off, c->curve_off.as<uint32_t>() + b, (n + 1) * 4, hipMemcpyDeviceToHost, s));
    if (d->vert && v1 > v0)
        WG_HIP(c, hipMemcpyAsync(d->vert, c->vert.as<uint32_t>() + v0, (v1 - v0) * 4, hipMemcpyDeviceToHost, s));
    if (d->curve && c1 > c0)
        WG_HIP(c, hipMemcpyAsync(d->curve, c->curve.as<wg_curve>() + c0, (c1 - c0) * sizeof(wg_curve), hipMemcpyDeviceToHost, s));
    if (d->curve_color && c1 > c0)
        WG_HIP(c, hipMemcpyAsync(d->curve_color, c->curve_color.as<uint8_t>() + c0, c1 - c0, hipMemcpyDeviceToHost, s));
    WG_HIP(c, hipStreamSynchronize(s));
    // offsets relative to the copied slice
    for (uint64_t i = 0; c->sh.on && i <= n; i++) {
        if (d->vert_off) d->vert_off[i] -= (uint32_t)v0;
        if (d->curve_off) d->curve_off[i] -= (uint32_t)c0;
    }
    return WG_OK;
}

// ---------------------------------------------------------------------------
// graph_cell (:803-908) tessellated per WG-TESS-1
// ---------------------------------------------------------------------------
int wg_emit_vertices(wg_ctx *c, uint64_t rb, uint64_t re, int64_t sel, const float *palette) {
    if (!c || !palette) return WG_E_INVALID;
    if (!c->have_geom) return wg_fail(c, WG_E_STATE, "no geometry");
    const ShardState &S = c->sh;
    if (rb > re || rb < S.s || re > S.e)
        return wg_fail(c, WG_E_INVALID, "row range [%llu,%llu) outside [%llu,%llu)", (unsigned long long)rb,
                       (unsigned long long)re, (unsigned long long)S.s, (unsigned long long)S.e);
    (void)hipSetDevice(c->device);
    c->have_vtx = false;
    if (c->pend.build) {   // a deferred build: validated by this call's vertex-total read (wg_stage_vertices)
        c->pend.emit = true;
        c->pend.rb = rb;
        c->pend.re = re;
        c->pend.sel = sel;
    }
    WG_ALLOC(c, c->palette, 2 * WG_PALETTE_SIZE * 4 * sizeof(float));
    if (!c->palette_valid || std::memcmp(c->palette_host, palette, WG_PALETTE_SIZE * 4 * sizeof(float)) != 0) {   // upload on change only
        // entries 8..15: the same colours at opacity WG_DIM_ALPHA (search dimming)
        std::memcpy(c->palette_host, palette, WG_PALETTE_SIZE * 4 * sizeof(float));
        for (int i = 0; i < 4 * WG_PALETTE_SIZE; i++)
            c->palette_host[4 * WG_PALETTE_SIZE + i] = (i & 3) == 3 ? palette[i] * WG_DIM_ALPHA : palette[i];
        WG_HIP(c, hipMemcpyAsync(c->palette.p, c->palette_host, sizeof(c->palette_host), hipMemcpyHostToDevice, c->stream));
        WG_HIP(c, hipStreamSynchronize(c->stream));   // palette_host may change before the copy ran
        c->palette_valid = true;
    }
    // global rows -> the context's row arrays (a shard's rows start at row_base)
    const uint64_t b = S.row_base;
    const int64_t sel_l = (sel >= 0 && (uint64_t)sel >= S.s && (uint64_t)sel < S.e) ? (int64_t)((uint64_t)sel - S.s + b) : -1;
    int rc = wg_stage_vertices(c, rb - S.s + b, re - S.s + b, sel_l);
    if (rc != WG_OK) return rc;
    c->vrow_begin = rb;
    c->vrow_end = re;
    c->selected = sel;
    c->have_vtx = true;
    return WG_OK;
}

int wg_vertex_summary_get(wg_ctx *c, wg_vertex_summary *out) {
    if (!c || !out) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_vtx) return wg_fail(c, WG_E_STATE, "no vertices emitted");
    out->row_begin = c->vrow_begin;
    out->row_end = c->vrow_end;
    out->n_vertices = c->n_vtx;
    uint64_t chk = 0;
    int rc = wg_vertex_checksum_run(c, &chk);
    if (rc != WG_OK) return rc;
    out->checksum = chk;
    return WG_OK;
}

int wg_copy_vertices(wg_ctx *c, uint64_t first, uint64_t count, wg_vertex *dst) {
    if (!c || (!dst && count)) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_vtx) return wg_fail(c, WG_E_STATE, "no vertices emitted");
    if (first > c->n_vtx || count > c->n_vtx - first) return wg_fail(c, WG_E_INVALID, "vertex range out of bounds");
    if (count)
        WG_HIP(c, hipMemcpyAsync(dst, c->vtx.as<wg_vertex>() + first, count * sizeof(wg_vertex), hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

int wg_copy_vertex_offsets(wg_ctx *c, uint64_t *dst) {
    if (!c || !dst) return WG_E_INVALID;
    WG_SETTLE(c);
    if (!c->have_vtx) return wg_fail(c, WG_E_STATE, "no vertices emitted");
    WG_HIP(c, hipMemcpyAsync(dst, c->vtx_off.p, (c->vrow_end - c->vrow_begin + 1) * 8, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    return WG_OK;
}

int wg_device_views_get(wg_ctx *c, wg_device_views *o) {
    if (!c || !o) return WG_E_INVALID;
    WG_SETTLE(c);
    std::memset(o, 0, sizeof(*o));
    const uint64_t b = c->sh.row_base;   // views start at the first own row
    if (c->have_layout) {
        o->lane = c->lane_out.as<uint32_t>() + b;
        o->color = c->color_out.as<uint8_t>() + b;
        o->edges = (c->sh.on && !c->sh.replicated) ? c->sh.own_edges.as<wg_edge>() : c->edges.as<wg_edge>();
    }
    if (c->have_geom) {
        o->height = c->g_height.as<float>() + b;
        o->node_y = c->g_node_y.as<float>() + b;
        o->row_top = c->g_row_top.as<float>() + b;
        o->vert_off = c->vert_off.as<uint32_t>() + b;
        o->vert = c->vert.as<uint32_t>();
        o->curve_off = c->curve_off.as<uint32_t>() + b;
        o->curve = c->curve.as<wg_curve>();
        o->curve_color = c->curve_color.as<uint8_t>();
    }
    if (c->have_vtx) {
        o->vtx_off = c->vtx_off.as<uint64_t>();
        o->vertices = c->vtx.as<wg_vertex>();
    }
    return WG_OK;
}

int wg_debug_counters(wg_ctx *c, uint32_t *out, int n) {
    if (!c || !out || n < 0) return WG_E_INVALID;
    WG_SETTLE(c);
    if (n > 16) n = 16;
    if (!c->lane_scalars.p) return wg_fail(c, WG_E_STATE, "no layout built");
    WG_HIP(c, hipMemcpyAsync(out, c->lane_scalars.p, (size_t)n * 4, hipMemcpyDeviceToHost, c->stream));
    WG_HIP(c, hipStreamSynchronize(c->stream));
    if (n > 3) out[3] = c->replay_iters;
    if (n > 4) out[4] = (uint32_t)c->n_events;
    if (n > 5) out[5] = c->sh.on ? (c->sh.replicated ? 2u : 1u) : 0u;
    if (n > 6) out[6] = c->spec_builds;
    if (n > 7) out[7] = c->spec_redo_lanes;
    if (n > 8) out[8] = c->spec_redo_geom;
    if (n > 9) out[9] = c->spec_replays_shard;
    if (n > 10) out[10] = c->last_serial ? 1u : 0u;
    if (n > 11) out[11] = c->sliced_emits;
    if (n > 12) out[12] = c->last_form;
    if (n > 13) out[13] = c->last_leaks;
    if (n > 14) out[14] = c->last_dc_warm;
    return WG_OK;
}

int wg_enable_timing(wg_ctx *c, int on) {
    if (!c) return WG_E_INVALID;
    c->timing = on != 0;
    for (int i = 0; i < on && i < WG_STAGE_MAX; i++)
        if (!c->stages[i].a) { WG_HIP(c, wg_timing_event(&c->stages[i].a)); WG_HIP(c, wg_timing_event(&c->stages[i].b)); }
    c->n_stages = 0;
    c->stage_depth = 0;
    return WG_OK;
}

int wg_stage_timings(wg_ctx *c, int *n_stages, const char **names, float *ms) {
    if (!c || !n_stages) return WG_E_INVALID;
    WG_HIP(c, hipStreamSynchronize(c->stream));
    *n_stages = c->n_stages;
    for (int i = 0; i < c->n_stages; i++) {
        if (names) names[i] = c->stages[i].name;
        if (ms) {
            float t = 0.0f;
            WG_HIP(c, hipEventElapsedTime(&t, c->stages[i].a, c->stages[i].b));
            ms[i] = t;
        }
    }
    return WG_OK;
}

}  // extern "C"
