// wg_internal.h — engine-internal declarations shared by the HIP sources.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>
#include <initializer_list>

#include "wgraph.h"

// ---- wave-level scans on DPP (no LDS round trip per step) --------------------
// __shfl_up compiles to ds_bpermute: every step of a shuffle scan is an LDS
// round trip (~50+ cycles), and the single-wave kernels (row_top walk, lane
// replay) are chains of such scans.  These use the GFX9 DPP row shifts and
// row broadcasts instead (the pattern of rocPRIM's warp scan); the combine is
// applied in order, comb(earlier, later), so it need not commute.
template <int CTRL, int ROWMASK, class T>
__device__ __forceinline__ T wg_dpp(const T &old, const T &x) {
    static_assert(sizeof(T) % 4 == 0, "DPP moves 32-bit words");
    constexpr int N = sizeof(T) / 4;
    uint32_t o[N], v[N], r[N];
    __builtin_memcpy(o, &old, sizeof(T));
    __builtin_memcpy(v, &x, sizeof(T));
#pragma unroll
    for (int i = 0; i < N; i++)
        r[i] = (uint32_t)__builtin_amdgcn_update_dpp((int)o[i], (int)v[i], CTRL, ROWMASK, 0xF, false);
    T out;
    __builtin_memcpy(&out, r, sizeof(T));
    return out;
}
// inclusive scan over the 64 lanes: lane i gets comb(x_0, ..., x_i); id = identity
template <class T, class C>
__device__ __forceinline__ T wg_wave_scan(T x, const T &id, C comb) {
    x = comb(wg_dpp<0x111, 0xF>(id, x), x);   // row_shr:1
    x = comb(wg_dpp<0x112, 0xF>(id, x), x);   // row_shr:2
    x = comb(wg_dpp<0x114, 0xF>(id, x), x);   // row_shr:4
    x = comb(wg_dpp<0x118, 0xF>(id, x), x);   // row_shr:8
    x = comb(wg_dpp<0x142, 0xA>(id, x), x);   // row_bcast:15 into rows 1, 3
    x = comb(wg_dpp<0x143, 0xC>(id, x), x);   // row_bcast:31 into rows 2, 3
    return x;
}
// lane i gets lane i - 1's value, lane 0 gets id (exclusive from inclusive)
template <class T>
__device__ __forceinline__ T wg_wave_shr1(const T &x, const T &id) { return wg_dpp<0x138, 0xF>(id, x); }
// lane `lane`'s value in every lane (lane wave-uniform)
__device__ __forceinline__ uint32_t wg_lane(uint32_t v, uint32_t lane) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}

#define WG_EMPTY 0xFFFFFFFFu   // "None" slot / empty hash entry / no row

// ---------------------------------------------------------------------------
// Device buffer that only grows (keeps HBM resident across frames).
// ---------------------------------------------------------------------------
struct DevBuf {
    void  *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) { hipError_t e = hipFree(p); p = nullptr; cap = 0; if (e != hipSuccess) return e; }
        // 1/16 headroom: a list that grows a little (a refresh prepending a few
        // commits) fits the buffers in place — no reallocation, and the
        // speculative build's capacity checks still pass
        size_t b = bytes < 256 ? 256 : bytes + bytes / 16;
        hipError_t e = hipMalloc(&p, b);
        if (e == hipSuccess) cap = b;
        return e;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
    template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

struct StageTimer {
    const char *name = nullptr;
    hipEvent_t  a = nullptr, b = nullptr;   // created on first use
};

// Crossing parent reference (row-sharded builds, wg_shard.hip): a reference
// from row c to a row p that lies beyond the shard of c.  kf: bits 0..15 the
// parent index within row c, bit 16 "first occurrence of p among row c's
// in-list parents" (the greedy ignores repeated parents, :435-459).
struct WgXEnt { uint32_t c, p, kf, pad; };
#define WG_XF_FIRST_IN_ROW 0x10000u
#define WG_XF_LLEAKY       0x20000u   // (a reference to an earlier row) the target's shard holds a leaky reference to it
// chain tokens of the lane fast path: an event id, a crossing entry (resolved
// once the other shards have reported), a row (pointer jumping) or nothing
#define WG_TOK_EV   0x80000000u
#define WG_TOK_X    0x40000000u
#define WG_TOK_NONE 0xFFFFFFFFu

// The rows one lane fast-path run owns: [s, e) of a list whose CSR and
// resolved parent rows are indexed globally.  A single-GPU build is s = 0,
// e = N with no crossing entries.
struct LfRange {
    uint64_t s = 0, nl = 0, e = 0;
    const uint32_t *poff = nullptr;   // parent_off, by global row
    const int32_t *prow = nullptr;    // parent row, by global ref index (own refs)
    const uint32_t *canon = nullptr;  // by global row, or null (ids known distinct)
    const WgXEnt *xall = nullptr;     // crossing entries of every shard, shard-major
    uint64_t xin_end = 0;             // [0, xin_end): entries of earlier shards
    uint64_t xown_begin = 0, xown_end = 0;   // this shard's own entries
    // device-resident bounds (the sharded X2 step, before any host read): when
    // set, xin_end = xown_begin = *xb_dev and xown_end = *xe_dev, and the host
    // fields above are upper bounds (grids, sizes) with xown_begin = 0
    const uint32_t *xb_dev = nullptr, *xe_dev = nullptr;
    uint8_t *isfb = nullptr;          // by global ref index: target beyond e and first reference to it
    uint32_t *xsec = nullptr;         // by global ref index: SECALLOC token of such a secondary reference
    // by target row - s: the first (row, parent index) reference to the target
    // from the target's own row or a later one (a parent at an earlier row:
    // clock skew, orphans re-sorted by time, self parents).  Null: such
    // references make the list "not well formed" (general walk).
    unsigned long long *lfirst = nullptr;
};

// Row-top transducer scan geometry (wg_rowtop.hip)
#define WG_RT_CHUNK   1024   // rows per chunk
#define WG_RT_NBIN    4      // binades tabulated per chunk (guess-1 .. guess+2)

// Sweep geometry (wg_geom.hip)
#define WG_SWEEP_CH   64     // rows per sweep chunk (one wave)
#define WG_SWEEP_CAP  2048   // active-edge capacity per wave (LDS)

// Vertex tiles (wg_vertex.hip)

// Row-sharded build state (wg_shard.hip)
struct ShardState {
    bool on = false;          // the last build was a wg_shard_build_* build
    bool replicated = false;  // ... that fell back to the whole-list build on every rank
    int world = 1, rank = 0, step = 0;
    uint64_t N = 0, s = 0, e = 0, Etot = 0;
    uint64_t E0 = 0, E1 = 0;  // own parent references [parent_off[s], parent_off[e])
    uint64_t row_base = 0;    // index of row s in the context's row arrays
    DevBuf msg;               // this rank's outgoing message
    const uint32_t *heads = nullptr;   // host copy of the gathered 16-byte headers (one exchange call)
    const uint64_t *sizes = nullptr;   // every rank's message length (one exchange call)
    uint64_t msg_bytes = 0;   // exact length, or (msg_dev) the buffer's capacity
    bool msg_dev = false;     // the length is on the device (msg_len), written by the producing kernels
    DevBuf msg_len;           // u64: device-resident message length
    DevBuf ptable;            // id partition table (global duplicate check)
    DevBuf prow;              // int32 [E1-E0] parent rows of own references
    DevBuf unres;             // unresolved-reference records of every rank (32 B each)
    uint64_t n_unres = 0;
    std::vector<uint64_t> uoffs;   // per-rank prefix of those records
    DevBuf flags, xcnt, refx, isfb, xsec;
    DevBuf dlist;   // the partition's rows {home slot, fingerprint, row} for the duplicate scan's settle pass
    DevBuf xall;              // WgXEnt [nx]: crossing entries of every rank
    std::vector<uint64_t> xoff, evoff, auxoff;   // per-rank prefixes (world + 1)
    DevBuf xtok, xt;          // chain token per crossing entry: shard-local / global
    DevBuf dev_small;
    DevBuf h_g, rt_g;         // heights / row_top of every row of the list (the crossing edges' far endpoints)
    bool rt_fresh = false;        // rt_g was computed at build begin (side stream) with the bands rt_band
    const float *rt_band = nullptr;
    const float *build_band = nullptr;   // wg_shard_build_frame_begin: the build's geometry takes these bands
    uint64_t local_gen = ~0ull;           // layout_gen of the local edges (c->edges / edge_cnt / in_scan)
    uint64_t local_ne = 0, local_nin = 0; // local edges, of which incoming
    DevBuf band_host;         // device copy of a host band array [N]
    const float *band_g = nullptr;
    DevBuf xchild, xpar;      // per crossing entry: child lane/colour/y, parent lane/y (built locally from etok)
    DevBuf lk;                // uint8 [nl]: an own row some own row at or after it references (a leaky reference)
    DevBuf etok;              // uint32 [2 nx]: per crossing entry the global token of its child row / parent row
    DevBuf elane;             // uint32 [2 nx]: ... and their lanes, after the replay
    DevBuf death;             // uint32 [nev]: consumption time of every global event's token (the replay's first iteration)
    DevBuf in_scan, edge_y, own_edges;
    uint64_t n_own_edges = 0;
    bool geom_spec_ready = false;   // an earlier sharded geometry pass sized the lists (speculation may start)
    bool geom_banded = false;       // the last local geometry pass took bands (c->band holds the local copy)
    bool replay_pending = false;    // X3 replayed speculatively: its words are checked with the local geometry's
    uint32_t rp_it = 0, rp_chunk = 0;
    const uint32_t *rp_flags = nullptr, *rp_scal = nullptr;
    bool rp_dc = false;       // ... by the compacted replay, at rp_nw words
    uint32_t rp_nw = 1, rp_warm = 0;
};

// SDF font atlas slot (wg_font.hip)
struct FontSlot {
    bool built = false;
    uint32_t W = 0, H = 0, spread = 0, R = 0, first_char = 0;
    uint64_t n_edges = 0;
    float em_px = 0, ascent = 0, descent = 0, line_gap = 0;
    std::vector<wg_glyph> glyphs;
    DevBuf edges, gdesc, cov, sdf, gin, gout, d2in, d2out, gtab;
    // the last build's font bytes (length + 64-bit hash) and parameters: a
    // rebuild of the same font at the same parameters skips the TrueType parse
    // and the uploads (the outlines and descriptors on the device still hold)
    bool have_key = false;
    uint64_t key_len = 0, key_hash = 0;
    std::vector<uint8_t> key_bytes;   // the last font's bytes: a hash match is confirmed by memcmp
    wg_atlas_params key_prm{};
    uint32_t n_gd = 0, max_ch = 0;
};

// workspace slots in wg_ctx::lf (wg_lanes_fast.hip; the sharded build reuses LF_EVREC / LF_AUX for the
// gathered event records)
enum { LF_FIRST, LF_FPC, LF_WINFO, LF_EVOFF, LF_SECEV, LF_CHOFF, LF_CHFILL, LF_CH, LF_SPA, LF_SPB, LF_EVREC,
       LF_SLOT, LF_FLAGS, LF_SLOTB, LF_OCC, LF_STATS, LF_RFLAGS, LF_AUXOFF, LF_AUX, LF_LFIRST, LF_SERREC, LF_DEATH,
       LF_DCVEC, LF_DCMASK, LF_DCPRE, LF_DCLIST, LF_DCSNAP, LF_DCSLOT, LF_COUNT };

// event replay to a fixed point (wg_lanes_replay.hip)
struct ReplayRun {
    uint64_t nev = 0, nch = 0;
    uint32_t chunk = 512, it = 0, max_iters = 0;
    const uint4 *ev = nullptr;
    const uint32_t *aux = nullptr;
    uint16_t *slots_a = nullptr, *slots_b = nullptr, *sp_prev = nullptr, *sp_next = nullptr;   // sp_prev: last written
    uint32_t nw = 1;                     // occupancy words (1, 4 or 16: up to 63, 255, 1023 slots)
    bool ser_w8 = false;                 // nw 16 on the serial pass with 8 words (511 slots; the last list used <= 448)
    bool ser_w3 = false;                 // nw 4 on the serial pass with 3 words (191 slots; the last list used <= 170)
    uint32_t warm = 0;                   // iteration 1 starts this many events before each chunk
    unsigned long long *occ_a = nullptr, *occ_b = nullptr, *op = nullptr, *on = nullptr;
    uint32_t *stats = nullptr, *flags = nullptr, *scal = nullptr;
    const uint32_t *nev_dev = nullptr;   // speculative build: event count on the device (nev = upper bound)
    const uint32_t *gate = nullptr;      // speculative build: nonzero = not well formed, replay nothing
    uint32_t switch_it = 0;              // exact replay at a short chunk: still moving at this iteration ->
    bool switched = false;               // stop; the caller replays at WG_REPLAY_CHUNK_LONG (wg_replay_resume)
    const uint32_t *death = nullptr;     // per event the time of the event consuming its token (0xFFFFFFFF: none),
                                         // or null: the first iteration then runs the general replay kernel
    uint32_t serial_it = 0;              // exact replay at the long chunk: still moving at this iteration ->
    bool to_serial = false;              // stop; the caller replays serially (wg_replay_resume)
    // compacted D-state chunked replay (wg_lanes_dchunk.hip): nw = words of positions (1, 2, 4)
    bool dc = false;
    uint32_t *dc_dvec[2] = {nullptr, nullptr};   // exit D-vectors per chunk, two iterations in turn
    unsigned long long *dc_lkmask = nullptr;     // per 64-event batch: the leaking events
    uint32_t *dc_bpre = nullptr;                 // per batch: leaks before it (k_dc_snap)
    uint32_t *dc_lklist = nullptr;               // the leaking events in order
    uint16_t *dc_snap = nullptr;                 // the non-leaked slots after each leak, [leak_cap + 1][64 nw]
    uint32_t dc_leak_cap = 0;
    uint16_t *dc_pos = nullptr;                  // the final positions (wg_dc_finish)
    uint16_t *dc_slot = nullptr;                 // the slots (wg_dc_finish; sp_prev points here after it)
    uint64_t dc_blocks = 0;                      // k_dc_fix blocks = stats records (3 words each)
};
// the compacted D-state chunked replay (wg_lanes_dchunk.hip): R.slots_a / b
// hold positions; wg_dc_init clears the flag words, wg_dc_iterate launches
// iterations (the first warm-started), wg_dc_finish turns the last positions
// into slots (R.sp_prev, R.stats per WG_DC_FIX_T events).  lane_scalars [4]
// the highest allocated position + 1, [5] leaks, [6] more leaks than dc_leak_cap.
constexpr uint32_t WG_DC_FIX_T = 256;
uint32_t wg_dc_words(uint32_t positions);   // 1, 2 or 4 words for that many positions below the sentinel; 0: none
constexpr uint32_t WG_DC_LEAK_CAP = 16384;   // leaks the snapshots hold (more: the serial pass)
// resets the run (positions in R.slots_a / b); flags: also clear the flag
// words (a speculative build's event kernel clears them otherwise)
hipError_t wg_dc_init(hipStream_t s, ReplayRun &R, bool flags);
hipError_t wg_dc_scalars(hipStream_t s, const ReplayRun &R);   // lane scalars [0..4] after wg_dc_finish (wg_lanes_replay.hip)
hipError_t wg_dc_iterate(hipStream_t s, ReplayRun &R, uint32_t n);
hipError_t wg_dc_finish(hipStream_t s, ReplayRun &R);
// The replay's chunk lengths (events).  Short chunks make iteration 1 short
// (its chunks replay serially, one wave each) and suit lists whose greedy
// state forgets a wrong entry within a chunk; on others (long-lived lanes
// carrying a wrong guess across many chunks: the Linux shape) the fixed point
// turns linear in the chunk count, and the list is replayed at the long chunk.
constexpr uint32_t WG_REPLAY_CHUNK_SHORT = 128, WG_REPLAY_CHUNK_LONG = 512;
constexpr uint32_t WG_REPLAY_SHORT_MAX_FP = 6;   // a short-chunk replay needing more iterations: long chunks next
constexpr uint32_t WG_REPLAY_SWITCH_IT = 12;     // exact replay: iterations at the short chunk before the switch
constexpr uint64_t WG_REPLAY_WIDE_EVENTS = 131072;   // 1024 short chunks: above, short chunks of twice the length

// small device -> host reads (wg_api.hip): one tiny kernel writes the values
// into mapped pinned host memory, then the stream is synchronised — instead of
// one blit per hipMemcpyAsync into pageable memory
struct WgFetch { const void *p; bool wide; };   // wide: 8-byte value, else 4-byte

// speculative build validation words: lanes + geometry + the edge count
constexpr int WG_LANES_SPEC_ITEMS = 12;
constexpr int WG_GEOM_SPEC_ITEMS = 8;
constexpr int WG_PENDING_ITEMS = WG_LANES_SPEC_ITEMS + WG_GEOM_SPEC_ITEMS + 1;

// A speculative build whose validation was deferred (WG_OPT_DEFER_VALIDATION)
// and what was queued after it: it is read with the next emission's vertex
// total (or by wg_settle), and a build that did not hold is redone then
struct PendingBuild {
    bool build = false;
    bool shard = false;             // a sharded build's speculative geometry pass only (its lanes are exact)
    int k = 0, kl = 0;              // validation items, of which the lane stage's
    WgFetch it[WG_PENDING_ITEMS];
    bool frame = false, frame_band = false;   // a frame geometry pass followed (its bands are in band_prev)
    bool emit = false;              // ... and an emission of rows [rb, re)
    uint64_t rb = 0, re = 0;
    int64_t sel = -1;
};

struct wg_ctx {
    int         device = 0;
    hipStream_t stream = nullptr;
    bool        own_stream = false;
    // side stream: the build's zero-band row_top (a function of the commit
    // times only) runs there, overlapping the latency-bound lane phases
    hipStream_t side = nullptr, side_main = nullptr;
    hipEvent_t  ev_fork = nullptr, ev_join = nullptr;
    hipEvent_t  ev_hash = nullptr;   // the side stream's hash table is built (wg_side_build_begin)
    bool        side_pending = false;
    std::string err;

    // ---- last layout build -------------------------------------------------
    uint64_t n = 0, e_refs = 0, n_edges = 0;
    uint64_t n_list = 0;      // rows of the whole list (n differs for a row shard)
    bool     have_layout = false;
    uint32_t max_lane = 0, n_slots = 0, lane_path = 1;
    uint32_t slots_last = 0;  // n_slots of the last completed lane build (a build in progress has cleared n_slots)
    // the slot count the next replay's width and narrow forms follow
    uint32_t slots_hint() const { return n_slots ? n_slots : slots_last; }
    float    graph_width = 24.0f;
    // inputs (device copies when the caller passed host memory)
    DevBuf in_oid, in_time, in_poff, in_poid, in_flags;
    DevBuf hs_time, hs_out;   // wg_compute_row_heights scratch (independent of the layout)
    const uint8_t  *d_oid = nullptr;
    const int64_t  *d_time = nullptr;
    const uint32_t *d_poff = nullptr;
    const uint8_t  *d_poid = nullptr;
    const uint8_t  *d_flags = nullptr;
    // hash join
    DevBuf hash;            // uint64 [hcap]  (fingerprint<<32 | row), then the duplicate flag word
    uint64_t hcap = 0;
    // single-GPU join (wg_hash.hip): two tables used in turn; the place pass
    // empties the one the next build uses.  htab_clean[k]: words known empty.
    DevBuf htab[2];
    uint64_t htab_clean[2] = {0, 0};
    int htab_cur = 0;
    const unsigned long long *htab_last = nullptr;   // the last join's table (hcap slots)
    DevBuf canon;           // uint32 [N]  last row holding the same id
    DevBuf rowmiss;         // uint8  [N]  a reference of the row missed the window probe (wg_hash.hip)
    unsigned long long *hash_table = nullptr;   // the table of this build (wg_hash_table_launch)
    // WG_OPT_JOIN_FUSED: the table's place pass in the window probe, settle on the main stream (r05 A/B on
    // wide16 1M: 1.438 / 1.444 ms/step against 1.434 / 1.434 with the table beside the probe: off)
    bool join_fused = false;
    uint32_t match_threads = 512;   // WG_OPT_MATCH_THREADS
    bool hash_built = false, hash_on_side = false;   // ... launched already (on the side stream)
    DevBuf prow;            // int32  [E]  canonical parent row or -1
    // lanes
    DevBuf lane_asg;        // uint32 [N]  lane assigned while processing row
    DevBuf lane_out;        // uint32 [N]  layouts.get(id).lane per row
    DevBuf color_out;       // uint8  [N]
    DevBuf lane_scalars;    // uint32 [8]  max_lane, n_slots, overflow, ...
    DevBuf lf[LF_COUNT];    // event-compressed lane path workspaces (wg_lanes_fast.hip), indexed by LF_*
    uint32_t replay_chunk = 512;   // events per replay chunk (WG_OPT_REPLAY_CHUNK)
    uint32_t replay_warm = 0;      // iteration 1's warm-up events before each chunk (WG_OPT_REPLAY_WARMUP)
    bool replay_auto = true;       // neither option set: chunk / warm-up follow the last build's event count
    // Auto: the short chunk with a warm-up first, the long chunk once a list
    // needed more than WG_REPLAY_SHORT_MAX_FP iterations at the short one
    // (replay_long; an exact replay still moving at WG_REPLAY_SWITCH_IT starts
    // over at the long chunk).  profiles/r03l_replay_tune.jsonl: wide16 1M
    // (46k events) 128 + 512 warm-up 0.160 ms (5 iterations) against 512 / 0
    // 0.203 (4); random13 100k (13.9k events) 128 + 256 0.092 against 0.117;
    // the Linux shape (93k events) needs 21+ iterations below 512: long.
    bool replay_long = false;
    void replay_geometry(uint32_t *chunk, uint32_t *warm) const {
        *chunk = replay_chunk;
        *warm = replay_warm;
        if (!replay_auto) return;
        if (!replay_long) {   // (short lists: 64-event chunks — random13 100k 0.093 -> 0.085 ms, r03l / r03q)
            *chunk = n_events >= 24576 ? WG_REPLAY_CHUNK_SHORT : WG_REPLAY_CHUNK_SHORT / 2;
            *warm = n_events >= 24576 ? 512u : 256u;
            // More chunks than SIMDs (a sharded build's global replay: 368k
            // events at 8 x 1M rows): iteration 1 turns throughput-bound on
            // the scalar units, and the warm-up is paid per chunk — double
            // chunks halve it (r03 emulation: 235 -> 207 us per step)
            if (n_events >= WG_REPLAY_WIDE_EVENTS) *chunk = 2 * WG_REPLAY_CHUNK_SHORT;
        }
        else { *chunk = WG_REPLAY_CHUNK_LONG; *warm = 0; }
    }
    // Serial replay (wg_lanes_serial.hip): lists whose greedy state does not
    // forget a wrong guess (long-lived lanes) need about one chunked
    // fixed-point iteration per chunk; their lanes come from one exact
    // single-wave pass instead.  Compacted replay (wg_lanes_dchunk.hip, r05):
    // the D-state chunked fixed point with the leaked slots struck out, for
    // the lists whose greedy state forgets once the leaks are gone (parents at
    // earlier rows, the Linux shape).  Auto: a short-chunk replay that needs
    // more than WG_REPLAY_SHORT_MAX_FP iterations moves the context to the
    // compacted replay; a compacted replay whose fixed point comes late
    // doubles its warm-up, and one whose iterations cost more than the serial
    // pass would moves it to the serial pass; the serial choice expires after
    // WG_SERIAL_RETRY builds (the compacted replay is tried again), and a list
    // of a very different length (mode_rows) starts over.
    uint32_t replay_mode = 0;      // WG_OPT_REPLAY_MODE: 0 auto, 1 chunked fixed point, 2 serial, 3 compacted
    bool replay_serial = false;    // auto: this list shape replays serially
    bool replay_dc = false;        // auto: this list shape replays by the compacted fixed point
    bool last_serial = false;      // the last lane replay was the serial pass (wg_debug_counters [10])
    uint32_t last_form = 0;        // the last replay's form (wg_debug_counters [12], WG_FORM_*)
    uint32_t last_leaks = 0;       // leaked slots struck out by the last compacted replay ([13])
    uint32_t last_dc_warm = 0;     // ... and its warm-up ([14])
    uint32_t serial_builds = 0;    // serial builds since the auto choice was made
    uint32_t dc_plain_builds = 0;  // compacted builds in a row that struck out no leak (the chunked replay is retried)
    static constexpr uint32_t WG_SERIAL_RETRY = 16;
    uint32_t dc_warm = 8192;       // the compacted replay's first-iteration warm-up (events)
    uint32_t dc_warm_fixed = 0;    // WG_OPT_DC_WARMUP (0: auto)
    static constexpr uint32_t WG_DC_WARM0 = 8192, WG_DC_WARM_MAX = 32768;
    uint32_t dc_nw = 1;            // words of positions of the next compacted replay (1, 2, 4)
    uint32_t dc_blind = 2;         // its iterations before the first check
    uint64_t mode_rows = 0;        // rows of the list the auto choices were made on
    // (mode 3: the compacted replay, or the serial pass where it does not apply)
    bool use_serial() const { return replay_mode == 2 || ((replay_mode == 0 || replay_mode == 3) && replay_serial); }
    bool use_dc() const { return (replay_mode == 3 || (replay_mode == 0 && replay_dc)) && !replay_serial; }
    // estimated cost of the serial pass (us) against one chunked iteration at the long chunk
    static double serial_cost_us(uint64_t nev, uint32_t nw) {
        return (double)nev * (nw <= 1 ? 0.016 : nw <= 2 ? 0.04 : nw <= 4 ? 0.07 : nw <= 16 ? 0.3 : 1.0);
    }
    static constexpr double WG_CHUNKED_ITER_US = 60.0;
    // The compacted replay's cost model (us): one wave replays an event in
    // about 25 / 40 / 72 ns at 1 / 2 / 4 words of positions (the D-step's
    // instruction count, profiles/r05_dc_*); iteration 1 replays warm + chunk
    // events per wave, every later one chunk events plus a launch.
    static double dc_step_us(uint32_t nw) { return nw <= 1 ? 0.025 : nw <= 2 ? 0.04 : 0.072; }
    static double dc_iter_us(uint32_t nw, uint32_t chunk) { return chunk * dc_step_us(nw) + 5.0; }
    static double dc_cost_us(uint32_t nw, uint32_t warm, uint32_t chunk, uint32_t fp) {
        return (warm + chunk) * dc_step_us(nw) + (fp > 1 ? fp - 1 : 0) * dc_iter_us(nw, chunk);
    }
    // a list of a very different length: the auto choices start over
    void replay_shape(uint64_t rows) {
        if (mode_rows && (rows > 2 * mode_rows || 2 * rows < mode_rows)) {
            replay_long = false;
            replay_serial = false;
            replay_dc = false;
            dc_warm = dc_warm_fixed ? dc_warm_fixed : WG_DC_WARM0;
            dc_probe = dc_probe_down = false;
            dc_warm_frozen = false;
            dc_blind = 2;
            replay_blind = 4;
        }
        if (!mode_rows || rows > 2 * mode_rows || 2 * rows < mode_rows) mode_rows = rows;
    }
    // a serial build done: after WG_SERIAL_RETRY of them the compacted replay is tried again
    void serial_done() {
        if ((replay_mode != 0 && replay_mode != 3) || !replay_serial) return;
        if (++serial_builds >= WG_SERIAL_RETRY) {
            replay_serial = false;
            replay_dc = true;
            dc_warm = dc_warm_fixed ? dc_warm_fixed : WG_DC_WARM0;
            dc_probe = dc_probe_down = false;
            dc_blind = 2;
            serial_builds = 0;
        }
    }
    // A compacted replay (nw words, its warm-up and chunk) that reached its
    // fixed point at iteration fp: the serial pass when the model prices the
    // serial pass lower (auto); else a fixed point later than iteration 3
    // tries a doubled warm-up once (kept only if the model prices it lower:
    // long-lived lanes need more than any affordable warm-up); the blind count.
    bool dc_probe = false;         // the last compacted replay tried a doubled warm-up
    bool dc_probe_down = false;    // ... or a halved one (r06)
    bool dc_warm_frozen = false;   // a probe did not pay: the warm-up stays
    double dc_cost_before = 0;     // the modelled cost before that probe
    static constexpr uint32_t WG_DC_WARM_MIN = 512;
    void dc_adapt(uint32_t fp, uint64_t nev, uint32_t nw, uint32_t warm, uint32_t chunk, uint32_t serial_nw) {
        if (fp == 0) return;
        const double cost = dc_cost_us(nw, warm, chunk, fp);
        if (replay_mode == 0 && fp > 2 && cost > serial_cost_us(nev, serial_nw)) {
            replay_serial = true;
            serial_builds = 0;
            dc_probe = dc_probe_down = false;
            return;
        }
        if (dc_probe || dc_probe_down) {
            // the probe's warm-up stays only if the model prices it lower
            // with the iterations it actually took; else back, and no more probes
            if (cost >= dc_cost_before) {
                dc_warm = dc_probe ? (warm / 2 >= 64 ? warm / 2 : 64) : warm * 2;
                dc_warm_frozen = true;
            }
            dc_probe = dc_probe_down = false;
        } else if (fp > 3 && warm < WG_DC_WARM_MAX && !dc_warm_fixed && !dc_warm_frozen) {
            dc_cost_before = cost;
            dc_warm = warm * 2;
            dc_probe = true;
        } else if (fp <= 3 && warm > WG_DC_WARM_MIN && !dc_warm_fixed && !dc_warm_frozen) {
            // (r06) iteration 1 is the warm-up's cost: a list whose state
            // forgets within a shorter window (the Linux shape: fixed point at
            // iteration 2 with 8192 events of warm-up, 205 of the replay's
            // 230 us) tries half of it
            dc_cost_before = cost;
            dc_warm = warm / 2;
            dc_probe_down = true;
        }
        dc_blind = fp >= dc_blind ? fp : (dc_blind + fp) / 2;
        if (dc_blind < 2) dc_blind = 2;
        // A changed warm-up may need more iterations than this one took: the
        // next speculative build launches generously many blind (an iteration
        // after the fixed point exits at once, k_dc_iter), so trying it never
        // costs an exact redo; the count adapts back down afterwards
        if (dc_warm != warm) {
            const uint32_t b = dc_warm < warm ? 4 * fp + 4 : 2 * fp + 2;
            if (dc_blind < b) dc_blind = b;
        }
    }
    uint32_t replay_iters = 0;     // iterations the last replay needed
    uint32_t replay_blind = 4;     // iterations launched before the first convergence check (adapts)
    uint32_t replay_nw = 1;        // occupancy words of the next replay (from the last build's slot count)
    // the narrowest occupancy (1, 4, 16 words) holding n_slots slots below the sentinel
    static uint32_t nw_for_slots(uint32_t slots) {
        return slots < 64 ? 1u : (slots < 256 ? 4u : (slots < 1024 ? 16u : 64u));   // (64: the serial workgroup, 4095 slots)
    }
    // After a replay that reached its fixed point at iteration fp (the first that
    // changed nothing), the next build's blind count: up at once, down by half
    // the excess per build (it used to fall by one per build: after a list that
    // needed hundreds of iterations, later builds launched hundreds of empty ones).
    void replay_adapt(uint32_t fp, uint32_t chunk = 0) {
        if (fp == 0) return;
        // auto: a long-chunk replay that needed more iterations than the serial pass costs
        if (replay_mode == 0 && chunk == WG_REPLAY_CHUNK_LONG && fp * WG_CHUNKED_ITER_US > serial_cost_us(n_events, replay_nw)) {
            replay_serial = true;
            return;
        }
        if (replay_auto && chunk < WG_REPLAY_CHUNK_LONG && fp > WG_REPLAY_SHORT_MAX_FP) {
            if (replay_mode == 0) replay_dc = true;   // this list shape wants the compacted replay
            else replay_long = true;                  // (held on the chunked replay: the long chunk)
            replay_blind = 4;
            return;
        }
        replay_blind = fp >= replay_blind ? fp : (fp > (replay_blind + fp) / 2 ? fp : (replay_blind + fp) / 2);
        if (replay_blind < 2) replay_blind = 2;
    }
    uint64_t n_events = 0;  // events of the last fast-path lane build
    uint64_t e_refs_own = 0;   // parent references of the rows this context owns
    bool lf_sp_b = false;   // chain sources ended in lf[LF_SPB] (else lf[LF_SPA])
    const uint16_t *lf_slot_of = nullptr;      // the last lane replay's slot per event (valid until the next replay)
    uint32_t *lf_death = nullptr;              // lf[LF_DEATH] when the last wg_lf_chain was a single-GPU one
    const uint32_t *replay_death = nullptr;    // the exact single-GPU replay's consumption times (replay_setup)
    bool lane_out_fused = false;
    bool lf_refs_done = false;     // the hash join's kernels did the lane stage's clear + reference pass (single GPU)
    bool edge_scan_pending = false;   // (r06) a speculative build's edge-count scan rides on the lane stage's (wg_lf_refs)
    bool edges_pending = false;    // the edge list is written by the next full geometry pass (k_edges_rows)   // the lane kernel wrote lane_out / color_out (speculative fast path)
    bool force_general_lanes = false;   // WG_LANES=general (testing the general walk)
    ReplayRun spec_run;     // the speculative build's replay (its iteration count and flag words)
    // speculative build (wg_layout_build): launches sized by upper bounds and
    // capacities, counts read by the kernels from the device, one host read at
    // the end validating them (the exact form redoes anything that failed)
    bool spec = false;          // the build in progress is speculative
    bool spec_ready = false;    // an exact build sized this context's buffers (speculation may start)
    bool defer_validation = false;   // WG_OPT_DEFER_VALIDATION
    bool spec_replay_shard = true;   // WG_OPT_SHARD_SPEC_REPLAY
    PendingBuild pend;
    uint64_t spec_nsuper_grid = 0;   // the speculative geometry pass's curve-record grid (its capacity)
    uint32_t spec_builds = 0, spec_redo_lanes = 0, spec_redo_geom = 0;   // speculative builds, of which lanes / geometry redone
    uint32_t spec_replays_shard = 0;   // sharded builds whose global replay ran blind (WG_OPT_SHARD_SPEC_REPLAY)
    // edges
    DevBuf edge_cnt;        // uint32 [N+1] -> edge_off after scan
    DevBuf edges;           // wg_edge [n_edges]
    // heights
    DevBuf heights;         // float [N]
    // row_geometry_with_bands on a list other than the built one (wg_row_geometry_list):
    // the frame passes take the heights of that list's times until the built list comes back
    DevBuf alt_heights, alt_time;
    bool alt_heights_on = false;
    const float *geom_heights() const { return alt_heights_on ? alt_heights.as<const float>() : heights.as<const float>(); }
    // ---- geometry ------------------------------------------------------------
    bool     have_geom = false;
    uint64_t n_vert = 0, n_curve = 0;
    uint32_t scan_path = 0;
    float    total_height = 0.0f;
    DevBuf band;            // float [N] device copy of caller bands
    DevBuf g_height, g_node_y, g_row_top;   // float [N], [N], [N+1]
    // wg_layout_build_frame: the build's own geometry pass took the frame's
    // bands (the band copy in band_prev); a redone build redoes it with them
    bool build_banded = false;
    DevBuf rt_chunk;        // per-chunk scan state
    DevBuf rt_tables;       // per-chunk transducer tables
    DevBuf rt_sup;          // super-chunk tables, binade bases and walk states
    DevBuf rt_flags;        // uint32 [4]
    DevBuf geom_zero;       // zeroed per pass: per-row counts / diff arrays, top fill, carry counts, sweep flags
    uint64_t geom_zero_n = ~0ull;   // rows the workspace was zeroed for ahead of the pass (wg_geom_prezero), or ~0
    DevBuf vert_off, curve_off;             // uint32 [N+1]
    DevBuf vert, curve, curve_color;
    DevBuf curve_ref;       // uint32 [n_curve] edge id per curve record
    DevBuf curve_row;       // uint32 [n_curve] row per curve record
    DevBuf curve_tb;        // float [n_curve] each record's t at its strip bottom (k_curves_tb)
    DevBuf carry_off, carry, carry_sorted;  // sweep carry-in lists (registration order / edge order)
    DevBuf curve_cnt;                       // uint32 [N+1] per-row curve counts (filter)
    uint64_t lists_nsuper = 0;              // curve superset records of the lists in place
    uint32_t *geom_err = nullptr;           // the last full pass's flag words (sweep error, overflow at +8)
    bool geom_sum_stale = false;            // total_height / scan_path / n_curve not read back yet
    const void *geom_sum_at[3] = {nullptr, nullptr, nullptr};   // where they are (row_top[n], scan flag, curve_off[n])
    DevBuf scan_tmp;        // scan workspace
    DevBuf scan_tmp_side;   // scan workspace of the side stream (geometry carry offsets)
    DevBuf bsum;            // producer tile sums of the wg_scan_bs_u32 scans (3 arrays of wg_bs_blocks(n) + 64)
    DevBuf scal;            // uint64 [16] device scalars (totals)
    DevBuf rowflags;        // uint8 [N] bit0 zero-height strip, bit1 child strip empty, bit2 parent strip empty
    // The ordered lists (vert, curve_ref/curve_row, offsets) depend on the
    // layout and the row flags only, not on row_top: a geometry pass on the
    // same layout whose flags equal those the lists were built with reuses
    // them and recomputes heights, row_top, node_y and the curves.
    uint64_t layout_gen = 0;            // bumped by every layout build
    uint64_t lists_gen = ~0ull;         // layout_gen the lists were built for (~0: none)
    uint64_t lists_n = 0, lists_ne = 0;
    DevBuf rowflags_lists;              // the flags the curve lists were filtered with
    DevBuf scurve_off, scurve_ref, scurve_row;   // curve superset (flags ignored), swept once per layout
    DevBuf geom_diff;                   // 2 x 16 uint32: flags differ (+ the pass's overflow word at 8), used in turn
    int geom_diff_par = 0;
    // per-frame reuse: the geometry in place was made for (layout geom_key_gen, bands or none)
    uint64_t geom_key_gen = ~0ull;
    bool     geom_key_band = false;
    DevBuf   band_prev;                 // float [N] the bands of that geometry
    float   *band_keep = nullptr;       // wg_row_geometry: k_row_basic writes the bands it reads here (band_prev)
    DevBuf   geom_diff_first;           // u64: first row whose band differs
    uint64_t geom_r0 = 0;               // that row, for the next geometry pass (0: whole pass)
    DevBuf sweep_big;       // uint32 [nch] chunks too wide for the register sweep
    uint32_t sweep_reg_cap = 512;   // edges per chunk the register sweep holds (WG_OPT_SWEEP_REG)
    const float *edge_y = nullptr;   // per edge {child_y, parent_y} override (row-sharded geometry), or null
    // Row-sliced lists (wg_geom_lists): a speculative full pass whose
    // validation rides on the emission leaves its list kernels (top halves,
    // sweep, curve clipping) to wg_stage_vertices, which runs rows [0, h) first
    // and rows [h, n) on the side stream beside the emission of the first
    // slice's tiles.  Any other call runs them whole first (WG_SETTLE).
    struct ListsDef {
        bool deferred = false;
        uint64_t n = 0, n_super_grid = 0;
        const uint32_t *cntF = nullptr, *cntT = nullptr;
        const uint32_t *vtot = nullptr, *stot = nullptr, *ctot = nullptr;   // the lists' scanned totals (capacity checks)
        uint32_t vcap = ~0u, scap = ~0u, ccap = ~0u;
        uint32_t *err = nullptr;   // the pass's flag words (geom_err)
        // a speculative pass after a list with no chunk past the register
        // sweep: the LDS sweep is not launched, and a chunk that needs it
        // raises the capacity-overflow word (the exact pass redoes the lists)
        bool lds_off = false;
    } glist;
    bool     slice_on = false;     // WG_OPT_SLICE_LISTS (measured slower on wide16 1M: DESIGN §3.2a)
    double   slice_frac = 0.25;
    uint64_t slice_min_rows = 1ull << 18;   // (WG_OPT_SLICE_LISTS = 2: every list of >= 4 chunks, for the tests)
    uint64_t vtx_t1_last = 0;      // the last sliced emission's first second-slice tile (part 1's grid)
    uint32_t sliced_emits = 0;     // emissions that ran row-sliced lists (wg_debug_counters [11])
    uint32_t sweep_wide_last = 0;  // the last read pass's chunks past the register sweep (sizes the LDS sweep's grid)
    hipEvent_t ev_slice = nullptr;
    // ---- vertices -------------------------------------------------------------
    bool     have_vtx = false;
    uint64_t vrow_begin = 0, vrow_end = 0, n_vtx = 0;
    uint64_t vtx_tiles_last = 0;   // tiles of the last emission (bounds the next one's early grid)
    uint32_t vtx_tile_last = 1024; // ... of this many vertices (wg_vertex.hip)
    uint32_t vtx_tile_opt = 0;     // WG_OPT_VTX_TILE: 0 auto, 1024 or 2048
    uint32_t vtx_place = 4;        // WG_OPT_VTX_PLACE: vertex buffer candidates (wg_vertex.hip wg_alloc_placed)
    uint32_t vtx_place_n = 0, vtx_place_pick = 0;   // the last placement: candidates probed, the one kept
    float    vtx_place_ms[8] = {};
    static constexpr uint64_t WG_VTX_BIG_VERTICES = 400000000ull;   // auto: 2048-vertex tiles past this many
    int64_t  selected = -1;
    DevBuf vtx_off;         // uint64 [rows+1]
    DevBuf vtx;             // wg_vertex [n_vtx]
    DevBuf palette;         // float [64]: palette, then the same at WG_DIM_ALPHA
    float   palette_host[2 * WG_PALETTE_SIZE * 4];   // last uploaded palette (+ dimmed)
    bool    palette_valid = false;
    DevBuf chk;             // uint64 [1]
    DevBuf tile_first;      // uint4 [tiles+1] per-tile record (first row, first vertical, first curve, straddles)
    // ---- host-side tables --------------------------------------------------------
    uint32_t h_thresh[32];  // delta thresholds for heights 29..56
    ShardState sh;
    FontSlot fonts[WG_FONT_SLOTS];
    // ---- glyph quads (wg_text.hip) ------------------------------------------------
    bool     have_text = false;
    uint64_t text_rb = 0, text_re = 0, n_quads = 0;
    DevBuf text_sum, text_sum_off, text_off, text_rec, text_vtx;
    int32_t text_slot = 0;          // atlas slot of the last glyph emission
    float    text_scale = 1.0f;     // its text_px / em_px
    // ---- rasteriser (wg_render.hip) -------------------------------------------------
    DevBuf render_small, render_img;
    // ---- search-match flags (wg_search.hip) -------------------------------------------
    bool     match_on = false;      // a non-empty query is active: emission dims non-matching rows
    uint64_t match_rb = 0, match_re = 0, match_count = 0;
    DevBuf   match_flags;           // uint8 [match_re - match_rb]
    DevBuf   match_q;               // {count u64, pad} + fail u16[m] + q u8[m]
    DevBuf match_flat;      // uint32 [WG_FLAT_N] lowercase | case classes of the BMP (search)
    DevBuf   match_txt[2], match_off[2];   // device copies of host summary / author text
    std::vector<uint64_t> match_rel[2];
    std::vector<uint8_t>  match_qhost;
    // ---- row order (wg_order.hip) ------------------------------------------------------
    DevBuf   ord[8];
    std::vector<uint32_t> ord_host;
    uint64_t ord_n = 0;
    // ---- timing ----------------------------------------------------------------------
    bool       timing = false;
    bool       timing_emit_only = false;   // WG_OPT_TIMING_EMIT_ONLY
    StageTimer stages[WG_STAGE_MAX];
    int        n_stages = 0;
    int        stage_stack[8] = {0};
    int        stage_depth = 0;
    uint64_t   scratch_host[16];
    uint64_t  *h_fetch = nullptr;   // mapped pinned host memory for wg_fetch / wg_fetch_begin
    hipEvent_t ev_fetch = nullptr;  // completion of the pending wg_fetch_begin
    int        fetch_pending = 0;   // words of the pending wg_fetch_begin
    bool       fetch_fused = false; // ... written by a producing kernel (wg_fetch_fused_begin): no event behind it
    bool       fused_read = true;   // WG_OPT_FUSED_READ: the emission's read folded into k_vtx_prep
    hipEvent_t ev_defer = nullptr;  // completion of the last wg_fetch_defer
    int        defer_pending = 0;   // words of the last wg_fetch_defer
    uint64_t  *d_fetch = nullptr;
    uint64_t   fetch_seq = 0;       // sequence number of the last k_fetch launch
    uint64_t   fetch_want[3] = {0, 0, 0};   // per fetch region: the launch whose words it holds
};

int wg_fetch(wg_ctx *c, std::initializer_list<WgFetch> items, uint64_t *out);
int wg_fetch_n(wg_ctx *c, int n, const WgFetch *items, uint64_t *out);   // n <= 64
// the same read without waiting: queue it, queue more work, then wg_fetch_end
// (one pending at a time)
int wg_fetch_begin(wg_ctx *c, std::initializer_list<WgFetch> items);
int wg_fetch_begin_n(wg_ctx *c, int n, const WgFetch *items);
// deferred validation (WG_OPT_DEFER_VALIDATION, wg_api.hip): wg_settle reads
// and checks a pending build's words; wg_validate_pending checks words read
// by the caller.  A build that did not hold is redone with the exact stages,
// followed by the frame pass and emission queued after it (*redone = true).
int wg_settle(wg_ctx *c);
int wg_validate_pending(wg_ctx *c, const uint64_t *v, bool *redone);
// a sharded geometry pass awaiting its validation (wg_shard.hip): check the
// words, redo the pass exactly when they do not hold (*redo)
int wg_shard_geom_validate(wg_ctx *c, const uint64_t *v, bool *redo);
#define WG_SETTLE(c)                                                               \
    do {                                                                           \
        if ((c)->pend.build || (c)->glist.deferred) {                              \
            const int _sr = wg_settle(c);                                          \
            if (_sr != WG_OK) return _sr;                                          \
        }                                                                          \
    } while (0)
int wg_fetch_end(wg_ctx *c, uint64_t *out);
// A read folded into a producing kernel instead of a k_fetch launch (and the
// event between that kernel and the next): wg_fetch_fused_begin fills the
// arguments for wg_fetch_begin's region, one device thread calls
// wg_fused_fetch_store after the words are final, wg_fetch_end reads them
// (its fallback wait is the stream's)
constexpr int WG_FETCH_MAX = 64;
struct WgFusedFetch {
    const void *p[WG_FETCH_MAX];
    unsigned long long wide;
    uint32_t n;
    unsigned long long *out, *seq_word, seq;
};
int wg_fetch_fused_begin(wg_ctx *c, int n, const WgFetch *items, WgFusedFetch *f);
__device__ __forceinline__ void wg_fused_fetch_store(const WgFusedFetch &f) {
    for (uint32_t i = 0; i < f.n; i++)
        f.out[i] = ((f.wide >> i) & 1ull) ? *reinterpret_cast<const volatile unsigned long long *>(f.p[i])
                                          : (unsigned long long)*reinterpret_cast<const volatile uint32_t *>(f.p[i]);
    __threadfence_system();
    __hip_atomic_store(f.seq_word, f.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
int wg_fetch_defer(wg_ctx *c, std::initializer_list<WgFetch> items);
int wg_fetch_deferred(wg_ctx *c, uint64_t *out);

// Batched device copies (+ a few host words) in ONE launch: the sharded
// exchanges move every rank's piece of a gathered buffer into place, which as
// one hipMemcpyAsync per piece was one blit launch each (~3 W launches per
// exchange); host words travel in the kernel arguments instead of a copy from
// pageable memory.  Byte counts and addresses are multiples of 4.
constexpr int WG_BCOPY_MAX = 48, WG_BCOPY_WORDS = 64;
struct WgCopyBatch {
    const void *src[WG_BCOPY_MAX];
    void       *dst[WG_BCOPY_MAX];
    uint64_t    bytes[WG_BCOPY_MAX];
    uint64_t   *wdst;                   // inline words -> wdst[0 .. nwords)
    uint64_t    words[WG_BCOPY_WORDS];
    uint32_t    n, nwords;
};
struct WgCopies {
    WgCopyBatch b{};
    bool overflow = false;
    void add(void *dst, const void *src, uint64_t bytes) {
        if (!bytes) return;
        if (b.n >= (uint32_t)WG_BCOPY_MAX) { overflow = true; return; }
        b.src[b.n] = src; b.dst[b.n] = dst; b.bytes[b.n] = bytes; b.n++;
    }
    // words [0, n) -> dst[at .. at + n) (one destination buffer per batch)
    void words(uint64_t *dst, uint32_t at, const uint64_t *w, uint32_t n) {
        if (b.wdst && b.wdst != dst) { overflow = true; return; }
        if (at + n > (uint32_t)WG_BCOPY_WORDS) { overflow = true; return; }
        b.wdst = dst;
        for (uint32_t i = 0; i < n; i++) b.words[at + i] = w[i];
        b.nwords = at + n > b.nwords ? at + n : b.nwords;
    }
};
int wg_copy_batch(wg_ctx *c, const WgCopies &cp, hipStream_t s);   // wg_api.hip

// error helpers -------------------------------------------------------------
int wg_fail(wg_ctx *c, int code, const char *fmt, ...);
#define WG_HIP(ctx, call)                                                          \
    do {                                                                           \
        hipError_t _e = (call);                                                    \
        if (_e != hipSuccess)                                                      \
            return wg_fail((ctx), WG_E_HIP, "%s:%d %s: %s", __FILE__, __LINE__,    \
                           #call, hipGetErrorString(_e));                          \
    } while (0)
#define WG_ALLOC(ctx, buf, bytes)                                                  \
    do {                                                                           \
        hipError_t _e = (buf).ensure(bytes);                                       \
        if (_e != hipSuccess)                                                      \
            return wg_fail((ctx), WG_E_NOMEM, "hipMalloc(%zu) failed: %s",         \
                           (size_t)(bytes), hipGetErrorString(_e));                \
    } while (0)

// stage timing
void wg_stage_begin(wg_ctx *c, const char *name);
void wg_stage_end(wg_ctx *c);

// scans (wg_scan.hip) -----------------------------------------------------------
// Exclusive scan of n uint32 in place into out[0..n] (out[n] = total).  The
// input may alias out.  tmp = c->scan_tmp after wg_scan_reserve(c, n).
size_t wg_scan_tmp_bytes(uint64_t n);
int wg_scan_reserve(wg_ctx *c, uint64_t n);   // grow c->scan_tmp for scans of up to n elements
hipError_t wg_exclusive_scan_u32(const uint32_t *in, uint32_t *out, uint64_t n, void *tmp, hipStream_t s);
// two independent arrays of the same length scanned in the same launches
hipError_t wg_exclusive_scan2_u32(const uint32_t *in0, uint32_t *out0, const uint32_t *in1, uint32_t *out1, uint64_t n,
                                  void *tmp, hipStream_t s);
hipError_t wg_exclusive_scan_u64(const uint64_t *in, uint64_t *out, uint64_t n, void *tmp, hipStream_t s);

// Scans whose tile sums come from the producer (no reduce launch): a producer
// kernel of WG_BS_THREADS-thread blocks, one element per thread, calls
// wg_bsum_store(v, bsum) with every thread of the block (it synchronises the
// block) and so leaves bsum[blockIdx.x] = the block's sum.  The down-sweep
// then needs one launch (up to WG_BS_SELF tile sums; more add a scan of the
// sums first).  Up to four arrays of the same length share the launches.
constexpr int WG_BS_THREADS = 256;
constexpr uint64_t WG_BS_SELF = 8192;
__device__ __forceinline__ void wg_bsum_store(uint32_t v, uint32_t *__restrict__ bsum) {
    __shared__ uint32_t wg_bs_w[WG_BS_THREADS / 64];
    v = wg_wave_scan(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
    if ((threadIdx.x & 63) == 63) wg_bs_w[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
#pragma unroll
        for (int w = 0; w < WG_BS_THREADS / 64; w++) t += wg_bs_w[w];
        bsum[blockIdx.x] = t;
    }
    __syncthreads();   // the staging words are reused by a following call
}
struct WgScanBs {
    int na = 0;
    const uint32_t *in[4] = {nullptr, nullptr, nullptr, nullptr};
    uint32_t *out[4] = {nullptr, nullptr, nullptr, nullptr};
    const uint32_t *bsum[4] = {nullptr, nullptr, nullptr, nullptr};   // [ceil(n / WG_BS_THREADS)] each
    uint64_t len[4] = {0, 0, 0, 0};   // an array shorter than n (0: n)
};
// out[a][0..n] = exclusive scan of in[a] (out[a][n] = total); in may alias out.
// tmp: c->scan_tmp after wg_scan_reserve(c, n).
hipError_t wg_scan_bs_u32(const WgScanBs &S, uint64_t n, void *tmp, hipStream_t s);
// tile sums (2048-element tiles) of two arrays, for a caller-fused down-sweep
hipError_t wg_tile_sums2_u32(const uint32_t *in0, const uint32_t *in1, uint64_t n, uint32_t *ts0, uint32_t *ts1,
                             hipStream_t s);
inline uint64_t wg_bs_blocks(uint64_t n) { return (n + WG_BS_THREADS - 1) / WG_BS_THREADS; }

// stages -------------------------------------------------------------------------
int wg_stage_hash_join(wg_ctx *c);            // wg_hash.hip
int wg_hash_table_launch(wg_ctx *c);          // wg_hash.hip: place + settle on c->stream
int wg_hash_clear_next(wg_ctx *c, hipStream_t s);   // the next build's table, emptied beside an emission
int wg_geom_prezero(wg_ctx *c, uint64_t n);   // wg_geom.hip: the next full pass's workspace zeroed on c->stream
// the build's side stream: the hash table (joined by the hash join's fix-up
// kernel), then the heights and the row_top (joined by the geometry)
int wg_side_build_begin(wg_ctx *c, uint64_t m, float *h, float *rt, const float *band, const float *band_host,
                        float *band_dev);
int wg_stage_lanes(wg_ctx *c, bool spec);     // wg_lanes.hip
int wg_lanes_fast(wg_ctx *c, bool *used, bool spec);   // wg_lanes_fast.hip

hipError_t wg_replay_start(wg_ctx *c, hipStream_t s, ReplayRun &R, uint32_t blind);
// speculative build: the replay's initial state is written by the event
// kernel (k_lf_events, WgReplayInit from wg_replay_prepare_spec), the
// iterations follow, and the scalars are reduced by the lanes kernel
// (wg_replay_finish_lanes, which also writes lane_out / colour: the fast path
// only runs on distinct ids, so every row is its own canonical row)
struct WgReplayInit {
    unsigned long long *occ = nullptr;
    uint64_t occ_words = 0;
    uint32_t *changed = nullptr;
    uint32_t nflags = 0;
    uint4 *slots16 = nullptr;
    uint64_t nslots16 = 0;
    const uint32_t *nev_dev = nullptr;   // zero records at ev[*nev_dev .. +256) (the replay prefetches past a chunk)
    uint64_t total = 0;                  // elements of the largest of these (grid-stride bound)
};
WgReplayInit wg_replay_prepare_spec(ReplayRun &R, uint32_t &blind);
hipError_t wg_replay_iterate_spec(hipStream_t s, ReplayRun &R, uint32_t blind);
hipError_t wg_replay_finish_lanes(hipStream_t s, const ReplayRun &R, uint64_t nl, const uint32_t *sp, uint32_t *lane,
                                  uint32_t *lane_out, uint8_t *color_out, const uint8_t *flags);
hipError_t wg_replay_resume(wg_ctx *c, hipStream_t s, ReplayRun &R, bool *converged);
// the serial replay (wg_lanes_serial.hip): R's buffers as for the chunked
// replay (R.nev, R.nw, R.ev, R.aux, R.slots_a/b, R.stats, R.flags, R.nev_dev,
// R.gate); rec: wg_replay_serial_rec_bytes(R.nev) of workspace.  Leaves R as a
// one-chunk replay that converged at iteration 1.
hipError_t wg_replay_serial(hipStream_t s, ReplayRun &R, uint4 *rec);
// the chunked replay's first iteration from R.death (one wave per chunk, the
// serial step from an empty table `warm` events ahead): slots and exit
// occupancies as k_lf_replay's iteration 1 would write them (NW = 1)
hipError_t wg_replay_first(hipStream_t s, const ReplayRun &R, uint16_t *slot_next, unsigned long long *occ_next);
uint64_t wg_replay_serial_rec_bytes(uint64_t nev);
int wg_stage_edges(wg_ctx *c, bool spec, int64_t ne_known = -1);   // wg_lanes.hip
// speculative build (wg_layout_build): validation words of the lane build
// (fills WG_LANES_SPEC_ITEMS items) and their check (wg_lanes_fast.hip)
int wg_lanes_spec_items(wg_ctx *c, WgFetch *it);
bool wg_lanes_spec_check(wg_ctx *c, const uint64_t *v);
// event-compressed lane phases over a row range (wg_lanes_fast.hip)
// scal: the lane scalars to clear with the stage's state (single-GPU build), or null
int wg_lf_refs(wg_ctx *c, const LfRange &R, bool read_back, uint32_t *scal = nullptr);   // + wg_lf_refs_end after queueing wg_lf_chain
int wg_lf_refs_end(wg_ctx *c, uint32_t *viol, uint64_t *nev, uint64_t *naux);
int wg_lf_chain(wg_ctx *c, const LfRange &R);
int wg_lf_export_tokens(wg_ctx *c, const LfRange &R, uint32_t *tok);
// sharded X3: the row token of every own crossing entry's child row (ctok, by
// own entry) and of every crossing entry's parent row in this shard (ptok, by
// global entry; WG_TOK_NONE elsewhere), xcap entries at most, *xtot on the device
int wg_lf_export_ends(wg_ctx *c, const LfRange &R, uint32_t *ctok, uint32_t *ptok, const uint32_t *xtot, uint64_t xcap);
// consumption time (event index + 1) of every token the nev global records consume; 0xFFFFFFFF: never
int wg_lf_death_from_records(wg_ctx *c, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *death);
int wg_lf_events(wg_ctx *c, const LfRange &R, uint32_t ev_base, const uint32_t *xt, uint4 *ev_out, uint32_t *aux_out,
                 uint32_t aux_base);
// sharded form: records with shard-local tokens / aux offsets (before the
// crossing tokens are resolved), then, on the gathered records of every rank,
// the global form (plus the own rows' chain tokens, for the lanes)
int wg_lf_events_local(wg_ctx *c, const LfRange &R, uint4 *ev_out, uint32_t *aux_out);
int wg_lf_events_finish(wg_ctx *c, const LfRange &R, uint32_t ev_base, const uint32_t *xt, uint64_t nx, uint64_t nev,
                        uint32_t world, const uint64_t *d_evoff, const uint64_t *d_auxoff, uint4 *ev, uint32_t *aux);
// replay + lanes of the range + their scalars; *ok = false: no fixed point or
// more than 63 slots (the caller takes its fallback)
int wg_lf_replay_lanes(wg_ctx *c, const LfRange &R, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *lane,
                       bool *ok);
int wg_lf_replay_lanes_spec(wg_ctx *c, const LfRange &R, uint64_t nev, const uint4 *ev, const uint32_t *aux, uint32_t *lane,
                            ReplayRun &run);
// a speculative sharded replay's words hold (run: its it, chunk, dc, nw, warm): the context takes them
void wg_lf_replay_spec_commit(wg_ctx *c, const ReplayRun &run, uint32_t max_lane, uint32_t n_slots, uint32_t first_still,
                              uint32_t positions, uint32_t leaks);
int wg_stage_heights(wg_ctx *c);              // wg_rowtop.hip
int wg_heights_run(wg_ctx *c, uint64_t m, uint64_t n, float *out,
                   const int64_t *time = nullptr);   // rows [0,m) of an n-row list (time: the layout's)
// side stream (wg_api.hip): wg_side_fork makes the context's launches go to
// the side stream (ordered after the work queued so far) until wg_side_done;
// wg_side_join orders the main stream after that work (no host wait).
int wg_side_fork(wg_ctx *c);
void wg_side_done(wg_ctx *c);
int wg_side_join(wg_ctx *c);
unsigned wg_event_scope();   // wg_api.hip: the release scope of the engine's stream-order events
// heights of rows [0, m) of the list + zero-band row_top into (h, rt), on the side stream
int wg_side_zero_rowtop(wg_ctx *c, uint64_t m, float *h, float *rt, uint64_t row_lo,
                        const float *band = nullptr,   // banded row_top (build_frame)
                        const float *band_host = nullptr, float *band_dev = nullptr);   // (a host band copied there first)
int wg_rowtop_run(wg_ctx *c, uint64_t n, const float *h, const float *d_band, float *row_top,
                  uint64_t row_lo,    // rows below row_lo: walked, not written
                  uint64_t r_from = 0);   // steps below r_from unchanged since row_top was last written: rescan from there
int wg_stage_rowtop(wg_ctx *c, const float *d_band, uint64_t r_from = 0);   // wg_rowtop.hip
int wg_stage_geometry(wg_ctx *c, const float *d_band); // wg_geom.hip
int wg_geom_summary_sync(wg_ctx *c);                   // read a frame pass's summary when asked for
int wg_geom_spec_items(wg_ctx *c, WgFetch *it);        // speculative full pass: WG_GEOM_SPEC_ITEMS validation words
bool wg_geom_spec_check(wg_ctx *c, const uint64_t *v);
int wg_stage_vertices(wg_ctx *c, uint64_t rb, uint64_t re, int64_t sel);  // wg_vertex.hip
// the full pass's list kernels for rows [r0, r1) (r0 a multiple of WG_SWEEP_CH;
// slice 0 or 1: its own wide-chunk list), and all of them when deferred
int wg_geom_lists(wg_ctx *c, uint64_t r0, uint64_t r1, int slice, hipStream_t s);
int wg_geom_lists_flush(wg_ctx *c);
int wg_vertex_checksum_run(wg_ctx *c, uint64_t *out);  // wg_vertex.hip
// an output buffer of >= 1 GiB chosen from WG_OPT_VTX_PLACE probed candidates
// (wg_vertex.hip); record: the vertex buffer's (wg_vertex_placement_get)
int wg_alloc_placed(wg_ctx *c, DevBuf &buf, size_t bytes, bool record);
int wg_words_checksum(wg_ctx *c, const uint32_t *w, uint64_t nwords, uint64_t *out);  // wg_vertex.hip
void wg_init_height_thresholds(uint32_t *th);  // wg_rowtop.hip
