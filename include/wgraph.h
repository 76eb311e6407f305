/*
 * wgraph.h — C ABI of the MI355X commit-graph render-prep engine.
 *
 * This is the drop-in boundary for whisper-git's `GraphLayout`
 * (/root/reference/src/commit_graph.rs:240-472) and the per-row paint
 * emission behind it (`graph_cell`, commit_graph.rs:803-908).  Each entry
 * point names the reference item it replaces.  Plain C: pointers + sizes,
 * int status codes (0 = OK, negative = error), no exceptions across the ABI.
 *
 * Threading: one wg_ctx per calling thread; a context is not re-entrant.
 * Every call is synchronous with respect to the host unless the caller has
 * installed its own stream with wg_set_stream(), in which case device-resident
 * outputs are ordered on that stream and host copies synchronise it.
 *
 * Ownership: the library owns every device output buffer.  Device pointers
 * returned by wg_device_views() stay valid until the next wg_layout_build(),
 * wg_row_geometry(), wg_emit_vertices() or wg_destroy() on the same context.
 */
#ifndef WGRAPH_H
#define WGRAPH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 2 (from 1): wg_shard_msg.bytes may be WG_SHARD_BYTES_ON_DEVICE (the
 * first build exchange of a multi-rank build always is; ask
 * wg_shard_msg_bytes); wg_shard_pack_slot / wg_shard_slot_heads take caps
 * and strides that are multiples of 16 only; wg_shard_exchange fails when a
 * message header announces more than that rank's sizes[] entry; an
 * exchange step may be sent again (msg.step repeats on every rank alike:
 * WG_OPT_SHARD_SPEC_REPLAY), so transports loop until msg.done. */
#define WGRAPH_ABI_VERSION 2

/* ---- status codes ------------------------------------------------------ */
#define WG_OK             0
#define WG_E_INVALID     -1  /* bad argument (null pointer, size mismatch)        */
#define WG_E_HIP         -2  /* HIP runtime error; see wg_last_error()             */
#define WG_E_NOMEM       -3  /* device allocation failed                           */
#define WG_E_STATE       -4  /* call order: e.g. geometry before a layout build    */
#define WG_E_UNSUPPORTED -5  /* input outside the engine's limits (see message)    */
#define WG_E_NODEVICE    -6  /* no gfx950 device / HIP code object not loadable    */

/* Opaque engine context (one per calling thread). */
typedef struct wg_ctx wg_ctx;

/* ---- residency of caller buffers --------------------------------------- */
#define WG_HOST   0
#define WG_DEVICE 1

/* ---- frozen constants (commit_graph.rs:30-54, 106, 775-780) ------------- */
#define WG_ROW_HEIGHT          28.0f   /* ROW_HEIGHT          :30  */
#define WG_LANE_W              24.0f   /* LANE_W              :33  */
#define WG_LANE_COUNT_VISUAL   6       /* LANE_COUNT_VISUAL   :37  */
#define WG_NODE_Y              14.0f   /* NODE_Y              :43  */
#define WG_MAX_EXTRA_HEIGHT    28.0f   /* MAX_EXTRA_HEIGHT    :47  */
#define WG_TIME_BASE_SECONDS   7200.0  /* TIME_BASE_SECONDS   :51  */
#define WG_TIME_MAX_DELTA      2592000.0 /* TIME_MAX_DELTA_SECONDS :54 */
#define WG_PILLS_BAND_HEIGHT   30.0f   /* PILLS_BAND_HEIGHT   :106 */
#define WG_LINE_WIDTH          2.0f    /* LINE_WIDTH          :775 */
#define WG_NODE_RADIUS         5.0f    /* NODE_RADIUS         :778 */
#define WG_SELECTED_RING_WIDTH 2.5f    /* SELECTED_RING_WIDTH :780 */

/* Colour indices.  The reference carries aetna theme tokens; the engine
 * carries the palette index and resolves RGBA from a caller palette at
 * vertex-emission time.  0..5 = LANE_COLORS[lane % 6] (:59-66),
 * 6 = ORPHAN_COLOR (:70), 7 = tokens::FOREGROUND (selected ring, :898). */
#define WG_COLOR_ORPHAN     6
#define WG_COLOR_FOREGROUND 7
#define WG_PALETTE_SIZE     8

/* commit flags (CommitInfo::is_orphaned / is_synthetic, git/mod.rs:256-269) */
#define WG_FLAG_ORPHAN    0x1u
#define WG_FLAG_SYNTHETIC 0x2u

/* ---- input: the commit list as structure-of-arrays ---------------------
 * Replaces `&[CommitInfo]` (git/mod.rs:246-270) as consumed by
 * GraphLayout::build.  Row order is the caller's (libgit2 revwalk
 * TOPOLOGICAL|TIME, newest first; git/mod.rs:570-596, 761-775).        */
typedef struct wg_commits {
    uint64_t        n_commits;    /* N rows                                   */
    uint64_t        n_parents;    /* E = parent_off[N]                        */
    const uint8_t  *oid;          /* [N][20] commit ids (CommitInfo::id)      */
    const int64_t  *time;         /* [N] seconds (CommitInfo::time)           */
    const uint32_t *parent_off;   /* [N+1] CSR offsets into parent_oid        */
    const uint8_t  *parent_oid;   /* [E][20] parent ids, in parent order      */
    const uint8_t  *flags;        /* [N] WG_FLAG_*; may be NULL (all zero)    */
    int32_t         residency;    /* WG_HOST or WG_DEVICE for all arrays      */
    int32_t         reserved;
} wg_commits;

/* GraphEdge (commit_graph.rs:173-180); colour = palette index */
typedef struct wg_edge {
    uint32_t child_row;
    uint32_t child_lane;
    uint32_t parent_row;
    uint32_t parent_lane;
    uint32_t color;
} wg_edge;

/* Summary of the last wg_layout_build (pub fields of GraphLayout, :244-257) */
typedef struct wg_layout_summary {
    uint64_t n_rows;
    uint64_t n_edges;
    uint32_t max_lane;        /* GraphLayout::max_lane                        */
    uint32_t n_slots;         /* length reached by active_lanes (diagnostic)  */
    float    graph_width;     /* GraphLayout::graph_width                     */
    uint32_t lane_path;       /* 0 = event-compressed fast path, 1 = general  */
    uint64_t row_begin;       /* first row of the rows reported (shard start)  */
} wg_layout_summary;

/* ---- row geometry layout (RowGeometry, commit_graph.rs:208-233) --------
 * Per-row CSR.  vert[] holds, per row and in this order, the
 * full_verticals, top_half_verticals and bottom_half_verticals entries
 * (the z-order graph_cell paints them in, :827-838); each entry packs
 *   bits  0..23 lane, bits 24..25 kind (WG_VERT_*), bits 28..31 colour.
 * curve[] holds CurveSegment records (:186-193) as 8 floats
 *   {p0.x, p0.y, p1.x, p1.y, p2.x, p2.y, p3.x, p3.y}, x in lane units,
 *   y row-local pixels; curve_color[] the matching palette indices.    */
#define WG_VERT_FULL   0u
#define WG_VERT_TOP    1u
#define WG_VERT_BOTTOM 2u
#define WG_VERT_LANE(v)  ((v) & 0xFFFFFFu)
#define WG_VERT_KIND(v)  (((v) >> 24) & 0x3u)
#define WG_VERT_COLOR(v) (((v) >> 28) & 0xFu)

typedef struct wg_curve { float p[8]; } wg_curve;

typedef struct wg_geometry_summary {
    uint64_t n_rows;
    uint64_t n_vert;          /* total vertical entries                       */
    uint64_t n_curve;         /* total curve segments                         */
    float    total_height;    /* row_top_y[N] (content height)                */
    uint32_t scan_path;       /* 0 = transducer scan, 1 = serial fallback     */
} wg_geometry_summary;

/* Host-side destination for wg_copy_geometry (any pointer may be NULL). */
typedef struct wg_geometry_host {
    float    *height;         /* [N]   RowGeometry::height                    */
    float    *node_y;         /* [N]   RowGeometry::node_y                    */
    float    *row_top;        /* [N+1] row_top_y (:329-335 / :374-381)        */
    uint32_t *vert_off;       /* [N+1]                                        */
    uint32_t *vert;           /* [n_vert]                                     */
    uint32_t *curve_off;      /* [N+1]                                        */
    wg_curve *curve;          /* [n_curve]                                    */
    uint8_t  *curve_color;    /* [n_curve]                                    */
} wg_geometry_host;

/* ---- vertex emission (frozen spec WG-TESS-1) -------------
 * SplineVertex (docs/render_engine.md:165-170): 24 bytes.                */
typedef struct wg_vertex { float x, y, r, g, b, a; } wg_vertex;

#define WG_TESS_CURVE_SEGMENTS 16   /* docs/render_engine.md:157          */
#define WG_TESS_NODE_SEGMENTS  24   /* README.md:22                       */
#define WG_VTX_PER_VERTICAL    6
#define WG_VTX_PER_CURVE       (6 * WG_TESS_CURVE_SEGMENTS)   /* 96  */
#define WG_VTX_PER_NODE        (3 * WG_TESS_NODE_SEGMENTS)    /* 72  */
#define WG_VTX_PER_RING        (6 * WG_TESS_NODE_SEGMENTS)    /* 144 */

typedef struct wg_vertex_summary {
    uint64_t row_begin, row_end;
    uint64_t n_vertices;
    uint64_t checksum;        /* order-sensitive 64-bit hash of the buffer   */
} wg_vertex_summary;

/* Device-resident views (valid until the next producing call). */
typedef struct wg_device_views {
    const uint32_t *lane;       /* [N] lane per row (layouts.get(id).lane)    */
    const uint8_t  *color;      /* [N] palette index per row                  */
    const wg_edge  *edges;      /* [n_edges]                                  */
    const float    *height;     /* [N]                                        */
    const float    *node_y;     /* [N]                                        */
    const float    *row_top;    /* [N+1]                                      */
    const uint32_t *vert_off;   /* [N+1]                                      */
    const uint32_t *vert;
    const uint32_t *curve_off;  /* [N+1]                                      */
    const wg_curve *curve;
    const uint8_t  *curve_color;
    const uint64_t *vtx_off;    /* [row_end-row_begin+1] vertex offsets       */
    const wg_vertex *vertices;
} wg_device_views;

/* ---- lifecycle ----------------------------------------------------------- */
/* GraphLayout::new (:261).  device_ordinal < 0 selects the current device. */
wg_ctx     *wg_create(int device_ordinal);
void        wg_destroy(wg_ctx *ctx);
const char *wg_last_error(const wg_ctx *ctx);
int         wg_abi_version(void);
/* Install a caller-owned hipStream_t (NULL = library-owned stream). */
int         wg_set_stream(wg_ctx *ctx, void *hip_stream);
int         wg_synchronize(wg_ctx *ctx);
/* Engine options.  WG_OPT_LANE_PATH: 0 = auto (event-compressed fast path
 * when the commit list is well formed, general walk otherwise), 1 = always
 * the general walk (for testing; results are identical). */
#define WG_OPT_LANE_PATH 1
/* WG_OPT_REPLAY_CHUNK: events per chunk of the parallel lane-event replay
 * (multiple of 64; default 512).  Affects speed only, never results. */
#define WG_OPT_REPLAY_CHUNK 2
/* WG_OPT_SWEEP_REG: edges per 64-row chunk the geometry sweep keeps in
 * registers (0..512, default 512); wider chunks use the LDS sweep.  Affects
 * speed only, never results. */
#define WG_OPT_SWEEP_REG 3
/* WG_OPT_TIMING_EMIT_ONLY: 1 = the stage-timing log (wg_enable_timing) keeps
 * only the vertex-emission stage ("vtx_emit"), so a timed loop carries two
 * events per step instead of two per stage; 0 = every stage (default). */
#define WG_OPT_TIMING_EMIT_ONLY 4
/* WG_OPT_DEFER_VALIDATION: 1 = a speculative wg_layout_build (every build
 * after one that sized the context's buffers) returns without its
 * end-of-build host read: its validation words are read with the vertex total
 * of the next wg_emit_vertices, or by the next call that needs the layout on
 * the host (summaries, copies, device views, glyphs, shards, ...).  A build
 * that did not hold is redone there by the exact stages, followed by the frame
 * pass (wg_row_geometry) and the emission queued after it: results are always
 * identical.  Device-resident commit inputs must stay valid until that call
 * (a redo reads them; device bands are kept by the engine).  Default 0: every
 * build validates before it returns. */
#define WG_OPT_DEFER_VALIDATION 5
/* WG_OPT_REPLAY_WARMUP: the lane-event replay's first iteration starts this
 * many events (multiple of 64, 0..3584) before each chunk, so chunk entry
 * states are mostly right before the second iteration.  Speed only, never
 * results. */
#define WG_OPT_REPLAY_WARMUP 6
/* WG_OPT_SHARD_SPEC_REPLAY: 1 (default) = once a sharded build sized the
 * context, the X3 step replays the global lane events for the blind
 * iteration count without a host read; the replay's convergence and width
 * words are read with the local geometry pass's validation words, and a
 * replay that did not reach its fixed point is redone exactly with that
 * pass (no extra exchange, same results).  0 = the replay is checked before
 * the geometry pass. */
#define WG_OPT_SHARD_SPEC_REPLAY 7
/* WG_OPT_REPLAY_MODE: how the lane events are replayed.  0 (default) = auto:
 * the chunked fixed point; for lists on which it needs many iterations
 * (parents at earlier rows, the Linux shape) the compacted fixed point (the
 * slots leaked by parents at earlier rows struck out, D-state chunks with a
 * long warm-up); for lists on which that still needs more iterations than an
 * exact single-wave pass costs (long-lived lanes) that pass; 1 = always the
 * chunked fixed point; 2 = always the single-wave pass; 3 = always the
 * compacted fixed point.  Speed only, never results. */
#define WG_OPT_REPLAY_MODE 8
/* WG_OPT_SLICE_LISTS: 1 = a speculative full geometry pass whose
 * validation rides on the emission (WG_OPT_DEFER_VALIDATION) leaves its list
 * kernels to the next wg_emit_vertices of the whole list, which builds rows
 * [0, h) first and rows [h, N) beside the emission of the first rows' tiles
 * (h about N / 6), for lists of at least 2^18 rows (2 = of any length past
 * four 64-row chunks); 0 (default: measured slower, the second slice's
 * kernels wait for slots beside the emission) = the lists are built in the
 * geometry pass.  Any other call builds deferred lists whole first.  Speed
 * only, never results. */
#define WG_OPT_SLICE_LISTS 9
/* WG_OPT_DC_WARMUP: the compacted replay's first-iteration warm-up in events
 * (a multiple of 64 in 64..1048576; 0 = auto, the default: 8192, doubled up
 * to 32768 while the fixed point comes late).  Speed only, never results. */
#define WG_OPT_DC_WARMUP 10
/* WG_OPT_JOIN_FUSED: 1 = the id table's place pass rides on the window
 * probe and its settle pass follows on the build's stream; 0 (default) = the
 * table is built on the side stream beside the probe.  Speed only. */
#define WG_OPT_JOIN_FUSED 11
/* WG_OPT_VTX_TILE: vertices per emission workgroup tile: 1024, 2048, 4096,
 * or 0 (default: auto, 2048 once the last emission wrote more than 4e8
 * vertices — its geometry no longer sits in the Infinity Cache — and 4096
 * past 1.6e9).  Speed only. */
#define WG_OPT_VTX_TILE 12
/* WG_OPT_FUSED_READ: 1 (default) = the emission's one host read (the vertex
 * total and a deferred build's validation words) is written to the host by
 * the kernel that computes the total; 0 = a separate read kernel.  Speed
 * only. */
#define WG_OPT_FUSED_READ 13
/* WG_OPT_MATCH_THREADS: threads per 256-row workgroup of the search-match
 * kernel (wg_match_rows): 512 (default, 0) or 256.  Speed only. */
#define WG_OPT_MATCH_THREADS 14
/* WG_OPT_VTX_PLACE: when the vertex buffer grows to 1 GiB or more, this
 * many candidate allocations (1..8, default 4; 0 or 1 = one; fewer when
 * device memory is short) are timed with a store probe and the fastest kept
 * (wg_vertex.hip wg_alloc_placed: the emission's store rate follows the
 * buffer's physical pages).  Setting it frees the vertex buffer (the last
 * emission is dropped; the next one allocates afresh).  Speed only. */
#define WG_OPT_VTX_PLACE 15
int         wg_set_option(wg_ctx *ctx, int option, int64_t value);

/* ---- layout (GraphLayout::build, :265-355) -------------------------------
 * Lane assignment, colours, edge list, default row geometry (bands = 0).  */
int wg_layout_build(wg_ctx *ctx, const wg_commits *commits);
int wg_layout_summary_get(wg_ctx *ctx, wg_layout_summary *out);
/* layouts: lane/colour per row = GraphLayout::get(&commits[row].id) (:357) */
int wg_copy_lanes(wg_ctx *ctx, uint32_t *lane, uint8_t *color);
/* GraphLayout::edges (:248) */
int wg_copy_edges(wg_ctx *ctx, wg_edge *edges);

/* compute_row_heights (:486-507) on the commits of the last build. */
int wg_copy_row_heights(wg_ctx *ctx, float *heights);
/* compute_row_heights(&[CommitInfo]) (:486-507), the free function: heights
 * of any n-row time list (`time`, `heights` both in `residency` memory),
 * independent of the context's layout.  Bit-exact (threshold table). */
int wg_compute_row_heights(wg_ctx *ctx, const int64_t *time, uint64_t n, int32_t residency, float *heights);

/* ---- per-frame geometry (row_geometry_with_bands, :367-399) --------------
 * band == NULL reproduces GraphLayout::row_geometry from build (:322-346);
 * otherwise band[N] (residency as given) is the per-row pills band.      */
int wg_row_geometry(wg_ctx *ctx, const float *band, int32_t band_residency);
/* row_geometry_with_bands(&self, commits, band_heights) (:367-399) with its
 * commits argument: the heights are compute_row_heights(commits) (:372) of
 * the list passed (only n_commits, time and residency are read), the edges and
 * lanes the built layout's.  commits must have the built list's length
 * (WG_E_INVALID otherwise: the engine keeps one geometry row per built row);
 * the built list itself (same times) takes wg_row_geometry's per-frame path. */
int wg_row_geometry_list(wg_ctx *ctx, const wg_commits *commits, const float *band, int32_t band_residency);
/* wg_layout_build then wg_row_geometry(band) — history_view's first frame
 * after a refresh (commit_graph.rs:1419-1421) — in one call: the frame's
 * banded row_top (heights and band only) is computed on the engine's side
 * stream beside the build.  Results identical to the two calls. */
int wg_layout_build_frame(wg_ctx *ctx, const wg_commits *commits, const float *band, int32_t band_residency);
int wg_geometry_summary_get(wg_ctx *ctx, wg_geometry_summary *out);
int wg_copy_geometry(wg_ctx *ctx, const wg_geometry_host *dst);

/* ---- vertex emission (graph_cell, :803-908 + WG-TESS-1) -----------------
 * Rows [row_begin, row_end) of the current geometry; selected_row < 0 for
 * none.  palette = WG_PALETTE_SIZE RGBA float quadruples (host memory).  */
int wg_emit_vertices(wg_ctx *ctx, uint64_t row_begin, uint64_t row_end,
                     int64_t selected_row, const float *palette);
int wg_vertex_summary_get(wg_ctx *ctx, wg_vertex_summary *out);
/* The vertex buffer's last placement (WG_OPT_VTX_PLACE): candidates probed
 * (0: plain allocation), the index kept, and each candidate's store-probe
 * time in ms (probe_ms: 8 floats, may be NULL). */
int wg_vertex_placement_get(wg_ctx *ctx, uint32_t *n_probed, uint32_t *kept, float *probe_ms);
/* Copy vertices [first, first+count) of the last emission to host memory. */
int wg_copy_vertices(wg_ctx *ctx, uint64_t first, uint64_t count, wg_vertex *dst);
/* Per-row vertex offsets (row_end-row_begin+1 entries) to host memory. */
int wg_copy_vertex_offsets(wg_ctx *ctx, uint64_t *dst);

int wg_device_views_get(wg_ctx *ctx, wg_device_views *out);

/* ---- row-sharded multi-GPU build --------------------------
 * One process per GPU.  Every rank holds the WHOLE commit list in device
 * memory; rank `rank` of `world` owns rows [row_begin, row_end) (contiguous
 * shards in rank order covering the list).  The build runs to a few
 * exchange points; at each one the engine exposes this rank's message
 * (wg_shard_msg.bytes long, copied out with wg_shard_copy_msg to device or
 * host memory), the caller all-gathers the messages of every rank — e.g.
 * torch.distributed all_gather over RCCL, each message padded to the
 * largest — and hands the gathered buffer (device memory, rank r's message
 * at r * stride, sizes[r] its length) to wg_shard_exchange, until done = 1.
 * Every rank must make the same sequence of calls.
 *
 * After a sharded build the per-row queries (wg_copy_lanes, _edges,
 * _row_heights, wg_copy_geometry, wg_emit_vertices) cover the own rows
 * only: lanes/heights/geometry have row_end-row_begin entries, edges are
 * those whose child is an own row (global row numbers), vertex emission
 * takes global rows inside the shard.  Results equal the single-GPU build of
 * the whole list restricted to the shard.  Lists the sharded path does not
 * take (duplicate ids, parents at earlier rows, > 63 lane slots) are built
 * whole on every rank instead, with the same results.                     */
typedef struct wg_shard_msg {
    const void *send;         /* engine-owned device buffer (diagnostic)      */
    uint64_t    bytes;        /* length of this rank's message, or
                                 WG_SHARD_BYTES_ON_DEVICE: written by the
                                 engine's kernels (wg_shard_msg_bytes reads it;
                                 wg_shard_pack_slot needs no host copy)        */
    int32_t     done;         /* 1: the call is complete, nothing to exchange */
    int32_t     step;         /* exchange index                               */
} wg_shard_msg;
/* GraphLayout::build (:265-355) of a row shard (+ zero-band geometry). */
int wg_shard_build_begin(wg_ctx *ctx, const wg_commits *commits, int world, int rank,
                         uint64_t row_begin, uint64_t row_end, wg_shard_msg *out);
/* wg_shard_build_begin then wg_shard_geometry_begin(band) in one sharded
 * call (history_view's first frame after a refresh, commit_graph.rs:1419-
 * 1421): the build's own geometry pass takes the bands — one geometry pass
 * fewer per step; the banded row_top runs on the side stream beside the
 * build.  Three exchanges (X1, X2, X3) either way.  band = the whole [N]
 * array; a device band must stay valid until the call is done (done = 1).
 * Results identical to the two calls. */
int wg_shard_build_frame_begin(wg_ctx *ctx, const wg_commits *commits, int world, int rank, uint64_t row_begin,
                               uint64_t row_end, const float *band, int32_t band_residency, wg_shard_msg *out);
/* row_geometry_with_bands (:367-399) of the shard; band = the whole [N]
 * array.  No exchange: the crossing edges' far endpoints (lanes from the
 * build's X3, y from the whole list's row_top) are local; done = 1 on return. */
int wg_shard_geometry_begin(wg_ctx *ctx, const float *band, int32_t band_residency, wg_shard_msg *out);
#define WG_SHARD_BYTES_ON_DEVICE UINT64_MAX
/* Copy this rank's current message (device or host destination). */
int wg_shard_copy_msg(wg_ctx *ctx, void *dst);
/* Exact length of this rank's current message (synchronises the engine's
 * stream when the length is still on the device).  Host transports, which
 * write the slot header themselves, call it when wg_shard_msg.bytes is
 * WG_SHARD_BYTES_ON_DEVICE. */
int wg_shard_msg_bytes(wg_ctx *ctx, uint64_t *out);
/* Write this rank's transport slot into device memory, queued on the
 * engine's stream without a host synchronisation: a 16-byte header (message
 * length as u64, then zeros), then the message when it fits in `cap` bytes
 * (the payload's first 16 bytes are zero for shorter messages).  `slot` is
 * 16-byte aligned and holds 16 + cap bytes; `cap` is a multiple of 16, >= 16
 * (WG_E_INVALID otherwise).  The caller orders its
 * all-gather after the engine's stream (e.g. RCCL on that same stream). */
int wg_shard_pack_slot(wg_ctx *ctx, void *slot, uint64_t cap);
/* Read the heads of all-gathered slots in the engine's stream order: per rank
 * r, out[3r] = the slot's u64 length and out[3r+1..3r+2] = its message's
 * 16-byte header (the `heads` wg_shard_exchange takes).  One small device
 * read the host polls for, instead of a copy + stream synchronisation by the
 * transport.  world <= 21; `gathered` 16-byte aligned; `stride` (= 16 + the
 * slots' cap) a multiple of 16, >= 32 (WG_E_INVALID otherwise).
 * wg_shard_exchange checks every length a message header announces against
 * that rank's entry of `sizes` and fails with WG_E_INVALID on a mismatch. */
int wg_shard_slot_heads(wg_ctx *ctx, const void *gathered, uint64_t stride, int world, uint64_t *out);
/* Deliver the all-gathered messages; runs to the next exchange or the end.
 * Every message starts with a 16-byte header; `heads` (may be NULL) is a host
 * copy of them (rank r's at heads[4r..4r+3]) that saves the engine a device
 * read when the transport already brought them to the host.  Reads of
 * `gathered` may still be queued on the engine's stream when the call
 * returns: keep the buffer until the next wg_shard_copy_msg returns (or
 * wg_synchronize). */
int wg_shard_exchange(wg_ctx *ctx, const void *gathered, uint64_t stride, const uint64_t *sizes,
                      const uint32_t *heads, wg_shard_msg *out);

/* ---- SDF font atlas (legacy TextRenderer atlas, docs/render_engine.md:105-112;
 * frozen spec WG-SDF-1) -------------------------------------
 * A TrueType font's characters [first_char, last_char] are rasterised at
 * em_px pixels per em (4x4 samples per pixel, non-zero winding), shelf-packed
 * into a width x height atlas with `spread` pixels of padding, and turned
 * into an R8 signed distance field by a two-pass separable EDT on the GPU.
 * Two slots: 0 = regular, 1 = bold (the legacy renderer's two instances). */
#define WG_FONT_SLOTS 2
typedef struct wg_atlas_params {
    uint32_t width, height;   /* atlas size (width <= 4096)                  */
    float    em_px;           /* pixels per em at atlas resolution          */
    uint32_t spread;          /* SDF range / cell padding in pixels (1..60) */
    uint32_t first_char, last_char;   /* e.g. 32, 126                        */
} wg_atlas_params;
typedef struct wg_glyph {     /* per character, atlas pixels (y down)       */
    uint32_t codepoint;
    float    advance;         /* advanceWidth * em_px / unitsPerEm          */
    int32_t  bearing_x;       /* bitmap left relative to the pen            */
    int32_t  bearing_top;     /* bitmap top above the baseline              */
    uint32_t w, h;            /* bitmap size (0 for blank glyphs)           */
    uint32_t atlas_x, atlas_y;/* cell origin; cell = (w, h) + 2 * spread    */
} wg_glyph;
typedef struct wg_atlas_info {
    uint32_t width, height, spread, n_glyphs, n_edges;
    uint32_t far_d2;          /* squared distances >= far_d2 mean "farther than 4*spread" */
    float    em_px, ascent, descent, line_gap;
    uint32_t first_char;
} wg_atlas_info;
int wg_font_atlas_build(wg_ctx *ctx, int slot, const uint8_t *ttf, uint64_t ttf_len, const wg_atlas_params *params);
int wg_font_atlas_info(wg_ctx *ctx, int slot, wg_atlas_info *out);
/* Any destination may be NULL: sdf/coverage width*height bytes (coverage =
 * inside samples 0..16), d2_in/d2_out width*height squared distances,
 * glyphs n_glyphs entries. */
int wg_copy_font_atlas(wg_ctx *ctx, int slot, uint8_t *sdf, uint8_t *coverage, uint16_t *d2_in, uint16_t *d2_out,
                       wg_glyph *glyphs);

/* ---- SDF glyph quads (legacy TextRenderer::layout_text, docs/render_engine.md:113-131;
 * frozen spec WG-TEXT-1) ----------------------------------
 * Per row of the current geometry, three runs on one baseline
 * (node_y + baseline_dy, row-local y like the SplineVertex buffers):
 *   short SHA (first 7 hex digits of the id, git/mod.rs:300; none for
 *   synthetic rows) at sha_x; summary (bytes; "(no summary)" when empty,
 *   commit_graph.rs:1003-1007) at summary_x, clipped at summary_max_x;
 *   relative time (format_relative_time(now, time), git/mod.rs:34-49)
 *   right-aligned at time_right_x.
 * Each visible glyph is one quad = 6 TextVertex, pen advanced in f32 in
 * reading order; bytes outside the atlas range draw as '?'.              */
typedef struct wg_text_vertex { float x, y, u, v, r, g, b, a; } wg_text_vertex;
typedef struct wg_text_params {
    int32_t slot;             /* font atlas slot                            */
    float   text_px;          /* font size in pixels                        */
    float   sha_x, summary_x, summary_max_x, time_right_x, baseline_dy;
    int64_t now;              /* unix seconds ("now" of the relative times) */
    float   color_sha[4], color_summary[4], color_time[4];
} wg_text_params;
typedef struct wg_glyph_summary {
    uint64_t row_begin, row_end, n_quads, n_vertices;
    uint64_t checksum;        /* same definition as wg_vertex_summary      */
} wg_glyph_summary;
/* summary_off: [N+1] byte offsets of every row's summary (NULL: all empty);
 * rows [row_begin, row_end) of the current geometry (global numbering).  */
int wg_emit_glyphs(wg_ctx *ctx, uint64_t row_begin, uint64_t row_end, const uint8_t *summary,
                   const uint64_t *summary_off, int32_t residency, const wg_text_params *params);
int wg_glyph_summary_get(wg_ctx *ctx, wg_glyph_summary *out);
int wg_copy_glyph_vertices(wg_ctx *ctx, uint64_t first, uint64_t count, wg_text_vertex *dst);
/* per-row first quad (row_end-row_begin+1 entries) */
int wg_copy_glyph_offsets(wg_ctx *ctx, uint64_t *dst);

/* ---- row order of the commit list -------------------
 * The order GraphLayout::build receives (repo_tab.rs:607-611, 975-980):
 * commit_graph_with_orphans (git/mod.rs:761-775) appends the reflog orphans
 * to the revwalk list and, when there are any, re-sorts everything by time,
 * newest first, with a stable sort; insert_synthetics_sorted (git/mod.rs:
 * 234-242) then inserts each synthetic row, in order, before the first row
 * whose time <= its time (or at the end).  perm[final row] = source row,
 * sources numbered walk rows [0, n_walk), orphans [n_walk, n_walk +
 * n_orphans), synthetics after them.  Times in host or device memory
 * (residency); perm (n_walk + n_orphans + n_syn entries) written to host or
 * device memory (out_residency).  n_syn <= 4096.                          */
int wg_order_rows(wg_ctx *ctx, const int64_t *walk_time, uint64_t n_walk, const int64_t *orphan_time,
                  uint64_t n_orphans, const int64_t *syn_time, uint64_t n_syn, int32_t residency,
                  uint32_t *perm, int32_t out_residency);

/* ---- search-match flags (history_view, commit_graph.rs:1320-1332;
 * commit_matches_query, :1509-1523) ------------------------
 * query = the raw search text (UTF-8); the engine lowers it with Rust's
 * str::to_lowercase semantics (:1326; Unicode tables of wgraph's
 * WG_UNICODE_VERSION) and flags every row r of [row_begin, row_end) of the
 * last build's commit list whose lowered summary or author contains it, whose
 * short id (first 7 hex digits, none for synthetic rows, git/mod.rs:300, 360)
 * contains it, or whose 40-digit hex id starts with it.  An empty query
 * matches every row and turns dimming off.  After a non-empty query,
 * wg_emit_vertices and wg_emit_glyphs draw rows flagged 0 at opacity
 * WG_DIM_ALPHA (:1467, 1482: row_el.opacity(0.3)): every vertex's alpha is
 * multiplied by it (rows outside [row_begin, row_end) are not dimmed; the
 * next layout build clears the flags).
 * Text fields: CSR bytes + [N+1] u64 offsets of the WHOLE list (host or
 * device, per residency); a NULL offset array = that field empty on every
 * row.  match_count (may be NULL) receives the number of flagged rows.     */
#define WG_DIM_ALPHA 0.3f
typedef struct wg_row_text {
    const uint8_t  *summary;      /* CommitInfo::summary bytes, concatenated   */
    const uint64_t *summary_off;  /* [N+1]                                      */
    const uint8_t  *author;       /* CommitInfo::author bytes                   */
    const uint64_t *author_off;   /* [N+1]                                      */
    int32_t         residency;    /* WG_HOST or WG_DEVICE                       */
    int32_t         reserved;
} wg_row_text;
int wg_match_rows(wg_ctx *ctx, const uint8_t *query, uint64_t query_len, uint64_t row_begin, uint64_t row_end,
                  const wg_row_text *text, uint64_t *match_count);
/* flags of the last wg_match_rows: row_end-row_begin bytes (1 = match) */
int wg_copy_match_flags(wg_ctx *ctx, uint8_t *dst);
/* str::to_lowercase of a UTF-8 byte string with the engine's tables (host):
 * writes min(len, cap) bytes to dst (may be NULL) and the full length to
 * *out_len. */
int wg_lower_utf8(const uint8_t *src, uint64_t len, uint8_t *dst, uint64_t cap, uint64_t *out_len);

/* ---- consumer adapter: rasterise the emitted buffers
 * The headless screenshot path (screenshot_mode.rs:101-141) renders the UI
 * into an offscreen image cleared to the theme colour and saves a PNG; the
 * reference's rasteriser (aetna-vulkano) is absent, so the engine freezes
 * WG-RAST-1 (wg_render.hip): rows in order, per row its
 * graph triangles then its glyph quads, one sample per pixel centre,
 * owner-edge rule, flat graph colours, bilinear SDF text coverage, "over"
 * blending in f32 onto the clear colour, RGBA8 output (alpha 255).
 * Row r of the last emissions lands at image y = ((row_top[r] -
 * row_top[top_row]) + origin_y) * scale; graph vertices are shifted by
 * graph_x, glyph vertices keep their x.                                   */
#define WG_RENDER_GRAPH 1
#define WG_RENDER_TEXT  2
typedef struct wg_render_params {
    uint32_t width, height;   /* image size in pixels (<= 16384)            */
    float    scale;           /* pixels per logical px (scale factor)       */
    float    graph_x;         /* x of the graph column (logical px)         */
    float    origin_y;        /* image y of top_row's top (logical px)      */
    uint64_t top_row;         /* global row at origin_y                     */
    float    clear[4];        /* background RGBA (alpha ignored: opaque)     */
    uint32_t layers;          /* WG_RENDER_GRAPH | WG_RENDER_TEXT            */
    uint32_t reserved;
} wg_render_params;
/* RGBA8 image (width * height * 4 bytes) into host or device memory. */
int wg_render(wg_ctx *ctx, const wg_render_params *params, uint8_t *rgba, int32_t out_residency);
/* Write an RGBA8 image as a PNG file (host; stored deflate, no compression). */
int wg_write_png(const char *path, const uint8_t *rgba, uint32_t width, uint32_t height);

/* ---- timing (HIP events on the context's stream) ------------------------ */
#define WG_STAGE_MAX 1024
/* on = 0 disables; on > 0 enables and restarts the stage log (on > 1 also
 * pre-creates that many stage event pairs, so none is created later).      */
int wg_enable_timing(wg_ctx *ctx, int on);
/* Per-stage milliseconds of every stage logged since wg_enable_timing, in
 * launch order (a multi-step run logs each step's stages); names[i] static;
 * names/ms hold WG_STAGE_MAX entries.                                      */
int wg_stage_timings(wg_ctx *ctx, int *n_stages, const char **names, float *ms);

/* ---- diagnostics ------------------------------------------------------------
 * Copies up to n (<= 16) 32-bit engine counters of the last layout build:
 * [0] max_lane, [1] slots, [2] lane-table overflow, [3] fixed-point
 * iterations of the lane-event replay, [4] lane events, [5] build mode
 * (0 single, 1 row-sharded, 2 row-sharded request built whole), [6]
 * speculative builds (one host read per build) on this context, [7] of
 * which the lanes and [8] the geometry were redone by the exact stages
 * (a sharded build's blind global replay redone exactly counts in [7]), [9]
 * sharded builds whose global lane replay ran blind (WG_OPT_SHARD_SPEC_REPLAY),
 * [10] 1 if the last lane replay was the single-wave serial pass
 * (WG_OPT_REPLAY_MODE), [11] emissions that built row-sliced geometry lists
 * (WG_OPT_SLICE_LISTS), [12] the last lane replay's form: 100 + words for the
 * chunked fixed point (101, 104, 116), 200 + words for the serial pass (201,
 * 203, 204, 208, 216; 264 the 16-wave workgroup), 300 + words for the
 * compacted fixed point (301, 302, 304), 0 none (the general walk), [13]
 * the slots the last compacted replay struck out as leaked, [14] its
 * first-iteration warm-up (events). */
int wg_debug_counters(wg_ctx *ctx, uint32_t *out, int n);

#ifdef __cplusplus
}
#endif
#endif /* WGRAPH_H */
