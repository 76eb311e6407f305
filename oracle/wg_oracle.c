/*
 * wg_oracle.c — CPU ORACLE for the commit-graph render-prep path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is a line-by-line restatement of the
 * reference's CPU algorithm in /root/reference/src/commit_graph.rs, used as
 * the checker for the HIP engine (tests/, __graft_entry__.smoke(), and the
 * `cpu_baseline` leg of bench.py).  The product never links or calls it.
 *
 * Pinning: the reference is a Rust crate that cannot be built here (no
 * cargo/rustc, libgit2 or Vulkan), so no reference-produced
 * vectors exist.  The restatement is pinned by (1) the reference's own
 * known-answer tests, ported in tests/test_oracle_kats.py
 * (commit_graph.rs:1593-1742), and (2) a second, independent restatement in
 * oracle/oracle_py.py (numpy float32, written separately) that must agree
 * bit-for-bit on every golden DAG.  Lane indices, edge order and path lists
 * are not covered by any reference test: parity there is "unpinned by
 * reference fixtures" and rests on (2).
 *
 * Numerics: compiled with -O2 -ffp-contract=off -fno-fast-math so every
 * f32 operation rounds as Rust's does (no FMA contraction, SSE f32, IEEE
 * denormals); f32::round == C roundf (half away from zero).
 *
 * The tessellation stage (wgo_emit_vertices) follows the frozen WG-TESS-1
 * spec: the reference tessellator is absent from the
 * snapshot (docs/aetna-port.md:58-63), so that stage is "parity unpinned".
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/wgraph.h"
#include "../include/wgraph_tess.h"
#include "wg_oracle.h"

/* ------------------------------------------------------------------------ */
/* HashMap<Oid, V> with 20-byte keys (std HashMap stand-in, :242, :272-274)  */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint8_t  *keys;    /* cap * 20 */
    int64_t  *vals;    /* cap; value */
    uint8_t  *used;
    uint64_t  cap, mask, len;
} oidmap;

static uint64_t oid_hash(const uint8_t *k) {
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < 20; i++) { h ^= k[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

static int map_init(oidmap *m, uint64_t n) {
    uint64_t cap = 16;
    while (cap < n * 2 + 16) cap <<= 1;
    m->keys = (uint8_t *)malloc(cap * 20);
    m->vals = (int64_t *)malloc(cap * sizeof(int64_t));
    m->used = (uint8_t *)calloc(cap, 1);
    m->cap = cap; m->mask = cap - 1; m->len = 0;
    return (m->keys && m->vals && m->used) ? 0 : -1;
}
static void map_free(oidmap *m) { free(m->keys); free(m->vals); free(m->used); }

/* insert-or-overwrite (HashMap::insert / collect: last write wins) */
static void map_put(oidmap *m, const uint8_t *k, int64_t v) {
    uint64_t i = oid_hash(k) & m->mask;
    while (m->used[i]) {
        if (memcmp(m->keys + i * 20, k, 20) == 0) { m->vals[i] = v; return; }
        i = (i + 1) & m->mask;
    }
    m->used[i] = 1; memcpy(m->keys + i * 20, k, 20); m->vals[i] = v; m->len++;
}
static int map_get(const oidmap *m, const uint8_t *k, int64_t *v) {
    uint64_t i = oid_hash(k) & m->mask;
    while (m->used[i]) {
        if (memcmp(m->keys + i * 20, k, 20) == 0) { if (v) *v = m->vals[i]; return 1; }
        i = (i + 1) & m->mask;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* active_lanes: Vec<Option<Oid>> (:243)                                      */
/* ------------------------------------------------------------------------ */
typedef struct { uint8_t some; uint8_t oid[20]; } slot_t;
typedef struct { slot_t *v; uint64_t len, cap; } lanes_t;

static void lanes_push_none(lanes_t *a) {
    if (a->len == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 16;
        a->v = (slot_t *)realloc(a->v, a->cap * sizeof(slot_t));
    }
    a->v[a->len].some = 0;
    a->len++;
}
static int slot_is(const slot_t *s, const uint8_t *oid) { return s->some && memcmp(s->oid, oid, 20) == 0; }

/* lowest_free_lane (:414-423) */
static uint64_t lowest_free_lane(lanes_t *a) {
    for (uint64_t l = 0; l < a->len; l++) if (!a->v[l].some) return l;
    uint64_t l = a->len;
    lanes_push_none(a);
    return l;
}
/* find_or_assign_lane (:401-412) */
static uint64_t find_or_assign_lane(lanes_t *a, const uint8_t *id) {
    for (uint64_t l = 0; l < a->len; l++) if (slot_is(&a->v[l], id)) return l;
    uint64_t l = lowest_free_lane(a);
    while (a->len <= l) lanes_push_none(a);
    return l;
}

/* ------------------------------------------------------------------------ */
/* Per-row lists of RowGeometry (:208-233)                                   */
/* ------------------------------------------------------------------------ */
typedef struct { uint32_t *v; uint32_t n, cap; } u32vec;
typedef struct { wg_curve *v; uint8_t *c; uint32_t n, cap; } curvevec;
static void u32_push(u32vec *a, uint32_t x) {
    if (a->n == a->cap) { a->cap = a->cap ? a->cap * 2 : 4; a->v = (uint32_t *)realloc(a->v, a->cap * 4); }
    a->v[a->n++] = x;
}
static void curve_push(curvevec *a, const wg_curve *cv, uint8_t color) {
    if (a->n == a->cap) {
        a->cap = a->cap ? a->cap * 2 : 4;
        a->v = (wg_curve *)realloc(a->v, a->cap * sizeof(wg_curve));
        a->c = (uint8_t *)realloc(a->c, a->cap);
    }
    a->v[a->n] = *cv; a->c[a->n] = color; a->n++;
}
typedef struct {
    float height, node_y;
    u32vec full, top, bottom;   /* entries packed lane | color<<28 */
    curvevec curves;
} rowgeom;

/* ------------------------------------------------------------------------ */
/* Cubic (:614-695) — exact f32 operation order                              */
/* ------------------------------------------------------------------------ */
typedef struct { float x, y; } pt;
typedef struct { pt p0, p1, p2, p3; } cubic;

static float y_at(const cubic *c, float t) {            /* :623-629 */
    float s = 1.0f - t;
    return s * s * s * c->p0.y + 3.0f * s * s * t * c->p1.y + 3.0f * s * t * t * c->p2.y + t * t * t * c->p3.y;
}
static float t_at_y(const cubic *c, float target) {     /* :635-654 */
    if (target <= c->p0.y) return 0.0f;
    if (target >= c->p3.y) return 1.0f;
    float lo = 0.0f, hi = 1.0f;
    for (int i = 0; i < 40; i++) {
        float mid = (lo + hi) * 0.5f;
        float y = y_at(c, mid);
        if (y < target) lo = mid; else hi = mid;
    }
    return (lo + hi) * 0.5f;
}
static pt lerp(pt a, pt b, float t) {                   /* :657 */
    pt r; r.x = a.x + (b.x - a.x) * t; r.y = a.y + (b.y - a.y) * t; return r;
}
static void split(const cubic *c, float t, cubic *left, cubic *right) {  /* :656-678 */
    pt q01 = lerp(c->p0, c->p1, t), q12 = lerp(c->p1, c->p2, t), q23 = lerp(c->p2, c->p3, t);
    pt r012 = lerp(q01, q12, t), r123 = lerp(q12, q23, t);
    pt s = lerp(r012, r123, t);
    if (left)  { left->p0 = c->p0; left->p1 = q01; left->p2 = r012; left->p3 = s; }
    if (right) { right->p0 = s; right->p1 = r123; right->p2 = q23; right->p3 = c->p3; }
}
static float clampf_rs(float x, float lo, float hi) {   /* f32::clamp */
    if (x < lo) x = lo;
    if (x > hi) x = hi;
    return x;
}
static cubic subcurve(const cubic *c, float a, float b) {  /* :683-694 */
    if (a <= 0.0f && b >= 1.0f) return *c;
    cubic right, left;
    split(c, clampf_rs(a, 0.0f, 1.0f), NULL, &right);
    if (b >= 1.0f) return right;
    float new_t = clampf_rs((b - a) / (1.0f - a), 0.0f, 1.0f);
    split(&right, new_t, &left, NULL);
    return left;
}

/* exported for the ported known-answer tests (:1593-1622) */
float wgo_cubic_y_at(const float *p8, float t) {
    cubic c = {{p8[0], p8[1]}, {p8[2], p8[3]}, {p8[4], p8[5]}, {p8[6], p8[7]}};
    return y_at(&c, t);
}
float wgo_cubic_t_at_y(const float *p8, float y) {
    cubic c = {{p8[0], p8[1]}, {p8[2], p8[3]}, {p8[4], p8[5]}, {p8[6], p8[7]}};
    return t_at_y(&c, y);
}
void wgo_cubic_subcurve(const float *p8, float a, float b, float *out8) {
    cubic c = {{p8[0], p8[1]}, {p8[2], p8[3]}, {p8[4], p8[5]}, {p8[6], p8[7]}};
    cubic s = subcurve(&c, a, b);
    float o[8] = {s.p0.x, s.p0.y, s.p1.x, s.p1.y, s.p2.x, s.p2.y, s.p3.x, s.p3.y};
    memcpy(out8, o, sizeof(o));
}

/* ------------------------------------------------------------------------ */
/* decompose_edge_into_rows (:525-608)                                        */
/* ------------------------------------------------------------------------ */
static void decompose_edge_into_rows(const wg_edge *edge, const float *row_top_y, rowgeom *rows, uint64_t nrows) {
    if (edge->child_row >= edge->parent_row) return;
    uint32_t color = edge->color;
    if (edge->child_lane == edge->parent_lane) {
        uint32_t e = edge->child_lane | (color << 28);
        if (edge->child_row < nrows) u32_push(&rows[edge->child_row].bottom, e);
        for (uint64_t r = (uint64_t)edge->child_row + 1; r < edge->parent_row; r++)
            if (r < nrows) u32_push(&rows[r].full, e);
        if (edge->parent_row < nrows) u32_push(&rows[edge->parent_row].top, e);
        return;
    }
    float child_node_y = edge->child_row < nrows ? rows[edge->child_row].node_y : WG_NODE_Y;
    float parent_node_y = edge->parent_row < nrows ? rows[edge->parent_row].node_y : WG_NODE_Y;
    float child_y = row_top_y[edge->child_row] + child_node_y;
    float parent_y = row_top_y[edge->parent_row] + parent_node_y;
    float dy = parent_y - child_y;
    cubic curve;
    curve.p0.x = (float)edge->child_lane;  curve.p0.y = child_y;
    curve.p1.x = (float)edge->child_lane;  curve.p1.y = child_y + dy * 0.4f;
    curve.p2.x = (float)edge->parent_lane; curve.p2.y = parent_y - dy * 0.4f;
    curve.p3.x = (float)edge->parent_lane; curve.p3.y = parent_y;
    for (uint64_t row = edge->child_row; row <= edge->parent_row; row++) {
        float row_top = row_top_y[row];
        float row_bot = row_top_y[row + 1];
        float strip_top = (row == edge->child_row) ? child_y : row_top;
        float strip_bot = (row == edge->parent_row) ? parent_y : row_bot;
        if (strip_bot - strip_top < 1e-4f) continue;
        float t_a = (row == edge->child_row) ? 0.0f : t_at_y(&curve, strip_top);
        float t_b = (row == edge->parent_row) ? 1.0f : t_at_y(&curve, strip_bot);
        cubic sub = subcurve(&curve, t_a, t_b);
        if (row < nrows) {
            wg_curve cv = {{sub.p0.x, sub.p0.y - row_top, sub.p1.x, sub.p1.y - row_top,
                            sub.p2.x, sub.p2.y - row_top, sub.p3.x, sub.p3.y - row_top}};
            curve_push(&rows[row].curves, &cv, (uint8_t)color);
        }
    }
}

/* ------------------------------------------------------------------------ */
/* compute_row_heights (:486-507)                                             */
/* ------------------------------------------------------------------------ */
void wgo_compute_row_heights(uint64_t n, const int64_t *time, float *heights) {
    if (n == 0) return;
    double log_max = log(1.0 + WG_TIME_MAX_DELTA / WG_TIME_BASE_SECONDS);
    for (uint64_t i = 0; i < n; i++) {
        float h;
        if (i + 1 < n) {
            int64_t d = time[i] - time[i + 1];            /* i64 wrapping sub */
            uint64_t ad = d < 0 ? (uint64_t)0 - (uint64_t)d : (uint64_t)d;  /* unsigned_abs */
            double delta = (double)ad;
            double clamped = delta < WG_TIME_MAX_DELTA ? delta : WG_TIME_MAX_DELTA;  /* f64::min */
            double ratio = log(1.0 + clamped / WG_TIME_BASE_SECONDS) / log_max;
            h = WG_ROW_HEIGHT + WG_MAX_EXTRA_HEIGHT * (float)ratio;
        } else {
            h = WG_ROW_HEIGHT;
        }
        heights[i] = roundf(h);
    }
}

/* ------------------------------------------------------------------------ */
/* Outputs                                                                    */
/* ------------------------------------------------------------------------ */
/* wgo_geometry / wgo_layout: oracle/wg_oracle.h */

static int flatten(rowgeom *rows, uint64_t n, const float *row_top_y, wgo_geometry *g) {
    memset(g, 0, sizeof(*g));
    g->n = n;
    g->height = (float *)malloc((n + 1) * sizeof(float));
    g->node_y = (float *)malloc((n + 1) * sizeof(float));
    g->row_top = (float *)malloc((n + 1) * sizeof(float));
    g->vert_off = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    g->curve_off = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    if (!g->height || !g->node_y || !g->row_top || !g->vert_off || !g->curve_off) return -1;
    uint64_t nv = 0, nc = 0;
    for (uint64_t r = 0; r < n; r++) { nv += rows[r].full.n + rows[r].top.n + rows[r].bottom.n; nc += rows[r].curves.n; }
    g->vert = (uint32_t *)malloc((nv + 1) * sizeof(uint32_t));
    g->curve = (wg_curve *)malloc((nc + 1) * sizeof(wg_curve));
    g->curve_color = (uint8_t *)malloc(nc + 1);
    if (!g->vert || !g->curve || !g->curve_color) return -1;
    uint64_t v = 0, c = 0;
    for (uint64_t r = 0; r < n; r++) {
        g->height[r] = rows[r].height; g->node_y[r] = rows[r].node_y; g->row_top[r] = row_top_y[r];
        g->vert_off[r] = (uint32_t)v; g->curve_off[r] = (uint32_t)c;
        for (uint32_t k = 0; k < rows[r].full.n; k++)   g->vert[v++] = rows[r].full.v[k] | (WG_VERT_FULL << 24);
        for (uint32_t k = 0; k < rows[r].top.n; k++)    g->vert[v++] = rows[r].top.v[k] | (WG_VERT_TOP << 24);
        for (uint32_t k = 0; k < rows[r].bottom.n; k++) g->vert[v++] = rows[r].bottom.v[k] | (WG_VERT_BOTTOM << 24);
        for (uint32_t k = 0; k < rows[r].curves.n; k++) { g->curve[c] = rows[r].curves.v[k]; g->curve_color[c] = rows[r].curves.c[k]; c++; }
        free(rows[r].full.v); free(rows[r].top.v); free(rows[r].bottom.v);
        free(rows[r].curves.v); free(rows[r].curves.c);
    }
    g->row_top[n] = row_top_y[n];
    g->vert_off[n] = (uint32_t)v; g->curve_off[n] = (uint32_t)c;
    g->n_vert = v; g->n_curve = c;
    return 0;
}

/* decompose_edge_into_rows over RowGeometry::default() rows (height
 * ROW_HEIGHT, node_y NODE_Y, :218-230) and the caller's row_top_y: the
 * reference's decomposition known-answer tests call it this way
 * (:1631-1702).  Exported for those tests only. */
int wgo_decompose_edges(const wg_edge *edges, uint64_t ne, const float *row_top_y, uint64_t nrows, wgo_geometry *out) {
    rowgeom *rows = (rowgeom *)calloc(nrows ? nrows : 1, sizeof(rowgeom));
    if (!rows) return -1;
    for (uint64_t r = 0; r < nrows; r++) { rows[r].height = WG_ROW_HEIGHT; rows[r].node_y = WG_NODE_Y; }
    for (uint64_t k = 0; k < ne; k++) decompose_edge_into_rows(&edges[k], row_top_y, rows, nrows);
    int rc = flatten(rows, nrows, row_top_y, out);
    free(rows);
    return rc;
}

void wgo_geometry_free(wgo_geometry *g) {
    if (!g) return;
    free(g->height); free(g->node_y); free(g->row_top); free(g->vert_off); free(g->vert);
    free(g->curve_off); free(g->curve); free(g->curve_color);
    memset(g, 0, sizeof(*g));
}
void wgo_layout_free(wgo_layout *L) {
    if (!L) return;
    free(L->lane); free(L->color); free(L->edges); free(L->heights);
    wgo_geometry_free(&L->geom);
    memset(L, 0, sizeof(*L));
}

/* ------------------------------------------------------------------------ */
/* GraphLayout::build (:265-355)                                              */
/* ------------------------------------------------------------------------ */
int wgo_layout_build(const wg_commits *in, wgo_layout *out) {
    memset(out, 0, sizeof(*out));
    const uint64_t n = in->n_commits;
    out->n = n;
    oidmap commit_set, row_by_oid, layouts;                 /* :272-274, :242 */
    if (map_init(&commit_set, n) || map_init(&row_by_oid, n) || map_init(&layouts, n)) return -1;
    for (uint64_t i = 0; i < n; i++) map_put(&commit_set, in->oid + i * 20, 0);
    for (uint64_t i = 0; i < n; i++) map_put(&row_by_oid, in->oid + i * 20, (int64_t)i);

    lanes_t al = {0};
    uint64_t max_lane = 0;
    for (uint64_t i = 0; i < n; i++) {                    /* :276-295 */
        const uint8_t *id = in->oid + i * 20;
        uint64_t lane = find_or_assign_lane(&al, id);
        int orphan = in->flags ? (in->flags[i] & WG_FLAG_ORPHAN) : 0;
        uint32_t color = orphan ? WG_COLOR_ORPHAN : (uint32_t)(lane % 6);
        map_put(&layouts, id, (int64_t)((lane << 8) | color));
        for (uint64_t l = 0; l < al.len; l++)              /* :287-291 */
            if (l != lane && slot_is(&al.v[l], id)) al.v[l].some = 0;
        /* update_lanes_for_parents (:425-460) */
        while (al.len <= lane) lanes_push_none(&al);
        uint32_t p0 = in->parent_off[i], p1 = in->parent_off[i + 1];
        if (p0 == p1) {
            al.v[lane].some = 0;
        } else {
            const uint8_t *fp = in->parent_oid + (uint64_t)p0 * 20;
            if (map_get(&commit_set, fp, NULL)) { al.v[lane].some = 1; memcpy(al.v[lane].oid, fp, 20); }
            else al.v[lane].some = 0;
            for (uint32_t k = p0 + 1; k < p1; k++) {
                const uint8_t *pid = in->parent_oid + (uint64_t)k * 20;
                if (!map_get(&commit_set, pid, NULL)) continue;
                int present = 0;
                for (uint64_t l = 0; l < al.len; l++) if (slot_is(&al.v[l], pid)) { present = 1; break; }
                if (present) continue;
                uint64_t nl = lowest_free_lane(&al);
                while (al.len <= nl) lanes_push_none(&al);
                al.v[nl].some = 1; memcpy(al.v[nl].oid, pid, 20);
            }
        }
        /* update_peak (:462-471) */
        for (uint64_t l = al.len; l-- > 0;) {
            if (al.v[l].some) { if (l > max_lane) max_lane = l; break; }
        }
    }
    out->max_lane = (uint32_t)max_lane;
    out->n_slots = (uint32_t)al.len;
    free(al.v);

    /* layouts as seen per row (history_view :1363-1367) */
    out->lane = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    out->color = (uint8_t *)malloc(n + 1);
    for (uint64_t i = 0; i < n; i++) {
        int64_t v = 0;
        map_get(&layouts, in->oid + i * 20, &v);
        out->lane[i] = (uint32_t)(v >> 8); out->color[i] = (uint8_t)(v & 0xFF);
    }

    /* edge list (:301-320) */
    uint64_t cap = (uint64_t)in->parent_off[n] + 1, ne = 0;
    out->edges = (wg_edge *)malloc(cap * sizeof(wg_edge));
    for (uint64_t i = 0; i < n; i++) {
        int64_t cl;
        if (!map_get(&layouts, in->oid + i * 20, &cl)) continue;
        for (uint32_t k = in->parent_off[i]; k < in->parent_off[i + 1]; k++) {
            const uint8_t *pid = in->parent_oid + (uint64_t)k * 20;
            int64_t prow, pl;
            if (!map_get(&row_by_oid, pid, &prow)) continue;
            if (!map_get(&layouts, pid, &pl)) continue;
            wg_edge e = {(uint32_t)i, (uint32_t)(cl >> 8), (uint32_t)prow, (uint32_t)(pl >> 8), (uint32_t)(cl & 0xFF)};
            out->edges[ne++] = e;
        }
    }
    out->n_edges = ne;

    /* heights, row_top_y, default geometry, decomposition (:326-346) */
    out->heights = (float *)malloc((n + 1) * sizeof(float));
    wgo_compute_row_heights(n, in->time, out->heights);
    float *row_top_y = (float *)malloc((n + 1) * sizeof(float));
    float acc = 0.0f;
    for (uint64_t i = 0; i < n; i++) { row_top_y[i] = acc; acc += out->heights[i]; }
    row_top_y[n] = acc;
    rowgeom *rows = (rowgeom *)calloc(n + 1, sizeof(rowgeom));
    for (uint64_t i = 0; i < n; i++) { rows[i].height = out->heights[i]; rows[i].node_y = WG_NODE_Y; }
    for (uint64_t k = 0; k < ne; k++) decompose_edge_into_rows(&out->edges[k], row_top_y, rows, n);
    int rc = flatten(rows, n, row_top_y, &out->geom);
    free(rows); free(row_top_y);

    /* graph_width (:353-354) */
    uint64_t vis = (uint64_t)out->max_lane + 1;
    if (vis > WG_LANE_COUNT_VISUAL) vis = WG_LANE_COUNT_VISUAL;
    float gw = (float)vis * WG_LANE_W;
    out->graph_width = gw > WG_LANE_W ? gw : WG_LANE_W;

    map_free(&commit_set); map_free(&row_by_oid); map_free(&layouts);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* row_geometry_with_bands (:367-399)                                         */
/* ------------------------------------------------------------------------ */
int wgo_row_geometry(const wgo_layout *L, const int64_t *time, const float *band, wgo_geometry *out) {
    const uint64_t n = L->n;
    float *heights = (float *)malloc((n + 1) * sizeof(float));
    wgo_compute_row_heights(n, time, heights);
    float *row_top_y = (float *)malloc((n + 1) * sizeof(float));
    float acc = 0.0f;
    for (uint64_t i = 0; i < n; i++) {
        float b = band ? band[i] : 0.0f;
        row_top_y[i] = acc;
        acc += heights[i] + b;
    }
    row_top_y[n] = acc;
    rowgeom *rows = (rowgeom *)calloc(n + 1, sizeof(rowgeom));
    for (uint64_t i = 0; i < n; i++) {
        float b = band ? band[i] : 0.0f;
        rows[i].height = roundf(heights[i] + b);
        rows[i].node_y = roundf(b + WG_NODE_Y);
    }
    for (uint64_t k = 0; k < L->n_edges; k++) decompose_edge_into_rows(&L->edges[k], row_top_y, rows, n);
    int rc = flatten(rows, n, row_top_y, out);
    free(rows); free(row_top_y); free(heights);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* graph_cell (:803-908) + WG-TESS-1 tessellation                             */
/* ------------------------------------------------------------------------ */
static const float UC_COS[25] = WG_UNIT_CIRCLE_COS_INIT;
static const float UC_SIN[25] = WG_UNIT_CIRCLE_SIN_INIT;

static uint64_t visible_lanes_of(float graph_width) {       /* :787, :846 */
    float q = roundf(graph_width / WG_LANE_W);
    uint64_t v = q <= 0.0f ? 0 : (uint64_t)q;               /* `as usize` saturates */
    return v > 1 ? v : 1;
}
static float lane_center_x(uint64_t lane, float graph_width) {   /* :786-790 */
    uint64_t vis = visible_lanes_of(graph_width);
    uint64_t visual = lane < vis - 1 ? lane : vis - 1;
    return (float)visual * WG_LANE_W + WG_LANE_W * 0.5f;
}

typedef struct { wg_vertex *v; uint64_t n, cap; } vtxbuf;
static void vput(vtxbuf *b, float x, float y, const float *rgba) {
    if (b->n == b->cap) { b->cap = b->cap ? b->cap * 2 : 1024; b->v = (wg_vertex *)realloc(b->v, b->cap * sizeof(wg_vertex)); }
    wg_vertex *o = &b->v[b->n++];
    o->x = x; o->y = y; o->r = rgba[0]; o->g = rgba[1]; o->b = rgba[2]; o->a = rgba[3];
}

static void emit_vertical(vtxbuf *b, float x, float y0, float y1, const float *rgba) {
    const float hw = WG_LINE_WIDTH * 0.5f;
    float xl = x - hw, xr = x + hw;
    vput(b, xl, y0, rgba); vput(b, xr, y0, rgba); vput(b, xl, y1, rgba);
    vput(b, xr, y0, rgba); vput(b, xr, y1, rgba); vput(b, xl, y1, rgba);
}

static void emit_curve(vtxbuf *b, const float *X, const float *Y, const float *rgba) {
    const float hw = WG_LINE_WIDTH * 0.5f;
    float Lx[17], Ly[17], Rx[17], Ry[17];
    for (int j = 0; j <= 16; j++) {
        float t = (float)j * WG_TESS_DT;
        float s = 1.0f - t;
        float px = s * s * s * X[0] + 3.0f * s * s * t * X[1] + 3.0f * s * t * t * X[2] + t * t * t * X[3];
        float py = s * s * s * Y[0] + 3.0f * s * s * t * Y[1] + 3.0f * s * t * t * Y[2] + t * t * t * Y[3];
        float dx = 3.0f * s * s * (X[1] - X[0]) + 6.0f * s * t * (X[2] - X[1]) + 3.0f * t * t * (X[3] - X[2]);
        float dy = 3.0f * s * s * (Y[1] - Y[0]) + 6.0f * s * t * (Y[2] - Y[1]) + 3.0f * t * t * (Y[3] - Y[2]);
        float len = sqrtf(dx * dx + dy * dy);
        float nx, ny;
        if (len > 0.0f) { nx = -dy / len; ny = dx / len; } else { nx = 1.0f; ny = 0.0f; }
        Lx[j] = px + hw * nx; Ly[j] = py + hw * ny;
        Rx[j] = px - hw * nx; Ry[j] = py - hw * ny;
    }
    for (int j = 0; j < 16; j++) {
        vput(b, Lx[j], Ly[j], rgba);         vput(b, Rx[j], Ry[j], rgba);         vput(b, Lx[j + 1], Ly[j + 1], rgba);
        vput(b, Rx[j], Ry[j], rgba);         vput(b, Rx[j + 1], Ry[j + 1], rgba); vput(b, Lx[j + 1], Ly[j + 1], rgba);
    }
}

static void emit_node(vtxbuf *b, float cx, float cy, const float *rgba) {
    const float r = WG_NODE_RADIUS;
    for (int j = 0; j < 24; j++) {
        vput(b, cx, cy, rgba);
        vput(b, cx + r * UC_COS[j], cy + r * UC_SIN[j], rgba);
        vput(b, cx + r * UC_COS[j + 1], cy + r * UC_SIN[j + 1], rgba);
    }
}

static void emit_ring(vtxbuf *b, float cx, float cy, const float *rgba) {
    const float ri = WG_NODE_RADIUS - WG_SELECTED_RING_WIDTH * 0.5f;
    const float ro = WG_NODE_RADIUS + WG_SELECTED_RING_WIDTH * 0.5f;
    for (int j = 0; j < 24; j++) {
        float ox0 = cx + ro * UC_COS[j], oy0 = cy + ro * UC_SIN[j];
        float ix0 = cx + ri * UC_COS[j], iy0 = cy + ri * UC_SIN[j];
        float ox1 = cx + ro * UC_COS[j + 1], oy1 = cy + ro * UC_SIN[j + 1];
        float ix1 = cx + ri * UC_COS[j + 1], iy1 = cy + ri * UC_SIN[j + 1];
        vput(b, ox0, oy0, rgba); vput(b, ix0, iy0, rgba); vput(b, ox1, oy1, rgba);
        vput(b, ix0, iy0, rgba); vput(b, ix1, iy1, rgba); vput(b, ox1, oy1, rgba);
    }
}

/* Emit rows [r0, r1).  node lane/colour per row come from L (layouts[i]).
 * *out_v / *out_off are malloc'd; off has (r1-r0+1) entries.             */
int wgo_emit_vertices(const wgo_layout *L, const wgo_geometry *g, uint64_t r0, uint64_t r1,
                      int64_t selected, const float *palette, wg_vertex **out_v, uint64_t **out_off,
                      uint64_t *out_n) {
    if (r1 > g->n || r0 > r1) return -1;
    vtxbuf b = {0};
    uint64_t *off = (uint64_t *)malloc((r1 - r0 + 1) * sizeof(uint64_t));
    const float gw = L->graph_width;
    const uint64_t vis = visible_lanes_of(gw);
    for (uint64_t r = r0; r < r1; r++) {
        off[r - r0] = b.n;
        float h = g->height[r], node_y = g->node_y[r];
        for (uint32_t k = g->vert_off[r]; k < g->vert_off[r + 1]; k++) {
            uint32_t e = g->vert[k];
            float x = lane_center_x(WG_VERT_LANE(e), gw);
            const float *rgba = palette + 4 * WG_VERT_COLOR(e);
            switch (WG_VERT_KIND(e)) {
            case WG_VERT_FULL:   emit_vertical(&b, x, 0.0f, h, rgba); break;
            case WG_VERT_TOP:    emit_vertical(&b, x, 0.0f, node_y, rgba); break;
            default:             emit_vertical(&b, x, node_y, h, rgba); break;
            }
        }
        for (uint32_t k = g->curve_off[r]; k < g->curve_off[r + 1]; k++) {
            const float *p = g->curve[k].p;
            float X[4], Y[4];
            for (int q = 0; q < 4; q++) {                      /* to_x (:847-850) */
                float cl = clampf_rs(p[2 * q], 0.0f, (float)(vis - 1));
                X[q] = cl * WG_LANE_W + WG_LANE_W * 0.5f;
                Y[q] = p[2 * q + 1];
            }
            emit_curve(&b, X, Y, palette + 4 * g->curve_color[k]);
        }
        float cx = lane_center_x(L->lane[r], gw);
        emit_node(&b, cx, node_y, palette + 4 * L->color[r]);
        if (selected >= 0 && (uint64_t)selected == r) emit_ring(&b, cx, node_y, palette + 4 * WG_COLOR_FOREGROUND);
    }
    off[r1 - r0] = b.n;
    *out_v = b.v; *out_off = off; *out_n = b.n;
    return 0;
}

void wgo_free(void *p) { free(p); }

/* Order-sensitive 64-bit checksum of a vertex buffer (shared definition
 * with the engine's on-device checksum).                   */
uint64_t wgo_vertex_checksum_at(const wg_vertex *v, uint64_t n, uint64_t first_vertex) {
    /* the sum over words is additive: a buffer checksummed in pieces, each
     * piece at its position (first_vertex) in the whole buffer            */
    const uint32_t *w = (const uint32_t *)v;
    uint64_t acc = 0;
    for (uint64_t j = 0; j < n * 6; j++) {
        const uint64_t i = first_vertex * 6 + j;
        uint64_t x = ((uint64_t)w[j] << 32) ^ (i * 0x9E3779B97F4A7C15ull);
        x ^= x >> 33; x *= 0xFF51AFD7ED558CCDull; x ^= x >> 33; x *= 0xC4CEB9FE1A85EC53ull; x ^= x >> 33;
        acc += x;
    }
    return acc;
}

uint64_t wgo_vertex_checksum(const wg_vertex *v, uint64_t n) { return wgo_vertex_checksum_at(v, n, 0); }
