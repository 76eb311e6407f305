/*
 * cpu_mt.c — the multi-threaded CPU BASELINE of the render-prep path.
 *
 * TEST / BASELINE INFRASTRUCTURE ONLY: bench.py's `cpu_baseline_threads` leg
 * and its bit-exactness test (tests/test_cpu_mt.py) use it; the product never
 * links or calls it.  It computes what the single-thread oracle (wg_oracle.c)
 * computes — GraphLayout::build (commit_graph.rs:265-355),
 * row_geometry_with_bands (:367-399) and graph_cell emission (:803-908) with
 * the WG-TESS-1 tessellation — bit for bit, on all the
 * threads OpenMP is given, the way a tuned CPU port of the reference would:
 *
 *   - id lookups: one concurrent open-addressing table of row indices
 *     (last row wins, HashMap::insert :272-274, :242), filled and probed in
 *     parallel; parents resolved to canonical rows once, in parallel;
 *   - the greedy lane walk (:276-295, :401-471): sequential, as the
 *     reference's semantics require, over int32 slots holding canonical rows
 *     instead of 20-byte ids (same equalities, auto-vectorised scans);
 *   - edges (:301-320): per-row counts, a prefix, a parallel fill;
 *   - heights (:486-507) in parallel; row_top_y (:329-335, :374-381): the
 *     sequential f32 prefix;
 *   - decomposition (:525-608): each thread owns a range of rows, walks the
 *     edges in edge order and keeps the pieces that land in its rows (count
 *     pass, prefix, write pass), so every row's lists are in edge order as
 *     in the sequential loop;
 *   - emission: every row's vertex count is fixed by its lists (6 per
 *     vertical, 96 per curve, 72 per node, 144 for the ring), so offsets are
 *     a prefix and the rows are written in parallel.
 *
 * Numerics: the same f32 expressions as wg_oracle.c, compiled with the same
 * flags (-ffp-contract=off -fno-fast-math), so outputs match bit for bit.
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/wgraph.h"
#include "../include/wgraph_tess.h"
#include "wg_oracle.h"

static double now_ms(void) { return omp_get_wtime() * 1e3; }
static double g_phase_ms[8];

/* phase times of the last calls (ms): 0 id table, 1 lane walk, 2 edges,
 * 3 heights + row_top, 4 decomposition (build), 5 banded geometry, 6 emission */
void wgm_phase_ms(double *out8) { memcpy(out8, g_phase_ms, sizeof(g_phase_ms)); }

/* ------------------------------------------------------------------------ */
/* Concurrent id table: slot = row + 1 (0 empty); equal ids keep the last row */
/* ------------------------------------------------------------------------ */
static uint64_t id_hash(const uint8_t *k) {
    uint64_t a, b;
    uint32_t c;
    memcpy(&a, k, 8); memcpy(&b, k + 8, 8); memcpy(&c, k + 16, 4);
    uint64_t h = (a ^ (b * 0x9E3779B97F4A7C15ull) ^ ((uint64_t)c << 17)) * 0xFF51AFD7ED558CCDull;
    return h ^ (h >> 31);
}

static void tab_insert(uint32_t *tab, uint64_t mask, const uint8_t *oid, uint32_t row) {
    const uint8_t *k = oid + (uint64_t)row * 20;
    uint64_t h = id_hash(k) & mask;
    for (;;) {
        uint32_t cur = __atomic_load_n(&tab[h], __ATOMIC_ACQUIRE);
        if (cur == 0) {
            if (__atomic_compare_exchange_n(&tab[h], &cur, row + 1, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) return;
            continue;   /* taken meanwhile: look at what is there */
        }
        if (memcmp(oid + (uint64_t)(cur - 1) * 20, k, 20) == 0) {
            while (cur < row + 1 &&
                   !__atomic_compare_exchange_n(&tab[h], &cur, row + 1, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
            }
            return;
        }
        h = (h + 1) & mask;
    }
}

static int64_t tab_find(const uint32_t *tab, uint64_t mask, const uint8_t *oid, const uint8_t *k) {
    uint64_t h = id_hash(k) & mask;
    for (;;) {
        uint32_t cur = tab[h];
        if (cur == 0) return -1;
        if (memcmp(oid + (uint64_t)(cur - 1) * 20, k, 20) == 0) return (int64_t)cur - 1;
        h = (h + 1) & mask;
    }
}

/* ------------------------------------------------------------------------ */
/* Cubic (:614-695), the same operation order as wg_oracle.c                 */
/* ------------------------------------------------------------------------ */
typedef struct { float x, y; } pt;
typedef struct { pt p0, p1, p2, p3; } cubic;

static float y_at(const cubic *c, float t) {
    float s = 1.0f - t;
    return s * s * s * c->p0.y + 3.0f * s * s * t * c->p1.y + 3.0f * s * t * t * c->p2.y + t * t * t * c->p3.y;
}
static float t_at_y(const cubic *c, float target) {
    if (target <= c->p0.y) return 0.0f;
    if (target >= c->p3.y) return 1.0f;
    float lo = 0.0f, hi = 1.0f;
    for (int i = 0; i < 40; i++) {
        float mid = (lo + hi) * 0.5f;
        if (y_at(c, mid) < target) lo = mid; else hi = mid;
    }
    return (lo + hi) * 0.5f;
}
static pt lerp(pt a, pt b, float t) { pt r; r.x = a.x + (b.x - a.x) * t; r.y = a.y + (b.y - a.y) * t; return r; }
static void split(const cubic *c, float t, cubic *left, cubic *right) {
    pt q01 = lerp(c->p0, c->p1, t), q12 = lerp(c->p1, c->p2, t), q23 = lerp(c->p2, c->p3, t);
    pt r012 = lerp(q01, q12, t), r123 = lerp(q12, q23, t);
    pt s = lerp(r012, r123, t);
    if (left)  { left->p0 = c->p0; left->p1 = q01; left->p2 = r012; left->p3 = s; }
    if (right) { right->p0 = s; right->p1 = r123; right->p2 = q23; right->p3 = c->p3; }
}
static float clampf_rs(float x, float lo, float hi) { if (x < lo) x = lo; if (x > hi) x = hi; return x; }
static cubic subcurve(const cubic *c, float a, float b) {
    if (a <= 0.0f && b >= 1.0f) return *c;
    cubic right, left;
    split(c, clampf_rs(a, 0.0f, 1.0f), NULL, &right);
    if (b >= 1.0f) return right;
    split(&right, clampf_rs((b - a) / (1.0f - a), 0.0f, 1.0f), &left, NULL);
    return left;
}

/* ------------------------------------------------------------------------ */
/* Heights (:486-507)                                                         */
/* ------------------------------------------------------------------------ */
static void heights_mt(uint64_t n, const int64_t *time, float *h, int threads) {
    const double log_max = log(1.0 + WG_TIME_MAX_DELTA / WG_TIME_BASE_SECONDS);
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        float v;
        if ((uint64_t)i + 1 < n) {
            int64_t d = time[i] - time[i + 1];
            uint64_t ad = d < 0 ? (uint64_t)0 - (uint64_t)d : (uint64_t)d;
            double delta = (double)ad;
            double clamped = delta < WG_TIME_MAX_DELTA ? delta : WG_TIME_MAX_DELTA;
            double ratio = log(1.0 + clamped / WG_TIME_BASE_SECONDS) / log_max;
            v = WG_ROW_HEIGHT + WG_MAX_EXTRA_HEIGHT * (float)ratio;
        } else {
            v = WG_ROW_HEIGHT;
        }
        h[i] = roundf(v);
    }
}

/* exclusive prefix of cnt[0..n) into off[0..n], in parallel (two passes) */
static uint64_t prefix_u32(const uint32_t *cnt, uint32_t *off, uint64_t n, int threads) {
    uint64_t part[1024];
    int T = threads > 1023 ? 1023 : threads;
#pragma omp parallel num_threads(T)
    {
        int t = omp_get_thread_num(), nt = omp_get_num_threads();
        uint64_t a = n * t / nt, b = n * (t + 1) / nt, s = 0;
        for (uint64_t i = a; i < b; i++) s += cnt[i];
        part[t + 1] = s;
#pragma omp barrier
#pragma omp single
        {
            part[0] = 0;
            for (int k = 1; k <= nt; k++) part[k] += part[k - 1];
        }
        uint64_t acc = part[t];
        for (uint64_t i = a; i < b; i++) { off[i] = (uint32_t)acc; acc += cnt[i]; }
    }
    uint64_t s = n ? (uint64_t)off[n - 1] + cnt[n - 1] : 0;
    off[n] = (uint32_t)s;
    return s;
}

/* ------------------------------------------------------------------------ */
/* Decomposition (:525-608) over owned row ranges, edges in edge order        */
/* ------------------------------------------------------------------------ */
typedef struct {
    const wg_edge *edges;
    uint64_t ne, n;
    const float *row_top, *node_y;
} decomp_in;

/* Visit the pieces edge k leaves in rows [R0, R1): kind 0 full, 1 top,
 * 2 bottom (entry = lane | colour << 28), 3 curve.  write == 0: count into
 * cnt[4 * (row - R0) + kind]; else write at cur[...] (post-incremented). */
static void decomp_edge(const decomp_in *D, const wg_edge *e, uint64_t R0, uint64_t R1, uint32_t *cnt, int write,
                        uint32_t *vert, wg_curve *curve, uint8_t *curve_color) {
    if (e->child_row >= e->parent_row) return;
    if (e->parent_row < R0 || e->child_row >= R1) return;
    const uint32_t color = e->color;
    if (e->child_lane == e->parent_lane) {
        const uint32_t v = e->child_lane | (color << 28);
        uint64_t lo = e->child_row, hi = e->parent_row;
        if (lo >= R0 && lo < R1 && lo < D->n) {
            uint32_t *c = &cnt[4 * (lo - R0) + 2];
            if (write) vert[(*c)++] = v | (WG_VERT_BOTTOM << 24); else (*c)++;
        }
        uint64_t a = lo + 1 > R0 ? lo + 1 : R0, b = hi < R1 ? hi : R1;
        for (uint64_t r = a; r < b; r++) {
            if (r >= D->n) break;
            uint32_t *c = &cnt[4 * (r - R0) + 0];
            if (write) vert[(*c)++] = v | (WG_VERT_FULL << 24); else (*c)++;
        }
        if (hi >= R0 && hi < R1 && hi < D->n) {
            uint32_t *c = &cnt[4 * (hi - R0) + 1];
            if (write) vert[(*c)++] = v | (WG_VERT_TOP << 24); else (*c)++;
        }
        return;
    }
    const float *row_top_y = D->row_top;
    float child_node_y = e->child_row < D->n ? D->node_y[e->child_row] : WG_NODE_Y;
    float parent_node_y = e->parent_row < D->n ? D->node_y[e->parent_row] : WG_NODE_Y;
    float child_y = row_top_y[e->child_row] + child_node_y;
    float parent_y = row_top_y[e->parent_row] + parent_node_y;
    float dy = parent_y - child_y;
    cubic cv;
    cv.p0.x = (float)e->child_lane;  cv.p0.y = child_y;
    cv.p1.x = (float)e->child_lane;  cv.p1.y = child_y + dy * 0.4f;
    cv.p2.x = (float)e->parent_lane; cv.p2.y = parent_y - dy * 0.4f;
    cv.p3.x = (float)e->parent_lane; cv.p3.y = parent_y;
    uint64_t a = e->child_row > R0 ? e->child_row : R0;
    uint64_t b = e->parent_row < R1 - 1 ? e->parent_row : R1 - 1;
    for (uint64_t row = a; row <= b; row++) {
        float row_top = row_top_y[row];
        float row_bot = row_top_y[row + 1];
        float strip_top = (row == e->child_row) ? child_y : row_top;
        float strip_bot = (row == e->parent_row) ? parent_y : row_bot;
        if (strip_bot - strip_top < 1e-4f) continue;
        if (row >= D->n) continue;
        uint32_t *c = &cnt[4 * (row - R0) + 3];
        if (!write) { (*c)++; continue; }
        float t_a = (row == e->child_row) ? 0.0f : t_at_y(&cv, strip_top);
        float t_b = (row == e->parent_row) ? 1.0f : t_at_y(&cv, strip_bot);
        cubic s = subcurve(&cv, t_a, t_b);
        wg_curve o = {{s.p0.x, s.p0.y - row_top, s.p1.x, s.p1.y - row_top,
                       s.p2.x, s.p2.y - row_top, s.p3.x, s.p3.y - row_top}};
        curve[*c] = o;
        curve_color[*c] = (uint8_t)color;
        (*c)++;
    }
}

/* height/node_y per row given; fills g (row_top copied from row_top_y[0..n]) */
static int decompose_mt(const wgo_layout *L, const float *row_top_y, const float *height, const float *node_y,
                        int threads, wgo_geometry *g) {
    const uint64_t n = L->n, ne = L->n_edges;
    memset(g, 0, sizeof(*g));
    g->n = n;
    g->height = (float *)malloc((n + 1) * sizeof(float));
    g->node_y = (float *)malloc((n + 1) * sizeof(float));
    g->row_top = (float *)malloc((n + 1) * sizeof(float));
    g->vert_off = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    g->curve_off = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    uint32_t *cnt = (uint32_t *)calloc(4 * (n + 1), sizeof(uint32_t));
    uint32_t *nv = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    uint32_t *nc = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    if (!g->height || !g->node_y || !g->row_top || !g->vert_off || !g->curve_off || !cnt || !nv || !nc) {
        free(cnt); free(nv); free(nc);
        return -1;
    }
    decomp_in D = {L->edges, ne, n, row_top_y, node_y};
    /* more ranges than threads: ranges stay balanced when a few hold the long edges */
    const int T = threads, NR = threads > 1 ? 4 * threads : 1;
#pragma omp parallel for num_threads(T) schedule(dynamic, 1)
    for (int q = 0; q < NR; q++) {
        uint64_t R0 = n * q / NR, R1 = n * (q + 1) / NR;
        if (R0 >= R1) continue;
        for (uint64_t k = 0; k < ne; k++) decomp_edge(&D, &L->edges[k], R0, R1, cnt + 4 * R0, 0, NULL, NULL, NULL);
    }
#pragma omp parallel for num_threads(T) schedule(static)
    for (int64_t r = 0; r < (int64_t)n; r++) {
        nv[r] = cnt[4 * r] + cnt[4 * r + 1] + cnt[4 * r + 2];
        nc[r] = cnt[4 * r + 3];
        g->height[r] = height[r];
        g->node_y[r] = node_y[r];
        g->row_top[r] = row_top_y[r];
    }
    g->row_top[n] = row_top_y[n];
    g->n_vert = prefix_u32(nv, g->vert_off, n, T);
    g->n_curve = prefix_u32(nc, g->curve_off, n, T);
    g->vert = (uint32_t *)malloc((g->n_vert + 1) * sizeof(uint32_t));
    g->curve = (wg_curve *)malloc((g->n_curve + 1) * sizeof(wg_curve));
    g->curve_color = (uint8_t *)malloc(g->n_curve + 1);
    if (!g->vert || !g->curve || !g->curve_color) { free(cnt); free(nv); free(nc); return -1; }
    /* cursors: full / top / bottom start at the row's list, in that order (flatten) */
#pragma omp parallel for num_threads(T) schedule(static)
    for (int64_t r = 0; r < (int64_t)n; r++) {
        uint32_t f = cnt[4 * r], t = cnt[4 * r + 1];
        cnt[4 * r + 0] = g->vert_off[r];
        cnt[4 * r + 1] = g->vert_off[r] + f;
        cnt[4 * r + 2] = g->vert_off[r] + f + t;
        cnt[4 * r + 3] = g->curve_off[r];
    }
#pragma omp parallel for num_threads(T) schedule(dynamic, 1)
    for (int q = 0; q < NR; q++) {
        uint64_t R0 = n * q / NR, R1 = n * (q + 1) / NR;
        if (R0 >= R1) continue;
        for (uint64_t k = 0; k < ne; k++)
            decomp_edge(&D, &L->edges[k], R0, R1, cnt + 4 * R0, 1, g->vert, g->curve, g->curve_color);
    }
    free(cnt); free(nv); free(nc);
    return 0;
}

void wgm_geometry_free(wgo_geometry *g) {
    if (!g) return;
    free(g->height); free(g->node_y); free(g->row_top); free(g->vert_off); free(g->vert);
    free(g->curve_off); free(g->curve); free(g->curve_color);
    memset(g, 0, sizeof(*g));
}
void wgm_layout_free(wgo_layout *L) {
    if (!L) return;
    free(L->lane); free(L->color); free(L->edges); free(L->heights);
    wgm_geometry_free(&L->geom);
    memset(L, 0, sizeof(*L));
}

/* ------------------------------------------------------------------------ */
/* GraphLayout::build (:265-355)                                              */
/* ------------------------------------------------------------------------ */
int wgm_layout_build(const wg_commits *in, int threads, wgo_layout *out) {
    memset(out, 0, sizeof(*out));
    const uint64_t n = in->n_commits, np = n ? in->parent_off[n] : 0;
    const int T = threads > 0 ? threads : omp_get_max_threads();
    out->n = n;
    double t0 = now_ms();
    uint64_t cap = 16;
    while (cap < 2 * n + 16) cap <<= 1;
    const uint64_t mask = cap - 1;
    uint32_t *tab = (uint32_t *)calloc(cap, sizeof(uint32_t));
    int32_t *canon = (int32_t *)malloc((n + 1) * sizeof(int32_t));
    int32_t *prow = (int32_t *)malloc((np + 1) * sizeof(int32_t));
    uint32_t *asg = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));   /* lane << 8 | colour, per row */
    if (!tab || !canon || !prow || !asg) { free(tab); free(canon); free(prow); free(asg); return -1; }
#pragma omp parallel num_threads(T)
    {
#pragma omp for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; i++) tab_insert(tab, mask, in->oid, (uint32_t)i);
#pragma omp for schedule(static)
        for (int64_t i = 0; i < (int64_t)n; i++) canon[i] = (int32_t)tab_find(tab, mask, in->oid, in->oid + i * 20);
#pragma omp for schedule(static)
        for (int64_t k = 0; k < (int64_t)np; k++)
            prow[k] = (int32_t)tab_find(tab, mask, in->oid, in->parent_oid + k * 20);
    }
    free(tab);
    double t1 = now_ms();

    /* the greedy walk (:276-295, :401-471); slot = canonical row or -1 */
    uint64_t scap = 64, len = 0, max_lane = 0;
    int32_t *s = (int32_t *)malloc(scap * sizeof(int32_t));
    for (uint64_t i = 0; i < n; i++) {
        const int32_t c = canon[i];
        uint64_t lane = len, fr = len;
        for (uint64_t l = 0; l < len; l++) if (s[l] == c) { lane = l; break; }
        if (lane == len) {
            for (uint64_t l = 0; l < len; l++) if (s[l] < 0) { fr = l; break; }
            lane = fr;
        }
        if (lane == len) {
            if (len == scap) { scap *= 2; s = (int32_t *)realloc(s, scap * sizeof(int32_t)); }
            s[len++] = -1;
        }
        const int orphan = in->flags ? (in->flags[i] & WG_FLAG_ORPHAN) : 0;
        asg[i] = (uint32_t)(lane << 8) | (orphan ? WG_COLOR_ORPHAN : (uint32_t)(lane % 6));
        for (uint64_t l = 0; l < len; l++) if (l != lane && s[l] == c) s[l] = -1;
        const uint32_t p0 = in->parent_off[i], p1 = in->parent_off[i + 1];
        if (p0 == p1) {
            s[lane] = -1;
        } else {
            s[lane] = prow[p0];   /* -1 when the first parent is outside the list */
            for (uint32_t k = p0 + 1; k < p1; k++) {
                const int32_t pr = prow[k];
                if (pr < 0) continue;
                int present = 0;
                for (uint64_t l = 0; l < len; l++) present |= s[l] == pr;
                if (present) continue;
                uint64_t nl = len;
                for (uint64_t l = 0; l < len; l++) if (s[l] < 0) { nl = l; break; }
                if (nl == len) {
                    if (len == scap) { scap *= 2; s = (int32_t *)realloc(s, scap * sizeof(int32_t)); }
                    s[len++] = -1;
                }
                s[nl] = pr;
            }
        }
        for (uint64_t l = len; l-- > 0;)
            if (s[l] >= 0) { if (l > max_lane) max_lane = l; break; }
    }
    free(s);
    out->max_lane = (uint32_t)max_lane;
    out->n_slots = (uint32_t)len;
    double t2 = now_ms();

    /* layouts per row and the edge list (:301-320) */
    out->lane = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    out->color = (uint8_t *)malloc(n + 1);
    uint32_t *ecnt = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    uint32_t *eoff = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    out->edges = (wg_edge *)malloc((np + 1) * sizeof(wg_edge));
    if (!out->lane || !out->color || !ecnt || !eoff || !out->edges) { free(ecnt); free(eoff); return -1; }
#pragma omp parallel for num_threads(T) schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        const uint32_t a = asg[canon[i]];
        out->lane[i] = a >> 8;
        out->color[i] = (uint8_t)(a & 0xFF);
        uint32_t c = 0;
        for (uint32_t k = in->parent_off[i]; k < in->parent_off[i + 1]; k++) c += prow[k] >= 0;
        ecnt[i] = c;
    }
    out->n_edges = prefix_u32(ecnt, eoff, n, T);
#pragma omp parallel for num_threads(T) schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        const uint32_t a = asg[canon[i]];
        uint32_t o = eoff[i];
        for (uint32_t k = in->parent_off[i]; k < in->parent_off[i + 1]; k++) {
            const int32_t pr = prow[k];
            if (pr < 0) continue;
            wg_edge e = {(uint32_t)i, a >> 8, (uint32_t)pr, asg[pr] >> 8, a & 0xFF};
            out->edges[o++] = e;
        }
    }
    free(ecnt); free(eoff); free(canon); free(prow); free(asg);
    double t3 = now_ms();

    /* heights, row_top_y, the build's geometry (:326-346) */
    out->heights = (float *)malloc((n + 1) * sizeof(float));
    float *row_top_y = (float *)malloc((n + 1) * sizeof(float));
    float *node_y = (float *)malloc((n + 1) * sizeof(float));
    heights_mt(n, in->time, out->heights, T);
    float acc = 0.0f;
    for (uint64_t i = 0; i < n; i++) { row_top_y[i] = acc; acc += out->heights[i]; }
    row_top_y[n] = acc;
    for (uint64_t i = 0; i < n; i++) node_y[i] = WG_NODE_Y;
    double t4 = now_ms();
    int rc = decompose_mt(out, row_top_y, out->heights, node_y, T, &out->geom);
    free(row_top_y); free(node_y);
    double t5 = now_ms();

    uint64_t vis = (uint64_t)out->max_lane + 1;     /* graph_width (:353-354) */
    if (vis > WG_LANE_COUNT_VISUAL) vis = WG_LANE_COUNT_VISUAL;
    float gw = (float)vis * WG_LANE_W;
    out->graph_width = gw > WG_LANE_W ? gw : WG_LANE_W;
    g_phase_ms[0] = t1 - t0; g_phase_ms[1] = t2 - t1; g_phase_ms[2] = t3 - t2;
    g_phase_ms[3] = t4 - t3; g_phase_ms[4] = t5 - t4;
    return rc;
}

/* ------------------------------------------------------------------------ */
/* row_geometry_with_bands (:367-399)                                         */
/* ------------------------------------------------------------------------ */
int wgm_row_geometry(const wgo_layout *L, const int64_t *time, const float *band, int threads, wgo_geometry *out) {
    const uint64_t n = L->n;
    const int T = threads > 0 ? threads : omp_get_max_threads();
    double t0 = now_ms();
    float *heights = (float *)malloc((n + 1) * sizeof(float));
    float *row_top_y = (float *)malloc((n + 1) * sizeof(float));
    float *height = (float *)malloc((n + 1) * sizeof(float));
    float *node_y = (float *)malloc((n + 1) * sizeof(float));
    if (!heights || !row_top_y || !height || !node_y) {
        free(heights); free(row_top_y); free(height); free(node_y);
        return -1;
    }
    heights_mt(n, time, heights, T);
    float acc = 0.0f;
    for (uint64_t i = 0; i < n; i++) {
        float b = band ? band[i] : 0.0f;
        row_top_y[i] = acc;
        acc += heights[i] + b;
    }
    row_top_y[n] = acc;
#pragma omp parallel for num_threads(T) schedule(static)
    for (int64_t i = 0; i < (int64_t)n; i++) {
        float b = band ? band[i] : 0.0f;
        height[i] = roundf(heights[i] + b);
        node_y[i] = roundf(b + WG_NODE_Y);
    }
    int rc = decompose_mt(L, row_top_y, height, node_y, T, out);
    free(heights); free(row_top_y); free(height); free(node_y);
    g_phase_ms[5] = now_ms() - t0;
    return rc;
}

/* ------------------------------------------------------------------------ */
/* graph_cell (:803-908) + WG-TESS-1, rows in parallel                        */
/* ------------------------------------------------------------------------ */
static const float UC_COS[25] = WG_UNIT_CIRCLE_COS_INIT;
static const float UC_SIN[25] = WG_UNIT_CIRCLE_SIN_INIT;

static uint64_t visible_lanes_of(float graph_width) {
    float q = roundf(graph_width / WG_LANE_W);
    uint64_t v = q <= 0.0f ? 0 : (uint64_t)q;
    return v > 1 ? v : 1;
}
static float lane_center_x(uint64_t lane, uint64_t vis) {
    uint64_t visual = lane < vis - 1 ? lane : vis - 1;
    return (float)visual * WG_LANE_W + WG_LANE_W * 0.5f;
}
static wg_vertex *vput(wg_vertex *o, float x, float y, const float *rgba) {
    o->x = x; o->y = y; o->r = rgba[0]; o->g = rgba[1]; o->b = rgba[2]; o->a = rgba[3];
    return o + 1;
}
static wg_vertex *emit_vertical(wg_vertex *o, float x, float y0, float y1, const float *rgba) {
    const float hw = WG_LINE_WIDTH * 0.5f;
    float xl = x - hw, xr = x + hw;
    o = vput(o, xl, y0, rgba); o = vput(o, xr, y0, rgba); o = vput(o, xl, y1, rgba);
    o = vput(o, xr, y0, rgba); o = vput(o, xr, y1, rgba); return vput(o, xl, y1, rgba);
}
static wg_vertex *emit_curve(wg_vertex *o, const float *X, const float *Y, const float *rgba) {
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
        o = vput(o, Lx[j], Ly[j], rgba);     o = vput(o, Rx[j], Ry[j], rgba);         o = vput(o, Lx[j + 1], Ly[j + 1], rgba);
        o = vput(o, Rx[j], Ry[j], rgba);     o = vput(o, Rx[j + 1], Ry[j + 1], rgba); o = vput(o, Lx[j + 1], Ly[j + 1], rgba);
    }
    return o;
}
static wg_vertex *emit_node(wg_vertex *o, float cx, float cy, const float *rgba) {
    const float r = WG_NODE_RADIUS;
    for (int j = 0; j < 24; j++) {
        o = vput(o, cx, cy, rgba);
        o = vput(o, cx + r * UC_COS[j], cy + r * UC_SIN[j], rgba);
        o = vput(o, cx + r * UC_COS[j + 1], cy + r * UC_SIN[j + 1], rgba);
    }
    return o;
}
static wg_vertex *emit_ring(wg_vertex *o, float cx, float cy, const float *rgba) {
    const float ri = WG_NODE_RADIUS - WG_SELECTED_RING_WIDTH * 0.5f;
    const float ro = WG_NODE_RADIUS + WG_SELECTED_RING_WIDTH * 0.5f;
    for (int j = 0; j < 24; j++) {
        float ox0 = cx + ro * UC_COS[j], oy0 = cy + ro * UC_SIN[j];
        float ix0 = cx + ri * UC_COS[j], iy0 = cy + ri * UC_SIN[j];
        float ox1 = cx + ro * UC_COS[j + 1], oy1 = cy + ro * UC_SIN[j + 1];
        float ix1 = cx + ri * UC_COS[j + 1], iy1 = cy + ri * UC_SIN[j + 1];
        o = vput(o, ox0, oy0, rgba); o = vput(o, ix0, iy0, rgba); o = vput(o, ox1, oy1, rgba);
        o = vput(o, ix0, iy0, rgba); o = vput(o, ix1, iy1, rgba); o = vput(o, ox1, oy1, rgba);
    }
    return o;
}

/* rows [r0, r1) into dst (cap vertices; NULL: a malloc'd buffer) with
 * offsets into off (r1 - r0 + 1 entries; NULL: malloc'd); the count in
 * *out_n.  A caller that draws frame after frame passes the same buffers (the
 * engine keeps its vertex buffers resident in HBM the same way), so the
 * timing is the emission, not the first touch of fresh pages.  Returns 1 when
 * dst is too small (nothing written but the offsets and the count). */
static int emit_impl(const wgo_layout *L, const wgo_geometry *g, uint64_t r0, uint64_t r1, int64_t selected,
                     const float *palette, int threads, wg_vertex *dst, uint64_t cap, uint64_t *off_dst,
                     wg_vertex **out_v, uint64_t **out_off, uint64_t *out_n) {
    if (r1 > g->n || r0 > r1) return -1;
    const int T = threads > 0 ? threads : omp_get_max_threads();
    double t0 = now_ms();
    const uint64_t m = r1 - r0;
    uint64_t *off = off_dst ? off_dst : (uint64_t *)malloc((m + 1) * sizeof(uint64_t));
    if (!off) return -1;
    uint64_t part[1025];
    const int TT = T > 1024 ? 1024 : T;
#pragma omp parallel num_threads(TT)
    {
        int t = omp_get_thread_num(), nt = omp_get_num_threads();
        uint64_t a = m * t / nt, b = m * (t + 1) / nt, acc = 0;
        for (uint64_t j = a; j < b; j++) {
            const uint64_t r = r0 + j;
            off[j] = acc;
            acc += 6ull * (g->vert_off[r + 1] - g->vert_off[r]) + 96ull * (g->curve_off[r + 1] - g->curve_off[r]) + 72 +
                   ((selected >= 0 && (uint64_t)selected == r) ? 144 : 0);
        }
        part[t + 1] = acc;
#pragma omp barrier
#pragma omp single
        {
            part[0] = 0;
            for (int k = 1; k <= nt; k++) part[k] += part[k - 1];
        }
        for (uint64_t j = a; j < b; j++) off[j] += part[t];
#pragma omp single
        off[m] = part[nt];
    }
    const uint64_t nv = off[m];
    *out_n = nv;
    if (dst && nv > cap) return 1;
    wg_vertex *v = dst ? dst : (wg_vertex *)malloc((nv + 1) * sizeof(wg_vertex));
    if (!v) { if (!off_dst) free(off); return -1; }
    const float gw = L->graph_width;
    const uint64_t vis = visible_lanes_of(gw);
#pragma omp parallel for num_threads(T) schedule(dynamic, 2048)
    for (int64_t j = 0; j < (int64_t)m; j++) {
        const uint64_t r = r0 + (uint64_t)j;
        wg_vertex *o = v + off[j];
        const float h = g->height[r], node_y = g->node_y[r];
        for (uint32_t k = g->vert_off[r]; k < g->vert_off[r + 1]; k++) {
            const uint32_t e = g->vert[k];
            const float x = lane_center_x(WG_VERT_LANE(e), vis);
            const float *rgba = palette + 4 * WG_VERT_COLOR(e);
            switch (WG_VERT_KIND(e)) {
            case WG_VERT_FULL:   o = emit_vertical(o, x, 0.0f, h, rgba); break;
            case WG_VERT_TOP:    o = emit_vertical(o, x, 0.0f, node_y, rgba); break;
            default:             o = emit_vertical(o, x, node_y, h, rgba); break;
            }
        }
        for (uint32_t k = g->curve_off[r]; k < g->curve_off[r + 1]; k++) {
            const float *p = g->curve[k].p;
            float X[4], Y[4];
            for (int q = 0; q < 4; q++) {
                float cl = clampf_rs(p[2 * q], 0.0f, (float)(vis - 1));
                X[q] = cl * WG_LANE_W + WG_LANE_W * 0.5f;
                Y[q] = p[2 * q + 1];
            }
            o = emit_curve(o, X, Y, palette + 4 * g->curve_color[k]);
        }
        const float cx = lane_center_x(L->lane[r], vis);
        o = emit_node(o, cx, node_y, palette + 4 * L->color[r]);
        if (selected >= 0 && (uint64_t)selected == r) o = emit_ring(o, cx, node_y, palette + 4 * WG_COLOR_FOREGROUND);
    }
    if (out_v) *out_v = v;
    if (out_off) *out_off = off;
    g_phase_ms[6] = now_ms() - t0;
    return 0;
}

int wgm_emit_vertices(const wgo_layout *L, const wgo_geometry *g, uint64_t r0, uint64_t r1, int64_t selected,
                      const float *palette, int threads, wg_vertex **out_v, uint64_t **out_off, uint64_t *out_n) {
    return emit_impl(L, g, r0, r1, selected, palette, threads, NULL, 0, NULL, out_v, out_off, out_n);
}

int wgm_emit_vertices_into(const wgo_layout *L, const wgo_geometry *g, uint64_t r0, uint64_t r1, int64_t selected,
                           const float *palette, int threads, wg_vertex *dst, uint64_t cap, uint64_t *off,
                           uint64_t *out_n) {
    if (!dst || !off) return -1;
    return emit_impl(L, g, r0, r1, selected, palette, threads, dst, cap, off, NULL, NULL, out_n);
}

void wgm_free(void *p) { free(p); }
int wgm_max_threads(void) { return omp_get_max_threads(); }
