/*
 * wg_oracle.h — C API of the CPU ORACLE (oracle/wg_oracle.c).
 *
 * TEST INFRASTRUCTURE ONLY: the checker the HIP engine is compared against
 * (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline).  The product
 * never includes or links it.  Each function restates the reference item
 * named beside it (/root/reference/src/commit_graph.rs).
 */
#ifndef WG_ORACLE_H
#define WG_ORACLE_H

#include <stdint.h>

#include "../include/wgraph.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct wgo_geometry {
    uint64_t  n, n_vert, n_curve;
    float    *height, *node_y, *row_top;
    uint32_t *vert_off, *vert, *curve_off;
    wg_curve *curve;
    uint8_t  *curve_color;
} wgo_geometry;

typedef struct wgo_layout {
    uint64_t  n, n_edges;
    uint32_t  max_lane, n_slots;
    float     graph_width;
    uint32_t *lane;       /* per row: layouts.get(&commits[row].id).lane  */
    uint8_t  *color;
    wg_edge  *edges;
    float    *heights;
    wgo_geometry geom;    /* self.row_geometry from build()               */
} wgo_layout;

/* GraphLayout::build (:265-355); 0 on success, *out freed by wgo_layout_free */
int  wgo_layout_build(const wg_commits *in, wgo_layout *out);
void wgo_layout_free(wgo_layout *L);
/* row_geometry_with_bands (:367-399); band NULL = zero bands */
int  wgo_row_geometry(const wgo_layout *L, const int64_t *time, const float *band, wgo_geometry *out);
void wgo_geometry_free(wgo_geometry *g);
/* decompose_edge_into_rows over default rows (the reference KATs, :1631-1702) */
int  wgo_decompose_edges(const wg_edge *edges, uint64_t ne, const float *row_top_y, uint64_t nrows, wgo_geometry *out);
/* compute_row_heights (:486-507) */
void wgo_compute_row_heights(uint64_t n, const int64_t *time, float *heights);
/* Cubic::{y_at, t_at_y, subcurve} (:614-695) on {p0.x, p0.y, ..., p3.y} */
float wgo_cubic_y_at(const float *p8, float t);
float wgo_cubic_t_at_y(const float *p8, float y);
void  wgo_cubic_subcurve(const float *p8, float a, float b, float *out8);
/* graph_cell (:803-908) + WG-TESS-1 for rows [r0, r1); outputs malloc'd (wgo_free) */
int  wgo_emit_vertices(const wgo_layout *L, const wgo_geometry *g, uint64_t r0, uint64_t r1, int64_t selected,
                       const float *palette, wg_vertex **out_v, uint64_t **out_off, uint64_t *out_n);
void wgo_free(void *p);
uint64_t wgo_vertex_checksum(const wg_vertex *v, uint64_t n);
uint64_t wgo_vertex_checksum_at(const wg_vertex *v, uint64_t n, uint64_t first_vertex);

#ifdef __cplusplus
}
#endif

#endif
