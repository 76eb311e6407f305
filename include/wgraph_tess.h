/*
 * wgraph_tess.h — frozen constant tables of the WG-TESS-1 tessellation spec
 * (DESIGN.md §5).  The reference tessellator (legacy src/ui/spline.rs) is
 * absent from the snapshot; only its prose survives (docs/render_engine.md:
 * 148-170, README.md:22).  These tables are data shared by the product and
 * the oracle so both tessellate from the same bits; no code lives here.
 *
 * Unit circle at 24 steps (15 degrees), entry 24 == entry 0.  Values are
 * float(cos/sin(2*pi*j/24)) rounded to nearest f32, with the three values
 * that are mathematically zero frozen to exactly 0.
 */
#ifndef WGRAPH_TESS_H
#define WGRAPH_TESS_H

#define WG_C15 0x1.ee8dd4p-1f   /* cos 15 deg = 0.96592581 */
#define WG_C30 0x1.bb67aep-1f   /* cos 30 deg = 0.86602539 */
#define WG_C45 0x1.6a09e6p-1f   /* cos 45 deg = 0.70710677 */
#define WG_S15 0x1.0907dcp-2f   /* sin 15 deg = 0.25881904 */

#define WG_UNIT_CIRCLE_COS_INIT { \
    1.0f,  WG_C15,  WG_C30,  WG_C45,  0.5f,  WG_S15,  0.0f, \
   -WG_S15, -0.5f, -WG_C45, -WG_C30, -WG_C15, -1.0f,         \
   -WG_C15, -WG_C30, -WG_C45, -0.5f, -WG_S15, 0.0f,          \
    WG_S15,  0.5f,  WG_C45,  WG_C30,  WG_C15,  1.0f }

#define WG_UNIT_CIRCLE_SIN_INIT { \
    0.0f,  WG_S15,  0.5f,  WG_C45,  WG_C30,  WG_C15,  1.0f, \
    WG_C15,  WG_C30,  WG_C45,  0.5f,  WG_S15,  0.0f,         \
   -WG_S15, -0.5f, -WG_C45, -WG_C30, -WG_C15, -1.0f,         \
   -WG_C15, -WG_C30, -WG_C45, -0.5f, -WG_S15, 0.0f }

/* Curve parameter step: t_j = (float)j * WG_TESS_DT, exact for j = 0..16 */
#define WG_TESS_DT 0.0625f

#endif /* WGRAPH_TESS_H */
