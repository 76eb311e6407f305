/*
 * wg_synth.h — seeded synthetic commit-DAG generator (workload, not engine).
 * See wg_synth.c for the model and the presets.
 */
#ifndef WG_SYNTH_H
#define WG_SYNTH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { WGS_LINEAR = 0, WGS_RANDOM13 = 1, WGS_LINUX = 2, WGS_WIDE16 = 3, WGS_ANOMALY = 4, WGS_SKEW = 5, WGS_LINUXWIDE = 6 };

typedef struct wgs_params {
    int32_t  kind;
    int32_t  max_lines;      /* cap on concurrently active lines          */
    uint64_t n;
    uint64_t seed;
    double   p_merge;        /* row gets a second parent                  */
    double   p_octopus;      /* a merge gets 1-6 extra parents            */
    double   p_newtip;       /* a new line starts at this row             */
    double   p_fork;         /* another line converges into this row      */
    double   main_weight;    /* selection weight of line 0 vs 1 per other */
    double   p_dup_oid;      /* anomaly: row reuses an earlier row's id   */
    double   p_skew;         /* anomaly: extra parent at an earlier row   */
    double   p_external;     /* anomaly: extra parent outside the list    */
    double   p_self;         /* anomaly: commit lists itself as parent    */
    double   p_dup_parent;   /* anomaly: a parent id repeated             */
    double   p_orphan_flag;  /* row flagged is_orphaned                   */
    double   band_frac;      /* rows with a 30 px pills band              */
    int32_t  truncated;      /* unresolved first parents point outside    */
    int32_t  reserved;
    double   p_feature;      /* a merge's second parent starts a new line */
    double   p_clock_skew;   /* a commit's time moved forward (1 h .. 30 d) */
    uint64_t n_orphans;      /* reflog orphans appended, then the whole list
                                stable-sorted by time desc (git/mod.rs:761-775) */
} wgs_params;

typedef struct wgs_dag {
    uint64_t  n, e;
    uint8_t  *oid;
    int64_t  *time;
    uint32_t *parent_off;
    uint8_t  *parent_oid;
    uint8_t  *flags;
    float    *band;
} wgs_dag;

/* fill *p with the preset's parameters; 0 on success */
int      wgs_preset(int kind, uint64_t n, uint64_t seed, wgs_params *p);
wgs_dag *wgs_generate(const wgs_params *p);
void     wgs_free(wgs_dag *d);
void     wgs_sizes(const wgs_dag *d, uint64_t *n, uint64_t *e);
void     wgs_copy(const wgs_dag *d, uint8_t *oid, int64_t *time, uint32_t *parent_off, uint8_t *parent_oid,
                  uint8_t *flags, float *band);

#ifdef __cplusplus
}
#endif

#endif
