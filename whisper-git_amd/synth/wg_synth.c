/*
 * wg_synth.c — seeded synthetic commit-DAG generator (bench/test workload).
 *
 * Produces the wg_commits structure-of-arrays (include/wgraph.h) in the row
 * order libgit2's revwalk TOPOLOGICAL|TIME gives the reference
 * (src/git/mod.rs:570-596): newest first, every commit before its parents.
 * It is workload infrastructure, not part of the engine: it models history
 * as a set of "lines" (branches seen backwards in time) that advance one
 * commit at a time, converge at fork points and receive merges.
 *
 * Presets follow SURVEY.md §8(d):
 *   WGS_LINEAR   C1  linear chain
 *   WGS_RANDOM13 C3  mean 1.3 parents, <= 8 branch tips
 *   WGS_LINUX    C4  ~7 % merges, many long-lived lines
 *   WGS_WIDE16   C5  wide DAG, lanes kept <= 16
 *   WGS_ANOMALY      edge cases the reference tolerates: duplicate ids,
 *                    parents at earlier rows (clock skew / orphans,
 *                    git/mod.rs:767-772), parents outside the list,
 *                    repeated parents, self-parents, octopus merges.
 *   WGS_SKEW         the LINUX shape as commit_graph_with_orphans delivers
 *                    it (git/mod.rs:761-775): ~1e-4 of the commits carry a
 *                    committer time moved forward by 1 h .. 30 days (clock
 *                    skew), 100 reflog orphans (short chains off random
 *                    commits, is_orphaned) are appended and the whole list is
 *                    stable-sorted by time, newest first — so every child
 *                    older than a skewed parent now sits BELOW it (a parent
 *                    at an earlier row), and each such reference holds a lane
 *                    slot for the rest of the list (commit_graph.rs:414-423).
 *   WGS_LINUXWIDE    the LINUX shape with up to 160 concurrently active lines
 *                    (more than 100 concurrent lanes).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "wg_synth.h"

/* splitmix64 */
static inline uint64_t sm64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline double urand(uint64_t *s) { return (double)(sm64(s) >> 11) * (1.0 / 9007199254740992.0); }
static inline uint64_t urange(uint64_t *s, uint64_t n) { return n ? sm64(s) % n : 0; }

int wgs_preset(int kind, uint64_t n, uint64_t seed, wgs_params *p) {
    memset(p, 0, sizeof(*p));
    p->kind = kind; p->n = n; p->seed = seed;
    p->band_frac = 0.02; p->main_weight = 4.0;
    switch (kind) {
    case WGS_LINEAR:   p->max_lines = 1;  break;
    case WGS_RANDOM13: p->max_lines = 8;  p->p_merge = 0.30; p->p_newtip = 0.06; p->p_fork = 0.10; p->main_weight = 2.0; p->p_feature = 0.3; break;
    case WGS_LINUX:    p->max_lines = 28; p->p_merge = 0.07; p->p_newtip = 0.02; p->p_fork = 0.04; p->p_octopus = 0.002; p->main_weight = 3.0; p->p_feature = 0.5; break;
    case WGS_WIDE16:   p->max_lines = 10; p->p_merge = 0.10; p->p_newtip = 0.01; p->p_fork = 0.03; p->main_weight = 2.0; p->p_feature = 0.3; break;
    case WGS_SKEW:     p->max_lines = 28; p->p_merge = 0.07; p->p_newtip = 0.02; p->p_fork = 0.04; p->p_octopus = 0.002; p->main_weight = 3.0; p->p_feature = 0.5;
                       p->p_clock_skew = 1e-4; p->n_orphans = n >= 1000 ? 100 : n / 10; break;
    case WGS_LINUXWIDE: p->max_lines = 160; p->p_merge = 0.07; p->p_newtip = 0.03; p->p_fork = 0.02; p->p_octopus = 0.002; p->main_weight = 3.0; p->p_feature = 0.5; break;
    case WGS_ANOMALY:  p->max_lines = 9;  p->p_merge = 0.25; p->p_newtip = 0.10; p->p_fork = 0.08; p->p_octopus = 0.05;
                       p->p_dup_oid = 0.03; p->p_skew = 0.04; p->p_external = 0.05; p->p_self = 0.01;
                       p->p_dup_parent = 0.03; p->p_orphan_flag = 0.05; p->band_frac = 0.1; p->truncated = 1; p->p_feature = 0.3; break;
    default: return -1;
    }
    return 0;
}

/* growable int64 vector */
typedef struct { int64_t *v; uint64_t n, cap; } vec64;
static int vpush(vec64 *a, int64_t x) {
    if (a->n == a->cap) {
        uint64_t nc = a->cap ? a->cap * 2 : 8;
        int64_t *nv = (int64_t *)realloc(a->v, nc * sizeof(int64_t));
        if (!nv) return -1;
        a->v = nv; a->cap = nc;
    }
    a->v[a->n++] = x;
    return 0;
}

/* Parent references are kept as int64 codes while the DAG grows:
 *   >= 0                 row index
 *   -1                   unresolved slot (filled when the line advances)
 *   <= -2                external id number (-2 - k)                    */
#define UNRES (-1)

void wgs_free(wgs_dag *d) {
    if (!d) return;
    free(d->oid); free(d->time); free(d->parent_off); free(d->parent_oid);
    free(d->flags); free(d->band); free(d);
}

static int orphans_and_time_sort(wgs_dag *d, const wgs_params *p, uint64_t *rs);

wgs_dag *wgs_generate(const wgs_params *p) {
    if (p->n_orphans > 0 || p->p_clock_skew > 0) {
        /* the revwalk list (n - n_orphans rows), then the reflog orphans */
        wgs_params b = *p;
        const uint64_t no = p->n_orphans < p->n ? p->n_orphans : p->n;
        b.n = p->n - no;
        b.n_orphans = 0;
        b.p_clock_skew = 0;
        wgs_dag *d = wgs_generate(&b);
        if (!d) return NULL;
        uint64_t rs = p->seed * 0xD1B54A32D192ED03ull + 0x0125ull;
        b.n_orphans = no;
        b.p_clock_skew = p->p_clock_skew;
        if (orphans_and_time_sort(d, &b, &rs)) { wgs_free(d); return NULL; }
        return d;
    }
    const uint64_t n = p->n;
    uint64_t rs = p->seed * 0x2545F4914F6CDD1Dull + 0x5EEDull;
    wgs_dag *d = (wgs_dag *)calloc(1, sizeof(wgs_dag));
    if (!d) return NULL;
    d->n = n;
    /* per-row parent lists: first parent in fp[], the rest in a side pool */
    int64_t *fp = (int64_t *)malloc((n ? n : 1) * sizeof(int64_t));
    uint32_t *xcount = (uint32_t *)calloc(n ? n : 1, sizeof(uint32_t));
    vec64 xrow = {0}, xval = {0};               /* extra parents: (row, code) */
    const int maxl = p->max_lines > 0 ? p->max_lines : 1;
    int64_t *line_last = (int64_t *)malloc(maxl * sizeof(int64_t));
    int *active = (int *)malloc(maxl * sizeof(int));
    vec64 *pend = (vec64 *)calloc(maxl, sizeof(vec64));  /* indices into xval */
    d->oid = (uint8_t *)malloc((n ? n : 1) * 20);
    d->time = (int64_t *)malloc((n ? n : 1) * sizeof(int64_t));
    d->flags = (uint8_t *)calloc(n ? n : 1, 1);
    d->band = (float *)calloc(n ? n : 1, sizeof(float));
    if (!fp || !xcount || !line_last || !active || !pend || !d->oid || !d->time || !d->flags || !d->band) goto fail;

    int nact = 0;
    int64_t ext_counter = 0;
    int64_t t = 1704067200;  /* 2024-01-01 */
    for (uint64_t i = 0; i < n; i++) {
        /* id */
        for (int k = 0; k < 20; k += 8) {
            uint64_t r = sm64(&rs);
            memcpy(d->oid + i * 20 + k, &r, (k + 8 <= 20) ? 8 : 4);
        }
        if (i > 0 && p->p_dup_oid > 0 && urand(&rs) < p->p_dup_oid)
            memcpy(d->oid + i * 20, d->oid + urange(&rs, i) * 20, 20);
        /* time: log-uniform gap 30 s .. 3 days */
        if (i > 0) {
            double lg = log(30.0) + urand(&rs) * (log(259200.0) - log(30.0));
            t -= (int64_t)exp(lg);
        }
        d->time[i] = t;
        if (p->band_frac > 0 && urand(&rs) < p->band_frac) d->band[i] = 30.0f;
        if (p->p_orphan_flag > 0 && urand(&rs) < p->p_orphan_flag) d->flags[i] |= 1;
        fp[i] = UNRES;

        /* which line does row i advance? */
        int L;
        if (nact == 0 || (nact < maxl && urand(&rs) < p->p_newtip)) {
            L = nact++;
            active[L] = 1;
            line_last[L] = -1;
            pend[L].n = 0;
        } else {
            double tot = p->main_weight + (double)(nact - 1), r = urand(&rs) * tot;
            L = (r < p->main_weight) ? 0 : 1 + (int)urange(&rs, (uint64_t)(nact - 1));
            if (L >= nact) L = nact - 1;
        }
        if (line_last[L] >= 0) fp[line_last[L]] = (int64_t)i;
        for (uint64_t k = 0; k < pend[L].n; k++) xval.v[pend[L].v[k]] = (int64_t)i;
        pend[L].n = 0;
        /* fork point: another line converges into row i */
        if (nact >= 2 && p->p_fork > 0 && urand(&rs) < p->p_fork) {
            int L2 = (int)urange(&rs, (uint64_t)nact);
            if (L2 != L && L2 != 0) {
                if (line_last[L2] >= 0) fp[line_last[L2]] = (int64_t)i;
                for (uint64_t k = 0; k < pend[L2].n; k++) xval.v[pend[L2].v[k]] = (int64_t)i;
                /* remove L2 by moving the last line into its place */
                int last = nact - 1;
                if (L == last) L = L2;
                line_last[L2] = line_last[last];
                vec64 tmp = pend[L2]; pend[L2] = pend[last]; pend[last] = tmp;
                pend[last].n = 0;
                nact--;
            }
        }
        /* merges: extra parents resolve to other lines' next commits */
        if (nact >= 1 && p->p_merge > 0 && urand(&rs) < p->p_merge) {
            int extra = 1;
            if (p->p_octopus > 0 && urand(&rs) < p->p_octopus) extra += 1 + (int)urange(&rs, 6);
            for (int k = 0; k < extra; k++) {
                int L3;
                if (nact < maxl && p->p_feature > 0 && urand(&rs) < p->p_feature) {
                    /* feature-branch merge: the merged tip starts a new line,
                     * so this merge is the first reference to it */
                    L3 = nact++;
                    active[L3] = 1;
                    line_last[L3] = -1;
                    pend[L3].n = 0;
                } else {
                    if (nact < 2) continue;
                    L3 = (int)urange(&rs, (uint64_t)nact);
                }
                if (L3 == L) continue;
                if (vpush(&xrow, (int64_t)i) || vpush(&xval, UNRES) || vpush(&pend[L3], (int64_t)(xval.n - 1))) goto fail;
                xcount[i]++;
            }
        }
        /* anomalies */
        if (p->p_skew > 0 && i > 0 && urand(&rs) < p->p_skew) {
            if (vpush(&xrow, (int64_t)i) || vpush(&xval, (int64_t)urange(&rs, i))) goto fail;
            xcount[i]++;
        }
        if (p->p_external > 0 && urand(&rs) < p->p_external) {
            if (vpush(&xrow, (int64_t)i) || vpush(&xval, -2 - (ext_counter++))) goto fail;
            xcount[i]++;
        }
        if (p->p_self > 0 && urand(&rs) < p->p_self) {
            if (vpush(&xrow, (int64_t)i) || vpush(&xval, (int64_t)i)) goto fail;
            xcount[i]++;
        }
        line_last[L] = (int64_t)i;
    }

    /* assemble CSR: first parent (if any) then extras in creation order */
    {
        uint64_t *xoff = (uint64_t *)calloc(n + 1, sizeof(uint64_t));
        if (!xoff) goto fail;
        for (uint64_t k = 0; k < xrow.n; k++) xoff[xrow.v[k] + 1]++;
        for (uint64_t i = 0; i < n; i++) xoff[i + 1] += xoff[i];
        int64_t *xs = (int64_t *)malloc((xrow.n ? xrow.n : 1) * sizeof(int64_t));
        uint64_t *fill = (uint64_t *)malloc((n ? n : 1) * sizeof(uint64_t));
        if (!xs || !fill) { free(xoff); free(xs); free(fill); goto fail; }
        for (uint64_t i = 0; i < n; i++) fill[i] = xoff[i];
        for (uint64_t k = 0; k < xrow.n; k++) xs[fill[xrow.v[k]]++] = xval.v[k];
        free(fill);

        d->parent_off = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
        uint64_t cap = n + xrow.n + n / 8 + 16;
        int64_t *codes = (int64_t *)malloc(cap * sizeof(int64_t));
        if (!d->parent_off || !codes) { free(xoff); free(xs); free(codes); goto fail; }
        uint64_t e = 0;
        for (uint64_t i = 0; i < n; i++) {
            d->parent_off[i] = (uint32_t)e;
            int64_t f = fp[i];
            if (f == UNRES && p->truncated && i + 1 < n && urand(&rs) < 0.5) f = -2 - (ext_counter++);
            if (f != UNRES) codes[e++] = f;
            for (uint64_t k = xoff[i]; k < xoff[i + 1]; k++) {
                int64_t c = xs[k];
                if (c == UNRES) { if (!p->truncated) continue; c = -2 - (ext_counter++); }
                codes[e++] = c;
            }
            if (p->p_dup_parent > 0 && e > d->parent_off[i] && urand(&rs) < p->p_dup_parent)
                codes[e++] = codes[d->parent_off[i]];
            if (e + 16 > cap) {
                cap *= 2;
                int64_t *nc = (int64_t *)realloc(codes, cap * sizeof(int64_t));
                if (!nc) { free(xoff); free(xs); free(codes); goto fail; }
                codes = nc;
            }
        }
        d->parent_off[n] = (uint32_t)e;
        d->e = e;
        d->parent_oid = (uint8_t *)malloc((e ? e : 1) * 20);
        if (!d->parent_oid) { free(xoff); free(xs); free(codes); goto fail; }
        for (uint64_t k = 0; k < e; k++) {
            int64_t c = codes[k];
            if (c >= 0) memcpy(d->parent_oid + k * 20, d->oid + c * 20, 20);
            else {
                uint64_t es = p->seed ^ 0xE47E4A1ull ^ ((uint64_t)(-2 - c) * 0x9E3779B97F4A7C15ull);
                for (int b = 0; b < 20; b += 8) {
                    uint64_t r = sm64(&es);
                    memcpy(d->parent_oid + k * 20 + b, &r, (b + 8 <= 20) ? 8 : 4);
                }
            }
        }
        free(xoff); free(xs); free(codes);
    }
    free(fp); free(xcount); free(xrow.v); free(xval.v); free(line_last); free(active);
    for (int k = 0; k < maxl; k++) free(pend[k].v);
    free(pend);
    return d;
fail:
    free(fp); free(xcount); free(xrow.v); free(xval.v); free(line_last); free(active);
    if (pend) { for (int k = 0; k < maxl; k++) free(pend[k].v); free(pend); }
    wgs_free(d);
    return NULL;
}

void wgs_sizes(const wgs_dag *d, uint64_t *n, uint64_t *e) { *n = d->n; *e = d->e; }

void wgs_copy(const wgs_dag *d, uint8_t *oid, int64_t *time, uint32_t *parent_off,
              uint8_t *parent_oid, uint8_t *flags, float *band) {
    if (oid) memcpy(oid, d->oid, d->n * 20);
    if (time) memcpy(time, d->time, d->n * sizeof(int64_t));
    if (parent_off) memcpy(parent_off, d->parent_off, (d->n + 1) * sizeof(uint32_t));
    if (parent_oid) memcpy(parent_oid, d->parent_oid, d->e * 20);
    if (flags) memcpy(flags, d->flags, d->n);
    if (band) memcpy(band, d->band, d->n * sizeof(float));
}

/* WGS_SKEW's second half (git/mod.rs:761-775 on a skewed history):
 * clock skew on the walk rows, the reflog orphans appended (newest first,
 * git/mod.rs:748-751), then a stable sort of the whole list by time desc. */
typedef struct { int64_t t; uint64_t row; } tkey;
static int tkey_cmp(const void *a, const void *b) {
    const tkey *x = (const tkey *)a, *y = (const tkey *)b;
    if (x->t != y->t) return x->t > y->t ? -1 : 1;   /* Reverse(time) */
    return x->row < y->row ? -1 : (x->row > y->row);   /* stable */
}

static int orphans_and_time_sort(wgs_dag *d, const wgs_params *p, uint64_t *rs) {
    const uint64_t nw = d->n, no = p->n_orphans, n = nw + no;
    /* clock skew: committer time moved forward by 1 h .. 30 days */
    for (uint64_t i = 0; i < nw; i++)
        if (urand(rs) < p->p_clock_skew) {
            double lg = log(3600.0) + urand(rs) * (log(2592000.0) - log(3600.0));
            d->time[i] += (int64_t)exp(lg);
        }
    /* orphans: chains of 1-8 commits, the oldest one's parent a walk row,
     * each newer than its parent by 1 min .. 2 days */
    uint8_t *oid = (uint8_t *)malloc(n * 20);
    int64_t *time = (int64_t *)malloc(n * sizeof(int64_t));
    uint8_t *flags = (uint8_t *)calloc(n, 1);
    float *band = (float *)calloc(n, sizeof(float));
    uint32_t *poff = (uint32_t *)malloc((n + 1) * sizeof(uint32_t));
    uint8_t *poid = (uint8_t *)malloc((d->e + no + 1) * 20);
    tkey *key = (tkey *)malloc(n * sizeof(tkey));
    uint64_t *src = (uint64_t *)malloc(n * sizeof(uint64_t));   /* source row per orphan-extended row */
    int64_t *opar = (int64_t *)malloc((no + 1) * sizeof(int64_t)); /* orphan parent: walk row or -(1 + orphan) */
    if (!oid || !time || !flags || !band || !poff || !poid || !key || !src || !opar) goto fail;
    memcpy(oid, d->oid, nw * 20);
    memcpy(time, d->time, nw * sizeof(int64_t));
    memcpy(flags, d->flags, nw);
    memcpy(band, d->band, nw * sizeof(float));
    {
        /* generated oldest first inside a chain, then listed newest first */
        uint64_t k = 0;
        while (k < no) {
            uint64_t len = 1 + urange(rs, 8);
            if (len > no - k) len = no - k;
            const uint64_t base = nw ? urange(rs, nw) : 0;
            int64_t t = nw ? d->time[base] : 1704067200;
            for (uint64_t j = 0; j < len; j++) {
                const uint64_t o = nw + k + j;
                for (int b = 0; b < 20; b += 8) {
                    uint64_t r = sm64(rs);
                    memcpy(oid + o * 20 + b, &r, (b + 8 <= 20) ? 8 : 4);
                }
                double lg = log(60.0) + urand(rs) * (log(172800.0) - log(60.0));
                t += (int64_t)exp(lg);
                time[o] = t;
                flags[o] = 1;   /* is_orphaned */
                opar[k + j] = j == 0 ? (nw ? (int64_t)base : INT64_MIN) : -(int64_t)(k + j);   /* previous orphan */
            }
            k += len;
        }
    }
    for (uint64_t i = 0; i < n; i++) { key[i].t = time[i]; key[i].row = i; }
    qsort(key, n, sizeof(tkey), tkey_cmp);
    {
        uint64_t e = 0;
        for (uint64_t r = 0; r < n; r++) {
            const uint64_t i = key[r].row;
            src[r] = i;
            poff[r] = (uint32_t)e;
            if (i < nw) {
                const uint64_t pa = d->parent_off[i], pb = d->parent_off[i + 1];
                memcpy(poid + e * 20, d->parent_oid + pa * 20, (pb - pa) * 20);
                e += pb - pa;
            } else {
                const int64_t q = opar[i - nw];
                if (q == INT64_MIN) continue;
                const uint64_t pr = q >= 0 ? (uint64_t)q : nw + (uint64_t)(-q - 1);
                memcpy(poid + e * 20, oid + pr * 20, 20);
                e++;
            }
        }
        poff[n] = (uint32_t)e;
        d->e = e;
    }
    {
        uint8_t *oid2 = (uint8_t *)malloc(n * 20);
        int64_t *time2 = (int64_t *)malloc(n * sizeof(int64_t));
        uint8_t *flags2 = (uint8_t *)malloc(n);
        float *band2 = (float *)malloc(n * sizeof(float));
        if (!oid2 || !time2 || !flags2 || !band2) { free(oid2); free(time2); free(flags2); free(band2); goto fail; }
        for (uint64_t r = 0; r < n; r++) {
            memcpy(oid2 + r * 20, oid + src[r] * 20, 20);
            time2[r] = time[src[r]];
            flags2[r] = flags[src[r]];
            band2[r] = band[src[r]];
        }
        free(d->oid); free(d->time); free(d->flags); free(d->band); free(d->parent_off); free(d->parent_oid);
        d->oid = oid2; d->time = time2; d->flags = flags2; d->band = band2; d->parent_off = poff; d->parent_oid = poid;
        d->n = n;
    }
    free(oid); free(time); free(flags); free(band); free(key); free(src); free(opar);
    return 0;
fail:
    free(oid); free(time); free(flags); free(band); free(poff); free(poid); free(key); free(src); free(opar);
    return -1;
}
