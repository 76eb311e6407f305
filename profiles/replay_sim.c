/*
 * replay_sim.c — CPU model of the chunked fixed-point lane replay
 * (whisper-git_amd/csrc/wg_lanes_replay.hip), for studying how many
 * iterations each way of guessing a chunk's entry occupancy needs on the
 * BASELINE list shapes.  Research tool (profiles/), not the engine, not the
 * oracle.
 *
 * The event stream is taken from a sequential run of the reference greedy
 * (commit_graph.rs:276-295, 401-471) that tracks, per slot, the token (event)
 * whose chain holds it — the same events the engine's event compression
 * builds (wg_lanes_fast.hip): ALLOC (w = 0), MIN (w >= 2), FREE (w = 1, first
 * parent outside the list), SECALLOC (first reference through a secondary
 * parent).  Then per iteration every chunk is replayed from a guessed entry
 * state, tokens born in earlier chunks read from the previous iteration:
 *
 *   exit   (the engine today) entry = previous iteration's exit occupancy of
 *          chunk c-1; iteration 1 warm-started `warm` events early from empty
 *   live   entry = OR of the previous iteration's slots of the tokens alive at
 *          the chunk's first event (structural: born before it, consumed at or
 *          after it, or never — leaked)
 *   livewarm  every iteration starts `warm` events early (a multiple of the
 *          chunk) from the live tokens' previous slots there
 *
 * usage: replay_sim <preset> <rows> <chunk> <warm> [scheme ...]
 * prints one JSON line per scheme: iterations to the fixed point, per
 * iteration [iteration, chunks still wrong, first wrong chunk, events whose
 * slot changed, the most changed events in one chunk, events still wrong].
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../whisper-git_amd/synth/wg_synth.h"

#define MAXW 16   /* 1024 slots */
typedef struct { uint64_t w[MAXW]; } occ_t;
static inline void occ_set(occ_t *o, uint32_t s) { o->w[s >> 6] |= 1ull << (s & 63); }
static inline void occ_clr(occ_t *o, uint32_t s) { o->w[s >> 6] &= ~(1ull << (s & 63)); }
static inline uint32_t occ_lowest_free(const occ_t *o) {
    for (int k = 0; k < MAXW; k++)
        if (~o->w[k]) return 64u * k + (uint32_t)__builtin_ctzll(~o->w[k]);
    return 64u * MAXW - 1;
}
static inline int occ_eq(const occ_t *a, const occ_t *b) { return memcmp(a, b, sizeof(occ_t)) == 0; }

typedef struct {
    uint8_t a, o;          /* allocates / occupies afterwards */
    uint32_t ntok, tok0;   /* consumed tokens: tokpool[tok0 .. tok0 + ntok) */
    uint16_t slot;         /* the sequential result */
} ev_t;

static ev_t *EV;
static uint32_t *TOK;
static uint64_t NEV, NTOK;
static uint64_t cap_ev, cap_tok;
static uint32_t push_ev(uint8_t a, uint8_t o) {
    if (NEV == cap_ev) { cap_ev = cap_ev ? 2 * cap_ev : 1024; EV = realloc(EV, cap_ev * sizeof(ev_t)); }
    EV[NEV].a = a; EV[NEV].o = o; EV[NEV].ntok = 0; EV[NEV].tok0 = (uint32_t)NTOK; EV[NEV].slot = 0;
    return (uint32_t)NEV++;
}
static void push_tok(uint32_t e, uint32_t t) {
    if (NTOK == cap_tok) { cap_tok = cap_tok ? 2 * cap_tok : 1024; TOK = realloc(TOK, cap_tok * 4); }
    TOK[NTOK++] = t;
    EV[e].ntok++;
}

/* oid -> row (ids are distinct in these presets; last occurrence wins) */
static uint64_t HC;
static int64_t *HROW;
static const uint8_t *OID;
static uint64_t hkey(const uint8_t *id) { uint64_t k; memcpy(&k, id, 8); return k * 0x9E3779B97F4A7C15ull; }
static void hput(uint64_t row) {
    uint64_t h = hkey(OID + row * 20) & (HC - 1);
    while (HROW[h] >= 0 && memcmp(OID + HROW[h] * 20, OID + row * 20, 20)) h = (h + 1) & (HC - 1);
    HROW[h] = (int64_t)row;
}
static int64_t hget(const uint8_t *id) {
    uint64_t h = hkey(id) & (HC - 1);
    while (HROW[h] >= 0) {
        if (!memcmp(OID + HROW[h] * 20, id, 20)) return HROW[h];
        h = (h + 1) & (HC - 1);
    }
    return -1;
}

static void build_events(const wgs_dag *d) {
    const uint64_t n = d->n;
    OID = d->oid;
    for (HC = 1; HC < 2 * n + 2; HC <<= 1) {}
    HROW = malloc(HC * sizeof(int64_t));
    for (uint64_t h = 0; h < HC; h++) HROW[h] = -1;
    for (uint64_t i = 0; i < n; i++) hput(i);
    uint64_t ns = 0, cs = 64;
    int64_t *tgt = malloc(cs * sizeof(int64_t));
    uint32_t *tok = malloc(cs * 4);
    for (uint64_t i = 0; i < n; i++) {
        uint32_t pa = d->parent_off[i], pb = d->parent_off[i + 1];
        int64_t fp = pa < pb ? hget(d->parent_oid + (uint64_t)pa * 20) : -1;
        uint32_t nwait = 0, lane = 0;
        for (uint64_t s = 0; s < ns; s++)
            if (tgt[s] == (int64_t)i) { if (!nwait) lane = (uint32_t)s; nwait++; }
        uint32_t t;   /* the token of row i's chain */
        if (nwait == 0) {
            uint64_t s = 0;
            while (s < ns && tgt[s] >= 0) s++;
            if (s == ns) { if (ns == cs) { cs *= 2; tgt = realloc(tgt, cs * 8); tok = realloc(tok, cs * 4); } tgt[ns++] = -1; }
            lane = (uint32_t)s;
            t = push_ev(1, fp >= 0);
            EV[t].slot = (uint16_t)lane;
        } else if (nwait == 1) {
            t = tok[lane];
            if (fp < 0) {
                const uint32_t e = push_ev(0, 0);
                push_tok(e, t);
                EV[e].slot = (uint16_t)lane;
            }
        } else {
            t = push_ev(0, fp >= 0);
            for (uint64_t s = 0; s < ns; s++)
                if (tgt[s] == (int64_t)i) { push_tok(t, tok[s]); if (s != lane) tgt[s] = -1; }
            EV[t].slot = (uint16_t)lane;
        }
        if (pa == pb || fp < 0) tgt[lane] = -1;
        else { tgt[lane] = fp; tok[lane] = t; }
        for (uint32_t k = pa + 1; k < pb; k++) {
            int64_t p = hget(d->parent_oid + (uint64_t)k * 20);
            if (p < 0) continue;
            int present = 0;
            for (uint64_t s = 0; s < ns; s++) if (tgt[s] == p) { present = 1; break; }
            if (present) continue;
            uint64_t s = 0;
            while (s < ns && tgt[s] >= 0) s++;
            if (s == ns) { if (ns == cs) { cs *= 2; tgt = realloc(tgt, cs * 8); tok = realloc(tok, cs * 4); } tgt[ns++] = -1; }
            const uint32_t e = push_ev(1, 1);
            EV[e].slot = (uint16_t)s;
            tgt[s] = p;
            tok[s] = e;
        }
    }
    free(tgt); free(tok); free(HROW);
    fprintf(stderr, "rows %lu events %lu slots %lu\n", (unsigned long)n, (unsigned long)NEV, (unsigned long)ns);
}

enum { S_EXIT, S_LIVE, S_LIVEWARM };

static void run(const char *name, int scheme, uint32_t CH, uint32_t warm) {
    const uint64_t nch = (NEV + CH - 1) / CH;
    uint16_t *prev = calloc(NEV, 2), *next = calloc(NEV, 2), *own = calloc(NEV, 2);
    occ_t *xprev = calloc(nch, sizeof(occ_t)), *xnext = calloc(nch, sizeof(occ_t));
    /* structural liveness: death[t] = consuming event (or NEV: never) */
    uint64_t *death = malloc(NEV * 8);
    for (uint64_t k = 0; k < NEV; k++) death[k] = NEV;
    for (uint64_t k = 0; k < NEV; k++)
        for (uint32_t q = 0; q < EV[k].ntok; q++) death[TOK[EV[k].tok0 + q]] = k;
    /* live lists per chunk boundary */
    uint64_t *lcnt = calloc(nch + 1, 8);
    for (uint64_t t = 0; t < NEV; t++) {
        if (!EV[t].o) continue;
        const uint64_t c0 = t / CH + 1, c1 = death[t] == NEV ? nch - 1 : death[t] / CH;   /* e0(c) in (t, death] */
        for (uint64_t c = c0; c <= c1 && c < nch; c++) lcnt[c + 1]++;
    }
    for (uint64_t c = 0; c < nch; c++) lcnt[c + 1] += lcnt[c];
    uint32_t *live = malloc((lcnt[nch] + 1) * 4);
    uint64_t *fill = calloc(nch, 8);
    for (uint64_t t = 0; t < NEV; t++) {
        if (!EV[t].o) continue;
        const uint64_t c0 = t / CH + 1, c1 = death[t] == NEV ? nch - 1 : death[t] / CH;
        for (uint64_t c = c0; c <= c1 && c < nch; c++) live[lcnt[c] + fill[c]++] = (uint32_t)t;
    }
    printf("{\"scheme\": \"%s\", \"chunk\": %u, \"warm\": %u, \"events\": %lu, \"chunks\": %lu, \"live_entries\": %lu, \"iters\": [",
           name, CH, warm, (unsigned long)NEV, (unsigned long)nch, (unsigned long)lcnt[nch]);
    int it;
    for (it = 1; it <= 100000; it++) {
        int changed = 0;
        uint64_t nchg = 0, maxchg = 0, wrong_chunks = 0, first_wrong = nch, wrong_ev = 0;
        for (uint64_t c = 0; c < nch; c++) {
            const uint64_t e0 = c * CH, e1 = e0 + CH < NEV ? e0 + CH : NEV;
            uint64_t ew = e0;
            occ_t o;
            memset(&o, 0, sizeof(o));
            if (it == 1) ew = e0 > warm ? e0 - warm : 0;
            else if (scheme == S_EXIT) { if (c) o = xprev[c - 1]; }
            else if (scheme == S_LIVE) for (uint64_t q = lcnt[c]; q < lcnt[c + 1]; q++) occ_set(&o, prev[live[q]]);
            else {   /* live tokens at the warm-up start (a chunk boundary), then the warm-up replayed */
                const uint64_t cw = c > warm / CH ? c - warm / CH : 0;
                ew = cw * CH;
                for (uint64_t q = lcnt[cw]; q < lcnt[cw + 1]; q++) occ_set(&o, prev[live[q]]);
            }
            uint64_t cc = 0, wrong = 0;
            for (uint64_t k = ew; k < e1; k++) {
                uint32_t s;
                if (EV[k].a) {
                    s = occ_lowest_free(&o);
                    if (EV[k].o) occ_set(&o, s);
                } else {
                    uint32_t m = 0xFFFFu;
                    for (uint32_t q = 0; q < EV[k].ntok; q++) {
                        const uint32_t t = TOK[EV[k].tok0 + q];
                        const uint32_t ts = t < ew ? prev[t] : own[t];
                        occ_clr(&o, ts);
                        if (ts < m) m = ts;
                    }
                    if (EV[k].o) occ_set(&o, m);
                    s = m;
                }
                own[k] = (uint16_t)s;
                if (k >= e0) {
                    next[k] = (uint16_t)s;
                    if (next[k] != prev[k]) cc++;
                    if (s != EV[k].slot) wrong++;
                }
            }
            xnext[c] = o;
            if (cc || (scheme == S_EXIT && !occ_eq(&xnext[c], &xprev[c])) || (ew < e0 && scheme != S_LIVEWARM && it == 1)) changed = 1;
            nchg += cc;
            if (cc > maxchg) maxchg = cc;
            if (wrong) { wrong_chunks++; if (c < first_wrong) first_wrong = c; }
            wrong_ev += wrong;
        }
        printf("%s[%d, %lu, %lu, %lu, %lu, %lu]", it > 1 ? ", " : "", it, (unsigned long)wrong_chunks, (unsigned long)first_wrong,
               (unsigned long)nchg, (unsigned long)maxchg, (unsigned long)wrong_ev);
        uint16_t *t = prev; prev = next; next = t;
        occ_t *x = xprev; xprev = xnext; xnext = x;
        if (!changed) break;
    }
    uint64_t bad = 0;
    for (uint64_t k = 0; k < NEV; k++) bad += prev[k] != EV[k].slot;
    printf("], \"fixed_point_at\": %d, \"wrong_at_end\": %lu}\n", it, (unsigned long)bad);
    fflush(stdout);
    free(prev); free(next); free(own); free(xprev); free(xnext); free(death); free(lcnt); free(live); free(fill);
}

/* longseed: the tokens whose life exceeds `warm` events (or that leak) get
 * their slots first, one after the other, each from a replay of the `warm`
 * events before its allocation seeded with the long tokens alive there
 * (level A); then iteration 1 replays every chunk from `warm` events early
 * seeded the same way, and later iterations take the exit scheme. */
static occ_t LAST_OCC;
static uint32_t replay_window(uint64_t ew, uint64_t e1, const uint32_t *seed_tok, const uint16_t *seed_slot, uint32_t nseed,
                              uint16_t *own, const uint16_t *prev) {
    occ_t o;
    memset(&o, 0, sizeof(o));
    static uint16_t *sslot = NULL;
    static uint64_t cap = 0;
    if (cap < NEV) { free(sslot); sslot = malloc(NEV * 2); cap = NEV; }
    for (uint32_t q = 0; q < nseed; q++) { occ_set(&o, seed_slot[q]); sslot[seed_tok[q]] = seed_slot[q]; }
    uint32_t s = 0;
    for (uint64_t k = ew; k < e1; k++) {
        if (EV[k].a) {
            s = occ_lowest_free(&o);
            if (EV[k].o) occ_set(&o, s);
        } else {
            uint32_t m = 0xFFFFu;
            for (uint32_t q = 0; q < EV[k].ntok; q++) {
                const uint32_t t = TOK[EV[k].tok0 + q];
                uint32_t ts;
                if (t >= ew) ts = own[t];
                else {
                    int seeded = 0;
                    for (uint32_t z = 0; z < nseed; z++) if (seed_tok[z] == t) { seeded = 1; break; }
                    if (!seeded) continue;   /* a ghost: its slot is not in the table */
                    ts = sslot[t];
                }
                occ_clr(&o, ts);
                if (ts < m) m = ts;
            }
            if (EV[k].o && m != 0xFFFFu) occ_set(&o, m);
            s = m;
        }
        own[k] = (uint16_t)s;
    }
    (void)prev;
    LAST_OCC = o;
    return s;
}

static void run_longseed(uint32_t CH, uint32_t warm) {
    uint64_t *death = malloc(NEV * 8);
    for (uint64_t k = 0; k < NEV; k++) death[k] = NEV;   /* never */
    for (uint64_t k = 0; k < NEV; k++)
        for (uint32_t q = 0; q < EV[k].ntok; q++) death[TOK[EV[k].tok0 + q]] = k;
    uint32_t *lt = malloc(NEV * 4), nl = 0;
    for (uint64_t k = 0; k < NEV; k++)
        if (EV[k].o && death[k] - k > warm) lt[nl++] = (uint32_t)k;
    uint16_t *ls = malloc((nl + 1) * 2), *own = calloc(NEV, 2);
    uint32_t *stok = malloc((nl + 1) * 4);
    uint16_t *sslot = malloc((nl + 1) * 2);
    uint64_t wrongA = 0, replayed = 0;
    for (uint32_t j = 0; j < nl; j++) {
        const uint64_t a = lt[j], ew = a > warm ? a - warm : 0;
        uint32_t ns = 0;
        for (uint32_t i = 0; i < j; i++)
            if (lt[i] < ew && death[lt[i]] >= ew) { stok[ns] = lt[i]; sslot[ns] = ls[i]; ns++; }
        ls[j] = (uint16_t)replay_window(ew, a + 1, stok, sslot, ns, own, NULL);
        replayed += a + 1 - ew;
        if (ls[j] != EV[a].slot) wrongA++;
    }
    /* iteration 1: every chunk from warm early, seeded with the long tokens alive there */
    const uint64_t nch = (NEV + CH - 1) / CH;
    occ_t *XP = calloc(nch, sizeof(occ_t)), *XN = calloc(nch, sizeof(occ_t));
    uint16_t *PV = calloc(NEV, 2), *NX = calloc(NEV, 2);
    uint64_t wrong_chunks = 0, wrong_ev = 0, first_wrong = nch;
    for (uint64_t c = 0; c < nch; c++) {
        const uint64_t e0 = c * CH, e1 = e0 + CH < NEV ? e0 + CH : NEV, ew = e0 > warm ? e0 - warm : 0;
        uint32_t ns = 0;
        for (uint32_t i = 0; i < nl; i++)
            if (lt[i] < ew && death[lt[i]] >= ew) { stok[ns] = lt[i]; sslot[ns] = ls[i]; ns++; }
        replay_window(ew, e1, stok, sslot, ns, own, NULL);
        XP[c] = LAST_OCC;
        for (uint64_t k = e0; k < e1; k++) PV[k] = own[k];
        uint64_t w = 0;
        for (uint64_t k = e0; k < e1; k++) w += own[k] != EV[k].slot;
        if (w) { wrong_chunks++; if (c < first_wrong) first_wrong = c; }
        wrong_ev += w;
    }
    printf("{\"scheme\": \"longseed\", \"chunk\": %u, \"warm\": %u, \"events\": %lu, \"long_tokens\": %u, "
           "\"level_a_events\": %lu, \"level_a_wrong\": %lu, \"it1_wrong_chunks\": %lu, \"it1_first_wrong\": %lu, "
           "\"it1_wrong_events\": %lu, \"chunks\": %lu}\n",
           CH, warm, (unsigned long)NEV, nl, (unsigned long)replayed, (unsigned long)wrongA, (unsigned long)wrong_chunks,
           (unsigned long)first_wrong, (unsigned long)wrong_ev, (unsigned long)nch);
    /* then the exit scheme to the fixed point */
    int it;
    for (it = 2; it <= 100000; it++) {
        int changed = 0;
        for (uint64_t c = 0; c < nch; c++) {
            const uint64_t e0 = c * CH, e1 = e0 + CH < NEV ? e0 + CH : NEV;
            occ_t o;
            memset(&o, 0, sizeof(o));
            if (c) o = XP[c - 1];
            uint64_t cc = 0;
            for (uint64_t k = e0; k < e1; k++) {
                uint32_t sl;
                if (EV[k].a) { sl = occ_lowest_free(&o); if (EV[k].o) occ_set(&o, sl); }
                else {
                    uint32_t m = 0xFFFFu;
                    for (uint32_t q = 0; q < EV[k].ntok; q++) {
                        const uint32_t t = TOK[EV[k].tok0 + q];
                        const uint32_t ts = t < e0 ? PV[t] : own[t];
                        occ_clr(&o, ts);
                        if (ts < m) m = ts;
                    }
                    if (EV[k].o) occ_set(&o, m);
                    sl = m;
                }
                own[k] = (uint16_t)sl;
                NX[k] = (uint16_t)sl;
                cc += NX[k] != PV[k];
            }
            XN[c] = o;
            if (cc || !occ_eq(&XN[c], &XP[c])) changed = 1;
        }
        uint16_t *t = PV; PV = NX; NX = t;
        occ_t *x = XP; XP = XN; XN = x;
        if (!changed) break;
    }
    uint64_t bad = 0;
    for (uint64_t k = 0; k < NEV; k++) bad += PV[k] != EV[k].slot;
    printf("{\"longseed_then_exit_fixed_point_at\": %d, \"wrong_at_end\": %lu}\n", it, (unsigned long)bad);
    free(XP); free(XN); free(PV); free(NX);
    free(death); free(lt); free(ls); free(own); free(stok); free(sslot);
}

/* compact: the D-state replay (wg_lanes_serial.hip: a slot holds D = the time
 * its holder is consumed) with leaked slots removed from the slot order — a
 * slot whose token is never consumed stays occupied for good, so the lowest
 * free slot is the lowest free one among the others; positions are ranks among
 * the non-leaked slots, and a leak removes its position (the ones above shift
 * down).  Chunked fixed point on the exit D-vectors (iteration 1 warm-started
 * from empty), then the real slots: S_j = the non-leaked slot indices in order
 * after j leaks, slot(k) = S_{leaks before k}[pos(k)]. */
#define CINF 0x7FFFFFFFu
static uint32_t CWID;   /* compact positions tracked */
static uint32_t cmaxpos;
static uint32_t creplay(uint64_t ew, uint64_t e1, const uint32_t *Din, uint32_t *Dout, uint32_t *pos, const uint64_t *death) {
    static uint32_t *D = NULL;
    if (!D) D = malloc(CWID * 4);
    memcpy(D, Din, CWID * 4);
    uint32_t hi = 0;   /* positions [0, hi) may be nonzero */
    for (uint32_t p = 0; p < CWID; p++) if (D[p]) hi = p + 1;
    for (uint64_t k = ew; k < e1; k++) {
        const uint32_t t = (uint32_t)k + 1;
        uint32_t x = 0xFFFFFFFFu;
        if (EV[k].a) { for (x = 0; x < CWID && D[x] >= t; x++) {} if (x == CWID) x = 0xFFFFFFFFu; }
        else for (uint32_t p = 0; p < hi; p++) if (D[p] == t) { x = p; break; }
        const uint32_t dv = EV[k].o ? (death[k] >= NEV ? CINF : (uint32_t)death[k] + 1) : t;
        pos[k] = x;
        if (x == 0xFFFFFFFFu) continue;
        if (x + 1 > cmaxpos) cmaxpos = x + 1;
        if (dv == CINF) { memmove(D + x, D + x + 1, (CWID - 1 - x) * 4); D[CWID - 1] = 0; if (hi) hi--; if (hi < x) hi = x; }
        else { D[x] = dv; if (x + 1 > hi) hi = x + 1; }
    }
    /* free positions (consumed at or before the last event) all read 0, so a
     * warm-started exit and the exact one compare equal */
    for (uint32_t p = 0; p < CWID; p++) if (D[p] <= (uint32_t)e1) D[p] = 0;
    memcpy(Dout, D, CWID * 4);
    return 0;
}
static void run_compact(uint32_t CH, uint32_t warm) {
    CWID = 1024;
    uint64_t *death = malloc(NEV * 8);
    for (uint64_t k = 0; k < NEV; k++) death[k] = NEV;
    for (uint64_t k = 0; k < NEV; k++)
        for (uint32_t q = 0; q < EV[k].ntok; q++) death[TOK[EV[k].tok0 + q]] = k;
    uint64_t nleak = 0;
    for (uint64_t k = 0; k < NEV; k++) if (EV[k].o && death[k] >= NEV) nleak++;
    const uint64_t nch = (NEV + CH - 1) / CH;
    uint32_t *XP = calloc(nch * CWID, 4), *XN = calloc(nch * CWID, 4);
    uint32_t *PP = malloc(NEV * 4), *PN = malloc(NEV * 4), *zero = calloc(CWID, 4);
    for (uint64_t k = 0; k < NEV; k++) PP[k] = 0xFFFFFFFEu;
    /* the sequential compact replay (for the width and the real-slot check) */
    uint32_t *PS = malloc(NEV * 4), *Dx = malloc(CWID * 4);
    cmaxpos = 0;
    creplay(0, NEV, zero, Dx, PS, death);
    const uint32_t seqw = cmaxpos;
    printf("{\"scheme\": \"compact\", \"chunk\": %u, \"warm\": %u, \"events\": %lu, \"leaks\": %lu, \"compact_width\": %u, \"iters\": [",
           CH, warm, (unsigned long)NEV, (unsigned long)nleak, seqw);
    int it;
    uint32_t *own = malloc(NEV * 4);
    for (it = 1; it <= 100000; it++) {
        int changed = 0;
        uint64_t wrong_chunks = 0, wrong_ev = 0, first_wrong = nch;
        for (uint64_t c = 0; c < nch; c++) {
            const uint64_t e0 = c * CH, e1 = e0 + CH < NEV ? e0 + CH : NEV;
            uint64_t ew = e0;
            const uint32_t *Din = zero;
            if (it == 1) ew = e0 > warm ? e0 - warm : 0;
            else if (c) Din = XP + (c - 1) * CWID;
            creplay(ew, e1, Din, XN + c * CWID, own, death);
            uint64_t w = 0;
            for (uint64_t k = e0; k < e1; k++) { PN[k] = own[k]; if (PN[k] != PP[k]) changed = 1; w += own[k] != PS[k]; }
            if (memcmp(XN + c * CWID, XP + c * CWID, CWID * 4)) changed = 1;
            if (w) { wrong_chunks++; if (c < first_wrong) first_wrong = c; }
            wrong_ev += w;
        }
        printf("%s[%d, %lu, %lu, %lu]", it > 1 ? ", " : "", it, (unsigned long)wrong_chunks, (unsigned long)first_wrong,
               (unsigned long)wrong_ev);
        uint32_t *t = PP; PP = PN; PN = t;
        t = XP; XP = XN; XN = t;
        if (!changed && it > 1) break;
    }
    /* real slots */
    uint32_t *S = malloc((CWID + nleak + 8) * 4);
    for (uint32_t p = 0; p < CWID; p++) S[p] = p;
    uint64_t bad = 0;
    for (uint64_t k = 0; k < NEV; k++) {
        const uint32_t x = PP[k];
        const uint32_t slot = x == 0xFFFFFFFFu ? 0xFFFFu : S[x];
        if (slot != EV[k].slot) bad++;
        if (x != 0xFFFFFFFFu && EV[k].o && death[k] >= NEV) {
            const uint32_t top = S[CWID - 1];
            memmove(S + x, S + x + 1, (CWID - 1 - x) * 4);
            S[CWID - 1] = top + 1;
        }
    }
    printf("], \"fixed_point_at\": %d, \"wrong_slots_at_end\": %lu}\n", it, (unsigned long)bad);
    fflush(stdout);
}

int main(int argc, char **argv) {
    if (argc < 5) { fprintf(stderr, "usage: %s preset rows chunk warm [exit|live ...]\n", argv[0]); return 2; }
    static const char *names[] = {"linear", "random13", "linux", "wide16", "anomaly", "skew", "linuxwide"};
    int kind = -1;
    for (int k = 0; k < 7; k++) if (!strcmp(argv[1], names[k])) kind = k;
    if (kind < 0) return 2;
    wgs_params p;
    wgs_preset(kind, strtoull(argv[2], 0, 10), 0x5EED + kind, &p);
    wgs_dag *d = wgs_generate(&p);
    build_events(d);
    const uint32_t CH = (uint32_t)atoi(argv[3]), warm = (uint32_t)atoi(argv[4]);
    if (!strcmp(argv[5 < argc ? 5 : 0], "lifetimes")) {   /* histogram of consumption distance (events) */
        uint64_t h[8] = {0}, leaked = 0, occupying = 0, cev = 0;
        static const uint64_t lim[8] = {1, 2, 4, 8, 16, 64, 256, ~0ull};
        uint64_t *death = malloc(NEV * 8);
        for (uint64_t k = 0; k < NEV; k++) death[k] = ~0ull;
        for (uint64_t k = 0; k < NEV; k++) { if (EV[k].ntok) cev++; for (uint32_t q = 0; q < EV[k].ntok; q++) death[TOK[EV[k].tok0 + q]] = k; }
        for (uint64_t k = 0; k < NEV; k++) {
            if (!EV[k].o) continue;
            occupying++;
            if (death[k] == ~0ull) { leaked++; continue; }
            const uint64_t dl = death[k] - k;
            for (int b = 0; b < 8; b++) if (dl <= lim[b]) { h[b]++; break; }
        }
        printf("{\"events\": %lu, \"c_events\": %lu, \"occupying\": %lu, \"leaked\": %lu, \"life_le\": {\"1\": %lu, \"2\": %lu, \"4\": %lu, \"8\": %lu, \"16\": %lu, \"64\": %lu, \"256\": %lu, \"more\": %lu}}\n",
               (unsigned long)NEV, (unsigned long)cev, (unsigned long)occupying, (unsigned long)leaked, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7]);
        return 0;
    }
    if (argc > 5 && !strcmp(argv[5], "wordhist")) {   /* which 64-slot word each event's slot lies in */
        uint64_t h[2][17] = {{0}};
        for (uint64_t k = 0; k < NEV; k++) { const uint32_t w = EV[k].slot / 64; h[EV[k].a ? 0 : 1][w < 16 ? w : 16]++; }
        for (int t = 0; t < 2; t++) {
            printf("%s:", t ? "consume" : "alloc");
            for (int w = 0; w < 17; w++) if (h[t][w]) printf(" w%d=%lu", w, (unsigned long)h[t][w]);
            printf("\n");
        }
        wgs_free(d);
        return 0;
    }
    if (argc > 5 && !strcmp(argv[5], "compact")) { run_compact(CH, warm); wgs_free(d); return 0; }
    if (argc > 5 && !strcmp(argv[5], "longseed")) { run_longseed(CH, warm); wgs_free(d); return 0; }
    for (int a = 5; a < argc || a == 5; a++) {
        const char *s = a < argc ? argv[a] : "exit";
        run(s, !strcmp(s, "live") ? S_LIVE : !strcmp(s, "livewarm") ? S_LIVEWARM : S_EXIT, CH, warm);
        if (a >= argc) break;
    }
    wgs_free(d);
    return 0;
}
