/*
 * edt_cpu.c — CPU baseline for BASELINE config C2 (TEST / BENCH
 * INFRASTRUCTURE, never part of the engine): the WG-SDF-1 distance pass of
 * the font atlas as a native exact Felzenszwalb–Huttenlocher
 * EDT — the CPU path BASELINE.md §2 plans for C2 ("C++ Felzenszwalb–
 * Huttenlocher EDT, 1 thread and all cores").  The reference's own
 * fontdue → EDT atlas is gone from its tree (legacy docs/render_engine.md:
 * 105-112 only), so there is no reference code to compile for it.
 *
 * Input: the atlas coverage (inside <=> coverage >= 8 of 16 samples).
 * Output: squared distances to the nearest pixel of the other class, capped
 * at far = (4*spread + 1)^2 (an exact EDT then min(d2, far) equals the
 * engine's window-bounded EDT: any distance below far is found inside the
 * window), and the R8 SDF byte
 *   floor(clamp(127.5 - (sqrt(d2_out) - sqrt(d2_in)) * (127.5 / spread), 0, 255) + 0.5)
 * in f32 — byte-identical to the engine's atlas (bench.py checks it).
 *
 * Pass 1: per column, distance to the nearest feature pixel (two sweeps).
 * Pass 2: per row, the lower envelope of the parabolas g(q) + (x - q)^2
 * (Felzenszwalb & Huttenlocher 2012, "Distance Transforms of Sampled
 * Functions"), exact in integers.  OpenMP over columns / rows.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#define EDT_INF (1ll << 40)

/* one row: f[0..n) squared column distances (EDT_INF = no feature) -> d[0..n) */
static void fh_row(const int64_t *f, int64_t *d, int n, int *v, double *z) {
    int k = -1;
    for (int q = 0; q < n; q++) {
        if (f[q] >= EDT_INF) continue;
        double s = 0.0;
        while (k >= 0) {
            const int p = v[k];
            s = ((double)(f[q] + (int64_t)q * q) - (double)(f[p] + (int64_t)p * p)) / (2.0 * (q - p));
            if (s <= z[k]) k--;
            else break;
        }
        k++;
        v[k] = q;
        z[k] = k == 0 ? -HUGE_VAL : s;
        z[k + 1] = HUGE_VAL;
    }
    if (k < 0) {
        for (int q = 0; q < n; q++) d[q] = EDT_INF;
        return;
    }
    int j = 0;
    for (int q = 0; q < n; q++) {
        while (z[j + 1] < (double)q) j++;
        const int64_t dx = q - v[j];
        d[q] = f[v[j]] + dx * dx;
    }
}

/* squared EDT of `feature` (1 = feature pixel), capped at cap, into out (u16) */
static void edt(const uint8_t *feature, int W, int H, int64_t cap, uint16_t *out, int threads) {
    int64_t *g = (int64_t *)malloc((size_t)W * H * sizeof(int64_t));
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int x = 0; x < W; x++) {
        int64_t dist = EDT_INF;
        for (int y = 0; y < H; y++) {
            dist = feature[(size_t)y * W + x] ? 0 : (dist >= EDT_INF ? EDT_INF : dist + 1);
            g[(size_t)y * W + x] = dist;
        }
        dist = EDT_INF;
        for (int y = H - 1; y >= 0; y--) {
            dist = feature[(size_t)y * W + x] ? 0 : (dist >= EDT_INF ? EDT_INF : dist + 1);
            int64_t *c = &g[(size_t)y * W + x];
            if (dist < *c) *c = dist;
            if (*c < EDT_INF) *c = *c * *c;
        }
    }
#pragma omp parallel num_threads(threads)
    {
        int64_t *f = (int64_t *)malloc((size_t)W * sizeof(int64_t));
        int64_t *d = (int64_t *)malloc((size_t)W * sizeof(int64_t));
        int *v = (int *)malloc((size_t)W * sizeof(int));
        double *z = (double *)malloc(((size_t)W + 1) * sizeof(double));
#pragma omp for schedule(static)
        for (int y = 0; y < H; y++) {
            memcpy(f, &g[(size_t)y * W], (size_t)W * sizeof(int64_t));
            fh_row(f, d, W, v, z);
            for (int x = 0; x < W; x++) out[(size_t)y * W + x] = (uint16_t)(d[x] < cap ? d[x] : cap);
        }
        free(f); free(d); free(v); free(z);
    }
    free(g);
}

/* WG-SDF-1 distances + SDF bytes of one atlas; returns 0 */
int edt_cpu_sdf(const uint8_t *cov, int W, int H, int spread, int threads, uint16_t *d2in, uint16_t *d2out,
                uint8_t *sdf) {
    if (threads < 1) threads = 1;
    const int64_t R = 4 * (int64_t)spread, cap = (R + 1) * (R + 1);
    uint8_t *outside = (uint8_t *)malloc((size_t)W * H), *inside = (uint8_t *)malloc((size_t)W * H);
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int i = 0; i < W * H; i++) {
        inside[i] = cov[i] >= 8;
        outside[i] = !inside[i];
    }
    edt(outside, W, H, cap, d2in, threads);    /* inside pixels: to the nearest outside pixel */
    edt(inside, W, H, cap, d2out, threads);
    const float k = 127.5f / (float)spread;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int i = 0; i < W * H; i++) {
        const float signed_d = sqrtf((float)d2out[i]) - sqrtf((float)d2in[i]);
        float v = 127.5f - signed_d * k;
        v = v < 0.0f ? 0.0f : (v > 255.0f ? 255.0f : v);
        sdf[i] = (uint8_t)floorf(v + 0.5f);
    }
    free(outside);
    free(inside);
    return 0;
}
