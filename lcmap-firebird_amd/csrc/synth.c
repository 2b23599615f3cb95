/* synth.c -- deterministic synthetic Landsat ARD chips (see include/ccdsynth.h).
 *
 * Input generator for benchmarks and parity tests only: it stands in for the chipmunk/merlin
 * fetch of ccdc/timeseries.py:120 (merlin.create), which needs network services.  Cadence and
 * class mix follow SURVEY.md §8(d).  Counter-based hashing (splitmix64 finaliser) makes every
 * sample a pure function of (seed, chip, pixel, obs, stream).
 */
#include "ccdsynth.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#define ORD_L4_START 723868 /* 1982-11-19 */
#define ORD_L4_END   727911 /* 1993-12-14 */
#define ORD_L5_START 724336 /* 1984-03-01 */
#define ORD_L5_END   734459 /* 2011-11-18 */
#define ORD_L7_START 729859 /* 1999-04-15 */
#define ORD_SLC_OFF  731366 /* 2003-05-31 */
#define ORD_L8_START 734969 /* 2013-04-11 */
#define ORD_END      736694 /* 2017-12-31 */

static const double TWO_PI = 6.283185307179586476925286766559;

static inline uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint64_t hash5(uint64_t seed, uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    uint64_t h = mix64(seed ^ 0x5851F42D4C957F2Dull);
    h = mix64(h ^ a);
    h = mix64(h ^ (b * 0x2545F4914F6CDD1Dull));
    h = mix64(h ^ (c * 0x9E3779B97F4A7C15ull));
    return mix64(h ^ (d * 0xD6E8FEB86659FD93ull));
}
static inline double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
static inline double gauss(uint64_t h) {
    double u1 = u01(h), u2 = u01(mix64(h));
    if (u1 < 1e-300) u1 = 1e-300;
    return sqrt(-2.0 * log(u1)) * cos(TWO_PI * u2);
}

static const double BASE[7] = {500, 800, 700, 2800, 2000, 1200, 2900};
static const double AMP[7] = {150, 200, 250, 600, 400, 300, 150};
static const double SIG[7] = {40, 50, 60, 150, 120, 90, 30};

enum { S_PIXEL = 1, S_CLASS = 2, S_NOISE = 3, S_BREAK = 4, S_DATE = 5, S_EXTRA = 6 };

int ccdsynth_config(int which, ccdsynth_cfg *c) {
    memset(c, 0, sizeof(*c));
    c->first_year_l4 = 1;
    c->p_clear = 0.55; c->p_cloud = 0.25; c->p_shadow = 0.08; c->p_snow = 0.04;
    c->p_water = 0.03; c->p_fill = 0.05;
    c->p_saturated = 0.003; c->p_hot_thermal = 0.001;
    c->seed = 20260101ull;
    switch (which) {
    case 2: c->n_obs_target = 1000; break;
    case 3: c->sidelap = 1; break;
    case 4:
        c->n_obs_target = 1000;
        c->p_clear = 0.25; c->p_cloud = 0.45; c->p_shadow = 0.0; c->p_snow = 0.20;
        c->p_water = 0.0; c->p_fill = 0.10; c->p_hot_thermal = 0.004;
        break;
    case 5: c->sidelap = 1; c->change_every_days = 1096; break;
    default: return -1;
    }
    return 0;
}

static int cmp_i64(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

int ccdsynth_dates(const ccdsynth_cfg *cfg, int32_t chip, int64_t *out, int32_t cap) {
    /* 16-day repeats: phase 0 = L4/L7, phase 8 = L5/L8; sidelap path +7 d on half the chips (the
     * sidelap acquisitions are per path, so every sidelap chip shares one date vector). */
    int64_t *buf = (int64_t *)malloc(sizeof(int64_t) * 8192);
    int n = 0;
    int side = cfg->sidelap && (mix64(cfg->seed ^ (uint64_t)chip * 77ull) & 1ull);
    for (int64_t d = ORD_L4_START; d <= ORD_END; d += 8) {
        int phase8 = (int)((d - ORD_L4_START) % 16) == 8;
        int on = 0;
        if (!phase8) on = (cfg->first_year_l4 && d <= ORD_L4_END) || d >= ORD_L7_START;
        else on = (d >= ORD_L5_START && d <= ORD_L5_END) || d >= ORD_L8_START;
        if (!on) continue;
        buf[n++] = d;
        if (side && d + 7 <= ORD_END && (hash5(cfg->seed, S_DATE, 0, (uint64_t)d, 0) & 1ull))
            buf[n++] = d + 7;
    }
    qsort(buf, (size_t)n, sizeof(int64_t), cmp_i64);
    if (cfg->n_obs_target > 0 && n > cfg->n_obs_target) {
        /* keep the n_obs_target dates with the smallest per-date hash key */
        uint64_t *key = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
        uint64_t *srt = (uint64_t *)malloc(sizeof(uint64_t) * (size_t)n);
        for (int i = 0; i < n; ++i) key[i] = srt[i] = hash5(cfg->seed, S_DATE, (uint64_t)chip, (uint64_t)buf[i], 1);
        /* threshold = n_obs_target-th smallest key (keys distinct with overwhelming probability) */
        for (int i = 1; i < n; ++i) { /* insertion sort is fine for ~3k keys */
            uint64_t k = srt[i]; int j = i - 1;
            while (j >= 0 && srt[j] > k) { srt[j + 1] = srt[j]; --j; }
            srt[j + 1] = k;
        }
        uint64_t thr = srt[cfg->n_obs_target - 1];
        int m = 0;
        for (int i = 0; i < n; ++i) if (key[i] <= thr) buf[m++] = buf[i];
        n = m;
        free(key); free(srt);
    }
    if (out) {
        int k = n < cap ? n : cap;
        for (int i = 0; i < k; ++i) out[i] = buf[n - 1 - i]; /* descending, as merlin delivers */
    }
    free(buf);
    return n;
}

static inline int16_t clip16(double v, double lo, double hi) {
    if (v < lo) v = lo;
    if (v > hi) v = hi;
    return (int16_t)lrint(v);
}

int ccdsynth_chip(const ccdsynth_cfg *cfg, int32_t chip, int32_t pix0, int32_t n_pix, int32_t n_obs,
                  const int64_t *dates, int16_t *spectra, uint16_t *qa) {
    const double w = TWO_PI / 365.2425;
    const uint64_t seed = cfg->seed;
#pragma omp parallel for schedule(static)
    for (int32_t pi = 0; pi < n_pix; ++pi) {
        const int32_t pix = pix0 + pi;
        const int32_t col = pix % 100;
        double base[7], amp[7], slope[7], phase[7];
        for (int b = 0; b < 7; ++b) {
            base[b] = BASE[b] * (0.8 + 0.4 * u01(hash5(seed, S_PIXEL, chip, pix, b)));
            amp[b] = AMP[b] * (0.5 + u01(hash5(seed, S_PIXEL, chip, pix, 10 + b)));
            slope[b] = (u01(hash5(seed, S_PIXEL, chip, pix, 20 + b)) - 0.5) * 1e-5 * BASE[b];
            phase[b] = 0.6 * (u01(hash5(seed, S_PIXEL, chip, pix, 30)) - 0.5)
                       + 0.1 * (u01(hash5(seed, S_PIXEL, chip, pix, 40 + b)) - 0.5);
        }
        /* break schedule (C5): first break 1-3 yr after the series start, then every ~N d +-0.5 yr */
        double brk_t[24]; double brk_step[24][7]; int n_brk = 0;
        if (cfg->change_every_days > 0) {
            double t = ORD_L4_START + 365.0 + 730.0 * u01(hash5(seed, S_BREAK, chip, pix, 999));
            while (t < ORD_END && n_brk < 24) {
                brk_t[n_brk] = t;
                for (int b = 0; b < 7; ++b) {
                    /* step of 25-100 % of the band's base level, signed back toward the undisturbed
                     * level so the cumulative shift stays inside the valid (0, 10000) range */
                    uint64_t h = hash5(seed, S_BREAK, chip, pix, (uint64_t)(n_brk * 16 + b));
                    double mag = (0.25 + 0.75 * u01(h)) * (b == 6 ? 0.05 * BASE[b] : base[b]);
                    double cum = 0.0;
                    for (int k = 0; k < n_brk; ++k) cum += brk_step[k][b];
                    int up = cum < 0.0 || (cum == 0.0 && (mix64(h) & 1ull));
                    brk_step[n_brk][b] = up ? mag : -mag;
                }
                ++n_brk;
                t += cfg->change_every_days + 365.0 * (u01(hash5(seed, S_BREAK, chip, pix, 5000 + n_brk)) - 0.5);
            }
        }
        for (int32_t i = 0; i < n_obs; ++i) {
            const int64_t d = dates[i];
            const double td = (double)d;
            const int ph = (int)((d - ORD_L4_START) % 16);
            const int l8 = (ph == 8 || ph == 15) && d >= ORD_L8_START;
            const int l7 = (ph == 0 || ph == 7) && d >= ORD_L7_START;
            double v[7];
            for (int b = 0; b < 7; ++b) {
                double s = 0.0;
                for (int k = 0; k < n_brk; ++k) if (td >= brk_t[k]) s += brk_step[k][b];
                v[b] = base[b] + amp[b] * cos(w * td + phase[b]) + slope[b] * (td - ORD_L4_START) + s
                       + SIG[b] * gauss(hash5(seed, S_NOISE, chip, ((uint64_t)pix << 20) | (uint64_t)i, b));
            }
            /* snow is winter weighted: peak near day-of-year 15 */
            double doy_phase = cos(w * (td - 15.0));
            double p_snow = cfg->p_snow * (1.0 + doy_phase);
            double p_clear = cfg->p_clear - (p_snow - cfg->p_snow);
            if (p_clear < 0) p_clear = 0;
            double u = u01(hash5(seed, S_CLASS, chip, pix, (uint64_t)i));
            double ue = u01(hash5(seed, S_EXTRA, chip, pix, (uint64_t)i));
            uint16_t q;
            int fill = 0;
            if (l7 && d >= ORD_SLC_OFF && ((col + (int)(d / 16)) % 9) < 2) fill = 1; /* SLC-off stripes */
            double c0 = cfg->p_fill, c1 = c0 + p_clear, c2 = c1 + cfg->p_cloud, c3 = c2 + cfg->p_shadow,
                   c4 = c3 + p_snow;
            const uint16_t l8b = l8 ? 256 : 0;
            if (fill || u < c0) {
                q = 1;
                for (int b = 0; b < 7; ++b) v[b] = -9999.0;
            } else if (u < c1) {
                q = (uint16_t)(66 + l8b);
                if (l8 && ue < 0.01) q = 832;       /* bits 6,8,9: cirrus rule -> clear */
                else if (l8 && ue < 0.015) q = 1088; /* bits 6,10: occlusion -> clear */
                if (ue > 1.0 - cfg->p_saturated) v[(int)(ue * 1e6) % 6] = 20000.0;
                else if (ue > 1.0 - cfg->p_saturated - cfg->p_hot_thermal) v[6] = 3300.0 + 200.0 * u01(mix64((uint64_t)i + pix));
            } else if (u < c2) {
                q = (uint16_t)(224 + l8b);
                for (int b = 0; b < 6; ++b) v[b] += 2500.0 + 500.0 * gauss(hash5(seed, S_EXTRA, chip, pix, (uint64_t)i * 8 + b));
                v[6] -= 300.0;
            } else if (u < c3) {
                q = (uint16_t)(72 + l8b);
                for (int b = 0; b < 6; ++b) v[b] *= 0.5;
            } else if (u < c4) {
                q = (uint16_t)(80 + l8b);
                v[0] += 5000; v[1] += 5000; v[2] += 5000; v[3] += 3500; v[4] = 300 + v[4] * 0.05;
                v[5] = 200 + v[5] * 0.05; v[6] -= 250;
            } else {
                q = (uint16_t)(68 + l8b);
                v[3] *= 0.2; v[4] *= 0.2; v[5] *= 0.2;
            }
            for (int b = 0; b < 7; ++b)
                spectra[((size_t)b * (size_t)n_pix + (size_t)pi) * (size_t)n_obs + (size_t)i] =
                    (v[b] == -9999.0) ? (int16_t)-9999 : clip16(v[b], -2000.0, 32000.0);
            qa[(size_t)pi * (size_t)n_obs + (size_t)i] = q;
        }
    }
    return 0;
}
