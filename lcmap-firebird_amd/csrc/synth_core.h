/* synth_core.h -- the per-value arithmetic of the synthetic ARD generator, shared by the host
 * generator (synth.c, gcc) and the device generator (ccd_synth.hip, hipcc), so both compute
 * every sample with the same operations in the same order (both built without FMA contraction).
 * The only inputs that can differ are the math library's cos / log results (glibc vs the ROCm
 * device library, <= 1-2 ulp apart); an int16 sample rounds the same unless its value lies within
 * ~1e-12 of a half-integer, so the two generators agree to the bit on practically every sample
 * (tests/test_gpu_synth.py checks whole chips).  See include/ccdsynth.h.
 */
#ifndef CCD_SYNTH_CORE_H
#define CCD_SYNTH_CORE_H
#include <math.h>
#include <stdint.h>

#include "ccdsynth.h"

#ifdef __HIPCC__
#define SYN_FN __host__ __device__ static inline
#else
#define SYN_FN static inline
#endif

#define ORD_L4_START 723868 /* 1982-11-19 */
#define ORD_L4_END   727911 /* 1993-12-14 */
#define ORD_L5_START 724336 /* 1984-03-01 */
#define ORD_L5_END   734459 /* 2011-11-18 */
#define ORD_L7_START 729859 /* 1999-04-15 */
#define ORD_SLC_OFF  731366 /* 2003-05-31 */
#define ORD_L8_START 734969 /* 2013-04-11 */
#define ORD_END      736694 /* 2017-12-31 */
#define SYN_MAX_BREAKS 24

#define SYN_TWO_PI 6.283185307179586476925286766559

enum { S_PIXEL = 1, S_CLASS = 2, S_NOISE = 3, S_BREAK = 4, S_DATE = 5, S_EXTRA = 6 };

SYN_FN uint64_t mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
SYN_FN uint64_t hash5(uint64_t seed, uint64_t a, uint64_t b, uint64_t c, uint64_t d) {
    uint64_t h = mix64(seed ^ 0x5851F42D4C957F2Dull);
    h = mix64(h ^ a);
    h = mix64(h ^ (b * 0x2545F4914F6CDD1Dull));
    h = mix64(h ^ (c * 0x9E3779B97F4A7C15ull));
    return mix64(h ^ (d * 0xD6E8FEB86659FD93ull));
}
SYN_FN double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
SYN_FN double gauss(uint64_t h) {
    double u1 = u01(h), u2 = u01(mix64(h));
    if (u1 < 1e-300) u1 = 1e-300;
    return sqrt(-2.0 * log(u1)) * cos(SYN_TWO_PI * u2);
}

SYN_FN double syn_base(int b) {
    return b == 0 ? 500 : b == 1 ? 800 : b == 2 ? 700 : b == 3 ? 2800 : b == 4 ? 2000 : b == 5 ? 1200 : 2900;
}
SYN_FN double syn_amp(int b) {
    return b == 0 ? 150 : b == 1 ? 200 : b == 2 ? 250 : b == 3 ? 600 : b == 4 ? 400 : b == 5 ? 300 : 150;
}
SYN_FN double syn_sig(int b) {
    return b == 0 ? 40 : b == 1 ? 50 : b == 2 ? 60 : b == 3 ? 150 : b == 4 ? 120 : b == 5 ? 90 : 30;
}

/* per-pixel level, seasonal amplitude, trend and phase of band b */
SYN_FN void syn_pixel_band(uint64_t seed, int32_t chip, int32_t pix, int b, double *base, double *amp, double *slope,
                           double *phase) {
    *base = syn_base(b) * (0.8 + 0.4 * u01(hash5(seed, S_PIXEL, chip, pix, b)));
    *amp = syn_amp(b) * (0.5 + u01(hash5(seed, S_PIXEL, chip, pix, 10 + b)));
    *slope = (u01(hash5(seed, S_PIXEL, chip, pix, 20 + b)) - 0.5) * 1e-5 * syn_base(b);
    *phase = 0.6 * (u01(hash5(seed, S_PIXEL, chip, pix, 30)) - 0.5) + 0.1 * (u01(hash5(seed, S_PIXEL, chip, pix, 40 + b)) - 0.5);
}

/* Break schedule (C5): first break 1-3 yr after the series start, then every ~N d +- 0.5 yr.
 * brk_t[k] = break day, step(k, b) = brk_step[k * 7 + b]; base[b] = the pixel's band levels.
 * Returns the number of breaks (0 without change_every_days). */
SYN_FN int syn_breaks(const ccdsynth_cfg *cfg, int32_t chip, int32_t pix, const double *base, double *brk_t,
                      double *brk_step) {
    const uint64_t seed = cfg->seed;
    int n_brk = 0;
    if (cfg->change_every_days <= 0) return 0;
    double t = ORD_L4_START + 365.0 + 730.0 * u01(hash5(seed, S_BREAK, chip, pix, 999));
    while (t < ORD_END && n_brk < SYN_MAX_BREAKS) {
        brk_t[n_brk] = t;
        for (int b = 0; b < 7; ++b) {
            /* step of 25-100 % of the band's base level, signed back toward the undisturbed
             * level so the cumulative shift stays inside the valid (0, 10000) range */
            uint64_t h = hash5(seed, S_BREAK, chip, pix, (uint64_t)(n_brk * 16 + b));
            double mag = (0.25 + 0.75 * u01(h)) * (b == 6 ? 0.05 * syn_base(b) : base[b]);
            double cum = 0.0;
            for (int k = 0; k < n_brk; ++k) cum += brk_step[k * 7 + b];
            int up = cum < 0.0 || (cum == 0.0 && (mix64(h) & 1ull));
            brk_step[n_brk * 7 + b] = up ? mag : -mag;
        }
        ++n_brk;
        t += cfg->change_every_days + 365.0 * (u01(hash5(seed, S_BREAK, chip, pix, 5000 + n_brk)) - 0.5);
    }
    return n_brk;
}

SYN_FN int16_t clip16(double v, double lo, double hi) {
    if (v < lo) v = lo;
    if (v > hi) v = hi;
    return (int16_t)lrint(v);
}

/* Observation i (date d) of pixel pix: the 7 band values (out[b]) and the QA word. */
SYN_FN uint16_t syn_obs(const ccdsynth_cfg *cfg, int32_t chip, int32_t pix, int32_t i, int64_t d, const double *base,
                        const double *amp, const double *slope, const double *phase, int n_brk, const double *brk_t,
                        const double *brk_step, int16_t *out) {
    const double w = SYN_TWO_PI / 365.2425;
    const uint64_t seed = cfg->seed;
    const int32_t col = pix % 100;
    const double td = (double)d;
    const int ph = (int)((d - ORD_L4_START) % 16);
    const int l8 = (ph == 8 || ph == 15) && d >= ORD_L8_START;
    const int l7 = (ph == 0 || ph == 7) && d >= ORD_L7_START;
    double v[7];
    for (int b = 0; b < 7; ++b) {
        double s = 0.0;
        for (int k = 0; k < n_brk; ++k)
            if (td >= brk_t[k]) s += brk_step[k * 7 + b];
        v[b] = base[b] + amp[b] * cos(w * td + phase[b]) + slope[b] * (td - ORD_L4_START) + s +
               syn_sig(b) * gauss(hash5(seed, S_NOISE, chip, ((uint64_t)pix << 20) | (uint64_t)i, b));
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
    double c0 = cfg->p_fill, c1 = c0 + p_clear, c2 = c1 + cfg->p_cloud, c3 = c2 + cfg->p_shadow, c4 = c3 + p_snow;
    const uint16_t l8b = l8 ? 256 : 0;
    if (fill || u < c0) {
        q = 1;
        for (int b = 0; b < 7; ++b) v[b] = -9999.0;
    } else if (u < c1) {
        q = (uint16_t)(66 + l8b);
        if (l8 && ue < 0.01) q = 832;        /* bits 6,8,9: cirrus rule -> clear */
        else if (l8 && ue < 0.015) q = 1088; /* bits 6,10: occlusion -> clear */
        if (ue > 1.0 - cfg->p_saturated) {
            const int sb = (int)(ue * 1e6) % 6;  /* (a constant-index loop: no dynamically indexed array) */
            for (int b = 0; b < 6; ++b) v[b] = b == sb ? 20000.0 : v[b];
        }
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
    for (int b = 0; b < 7; ++b) out[b] = (v[b] == -9999.0) ? (int16_t)-9999 : clip16(v[b], -2000.0, 32000.0);
    return q;
}

#endif
