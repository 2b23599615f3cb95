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
#include <emmintrin.h>

#include "synth_core.h"

/* dst = src (n bytes) with streaming (non-temporal) 16-byte stores: the destination is a pinned
 * upload buffer the CPU will not read again, so its lines are not fetched before being written
 * (a plain copy of a few-KB row costs a read of the destination line per line written) */
static void copy_stream(void *dst, const void *src, size_t n) {
    char *d = (char *)dst;
    const char *s = (const char *)src;
    const size_t head = (16 - ((uintptr_t)d & 15)) & 15;
    if (n < 64 + head) {
        memcpy(d, s, n);
        return;
    }
    memcpy(d, s, head);
    d += head, s += head, n -= head;
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
        const __m128i a = _mm_loadu_si128((const __m128i *)(s + i));
        const __m128i b = _mm_loadu_si128((const __m128i *)(s + i + 16));
        const __m128i c = _mm_loadu_si128((const __m128i *)(s + i + 32));
        const __m128i e = _mm_loadu_si128((const __m128i *)(s + i + 48));
        _mm_stream_si128((__m128i *)(d + i), a);
        _mm_stream_si128((__m128i *)(d + i + 16), b);
        _mm_stream_si128((__m128i *)(d + i + 32), c);
        _mm_stream_si128((__m128i *)(d + i + 48), e);
    }
    memcpy(d + i, s + i, n - i);
}

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

int ccdsynth_chip(const ccdsynth_cfg *cfg, int32_t chip, int32_t pix0, int32_t n_pix, int32_t n_obs,
                  const int64_t *dates, int16_t *spectra, uint16_t *qa) {
#pragma omp parallel for schedule(static)
    for (int32_t pi = 0; pi < n_pix; ++pi) {
        const int32_t pix = pix0 + pi;
        double base[7], amp[7], slope[7], phase[7];
        for (int b = 0; b < 7; ++b) syn_pixel_band(cfg->seed, chip, pix, b, &base[b], &amp[b], &slope[b], &phase[b]);
        double brk_t[SYN_MAX_BREAKS], brk_step[SYN_MAX_BREAKS * 7];
        const int n_brk = syn_breaks(cfg, chip, pix, base, brk_t, brk_step);
        for (int32_t i = 0; i < n_obs; ++i) {
            int16_t v[7];
            const uint16_t q = syn_obs(cfg, chip, pix, i, dates[i], base, amp, slope, phase, n_brk, brk_t, brk_step, v);
            for (int b = 0; b < 7; ++b) spectra[((size_t)b * (size_t)n_pix + (size_t)pi) * (size_t)n_obs + (size_t)i] = v[b];
            qa[(size_t)pi * (size_t)n_obs + (size_t)i] = q;
        }
    }
    return 0;
}

int ccdsynth_rotate(const int16_t *spectra, const uint16_t *qa, int32_t n_pix, int32_t n_obs, int32_t shift,
                    int16_t *spectra_out, uint16_t *qa_out, int32_t threads) {
    if (n_pix <= 0 || n_obs <= 0 || !spectra || !qa || !spectra_out || !qa_out) return -1;
    const int32_t k = ((shift % n_obs) + n_obs) % n_obs;
    if (k == 0) {
        /* a plain copy: both arrays in large contiguous pieces, one per thread, streamed */
        const size_t ns = (size_t)7 * (size_t)n_pix * (size_t)n_obs * sizeof(int16_t);
        const size_t nq = (size_t)n_pix * (size_t)n_obs * sizeof(uint16_t);
        const int nt = threads > 0 ? threads : 1;
        const size_t piece = ((ns + nq) / (size_t)nt + 4095) & ~(size_t)4095;
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int t = 0; t < nt; ++t) {
            size_t a = (size_t)t * piece, e = a + piece;
            if (e > ns + nq) e = ns + nq;
            if (a >= e) continue;
            if (a < ns) copy_stream((char *)spectra_out + a, (const char *)spectra + a, (e < ns ? e : ns) - a);
            if (e > ns) {
                const size_t qa0 = a > ns ? a - ns : 0;
                copy_stream((char *)qa_out + qa0, (const char *)qa + qa0, e - ns - qa0);
            }
            _mm_sfence();  /* this thread's streaming stores are visible before the upload reads them */
        }
        return 0;
    }
    const size_t rows = (size_t)8 * (size_t)n_pix;  /* 7 band rows + the qa row per pixel */
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1)
    for (long long r = 0; r < (long long)rows; ++r) {
        const size_t o = (size_t)(r % n_pix) * (size_t)n_obs;
        const int b = (int)(r / n_pix);
        if (b < 7) {
            const int16_t *src = spectra + (size_t)b * (size_t)n_pix * (size_t)n_obs + o;
            int16_t *dst = spectra_out + (size_t)b * (size_t)n_pix * (size_t)n_obs + o;
            memcpy(dst, src + k, sizeof(int16_t) * (size_t)(n_obs - k));
            memcpy(dst + (n_obs - k), src, sizeof(int16_t) * (size_t)k);
        } else {
            memcpy(qa_out + o, qa + o + k, sizeof(uint16_t) * (size_t)(n_obs - k));
            memcpy(qa_out + o + (n_obs - k), qa + o, sizeof(uint16_t) * (size_t)k);
        }
    }
    return 0;
}
