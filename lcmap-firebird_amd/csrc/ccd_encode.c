/* ccd_encode.c -- transport encoding of ARD chips for the PCIe upload (host side).
 *
 * The tile path is bound by the host-to-device link (16 bytes per observation: 7 int16 bands +
 * a uint16 QA word).  The encoding sends less of it:
 *   - the band values of an observation whose QA word has any of `drop_bits` set are not sent;
 *     the device writes -9999 (the ARD fill value) in their place.  With drop_bits = the fill bit
 *     (and strict_bits = the same: such an observation must hold -9999 in every band, or its chip
 *     goes raw) the encoding is lossless.  With the fill, cloud and shadow bits it drops values
 *     the detection never reads: pyccd's procedures (qa.standard_procedure_filter and the snow
 *     and insufficient-clear filters) keep only clear / water (/ snow) observations -- the class
 *     qabitval gives a word, fill > cloud > shadow > snow > water > clear -- so a word with the
 *     fill, cloud or shadow bit is never in a processing mask and its band values never enter a
 *     test or a fit (px_setup in ccd_kernels.hip: keep = class clear or water (or snow) and the
 *     range tests), and the results are the same (tests/test_gpu_encode.py, test_gpu_tile.py);
 *   - a chip's QA words take a handful of distinct values: each becomes a 4-bit index into a
 *     16-entry palette (a chip with more distinct words is sent raw, mode 0).
 * The device decoder (ccd_decode_enc in ccd_pack.hip) rebuilds the standard band-major
 * [7][n_pix][n_obs] spectra and [n_pix][n_obs] QA of every chip (tests/test_encode.py: round
 * trips against a numpy decoder).  Layout: include/ccdgpu.h.
 *
 * The encode replaces the copy into pinned memory that every upload from a fetched (pageable)
 * chip needs anyway; it runs one pass over the QA words (counts, palette, fill check) and one
 * over the bands (stream compaction: AVX-512 VBMI2 compress-store where the CPU has it).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ccdgpu.h"
#ifdef _OPENMP
#include <omp.h>
#endif

#define ENC_HDR 128
#define ENC_ALIGN 256

static size_t up(size_t x, size_t a) { return (x + a - 1) / a * a; }

/* bytes of a chip section in mode 1 for kept observations, and in mode 0 */
static size_t sec_mode1(int64_t n_pix, int64_t n_obs, int64_t kept) {
    return ENC_HDR + up(4 * (size_t)(n_pix + 1), 16) + up((size_t)n_pix * (size_t)((n_obs + 1) / 2), 16) +
           7 * 2 * up((size_t)kept, 8);
}
static size_t sec_mode0(int64_t n_pix, int64_t n_obs) {
    const size_t d = (size_t)n_pix * (size_t)n_obs;
    return ENC_HDR + up(2 * d, 16) + 7 * 2 * d;
}
static size_t table_bytes(int32_t n_chips) { return up(8 + 16 * ((size_t)n_chips + 1), ENC_ALIGN); }

int64_t ccdgpu_encoded_bound(int32_t n_chips, const int32_t *n_pix, const int32_t *n_obs) {
    if (n_chips <= 0 || !n_pix || !n_obs) return -1;
    size_t t = table_bytes(n_chips);
    for (int32_t c = 0; c < n_chips; ++c) {
        const size_t a = sec_mode0(n_pix[c], n_obs[c]), b = sec_mode1(n_pix[c], n_obs[c], (int64_t)n_pix[c] * n_obs[c]);
        t += up(a > b ? a : b, ENC_ALIGN);
    }
    return (int64_t)t;
}

/* ---- band compaction: dst[k++] = src[i] for the observations kept (keep[i] = 1); *bad is set
 * when a dropped observation that must hold the fill value (strict[i] = 1) holds another one
 * (the chip then goes raw).  Only kept values are written: dst has room for exactly this pixel's
 * kept run, and the next pixel's run (another thread's, under the static schedule) follows it. */
static size_t compact_scalar(const int16_t *src, const uint8_t *keep, const uint8_t *strict, int n, int16_t *dst,
                             int *bad) {
    size_t k = 0;
    int b = 0;
    for (int i = 0; i < n; ++i) {
        if (keep[i]) dst[k++] = src[i];
        b |= strict[i] & (src[i] != -9999);
    }
    *bad |= b;
    return k;
}

#if defined(__x86_64__)
#include <immintrin.h>
/* Streaming writer of one contiguous output range (a block's run of one band): the compressed
 * values are staged in a small L1-resident buffer laid out like the destination lines, and every
 * destination line that lies wholly inside the range leaves with a non-temporal store -- no
 * read-for-ownership of the pinned destination, which costs a DRAM read of every line written
 * (the encoded batch, ~15 KB per tile pixel, is far larger than the caches).  The range's first
 * and last lines, which it may share with a neighbouring range (another block, possibly another
 * thread's), are written with masked ordinary stores of its own elements only. */
#define NTW_LINES 32
typedef struct {
    int16_t stage[(NTW_LINES + 1) * 32] __attribute__((aligned(64)));
    int16_t *dst; /* destination line of stage[0] (64-byte aligned) */
    int first;    /* elements of the range's first line below its start (0 once that line is out) */
    int k;        /* elements staged, counted from stage[0] */
} ntw_t;

__attribute__((target("avx512f,avx512bw"))) static inline void ntw_begin(ntw_t *w, int16_t *dst) {
    const uintptr_t a = (uintptr_t)dst;
    w->dst = (int16_t *)(a & ~(uintptr_t)63);
    w->first = (int)((a & 63) >> 1);
    w->k = w->first;
}
/* CCDGPU_ENCODE_NT=0: ordinary stores for the full lines too (A/B) */
static int ntw_stream(void) {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("CCDGPU_ENCODE_NT");
        v = !(e && *e == '0');
    }
    return v;
}
__attribute__((target("avx512f,avx512bw"))) static inline void ntw_lines(ntw_t *w, int nl) {
    const int nt = ntw_stream();
    for (int i = 0; i < nl; ++i) {
        const __m512i v = _mm512_load_si512((const void *)(w->stage + 32 * i));
        if (w->first) {
            _mm512_mask_storeu_epi16(w->dst, (__mmask32)(0xFFFFFFFFu << w->first), v);
            w->first = 0;
        } else if (nt) {
            _mm512_stream_si512((__m512i *)w->dst, v);
        } else {
            _mm512_store_si512((void *)w->dst, v);
        }
        w->dst += 32;
    }
}
/* c compressed values (the low lanes of v) onto the range */
__attribute__((target("avx512f,avx512bw"))) static inline void ntw_put(ntw_t *w, __m512i v, int c) {
    _mm512_mask_storeu_epi16(w->stage + w->k, (__mmask32)(c == 32 ? 0xFFFFFFFFu : (1u << c) - 1u), v);
    w->k += c;
    if (w->k >= NTW_LINES * 32) {
        const int nl = w->k >> 5;
        ntw_lines(w, nl);
        _mm512_store_si512((void *)w->stage, _mm512_load_si512((const void *)(w->stage + 32 * nl)));
        w->k -= 32 * nl;
    }
}
/* the range is complete: its full lines, then its partial last line */
__attribute__((target("avx512f,avx512bw"))) static inline void ntw_end(ntw_t *w) {
    const int nl = w->k >> 5;
    ntw_lines(w, nl);
    const int rem = w->k - 32 * nl;
    if (rem > 0) {
        const __m512i v = _mm512_load_si512((const void *)(w->stage + 32 * nl));
        _mm512_mask_storeu_epi16(w->dst, (__mmask32)(((1u << rem) - 1u) & (0xFFFFFFFFu << w->first)), v);
    }
    w->first = 0;
    w->k = 0;
}

/* the same with AVX-512 VBMI2, 32 observations at a time; m[] = keep bit masks, sm[] = the strict
 * observations' bit masks.  The kept values are compressed in a register and appended to the
 * range's streaming writer (a compress with a memory destination is microcoded and slow on Zen
 * 4/5). */
__attribute__((target("avx512f,avx512bw,avx512vbmi2"))) static size_t compact_vbmi2(const int16_t *src,
                                                                                   const uint32_t *m,
                                                                                   const uint32_t *sm, int n,
                                                                                   ntw_t *out, int *bad) {
    size_t k = 0;
    int i = 0, w = 0;
    const __m512i fillv = _mm512_set1_epi16(-9999);
    __mmask32 nb = 0;  /* dropped observations whose value is not the fill value */
    for (; i + 32 <= n; i += 32, ++w) {
        const __m512i v = _mm512_loadu_si512((const void *)(src + i));
        const int c = __builtin_popcount(m[w]);
        ntw_put(out, _mm512_maskz_compress_epi16((__mmask32)m[w], v), c);
        k += (size_t)c;
        nb |= _mm512_mask_cmpneq_epi16_mask((__mmask32)sm[w], v, fillv);
    }
    if (i < n) {
        const __mmask32 tail = (__mmask32)((1ull << (n - i)) - 1ull);
        const __m512i v = _mm512_maskz_loadu_epi16(tail, (const void *)(src + i));
        const int c = __builtin_popcount(m[w] & tail);
        ntw_put(out, _mm512_maskz_compress_epi16((__mmask32)(m[w] & tail), v), c);
        k += (size_t)c;
        nb |= _mm512_mask_cmpneq_epi16_mask((__mmask32)(sm[w] & tail), v, fillv);
    }
    *bad |= nb != 0;
    return k;
}
/* 4-bit palette codes (two per byte, even observation in the low nibble) and the keep bit masks
 * of one pixel's QA row, 32 observations at a time: a code is the index of the palette entry its
 * word equals (at most 16 compares); the codes' 16-bit lanes, read as 32-bit pairs, fold into
 * bytes with one down-convert.  Returns nonzero if a word is not in the palette (it got code 0
 * without being pal[0]): the palette came from a sample of the chip's pixels and misses it. */
__attribute__((target("avx512f,avx512bw,avx512vl,avx512vbmi2"))) static int qa_codes_avx512(const uint16_t *q, int n,
                                                                                  const uint16_t *pal, int npal,
                                                                                  uint16_t drop, uint16_t strict,
                                                                                  uint8_t *r, uint32_t *km,
                                                                                  uint32_t *sm) {
    int i = 0, w = 0;
    const __m512i dropv = _mm512_set1_epi16((short)drop), strictv = _mm512_set1_epi16((short)strict);
    const __m512i pal0 = _mm512_set1_epi16((short)pal[0]);
    __mmask32 miss = 0;
    for (; i < n; i += 32, ++w) {
        const __mmask32 lm = n - i >= 32 ? (__mmask32)0xFFFFFFFFu : (__mmask32)((1u << (n - i)) - 1u);
        const __m512i v = _mm512_maskz_loadu_epi16(lm, (const void *)(q + i));
        __m512i code = _mm512_setzero_si512();
        for (int j = 1; j < npal; ++j)
            code = _mm512_mask_mov_epi16(code, _mm512_cmpeq_epi16_mask(v, _mm512_set1_epi16((short)pal[j])),
                                         _mm512_set1_epi16((short)j));
        miss |= _mm512_mask_cmpneq_epi16_mask(_mm512_cmpeq_epi16_mask(code, _mm512_setzero_si512()) & lm, v, pal0);
        km[w] = (uint32_t)(_mm512_testn_epi16_mask(v, dropv) & lm);
        sm[w] = (uint32_t)(_mm512_test_epi16_mask(v, strictv) & lm);
        const __m512i pr = _mm512_or_si512(_mm512_and_si512(code, _mm512_set1_epi32(0xF)),
                                           _mm512_and_si512(_mm512_srli_epi32(code, 12), _mm512_set1_epi32(0xF0)));
        const __m128i bytes = _mm512_cvtepi32_epi8(pr);
        const int nb = (n - i >= 32 ? 32 : n - i + 1) / 2;  /* bytes of this chunk's codes */
        _mm_mask_storeu_epi8(r + (i >> 1), (__mmask16)(nb == 16 ? 0xFFFFu : (1u << nb) - 1u), bytes);
    }
    return miss != 0;
}
/* pass 1 of a pixel's QA row outside the palette sample: the dropped count only */
__attribute__((target("avx512f,avx512bw,avx512vl"))) static uint32_t qa_count_avx512(const uint16_t *q, int n,
                                                                                   uint16_t drop) {
    uint32_t fill = 0;
    const __m512i dv = _mm512_set1_epi16((short)drop);
    int i = 0;
    for (; i + 32 <= n; i += 32)
        fill += (uint32_t)__builtin_popcount(_mm512_test_epi16_mask(_mm512_loadu_si512((const void *)(q + i)), dv));
    if (i < n) {
        const __mmask32 lm = (__mmask32)((1u << (n - i)) - 1u);
        fill += (uint32_t)__builtin_popcount(_mm512_test_epi16_mask(_mm512_maskz_loadu_epi16(lm, (const void *)(q + i)), dv) & lm);
    }
    return fill;
}
/* pass 1 of one pixel's QA row, vector path: dropped count, and every word not yet in the thread's
 * list s_pal (compared 32 at a time against the list; the rare new word is added) */
__attribute__((target("avx512f,avx512bw,avx512vl,avx512vbmi2"))) static uint32_t qa_scan_avx512(const uint16_t *q,
                                                                                               int n, uint16_t drop,
                                                                                               uint16_t *s_pal,
                                                                                               int *s_npal) {
    uint32_t fill = 0;
    const __m512i one = _mm512_set1_epi16((short)drop);
    int np = *s_npal;
    for (int i = 0; i < n; i += 32) {
        const __mmask32 lm = n - i >= 32 ? (__mmask32)0xFFFFFFFFu : (__mmask32)((1u << (n - i)) - 1u);
        const __m512i v = _mm512_maskz_loadu_epi16(lm, (const void *)(q + i));
        fill += (uint32_t)__builtin_popcount(_mm512_test_epi16_mask(v, one) & lm);
        __mmask32 hit = 0;  /* independent compares (an early-exit chain measured 1.7x slower) */
        for (int j = 0; j < np; ++j) hit |= _mm512_cmpeq_epi16_mask(v, _mm512_set1_epi16((short)s_pal[j]));
        __mmask32 un = lm & ~hit;
        while (un) {
            const uint16_t w = q[i + __builtin_ctz(un)];
            if (np < 17) s_pal[np++] = w;
            un &= ~_mm512_cmpeq_epi16_mask(v, _mm512_set1_epi16((short)w));
            if (np >= 17) un = 0;  /* more than a palette: the chip goes raw */
        }
    }
    *s_npal = np;
    return fill;
}
static int have_vbmi2(void) {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("CCDGPU_ENCODE_SCALAR");
        v = (e && *e && *e != '0') ? 0 : __builtin_cpu_supports("avx512vbmi2") && __builtin_cpu_supports("avx512bw") &&
                                                  __builtin_cpu_supports("avx512vl");
    }
    return v;
}
#else
static int have_vbmi2(void) { return 0; }
#endif

int32_t ccdgpu_encode_vector_path(void) { return have_vbmi2(); }

/* pixels per block of the vector pass 2 (CCDGPU_ENCODE_BLOCK overrides the default 32; 1 = the
 * bands of one pixel after another) */
static int enc_block(void) {
    static int b = 0;
    if (!b) {
        const char *e = getenv("CCDGPU_ENCODE_BLOCK");
        int v = e ? atoi(e) : 32;
        b = v < 1 ? 1 : v > 256 ? 256 : v;
    }
    return b;
}

/* per-thread pass-1 state: the QA words seen (a 65536-bit set), a fill observation with a band
 * value other than -9999 */
typedef struct {
    uint8_t seen[65536];  /* scalar path: byte flags (independent stores, no read-modify-write chain) */
    uint16_t pal[17];     /* vector path: the distinct words met so far (17 = more than a palette holds) */
    int npal;
    int bad_fill;
} pass1_t;

/* mode 0: the chip as it is (header fields other than the mode already written) */
static size_t encode_raw(int32_t n_pix, int32_t n_obs, const int16_t *spectra, const uint16_t *qa, uint8_t *sec,
                         int nt) {
    const size_t plane = (size_t)n_pix * (size_t)n_obs;
    int32_t *h = (int32_t *)sec;
    h[0] = 0;
    h[3] = 0;
    int64_t *h64 = (int64_t *)(sec + 48);
    h64[0] = 0;
    h64[2] = 0;
    memset(sec + 16, 0, 32);
    uint16_t *oq = (uint16_t *)(sec + ENC_HDR);
    int16_t *os = (int16_t *)(sec + ENC_HDR + up(2 * plane, 16));
    memset((uint8_t *)(oq + plane), 0, up(2 * plane, 16) - 2 * plane);
#pragma omp parallel for schedule(static) num_threads(nt)
    for (int32_t p = 0; p < n_pix; ++p) {
        memcpy(oq + (size_t)p * n_obs, qa + (size_t)p * n_obs, 2 * (size_t)n_obs);
        for (int b = 0; b < 7; ++b)
            memcpy(os + (size_t)b * plane + (size_t)p * n_obs, spectra + (size_t)b * plane + (size_t)p * n_obs,
                   2 * (size_t)n_obs);
    }
    return sec_mode0(n_pix, n_obs);
}

/* pixels of a chip whose QA rows pass 1 scans for the palette (vector path): every
 * ENC_SAMPLE-th; pass 2 checks every word against it and, when one is missing, the chip is
 * encoded again from a scan of every pixel.  The palette is the chip's sorted set of distinct
 * words either way, so the bytes are the same. */
#define ENC_SAMPLE 16

/* one chip into sec (room for the larger of its two modes); returns the section's bytes */
static size_t encode_chip(int32_t n_pix, int32_t n_obs, const int16_t *spectra, const uint16_t *qa, int64_t pix_base,
                          int64_t data_off, uint8_t *sec, int threads, uint32_t *kept_scratch, uint16_t drop,
                          uint16_t strict) {
    const size_t plane = (size_t)n_pix * (size_t)n_obs;
    int nt = threads > 0 ? threads : 1;
    if (nt > 64) nt = 64;
    pass1_t *st = (pass1_t *)malloc((size_t)nt * sizeof(pass1_t));
    uint8_t *lut = (uint8_t *)malloc(65536);  /* QA word -> palette index */
    if (!st || !lut) {
        free(st);
        free(lut);
        return 0;
    }
    const int vec1 = have_vbmi2();
    size_t ret = 0;
    for (int full = vec1 ? 0 : 1; full < 2; ++full) {
        const int sample = full ? 1 : ENC_SAMPLE;
        memset(st, 0, (size_t)nt * sizeof(pass1_t));
        /* pass 1: kept counts, distinct QA words (of the sampled pixels) */
#pragma omp parallel for schedule(static) num_threads(nt)
        for (int32_t p = 0; p < n_pix; ++p) {
#ifdef _OPENMP
            pass1_t *s = &st[omp_get_thread_num()];
#else
            pass1_t *s = &st[0];
#endif
            const uint16_t *q = qa + (size_t)p * n_obs;
            uint32_t fill = 0;
#if defined(__x86_64__)
            if (vec1) {
                fill = p % sample == 0 ? qa_scan_avx512(q, n_obs, drop, s->pal, &s->npal) : qa_count_avx512(q, n_obs, drop);
            } else
#endif
            {
                for (int32_t i = 0; i < n_obs; ++i) {
                    const uint16_t v = q[i];
                    s->seen[v] = 1;
                    fill += (v & drop) != 0;
                }
            }
            kept_scratch[p] = (uint32_t)n_obs - fill;
        }
        int bad = 0;  /* (pass 2 checks the fill observations' band values) */
        uint16_t palv[16];
        int npal = 0;
        for (int t = 0; t < nt; ++t) bad |= st[t].bad_fill;
        if (vec1)  /* the threads' word lists into the byte set the scalar path fills */
            for (int t = 0; t < nt; ++t)
                for (int j = 0; j < st[t].npal; ++j) st[t].seen[st[t].pal[j]] = 1;
        for (int t = 0; t < nt; ++t)
            if (st[t].npal > 16) bad = 1;  /* (vector path: one thread alone met more than 16 words) */
        {
            uint64_t *s0 = (uint64_t *)st[0].seen;
            for (int t = 1; t < nt; ++t) {
                const uint64_t *st_ = (const uint64_t *)st[t].seen;
                for (int w = 0; w < 8192; ++w) s0[w] |= st_[w];
            }
            for (int w = 0; w < 8192 && npal <= 16; ++w)  /* ascending: the palette is sorted */
                if (s0[w])
                    for (int j = 0; j < 8 && npal <= 16; ++j)
                        if (st[0].seen[8 * w + j]) {
                            if (npal < 16) palv[npal] = (uint16_t)(8 * w + j);
                            ++npal;
                        }
        }
        int32_t *h = (int32_t *)sec;
        memset(sec, 0, ENC_HDR);
        h[1] = n_pix;
        h[2] = n_obs;
        int64_t *h64 = (int64_t *)(sec + 48);
        h64[1] = data_off;
        h64[3] = pix_base;
        if (bad || npal > 16) {
            ret = encode_raw(n_pix, n_obs, spectra, qa, sec, nt);
            break;
        }
        h[0] = 1;
        h[3] = npal;
        *(uint32_t *)(sec + 80) = drop;  /* the decoder's keep test */
        uint16_t *pal = (uint16_t *)(sec + 16);
        for (int j = 0; j < npal; ++j) {
            pal[j] = palv[j];
            lut[palv[j]] = (uint8_t)j;
        }
        uint32_t *koff = (uint32_t *)(sec + ENC_HDR);
        uint64_t tot = 0;
        for (int32_t p = 0; p < n_pix; ++p) {
            koff[p] = (uint32_t)tot;
            tot += kept_scratch[p];
        }
        koff[n_pix] = (uint32_t)tot;
        /* padding after the offsets and after the code rows: deterministic bytes */
        memset(koff + n_pix + 1, 0, up(4 * ((size_t)n_pix + 1), 16) - 4 * ((size_t)n_pix + 1));
        const size_t bstride = up((size_t)tot, 8);
        h64[0] = (int64_t)tot;
        h64[2] = (int64_t)bstride;
        uint8_t *q4 = sec + ENC_HDR + up(4 * ((size_t)n_pix + 1), 16);
        const size_t rowb = (size_t)(n_obs + 1) / 2;
        int16_t *bands = (int16_t *)(q4 + up((size_t)n_pix * rowb, 16));
        memset(q4 + (size_t)n_pix * rowb, 0, up((size_t)n_pix * rowb, 16) - (size_t)n_pix * rowb);
        const int vec = have_vbmi2();
        int bad2 = 0, miss = 0;
        /* pass 2: 4-bit QA codes and the kept band values (and the fill observations' values checked).
         * Vector path in blocks of enc_block() pixels: the block's keep / strict masks first, then one
         * band at a time over the whole block, so the loads and stores run as two long sequential
         * streams (band rows of consecutive pixels are contiguous in the input plane and in the
         * output) instead of seven of each interleaved per pixel. */
        const int mw = n_obs / 32 + 2;  /* mask words per pixel */
        const int pb = enc_block();
#pragma omp parallel num_threads(nt) reduction(| : bad2, miss)
        {
            uint8_t *keep = (uint8_t *)malloc(2 * (size_t)n_obs + 64), *strictm = keep + n_obs + 32;
            uint32_t *km = (uint32_t *)malloc((size_t)mw * 8 * pb), *sm = km + (size_t)mw * pb;
#if defined(__x86_64__)
            ntw_t ntw_s; /* (2 KB, 64-byte aligned, on the thread's stack) */
            ntw_t *ntw = &ntw_s;
            if (vec) {
#pragma omp for schedule(static)
                for (int32_t p0 = 0; p0 < n_pix; p0 += pb) {
                    const int32_t pe = p0 + pb < n_pix ? p0 + pb : n_pix;
                    for (int32_t p = p0; p < pe; ++p)
                        miss |= qa_codes_avx512(qa + (size_t)p * n_obs, n_obs, pal, npal, drop, strict, q4 + (size_t)p * rowb,
                                                km + (size_t)(p - p0) * mw, sm + (size_t)(p - p0) * mw);
                    if (miss) continue;  /* the chip is encoded again */
                    for (int b = 0; b < 7; ++b) {
                        const int16_t *src = spectra + (size_t)b * plane;
                        /* the block's run of band b is one contiguous range (koff[p0] .. koff[pe]) */
                        ntw_begin(ntw, bands + (size_t)b * bstride + koff[p0]);
                        for (int32_t p = p0; p < pe; ++p)
                            compact_vbmi2(src + (size_t)p * n_obs, km + (size_t)(p - p0) * mw, sm + (size_t)(p - p0) * mw,
                                          n_obs, ntw, &bad2);
                        ntw_end(ntw);
                    }
                }
            } else
#endif
#pragma omp for schedule(static)
            for (int32_t p = 0; p < n_pix; ++p) {
                const uint16_t *q = qa + (size_t)p * n_obs;
                uint8_t *r = q4 + (size_t)p * rowb;
                memset(km, 0, ((size_t)n_obs / 32 + 1) * 4);
                int32_t i = 0;
                for (; i + 1 < n_obs; i += 2) {
                    const uint16_t v0 = q[i], v1 = q[i + 1];
                    r[i >> 1] = (uint8_t)(lut[v0] | (lut[v1] << 4));
                    const uint32_t k0 = !(v0 & drop), k1 = !(v1 & drop);
                    keep[i] = (uint8_t)k0;
                    keep[i + 1] = (uint8_t)k1;
                    strictm[i] = (uint8_t)((v0 & strict) != 0);
                    strictm[i + 1] = (uint8_t)((v1 & strict) != 0);
                    km[i >> 5] |= (k0 | (k1 << 1)) << (i & 31);
                }
                if (i < n_obs) {
                    const uint16_t v0 = q[i];
                    r[i >> 1] = lut[v0];
                    const uint32_t k0 = !(v0 & drop);
                    keep[i] = (uint8_t)k0;
                    strictm[i] = (uint8_t)((v0 & strict) != 0);
                    km[i >> 5] |= k0 << (i & 31);
                }
                for (int b = 0; b < 7; ++b)
                    compact_scalar(spectra + (size_t)b * plane + (size_t)p * n_obs, keep, strictm, n_obs,
                                   bands + (size_t)b * bstride + koff[p], &bad2);
            }
#if defined(__x86_64__)
            if (vec) _mm_sfence();  /* the streamed lines are visible before the batch is uploaded */
#endif
            free(keep);
            free(km);
        }
        if (miss && !full) continue;  /* a word the sample missed: every pixel's words this time */
        if (bad2) {
            ret = encode_raw(n_pix, n_obs, spectra, qa, sec, nt);  /* a strict observation with data */
            break;
        }
        for (int b = 0; b < 7; ++b)  /* band padding: deterministic bytes */
            memset(bands + (size_t)b * bstride + tot, 0, 2 * (bstride - (size_t)tot));
        ret = sec_mode1(n_pix, n_obs, (int64_t)tot);
        break;
    }
    free(st);
    free(lut);
    return ret;
}

int64_t ccdgpu_encode_chips(int32_t n_chips, const int32_t *n_pix, const int32_t *n_obs, const int16_t *const *spectra,
                            const uint16_t *const *qa, uint8_t *out, int64_t out_cap, int32_t threads,
                            uint16_t drop_bits, uint16_t strict_bits) {
    if (n_chips <= 0 || !n_pix || !n_obs || !spectra || !qa || !out) return -1;
    if ((strict_bits & ~drop_bits) != 0) return -1;  /* a strict observation is a dropped one */
    const int64_t need = ccdgpu_encoded_bound(n_chips, n_pix, n_obs);
    if (need < 0 || out_cap < need) return -2;
    int64_t *tab = (int64_t *)out;
    tab[0] = n_chips;
    int64_t *off = tab + 1, *pix = tab + 2 + n_chips;
    int32_t maxp = 0;
    for (int32_t c = 0; c < n_chips; ++c) {
        if (n_pix[c] <= 0 || n_obs[c] <= 0 || !spectra[c] || !qa[c]) return -1;
        maxp = n_pix[c] > maxp ? n_pix[c] : maxp;
    }
    uint32_t *kept = (uint32_t *)malloc(4 * (size_t)maxp);
    if (!kept) return -3;
    size_t pos = table_bytes(n_chips);
    memset(out + 8 + 16 * ((size_t)n_chips + 1), 0, pos - (8 + 16 * ((size_t)n_chips + 1)));  /* table padding */
    int64_t pbase = 0, dbase = 0;
    for (int32_t c = 0; c < n_chips; ++c) {
        off[c] = (int64_t)pos;
        pix[c] = pbase;
        const size_t sz = encode_chip(n_pix[c], n_obs[c], spectra[c], qa[c], pbase, dbase, out + pos, threads, kept,
                                      drop_bits, strict_bits);
        if (!sz) {
            free(kept);
            return -3;
        }
        memset(out + pos + sz, 0, up(sz, ENC_ALIGN) - sz);  /* section padding */
        pos += up(sz, ENC_ALIGN);
        pbase += n_pix[c];
        dbase += (int64_t)n_pix[c] * n_obs[c];
    }
    off[n_chips] = (int64_t)pos;
    pix[n_chips] = pbase;
    free(kept);
    return (int64_t)pos;
}
