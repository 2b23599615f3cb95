/* ccdgpu.h -- C-ABI of libccdgpu.so: MI355X (gfx950) CCDC change detection.
 *
 * Drop-in replacement for the per-pixel call the reference makes at
 *     ccdc/pyccd.py:168   ccdresult = ccd.detect(**second(timeseries))
 * (lcmap-pyccd 2018.03.12.dev-ncompare.b2, setup.py:32) over the records that
 *     ccdc/timeseries.py:92-126   (merlin.create -> ((cx,cy,px,py), {dates, blues..thermals, qas}))
 * builds.  One call processes a batch of pixels that share one acquisition-date vector (a chip
 * or part of one, as merlin builds them per chip).  The Python side (lcmap-firebird_amd/ccd,
 * lcmap-firebird_amd/ccdc/pyccd.py) binds these symbols with ctypes; INTEGRATION.md shows the
 * binding.  Plain C types only; no C++ or torch types cross this boundary.
 *
 * Errors: every entry point returns 0 on success or a negative CCDGPU_E* code; the message of the
 * last failure on the calling thread is ccdgpu_last_error().  An unsupported bit-packed QA value
 * is CCDGPU_EQA -- the analogue of pyccd's ValueError from qa.qabitval -- and the offending
 * pixel is reported in ccdgpu_result.error_pixel.
 */
#ifndef CCDGPU_H
#define CCDGPU_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define CCDGPU_OK 0
#define CCDGPU_EINVAL (-1)   /* bad argument / size                                    */
#define CCDGPU_EHIP (-2)     /* HIP runtime error (no device, launch failure, ...)     */
#define CCDGPU_EQA (-3)      /* unsupported bit-packed QA value (pyccd ValueError)     */
#define CCDGPU_ENOMEM (-4)   /* device or host allocation failed                       */
#define CCDGPU_EOVERFLOW (-5)/* capacity exceeded (adaptive peek > CCDGPU_MAX_PEEK)    */

#define CCDGPU_NBANDS 7      /* blue, green, red, nir, swir1, swir2, thermal            */
#define CCDGPU_MAX_OBS 4096  /* observations per pixel the kernels accept              */
/* Largest (adaptive) look-ahead window.  The ncompare peek is round(16 PEEK_SIZE / median gap)
 * over the filtered, duplicate-free dates, so with the default PEEK_SIZE 6 it never exceeds 96
 * (median gap >= 1 day): every default-parameter pixel is supported.  A configured PEEK_SIZE > 6
 * can push it past 96 on dense dates; that pixel fails the call with CCDGPU_EOVERFLOW. */
#define CCDGPU_MAX_PEEK 96

/* ccd/parameters.yaml defaults; ccdgpu_params_default() fills them. */
typedef struct ccdgpu_params {
    int32_t meow_size;          /* 12   MEOW_SIZE                                       */
    int32_t peek_size;          /* 6    PEEK_SIZE (default; ncompare may enlarge it)     */
    int32_t day_delta;          /* 365  DAY_DELTA                                        */
    int32_t coef_min, coef_mid, coef_max; /* 4 / 6 / 8                                    */
    int32_t num_obs_factor;     /* 3                                                     */
    uint32_t detection_bands;   /* bit mask, default bands 1..5 = 0x3E                   */
    uint32_t tmask_bands;       /* bit mask, default bands 1 and 4 = 0x12                */
    int32_t lasso_max_iter;     /* 1000                                                  */
    int32_t thermal_min, thermal_max; /* -9320 / 7070 (deg C x 100)                        */
    int32_t median_green_filter;/* 400                                                   */
    int32_t curve_qa_start, curve_qa_end, curve_qa_insuf_clear, curve_qa_persist_snow; /* 14/24/44/54 */
    int32_t qa_fill, qa_clear, qa_water, qa_shadow, qa_snow, qa_cloud; /* bit offsets 0..5 */
    int32_t qa_cirrus1, qa_cirrus2, qa_occlusion;                      /* 8, 9, 10         */
    int32_t qa_bitpacked;       /* 1: qas are PIXELQA bit fields; 0: already class ids   */
    int32_t adaptive_peek;      /* 1: "ncompare" density-adaptive peek + threshold        */
    int32_t rmse_dof;           /* 1: rmse denominator n - num_coefficients              */
    int32_t kelvin_to_celsius;  /* 1: standard procedure converts thermal (int16 wrap)   */
    double avg_days_yr;         /* 365.2425                                              */
    double change_probability;  /* 0.99                                                  */
    double change_threshold;    /* chi2.ppf(0.99, 5)                                     */
    double outlier_threshold;   /* chi2.ppf(0.999999, 5)                                 */
    double t_const;             /* 4.42 Tmask                                            */
    double lasso_alpha;         /* 1.0 (sklearn Lasso alpha; l1 = alpha * n_samples)     */
    double lasso_tol;           /* 1e-4                                                  */
    double clear_pct_threshold; /* 0.25                                                  */
    double snow_pct_threshold;  /* 0.75                                                  */
    /* tie order of the date sort (ccd/__init__.py detect) and of find_closest_doy
       (change.py): 0 = numpy's argsort kind='quicksort' as the pinned reference image ran it
       (numpy < 1.17 introsort-free aquicksort), 1 = stable (ties by position) */
    int32_t argsort_stable;     /* 0                                                     */
    int32_t reserved0;          /* 0                                                     */
} ccdgpu_params;

/* One change model (pyccd change_model dict; ccdc/pyccd.py:106-148 formats it). */
typedef struct ccdgpu_segment {
    int32_t start_day, end_day, break_day; /* proleptic ordinals                       */
    int32_t observation_count;
    int32_t curve_qa;
    int32_t pixel;                          /* pixel index within the batch             */
    double change_probability;
    double magnitude[CCDGPU_NBANDS];
    double rmse[CCDGPU_NBANDS];
    double intercept[CCDGPU_NBANDS];
    double coef[CCDGPU_NBANDS][7];          /* [band][t, cos, sin, cos2, sin2, cos3, sin3] */
} ccdgpu_segment;

enum { CCDGPU_PROC_STANDARD = 0, CCDGPU_PROC_PERMANENT_SNOW = 1, CCDGPU_PROC_INSUFFICIENT_CLEAR = 2 };

/* Results, CSR by pixel.  Owned by the library until ccdgpu_result_free. */
typedef struct ccdgpu_result {
    int32_t n_pix, n_obs;
    int64_t n_seg;
    int64_t *seg_offsets;       /* [n_pix + 1]                                            */
    ccdgpu_segment *segments;   /* [n_seg], pixel-major, in detection order               */
    uint32_t *mask_bits;        /* [n_pix][mask_words] processing_mask, SORTED date order  */
    int32_t mask_words;         /* (n_obs + 31) / 32                                      */
    int32_t *procedure;         /* [n_pix] CCDGPU_PROC_*                                  */
    double *probs;              /* [n_pix][3] cloud, snow, water                          */
    int64_t *sorted_dates;      /* [n_obs] ascending (argsort of the input dates, ties in */
                                /* params.argsort_stable's order)                         */
    int32_t *sort_index;        /* [n_obs] input position of each sorted observation      */
    int32_t error_pixel;        /* first pixel with an unsupported QA value, else -1      */
    double seconds_kernel;      /* device time of the detection kernels (HIP events)      */
    double seconds_total;       /* wall time of the call                                  */
} ccdgpu_result;

/* One row of the reference's segment table with its storage types (ccdc/segment.py:16-55,
 * resources/schema.cql segment; rows of ccdc/pyccd.py:106-148): float columns rounded to
 * float32 as Spark's FloatType cast does, days as proleptic ordinals (ISO text on the host).
 * A pixel without change models has one row of pyccd.default (pyccd.py:99-103): days 1/1/1 and
 * has_model 0, every band / chprob / curqa column null. */
typedef struct ccdgpu_row {
    int32_t px, py;                 /* cx + 30 col, cy - 30 row (test/__init__.py:37)          */
    int32_t sday, eday, bday;
    int32_t curqa;
    int32_t has_model;
    float chprob;
    float mag[CCDGPU_NBANDS], rmse[CCDGPU_NBANDS];
    float coef[CCDGPU_NBANDS][7];
    float intercept[CCDGPU_NBANDS];
} ccdgpu_row;

/* Segment + pixel table rows of one chip.  Owned by the library until ccdgpu_rows_free. */
typedef struct ccdgpu_rows {
    int32_t n_pix, n_obs;
    int64_t n_rows;
    int64_t *row_offsets;       /* [n_pix + 1]                                             */
    ccdgpu_row *rows;           /* [n_rows], pixel-major                                   */
    int8_t *mask;               /* [n_pix][n_obs] processing mask 0/1, sorted date order   */
                                /* (pixel table, resources/schema.cql pixel.mask); NULL    */
                                /* for a batch fetch, which returns mask_bits instead      */
    uint32_t *mask_bits;        /* batch fetch: [n_pix][mask_words] the same mask as bits  */
    int32_t mask_words;         /* (bit i of word i/32 = sorted observation i), 8x smaller */
} ccdgpu_rows;

typedef struct ccdgpu_ctx ccdgpu_ctx;

const char *ccdgpu_version(void);
const char *ccdgpu_last_error(void);
void ccdgpu_params_default(ccdgpu_params *p);

/* Create a context bound to HIP device `device`.  A context is used by one host thread at a
 * time; up to 16 contexts may live in a process, and contexts on the same device run their
 * detections concurrently (each has its own stream, buffers and launch-argument slot), so a
 * second context's launch fills the CUs the first one's launch tail leaves idle. */
int ccdgpu_init(int device, ccdgpu_ctx **ctx);
/* ccdgpu_init with `copy_cus` CUs reserved for everything of the context but the detection kernel
 * -- the encoded upload's decode kernel, the launch's prep, CSR scan and scatter, the row packing
 * and the small copies -- and the rest for the detection kernel; 0 = no reservation
 * (ccdgpu_init: all on one stream).  Persistent detection waves hold every wave slot of their
 * CUs until the launch drains, so with several contexts one context's short kernels otherwise
 * wait for wave slots behind the others' whole detections; the tile driver (ccdc.runner)
 * reserves 8 of 256.  CCDGPU_COPY_CUS in the
 * environment overrides the value.  (No reference counterpart: an execution detail of the
 * pipelined driver that replaces ccdc/pyccd.py:168's per-chip map.) */
int ccdgpu_init_copy_cus(int device, int copy_cus, ccdgpu_ctx **ctx);
int ccdgpu_destroy(ccdgpu_ctx *ctx);
int ccdgpu_device_count(int *count);
/* NUMA node of HIP device `device`'s PCIe attachment (sysfs numa_node of its bus id; -1 when the
 * platform does not say).  The tile driver (ccdc.runner) keeps its host threads and pinned upload
 * buffers on that node, so the chip copies and the DMA reads of them stay on the socket the GPU
 * hangs off.  (No reference counterpart: Spark placed executors, ccdc/core.py:97-108.) */
int ccdgpu_device_numa_node(int device, int *node);
int ccdgpu_synchronize(ccdgpu_ctx *ctx);

/* Host-buffer entry point (the pyccd.detect / ccd.detect path).
 *   dates   [n_obs]                 ordinals, any order (merlin delivers them descending)
 *   spectra [7][n_pix][n_obs]       int16, band-major, observation-contiguous, input order
 *   qa      [n_pix][n_obs]          uint16 bit-packed PIXELQA (or class ids if !qa_bitpacked)
 * Synchronous: H2D, kernels, D2H.  *out must be released with ccdgpu_result_free. */
int ccdgpu_detect_batch(ccdgpu_ctx *ctx, const ccdgpu_params *params, int32_t n_pix, int32_t n_obs,
                        const int64_t *dates, const int16_t *spectra, const uint16_t *qa,
                        ccdgpu_result *out);
void ccdgpu_result_free(ccdgpu_result *out);

/* Device-resident path (tile runner, benchmarks, batched Spark partitions): stage a batch once,
 * run the detection as often as wanted on the resident copy, fetch results separately.
 *
 * A batch is `n_chips` chips -- pixel groups that share one date vector, as merlin builds them
 * per chip (ccdc/timeseries.py:107-115) -- with their own sizes: chip c has n_pix[c] pixels and
 * n_obs[c] observations, so a tile's base-cadence and sidelap chips (and the date groups of a
 * Spark partition) run in one launch.  Their arrays are packed back to back:
 *   dates   chip c at  O_c = sum_{c' < c} n_obs[c']               [n_obs[c]]
 *   spectra chip c at  7 * D_c, D_c = sum_{c' < c} n_pix[c'] n_obs[c']   [7][n_pix[c]][n_obs[c]]
 *   qa      chip c at  D_c                                          [n_pix[c]][n_obs[c]]
 * Pixel p of the batch is pixel p - sum_{c' < c} n_pix[c'] of chip c. */
int ccdgpu_stage_chips(ccdgpu_ctx *ctx, const ccdgpu_params *params, int32_t n_chips, const int32_t *n_pix,
                       const int32_t *n_obs, const int64_t *dates, const int16_t *spectra, const uint16_t *qa);
/* ccdgpu_stage_chips with every chip of shape (n_pix, n_obs). */
int ccdgpu_stage(ccdgpu_ctx *ctx, const ccdgpu_params *params, int32_t n_chips, int32_t n_pix,
                 int32_t n_obs, const int64_t *dates, const int16_t *spectra, const uint16_t *qa);
int ccdgpu_run_staged(ccdgpu_ctx *ctx, double *kernel_seconds);

/* Chip packer: stage a batch straight from the chipmunk wire format (replaces merlin.create's
 * per-pixel pivot and the repartition shuffle of ccdc/timeseries.py:120-125; payloads as in the
 * reference fixture test/data/chip_response.json).  Layer l (0..6 = blues, greens, reds, nirs,
 * swir1s, swir2s, thermals; 7 = pixel QA) of observation o of chip c is the base64 text (standard
 * alphabet, '=' padded) starting at byte text_offsets[(c * n_obs + o) * 8 + l] of `text`; it
 * decodes to n_pix little-endian int16 (uint16 for QA) values in row-major pixel order.  A
 * negative offset is a missing layer: its pixels become fill (-9999, QA 1).  dates as in
 * ccdgpu_stage.  The text is copied to the device, decoded and pivoted there to the
 * [7][n_pix][n_obs] / [n_pix][n_obs] layout; *unpack_seconds (may be NULL) gets the kernel time.
 * CCDGPU_EINVAL for a payload that runs past text_bytes or is not base64. */
int ccdgpu_stage_chipmunk(ccdgpu_ctx *ctx, const ccdgpu_params *params, int32_t n_chips, int32_t n_pix,
                          int32_t n_obs, const int64_t *dates, const char *text, int64_t text_bytes,
                          const int64_t *text_offsets, double *unpack_seconds);

/* Overlapped upload (HIP copy stream): ccdgpu_stage_slot uploads a batch into input slot
 * 0 .. CCDGPU_UPLOAD_SLOTS-1 and returns at once; ccdgpu_run_slot detects the batch of a slot
 * (after its upload) exactly like ccdgpu_run_staged, results fetched with ccdgpu_fetch_staged /
 * ccdgpu_fetch_rows.  The streaming loop  stage_slot(0, b0); for i: { stage_slot((i+1)&1,
 * b_{i+1}); run_slot(i&1); fetch }  overlaps each upload with the previous batch's detection;
 * with S slots up to S-1 uploads can be queued ahead of the running batch (the tile driver keeps
 * two queued, so the PCIe link stays busy while detection and the row fetch run).  Host inputs must stay valid and
 * unchanged until the run_slot of their slot returns; they should be pinned (ccdgpu_host_alloc),
 * or the upload is synchronous.  Each slot keeps the params it was staged with. */
#define CCDGPU_UPLOAD_SLOTS 4
int ccdgpu_host_alloc(size_t bytes, void **ptr);
int ccdgpu_host_free(void *ptr);
int ccdgpu_stage_slot_chips(ccdgpu_ctx *ctx, int32_t slot, const ccdgpu_params *params, int32_t n_chips,
                            const int32_t *n_pix, const int32_t *n_obs, const int64_t *dates, const int16_t *spectra,
                            const uint16_t *qa);
int ccdgpu_stage_slot(ccdgpu_ctx *ctx, int32_t slot, const ccdgpu_params *params, int32_t n_chips, int32_t n_pix,
                      int32_t n_obs, const int64_t *dates, const int16_t *spectra, const uint16_t *qa);
int ccdgpu_run_slot(ccdgpu_ctx *ctx, int32_t slot, double *kernel_seconds);
/* ccdgpu_run_slot in two halves, so the calling thread can stage further slots while the
 * detection runs: _begin launches it and returns at once, ccdgpu_run_query returns 1 once it has
 * completed (0 while it runs; 1 with nothing begun), _end waits for it and does the rest of
 * ccdgpu_run_slot (status, CSR of the segments; same return codes).  Between _begin and _end only
 * ccdgpu_stage_slot* of other slots and ccdgpu_run_query may be called on the context.  The tile
 * driver (ccdc.runner) stages the batches its fetch thread finishes during the detection. */
int ccdgpu_run_slot_begin(ccdgpu_ctx *ctx, int32_t slot);
int ccdgpu_run_query(ccdgpu_ctx *ctx);
int ccdgpu_run_slot_end(ccdgpu_ctx *ctx, double *kernel_seconds);
/* The split run with the batch's rows in the same device chain (the tile driver's path; rows as
 * ccdgpu_fetch_batch_rows_into gives them, chip c at (cx[c], cy[c])): _begin_rows enqueues the
 * detection and behind it the CSR, the row packing and the copies of the row offsets
 * [total_pixels + 1], the rows (up to rows_cap) and the mask words [total_pixels][mask_words]
 * into the caller's buffers (pinned: ccdgpu_host_alloc), then returns; _end_rows waits once for
 * the whole chain and returns what ccdgpu_run_slot_end returns, with the row count in *n_rows.
 * More rows than rows_cap: CCDGPU_EOVERFLOW with *n_rows set -- the run is complete and
 * ccdgpu_fetch_batch_rows_into fetches its rows into larger buffers.  rows_cap is also what the
 * chain copies back (the whole rows_cap rows, written or not): pass the rows a batch is expected
 * to hold, not the buffer's room (ccdgpu.RowsBuffers learns it: 1.25 x the highest rows per
 * pixel seen).  The buffers must stay alive and untouched until _end_rows returns;
 * ccdgpu_run_query works as for _begin. */
int ccdgpu_run_slot_begin_rows(ccdgpu_ctx *ctx, int32_t slot, const int32_t *cx, const int32_t *cy, int32_t width,
                               int64_t *row_offsets, int64_t offsets_cap, ccdgpu_row *rows, int64_t rows_cap,
                               uint32_t *mask_bits, int64_t mask_cap);
int ccdgpu_run_slot_end_rows(ccdgpu_ctx *ctx, double *kernel_seconds, int64_t *n_rows);

/* Transport-encoded uploads (no reference counterpart -- the tile path's PCIe link is its bound,
 * DESIGN.md §5).  ccdgpu_encode_chips packs chips given as per-chip pointers (spectra
 * [7][n_pix][n_obs] int16, qa [n_pix][n_obs] uint16, the ccdgpu_stage_chips layout of one chip)
 * into `out` (>= ccdgpu_encoded_bound bytes; pinned for an asynchronous upload) and returns the
 * bytes written (< 0 on bad arguments).  Per chip: an observation whose QA word has any of
 * `drop_bits` set sends no band values (the decoder writes -9999); if it also has any of
 * `strict_bits` (a subset of drop_bits) its 7 bands must all be -9999 or the chip is sent raw --
 * drop_bits = strict_bits = the fill bit is lossless; adding the cloud and shadow bits drops
 * only values the detection never reads (ccd_encode.c); QA words become 4-bit indices into the
 * chip's palette when it has at most 16 distinct words, else the chip is sent raw.  Layout:
 *   int64 n_chips; int64 chip_off[n_chips + 1] (bytes from `out`, 256-aligned);
 *   int64 chip_pix[n_chips + 1] (pixel prefix); chip sections:
 *   header (128 B): int32 mode (0 raw, 1 encoded), n_pix, n_obs, n_pal; uint16 pal[16];
 *                   int64 kept, data_off (the chip's offset in the standard layout), band_stride,
 *                   pix_base; uint32 drop_bits
 *   mode 1: uint32 kept_off[n_pix + 1]; uint8 qa4[n_pix][(n_obs + 1) / 2] (low nibble = even
 *           observation); int16 bands[7][band_stride] (kept observations, pixel-major) -- each
 *           part 16-byte aligned
 *   mode 0: uint16 qa[n_pix][n_obs]; int16 spectra[7][n_pix][n_obs].
 * ccdgpu_stage_slot_encoded uploads such a batch (and the dates) into a slot and decodes it on the
 * device, on the copy stream, into exactly the buffers ccdgpu_stage_slot_chips would fill; run it
 * with ccdgpu_run_slot.  ccdgpu_encode_vector_path: 1 if the encoder uses AVX-512 VBMI2. */
int64_t ccdgpu_encoded_bound(int32_t n_chips, const int32_t *n_pix, const int32_t *n_obs);
int64_t ccdgpu_encode_chips(int32_t n_chips, const int32_t *n_pix, const int32_t *n_obs, const int16_t *const *spectra,
                            const uint16_t *const *qa, uint8_t *out, int64_t out_cap, int32_t threads,
                            uint16_t drop_bits, uint16_t strict_bits);
int32_t ccdgpu_encode_vector_path(void);
/* The checks ccdgpu_stage_slot_encoded makes before an encoded batch is uploaded (no device
 * needed): the chip table, every section's header against the chip's shape, every section long
 * enough for its mode's layout, and each encoded section's kept-offset table a run per pixel
 * ending at its kept count.  0, or CCDGPU_EINVAL with the reason in ccdgpu_last_error(). */
int ccdgpu_encoded_check(int32_t n_chips, const int32_t *n_pix, const int32_t *n_obs, const uint8_t *enc,
                         int64_t enc_bytes);
int ccdgpu_stage_slot_encoded(ccdgpu_ctx *ctx, int32_t slot, const ccdgpu_params *params, int32_t n_chips,
                              const int32_t *n_pix, const int32_t *n_obs, const int64_t *dates, const uint8_t *enc,
                              int64_t enc_bytes);

/* Copy the staged pixel inputs back to the host in the ccdgpu_stage_chips layout; either
 * pointer may be NULL. */
int ccdgpu_staged_inputs(ccdgpu_ctx *ctx, int16_t *spectra, uint16_t *qa);
/* CSR result of staged chip `chip` (n_pix / n_obs of that chip). */
int ccdgpu_fetch_staged(ccdgpu_ctx *ctx, int32_t chip, ccdgpu_result *out);

/* Output writer: the segment / pixel table rows of staged chip `chip` of the last run, packed on
 * the device (ccd_rows.hip) for the chip at (cx, cy) with `width` pixels per chip row (100).
 * Replaces the per-segment Python formatting of ccdc/pyccd.py:106-148 + Spark's float cast. */
int ccdgpu_fetch_rows(ccdgpu_ctx *ctx, int32_t chip, int32_t cx, int32_t cy, int32_t width, ccdgpu_rows *out);
/* The same for every chip of the batch in one device pass and one copy (the tile runner's
 * gather): chip c at (cx[c], cy[c]); row_offsets over all pixels of the batch; the masks come
 * back bit-packed (out->mask_bits [n_pix of the batch][out->mask_words], out->mask NULL);
 * out->n_obs is 0 for a multi-chip batch. */
int ccdgpu_fetch_batch_rows(ccdgpu_ctx *ctx, const int32_t *cx, const int32_t *cy, int32_t width, ccdgpu_rows *out);
/* ccdgpu_fetch_batch_rows into the caller's buffers (no library allocation, no host copy of the
 * rows or mask words: with pinned buffers from ccdgpu_host_alloc they arrive by DMA):
 * row_offsets [total_pixels + 1], rows [*n_rows], mask_bits [total_pixels][mask_words].  The
 * row count is set in *n_rows even when a buffer is too small (CCDGPU_EINVAL, nothing fetched:
 * grow and call again).  The tile driver reuses one set of pinned buffers per context. */
int ccdgpu_fetch_batch_rows_into(ccdgpu_ctx *ctx, const int32_t *cx, const int32_t *cy, int32_t width,
                                 int64_t *row_offsets, int64_t offsets_cap, ccdgpu_row *rows, int64_t rows_cap,
                                 uint32_t *mask_bits, int64_t mask_cap, int64_t *n_rows);
void ccdgpu_rows_free(ccdgpu_rows *out);

/* Kernel statistics of the last run (per launch of the main detection kernel). */
typedef struct ccdgpu_stats {
    double detect_ms;           /* average duration of the detection kernel (HIP events)   */
    double prep_ms;             /* average duration of the per-chip preparation kernel     */
    int64_t pixels;             /* pixels processed by the last run                        */
    int64_t segments;           /* segments written                                        */
    int64_t lasso_fits;         /* band-model fits (7 per model)                           */
    int64_t cd_sweeps;          /* coordinate-descent sweeps summed over fits              */
    int64_t flops;              /* counted FP64 flops (SURVEY.md §8(d) op-count model)     */
    int64_t bytes;              /* algorithmic HBM bytes read+written                      */
    double detect_ms_device;    /* the detection kernel's execution window, first wave in to
                                   last wave out, on the device's 100 MHz clock (excludes time
                                   queued behind another context's launch)                 */
    int64_t pool_reruns;        /* launches rerun because the segment pool overflowed      */
    int64_t pool_cap;           /* segment-pool capacity after the run (segments)          */
    int64_t wave_slots;         /* persistent detection waves of the launch (resident slots) */
    int64_t n_cu;               /* compute units the detection kernel may use              */
} ccdgpu_stats;
int ccdgpu_last_stats(ccdgpu_ctx *ctx, ccdgpu_stats *stats);

/* Raw device counters of the last run (up to 48 words): [0] band fits, [1] CD sweeps, [2] counted
 * flops, [8 + k] phase-k cycle totals (only in the diagnostic build lib/libccdgpu_diag.so). */
int ccdgpu_diag_counters(ccdgpu_ctx *ctx, uint64_t *out, int32_t n);

#ifdef __cplusplus
}
#endif
#endif
