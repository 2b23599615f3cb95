// ccd_device.h -- device-side data contract shared by the HIP kernels and the host API.
//
// Layout in HBM.  One "staged batch" = n_chips chips (pixel groups sharing one date vector);
// chip c has np_c = chip_npix[c] pixels and n_c = chip_nobs[c] observations, and its arrays are
// packed back to back (a tile's base-cadence and sidelap chips stage together):
//   dates     int64 [n_c]            at chip_obs_off[c]       input order (merlin: descending)
//   spectra   int16 [7][np_c][n_c]   at 7 * chip_data_off[c]  band-major, observation-contiguous
//   qa        uint16[np_c][n_c]      at chip_data_off[c]
//   order     int32 [n_c]            at chip_obs_off[c]       sorted position -> input position
//   sdates    int64 [n_c]            at chip_obs_off[c]       sorted dates
//   basis     f64   [n_c][8]         at 8 * chip_obs_off[c]   t, cos wt, sin wt, cos 2wt, sin 2wt,
//                                    cos 3wt, sin 3wt, 0 (models/lasso.coefficient_matrix rows,
//                                    shared by all pixels of the chip)
//   chip_obs_off = prefix sum of n_c, chip_pix_off = prefix sum of np_c (pixel p of the batch is
//   pixel p - chip_pix_off[c] of chip c), chip_data_off = prefix sum of np_c * n_c.
//   per wave slot scratch (persistent grid, sized by the largest n_c): compacted period of the
//     current pixel, cdate int32[n], row {int16 v[7]; uint16 cidx}[n]  (20 B / observation)
//   outputs: mask bits ([pixel][mask_words], mask_words from the largest n_c), procedure, probs,
//   per-pixel segment count, segment pool (+ seq numbers)
#pragma once
#include <stdint.h>

#include "../../include/ccdgpu.h"

// launch statistics words: 8 counters + CCD_NSTATS - 8 diagnostic phase slots
#define CCD_NSTATS 48
#define CCD_NB 7
#define CCD_WAVE 64
#define CCD_BASIS_STRIDE 8
// per-slot double scratch: [8][n_obs_max] (Tmask columns / closest-DOY r^2) + the overflow of
// the peek-residual ring (7 bands x (CCDGPU_MAX_PEEK - 64) observations)
#define CCD_RING_OVF 256
#define CCD_SLOT_F64(nmax) ((size_t)8 * (size_t)(nmax) + CCD_RING_OVF)
// launch-argument slots in constant memory: contexts of one process that can run at once
#define CCD_ARG_SLOTS 16

struct CcdDetectArgs {
    ccdgpu_params p;
    int32_t n_chips, n_obs_max, mask_words;
    int32_t n_slots;
    int32_t poison;  // 1: every pixel starts from an LDS block filled with NaN bytes (test mode)
    int32_t pad0;
    int64_t total_pix;
    int64_t pool_cap;
    const int32_t *chip_nobs;      // [n_chips]
    const int64_t *chip_obs_off;   // [n_chips + 1]
    const int64_t *chip_pix_off;   // [n_chips + 1]
    const int64_t *chip_data_off;  // [n_chips + 1]
    const int16_t *spectra;
    const uint16_t *qa;
    // non-null: the batch's inputs are a transport-encoded batch (include/ccdgpu.h) read in place
    // by the detection kernel (spectra / qa unused)
    const unsigned char *enc;
    const int32_t *order;
    const int64_t *sdates;
    const double *basis;
    // work queue + global flags: [0] next pixel, [1] pool count, [2] first QA-error pixel (min),
    // [3] pool overflow, [4] first source line whose index guard tripped (0 = none),
    // [5] / [6] s_memrealtime of the first wave's start / the last wave's end (100 MHz),
    // [7] first pixel whose adaptive peek exceeds CCDGPU_MAX_PEEK (min; ~0 = none)
    unsigned long long *counters;
    // per-slot scratch
    int32_t *s_date;
    uint16_t *s_row;  // [n_slots][n_obs][8]: int16 band values 0..6, uint16 sorted index
    double *s_f64;   // [n_slots][CCD_SLOT_F64(n_obs)] Tmask scratch / closest-DOY squared residuals / ring overflow
    uint16_t *s_bk;  // [n_slots][n_obs] closest-DOY bucket list
    // outputs
    uint32_t *mask_bits;
    int32_t *procedure;
    double *probs;
    int32_t *nseg;
    ccdgpu_segment *pool;
    int32_t *pool_seq;
    // instrumentation: [0] fits (band models), [1] CD sweeps, [2] counted flops
    unsigned long long *stats;
    // change threshold per (adaptive) peek size, index = peek (<= CCDGPU_MAX_PEEK)
    double thr_table[CCDGPU_MAX_PEEK + 1];
};

#ifdef __cplusplus
extern "C" {
#endif
// kernel launchers (ccd_kernels.hip)
int ccdk_prep(const int64_t *dates, int32_t n_chips, const int32_t *chip_nobs, const int64_t *chip_obs_off,
              double avg_days_yr, int32_t argsort_stable, int32_t *order, int64_t *sdates, double *basis,
              void *stream);
// the detection kernel reads its arguments from slot arg_slot of a __constant__ array (one slot
// per live context, so contexts on one device may launch concurrently from their own streams)
int ccdk_set_args(const CcdDetectArgs *host_args, int arg_slot, void *stream);
int ccdk_detect(int32_t grid, int variant, int32_t n_obs_max, int arg_slot, void *stream);
// dynamic LDS bytes per wave and resident waves per CU for a period of n_obs observations
size_t ccdk_lds_bytes(int32_t n_obs);
int ccdk_occupancy(int variant, int32_t n_obs);
// chipmunk wire format -> spectra / qa (ccd_pack.hip); err: set to 1 on invalid base64
int ccdk_unpack_b64(const unsigned char *text, int64_t text_bytes, const int64_t *offsets, int32_t n_chips,
                    int32_t n_obs, int32_t n_pix, int16_t *spectra, uint16_t *qa, unsigned long long *err,
                    void *stream);
// transport-encoded batch (ccd_encode.c) -> spectra / qa in the standard layout (ccd_pack.hip)
int ccdk_decode_enc(const unsigned char *enc, int64_t total_pix, int16_t *spectra, uint16_t *qa, void *stream);
// detection results -> segment / pixel table rows (ccd_rows.hip)
// (skip: nullptr, or a device flag that makes the launch write nothing; seg_cap / rows_cap bound
// the segment reads and row writes)
int ccdk_pack_rows(const ccdgpu_segment *seg, const int64_t *seg_off, const int64_t *row_off, const uint32_t *mask_bits,
                   int32_t mask_words, int32_t n_pix, int32_t n_obs, int32_t cx, int32_t cy, int32_t width,
                   ccdgpu_row *rows, int8_t *mask, const unsigned long long *skip, int64_t seg_cap, int64_t rows_cap,
                   void *stream);
// the batch chain of ccdgpu_run_slot_begin_rows (ccd_rows.hip): pool -> CSR with the segment
// count read on the device (counters[1], at most cap); rows per pixel for the row-offset scan
// (overflow: the detection's pool-overflow flag -- set, the chain's kernels write nothing and the
// host reruns the batch with a larger pool)
int ccdk_scatter_dev(const ccdgpu_segment *pool, const int32_t *pool_seq, const unsigned long long *n_pool_dev,
                     const unsigned long long *overflow, int64_t cap, const int64_t *offsets,
                     const int64_t *chip_pix_off, int32_t n_chips, ccdgpu_segment *out, void *stream);
int ccdk_row_counts(const int32_t *nseg, int64_t *offsets, int64_t n_pix, int64_t *rc, void *stream);
// pool -> CSR (and, rows != nullptr, the float32 rows) in one pass; segment count from n_pool_dev
// when given, else n_pool_host; writes nothing when *overflow (ccd_rows.hip)
int ccdk_pool_rows(const ccdgpu_segment *pool, const int32_t *pool_seq, const unsigned long long *n_pool_dev,
                   int64_t n_pool_host, const unsigned long long *overflow, int64_t cap, const int64_t *offsets,
                   const int64_t *chip_pix_off, int32_t n_chips, ccdgpu_segment *out, const int64_t *row_off,
                   const int32_t *chip_xy, int32_t width, ccdgpu_row *rows, int64_t rows_cap, int32_t blocks, void *stream);
// pyccd.default's row for every pixel without a change model
int ccdk_default_rows(const int32_t *nseg, int64_t n_pix, const unsigned long long *overflow,
                      const int64_t *chip_pix_off, int32_t n_chips, const int64_t *row_off, const int32_t *chip_xy,
                      int32_t width, ccdgpu_row *rows, int64_t rows_cap, void *stream);
// pool -> CSR; the segment's pixel field becomes the pixel index within its chip
int ccdk_scatter(const ccdgpu_segment *pool, const int32_t *pool_seq, int64_t n_pool,
                 const int64_t *offsets, const int64_t *chip_pix_off, int32_t n_chips, ccdgpu_segment *out,
                 void *stream);
#ifdef __cplusplus
}
#endif
