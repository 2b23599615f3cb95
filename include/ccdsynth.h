/* ccdsynth.h -- deterministic synthetic Landsat ARD chip generator (bench / test input only).
 *
 * Produces the per-chip record layout that ccdc/timeseries.py:92-126 builds through
 * merlin.create (dates descending as merlin delivers them, timeseries.py:115; int16 spectra
 * with fill -9999; uint16 bit-packed PIXELQA), in the band-major, observation-contiguous layout
 * the detection ABI consumes (include/ccdgpu.h).  Configs follow SURVEY.md §8(d): C2 (chip,
 * n~1000), C3 (tile cadence L4-L8 1982-2017 + sidelap), C4 (high cloud/snow), C5 (breaks every
 * ~3 yr).  Counter-based RNG: every value depends only on (seed, chip, pixel, obs), so any subset
 * of pixels regenerates bit-identically on any host.
 */
#ifndef CCDSYNTH_H
#define CCDSYNTH_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ccdsynth_cfg {
    int32_t n_obs_target;      /* subsample the cadence down to this many dates (0 = natural) */
    int32_t sidelap;           /* 1: add the +7 day sidelap path (50 % of its acquisitions)   */
    int32_t change_every_days; /* 0: no abrupt change; else mean days between breaks          */
    int32_t first_year_l4;     /* 1: include Landsat 4 (1982-1993)                             */
    double p_clear, p_cloud, p_shadow, p_snow, p_water, p_fill; /* per-observation class mix  */
    double p_saturated;        /* share of clear obs with one optical band saturated          */
    double p_hot_thermal;      /* share of clear obs with thermal > 327.6 K (int16 wrap path)  */
    uint64_t seed;
} ccdsynth_cfg;

/* Fill cfg with a named config: 2 = C2 chip, 3 = C3 tile chip, 4 = C4 stress, 5 = C5 change-dense. */
int ccdsynth_config(int which, ccdsynth_cfg *cfg);

/* Acquisition dates of chip `chip_index` (proleptic Gregorian ordinals, DESCENDING).
 * Writes at most `cap` values; returns the count (or the required count if dates == NULL). */
int ccdsynth_dates(const ccdsynth_cfg *cfg, int32_t chip_index, int64_t *dates, int32_t cap);

/* Spectra [7][n_pix][n_obs] (blue, green, red, nir, swir1, swir2, thermal K*10) and
 * qa [n_pix][n_obs] for pixels pix0 .. pix0+n_pix-1 of the chip (pixel = row*100 + col). */
int ccdsynth_chip(const ccdsynth_cfg *cfg, int32_t chip_index, int32_t pix0, int32_t n_pix,
                  int32_t n_obs, const int64_t *dates, int16_t *spectra, uint16_t *qa);

/* A chip whose every pixel series (7 bands and QA) is the given chip's rotated left by `shift`
 * observations against the same dates: out[i] = in[(i + shift) mod n_obs].  The bench's source of
 * a tile's distinct chips (ccdgpu.synth.TileSource 'pool' mode): a pool of generated chips, each
 * tile position a different rotation, produced by copies at memory speed.  OpenMP, `threads`. */
int ccdsynth_rotate(const int16_t *spectra, const uint16_t *qa, int32_t n_pix, int32_t n_obs, int32_t shift,
                    int16_t *spectra_out, uint16_t *qa_out, int32_t threads);

/* ---- device generator (lib/libccdsynth.so, csrc/ccd_synth.hip): the same samples computed on
 * a gfx950 GPU and copied into host buffers (pinned for full PCIe rate), for inputs too large to
 * generate on the host (a tile's 2500 distinct chips).  Same arithmetic as ccdsynth_chip
 * (csrc/synth_core.h); see there for how close the two agree.  One handle per thread. */
typedef struct ccdsynth_gpu ccdsynth_gpu;
int ccdsynth_gpu_create(int device, ccdsynth_gpu **out);
void ccdsynth_gpu_destroy(ccdsynth_gpu *g);
/* last error of this thread's calls (static string) */
const char *ccdsynth_gpu_error(void);
/* n_chips chips: chip c is tile chip chip_ids[c] with pixels pix0[c] .. pix0[c]+n_pix[c]-1 and the
 * n_obs[c] dates at dates + obs_off[c] (host, as ccdsynth_dates writes them).  Writes spectra
 * [7][n_pix][n_obs] at spectra + 7 * data_off[c] and qa [n_pix][n_obs] at qa + data_off[c] (host
 * buffers: the layout of a staged batch, ccdgpu_stage_chips).  Returns 0 when the copies are done. */
int ccdsynth_gpu_batch(ccdsynth_gpu *g, const ccdsynth_cfg *cfg, int32_t n_chips, const int32_t *chip_ids,
                       const int32_t *pix0, const int32_t *n_pix, const int32_t *n_obs, const int64_t *obs_off,
                       const int64_t *data_off, const int64_t *dates, int16_t *spectra, uint16_t *qa);

#ifdef __cplusplus
}
#endif
#endif
