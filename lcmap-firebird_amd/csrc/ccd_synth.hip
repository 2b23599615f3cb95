// ccd_synth.hip -- the synthetic ARD generator on a gfx950 GPU (include/ccdsynth.h,
// ccdsynth_gpu_*): bench / test input only.  A tile's 2500 distinct chips are ~0.7 TB of ARD,
// hours of host generation; here every sample is computed by the same arithmetic as the host
// generator (csrc/synth_core.h) in HBM and then copied to the caller's host buffers, so the
// inputs reach the detection path through host memory and PCIe exactly like fetched ARD would.
//
// Mapping: one 64-lane wave per pixel.  Lanes 0..6 derive the pixel's per-band parameters and
// lane 0 its break schedule into the wave's LDS block; then lane = observation, so every band's
// int16 row [band][pixel][obs] and the QA row are written by coalesced stores.  Built without FMA
// contraction, as synth.c is.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "synth_core.h"

namespace {

constexpr int WAVES = 4;  // pixels per 256-thread block

struct ChipJob {
    int32_t chip, pix0, n_pix, n_obs;
    int64_t obs_off, data_off;
};

struct PixelLds {
    double base[7], amp[7], slope[7], phase[7];
    double brk_t[SYN_MAX_BREAKS];
    double brk_step[SYN_MAX_BREAKS * 7];
    int n_brk;
};

__global__ __launch_bounds__(256) void synth_chips(ccdsynth_cfg cfg, const ChipJob *jobs, const int64_t *dates,
                                                   int16_t *spectra, uint16_t *qa) {
    __shared__ PixelLds lds[WAVES];
    const ChipJob J = jobs[blockIdx.y];
    const int wv = threadIdx.x / 64, l = threadIdx.x % 64;
    const int pi = blockIdx.x * WAVES + wv;  // pixel within the job
    PixelLds &P = lds[wv];
    const bool live = pi < J.n_pix;
    const int32_t pix = J.pix0 + pi;
    if (live && l < 7) syn_pixel_band(cfg.seed, J.chip, pix, l, &P.base[l], &P.amp[l], &P.slope[l], &P.phase[l]);
    __syncthreads();
    if (live && l == 0) P.n_brk = syn_breaks(&cfg, J.chip, pix, P.base, P.brk_t, P.brk_step);
    __syncthreads();
    if (!live) return;
    const int n = J.n_obs, np = J.n_pix;
    const int64_t *d = dates + J.obs_off;
    int16_t *sp = spectra + 7 * J.data_off;
    uint16_t *q = qa + J.data_off;
    for (int i = l; i < n; i += 64) {
        int16_t v[7];
        const uint16_t qw = syn_obs(&cfg, J.chip, pix, i, d[i], P.base, P.amp, P.slope, P.phase, P.n_brk, P.brk_t,
                                    P.brk_step, v);
#pragma unroll
        for (int b = 0; b < 7; ++b) sp[((size_t)b * np + pi) * n + i] = v[b];
        q[(size_t)pi * n + i] = qw;
    }
}

thread_local std::string t_err;

int fail(const std::string &m) {
    t_err = m;
    return -1;
}

}  // namespace

struct ccdsynth_gpu {
    int device = 0;
    hipStream_t stream = nullptr;
    void *d_dates = nullptr, *d_spectra = nullptr, *d_qa = nullptr, *d_jobs = nullptr;
    size_t cap_dates = 0, cap_data = 0, cap_qa = 0, cap_jobs = 0;
};

static int grow(void **p, size_t &cap, size_t need) {
    if (need <= cap) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    if (hipMalloc(p, need) != hipSuccess) return fail("hipMalloc of " + std::to_string(need) + " bytes failed");
    cap = need;
    return 0;
}

#define HCK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_)); \
    } while (0)

extern "C" const char *ccdsynth_gpu_error(void) { return t_err.c_str(); }

extern "C" int ccdsynth_gpu_create(int device, ccdsynth_gpu **out) {
    if (!out) return fail("out is NULL");
    int n = 0;
    HCK(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) return fail("device " + std::to_string(device) + " not present");
    HCK(hipSetDevice(device));
    ccdsynth_gpu *g = new ccdsynth_gpu;
    g->device = device;
    if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
        delete g;
        return fail("hipStreamCreate failed");
    }
    *out = g;
    return 0;
}

extern "C" void ccdsynth_gpu_destroy(ccdsynth_gpu *g) {
    if (!g) return;
    (void)hipSetDevice(g->device);
    if (g->stream) (void)hipStreamSynchronize(g->stream);
    for (void *p : {g->d_dates, g->d_spectra, g->d_qa, g->d_jobs})
        if (p) (void)hipFree(p);
    if (g->stream) (void)hipStreamDestroy(g->stream);
    delete g;
}

extern "C" int ccdsynth_gpu_batch(ccdsynth_gpu *g, const ccdsynth_cfg *cfg, int32_t n_chips, const int32_t *chip_ids,
                                  const int32_t *pix0, const int32_t *n_pix, const int32_t *n_obs, const int64_t *obs_off,
                                  const int64_t *data_off, const int64_t *dates, int16_t *spectra, uint16_t *qa) {
    if (!g || !cfg || n_chips <= 0 || !chip_ids || !pix0 || !n_pix || !n_obs || !obs_off || !data_off || !dates ||
        !spectra || !qa)
        return fail("invalid arguments");
    if (n_chips > 65535) return fail("at most 65535 chips per call");
    HCK(hipSetDevice(g->device));
    // the batch's extent: dates [0, max(obs_off + n_obs)), data [0, max(data_off + n_pix * n_obs))
    int64_t n_dates = 0, n_data = 0, max_pix = 0;
    ChipJob *jobs = new ChipJob[n_chips];
    for (int c = 0; c < n_chips; ++c) {
        if (n_pix[c] <= 0 || n_obs[c] <= 0 || obs_off[c] < 0 || data_off[c] < 0 || pix0[c] < 0) {
            delete[] jobs;
            return fail("chip " + std::to_string(c) + ": invalid pixel / observation counts or offsets");
        }
        jobs[c] = ChipJob{chip_ids[c], pix0[c], n_pix[c], n_obs[c], obs_off[c], data_off[c]};
        n_dates = std::max<int64_t>(n_dates, obs_off[c] + n_obs[c]);
        n_data = std::max<int64_t>(n_data, data_off[c] + (int64_t)n_pix[c] * n_obs[c]);
        max_pix = std::max<int64_t>(max_pix, n_pix[c]);
    }
    int rc = grow(&g->d_dates, g->cap_dates, sizeof(int64_t) * n_dates);
    if (!rc) rc = grow(&g->d_spectra, g->cap_data, sizeof(int16_t) * 7 * n_data);
    if (!rc) rc = grow(&g->d_qa, g->cap_qa, sizeof(uint16_t) * n_data);
    if (!rc) rc = grow(&g->d_jobs, g->cap_jobs, sizeof(ChipJob) * n_chips);
    if (rc) {
        delete[] jobs;
        return rc;
    }
    hipError_t e = hipMemcpyAsync(g->d_jobs, jobs, sizeof(ChipJob) * n_chips, hipMemcpyHostToDevice, g->stream);
    if (e == hipSuccess)
        e = hipMemcpyAsync(g->d_dates, dates, sizeof(int64_t) * n_dates, hipMemcpyHostToDevice, g->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(g->stream);  // jobs[] is a host temporary
    delete[] jobs;
    HCK(e);
    const dim3 grid((unsigned)((max_pix + WAVES - 1) / WAVES), (unsigned)n_chips);
    // Page-locked host buffers are written by the kernel itself, straight over PCIe (no DMA copy:
    // the copy engines stay free for the detection path's uploads); pageable ones through HBM and a
    // device-to-host copy.  CCDSYNTH_D2H=copy forces the latter (A/B measurements).
    hipPointerAttribute_t as{}, aq{};
    const char *mode = getenv("CCDSYNTH_D2H");
    const bool direct = !(mode && !strcmp(mode, "copy")) && hipPointerGetAttributes(&as, spectra) == hipSuccess &&
                        hipPointerGetAttributes(&aq, qa) == hipSuccess && as.type == hipMemoryTypeHost &&
                        aq.type == hipMemoryTypeHost && as.devicePointer && aq.devicePointer;
    (void)hipGetLastError();  // (a pageable pointer leaves an error from the attribute query)
    if (direct) {
        hipLaunchKernelGGL(synth_chips, grid, dim3(64 * WAVES), 0, g->stream, *cfg, (const ChipJob *)g->d_jobs,
                           (const int64_t *)g->d_dates, (int16_t *)as.devicePointer, (uint16_t *)aq.devicePointer);
        HCK(hipGetLastError());
    } else {
        hipLaunchKernelGGL(synth_chips, grid, dim3(64 * WAVES), 0, g->stream, *cfg, (const ChipJob *)g->d_jobs,
                           (const int64_t *)g->d_dates, (int16_t *)g->d_spectra, (uint16_t *)g->d_qa);
        HCK(hipGetLastError());
        HCK(hipMemcpyAsync(spectra, g->d_spectra, sizeof(int16_t) * 7 * n_data, hipMemcpyDeviceToHost, g->stream));
        HCK(hipMemcpyAsync(qa, g->d_qa, sizeof(uint16_t) * n_data, hipMemcpyDeviceToHost, g->stream));
    }
    HCK(hipStreamSynchronize(g->stream));
    return 0;
}
