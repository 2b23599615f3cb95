// ccd_rows.hip -- MI355X (gfx950) output writer: detection results -> the rows of the reference's
// segment and pixel tables with their storage types.
//
// Reference: ccdc/pyccd.py:106-148 formats one row dict per change model (pyccd.default's day-1
// row for a pixel without any), Spark casts every FloatType column to float32
// (ccdc/segment.py:16-55, pyccd.py:39-96) and Cassandra stores them as float / tinyint /
// list<float> (resources/schema.cql segment, pixel).  Here one wave per pixel writes the
// pixel's rows as ccdgpu_row records (float32 by round-to-nearest, the Python float -> Java
// float cast) and the pixel table's processing mask as one byte per date (sorted order), so the
// host only formats the ISO day strings.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ccdgpu.h"

namespace {

constexpr int W = 64;

__global__ __launch_bounds__(256) void ccd_pack_rows(const ccdgpu_segment *__restrict__ seg, const int64_t *__restrict__ seg_off,
                                                     const int64_t *__restrict__ row_off, const uint32_t *__restrict__ mask_bits,
                                                     int mask_words, int n_pix, int n_obs, int cx, int cy, int width,
                                                     ccdgpu_row *__restrict__ rows, int8_t *__restrict__ mask) {
    const int wave = (int)(blockIdx.x * (blockDim.x / W) + threadIdx.x / W);
    const int l = threadIdx.x % W;
    const int nwaves = (int)(gridDim.x * (blockDim.x / W));
    for (int p = wave; p < n_pix; p += nwaves) {
        const int64_t s0 = seg_off[p], s1 = seg_off[p + 1];
        const int64_t r0 = row_off[p];
        const int px = cx + 30 * (p % width), py = cy - 30 * (p / width);
        const int ns = (int)(s1 - s0);
        // one lane per row; a pixel without change models gets pyccd.default's row
        for (int j = l; j < (ns > 0 ? ns : 1); j += W) {
            ccdgpu_row r;
            r.px = px;
            r.py = py;
            if (ns == 0) {
                r.sday = r.eday = r.bday = 1;
                r.curqa = 0;
                r.has_model = 0;
                r.chprob = 0.f;
                for (int b = 0; b < CCDGPU_NBANDS; ++b) {
                    r.mag[b] = r.rmse[b] = r.intercept[b] = 0.f;
                    for (int k = 0; k < 7; ++k) r.coef[b][k] = 0.f;
                }
            } else {
                const ccdgpu_segment &s = seg[s0 + j];
                r.sday = s.start_day;
                r.eday = s.end_day;
                r.bday = s.break_day;
                r.curqa = s.curve_qa;
                r.has_model = 1;
                r.chprob = __double2float_rn(s.change_probability);
                for (int b = 0; b < CCDGPU_NBANDS; ++b) {
                    r.mag[b] = __double2float_rn(s.magnitude[b]);
                    r.rmse[b] = __double2float_rn(s.rmse[b]);
                    r.intercept[b] = __double2float_rn(s.intercept[b]);
                    for (int k = 0; k < 7; ++k) r.coef[b][k] = __double2float_rn(s.coef[b][k]);
                }
            }
            rows[r0 + j] = r;
        }
        // pixel table: processing mask, one byte per date (sorted order); skipped when the
        // caller fetches the bit-packed mask instead
        if (!mask) continue;
        const uint32_t *mb = mask_bits + (int64_t)p * mask_words;
        int8_t *mo = mask + (int64_t)p * n_obs;
        for (int i = l; i < n_obs; i += W) mo[i] = (int8_t)((mb[i >> 5] >> (i & 31)) & 1u);
    }
}

}  // namespace

extern "C" int ccdk_pack_rows(const ccdgpu_segment *seg, const int64_t *seg_off, const int64_t *row_off,
                              const uint32_t *mask_bits, int32_t mask_words, int32_t n_pix, int32_t n_obs, int32_t cx,
                              int32_t cy, int32_t width, ccdgpu_row *rows, int8_t *mask, void *stream) {
    const int waves = n_pix < 4096 ? n_pix : 4096;
    const int blocks = (waves + 3) / 4;
    hipLaunchKernelGGL(ccd_pack_rows, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, (hipStream_t)stream, seg, seg_off,
                       row_off, mask_bits, mask_words, n_pix, n_obs, cx, cy, width, rows, mask);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
