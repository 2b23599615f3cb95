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
#include <stddef.h>
#include <stdint.h>

#include "../../include/ccdgpu.h"

namespace {

constexpr int W = 64;

// skip: the detection's pool-overflow flag (batch chain: the segment counts then exceed what the
// pool holds, and the host reruns the batch), nullptr when the host checked it first; seg_cap /
// rows_cap bound every segment read and row write.
__global__ __launch_bounds__(256) void ccd_pack_rows(const ccdgpu_segment *__restrict__ seg, const int64_t *__restrict__ seg_off,
                                                     const int64_t *__restrict__ row_off, const uint32_t *__restrict__ mask_bits,
                                                     int mask_words, int n_pix, int n_obs, int cx, int cy, int width,
                                                     ccdgpu_row *__restrict__ rows, int8_t *__restrict__ mask,
                                                     const unsigned long long *__restrict__ skip, int64_t seg_cap,
                                                     int64_t rows_cap) {
    if (skip && *skip) return;
    const int wave = (int)(blockIdx.x * (blockDim.x / W) + threadIdx.x / W);
    const int l = threadIdx.x % W;
    const int nwaves = (int)(gridDim.x * (blockDim.x / W));
    for (int p = wave; p < n_pix; p += nwaves) {
        const int64_t s0 = seg_off[p], s1 = seg_off[p + 1];
        const int64_t r0 = row_off[p];
        const int px = cx + 30 * (p % width), py = cy - 30 * (p / width);
        // (offsets outside the segment array -- a batch chain after a pool overflow -- write nothing)
        if (s1 < s0 || s0 < 0 || (s1 > s0 && s1 > seg_cap) || s1 - s0 > 4096 || r0 < 0 || r0 >= rows_cap) continue;
        const int ns = (int)(s1 - s0);
        // one lane per row; a pixel without change models gets pyccd.default's row
        for (int j = l; j < (ns > 0 ? ns : 1); j += W) {
            if (r0 + j >= rows_cap || (ns > 0 && s0 + j >= seg_cap)) continue;
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

// Pool -> CSR with the segment count read on the device (counters[1] of the detection, for the
// batch chain that is enqueued before the count is known): grid-stride over the pooled segments,
// one wave per segment, its dwords copied lane-parallel; the pixel field becomes the pixel index
// within its chip (the same result as ccd_scatter in ccd_kernels.hip).
__global__ __launch_bounds__(256) void ccd_scatter_dev(const ccdgpu_segment *__restrict__ pool, const int32_t *__restrict__ seq,
                                                       const unsigned long long *__restrict__ n_pool_dev,
                                                       const unsigned long long *__restrict__ overflow, int64_t cap,
                                                       const int64_t *__restrict__ offsets, const int64_t *__restrict__ chip_pix_off,
                                                       int n_chips, ccdgpu_segment *__restrict__ out) {
    if (overflow && *overflow) return;  // the pool overflowed: the host reruns the batch
    const int64_t n = (int64_t)(*n_pool_dev < (unsigned long long)cap ? *n_pool_dev : (unsigned long long)cap);
    const int l = threadIdx.x % W;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / W);
    for (int64_t s = (int64_t)blockIdx.x * (blockDim.x / W) + threadIdx.x / W; s < n; s += nw) {
        const int gp = pool[s].pixel;
        int lo = 0, hi = n_chips - 1;  // chip of the pixel
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (chip_pix_off[mid] <= gp) lo = mid;
            else hi = mid - 1;
        }
        const int64_t dst = offsets[gp] + seq[s];
        if (dst < 0 || dst >= cap) continue;
        const uint32_t *src = reinterpret_cast<const uint32_t *>(pool + s);
        uint32_t *dd = reinterpret_cast<uint32_t *>(out + dst);
        constexpr int NW = (int)(sizeof(ccdgpu_segment) / 4);
        constexpr int PIXW = (int)(offsetof(ccdgpu_segment, pixel) / 4);
        for (int i = l; i < NW; i += W) dd[i] = (i == PIXW) ? (uint32_t)(gp - chip_pix_off[lo]) : src[i];
    }
}

// Rows per pixel (max(1, segments): pyccd.default's row for a pixel without a change model) with
// a trailing zero, for the exclusive scan into row offsets; and the CSR offsets' closing entry.
__global__ __launch_bounds__(256) void ccd_row_counts(const int32_t *__restrict__ nseg, int64_t *__restrict__ offsets,
                                                      int64_t n_pix, int64_t *__restrict__ rc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_pix) rc[i] = nseg[i] > 0 ? nseg[i] : 1;
    if (i == n_pix) {
        rc[n_pix] = 0;
        offsets[n_pix] = n_pix > 0 ? offsets[n_pix - 1] + nseg[n_pix - 1] : 0;
    }
}

}  // namespace

extern "C" int ccdk_scatter_dev(const ccdgpu_segment *pool, const int32_t *pool_seq, const unsigned long long *n_pool_dev,
                                const unsigned long long *overflow, int64_t cap, const int64_t *offsets,
                                const int64_t *chip_pix_off, int32_t n_chips, ccdgpu_segment *out, void *stream) {
    hipLaunchKernelGGL(ccd_scatter_dev, dim3(256), dim3(256), 0, (hipStream_t)stream, pool, pool_seq, n_pool_dev, overflow,
                       cap, offsets, chip_pix_off, n_chips, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ccdk_row_counts(const int32_t *nseg, int64_t *offsets, int64_t n_pix, int64_t *rc, void *stream) {
    const int64_t blocks = (n_pix + 1 + 255) / 256;
    hipLaunchKernelGGL(ccd_row_counts, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, nseg, offsets, n_pix, rc);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ccdk_pack_rows(const ccdgpu_segment *seg, const int64_t *seg_off, const int64_t *row_off,
                              const uint32_t *mask_bits, int32_t mask_words, int32_t n_pix, int32_t n_obs, int32_t cx,
                              int32_t cy, int32_t width, ccdgpu_row *rows, int8_t *mask, const unsigned long long *skip,
                              int64_t seg_cap, int64_t rows_cap, void *stream) {
    const int waves = n_pix < 4096 ? n_pix : 4096;
    const int blocks = (waves + 3) / 4;
    hipLaunchKernelGGL(ccd_pack_rows, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, (hipStream_t)stream, seg, seg_off,
                       row_off, mask_bits, mask_words, n_pix, n_obs, cx, cy, width, rows, mask, skip, seg_cap, rows_cap);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
