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

// Pool -> CSR and rows in one pass (batch chain): each wave takes 64 pooled segments, every lane
// resolves one of them (pixel, chip, position in the CSR and in the rows: the dependent loads
// of 64 segments in flight at once), then the wave copies them one after the other, all lanes
// over one segment's dwords -- the CSR record (the pixel field becoming the pixel index within
// its chip) and, with rows != nullptr, its float32 row (lanes over the row's 78 dwords, each
// converting its double; the same values as ccd_pack_rows).  n_pool_dev / overflow as
// ccd_scatter_dev; chip_xy [2 n_chips] the chips' (cx, cy).
constexpr int SEG_DW = (int)(sizeof(ccdgpu_segment) / 4);
constexpr int ROW_DW = (int)(sizeof(ccdgpu_row) / 4);
static_assert(ROW_DW == 8 + 10 * CCDGPU_NBANDS, "ccdgpu_row layout");
static_assert(offsetof(ccdgpu_row, chprob) == 28 && offsetof(ccdgpu_row, mag) == 32, "ccdgpu_row layout");
static_assert(offsetof(ccdgpu_segment, change_probability) == 24, "ccdgpu_segment layout");

// source double (index into the segment's doubles from change_probability) of row dword r >= 8
__device__ __forceinline__ int row_src(int r) {
    const int f = r - 8;  // mag[7], rmse[7], coef[7][7], intercept[7]
    constexpr int NB = CCDGPU_NBANDS;
    const int mag = 1, rmse = 1 + NB, icpt = 1 + 2 * NB, coef = 1 + 3 * NB;
    return f < NB ? mag + f : f < 2 * NB ? rmse + (f - NB) : f < 9 * NB ? coef + (f - 2 * NB) : icpt + (f - 9 * NB);
}

__global__ __launch_bounds__(256) void ccd_pool_rows(const ccdgpu_segment *__restrict__ pool, const int32_t *__restrict__ seq,
                                                     const unsigned long long *__restrict__ n_pool_dev, int64_t n_pool_host,
                                                     const unsigned long long *__restrict__ overflow, int64_t cap,
                                                     const int64_t *__restrict__ offsets, const int64_t *__restrict__ chip_pix_off,
                                                     int n_chips, ccdgpu_segment *__restrict__ out,
                                                     const int64_t *__restrict__ row_off, const int32_t *__restrict__ chip_xy,
                                                     int width, ccdgpu_row *__restrict__ rows, int64_t rows_cap) {
    if (overflow && *overflow) return;  // the pool overflowed: the host reruns the batch
    int64_t n = n_pool_host;
    if (n_pool_dev) n = (int64_t)*n_pool_dev;
    if (n > cap) n = cap;
    const int l = threadIdx.x % W;
    const int64_t nw = (int64_t)gridDim.x * (blockDim.x / W);
    for (int64_t base = ((int64_t)blockIdx.x * (blockDim.x / W) + threadIdx.x / W) * W; base < n; base += nw * W) {
        // lane l resolves segment base + l
        const int64_t s = base + l;
        int64_t dst = -1, rdst = -1;
        int lp = 0, px = 0, py = 0;
        if (s < n) {
            const int gp = pool[s].pixel;
            int lo = 0, hi = n_chips - 1;  // chip of the pixel
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (chip_pix_off[mid] <= gp) lo = mid;
                else hi = mid - 1;
            }
            const int sq = seq[s];
            dst = offsets[gp] + sq;
            if (dst < 0 || dst >= cap) dst = -1;
            lp = gp - (int)chip_pix_off[lo];
            if (rows) {
                rdst = row_off[gp] + sq;
                if (rdst < 0 || rdst >= rows_cap) rdst = -1;
                px = chip_xy[2 * lo] + 30 * (lp % width);
                py = chip_xy[2 * lo + 1] - 30 * (lp / width);
            }
        }
        const int cnt = n - base < W ? (int)(n - base) : W;
        for (int k = 0; k < cnt; ++k) {
            const int64_t d = __shfl(dst, k);
            const int64_t rd = __shfl(rdst, k);
            const int lpk = __shfl(lp, k);
            const uint32_t *src = reinterpret_cast<const uint32_t *>(pool + base + k);
            if (d >= 0 && out) {  // (out == nullptr: rows only)
                uint32_t *dd = reinterpret_cast<uint32_t *>(out + d);
                constexpr int PIXW = (int)(offsetof(ccdgpu_segment, pixel) / 4);
                for (int i = l; i < SEG_DW; i += W) dd[i] = (i == PIXW) ? (uint32_t)lpk : src[i];
            }
            if (rows && rd >= 0) {
                const int pxk = __shfl(px, k), pyk = __shfl(py, k);
                const ccdgpu_segment &sg = pool[base + k];
                const double *dv = &sg.change_probability;
                uint32_t *rw = reinterpret_cast<uint32_t *>(rows + rd);
                for (int r = l; r < ROW_DW; r += W) {
                    uint32_t v;
                    if (r >= 7) {
                        v = __float_as_uint(__double2float_rn(dv[r == 7 ? 0 : row_src(r)]));
                    } else {
                        // px, py, sday, eday, bday, curqa, has_model
                        v = r == 0 ? (uint32_t)pxk : r == 1 ? (uint32_t)pyk : r == 2 ? (uint32_t)sg.start_day
                          : r == 3 ? (uint32_t)sg.end_day : r == 4 ? (uint32_t)sg.break_day : r == 5 ? (uint32_t)sg.curve_qa : 1u;
                    }
                    rw[r] = v;
                }
            }
        }
    }
}

// pyccd.default's row for the pixels without a change model (batch chain, after ccd_pool_rows):
// one lane per pixel; such pixels are rare, each writes its row alone.
__global__ __launch_bounds__(256) void ccd_default_rows(const int32_t *__restrict__ nseg, int64_t n_pix,
                                                        const unsigned long long *__restrict__ overflow,
                                                        const int64_t *__restrict__ chip_pix_off, int n_chips,
                                                        const int64_t *__restrict__ row_off, const int32_t *__restrict__ chip_xy,
                                                        int width, ccdgpu_row *__restrict__ rows, int64_t rows_cap) {
    if (overflow && *overflow) return;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t gp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; gp < n_pix; gp += stride) {
        if (nseg[gp] != 0) continue;
        const int64_t r0 = row_off[gp];
        if (r0 < 0 || r0 >= rows_cap) continue;
        int lo = 0, hi = n_chips - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (chip_pix_off[mid] <= gp) lo = mid;
            else hi = mid - 1;
        }
        const int lp = (int)(gp - chip_pix_off[lo]);
        uint32_t *rw = reinterpret_cast<uint32_t *>(rows + r0);
        rw[0] = (uint32_t)(chip_xy[2 * lo] + 30 * (lp % width));
        rw[1] = (uint32_t)(chip_xy[2 * lo + 1] - 30 * (lp / width));
        rw[2] = rw[3] = rw[4] = 1u;  // sday, eday, bday
        for (int r = 5; r < ROW_DW; ++r) rw[r] = 0u;  // curqa, has_model, chprob and every float 0
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

extern "C" int ccdk_pool_rows(const ccdgpu_segment *pool, const int32_t *pool_seq, const unsigned long long *n_pool_dev,
                              int64_t n_pool_host, const unsigned long long *overflow, int64_t cap, const int64_t *offsets,
                              const int64_t *chip_pix_off, int32_t n_chips, ccdgpu_segment *out, const int64_t *row_off,
                              const int32_t *chip_xy, int32_t width, ccdgpu_row *rows, int64_t rows_cap, int32_t blocks,
                              void *stream) {
    if (!n_pool_dev && n_pool_host <= 0) return 0;
    if (blocks <= 0) blocks = 1;
    hipLaunchKernelGGL(ccd_pool_rows, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, pool, pool_seq, n_pool_dev,
                       n_pool_host, overflow, cap, offsets, chip_pix_off, n_chips, out, row_off, chip_xy, width, rows, rows_cap);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ccdk_default_rows(const int32_t *nseg, int64_t n_pix, const unsigned long long *overflow,
                                 const int64_t *chip_pix_off, int32_t n_chips, const int64_t *row_off, const int32_t *chip_xy,
                                 int32_t width, ccdgpu_row *rows, int64_t rows_cap, void *stream) {
    if (n_pix <= 0) return 0;
    const int64_t b = (n_pix + 255) / 256;
    const unsigned blocks = (unsigned)(b < 256 ? b : 256);
    hipLaunchKernelGGL(ccd_default_rows, dim3(blocks), dim3(256), 0, (hipStream_t)stream, nseg, n_pix, overflow, chip_pix_off,
                       n_chips, row_off, chip_xy, width, rows, rows_cap);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
