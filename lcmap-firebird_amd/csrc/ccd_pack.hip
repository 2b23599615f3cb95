// ccd_pack.hip -- MI355X (gfx950) chip packer: chipmunk wire format -> the detection kernel's
// band-major, observation-contiguous input buffers, on the device.
//
// Reference: ccdc/timeseries.py:120-125 builds per-pixel records with merlin.create (chipmunk
// chips per ubid and acquisition date, base64 int16/uint16 100x100 payloads; fixtures
// test/data/chip_response.json + registry_response.json) and then re-partitions them across
// the cluster.  Here the payloads of a chip's layers (7 spectral + pixel QA) for all of its
// acquisition dates are copied to HBM as text and one kernel decodes and pivots them:
//
//   text[(chip, obs, layer) payload]  base64 of n_pix little-endian 16-bit values, pixel order
//   -> spectra[chip][band][pix][obs] int16, qa[chip][pix][obs] uint16  (include/ccdgpu.h layout)
//
// One 256-thread block per (chip, layer, tile of 64 observations, tile of 96 pixels): 96 pixels
// are 192 bytes = 64 base64 quanta, so each observation row of the tile is one wave-wide decode
// (lane = 4-character quantum -> 3 bytes into LDS); the tile is then written pixel-major with
// consecutive threads on consecutive observations (128-byte runs per pixel).  HBM-bound byte
// work: no MFMA, no FP.  A missing layer (offset < 0) decodes as fill (-9999, QA bit 0 = fill).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int OBS_T = 64;   // observations per tile
constexpr int PIX_T = 96;   // pixels per tile = 192 bytes = 64 base64 quanta
constexpr int QUANTA = PIX_T * 2 / 3;
constexpr int NLAYER = 8;   // blues greens reds nirs swir1s swir2s thermals qas

// base64 character -> 6-bit value; 64 for '=' (padding), 255 for anything else
__device__ __forceinline__ unsigned b64v(unsigned c) {
    if (c >= 'A' && c <= 'Z') return c - 'A';
    if (c >= 'a' && c <= 'z') return c - 'a' + 26;
    if (c >= '0' && c <= '9') return c - '0' + 52;
    if (c == '+') return 62;
    if (c == '/') return 63;
    if (c == '=') return 64;
    return 255;
}

__global__ __launch_bounds__(256) void ccd_unpack_b64(const unsigned char *__restrict__ text, int64_t text_bytes,
                                                       const int64_t *__restrict__ offsets, int n_obs, int n_pix,
                                                       int16_t *__restrict__ spectra, uint16_t *__restrict__ qa,
                                                       unsigned long long *__restrict__ err) {
    __shared__ uint16_t tile[OBS_T][PIX_T + 2];  // +2: odd row pitch in 32-bit words
    const int ptile = blockIdx.x, otile = blockIdx.y;
    const int chip = blockIdx.z / NLAYER, layer = blockIdx.z % NLAYER;
    const int p0 = ptile * PIX_T, o0 = otile * OBS_T;
    const int tid = threadIdx.x;
    const int nbytes = 2 * n_pix;                    // decoded payload bytes
    const int64_t nchars = 4 * (int64_t)((nbytes + 2) / 3);  // encoded length incl. padding
    const uint16_t fill = layer == NLAYER - 1 ? (uint16_t)1 : (uint16_t)(int16_t)-9999;
    bool bad = false;
    // decode: thread -> (observation row, quantum); 64 rows x 64 quanta per tile
    for (int e = tid; e < OBS_T * QUANTA; e += 256) {
        const int r = e / QUANTA, q = e % QUANTA;
        const int o = o0 + r;
        if (o >= n_obs) continue;
        const int64_t off = offsets[((int64_t)chip * n_obs + o) * NLAYER + layer];
        const int64_t qg = (int64_t)ptile * QUANTA + q;  // quantum index within the payload
        uint16_t *row = tile[r];
        const int pb = 3 * q;                            // first decoded byte of this quantum, tile-relative
        unsigned char by[3] = {0, 0, 0};
        bool have = false;
        if (off >= 0 && 4 * qg < nchars) {
            const int64_t at = off + 4 * qg;
            if (at + 4 <= text_bytes) {
                const unsigned v0 = b64v(text[at]), v1 = b64v(text[at + 1]);
                const unsigned v2 = b64v(text[at + 2]), v3 = b64v(text[at + 3]);
                bad |= (v0 | v1) >= 64 || v2 > 64 || v3 > 64;
                const unsigned w = (v0 << 18) | (v1 << 12) | ((v2 & 63) << 6) | (v3 & 63);
                by[0] = (unsigned char)(w >> 16);
                by[1] = (unsigned char)(w >> 8);
                by[2] = (unsigned char)w;
                have = true;
            } else {
                bad = true;
            }
        }
        // bytes of this quantum -> 16-bit little-endian pixel values of the tile row
        for (int k = 0; k < 3; ++k) {
            const int b = pb + k;
            const int pix = b >> 1;
            if (pix >= PIX_T) continue;
            unsigned char *rb = reinterpret_cast<unsigned char *>(row);
            rb[b] = have ? by[k] : (unsigned char)((b & 1) ? (fill >> 8) : (fill & 0xFF));
        }
    }
    __syncthreads();
    // write: thread -> (pixel, observation), observations fastest (contiguous per pixel)
    const bool is_qa = layer == NLAYER - 1;
    const int64_t pstride = n_obs;
    for (int e = tid; e < PIX_T * OBS_T; e += 256) {
        const int pl = e / OBS_T, r = e % OBS_T;
        const int pix = p0 + pl, o = o0 + r;
        if (pix >= n_pix || o >= n_obs) continue;
        const uint16_t v = tile[r][pl];
        if (is_qa)
            qa[((int64_t)chip * n_pix + pix) * pstride + o] = v;
        else
            spectra[(((int64_t)chip * 7 + layer) * n_pix + pix) * pstride + o] = (int16_t)v;
    }
    if (bad) atomicOr(err, 1ull);
}

// ---- transport-encoded batches (ccd_encode.c; layout in include/ccdgpu.h) -> the standard
// band-major spectra [7][n_pix][n_obs] and QA [n_pix][n_obs] of every chip.  One wave per
// pixel, lane = observation: the 4-bit QA code through the chip's palette, the kept
// observations' (no drop bit) rank by ballot / mbcnt, band values gathered from the compacted
// band columns (consecutive ranks: coalesced) and -9999 written for the dropped ones.  Byte
// work at HBM speed: ~13 B read and 16 B written per observation.
constexpr int ENC_HDR = 128;
__device__ __forceinline__ int64_t up16(int64_t x) { return (x + 15) & ~(int64_t)15; }

__global__ __launch_bounds__(256) void ccd_decode_enc(const unsigned char *__restrict__ enc, int64_t total_pix,
                                                       int16_t *__restrict__ spectra, uint16_t *__restrict__ qa) {
    const int64_t pix = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (pix >= total_pix) return;
    const int l = threadIdx.x & 63;
    const int64_t *tab = reinterpret_cast<const int64_t *>(enc);
    const int64_t nc = tab[0];
    const int64_t *off = tab + 1, *pixo = tab + 2 + nc;
    int64_t lo = 0, hi = nc - 1;  // the pixel's chip (wave-uniform binary search)
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (pixo[mid] <= pix) lo = mid;
        else hi = mid - 1;
    }
    const unsigned char *sec = enc + off[lo];
    const int32_t *h = reinterpret_cast<const int32_t *>(sec);
    const int mode = h[0], n_pix = h[1], n_obs = h[2];
    const int64_t *h64 = reinterpret_cast<const int64_t *>(sec + 48);
    const int64_t data_off = h64[1], bstride = h64[2];
    const int64_t p = pix - pixo[lo];
    const int64_t plane = (int64_t)n_pix * n_obs;
    int16_t *sp = spectra + 7 * data_off + p * n_obs;
    uint16_t *qo = qa + data_off + p * n_obs;
    if (mode == 0) {
        const uint16_t *rq = reinterpret_cast<const uint16_t *>(sec + ENC_HDR) + p * n_obs;
        const int16_t *rs = reinterpret_cast<const int16_t *>(sec + ENC_HDR + up16(2 * plane)) + p * n_obs;
        for (int i = l; i < n_obs; i += 64) {
            qo[i] = rq[i];
#pragma unroll
            for (int b = 0; b < 7; ++b) sp[(int64_t)b * plane + i] = rs[(int64_t)b * plane + i];
        }
        return;
    }
    // the palette in registers (lane j < 16 holds entry j): a code is looked up with one lane
    // permute instead of a dependent global load
    const uint16_t palr = l < 16 ? reinterpret_cast<const uint16_t *>(sec + 16)[l] : (uint16_t)0;
    const unsigned drop = *reinterpret_cast<const uint32_t *>(sec + 80);  // QA bits whose bands were not sent
    const uint32_t *koff = reinterpret_cast<const uint32_t *>(sec + ENC_HDR);
    const unsigned char *q4 = sec + ENC_HDR + up16(4 * ((int64_t)n_pix + 1));
    const int64_t rowb = (n_obs + 1) / 2;
    const int16_t *bands = reinterpret_cast<const int16_t *>(q4 + up16((int64_t)n_pix * rowb)) + koff[p];
    // the pixel's kept run (the host checked the table); a code row that claims more kept
    // observations than the run holds reads no further than the run (its excess gets -9999)
    const int kcount = (int)(koff[p + 1] - koff[p]);
    const unsigned char *qr = q4 + p * rowb;
    int carry = 0;
    // four 64-observation chunks per round: their code bytes load together, then their ranks,
    // then all 28 band loads go out before the first store (latency once per round, not per chunk)
    constexpr int U = 4;
    for (int i0 = 0; i0 < n_obs; i0 += U * 64) {
        unsigned cb[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * 64 + l;
            cb[u] = i < n_obs ? (unsigned)qr[i >> 1] : 0u;
        }
        uint16_t q[U];
        bool keep[U];
        int rank[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * 64 + l;
            const bool in = i < n_obs;
            const int code = (int)((cb[u] >> ((i & 1) * 4)) & 15u);
            q[u] = (uint16_t)__shfl((int)palr, code, 64);
            keep[u] = in && !(q[u] & drop);
            const unsigned long long km = __ballot(keep[u]);
            rank[u] = carry + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(km >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)km, 0));
            carry += __popcll(km);
        }
        int16_t v[U][7];
#pragma unroll
        for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int b = 0; b < 7; ++b) v[u][b] = (int16_t)-9999;
            if (keep[u] && rank[u] < kcount) {  // (loads under the lane's own mask: a dropped lane's rank may point past the column)
#pragma unroll
                for (int b = 0; b < 7; ++b) v[u][b] = bands[b * bstride + rank[u]];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * 64 + l;
            if (i < n_obs) {
                qo[i] = q[u];
#pragma unroll
                for (int b = 0; b < 7; ++b) sp[(int64_t)b * plane + i] = v[u][b];
            }
        }
    }
}

}  // namespace

extern "C" int ccdk_decode_enc(const unsigned char *enc, int64_t total_pix, int16_t *spectra, uint16_t *qa,
                               void *stream) {
    if (total_pix <= 0) return 0;
    hipLaunchKernelGGL(ccd_decode_enc, dim3((unsigned)((total_pix + 3) / 4)), dim3(256), 0, (hipStream_t)stream, enc,
                       total_pix, spectra, qa);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ccdk_unpack_b64(const unsigned char *text, int64_t text_bytes, const int64_t *offsets, int32_t n_chips,
                               int32_t n_obs, int32_t n_pix, int16_t *spectra, uint16_t *qa,
                               unsigned long long *err, void *stream) {
    const dim3 grid((unsigned)((n_pix + PIX_T - 1) / PIX_T), (unsigned)((n_obs + OBS_T - 1) / OBS_T),
                    (unsigned)(n_chips * NLAYER));
    hipLaunchKernelGGL(ccd_unpack_b64, grid, dim3(256), 0, (hipStream_t)stream, text, text_bytes, offsets, n_obs,
                       n_pix, spectra, qa, err);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
