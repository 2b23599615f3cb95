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
// One 256-thread block per (chip, layer, tile of 128 observations, tile of 96 pixels): 96
// pixels are 192 bytes = 64 base64 quanta = 32 pairs of quanta = 3 pixels per pair.
//   decode: lane = (observation row, pair of quanta): 8 characters in one load, mapped to 6-bit
//           values through a 256-byte table in LDS (one dword per bank: conflict-free), -> 3
//           pixels as 16-bit LDS stores into a pixel-major tile;
//   write:  wave = pixel row, lane = 32-bit word of the output row (256 contiguous bytes per
//           pixel per block; the tile rows are shifted by the output's word alignment).
// HBM-bound byte work: no MFMA, no FP.  A missing layer (offset < 0) decodes as fill (-9999,
// QA bit 0 = fill).  Round 6: from a lane-per-quantum form with 64-observation tiles, byte
// loads and a branchy character decode (1.06 TB/s) to 3.5 TB/s of algorithmic bytes -- the
// table lookup halved the time (the old decode was VALU-bound), DESIGN.md §6b.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int OBS_T = 128;  // observations per tile
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

static_assert(256 % (QUANTA / 2) == 0 && OBS_T * (QUANTA / 2) % 256 == 0, "decode items per thread");
constexpr int PAIRS = QUANTA / 2;      // 32 quantum pairs = 96 pixels
constexpr int OPITCH = OBS_T + 2;      // LDS row pitch in 16-bit words: 65 dwords (odd)
static_assert(OBS_T == 128, "the write phase gives each lane two observations of a row");

__global__ __launch_bounds__(256, 6) void ccd_unpack_b64(const unsigned char *__restrict__ text, int64_t text_bytes,
                                                         const int64_t *__restrict__ offsets, int n_obs, int n_pix,
                                                         int16_t *__restrict__ spectra, uint16_t *__restrict__ qa,
                                                         unsigned long long *__restrict__ err, unsigned n_ptiles,
                                                         unsigned n_otiles, unsigned n_tiles) {
    __shared__ uint16_t tile[PIX_T][OPITCH];  // pixel-major: the write phase reads along a row
    __shared__ unsigned char lut[256];        // character -> b64v; 64 dwords = one per LDS bank
    __shared__ int64_t roff[OBS_T];           // payload offset of each observation row
    // XCD-aware order: the hardware deals block ids round-robin over the 8 XCDs, so ids
    // id, id + 8, ..., id + 56 of each run of 64 share an XCD; they take 8 consecutive tiles
    // (pixel tile fastest), whose text rows are adjacent and share cache lines at their ends:
    // those lines are then fetched into one L2, not two
    const unsigned lt = (blockIdx.x & ~63u) + (blockIdx.x % 8) * 8 + (blockIdx.x / 8) % 8;
    if (lt >= n_tiles) return;
    const int ptile = (int)(lt % n_ptiles);
    const int otile = (int)(lt / n_ptiles % n_otiles);
    const int cl = (int)(lt / (n_ptiles * n_otiles));
    const int chip = cl / NLAYER, layer = cl % NLAYER;
    const int p0 = ptile * PIX_T, o0 = otile * OBS_T;
    const int tid = threadIdx.x;
    const int nbytes = 2 * n_pix;
    const int64_t nchars = 4 * (int64_t)((nbytes + 2) / 3);
    const uint16_t fill = layer == NLAYER - 1 ? (uint16_t)1 : (uint16_t)(int16_t)-9999;
    const unsigned flo = fill & 0xFF, fhi = fill >> 8;
    // the block's 128 payload offsets go to LDS once (rows past n_obs repeat the last one;
    // they are never written out).  ccdgpu_stage_chipmunk has checked that every payload lies
    // inside the text, so a quantum of the payload is always loadable; the 8-character load of
    // a pair whose second quantum is past the payload reads at most 4 bytes past it (the text
    // buffer carries 8 bytes of slack).  A missing layer loads text[0] and takes fill bytes.
    lut[tid] = (unsigned char)b64v(tid);
    if (tid < OBS_T) roff[tid] = offsets[((int64_t)chip * n_obs + min(o0 + tid, n_obs - 1)) * NLAYER + layer];
    __syncthreads();
    constexpr int ITEMS = OBS_T * PAIRS / 256, BATCH = 8;
    static_assert(ITEMS % BATCH == 0, "batches");
    const int pp = tid % PAIRS, r0 = tid / PAIRS;
    const int64_t c0 = 4 * ((int64_t)ptile * QUANTA + 2 * pp);  // character offset of the pair in a payload
    const bool in0 = c0 < nchars, in1 = c0 + 4 < nchars;
    // output rows: row pl starts at element pl * n_obs of the block's first row; h(pl) = 1 when
    // that element sits in the high half of a 32-bit word.  Observation r of row pl goes to tile
    // position r + h(pl), so that tile word l is output word l of the row (elements 2l - h and
    // 2l + 1 - h) and the write phase moves aligned words only.
    const bool is_qa = layer == NLAYER - 1;
    uint16_t *base = (is_qa ? qa + (int64_t)chip * n_pix * n_obs
                            : reinterpret_cast<uint16_t *>(spectra) + ((int64_t)chip * 7 + layer) * n_pix * n_obs) +
                     (int64_t)p0 * n_obs + o0;
    const int hb = (int)(((uintptr_t)base >> 1) & 1), odd = n_obs & 1;
    uint16_t *t0 = &tile[3 * pp][hb ^ (3 * pp & odd)];
    uint16_t *t1 = &tile[3 * pp + 1][hb ^ ((3 * pp + 1) & odd)];
    uint16_t *t2 = &tile[3 * pp + 2][hb ^ ((3 * pp + 2) & odd)];
    // fill bytes of a missing quantum, as the quantum's 24-bit word: bytes 6pp .. 6pp+5 of the
    // row alternate low / high bytes of the fill value, starting with a low byte
    const unsigned fw0 = (flo << 16) | (fhi << 8) | flo, fw1 = (fhi << 16) | (flo << 8) | fhi;
    unsigned acc01 = 0, acc23 = 0;  // OR of the 6-bit values: '=' or bad in places 0-1, bad in 2-3
#pragma unroll 1
    for (int i0 = 0; i0 < ITEMS; i0 += BATCH) {
        unsigned long long cw[BATCH];
        bool have[BATCH];
#pragma unroll
        for (int i = 0; i < BATCH; ++i) {
            const int64_t off = roff[r0 + (i0 + i) * (256 / PAIRS)];
            have[i] = off >= 0;
            __builtin_memcpy(&cw[i], text + (have[i] && in0 ? off + c0 : 0), 8);
        }
#pragma unroll
        for (int i = 0; i < BATCH; ++i) {
            const int r = r0 + (i0 + i) * (256 / PAIRS);
            unsigned w[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const bool ok = have[i] && (k ? in1 : in0);
                const unsigned c = ok ? (unsigned)(cw[i] >> (32 * k)) : 0x41414141u;  // "AAAA" decodes to 0
                const unsigned v0 = lut[c & 0xFF], v1 = lut[(c >> 8) & 0xFF], v2 = lut[(c >> 16) & 0xFF],
                               v3 = lut[c >> 24];
                acc01 |= v0 | v1;
                acc23 |= v2 | v3;
                const unsigned d = (v0 << 18) | (v1 << 12) | ((v2 & 63) << 6) | (v3 & 63);
                w[k] = ok ? d : (k ? fw1 : fw0);
            }
            t0[r] = (uint16_t)(((w[0] >> 16) & 0xFF) | (w[0] & 0xFF00));
            t1[r] = (uint16_t)((w[0] & 0xFF) | ((w[1] >> 8) & 0xFF00));
            t2[r] = (uint16_t)(((w[1] >> 8) & 0xFF) | ((w[1] & 0xFF) << 8));
        }
    }
    const bool bad = (acc01 & 0xC0) || (acc23 & 0x80);
    __syncthreads();
    const int cnt = min(OBS_T, n_obs - o0);
    // wave w writes pixel rows w, w + 4, ...: lane l stores tile word l as output word l (one
    // 32-bit store; the halves alone at the row's ends), lane 0 also element 127 when h = 1
    const int wv = tid >> 6, l = tid & 63;
    for (int pl = wv; pl < PIX_T && p0 + pl < n_pix; pl += 4) {
        uint16_t *row = base + (int64_t)pl * n_obs;
        const int h = hb ^ (pl & odd);
        const unsigned *tw = reinterpret_cast<const unsigned *>(tile[pl]);
        const unsigned wd = tw[l];
        const int e = 2 * l - h;
        if (e >= 0 && e + 1 < cnt) {
            *reinterpret_cast<unsigned *>(row + e) = wd;
        } else {
            if (e >= 0 && e < cnt) row[e] = (uint16_t)wd;
            if (e < 0 && cnt > 0) row[0] = (uint16_t)(wd >> 16);
        }
        if (h && l == 0 && cnt == OBS_T) row[OBS_T - 1] = (uint16_t)tw[OBS_T / 2];
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
    const int64_t n_tiles = (int64_t)grid.x * grid.y * grid.z;
    if (n_tiles > (int64_t)1 << 30) return -1;  // one 1-D grid of tiles (a 10^4-pixel chip has 1000)
    hipLaunchKernelGGL(ccd_unpack_b64, dim3((unsigned)((n_tiles + 63) / 64 * 64)), dim3(256), 0, (hipStream_t)stream,
                       text, text_bytes, offsets, n_obs, n_pix, spectra, qa, err, grid.x, grid.y, (unsigned)n_tiles);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
