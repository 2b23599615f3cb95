// ccd_kernels.hip -- MI355X (gfx950) CCDC change detection: the whole per-pixel pyccd state
// machine on device, one wavefront per pixel.
//
// What runs here (reference: ccd.detect called at ccdc/pyccd.py:168; pyccd module names in the
// comments are lcmap-pyccd 2018.03.12.dev-ncompare.b2, restated in oracle/ccd_ref.py):
//   ccdk_prep    -- per chip: stable argsort of the acquisition dates (ccd/__init__.py detect) and
//                   the Lasso design rows cos/sin(k w t) (models/lasso.coefficient_matrix), shared
//                   by every pixel of the chip.
//   ccd_detect   -- persistent kernel, one 64-lane wavefront per pixel pulled from a device work
//                   queue (active-pixel compaction: a wave that finishes a short pixel takes the
//                   next one, so divergent pixels never idle lanes of a long one):
//                   QA unpack/filter/dedup + compaction (qa.py), variogram (math_utils.py),
//                   ncompare peek (change.py), initialize + Tmask IRLS (procedures.py,
//                   models/tmask.py, models/robust_fit.py), stability (change.stable), lookback,
//                   lookforward with closest-DOY comparison RMSE, catch (change.py), 4/6/8-coef
//                   Lasso (models/lasso.py = sklearn 0.18 coordinate descent, here in Gram form),
//                   permanent-snow / insufficient-clear single fits (procedures.py).
//   ccdk_scatter -- segment pool -> CSR by pixel.
//
// Parallel mapping inside a wave (all control flow is wave-uniform; every reduction is a
// shuffle butterfly whose result is bit-identical in all lanes):
//   * observation loops: lane = observation (coalesced loads of the compacted period);
//   * Gram build: design rows staged in LDS, lane = Gram / X'y entry, sequential over rows;
//   * coordinate descent: lane = band (7 independent Lasso problems sharing one Gram);
//   * medians / 24-closest selection: counting selection with ballots (no sorting);
//   * peek windows: lane = peek observation.
// FP64 vector ALU throughout (tiny latency-bound solves; no MFMA shape exists).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stddef.h>
#include <stdint.h>

#include "ccd_device.h"

namespace {

constexpr int NB = CCD_NB;
constexpr int W = CCD_WAVE;
constexpr int RW = 16;  // doubles per staged design row: t c1 s1 c2 s2 c3 s3 _ y0..y6 _
constexpr int TR = 32;  // rows per LDS staging tile
constexpr int MAXW = CCDGPU_MAX_OBS / 32;
constexpr int PSTR = CCD_WAVE;  // band stride of the LDS peek-residual ring (a batch's 64 rows)
// Peek observations past the ring's 64 (an adaptive peek of 65 .. CCDGPU_MAX_PEEK, evaluated one
// step at a time) keep their residuals in the slot's global scratch, after its [8][n] block.
constexpr int POVF = CCDGPU_MAX_PEEK - PSTR;
static_assert(NB * POVF <= CCD_RING_OVF, "ring overflow fits the slot scratch tail");
#define CCD_NPHASE (CCD_NSTATS - 8)

// Global-memory pointers kept in the per-pixel state are typed address_space(1) so every access
// is a global_* instruction (a generic pointer would compile to flat_*, which also counts against
// lgkmcnt and makes every later LDS wait wait for the global load too).
#define GLOBAL_AS __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ GLOBAL_AS T *as_global(T *p) { return (GLOBAL_AS T *)p; }

struct __attribute__((aligned(16))) Lds {
    union {
        double row[TR][RW];       // staging tile (Gram, Tmask, speculative fits, variogram counts)
        double ring[NB * PSTR];   // peek residuals, band-major [band][PSTR] (never live with a tile)
    };
    union {
        struct {
            double G[8][8];
            double Q[8][8];  // Q[j][band] = Xc_j . yc_band
        };
        // lookforward between two fits (G / Q are rebuilt at every fit): per band, the inclusive
        // prefix over blocks of 46 bins of u = 4 t mod 1461 of the fit window's squared residuals
        // of the current models, in float, every term rounded up (fit_bounds)
        float blk[32][8];
    };
    double YY[8];
    double xm[8];
    double ym[8];
    double coef[NB][8];  // [band][0..6] = w, [band][7] = intercept
    double rmse[8];
    double vario[8];
    double comp[8];        // comparison rmse per band (change_magnitude)
    double med1[8], med2[8];
    double chg;            // change threshold of the pixel's (adaptive) peek (change.py)
    int sel[32];           // qs_ties: pending parts of the replayed quicksort
#ifdef CCD_PHASE_TIMERS
    unsigned long long tph[CCD_NPHASE];  // diagnostic build: per-phase cycle totals of this wave
#endif
    double S[98];          // raw Gram sums of the accumulated window (entry map: gram_entry)
    int y0[8];             // per-band value shift of the accumulated window
    union {                // Tmask (initialize) and the closest-DOY buckets (lookforward) never overlap
        uint32_t hist2[732];   // closest-DOY: fit-window counts per (4 t mod 1461) bin, 2 x u16 per word
        uint16_t hist16[1464]; // the same bins read one u16 at a time (ds_read_u16: no shift / mask)
        struct {
            uint32_t tflag[MAXW];  // Tmask outlier flags of the current window
            double tchol[5][5];    // Tmask: Cholesky factor of the unweighted normal matrix
            double tsys[2][5][6];  // paired Tmask: each band's weighted normal matrix | rhs
        };
        struct {                   // px_setup of a transport-encoded pixel (read in place):
            unsigned long long ekm[CCDGPU_MAX_OBS / 64];  // sent-band bits per 64 input observations
            uint16_t ekp[CCDGPU_MAX_OBS / 64];            // sent observations before each chunk
            uint16_t epal[16];                            // the chip's QA palette
        };
    };
    // launch statistics of this wave (kept here, not in registers: they are only touched per fit
    // and at the end): [0] band fits, [1] CD sweeps, [2] counted FP64 flops.  Last member: the
    // poison test mode fills everything before it.
    unsigned long long stat[4];
};
#ifndef CCD_PHASE_TIMERS
// <= 10 KB: 16 waves per CU fit in the 160 KB LDS (the 128-VGPR variant's register occupancy)
static_assert(sizeof(Lds) <= 10240, "per-wave LDS block within 160 KB / 16 waves");
#endif

// Launch arguments live in constant memory (uniform scalar loads from every device function),
// one slot per host context so that contexts sharing a device can run concurrently; the launch
// passes its slot as the kernel's only argument.  The per-wave LDS block is the dynamic shared
// segment (so every access is a ds_* instruction).
__constant__ CcdDetectArgs c_args[CCD_ARG_SLOTS];
// Every device function reads the launch arguments through ARGS(): the slot index is read from
// the kernel-argument segment and made opaque, which keeps the compiler from hoisting the
// (invariant) constant loads to the top of the persistent kernel, where they would stay live in
// SGPRs for its whole length and be spilled; re-reading them at the use is a scalar-cache hit.
__device__ __forceinline__ const CcdDetectArgs &ARGS() {
    int z = *(const int *)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(z));
    return c_args[z];
}
extern __shared__ __attribute__((aligned(16))) char ccd_smem[];
__device__ __forceinline__ Lds &LDS() { return *reinterpret_cast<Lds *>(ccd_smem); }
// statistics (Lds::stat): a wave-uniform amount added once (lane 0), a per-lane amount from the
// lanes that carry one
enum { ST_FITS = 0, ST_SWEEPS = 1, ST_FLOPS = 2 };
__device__ __forceinline__ int lane();
__device__ __forceinline__ void stat_uniform(int s, unsigned long long v) {
    if (lane() == 0) LDS().stat[s] += v;
}
__device__ __forceinline__ void stat_lane(int s, unsigned long long v) { atomicAdd(&LDS().stat[s], v); }
// Peek-residual ring, band-major [band][PSTR observations], aliased with the row staging tile
// (the Gram staging never overlaps a live ring): lane-contiguous, so lane-per-observation access
// is bank-conflict free.
__device__ __forceinline__ double *PRES(Lds *L) { return &L->ring[0]; }

// One compacted observation: the 7 band values and its sorted-date index in one 16-byte row, so a
// random gather (closest-DOY, peek) touches one cache line instead of eight.
struct __attribute__((aligned(16))) CRow {
    int16_t v[NB];
    uint16_t ci;
};
static_assert(sizeof(CRow) == 16, "CRow is one dwordx4");

struct Px {
    int n;      // observations (sorted)
    int m;      // current compacted period length (logical rows 0 .. m-1)
    // Gap buffer: logical row j lives at physical row j (j < gp) or j + gl (j >= gp).  Removing
    // observations (Tmask, outliers) compacts only the rows between the first removal and the
    // gap and widens the gap, instead of shifting the whole tail of the period.
    int gp, gl;
    int peek;   // (adaptive) peek size
    const GLOBAL_AS double *basis;
    const int64_t *sd;
    int32_t *cd;  // compacted dates
    CRow *cr;     // compacted rows: 7 band values + sorted index, one 16-byte load per observation
    // (the slot's double scratch -- Tmask columns, bucket records, ring overflow -- and its bucket
    // list are addressed from the launch arguments where used: PFS, PBK)
    int64_t gpix;
    int nseg;
    int acc_a, acc_b;  // window [acc_a, acc_b) whose raw sums L->S holds (acc_a < 0: none)
    int acc_t0;        // date shift of those sums
    int fit_k;         // coefficients of the models in L->coef when they describe [acc_a, acc_b)
    mutable int bad;             // source line of a tripped index guard (0 = none), per lane
};
// the pixel's processing mask: its output words, updated in place (Tmask / outlier removals)
__device__ __forceinline__ GLOBAL_AS unsigned *pmask(const Px &P) {
    return as_global(ARGS().mask_bits) + (size_t)P.gpix * ARGS().mask_words;
}
// peek residuals of observations 64 .. CCDGPU_MAX_PEEK-1, band-major [band][POVF], after the
// slot's [8][n] double scratch
// The wave's slot (its workgroup: one wave per workgroup) and the slot's double scratch and
// bucket list, recomputed at every use from the launch arguments (scalar loads) instead of two
// 64-bit pointers held in scalar registers for the whole kernel; none is read in the hottest loops
// (the period rows and dates, PCD / PCR, are: those stay in Px).
__device__ __forceinline__ size_t slot_no() {
    int s = (int)__builtin_amdgcn_workgroup_id_x();
    asm volatile("" : "+s"(s));
    return (size_t)s;
}
__device__ __forceinline__ GLOBAL_AS double *PFS(const Px &) {
    const CcdDetectArgs &A = ARGS();
    return as_global(A.s_f64 + slot_no() * CCD_SLOT_F64(A.n_obs_max));
}
__device__ __forceinline__ GLOBAL_AS uint16_t *PBK(const Px &) {
    const CcdDetectArgs &A = ARGS();
    return as_global(A.s_bk + slot_no() * (size_t)A.n_obs_max);
}
__device__ __forceinline__ GLOBAL_AS double *ring_ovf(const Px &P) { return PFS(P) + (size_t)8 * ARGS().n_obs_max; }

// The compacted period lives in the per-slot global scratch (round 2 measured it in LDS: one wave
// per SIMD, slower).
__device__ __forceinline__ int32_t *PCD(const Px &P) { return P.cd; }
__device__ __forceinline__ CRow *PCR(const Px &P) { return P.cr; }

// ------------------------------------------------------------------ diagnostic phase timers
// Built only into lib/libccdgpu_diag.so (-DCCD_PHASE_TIMERS): s_memtime cycle totals per phase,
// summed over waves into stats[8 + phase].  Phases: 0 pixel total, 1 QA/filter/compaction,
// 2 variogram + peek, 3 Tmask, 4 Lasso Gram, 5 Lasso CD, 6 Lasso rmse, 7 lookforward batch
// (13 ring residuals + 14 per-lane closest-DOY rmse + 15 magnitudes + decisions), 8 single-step
// peek evaluation, 9 outlier compaction, 10 stability, 11 medians + emit, 12 closest-DOY bucket
// build; event counts: 16 batched steps executed, 17 batches, 18 single-step peek evaluations,
// 19 fits; 20 speculative early fits.  Per-lane phases (14, 15) are summed in lane 0 only.
#ifdef CCD_PHASE_TIMERS
// s_memtime returns through lgkmcnt out of order with LDS traffic: drain every counter around
// each stamp so no LDS result can be consumed early.
// (CCD_PHASE_TIMERS_RAW: no draining -- outstanding memory latency is then charged to the phase
// that waits for it; closer to the undisturbed schedule of an issue-bound kernel)
__device__ __forceinline__ unsigned long long ph_stamp() {
#ifndef CCD_PHASE_TIMERS_RAW
    __builtin_amdgcn_s_waitcnt(0);
#endif
    const unsigned long long t = __builtin_amdgcn_s_memtime();
#ifndef CCD_PHASE_TIMERS_RAW
    __builtin_amdgcn_s_waitcnt(0);
#endif
    return t;
}
#define PH_BEGIN(id) const unsigned long long _ph_##id = ph_stamp();
// (totals live in LDS, not in the pixel state, so the diagnostic build keeps the product's
// register allocation as far as possible; lane 0 accumulates)
#define PH_END(P, id, slot) { const unsigned long long _d = ph_stamp() - _ph_##id; if (lane() == 0) LDS().tph[slot] += _d; }
#define PH_COUNT(P, slot, v) { if (lane() == 0) LDS().tph[slot] += (unsigned long long)(v); }
#else
#define PH_COUNT(P, slot, v)
#define PH_BEGIN(id)
#define PH_END(P, id, slot)
#endif

// ------------------------------------------------------------------ index guards
// Every read of the compacted period and of the slot scratch goes through these: an index past
// the end is clamped into [0, lim) (one v_min_u32), so a logic error can never fault the GPU.
// The checking build (-DCCD_GUARD_LINES, lib/libccdgpu_guard.so, run over the golden vectors by
// tests/test_gpu_batches.py) also keeps the offending source line in a register (P.bad); at the
// end of the pixel the wave publishes it to counters[4], which the host turns into CCDGPU_EHIP
// naming the line.  (The line bookkeeping costs the product build ~2 %: a compare, two selects
// and a live register per access.)
__device__ __forceinline__ int gidx(const Px &P, int j, int lim, int line) {
#if defined(CCD_NOGUARD)  // measurement build only: what the clamp costs
    return j;
#elif defined(CCD_GUARD_LINES)
    const bool ok = (unsigned)j < (unsigned)lim;
    P.bad = ok ? P.bad : line;
    return ok ? j : 0;
#else
    (void)P;
    (void)line;
    const unsigned u = (unsigned)j, c = (unsigned)(lim > 0 ? lim - 1 : 0);  // (lim: wave-uniform, SALU)
    return (int)(u < c ? u : c);
#endif
}
// physical row of logical row j (gap buffer)
__device__ __forceinline__ int ph(const Px &P, int j) {
    return j + (j >= P.gp ? P.gl : 0);
}
// guarded logical row -> physical row
__device__ __forceinline__ int prow(const Px &P, int j, int line) { return ph(P, gidx(P, j, P.m, line)); }
__device__ __forceinline__ int32_t cdr(const Px &P, int j, int line) { return PCD(P)[prow(P, j, line)]; }
__device__ __forceinline__ int cir(const Px &P, int j, int line) {
    const int c = PCR(P)[prow(P, j, line)].ci;
    return gidx(P, c, P.n, line);
}
__device__ __forceinline__ int16_t cvr(const Px &P, int b, int j, int line) {
    return PCR(P)[prow(P, j, line)].v[b];
}
__device__ __forceinline__ CRow crow(const Px &P, int j, int line) {
    CRow r = PCR(P)[prow(P, j, line)];
    r.ci = (uint16_t)gidx(P, r.ci, P.n, line);
    return r;
}
// the 16-byte row of logical row j as one vector load
__device__ __forceinline__ uint4 crow4(const Px &P, int j, int line) {
    return reinterpret_cast<const uint4 *>(PCR(P))[prow(P, j, line)];
}
#define CROW4(P, j) crow4(P, (j), __LINE__)
#define CROW(P, j) crow(P, (j), __LINE__)
#define CDR(P, j) cdr(P, (j), __LINE__)
// the date of a row whose index is wave-uniform, as a scalar (see uni)
#define CDRU(P, j) uni(cdr(P, (j), __LINE__))
#define CIR(P, j) cir(P, (j), __LINE__)
#define CVR(P, b, j) cvr(P, (b), (j), __LINE__)

// ------------------------------------------------------------------ wave primitives
// Every primitive below that reads other lanes' registers (DPP, readlane, bpermute) is only
// correct with all 64 lanes enabled: a disabled lane's register holds whatever the register
// allocator left there.  (Ballots and mbcnt are lane-local -- a v_cmp writes 0 for a disabled
// lane -- and need no full EXEC.)  All control flow around them is wave-uniform by construction;
// the checking build asserts it: each primitive takes its call site's line (XL) and, when EXEC
// is not all ones, records 100000 + line in counters[4] (the first; CCDGPU_EHIP names it) and
// sets bit line / 2 of the bitmap in stats[8 ..] (all of them; the host lists them).
#ifdef CCD_GUARD_LINES
__device__ __forceinline__ void exec_full(int line) {
    if (__builtin_amdgcn_read_exec() != ~0ull) {
        atomicCAS(&ARGS().counters[4], 0ull, 100000ull + (unsigned long long)line);
        const int bit = line >> 1;
        if (bit < 64 * (CCD_NSTATS - 8)) atomicOr(&ARGS().stats[8 + (bit >> 6)], 1ull << (bit & 63));
    }
}
#define XL , int xline_ = __builtin_LINE()
#define EXEC_FULL() exec_full(xline_)
#else
#define XL
#define EXEC_FULL()
#endif
// Opaque like ARGS(): lane-derived masks and index maps are recomputed where they are used
// instead of being hoisted to the kernel entry and kept live (spilled) for the whole kernel.
__device__ __forceinline__ int lane() {
    int l = (int)__lane_id();
    asm volatile("" : "+v"(l));
    return l;
}
__device__ __forceinline__ unsigned long long bal(bool p) { return __ballot(p); }
__device__ __forceinline__ int popc(unsigned long long x) { return __popcll(x); }
// lane shuffles (ds_bpermute): the source lane must be enabled
template <class T>
__device__ __forceinline__ T shf(T v, int src XL) {
    EXEC_FULL();
    return __shfl(v, src);
}
template <class T>
__device__ __forceinline__ T shfx(T v, int m XL) {
    EXEC_FULL();
    return __shfl_xor(v, m);
}

__device__ __forceinline__ int below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0));
}
// DPP lane moves on a double (two 32-bit halves).  Controls: 0xB1 quad_perm [1,0,3,2] (xor 1),
// 0x4E quad_perm [2,3,0,1] (xor 2), 0x141 row_half_mirror (lane i <-> 7-i in each 8),
// 0x140 row_mirror (lane i <-> 15-i in each 16).
// (Every lane's source is valid for the permutations used with dpp<>, so bound_ctrl only saves
// the compiler a zero "old" operand.)
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rdlane(double v, int l XL) {
    EXEC_FULL();
    return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                            __builtin_amdgcn_readlane(__double2loint(v), l));
}
// Inclusive prefix sum over the 64 lanes in DPP only (no LDS round trip): Hillis-Steele with
// row_shr 1/2/4/8 inside each row of 16, then row_bcast:15 (rows 1, 3) and row_bcast:31
// (rows 2, 3) carry the row totals across.
__device__ __forceinline__ int wscan_incl(int v XL) {
    EXEC_FULL();
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);
    // row_bcast with a full row mask, rows selected by lane id: a partial row_mask leaves the
    // disabled rows' destination unwritten, and the compiler's choice of "old" register for
    // them is not reliably zero (observed wrong scans on gfx950).
    const int row = (int)__lane_id() >> 4;
    const int t15 = __builtin_amdgcn_update_dpp(0, v, 0x142, 0xF, 0xF, false);
    v += (row & 1) ? t15 : 0;
    const int t31 = __builtin_amdgcn_update_dpp(0, v, 0x143, 0xF, 0xF, false);
    v += (row & 2) ? t31 : 0;
    return v;
}
// Inclusive prefix sum of a float over each 32-lane half of the wave, in DPP only (wscan_incl
// without the row_bcast:31 step that carries the first half into the second).
__device__ __forceinline__ float fscan32(float v XL) {
    EXEC_FULL();
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x111, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x112, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x114, 0xF, 0xF, false));
    v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x118, 0xF, 0xF, false));
    const int row = (int)__lane_id() >> 4;
    const float t15 = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x142, 0xF, 0xF, false));
    v += (row & 1) ? t15 : 0.0f;
    return v;
}
// a wave-uniform value (every lane holds the same) as a scalar: the compiler's divergence
// analysis cannot see through lane shuffles and DPP reductions, and a value it takes for
// divergent lives in a VGPR (two for a pointer) -- and so does everything computed from it
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ unsigned long long uni(unsigned long long v) {
    return ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
           (unsigned)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ double unid(double v) {
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
}
// value of v in a (wave-uniform) lane, as a scalar
__device__ __forceinline__ int rdl(int v, int src XL) {
    EXEC_FULL();
    return __builtin_amdgcn_readlane(v, src);
}

// wave-wide sum, identical (wave-uniform) result in every lane
__device__ __forceinline__ double wsum(double v XL) {
    EXEC_FULL();
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    return (rdlane(v, 0) + rdlane(v, 16)) + (rdlane(v, 32) + rdlane(v, 48));
}
// wsync: order LDS traffic between the lanes of this (single-wave) workgroup -- the LDS
// executes a wave's ds_* operations in order, so only compiler motion must be stopped.
// gsync: hand-off of GLOBAL scratch written by one lane and read by another (compaction,
// Tmask scratch): workgroup release/acquire (vmcnt drain) + barrier.
__device__ __forceinline__ void wsync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}
__device__ __forceinline__ void gsync() { __syncthreads(); }
// psync: hand-off of compacted-period data written by one lane and read by another
__device__ __forceinline__ void psync() { gsync(); }

#define cvalf(P, b, j) ((double)CVR(P, b, j))

// k-th smallest (0-based) of integer values in [lo, hi] produced by gen(i, &v) (returns valid).
template <class F>
__device__ __forceinline__ int kth_int(F gen, int N, int k, int lo, int hi) {
    const int l = lane();
    while (lo < hi) {
        const int mid = lo + ((hi - lo) >> 1);
        int c = 0;
        for (int base = 0; base < N; base += W) {
            const int i = base + l;
            int v = 0;
            bool ok = false;
            if (i < N) ok = gen(i, v);
            c += popc(bal(ok && v <= mid));
        }
        if (c >= k + 1) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

template <class F>
__device__ __forceinline__ double median_int(F gen, int N, int cnt, int lo, int hi) {
    if (cnt <= 0) return __builtin_nan("");
    if (cnt & 1) return (double)kth_int(gen, N, cnt / 2, lo, hi);
    const int a = kth_int(gen, N, cnt / 2 - 1, lo, hi);
    const int b = kth_int(gen, N, cnt / 2, lo, hi);
    return ((double)a + (double)b) / 2.0;
}

// k-th smallest of non-negative doubles vals[0..N) (bit patterns are monotone for x >= 0).
__device__ __forceinline__ double kth_nonneg(const GLOBAL_AS double *vals, int N, int k) {
    const int l = lane();
    unsigned long long lo = 0ull, hi = 0x7FF0000000000000ull;
    while (lo < hi) {
        const unsigned long long mid = lo + ((hi - lo) >> 1);
        int c = 0;
        for (int base = 0; base < N; base += W) {
            const int i = base + l;
            bool ok = false;
            if (i < N) ok = (unsigned long long)__double_as_longlong(vals[i]) <= mid;
            c += popc(bal(ok));
        }
        if (c >= k + 1) hi = mid;
        else lo = mid + 1;
    }
    return __longlong_as_double((long long)lo);
}

// ascending bitonic sort of one double per lane across the 64-lane wave (21 exchange stages)
__device__ __forceinline__ double bitonic64(double v XL) {
    EXEC_FULL();
    const int l = lane();
#pragma unroll
    for (int k = 2; k <= W; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const double o = shfx(v, j);
            const bool up = (l & k) == 0;
            const bool lower = (l & j) == 0;
            const double mn = o < v ? o : v;
            const double mx = o < v ? v : o;
            v = (lower == up) ? mn : mx;
        }
    }
    return v;
}

// two independent ascending bitonic sorts, lanes 0..31 and 32..63 (the 64-lane network without
// its last merge, the k = 32 stage ascending in both halves): the same sorted sequence per half as
// bitonic64 gives for 32 values padded with +inf
__device__ __forceinline__ double bitonic32x2(double v XL) {
    EXEC_FULL();
    const int l = lane();
#pragma unroll
    for (int k = 2; k <= 32; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const double o = shfx(v, j);
            const bool up = k == 32 || (l & k) == 0;
            const bool lower = (l & j) == 0;
            const double mn = o < v ? o : v;
            const double mx = o < v ? v : o;
            v = (lower == up) ? mn : mx;
        }
    }
    return v;
}

__device__ __forceinline__ int qabitval(const ccdgpu_params &p, unsigned v) {
#define BIT(o) ((v >> (o)) & 1u)
    if (BIT(p.qa_fill)) return p.qa_fill;
    if (BIT(p.qa_cloud)) return p.qa_cloud;
    if (BIT(p.qa_shadow)) return p.qa_shadow;
    if (BIT(p.qa_snow)) return p.qa_snow;
    if (BIT(p.qa_water)) return p.qa_water;
    if (BIT(p.qa_clear)) return p.qa_clear;
    if (BIT(p.qa_cirrus1) && BIT(p.qa_cirrus2)) return p.qa_clear;
    if (BIT(p.qa_occlusion)) return p.qa_clear;
    return -1;
#undef BIT
}

// ------------------------------------------------------------------ compaction
// Drop the observations j in [lo, hi) for which drop(j) is true (logical indices).  Gap buffer:
// only the logical rows of [min(lo, gp), max(hi, gp)) are rewritten -- the kept ones packed
// down from physical row min(lo, gp) in one ascending pass -- and the gap moves to the end of
// that range, widened by the number dropped; rows past the range keep their physical place.
// The dropped rows leave the processing mask.  Removals happen at the front of the growing
// window, so the range is a few dozen rows instead of the whole tail of the period.
template <class F>
__device__ __forceinline__ int compact_drop(Px &P, int lo, int hi, F drop) {
    const int l = lane();
    if (lo < P.acc_b) P.acc_a = -1;  // rows of the accumulated Gram window may move
    hi = hi < P.m ? hi : P.m;
    if (P.gl == 0) P.gp = lo;  // an empty gap moves for free: start it at the first removal
    const int a = lo < P.gp ? lo : P.gp;
    const int e = hi > P.gp ? hi : (P.gp < P.m ? P.gp : P.m);
    PH_COUNT(P, 31, e - a)
    int out = a;
    // four 64-row chunks per round: all their loads go out before the first store (a row's
    // store lands at or below its own physical position, and physical positions grow with the
    // logical index, so a store never overwrites a row still to be read)
    constexpr int U = 4;
    for (int base = a; base < e; base += U * W) {
        int32_t d[U];
        uint4 r[U];  // the 16-byte row as one vector (ci = high half of .w)
        bool in[U], dr[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int j = base + u * W + l;
            in[u] = j < e;
            d[u] = 0;
            r[u] = uint4{0u, 0u, 0u, 0u};
            dr[u] = false;
            if (in[u]) {
                const int pj = ph(P, j);
                d[u] = PCD(P)[pj];
                r[u] = reinterpret_cast<const uint4 *>(PCR(P))[pj];
                dr[u] = j >= lo && j < hi && drop(j);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const unsigned long long keep = bal(in[u] && !dr[u]);
            const unsigned ci = r[u].w >> 16;
            if (in[u] && dr[u])
                __hip_atomic_fetch_and(pmask(P) + (ci >> 5), ~(1u << (ci & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (in[u] && !dr[u]) {
                const int pos = gidx(P, out + below(keep), P.n, __LINE__);
                PCD(P)[pos] = d[u];
                reinterpret_cast<uint4 *>(PCR(P))[pos] = r[u];
            }
            out += popc(keep);
        }
    }
    const int removed = (e - a) - (out - a);
    P.m -= removed;
    P.gl += removed;
    P.gp = out;
    psync();
    return P.m;
}

// ------------------------------------------------------------------ Lasso (models/lasso.py)
// gram_accumulate stages period rows into the LDS tile as
// [t - t0, cos wt, sin wt, cos 2wt, sin 2wt, cos 3wt, sin 3wt, 1, y0 - s0 .. y6 - s6, 0]
// (t0, s = the accumulated window's integer shifts: exact, and they keep the raw sums small).
// Raw-sum entry e of the accumulated Gram: products of staged columns (ca, cb).  0..27 design
// x design (upper triangle), 28..76 design x band, 77..83 band x band, 84..90 design sums,
// 91..97 band sums; e >= 98 maps to the zero column.
__device__ __forceinline__ void gram_entry(int e, int &ca, int &cb) {
    if (e < 28) {
        int j = 0;
        while (e >= 7 - j) { e -= 7 - j; ++j; }
        ca = j;
        cb = j + e;
    } else if (e < 77) {
        e -= 28;
        ca = e / 7;
        cb = 8 + e % 7;
    } else if (e < 84) {
        ca = cb = 8 + (e - 77);
    } else if (e < 91) {
        ca = e - 84;
        cb = 7;
    } else if (e < 98) {
        ca = 8 + (e - 91);
        cb = 7;
    } else {
        ca = cb = 15;
    }
}

// Make L->S the raw sums of window [a, b): extend the accumulated window when it is a prefix of
// [a, b) (the lookforward case: the window only grows at its end), otherwise start over with
// the date / value shifts of observation a.  Lane = entry (two per lane), sequential over rows.
__device__ __forceinline__ void gram_accumulate(Px &P, int a, int b) {
    Lds *L = &LDS();
    const int l = lane();
    int from = P.acc_b;
    if (!(P.acc_a == a && P.acc_b <= b)) {
        P.acc_a = a;
        P.acc_t0 = CDRU(P, a);
        if (l < NB) L->y0[l] = (int)CVR(P, l, a);
        L->S[l] = 0.0;
        if (l + W < 98) L->S[l + W] = 0.0;
        wsync();
        from = a;
    }
    P.acc_b = b;
    if (from >= b) return;
    int ca0, cb0, ca1, cb1;
    gram_entry(l, ca0, cb0);
    gram_entry(l + W, ca1, cb1);
    double s0 = L->S[l], s1 = l + W < 98 ? L->S[l + W] : 0.0;
    // 64 rows per round: every lane loads one row (period row + design row) up front, then the
    // two 32-row halves are staged through the LDS tile in turn (one memory round trip per 64)
    for (int t0 = from; t0 < b; t0 += 2 * TR) {
        const int cnt = b - t0 < 2 * TR ? b - t0 : 2 * TR;
        CRow cw{};
        double x[7];
#pragma unroll
        for (int c = 0; c < 7; ++c) x[c] = 0.0;
        if (l < cnt) {
            cw = CROW(P, t0 + l);
            const GLOBAL_AS double *bs = P.basis + (size_t)cw.ci * CCD_BASIS_STRIDE;
#pragma unroll
            for (int c = 0; c < 7; ++c) x[c] = bs[c];
        }
        for (int h = 0; h < 2; ++h) {
            const int hc = cnt - h * TR < TR ? cnt - h * TR : TR;
            if (hc <= 0) break;
            const int hc4 = (hc + 3) & ~3;  // rows hc .. hc4 - 1 are staged as zeros (add nothing)
            if (l >= h * TR && l < h * TR + hc4) {
                const bool rv = l < h * TR + hc;
                double *r = L->row[l - h * TR];
                r[0] = rv ? x[0] - (double)P.acc_t0 : 0.0;
#pragma unroll
                for (int c = 1; c < 7; ++c) r[c] = rv ? x[c] : 0.0;
                r[7] = rv ? 1.0 : 0.0;
#pragma unroll
                for (int bb = 0; bb < NB; ++bb) r[8 + bb] = rv ? (double)((int)cw.v[bb] - L->y0[bb]) : 0.0;
                r[15] = 0.0;
            }
            wsync();
            // four rows per round, all sixteen LDS reads issued before the first FMA (the sums
            // stay sequential over the rows)
            for (int r = 0; r < hc4; r += 4) {
                double a0[4], b0[4], a1[4], b1[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    a0[u] = L->row[r + u][ca0];
                    b0[u] = L->row[r + u][cb0];
                    a1[u] = L->row[r + u][ca1];
                    b1[u] = L->row[r + u][cb1];
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    s0 += a0[u] * b0[u];
                    s1 += a1[u] * b1[u];
                }
            }
            wsync();
        }
    }
    L->S[l] = s0;
    if (l + W < 98) L->S[l + W] = s1;
    wsync();
}

// Centred Gram (sklearn's centred design / targets) and the means of the raw columns from the
// raw sums of [acc_a, acc_b): entry = S_ab - S_a S_b / n; means = (shifted sum + n shift) / n
// (exact integer shifts, so the means equal the plain column means).
__device__ __forceinline__ void gram_finalize(const Px &P, int nw) {
    Lds *L = &LDS();
    const int l = lane();
    const double n = (double)nw;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int e = l + h * W;
        int ca, cb;
        gram_entry(e, ca, cb);
        if (e < 98) {
            const double se = L->S[e];
            if (e < 28) {
                const double v = se - L->S[84 + ca] * (L->S[84 + cb] / n);
                L->G[ca][cb] = v;
                L->G[cb][ca] = v;
            } else if (e < 77) {
                L->Q[ca][cb - 8] = se - L->S[84 + ca] * (L->S[91 + cb - 8] / n);
            } else if (e < 84) {
                L->YY[ca - 8] = se - L->S[91 + ca - 8] * (L->S[91 + ca - 8] / n);
            } else if (e < 91) {
                L->xm[ca] = (se + (ca == 0 ? n * (double)P.acc_t0 : 0.0)) / n;
            } else {
                L->ym[ca - 8] = (se + n * (double)L->y0[ca - 8]) / n;
            }
        }
    }
    wsync();
}

// 8-lane group reductions (a band's lanes 8b .. 8b+7); results identical in all 8 lanes.
__device__ __forceinline__ double gsum8(double v XL) {
    EXEC_FULL();
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    return v + dpp<0x141>(v);
}
// one v_max_f64 per level: every operand here is a non-NaN magnitude, so the sNaN quieting fmax
// would add (a canonicalising max of each DPP operand) is left out
__device__ __forceinline__ double vmax(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double gmax8(double v XL) {
    EXEC_FULL();
    v = vmax(v, dpp<0xB1>(v));
    v = vmax(v, dpp<0x4E>(v));
    return vmax(v, dpp<0x141>(v));
}

// float max over a band's 8 lanes, one DPP-modified v_max_f32 per level (a 64-bit max needs two
// lane moves and a max per level); s_nop 1: a DPP source read 2 wait states after its VALU write
__device__ __forceinline__ float gmax8f(float v XL) {
    EXEC_FULL();
    float r;
    asm("s_nop 1\n\t"
        "v_max_f32_dpp %0, %1, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 1\n\t"
        "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf"
        : "=&v"(r) : "v"(v));
    return r;
}

// gmax8f of two values at once: the two reductions' DPP maxima interleaved, so each level's
// second operation supplies one of the two wait states the next level's DPP read needs
__device__ __forceinline__ void gmax8f2(float u, float v, float &ru, float &rv XL) {
    EXEC_FULL();
    asm("s_nop 1\n\t"
        "v_max_f32_dpp %0, %2, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %1, %3, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_max_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %1, %1, %1 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf\n\t"
        "s_nop 0\n\t"
        "v_max_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf\n\t"
        "v_max_f32_dpp %1, %1, %1 row_half_mirror row_mask:0xf bank_mask:0xf"
        : "=&v"(ru), "=&v"(rv) : "v"(u), "v"(v));
}

// One coordinate of the cyclic sweep (coordinate J of every band group).  Lane (b, k) holds
// h_k = g_k + G_kk w_k, where g_k = q_k - sum_m G_km w_m is the correlation X_k . R of sklearn's
// residual form: h_J is sklearn's tmp = X_J . (R + w_J X_J) for coordinate J as it stands, so the
// update reads it directly.  A change d of w_J moves h_k by -G_kJ d for k != J and leaves h_J as
// it is (the G_JJ terms cancel), so the broadcast column carries a zero on its diagonal.
// Per coordinate: soft threshold (3 VALU), d (1 fused), lane J's w (1, exec-masked), 2 DPP FMAs.
// HALF: 0 = both band groups of each 16-lane row take the broadcast; 1 / 2 = only the even (lanes
// 0-7 of the row) / odd (lanes 8-15) groups are live, so the other group's FMA (which would add
// zeros to a finished group) is left out.
template <int J, int HALF = 0>
__device__ __forceinline__ void cd_coord(unsigned long long mJ /* live lanes of coordinate J */,
                                         double alpha, double rgkk, double ngcolJ, double &h, double &w XL) {
    EXEC_FULL();
    // sklearn: fsign(tmp) * fmax(|tmp| - alpha, 0) / norm (a signed zero below alpha, as there)
    const double s = copysign(fmax(fabs(h) - alpha, 0.0), h);
    // d = w_new - w_old in one rounding (read from lane J only; a finished group's column is
    // zero, so d needs no gating)
    const double d = fma(s, rgkk, -w);
    // w_J = S(tmp) / G_JJ as a multiply, in the live lanes of coordinate J only: one VALU under
    // an exec mask instead of a 64-bit select (two v_cndmask).  s_and_saveexec keeps any lane the
    // caller had disabled disabled.
    unsigned long long sv;
    asm volatile("s_and_saveexec_b64 %[sv], %[m]\n\t"
                 "v_mul_f64 %[w], %[s], %[r]\n\t"
                 "s_mov_b64 exec, %[sv]"
                 : [w] "+v"(w), [sv] "=&s"(sv)
                 : [m] "s"(mJ), [s] "v"(s), [r] "v"(rgkk));
    // h += (-G_kJ) * d_J: two 64-bit DPP FMAs, row_newbcast (lane J of the 16-lane row to the
    // row) with the bank mask of the band group that owns that lane -- lanes 0-7 of each row take
    // lane J, lanes 8-15 lane 8 + J.  s_nop 1 before each: a DPP FMA reads its operands (the
    // accumulator included) 2 wait states behind a VALU write of them -- back to back, the second
    // FMA loses the first one's result (tools/probe/dpp64.hip, measured on gfx950).
    if (HALF == 0)
        asm volatile("s_nop 1\n\t"
                     "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0x3\n\t"
                     "s_nop 1\n\t"
                     "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%4 row_mask:0xf bank_mask:0xc"
                     : "+v"(h) : "v"(d), "v"(ngcolJ), "i"(J), "i"(J + 8));
    else if (HALF == 1)
        asm volatile("s_nop 1\n\t"
                     "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0x3"
                     : "+v"(h) : "v"(d), "v"(ngcolJ), "i"(J));
    else
        asm volatile("s_nop 1\n\t"
                     "v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xc"
                     : "+v"(h) : "v"(d), "v"(ngcolJ), "i"(J + 8));
}

// one cyclic sweep over the PC active coordinates (pc at run time when PC = 0)
template <int PC, int HALF>
__device__ __forceinline__ void cd_coords(int pc, unsigned long long lm, double alpha, double rgkk,
                                          const double (&gcol)[7], double &h, double &w XL) {
    constexpr unsigned long long COL = 0x0001010101010101ull;  // coordinate J's lanes (b, J): one bit per group
    cd_coord<0, HALF>(lm & COL, alpha, rgkk, gcol[0], h, w);
    if (pc > 1) cd_coord<1, HALF>(lm & (COL << 1), alpha, rgkk, gcol[1], h, w);
    if (pc > 2) cd_coord<2, HALF>(lm & (COL << 2), alpha, rgkk, gcol[2], h, w);
    if (pc > 3) cd_coord<3, HALF>(lm & (COL << 3), alpha, rgkk, gcol[3], h, w);
    if (pc > 4) cd_coord<4, HALF>(lm & (COL << 4), alpha, rgkk, gcol[4], h, w);
    if (pc > 5) cd_coord<5, HALF>(lm & (COL << 5), alpha, rgkk, gcol[5], h, w);
    if (pc > 6) cd_coord<6, HALF>(lm & (COL << 6), alpha, rgkk, gcol[6], h, w);
}

// sklearn 0.18 enet_coordinate_descent (beta = 0, cyclic, duality-gap stop) in gradient form,
// 7 bands at once: lane = band * 8 + coordinate.  Lane (b, k) holds Gram column k, g_k and w_k;
// a coordinate update is broadcast to its band group by DPP and folded into every g (no
// per-coordinate reduction).  Writes L->coef[b][0..6]; returns the sweep count (every lane of
// the band's group).
template <int PC>  // active columns as a constant (3, 5, 7: 4, 6, 8 coefficients), 0 = runtime pc
__device__ __forceinline__ int cd_sweep(Lds *L, int pc_rt, double alpha, int max_iter, double tol) {
    const int pc = PC ? PC : pc_rt;
    const int l = lane();
    const int b = l >> 3, k = l & 7;
    const bool act = b < NB && k < pc;
    double gcol[7];
    // negated (h += gcol * d), zero on the diagonal (a coordinate's own h does not move)
#pragma unroll
    for (int j = 0; j < 7; ++j) gcol[j] = (act && j < pc && j != k) ? -L->G[j][k] : 0.0;
    const double gkk = act ? L->G[k][k] : 0.0;
    const double rgkk = gkk != 0.0 ? 1.0 / gkk : 0.0;  // w_k = S(tmp, alpha) / G_kk as a multiply
    const double q = act ? L->Q[k][b] : 0.0;
    const double yy = b < NB ? L->YY[b] : 0.0;
    const double tol_s = tol * yy;
    const double tol_m = -0x1p-45 * tol;  // exact (a power of two)
    const float tol_f = (float)tol;
    const bool can = act && gkk != 0.0;  // sklearn skips zero-norm columns
    double w = 0.0, h = q;  // h = g + G_kk w = q at w = 0
    // loop control in wave-uniform lane masks (SALU): finished groups (all 8 lanes of a band
    // whose duality gap met tol, and lanes 56-63), and the lanes sklearn updates at all
    unsigned long long dmask = bal(b >= NB);
    const unsigned long long cmask = bal(can);
    int sweeps = max_iter;
#ifdef CCD_CD_CYCLES
    // diagnostic: Brent cycle detection on each band group's sweep state (w, h of its 8 lanes,
    // bitwise); det_it / det_per = sweep at which the group's state first repeated, and the period
    long long ws = __double_as_longlong(w), hs = __double_as_longlong(h);
    int power = 1, lam = 0, det_it = 0, det_per = 0;
    unsigned long long cyc = 0ull;
#endif
    for (int it = 0; it < max_iter; ++it) {
        if (dmask == ~0ull) break;
#ifdef CCD_CD_CYCLES
        if (it > 0) {
            ++lam;
            const unsigned long long eq = bal(__double_as_longlong(w) == ws && __double_as_longlong(h) == hs);
            unsigned long long newg = 0ull;
            for (int g = 0; g < NB; ++g)
                if (((eq >> (8 * g)) & 0xFFull) == 0xFFull && !((cyc >> (8 * g)) & 1ull) && !((dmask >> (8 * g)) & 1ull))
                    newg |= 0xFFull << (8 * g);
            if ((newg >> l) & 1ull) {
                det_it = it;
                det_per = lam;
            }
            cyc |= newg;
            if (power == lam) {
                ws = __double_as_longlong(w);
                hs = __double_as_longlong(h);
                power *= 2;
                lam = 0;
            }
        }
#endif
        const unsigned long long lm = cmask & ~dmask;  // live lanes (all coordinates)
        const double w0 = w;
        // (one sweep body for every live-group pattern: a second body for live groups all in one
        // half of their rows -- one broadcast FMA per coordinate, 36 % of C3 sweeps -- measured 5 %
        // slower, profiles/r06/ab/half_row_skip_*)
        cd_coords<PC, 0>(pc, lm, alpha, rgkk, gcol, h, w);
        // every coordinate moves once per sweep: d_w_ii = |w_new - w_old| of the lane's own one.
        // sklearn's d_w_max / w_max < tol (w_max = 0 is the check's own first clause), decided
        // first on the float32 roundings of the two maxima (max commutes with the monotone
        // rounding, so they are fl32(d_w_max) and fl32(w_max), each within 2^-24 relative): with
        // w_max in [2^-100, 2^100], D < fl(tol) W (1 - 2^-16) implies d/w < tol (1 - 2^-17), so
        // fl64(d/w) < tol, and D > fl(tol) W (1 + 2^-16) implies fl64(d/w) >= tol.  Groups whose
        // ratio falls in that band (or whose w_max is 0 or out of range) take the exact test.
        // The bound needs tw = fl(tol) W and tw (1 -+ 2^-16) normal floats: with a tolerance
        // below ~1e-8 (or flushed denormals) tw can be subnormal, so tw < 2^-125 also goes exact.
        unsigned long long rl, wz = 0ull;  // groups with d_w_max / w_max < tol, with w_max = 0
        {
            float D, Wf;  // w stays 0 in lanes outside the model
            gmax8f2((float)fabs(w - w0), (float)fabs(w), D, Wf);
            const float tw = tol_f * Wf;
            // (one ballot per comparison: each v_cmp writes its lane mask straight to SGPRs)
            const unsigned long long wokm = bal(Wf >= 0x1p-100f) & bal(Wf <= 0x1p100f) & bal(tw >= 0x1p-125f);
            const unsigned long long ltm = wokm & bal(D < tw * (1.0f - 0x1p-16f));
            const unsigned long long gem = wokm & bal(D > tw * (1.0f + 0x1p-16f));
            rl = ltm;
            const unsigned long long ambm = ~dmask & ~ltm & ~gem;
#ifdef CCD_CD_CHKSTAT
            PH_COUNT(P, 27, ambm ? 1 : 0)
#endif
            if (ambm) {
                const double d_w_max = gmax8(fabs(w - w0));
                const double w_max = gmax8(fabs(w));
                // the sign of the fused d_w_max - tol w_max (one rounding of the exact value)
                // decides it outside a sliver of relative width 2^-45 around tol, where the
                // quotient itself is taken: r >= 0 -> fl(d/w) >= tol; r < -2^-45 tol w -> fl(d/w) < tol.
                const double r = fma(-tol, w_max, d_w_max);
                bool ex = r < tol_m * w_max;
                const bool amb = !(r >= 0.0) && !ex;
                if (bal(amb)) ex = amb ? d_w_max / w_max < tol : ex;
                rl = (rl & ~ambm) | (bal(ex) & ambm);
                wz = bal(w_max == 0.0) & ambm;
            }
        }
        const unsigned long long chk = ~dmask & (wz | rl | (it == max_iter - 1 ? ~0ull : 0ull));
#ifdef CCD_CD_CHKSTAT
        {
            // diagnostic: sweeps, sweeps that take the duality-gap test, sweeps whose live band
            // groups all sit in one half of their 16-lane rows (even groups 0, 2, 4, 6 or odd 1, 3, 5:
            // one of the two broadcast FMAs would do); slot 27: sweeps whose float pre-check of the
            // stopping ratio is ambiguous (the 64-bit reductions)
            constexpr unsigned long long EVEN = 0x00FF00FF00FF00FFull;
            const unsigned long long live = ~dmask;
            PH_COUNT(P, 24, 1)
            PH_COUNT(P, 25, chk ? 1 : 0)
            PH_COUNT(P, 26, ((live & EVEN) == 0ull || (live & ~EVEN) == 0ull) ? 1 : 0)
        }
#endif
        if (chk) {
            const double xta = act ? fma(-gkk, w, h) : 0.0;  // X^T R = g = h - G_kk w
            const double dual = gmax8(fabs(xta));
            const double wq = gsum8(w * q);
            const double wxta = gsum8(w * xta);
            const double l1 = gsum8(fabs(w));
            const double ry = yy - wq;    // R . y
            const double rr = ry - wxta;  // R . R = yy - 2 w.q + w.G.w
            double cst, gap;
            if (dual > alpha) {
                cst = alpha / dual;
                gap = 0.5 * (rr + rr * cst * cst);
            } else {
                cst = 1.0;
                gap = rr;
            }
            gap += alpha * l1 - cst * ry;
            const unsigned long long fin = chk & bal(gap < tol_s);
            if (fin) {
                const bool f = (fin >> l) & 1ull;
                sweeps = f ? it + 1 : sweeps;
#pragma unroll
                for (int j = 0; j < 7; ++j) gcol[j] = f ? 0.0 : gcol[j];  // h and w of the group stay as they are
                dmask |= fin;
            }
        }
    }
    if (b < NB && k < 7) L->coef[b][k] = act ? w : 0.0;
#ifdef CCD_CD_CYCLES
    {
        // groups that ran max_iter sweeps: how many, how many of them had cycled, and the sums
        // of their detection sweeps and periods (lane 8b stands for group b)
        const bool mx = k == 0 && b < NB && sweeps >= max_iter;
        const bool mc = mx && det_it > 0;
        int v0 = mx ? 1 : 0, v1 = mc ? 1 : 0, v2 = mc ? det_it : 0, v3 = mc ? det_per : 0;
        for (int o = 32; o > 0; o >>= 1) {
            v0 += shfx(v0, o);
            v1 += shfx(v1, o);
            v2 += shfx(v2, o);
            v3 += shfx(v3, o);
        }
        PH_COUNT(P, 24, v0)
        PH_COUNT(P, 25, v1)
        PH_COUNT(P, 26, v2)
        PH_COUNT(P, 27, v3)
    }
#endif
    return sweeps;
}
// the sweep with its coordinate count unrolled for the three model sizes (no per-coordinate branch)
__device__ __forceinline__ int cd_lanes(Lds *L, int pc, double alpha, int max_iter, double tol) {
    switch (pc) {
    case 3: return cd_sweep<3>(L, pc, alpha, max_iter, tol);
    case 5: return cd_sweep<5>(L, pc, alpha, max_iter, tol);
    case 7: return cd_sweep<7>(L, pc, alpha, max_iter, tol);
    default: return cd_sweep<0>(L, pc, alpha, max_iter, tol);
    }
}

// residual of band b at compacted observation j for the current models (lasso.predict)
__device__ __forceinline__ double resid_at(const Px &P, int band, int j) {
    const int g = prow(P, j, __LINE__);
    const CRow *rw = PCR(P) + g;  // band value and index read in place (no dynamically indexed copy)
    const GLOBAL_AS double *bs = P.basis + (size_t)gidx(P, rw->ci, P.n, __LINE__) * CCD_BASIS_STRIDE;
    const double *c = LDS().coef[band];
    double pr = bs[0] * c[0];  // bs[0] = (double) date
#pragma unroll
    for (int jj = 1; jj < 7; ++jj) pr += bs[jj] * c[jj];
    pr += c[7];
    return (double)rw->v[band] - pr;
}

// lasso.fitted_model for the 7 bands over compacted window [a, b) with k coefficients.
// with_rmse = false leaves L->rmse to the caller (fit_bounds computes it from the same
// residuals).  A window and k equal to the last fit's keep the models as they are.
__device__ __forceinline__ void fit_models(Px &P, int a, int b, int k, bool with_rmse = true) {
    const ccdgpu_params &p = ARGS().p;
    Lds *L = &LDS();
    const int l = lane();
    const int nw = b - a;
    const int pc = k - 1;  // active design columns (t + harmonics)
    if (P.acc_a == a && P.acc_b == b && P.fit_k == k) return;  // same rows, same model
    PH_BEGIN(gram)
    gram_accumulate(P, a, b);
    gram_finalize(P, nw);
    P.fit_k = k;
    PH_END(P, gram, 4)
    PH_BEGIN(cd)
    // coordinate descent: lane = band * 8 + coordinate
    const int sw = cd_lanes(L, pc, p.lasso_alpha * nw, p.lasso_max_iter, p.lasso_tol);
    if ((l & 7) == 0 && (l >> 3) < NB) {
        stat_lane(ST_SWEEPS, (unsigned long long)sw);
        stat_lane(ST_FLOPS, (unsigned long long)sw * (unsigned long long)(2 * k * k + 6 * k));  // CD: iters (2k^2 + 6k)
    }
#ifdef CCD_PHASE_TIMERS
    {
        int wsw = (l >> 3) < NB ? sw : 0;  // the wave's sweep count: max over the band groups
        for (int o = 32; o > 0; o >>= 1) {
            const int t = shfx(wsw, o);
            wsw = t > wsw ? t : wsw;
        }
        PH_COUNT(P, 28, wsw >= p.lasso_max_iter ? 1 : 0)
        PH_COUNT(P, 29, wsw)
        PH_COUNT(P, 30, wsw >= p.lasso_max_iter ? wsw : 0)
    }
#endif
    wsync();
    if (l < NB) {
        double dot = 0.0;
#pragma unroll
        for (int j = 0; j < 7; ++j) dot += L->xm[j] * L->coef[l][j];
        L->coef[l][7] = L->ym[l] - dot;
    }
    stat_uniform(ST_FITS, NB);
    PH_COUNT(P, 19, 1)
    // SURVEY.md 8(d) op-count model: Gram + column sums n k (k+1), RHS 7 * 2 n k,
    // residual / rmse 7 (2 n k + 3 n)  (k = number of coefficients incl. intercept)
    stat_uniform(ST_FLOPS, (unsigned long long)nw * (unsigned long long)(k * (k + 1) + 14 * k + 7 * (2 * k + 3)));
    wsync();
    PH_END(P, cd, 5)
    PH_BEGIN(rmse)
    // rmse from residuals of the raw design (predict = X @ coef + intercept);
    // lane = (observation sub-index, band), 8 observations per pass
    if (with_rmse) {
        const int bnd = l >> 3, osub = l & 7;  // band-major: DPP reduction over the 8 partials
        double ss = 0.0;
        if (bnd < NB)
            for (int t0 = osub; t0 < nw; t0 += 8) {
                const double r = resid_at(P, bnd, a + t0);
                ss += r * r;
            }
        ss = gsum8(ss);
        const double den = (double)(nw - (p.rmse_dof ? k : 0));
        if (osub == 0 && bnd < NB) L->rmse[bnd] = sqrt(ss / den);
    }
    wsync();
    PH_END(P, rmse, 6)
}


// ------------------------------------------------------------------ segment output
__device__ __forceinline__ void emit(Px &P, int sday, int eday, int bday, int count, double chprob, int cqa,
                     double mag_lane /* lane b: magnitude of band b */) {
    const CcdDetectArgs &A = ARGS();
    const int l = lane();
    unsigned long long slot = 0;
    if (l == 0) slot = atomicAdd(&A.counters[1], 1ull);
    slot = uni(slot);  // lane 0's
    if (slot >= (unsigned long long)A.pool_cap) {
        if (l == 0) atomicOr(&A.counters[3], 1ull);
        P.nseg++;
        return;
    }
    ccdgpu_segment *s = A.pool + slot;
    if (l < NB) {
        s->magnitude[l] = mag_lane;
        s->rmse[l] = LDS().rmse[l];
        s->intercept[l] = LDS().coef[l][7];
#pragma unroll
        for (int j = 0; j < 7; ++j) s->coef[l][j] = LDS().coef[l][j];
    }
    if (l == 0) {
        s->start_day = sday;
        s->end_day = eday;
        s->break_day = bday;
        s->observation_count = count;
        s->curve_qa = cqa;
        s->pixel = (int32_t)P.gpix;
        s->change_probability = chprob;
        A.pool_seq[slot] = P.nseg;
    }
    P.nseg++;
}

// change.catch (a segment fit with the minimum coefficients over compacted [a, b)).  whole: the
// permanent-snow / insufficient-clear procedures' single segment, which spans the input's sorted
// dates (first to last, all observations) with break day 0.
__device__ __forceinline__ void catch_(Px &P, int a, int b, int cqa, bool whole = false) {
    fit_models(P, a, b, ARGS().p.coef_min);
    const int bday = whole ? 0 : b < P.m ? CDR(P, b) : CDR(P, P.m - 1);
    const int sday = whole ? (int)P.sd[0] : CDR(P, a);
    const int eday = whole ? (int)P.sd[P.n - 1] : CDR(P, b - 1);
    emit(P, sday, eday, bday, b - a, 0.0, cqa, 0.0);
}

// Bin of the 256-bin histogram L->hist2[0..255] holding the rank-th smallest entry; rank becomes
// the rank within that bin.
__device__ __forceinline__ int hist_find(const Lds *L, int &rank) {
    const int l = lane();
    int carry = 0;
    for (int b0 = 0; b0 < 256; b0 += W) {
        const int c = (int)L->hist2[b0 + l];
        const int cum = wscan_incl(c) + carry;
        const unsigned long long hit = bal(cum > rank);
        if (hit) {
            const int src = __ffsll((long long)hit) - 1;
            rank -= rdl(cum, src) - rdl(c, src);
            return b0 + src;
        }
        carry = rdl(cum, W - 1);
    }
    return 0;
}

// hist_find over a 256-bin histogram of u16 counters packed two per word.
__device__ __forceinline__ int hist_find16(const uint32_t *h, int &rank) {
    const int l = lane();
    int carry = 0;
    for (int b0 = 0; b0 < 256; b0 += W) {
        const int x = b0 + l;
        const int c = (int)((h[x >> 1] >> ((x & 1) * 16)) & 0xFFFFu);
        const int cum = wscan_incl(c) + carry;
        const unsigned long long hit = bal(cum > rank);
        if (hit) {
            const int src = __ffsll((long long)hit) - 1;
            rank -= rdl(cum, src) - rdl(c, src);
            return b0 + src;
        }
        carry = rdl(cum, W - 1);
    }
    return 0;
}

// Histogram (L->hist2[0..255]) of the low bytes (pass 1, high byte hb) or the high bytes
// (pass 0, hb < 0) of the values gen produces.
template <class F>
__device__ __forceinline__ void hist_u16(F gen, int N, int hb) {
    Lds *L = &LDS();
    const int l = lane();
    for (int i = l; i < 256; i += W) L->hist2[i] = 0u;
    wsync();
#pragma unroll 4
    for (int base = 0; base < N; base += W) {
        const int i = base + l;
        int v = 0;
        if (i < N && gen(i, v) && (hb < 0 || (v >> 8) == hb))
            atomicAdd(&L->hist2[hb < 0 ? (v >> 8) : (v & 255)], 1u);
    }
    wsync();
}

// The k0-th and k1-th smallest (0-based, k0 <= k1) of 16-bit unsigned values produced by
// gen(i, &v) for i < N: radix select over 256-bin LDS histograms (L->hist2 as scratch), the two
// ranks sharing every pass whose bin they share.  small_first: when both ranks lie among the
// values below 256 (counted with ballots, no histogram) the high-byte pass is skipped -- the
// common case for absolute differences, where a high-byte histogram would put every lane on
// bin 0.
template <class F>
__device__ __forceinline__ void select2_u16(F gen, int N, int k0, int k1, bool small_first, int &v0, int &v1) {
    Lds *L = &LDS();
    int h0 = 0, h1 = 0, r0 = k0, r1 = k1;
    bool known = false;
    if (small_first) {
        int c = 0;
        for (int base = 0; base < N; base += W) {
            const int i = base + lane();
            int v = 0;
            c += popc(bal(i < N && gen(i, v) && v < 256));
        }
        known = k1 < c;
    }
    if (!known) {
        hist_u16(gen, N, -1);
        h0 = hist_find(L, r0);
        h1 = hist_find(L, r1);
        wsync();
    }
    hist_u16(gen, N, h0);
    v0 = (h0 << 8) | hist_find(L, r0);
    if (h1 == h0) {
        v1 = (h1 << 8) | hist_find(L, r1);
    } else {
        wsync();
        hist_u16(gen, N, h1);
        v1 = (h1 << 8) | hist_find(L, r1);
    }
    wsync();
}

template <class F>
__device__ __forceinline__ double median_u16(F gen, int N, int cnt, bool small_first = false) {
    if (cnt <= 0) return __builtin_nan("");
    int a, b;
    select2_u16(gen, N, (cnt - 1) / 2, cnt / 2, small_first, a, b);
    if (cnt & 1) return (double)a;
    return ((double)a + (double)b) / 2.0;
}

// ------------------------------------------------------------------ variogram / peek
__device__ __forceinline__ void variogram(Px &P) {
    Lds *L = &LDS();
    const int l = lane();
    const int m = P.m;
    if (m < 2) {
        if (l < NB) L->vario[l] = __builtin_nan("");
        wsync();
        return;
    }
    int lag = 0;
    {
        // lags 1..4 (where the lag is found nearly always) counted in one pass over the dates
        int c4[4] = {0, 0, 0, 0};
        for (int base = 0; base < m - 1; base += W) {
            const int i = base + l;
            const int d0 = i < m ? CDR(P, i) : 0;
            int dk[4];
#pragma unroll
            for (int k = 1; k <= 4; ++k) dk[k - 1] = i + k < m ? CDR(P, i + k) : 0;
#pragma unroll
            for (int k = 1; k <= 4; ++k) c4[k - 1] += popc(bal(i + k < m && dk[k - 1] - d0 > 30));
        }
#pragma unroll
        for (int k = 1; k <= 4; ++k)
            if (!lag && k < m && 2 * c4[k - 1] >= m - k) lag = k;
    }
    for (int k = 5; !lag && k < m; ++k) {
        int cnt = 0;
        for (int base = 0; base < m - k; base += W) {
            const int i = base + l;
            cnt += popc(bal(i < m - k && (CDR(P, i + k) - CDR(P, i)) > 30));
        }
        if (2 * cnt >= m - k) { lag = k; break; }
    }
    const int kk = lag ? lag : 1;
    const bool all = lag == 0;
    // the qualifying absolute differences of all 7 bands, compacted once into the slot's scratch
    // (band-major u16 [7][n]); the same pass histograms every band's differences below 256 in
    // LDS (u16 counters, 128 words per band, in the row tile) and counts them, so a band whose two
    // middle ranks lie below 256 -- nearly always -- needs no further pass over its differences
    GLOBAL_AS uint16_t *dv = reinterpret_cast<GLOBAL_AS uint16_t *>(PFS(P));
    uint32_t *h16w = reinterpret_cast<uint32_t *>(&L->row[0][0]);
    for (int i = l; i < NB * 128; i += W) h16w[i] = 0u;
    wsync();
    const int stride = P.n;
    int cnt = 0;
    int small[NB];
#pragma unroll
    for (int band = 0; band < NB; ++band) small[band] = 0;
    // two chunks per round, loads before the stores; the next round's loads go out before this
    // round's stores
    constexpr int U = 2;
    bool okn[U];
    uint4 r0n[U], r1n[U];
    auto load = [&](int base0, bool (&okv)[U], uint4 (&r0v)[U], uint4 (&r1v)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base0 + u * W + l;
            okv[u] = false;
            r0v[u] = uint4{0u, 0u, 0u, 0u};
            r1v[u] = uint4{0u, 0u, 0u, 0u};
            if (i < m - kk) {
                okv[u] = all || (CDR(P, i + kk) - CDR(P, i)) > 30;
                r0v[u] = CROW4(P, i);
                r1v[u] = CROW4(P, i + kk);
            }
        }
    };
    load(0, okn, r0n, r1n);
    for (int base0 = 0; base0 < m - kk; base0 += U * W) {
        bool okv[U];
        uint4 r0v[U], r1v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            okv[u] = okn[u];
            r0v[u] = r0n[u];
            r1v[u] = r1n[u];
        }
        load(base0 + U * W, okn, r0n, r1n);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool ok = okv[u];
            const uint4 r0 = r0v[u], r1 = r1v[u];
            const unsigned long long km = bal(ok);
            const unsigned a0[4] = {r0.x, r0.y, r0.z, r0.w}, a1[4] = {r1.x, r1.y, r1.z, r1.w};
#pragma unroll
            for (int band = 0; band < NB; ++band) {
                const int v0 = (int)(int16_t)(a0[band >> 1] >> ((band & 1) * 16));
                const int v1 = (int)(int16_t)(a1[band >> 1] >> ((band & 1) * 16));
                const int d = v1 - v0;
                const int ad = d < 0 ? -d : d;
                const bool lo = ok && ad < 256;
                small[band] += popc(bal(lo));
                if (ok) dv[band * stride + cnt + below(km)] = (uint16_t)ad;
                if (lo) atomicAdd(&h16w[band * 128 + (ad >> 1)], 1u << ((ad & 1) * 16));
            }
            cnt += popc(km);
        }
    }
    gsync();
    for (int band = 0; band < NB; ++band) {
        double med;
        if (cnt <= 0) {
            med = __builtin_nan("");
        } else if (cnt / 2 < small[band]) {
            // both middle ranks among the differences below 256: read them off the histogram
            int r0 = (cnt - 1) / 2, r1 = cnt / 2;
            const int a = hist_find16(h16w + band * 128, r0);
            const int b2 = hist_find16(h16w + band * 128, r1);
            med = (cnt & 1) ? (double)a : ((double)a + (double)b2) / 2.0;
        } else {
            const GLOBAL_AS uint16_t *col = dv + band * stride;
            auto gen = [&](int i, int &val) -> bool {
                val = (int)col[i];
                return true;
            };
            med = median_u16(gen, cnt, cnt, true);
        }
        if (l == 0) L->vario[band] = med;
        stat_uniform(ST_FLOPS, 2ull * (unsigned long long)(m - kk));  // 2 per difference per band
    }
    wsync();
}

__device__ __forceinline__ void adjust_peek(Px &P) {
    const ccdgpu_params &p = ARGS().p;
    P.peek = p.peek_size;
    if (lane() == 0) LDS().chg = p.change_threshold;  // (in LDS: read where compared, never spilled)
    if (!p.adaptive_peek || P.m < 2) return;
    auto gen = [&](int i, int &val) -> bool {
        val = CDR(P, i + 1) - CDR(P, i);
        return true;
    };
    const bool narrow = CDR(P, P.m - 1) - CDR(P, 0) <= 65535;  // every gap fits 16 bits
    const double delta = narrow ? median_u16(gen, P.m - 1, P.m - 1, true) : median_int(gen, P.m - 1, P.m - 1, 0, 1 << 30);
    const double adj = rint((double)(p.peek_size * 16) / delta);
    if (adj > (double)p.peek_size) {
        // With the default PEEK_SIZE (6) the peek is at most 96 = CCDGPU_MAX_PEEK: the compacted
        // period has distinct dates, so the median gap is >= 1 day.  A larger configured
        // PEEK_SIZE can exceed it: the pixel is reported (the call fails with CCDGPU_EOVERFLOW)
        // and finished with the largest supported peek so the launch still drains.
        if (adj > (double)CCDGPU_MAX_PEEK && lane() == 0) atomicMin(&ARGS().counters[7], (unsigned long long)P.gpix);
        P.peek = uni(adj > (double)CCDGPU_MAX_PEEK ? CCDGPU_MAX_PEEK : (int)adj);
        if (lane() == 0) LDS().chg = ARGS().thr_table[P.peek];
    }
}

// ------------------------------------------------------------------ Tmask (models/tmask.py + robust_fit.py)
// Tmask design row: [cos wt, sin wt, cos (w/N) t, sin (w/N) t, 1]; when N = 1 the annual and the
// observation cycle coincide (rank-deficient 5-column design) and the row is [cos, sin, 1, 0, 0]
// with the two unused normal-matrix diagonals pinned to 1 (Tmask).
__device__ __forceinline__ void tm_row(const Px &P, int j, int i, int ncol, const GLOBAL_AS double *xoc,
                                       const GLOBAL_AS double *xos, double (&x)[5]) {
    const GLOBAL_AS double *bs = P.basis + (size_t)CIR(P, j) * CCD_BASIS_STRIDE;
    x[0] = bs[1];
    x[1] = bs[2];
    if (ncol == 5) {
        x[2] = xoc[i];
        x[3] = xos[i];
        x[4] = 1.0;
    } else {
        x[2] = 1.0;
        x[3] = 0.0;
        x[4] = 0.0;
    }
}

// acc += w x_ea x_eb over staged rows 0 .. cnt4 - 1 (cnt4 a multiple of 4), sequential over the
// rows, four rows per round with all their LDS reads issued before the first multiply
__device__ __forceinline__ void tm_rows_acc(const Lds *L, int cnt4, int ea, int eb, double &acc) {
    for (int r = 0; r < cnt4; r += 4) {
        double wv[4], xa[4], xb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            wv[u] = L->row[r + u][5];
            xa[u] = L->row[r + u][ea];
            xb[u] = L->row[r + u][eb];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += wv[u] * xa[u] * xb[u];
    }
}

// normal equations sum w x x^T and sum w x y over the window into L->G[0..4][0..4] and
// L->Q[0..4][0]: rows [x0..x4, w, y] staged in LDS 64 at a time, lane = matrix entry,
// sequential over rows (same scheme as the Lasso Gram in fit_models).
__device__ __forceinline__ void tm_normal(const Px &P, int a, int nw, int ncol, const GLOBAL_AS double *xoc,
                                       const GLOBAL_AS double *xos, int band, const GLOBAL_AS double *wv) {
    Lds *L = &LDS();
    const int l = lane();
    int ea = -1, eb = -1;
    if (l < 15) {
        int e = l, r = 0;
        while (e > r) { e -= r + 1; ++r; }
        ea = r;
        eb = e;
    } else if (l < 20) {
        ea = l - 15;
        eb = 6;
    }
    double acc = 0.0;
    for (int t0 = 0; t0 < nw; t0 += TR) {
        const int cnt = nw - t0 < TR ? nw - t0 : TR;
        const int cnt4 = (cnt + 3) & ~3;  // rows cnt .. cnt4 - 1 staged as zeros (add nothing)
        if (l < cnt) {
            const int i = t0 + l;
            double x[5];
            tm_row(P, a + i, i, ncol, xoc, xos, x);
            double *row = L->row[l];
#pragma unroll
            for (int r = 0; r < 5; ++r) row[r] = x[r];
            row[5] = wv ? wv[i] : 1.0;
            row[6] = band >= 0 ? cvalf(P, band, a + i) : 0.0;
        } else if (l < cnt4) {
            double *row = L->row[l];
#pragma unroll
            for (int r = 0; r < 7; ++r) row[r] = 0.0;
        }
        wsync();
        if (ea >= 0) tm_rows_acc(L, cnt4, ea, eb, acc);
        wsync();
    }
    if (l < 15) {
        L->G[ea][eb] = acc;
        L->G[eb][ea] = acc;
    } else if (l < 20) {
        L->Q[ea][0] = acc;
    }
    wsync();
    if (ncol == 3 && l == 0) {
        L->G[3][3] = 1.0;
        L->G[4][4] = 1.0;
    }
    wsync();
}

__device__ __forceinline__ void tm_load(const Lds *L, double (&A)[5][5], double (&rhs)[5]) {
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        rhs[r] = L->Q[r][0];
#pragma unroll
        for (int c = 0; c < 5; ++c) A[r][c] = L->G[r][c];
    }
}

// in-place lower Cholesky factor of a 5x5 SPD matrix; false if not positive definite.  Each
// column divides by its pivot as a multiply by the pivot's reciprocal (one IEEE division per
// column instead of one per entry: a division is ~10 VALU instructions on gfx950).
__device__ __forceinline__ bool chol5(double (&a)[5][5]) {
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        double d = a[j][j];
#pragma unroll
        for (int k = 0; k < j; ++k) d -= a[j][k] * a[j][k];
        if (!(d > 0.0)) return false;
        d = sqrt(d);
        a[j][j] = d;
        const double rd = 1.0 / d;
#pragma unroll
        for (int i = j + 1; i < 5; ++i) {
            double s = a[i][j];
#pragma unroll
            for (int k = 0; k < j; ++k) s -= a[i][k] * a[j][k];
            a[i][j] = s * rd;
        }
    }
    return true;
}
// forward / back substitution with the factor: the 5 pivot reciprocals once, shared by both
__device__ __forceinline__ void chol5_solve(const double (&c)[5][5], const double (&b)[5], double (&x)[5]) {
    double z[5], r[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) r[i] = 1.0 / c[i][i];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        double s = b[i];
#pragma unroll
        for (int k = 0; k < i; ++k) s -= c[i][k] * z[k];
        z[i] = s * r[i];
    }
#pragma unroll
    for (int i = 4; i >= 0; --i) {
        double s = z[i];
#pragma unroll
        for (int k = i + 1; k < 5; ++k) s -= c[k][i] * x[k];
        x[i] = s * r[i];
    }
}

// solve with a fallback for a (numerically) singular weighted system: zero coefficients
__device__ __forceinline__ void tm_solve(double (&A)[5][5], const double (&rhs)[5], double (&coef)[5]) {
    if (chol5(A)) {
        chol5_solve(A, rhs, coef);
    } else {
#pragma unroll
        for (int r = 0; r < 5; ++r) coef[r] = 0.0;
    }
}

__device__ __forceinline__ double tm_pred(const Px &P, int j, int i, int ncol, const GLOBAL_AS double *xoc,
                                          const GLOBAL_AS double *xos, const double (&coef)[5]) {
    double x[5];
    tm_row(P, j, i, ncol, xoc, xos, x);
    double pr = 0.0;
#pragma unroll
    for (int r = 0; r < 5; ++r) pr += x[r] * coef[r];
    return pr;
}

// cos / sin of the observation-cycle harmonic (w / N) t for the window (lane = obs)
__device__ __forceinline__ void tm_trig(const Px &P, int a, int nw, double oc, GLOBAL_AS double *xoc, GLOBAL_AS double *xos) {
    for (int i = lane(); i < nw; i += W) {
        double sv, cv;
        sincos(oc * (double)CDR(P, a + i), &sv, &cv);
        xoc[i] = cv;
        xos[i] = sv;
    }
}

// ---- Tmask for windows of at most 64 observations (the initialize windows): lane = window
// observation, its design row, value and weights held in registers for the whole call, so the
// IRLS iterations re-read nothing from memory; the normal equations are summed through the LDS
// row tile as in tm_normal (same order, same arithmetic: results equal the generic path's).
__device__ __forceinline__ void tm_normal_reg(const double (&x)[5], double wv, double yv, int nw, int ncol) {
    Lds *L = &LDS();
    const int l = lane();
    int ea = -1, eb = -1;
    if (l < 15) {
        int e = l, r = 0;
        while (e > r) { e -= r + 1; ++r; }
        ea = r;
        eb = e;
    } else if (l < 20) {
        ea = l - 15;
        eb = 6;
    }
    double acc = 0.0;
    for (int t0 = 0; t0 < nw; t0 += TR) {
        const int cnt = nw - t0 < TR ? nw - t0 : TR;
        const int cnt4 = (cnt + 3) & ~3;  // rows cnt .. cnt4 - 1 staged as zeros (add nothing)
        if (l >= t0 && l < t0 + cnt4) {
            const bool rv = l < t0 + cnt;
            double *row = L->row[l - t0];
#pragma unroll
            for (int r = 0; r < 5; ++r) row[r] = rv ? x[r] : 0.0;
            row[5] = rv ? wv : 0.0;
            row[6] = rv ? yv : 0.0;
        }
        wsync();
        if (ea >= 0) tm_rows_acc(L, cnt4, ea, eb, acc);
        wsync();
    }
    if (l < 15) {
        L->G[ea][eb] = acc;
        L->G[eb][ea] = acc;
    } else if (l < 20) {
        L->Q[ea][0] = acc;
    }
    wsync();
    if (ncol == 3 && l == 0) {
        L->G[3][3] = 1.0;
        L->G[4][4] = 1.0;
    }
    wsync();
}

__device__ __forceinline__ double tm_dot(const double (&x)[5], const double (&coef)[5]) {
    double pr = 0.0;
#pragma unroll
    for (int r = 0; r < 5; ++r) pr += x[r] * coef[r];
    return pr;
}

__device__ __forceinline__ int tmask_reg(Px &P, int a, int b) {
    const ccdgpu_params &p = ARGS().p;
    Lds *L = &LDS();
    const int l = lane();
    const int nw = b - a;
    const double w = 2.0 * M_PI / p.avg_days_yr;
    const double oc = w / ceil(((double)CDR(P, b - 1) - (double)CDR(P, a)) / p.avg_days_yr);
    const int ncol = (oc == w) ? 3 : 5;
    const bool in = l < nw;
    double x[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    uint4 q = {0u, 0u, 0u, 0u};  // the observation's row: band values + sorted index
    if (in) {
        q = CROW4(P, a + l);
        const GLOBAL_AS double *bs = P.basis + (size_t)gidx(P, (int)(q.w >> 16), P.n, __LINE__) * CCD_BASIS_STRIDE;
        x[0] = bs[1];
        x[1] = bs[2];
        if (ncol == 5) {
            double sv, cv;
            sincos(oc * (double)CDR(P, a + l), &sv, &cv);
            x[2] = cv;
            x[3] = sv;
            x[4] = 1.0;
        } else {
            x[2] = 1.0;
        }
    }
    if (l < (nw + 31) / 32) L->tflag[l] = 0u;
    // unweighted normal matrix: OLS solves and leverage h = diag(X (X'X)^-1 X') (robust_fit.RLM)
    bool ok0;
    {
        double G0[5][5], rhs0[5];
        tm_normal_reg(x, 1.0, 0.0, nw, ncol);
        tm_load(L, G0, rhs0);
        ok0 = chol5(G0);
        if (l == 0)
#pragma unroll
            for (int r = 0; r < 5; ++r)
#pragma unroll
                for (int c = 0; c < 5; ++c) L->tchol[r][c] = G0[r][c];
    }
    wsync();
    double adj = 0.0;
    if (in) {
        double h = 0.9999;
        if (ok0) {
            double z[5], hh = 0.0;
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                double s2 = x[r];
#pragma unroll
                for (int k = 0; k < r; ++k) s2 -= L->tchol[r][k] * z[k];
                z[r] = s2 / L->tchol[r][r];
                hh += z[r] * z[r];
            }
            h = hh < 0.9999 ? hh : 0.9999;
        }
        adj = 1.0 / sqrt(1.0 - h);
    }
    for (int band = 0; band < NB; ++band) {
        if (!((p.tmask_bands >> band) & 1u)) continue;
        const unsigned word = (band >> 1) == 0 ? q.x : (band >> 1) == 1 ? q.y : (band >> 1) == 2 ? q.z : q.w;
        const double yv = in ? (double)(int16_t)(word >> ((band & 1) * 16)) : 0.0;
        // y statistics (np.std, population)
        const double ym = wsum(yv) / nw;
        const double dy = in ? yv - ym : 0.0;
        const double ystd = sqrt(wsum(dy * dy) / nw);
        double coef[5], coef0[5];
        {
            double Gt[5][5], r0[5];
            tm_normal_reg(x, 1.0, yv, nw, ncol);
            tm_load(L, Gt, r0);
            if (ok0) {
#pragma unroll
                for (int r = 0; r < 5; ++r)
#pragma unroll
                    for (int c = 0; c < 5; ++c) Gt[r][c] = L->tchol[r][c];
                chol5_solve(Gt, r0, coef);
            } else {
                tm_solve(Gt, r0, coef);
            }
        }
        // every lane solved the same system (LDS-broadcast normal equations): the coefficients and
        // the convergence test below are wave-uniform -- as scalars
#pragma unroll
        for (int r = 0; r < 5; ++r) coef[r] = unid(coef[r]);
        stat_uniform(ST_FLOPS, (unsigned long long)nw * 35 + 125);  // OLS fit: n_w 35 + 5^3
        int iteration = 1;
        bool converged = false;
        while (!converged && iteration < 5) {
#pragma unroll
            for (int r = 0; r < 5; ++r) coef0[r] = coef[r];
            const double rr = in ? (yv - tm_dot(x, coef0)) * adj : 0.0;  // signed, adjusted residual
            // mad = median(sort(|r|)[4:]) / 0.6745: one value per lane, bitonic sort across the wave
            const int c = nw - 4;
            const double v = bitonic64(in ? fabs(rr) : __builtin_inf());
            const double hi = shf(v, 4 + c / 2);
            const double lo = shf(v, 4 + (c - 1) / 2);
            const double med = (c & 1) ? hi : (lo + hi) / 2.0;
            const double mad = med / 0.6745;
            const double floor_ = 2.220446049250313e-16 * ystd;
            const double scale = mad > floor_ ? mad : floor_;
            const double u = rr / scale;
            const double qq = u / 4.685;
            const double om = 1.0 - qq * qq;
            const double wt = fabs(u) < 4.685 ? om * om : 0.0;
            double Gw[5][5], rw[5];
            tm_normal_reg(x, in ? wt : 0.0, yv, nw, ncol);
            tm_load(L, Gw, rw);
            tm_solve(Gw, rw, coef);
#pragma unroll
            for (int r = 0; r < 5; ++r) coef[r] = unid(coef[r]);
            stat_uniform(ST_FLOPS, (unsigned long long)nw * 35 + 125);  // each IRLS refit: n_w 35 + 5^3
            iteration += 1;
            converged = true;
#pragma unroll
            for (int r = 0; r < 5; ++r)
                if (coef[r] - coef0[r] > 1e-8) converged = false;
        }
        const double thr = L->vario[band] * p.t_const;
        const double pr = tm_dot(x, coef) + 0.0;
        const unsigned long long bm = bal(in && fabs(pr - yv) > thr);
        if (l == 0) {
            L->tflag[0] |= (unsigned)bm;
            if (32 < nw) L->tflag[1] |= (unsigned)(bm >> 32);
        }
        wsync();
    }
    int cnt = 0;
    for (int i = l; i < (nw + 31) / 32; i += W) cnt += __popc(L->tflag[i]);
    for (int o = 32; o > 0; o >>= 1) cnt += shfx(cnt, o);
    wsync();
    return uni(cnt);
}

// ---- Tmask of the two default Tmask bands at once, for windows of at most 32 observations (the
// initialize windows, nearly always): band A (the lower band) in lanes 0..31, band B in lanes
// 32..63, lane = window observation within the half.  Every per-band quantity is computed with
// the arithmetic of tmask_reg, in the same order: the half-wave sums equal wsum's value when the
// other half is zero, the two 32-lane sorts give bitonic64's first 32 values, the weighted normal
// equations of both bands accumulate in one pass over the staged rows (row = x0..x4, wA, yA, wB,
// yB; lane = (band, matrix entry)), and each half solves its band's system.  A band whose IRLS
// has converged (or reached its 5th fit) keeps its coefficients while the other one iterates.
// Half-wave sum (wsum's butterfly, then the two row totals of the lane's half).
__device__ __forceinline__ double hsum2(double v XL) {
    EXEC_FULL();
    v += dpp<0xB1>(v);
    v += dpp<0x4E>(v);
    v += dpp<0x141>(v);
    v += dpp<0x140>(v);
    const double s0 = rdlane(v, 0) + rdlane(v, 16);
    const double s1 = rdlane(v, 32) + rdlane(v, 48);
    return lane() >= 32 ? s1 : s0;
}

// acc += w x_ea x_eb over staged rows 0 .. cnt4 - 1 with the weight in column wc (tm_rows_acc's
// arithmetic and order)
__device__ __forceinline__ void tm_rows_acc_w(const Lds *L, int cnt4, int wc, int ea, int eb, double &acc) {
    for (int r = 0; r < cnt4; r += 4) {
        double wv[4], xa[4], xb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            wv[u] = L->row[r + u][wc];
            xa[u] = L->row[r + u][ea];
            xb[u] = L->row[r + u][eb];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += wv[u] * xa[u] * xb[u];
    }
}

// both bands' normal systems [G | rhs] into L->tsys[half]: rows staged by the observation lanes
// (x, each half its weight and value), entries accumulated by lanes (half, e), e < 20 (e < 15: the
// upper triangle of G, 15..19: rhs); with_g = false sums the rhs only
__device__ __forceinline__ void tm_normal_pair(const double (&x)[5], double wv, double yv, int nw, int ncol, bool with_g) {
    Lds *L = &LDS();
    const int l = lane();
    const int hf = l >> 5, i = l & 31;
    const int cnt4 = (nw + 3) & ~3;  // rows nw .. cnt4 - 1 staged as zeros (add nothing)
    if (i < cnt4) {
        const bool rv = i < nw;
        double *row = L->row[i];
        if (hf == 0) {
#pragma unroll
            for (int r = 0; r < 5; ++r) row[r] = rv ? x[r] : 0.0;
        }
        row[5 + 2 * hf] = rv ? wv : 0.0;
        row[6 + 2 * hf] = rv ? yv : 0.0;
    }
    wsync();
    int ea = -1, eb = -1;
    if (i < 15) {
        int e = i, r = 0;
        while (e > r) { e -= r + 1; ++r; }
        ea = r;
        eb = e;
    } else if (i < 20) {
        ea = i - 15;
        eb = 6 + 2 * hf;
    }
    double acc = 0.0;
    if (ea >= 0 && (with_g || i >= 15)) tm_rows_acc_w(L, cnt4, 5 + 2 * hf, ea, eb, acc);
    wsync();
    if (i < 15) {
        if (with_g) {
            L->tsys[hf][ea][eb] = acc;
            L->tsys[hf][eb][ea] = acc;
        }
    } else if (i < 20) {
        L->tsys[hf][ea][5] = acc;
    }
    wsync();
    if (with_g && ncol == 3 && i == 0) {
        L->tsys[hf][3][3] = 1.0;
        L->tsys[hf][4][4] = 1.0;
    }
    wsync();
}

__device__ __forceinline__ int tmask_pair(Px &P, int a, int b, int bandA, int bandB) {
    const ccdgpu_params &p = ARGS().p;
    Lds *L = &LDS();
    const int l = lane();
    const int hf = l >> 5, i = l & 31;
    const int band = hf ? bandB : bandA;
    const int nw = b - a;
    const double w = 2.0 * M_PI / p.avg_days_yr;
    const double oc = w / ceil(((double)CDR(P, b - 1) - (double)CDR(P, a)) / p.avg_days_yr);
    const int ncol = (oc == w) ? 3 : 5;
    const bool in = i < nw;
    double x[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    uint4 q = {0u, 0u, 0u, 0u};  // the observation's row: band values + sorted index
    if (in) {
        q = CROW4(P, a + i);
        const GLOBAL_AS double *bs = P.basis + (size_t)gidx(P, (int)(q.w >> 16), P.n, __LINE__) * CCD_BASIS_STRIDE;
        x[0] = bs[1];
        x[1] = bs[2];
        if (ncol == 5) {
            double sv, cv;
            sincos(oc * (double)CDR(P, a + i), &sv, &cv);
            x[2] = cv;
            x[3] = sv;
            x[4] = 1.0;
        } else {
            x[2] = 1.0;
        }
    }
    if (l == 0) L->tflag[0] = 0u;
    // unweighted normal matrix (tmask_reg's: rows from lanes 0 .. nw-1, which are half A's)
    bool ok0;
    {
        double G0[5][5], rhs0[5];
        tm_normal_reg(x, 1.0, 0.0, nw, ncol);
        tm_load(L, G0, rhs0);
        ok0 = chol5(G0);
        if (l == 0)
#pragma unroll
            for (int r = 0; r < 5; ++r)
#pragma unroll
                for (int c = 0; c < 5; ++c) L->tchol[r][c] = G0[r][c];
    }
    wsync();
    double adj = 0.0;
    if (in) {
        double h = 0.9999;
        if (ok0) {
            double z[5], hh = 0.0;
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                double s2 = x[r];
#pragma unroll
                for (int k = 0; k < r; ++k) s2 -= L->tchol[r][k] * z[k];
                z[r] = s2 / L->tchol[r][r];
                hh += z[r] * z[r];
            }
            h = hh < 0.9999 ? hh : 0.9999;
        }
        adj = 1.0 / sqrt(1.0 - h);
    }
    const unsigned word = (band >> 1) == 0 ? q.x : (band >> 1) == 1 ? q.y : (band >> 1) == 2 ? q.z : q.w;
    const double yv = in ? (double)(int16_t)(word >> ((band & 1) * 16)) : 0.0;
    // y statistics (np.std, population)
    const double ym = hsum2(yv) / nw;
    const double dy = in ? yv - ym : 0.0;
    const double ystd = sqrt(hsum2(dy * dy) / nw);
    // OLS: the unweighted matrix's factor and each band's rhs
    double coef[5], coef0[5];
    tm_normal_pair(x, 1.0, yv, nw, ncol, false);
    {
        double rhs[5];
#pragma unroll
        for (int r = 0; r < 5; ++r) rhs[r] = L->tsys[hf][r][5];
        if (ok0) {
            double Gt[5][5];
#pragma unroll
            for (int r = 0; r < 5; ++r)
#pragma unroll
                for (int c = 0; c < 5; ++c) Gt[r][c] = L->tchol[r][c];
            chol5_solve(Gt, rhs, coef);
        } else {
#pragma unroll
            for (int r = 0; r < 5; ++r) coef[r] = 0.0;  // tm_solve of the unweighted matrix: not SPD
        }
    }
    int iteration = 1;
    bool converged = false;
    while (bal(!converged && iteration < 5)) {
        const bool run = !converged && iteration < 5;  // this half's band still iterates
#pragma unroll
        for (int r = 0; r < 5; ++r) coef0[r] = coef[r];
        const double rr = in ? (yv - tm_dot(x, coef0)) * adj : 0.0;  // signed, adjusted residual
        // mad = median(sort(|r|)[4:]) / 0.6745: each half sorts its band's 32 values
        const int c = nw - 4;
        const double v = bitonic32x2(in ? fabs(rr) : __builtin_inf());
        const double hi = shf(v, (l & 32) + 4 + c / 2);
        const double lo = shf(v, (l & 32) + 4 + (c - 1) / 2);
        const double med = (c & 1) ? hi : (lo + hi) / 2.0;
        const double mad = med / 0.6745;
        const double floor_ = 2.220446049250313e-16 * ystd;
        const double scale = mad > floor_ ? mad : floor_;
        const double u = rr / scale;
        const double qq = u / 4.685;
        const double om = 1.0 - qq * qq;
        const double wt = fabs(u) < 4.685 ? om * om : 0.0;
        tm_normal_pair(x, in ? wt : 0.0, yv, nw, ncol, true);
        double Gw[5][5], rw[5], cn[5];
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            rw[r] = L->tsys[hf][r][5];
#pragma unroll
            for (int cc = 0; cc < 5; ++cc) Gw[r][cc] = L->tsys[hf][r][cc];
        }
        tm_solve(Gw, rw, cn);
        bool conv = true;
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            coef[r] = run ? cn[r] : coef0[r];
            if (coef[r] - coef0[r] > 1e-8) conv = false;
        }
        converged = run ? conv : converged;
        iteration += run ? 1 : 0;
    }
    // counted flops: per band an OLS fit and each IRLS refit, n_w 35 + 5^3 each
    {
        const int fits = rdl(iteration, 0) + rdl(iteration, 32);  // (1 + refits) per band
        stat_uniform(ST_FLOPS, (unsigned long long)fits * ((unsigned long long)nw * 35 + 125));
    }
    const double thr = L->vario[band] * p.t_const;
    const double pr = tm_dot(x, coef) + 0.0;
    const unsigned long long bm = bal(in && fabs(pr - yv) > thr);
    const unsigned fl = (unsigned)bm | (unsigned)(bm >> 32);
    if (l == 0) L->tflag[0] = fl;
    wsync();
    return __popc(fl);
}

// Returns the outlier count; outlier flags in L->tflag (bit i = window observation i).
__device__ __forceinline__ int tmask(Px &P, int a, int b) {
    const ccdgpu_params &p = ARGS().p;
    Lds *L = &LDS();
    const int l = lane();
    const int nw = b - a;
    if (nw <= 32 && __builtin_popcount(p.tmask_bands & 0x7Fu) == 2) {
        const int bA = __builtin_ctz(p.tmask_bands), bB = 31 - __builtin_clz(p.tmask_bands & 0x7Fu);
        return tmask_pair(P, a, b, bA, bB);
    }
    if (nw <= W) return tmask_reg(P, a, b);
    const double w = 2.0 * M_PI / p.avg_days_yr;
    const double oc = w / ceil(((double)CDR(P, b - 1) - (double)CDR(P, a)) / p.avg_days_yr);
    const int ncol = (oc == w) ? 3 : 5;
    GLOBAL_AS double *xoc = PFS(P), *xos = PFS(P) + P.n, *adj = PFS(P) + 2 * P.n, *absr = PFS(P) + 3 * P.n,
           *wt = PFS(P) + 4 * P.n;
    if (ncol == 5) tm_trig(P, a, nw, oc, xoc, xos);
    for (int i = l; i < (nw + 31) / 32; i += W) L->tflag[i] = 0u;
    gsync();
    // unweighted normal matrix: OLS solves and leverage h = diag(X (X'X)^-1 X') (robust_fit.RLM);
    // its Cholesky factor is kept in LDS (L->tchol) for the per-band OLS solves
    bool ok0;
    {
        double G0[5][5], rhs0[5];
        tm_normal(P, a, nw, ncol, xoc, xos, -1, nullptr);
        tm_load(&LDS(), G0, rhs0);
        ok0 = chol5(G0);
        if (l == 0)
#pragma unroll
            for (int r = 0; r < 5; ++r)
#pragma unroll
                for (int c = 0; c < 5; ++c) L->tchol[r][c] = G0[r][c];
    }
    wsync();
    for (int i = l; i < nw; i += W) {
        double x[5];
        tm_row(P, a + i, i, ncol, xoc, xos, x);
        double h = 0.9999;
        if (ok0) {
            double z[5], hh = 0.0;
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                double s2 = x[r];
#pragma unroll
                for (int k = 0; k < r; ++k) s2 -= L->tchol[r][k] * z[k];
                z[r] = s2 / L->tchol[r][r];
                hh += z[r] * z[r];
            }
            h = hh < 0.9999 ? hh : 0.9999;
        }
        adj[i] = 1.0 / sqrt(1.0 - h);
    }
    for (int band = 0; band < NB; ++band) {
        if (!((p.tmask_bands >> band) & 1u)) continue;
        // y statistics (np.std, population)
        double sy = 0.0;
        for (int i = l; i < nw; i += W) sy += cvalf(P, band, a + i);
        const double ym = wsum(sy) / nw;
        double sv = 0.0;
        for (int i = l; i < nw; i += W) {
            const double d = cvalf(P, band, a + i) - ym;
            sv += d * d;
        }
        const double ystd = sqrt(wsum(sv) / nw);
        double coef[5], coef0[5];
        {
            double Gt[5][5], r0[5];
            tm_normal(P, a, nw, ncol, xoc, xos, band, nullptr);
            tm_load(&LDS(), Gt, r0);
            if (ok0) {
#pragma unroll
                for (int r = 0; r < 5; ++r)
#pragma unroll
                    for (int c = 0; c < 5; ++c) Gt[r][c] = L->tchol[r][c];
                chol5_solve(Gt, r0, coef);
            } else {
                tm_solve(Gt, r0, coef);
            }
        }
        // every lane solved the same system (LDS-broadcast normal equations): the coefficients and
        // the convergence test below are wave-uniform -- as scalars
#pragma unroll
        for (int r = 0; r < 5; ++r) coef[r] = unid(coef[r]);
        stat_uniform(ST_FLOPS, (unsigned long long)nw * 35 + 125);  // OLS fit: n_w 35 + 5^3
        int iteration = 1;
        bool converged = false;
        while (!converged && iteration < 5) {
#pragma unroll
            for (int r = 0; r < 5; ++r) coef0[r] = coef[r];
            for (int i = l; i < nw; i += W) {
                const double r = (cvalf(P, band, a + i) - tm_pred(P, a + i, i, ncol, xoc, xos, coef0)) * adj[i];
                wt[i] = r;  // signed, adjusted residual
                absr[i] = fabs(r);
            }
            // mad = median(sort(|r|)[4:]) / 0.6745
            const int c = nw - 4;
            double med;
            if (nw <= W) {
                // one value per lane (lane i wrote absr[i]): bitonic sort across the wave
                const double v = bitonic64(l < nw ? absr[l] : __builtin_inf());
                const double hi = shf(v, 4 + c / 2);
                const double lo = shf(v, 4 + (c - 1) / 2);
                med = (c & 1) ? hi : (lo + hi) / 2.0;
            } else if (c & 1) {
                med = kth_nonneg(absr, nw, 4 + c / 2);
            } else {
                med = (kth_nonneg(absr, nw, 4 + c / 2 - 1) + kth_nonneg(absr, nw, 4 + c / 2)) / 2.0;
            }
            const double mad = med / 0.6745;
            const double floor_ = 2.220446049250313e-16 * ystd;
            const double scale = mad > floor_ ? mad : floor_;
            for (int i = l; i < nw; i += W) {
                const double u = wt[i] / scale;
                const double q = u / 4.685;
                const double om = 1.0 - q * q;
                wt[i] = fabs(u) < 4.685 ? om * om : 0.0;
            }
            double Gw[5][5], rw[5];
            gsync();  // weights written lane-strided, read tile-strided
            tm_normal(P, a, nw, ncol, xoc, xos, band, wt);
            tm_load(&LDS(), Gw, rw);
            tm_solve(Gw, rw, coef);
#pragma unroll
            for (int r = 0; r < 5; ++r) coef[r] = unid(coef[r]);
            stat_uniform(ST_FLOPS, (unsigned long long)nw * 35 + 125);  // each IRLS refit: n_w 35 + 5^3
            iteration += 1;
            converged = true;
#pragma unroll
            for (int r = 0; r < 5; ++r)
                if (coef[r] - coef0[r] > 1e-8) converged = false;
        }
        const double thr = L->vario[band] * p.t_const;
        for (int t0 = 0; t0 < nw; t0 += W) {
            const int i = t0 + l;
            bool out = false;
            if (i < nw) {
                const double pr = tm_pred(P, a + i, i, ncol, xoc, xos, coef) + 0.0;
                out = fabs(pr - cvalf(P, band, a + i)) > thr;
            }
            const unsigned long long bm = bal(out);
            if (l == 0) {
                L->tflag[t0 >> 5] |= (unsigned)bm;
                if (t0 + 32 < nw) L->tflag[(t0 >> 5) + 1] |= (unsigned)(bm >> 32);
            }
        }
        wsync();
    }
    int cnt = 0;
    for (int i = l; i < (nw + 31) / 32; i += W) cnt += __popc(L->tflag[i]);
    for (int o = 32; o > 0; o >>= 1) cnt += shfx(cnt, o);
    wsync();
    return uni(cnt);
}

__device__ __forceinline__ bool tflag_at(const Lds *L, int i) { return (L->tflag[i >> 5] >> (i & 31)) & 1u; }

// ------------------------------------------------------------------ change.py
__device__ __forceinline__ int num_coefs(const ccdgpu_params &p, int n) {
    const double span = (double)n / p.num_obs_factor;
    if (span < p.coef_mid) return p.coef_min;
    if (span < p.coef_max) return p.coef_mid;
    return p.coef_max;
}

__device__ __forceinline__ bool stable(const Px &P, int a, int b) {
    const ccdgpu_params &p = ARGS().p;
    const Lds *L = &LDS();
    const int l = lane();
    double v2 = 0.0;
    if (l < NB && ((p.detection_bands >> l) & 1u)) {
        const double rm = L->rmse[l];
        const double vr = L->vario[l];
        const double rn = rm > vr ? rm : vr;
        const double slope = L->coef[l][0] * ((double)CDR(P, b - 1) - (double)CDR(P, a));
        const double v = (fabs(slope) + fabs(resid_at(P, l, a)) + fabs(resid_at(P, l, b - 1))) / rn;
        v2 = v * v;
    }
    return uni(sqrt(wsum(v2)) < LDS().chg ? 1 : 0) != 0;
}
__device__ __forceinline__ void count_stable(Px &P) {}

__device__ __forceinline__ bool initialize(Px &P, int &wa, int &wb) {
    const ccdgpu_params &p = ARGS().p;
    const Lds *L = &LDS();
    const int l = lane();
    int a = wa, b = wb;
    bool ok = false;
    while (b + p.meow_size < P.m) {
        if (CDRU(P, b - 1) - CDRU(P, a) < p.day_delta) { b += 1; continue; }
        PH_BEGIN(tm)
        const int cnt = tmask(P, a, b);
        PH_END(P, tm, 3)
        PH_COUNT(P, 32, 1)
        const int nw = b - a;
        if (cnt == nw) { b += 1; continue; }
        // first / last kept observation of the window
        int first = 1 << 30, last = -1;
        for (int t0 = 0; t0 < nw; t0 += W) {
            const int i = t0 + l;
            const bool kept = i < nw && !tflag_at(L, i);
            const unsigned long long km = bal(kept);
            if (km) {
                const int f = t0 + __ffsll((long long)km) - 1;
                const int la = t0 + 63 - __clzll(km);
                first = f < first ? f : first;
                last = la;
            }
        }
        if (CDRU(P, a + last) - CDRU(P, a + first) < p.day_delta || nw - cnt < p.meow_size) { b += 1; continue; }
        if (cnt) {
            const int aa = a, bb = b;
            compact_drop(P, a, bb, [&](int j) { return tflag_at(L, j - aa); });
            b -= cnt;
        }
        fit_models(P, a, b, 4);
        PH_COUNT(P, 33, 1)
        count_stable(P);
        PH_BEGIN(st)
        const bool stb = stable(P, a, b);
        PH_END(P, st, 10)
        if (!stb) { a += 1; b += 1; continue; }
        ok = true;
        break;
    }
    wa = a;
    wb = b;
    return ok;
}

// Peek evaluation shared by lookback and lookforward: lane = (peek observation jj, band),
// 8 observations per pass, jj = pass * 8 + (lane >> 3).  Residuals of the current models
// (lasso.predict), change magnitude = sum over detection bands of (r / max(vario, comp))^2
// (change.change_magnitude) reduced over the 8 band lanes.  rl[pass] keeps each lane's residual
// for the segment's magnitude medians.  Returns true iff every peek observation exceeds the
// change threshold (change.detect_change); mag0 = magnitude of observation 0 (detect_outlier).
__device__ __forceinline__ bool eval_peek(Px &P, int k, int start, int dir, double &mag0) {
    const ccdgpu_params &p = ARGS().p;
    Lds *L = &LDS();
    const int l = lane();
    const int bnd = l & 7, osub = l >> 3;
    const bool det = bnd < NB && ((p.detection_bands >> bnd) & 1u);
    double rm = 1.0;
    if (bnd < NB) {
        const double vr = L->vario[bnd], cr = L->comp[bnd];
        rm = (vr != vr || cr != cr) ? __builtin_nan("") : (vr > cr ? vr : cr);
    }
    bool all = true;
    mag0 = 0.0;
    // gathers of up to 4 rounds first (all in flight together), then the magnitudes
    double rr[4];
#pragma unroll
    for (int pass = 0; pass < 4; ++pass) {
        const int jj = pass * 8 + osub;
        rr[pass] = (pass * 8 < k && jj < k && bnd < NB) ? resid_at(P, bnd, start + dir * jj) : 0.0;
    }
#pragma unroll
    for (int pass = 0; pass < CCDGPU_MAX_PEEK / 8; ++pass) {
        if (pass * 8 >= k) break;
        const int jj = pass * 8 + osub;
        const bool valid = jj < k && bnd < NB;
        double r = 0.0;
        if (pass < 4) r = rr[pass < 4 ? pass : 0];
        else if (valid) r = resid_at(P, bnd, start + dir * jj);
        if (jj < k && bnd < NB) {  // kept for the segment's magnitude medians
            if (pass < PSTR / 8) PRES(L)[bnd * PSTR + jj] = r;
            else ring_ovf(P)[bnd * POVF + jj - PSTR] = r;
        }
        const double v = r / rm;
        const double mag = gsum8((valid && det) ? v * v : 0.0);
        if (bal(bnd == 0 && jj < k && !(mag > L->chg))) all = false;
        if (pass == 0) mag0 = unid(mag);  // lane 0's: observation 0 (full EXEC here)
    }
    stat_uniform(ST_FLOPS, (unsigned long long)k * (7 * 2 * 8 + 5 * 3));
    PH_COUNT(P, 18, 1)  // predict 7*2*8 + magnitude 5*3 per peek obs
    wsync();
    return all;
}

// Median over the k peek residuals of each band of the window whose residuals start at ring
// offset off (band-major ring PRES, written by eval_peek or ring_rows); returns band l's median in
// lane l (l < 7).
__device__ __forceinline__ double peek_medians(Px &P, int k, int off) {
    Lds *L = &LDS();
    const int l = lane();
    const int bnd = l & 7, osub = l >> 3;
    const int t1 = (k - 1) / 2, t2 = k / 2;
    const double *R = PRES(L) + bnd * PSTR + off;
    // observations past the LDS ring (k > 64: off is 0 then) are in the global overflow
    const int kl = k < PSTR - off ? k : PSTR - off;
    const GLOBAL_AS double *Ro = ring_ovf(P) + bnd * POVF - PSTR;
    for (int jj = osub; jj < k; jj += 8) {
        if (bnd >= NB) continue;
        const double v = jj < kl ? R[jj] : Ro[jj];
        int rank = 0;
        for (int i = 0; i < kl; ++i) {
            const double u = R[i];
            rank += (u < v || (u == v && i < jj)) ? 1 : 0;
        }
        for (int i = kl; i < k; ++i) {
            const double u = Ro[i];
            rank += (u < v || (u == v && i < jj)) ? 1 : 0;
        }
        if (rank == t1) L->med1[bnd] = v;
        if (rank == t2) L->med2[bnd] = v;
    }
    wsync();
    double out = 0.0;
    if (l < NB) out = (k & 1) ? L->med1[l] : (L->med1[l] + L->med2[l]) / 2.0;
    wsync();
    return out;
}

__device__ __forceinline__ void lookback(Px &P, int &wa, int &wb, int prev) {
    const ccdgpu_params &p = ARGS().p;
    const int l = lane();
    int a = wa, b = wb;
    if (l < NB) LDS().comp[l] = LDS().rmse[l];  // change.lookback: comparison rmse = model rmse
    wsync();
    while (a > prev) {
        int lo;
        if (a - prev > P.peek) lo = a - P.peek + 1;
        else if (a - P.peek <= 0) lo = 0;
        else lo = prev;
        const int k = a - lo;
        double m0;
        PH_BEGIN(ep)
        const bool change = eval_peek(P, k, a - 1, -1, m0);
        PH_END(P, ep, 8)
        if (change) break;
        if (m0 > p.outlier_threshold) {
            const int rm = a - 1;
            PH_BEGIN(cp)
            compact_drop(P, rm, rm + 1, [&](int j) { return j == rm; });
            PH_END(P, cp, 9)
            a -= 1;
            b -= 1;
            continue;
        }
        a -= 1;
    }
    wa = a;
    wb = b;
}

// find_closest_doy(period, ref, fit_window, 24) -> comparison rmse sqrt(sum r^2) / 4 per detection
// band.  The key |round(d / 365.25) * 365.25 - d| of d = t - t_ref is exactly min(r, 1461 - r) / 4
// with r = (4 t - 4 t_ref) mod 1461 (verified over all |d| <= 20000), so with u = 4 t mod 1461 the
// 24 closest observations are the entries of the bins within distance K of u_ref -- K the
// smallest distance holding 24 -- and, when the two bins at distance exactly K hold more entries
// than the 24 still need, the ones numpy's argsort puts first (qs_ties below).
//
// Per fit the window is counted into the 1461 bins (L->hist2, bin end positions: fit_bounds), and
// the comparison rmse is first bounded (comp_bound); only a step the bounds leave open gets the
// exact value (coop_comp), from bucket records -- the fit window's 16-byte period rows
// counting-sorted by u (build_buckets) -- so the entries closer than K are one circular run of
// bucket positions.
__device__ __forceinline__ int u1461(int t) { return (4 * t) % 1461; }
__device__ __forceinline__ unsigned det_mask() { return ARGS().p.detection_bands & 0x7Fu; }
// L->hist2 holds two u16 per word: plain counts (build_hist) or the end position of each bin in
// the bucket list (bins_prefix).
__device__ __forceinline__ int h16(const Lds *L, int u) { return (int)L->hist16[u]; }  // = hist2[u/2] half u%2
__device__ __forceinline__ int bend(const Lds *L, int u) { return h16(L, u); }
__device__ __forceinline__ int bstart(const Lds *L, int u) { return u == 0 ? 0 : h16(L, u - 1); }
__device__ __forceinline__ int bcount(const Lds *L, int u) { return bend(L, u) - bstart(L, u); }

__device__ __forceinline__ void build_hist(const Px &P, int fa, int fb) {
    Lds *L = &LDS();
    const int l = lane();
    for (int i = l; i < 732; i += W) L->hist2[i] = 0u;
    wsync();
    // (four chunks per round: the date loads go out together)
    for (int i0 = fa; i0 < fb; i0 += 4 * W) {
        int dt[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) dt[u] = i0 + u * W + l < fb ? CDR(P, i0 + u * W + l) : 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (i0 + u * W + l < fb) {
                const int b = u1461(dt[u]);
                atomicAdd(&L->hist2[b >> 1], 1u << ((b & 1) * 16));
            }
        }
    }
    wsync();
}

// 16-byte bucket records in the slot's global scratch (a native vector type: loads and stores
// through the address_space(1) pointer are single dwordx4 instructions)
typedef unsigned rec4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void rec_store(GLOBAL_AS double *fs, int pos, uint4 q) {
    reinterpret_cast<GLOBAL_AS rec4 *>(fs)[pos] = rec4{q.x, q.y, q.z, q.w};
}
__device__ __forceinline__ uint4 rec_load(const GLOBAL_AS double *fs, int pos) {
    const rec4 v = reinterpret_cast<const GLOBAL_AS rec4 *>(fs)[pos];
    return uint4{v.x, v.y, v.z, v.w};
}

// L->hist2 (bin counts of build_hist) -> bin start positions (ends = false: the cursors of a
// counting-sort fill, which leaves the ends) or bin end positions (ends = true).  Lane l owns
// words [12 l, 12 l + 12) (24 bins; 732 = 61 lanes x 12).
__device__ __forceinline__ void bins_prefix(bool ends) {
    Lds *L = &LDS();
    const int l = lane();
    unsigned hv[12];
    const bool hl = l < 61;
#pragma unroll
    for (int i = 0; i < 12; ++i) hv[i] = hl ? L->hist2[12 * l + i] : 0u;
    int tot = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) tot += (int)(hv[i] & 0xFFFFu) + (int)(hv[i] >> 16);
    int run = wscan_incl(tot) - tot;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const int s0 = run;
        const int s1 = run + (int)(hv[i] & 0xFFFFu);
        run = s1 + (int)(hv[i] >> 16);
        if (hl) L->hist2[12 * l + i] = ends ? ((unsigned)s1 | ((unsigned)run << 16)) : ((unsigned)s0 | ((unsigned)s1 << 16));
    }
    wsync();
}

// Counting sort of the fit window [fa, fb) by u = 4 t mod 1461 (L->hist2: bin end positions
// afterwards) into bucket records: P.fs viewed as 16-byte rows, record pos = the period row (7
// band values + sorted index) of the pos-th entry in bucket order.  The records depend on the fit
// window's rows only, not on the model: a step that needs its comparison rmse recomputes the
// residuals of its 24 entries from them (coop_comp), so a refit writes 16 B per fit observation
// instead of the squared residuals of every detection band (40 B) and computes no residuals --
// and only when some step of its batches needs the exact comparison rmse.  Removals after the
// window (lookforward outliers) leave the window's rows as they are.
__device__ __forceinline__ void build_buckets(const Px &P, int fa, int fb) {
    Lds *L = &LDS();
    const int l = lane();
    const int nf = fb - fa;
    build_hist(P, fa, fb);
    bins_prefix(false);
    // four chunks per round: the row and date loads go out together, then the bin cursors
    constexpr int U = 4;
    for (int i0 = fa; i0 < fb; i0 += U * W) {
        uint4 q[U];
        int dt[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * W + l;
            q[u] = uint4{0u, 0u, 0u, 0u};
            dt[u] = 0;
            if (i < fb) {
                q[u] = CROW4(P, i);
                dt[u] = CDR(P, i);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * W + l;
            if (i < fb) {
                const int ub = u1461(dt[u]);
                const unsigned old = atomicAdd(&L->hist2[ub >> 1], 1u << ((ub & 1) * 16));
                rec_store(PFS(P), gidx(P, (int)((old >> ((ub & 1) * 16)) & 0xFFFFu), nf, __LINE__), q[u]);
            }
        }
    }
    gsync();  // the records are read by other lanes
}

// Per fit (lookforward, more than 24 fit observations), once it is needed: lasso.fitted_model's
// rmse of the current models over the fit window [fa, fb) -- lane l sums observations fa + l,
// fa + l + 64, ... in order, then one wave sum: the order of round 4's bucket build, so the emitted
// rmse of these fits is unchanged since then -- and, from the same residuals, the comparison-rmse bounds of
// the batched steps: the window's bin end positions (L->hist2) and per block of 46 bins the sum
// of its squared residuals per detection band (L->blk, float, every term rounded up).
__device__ __forceinline__ void fit_bounds(const Px &P, int fa, int fb, int k) {
    Lds *L = &LDS();
    const int l = lane();
    const int nf = fb - fa;
    const unsigned dm = det_mask();
    // the bin counts (L->hist2) are gathered in the residual pass (one pass over the window's
    // dates, not two) and turned into bin ends after it
    for (int i = l; i < 732; i += W) L->hist2[i] = 0u;
    float *bz = &L->blk[0][0];
    for (int i = l; i < 32 * 8; i += W) bz[i] = 0.0f;
    wsync();
    double ssq[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) ssq[b] = 0.0;
    // FU chunks per round, software-pipelined: the next round's rows and dates load while this
    // round's design rows load (lane l still adds fa + l, fa + l + 64, ... in order); one or three
    // chunks per round measured slower
    constexpr int FU = 2;
    uint4 qn[FU];
    int dn[FU];
#pragma unroll
    for (int u = 0; u < FU; ++u) {
        const int i = fa + u * W + l;
        qn[u] = uint4{0u, 0u, 0u, 0u};
        dn[u] = 0;
        if (i < fb) {
            qn[u] = CROW4(P, i);
            dn[u] = CDR(P, i);
        }
    }
    for (int i0 = fa; i0 < fb; i0 += FU * W) {
        uint4 qv[FU];
        int dt[FU];
        double xv[FU][7];
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            qv[u] = qn[u];
            dt[u] = dn[u];
        }
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const int i = i0 + u * W + l;
            const GLOBAL_AS double *bs = P.basis + (size_t)gidx(P, i < fb ? (int)(qv[u].w >> 16) : 0, P.n, __LINE__) * CCD_BASIS_STRIDE;
#pragma unroll
            for (int c = 0; c < 7; ++c) xv[u][c] = bs[c];
        }
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const int i = i0 + (FU + u) * W + l;
            qn[u] = uint4{0u, 0u, 0u, 0u};
            dn[u] = 0;
            if (i < fb) {
                qn[u] = CROW4(P, i);
                dn[u] = CDR(P, i);
            }
        }
#pragma unroll
        for (int u = 0; u < FU; ++u) {
            const int i = i0 + u * W + l;
            if (i >= fb) continue;
            const int ub = u1461(dt[u]);
            const int blk = ub / 46;
            atomicAdd(&L->hist2[ub >> 1], 1u << ((ub & 1) * 16));
            const double *x = xv[u];
            const unsigned qw[4] = {qv[u].x, qv[u].y, qv[u].z, qv[u].w};
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                const double *c = L->coef[b];
                double pr = x[0] * c[0];
#pragma unroll
                for (int jj = 1; jj < 7; ++jj) pr += x[jj] * c[jj];
                pr += c[7];
                const double y = (double)(int16_t)(qw[b >> 1] >> ((b & 1) * 16));
                const double r = y - pr;
                ssq[b] += r * r;
                if ((dm >> b) & 1u) {
                // r^2 rounded up to float without a rounding-mode switch: the nearest float, one
                // ulp up when below (r^2 >= 0; NaN / inf pass through)
                const double r2 = r * r;
                float f = (float)r2;
                f = (double)f < r2 ? __int_as_float(__float_as_int(f) + 1) : f;
                atomicAdd(&L->blk[blk][b], f);
            }
            }
        }
    }
    wsync();
    bins_prefix(true);
    // per band, the block sums -> their inclusive prefix over the 32 blocks (two bands a pass,
    // one per 32-lane half; float, the rounding is covered in comp_bound)
#pragma unroll
    for (int b2 = 0; b2 < NB; b2 += 2) {
        const int b = b2 + (l >> 5), g = l & 31;
        float v = b < NB ? L->blk[g][b] : 0.0f;
        v = fscan32(v);
        if (b < NB) L->blk[g][b] = v;
    }
    const double den = (double)(nf - (ARGS().p.rmse_dof ? k : 0));
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        const double t = wsum(ssq[b]);
        if (l == b) L->rmse[b] = sqrt(t / den);
    }
    wsync();
}

// ---- the reference's argsort tie order at distance K (change.find_closest_doy)
// np.argsort(d_yr)[:24] with numpy's default quicksort as the pinned reference image ran it (numpy
// < 1.17 aquicksort, restated and pinned against a real numpy build in oracle/ccd_oracle.c
// ccdoracle_np_argsort): its tie order decides WHICH of the entries at exactly distance K enter
// the comparison rmse when the two bins at K hold more entries than the 24 still need.  That
// order depends on the whole sort, so the wave replays it on the fit window's keys -- element
// key << 12 | sorted index in fit-window order (the order np.argsort sees), in the slot's scratch
// after the bucket records -- partitioning only the parts that overlap positions [less, 24), the
// ones whose content is wanted (parts are disjoint ranges permuted within themselves, so the
// others do not matter).  A partition (median of three parked at pr - 1, Sedgewick's scans that
// stop on keys equal to the pivot) is computed in parallel: with S the positions in (pl, pr - 1]
// whose key is >= the pivot (ascending, s_k) and T those in [pl, pr - 2] whose key is <= it
// (descending, t_k), the sequential scans swap s_k <-> t_k for every k with s_k < t_k (a prefix
// of k: K1 pairs) and stop at pi = min(s_{K1+1}, t_{K1}) -- the scans only ever meet untouched
// positions before that -- then pi <-> pr - 1.  Parts of <= 16 entries are insertion-sorted
// (= stably by key).  Returns in lane j < 24 - less the sorted index of the entry numpy puts at
// position less + j (the taken ties), -1 elsewhere.  Only steps whose exact comparison rmse is
// needed AND whose ties straddle the 24th position get here.
__device__ __forceinline__ unsigned qkey(unsigned x) { return x >> 12; }
__device__ __forceinline__ int qs_ties(const Px &P, int fa, int nf, int dref, int less) {
    Lds *L = &LDS();
    const int l = lane();
    GLOBAL_AS uint32_t *A = reinterpret_cast<GLOBAL_AS uint32_t *>(PFS(P) + 2 * (size_t)P.n);
    GLOBAL_AS uint16_t *MS = reinterpret_cast<GLOBAL_AS uint16_t *>(A + P.n);  // s_k by k - 1
    const int ur = u1461(dref);
    for (int i0 = 0; i0 < nf; i0 += W) {
        const int i = i0 + l;
        if (i < nf) {
            int r = u1461(CDR(P, fa + i)) - ur;
            r += r < 0 ? 1461 : 0;
            const int key = r < 1461 - r ? r : 1461 - r;
            A[i] = ((unsigned)key << 12) | (unsigned)CIR(P, fa + i);
        }
    }
    gsync();
    const int lo = less, hi = 24;  // positions whose content is wanted
    int sp = 0;                    // pending parts: L->sel as pl | pr << 16
    int pl = 0, pr = nf - 1;
    for (;;) {
        while (pr - pl > 15) {
            const int pm = pl + ((pr - pl) >> 1);
            unsigned a0 = (unsigned)uni((int)A[pl]), am = (unsigned)uni((int)A[pm]);
            unsigned ar = (unsigned)uni((int)A[pr]);
            const unsigned ap = (unsigned)uni((int)A[pr - 1]);
            unsigned t;
            if (qkey(am) < qkey(a0)) { t = am; am = a0; a0 = t; }
            if (qkey(ar) < qkey(am)) { t = ar; ar = am; am = t; }
            if (qkey(am) < qkey(a0)) { t = am; am = a0; a0 = t; }
            const unsigned vp = qkey(am);
            if (l == 0) {  // median of three in place, the pivot parked at pr - 1
                A[pl] = a0;
                A[pr] = ar;
                A[pm] = ap;
                A[pr - 1] = am;
            }
            gsync();
            int nT = 0;  // T: positions in [pl, pr - 2] with key <= pivot
            for (int p0 = pl; p0 <= pr - 2; p0 += W) {
                const int q = p0 + l;
                const bool in = q <= pr - 2 && qkey(A[q]) <= vp;
                nT += popc(bal(in));
            }
            // S ascending: s_k (k = rank) swaps with t_k while t_k > s_k, i.e. while more than
            // k - 1 positions of T lie past s_k; the first S position failing that is s_{K1+1}
            int cS = 0, cT = 0, K1 = -1, sfail = pr - 1;
            for (int p0 = pl; p0 <= pr - 1 && K1 < 0; p0 += W) {
                const int q = p0 + l;
                const unsigned x = q <= pr - 1 ? A[q] : 0u;
                const unsigned kx = qkey(x);
                const bool inS = q >= pl + 1 && q <= pr - 1 && kx >= vp;
                const bool inT = q <= pr - 2 && kx <= vp;
                const unsigned long long bS = bal(inS), bT = bal(inT);
                const int rs = cS + below(bS) + 1;
                const int tgt = nT - (cT + below(bT) + (inT ? 1 : 0));  // T positions past q
                const bool ok = inS && tgt >= rs;
                if (ok) MS[gidx(P, rs - 1, P.n, __LINE__)] = (uint16_t)q;
                const unsigned long long bF = bal(inS && !ok);
                if (bF) {
                    const int f = __ffsll((long long)bF) - 1;
                    sfail = p0 + f;
                    K1 = rdl(rs, f) - 1;
                }
                cS += popc(bS);
                cT += popc(bT);
            }
            K1 = K1 < 0 ? 0 : K1;  // (pr - 1 holds the pivot: it always fails)
            // T descending: t_k (k = rank from the right) <-> s_k for k <= K1
            int tK = pr - 1;
            if (K1 > 0) {
                gsync();  // MS
                int cR = 0;
                for (int p1 = pr - 2; p1 >= pl && cR < K1; p1 -= W) {
                    const int q = p1 - l;  // lane 0 rightmost
                    const unsigned x = q >= pl ? A[q] : 0u;
                    const bool inT = q >= pl && qkey(x) <= vp;
                    const unsigned long long bT = bal(inT);
                    const int rt = cR + below(bT) + 1;
                    if (inT && rt <= K1) {
                        const int sq = gidx(P, (int)MS[gidx(P, rt - 1, P.n, __LINE__)], nf, __LINE__);
                        const unsigned xs = A[sq];
                        A[sq] = x;
                        A[q] = xs;
                    }
                    const unsigned long long bK = bal(inT && rt == K1);
                    if (bK) tK = p1 - (__ffsll((long long)bK) - 1);
                    cR += popc(bT);
                }
            }
            gsync();
            const int pi = K1 > 0 && tK < sfail ? tK : sfail;
            {
                const unsigned xpi = (unsigned)uni((int)A[pi]), xp1 = (unsigned)uni((int)A[pr - 1]);
                if (l == 0) {
                    A[pi] = xp1;
                    A[pr - 1] = xpi;
                }
                gsync();
            }
            // the parts that overlap [lo, hi): continue with one, keep the other
            const bool rl = pl < hi && pi - 1 >= lo && pi - 1 >= pl;
            const bool rr = pi + 1 < hi && pr >= lo && pr >= pi + 1;
            if (rl && rr) {
                if (l == 0) L->sel[sp < 31 ? sp : 31] = (pi + 1) | (pr << 16);
                sp += 1;
                pr = pi - 1;
            } else if (rl) {
                pr = pi - 1;
            } else if (rr) {
                pl = pi + 1;
            } else {
                pl = 1;
                pr = 0;
                break;
            }
        }
        if (pr >= pl) {  // insertion sort of a part of <= 16 entries: stable by key
            const int cnt = pr - pl + 1;
            const unsigned x = l < cnt ? A[pl + l] : 0xFFFFFFFFu;
            const unsigned kx = qkey(x);
            int pos = 0;
            for (int j = 0; j < cnt; ++j) {
                const unsigned kj = qkey((unsigned)rdl((int)x, j));
                pos += (kj < kx || (kj == kx && j < l)) ? 1 : 0;
            }
            if (l < cnt) A[pl + pos] = x;
            gsync();
        }
        if (sp == 0) break;
        sp -= 1;
        wsync();
        const int e = uni(L->sel[sp < 31 ? sp : 31]);
        pl = e & 0xFFFF;
        pr = e >> 16;
    }
    const int need = hi - lo;
    return l < need ? (int)(A[lo + l] & 0xFFFu) : -1;
}

// find_closest_doy comparison rmse of ONE batched step (reference date dref) from the bucket
// records, the whole wave working on it: the distance K of the 24th closest entry by a scan over
// the bin ends, then lane = entry -- the circular run of bucket positions
// closer than K and the entries at exactly K (when more are there than needed: the ones numpy's
// quicksort puts first, qs_ties; with argsort_stable the lowest sorted indices -- sorted index
// order is fit-window order) -- each taken lane recomputes its residuals of the detection bands
// from its record and design row (resid_at's arithmetic) and the squares are summed over the
// wave.  Returns sqrt(sum) / 4 of the s-th detection band in out[s] (every lane).  Fit window
// [fa, fa + nf), nf > 24.
__device__ __forceinline__ void coop_comp(const Px &P, int fa, int nf, int dref, const int (&bs)[NB], int nd,
                                          double (&out)[NB]) {
    const unsigned dm = det_mask();
    const Lds *L = &LDS();
    const int l = lane();
    const int u = u1461(dref);
    int K = 0, less = 0;
    {
        int carry = 0;
        for (int base = 0; base <= 730; base += W) {
            const int dd = base + l;
            int c = 0;
            if (dd == 0) c = bcount(L, u);
            else if (dd <= 730) c = bcount(L, (u + dd) % 1461) + bcount(L, (u - dd + 1461) % 1461);
            const int cum = wscan_incl(c) + carry;
            const unsigned long long hit = bal(cum >= 24);
            if (hit) {
                const int src = __ffsll((long long)hit) - 1;
                K = base + src;
                less = rdl(cum, src) - rdl(c, src);
                break;
            }
            carry = rdl(cum, W - 1);
        }
    }
    const int need = 24 - less;
    const int s0 = K > 0 ? bstart(L, (u - K + 1 + 1461) % 1461) : 0;
    const int b1 = (u - K + 1461) % 1461, b2 = (u + K) % 1461;
    const int c1 = bcount(L, b1), c2 = K > 0 ? bcount(L, b2) : 0;
    const int st1 = bstart(L, b1), st2 = bstart(L, b2);
    const int T = c1 + c2, E = less + T;
    // numpy's choice among the ties (lane j < need: the sorted index of the j-th one taken)
    const bool qs = T > need && !ARGS().p.argsort_stable;
    const int tk = qs ? qs_ties(P, fa, nf, dref, less) : -1;
    PH_COUNT(P, 22, E > W ? 1 : 0)     // (diagnostic build) selections of more entries than a wave
    PH_COUNT(P, 23, T > need ? 1 : 0)  // ... and with more ties at the cut-off than still needed
    double acc[NB];  // per band (detection bands only)
#pragma unroll
    for (int b = 0; b < NB; ++b) acc[b] = 0.0;
    for (int e0 = 0; e0 < E; e0 += W) {
        const int e = e0 + l;
        const bool tie = e >= less && e < E;
        int pos = 0;
        if (e < less) {
            pos = s0 + e;
            pos = pos >= nf ? pos - nf : pos;
        } else if (tie) {
            const int te = e - less;
            pos = te < c1 ? st1 + te : st2 + (te - c1);
        }
        uint4 q = uint4{0u, 0u, 0u, 0u};
        if (e < E) q = rec_load(PFS(P), gidx(P, pos, nf, __LINE__));
        const int ci = (int)(q.w >> 16);
        bool take = e < E;
        if (qs) {
            // more entries at distance K than needed: a tie entry is taken when numpy's argsort
            // puts it among the first 24
            bool in = false;
            for (int j = 0; j < need; ++j) {
                const int cj = rdl(tk, j);  // (full EXEC: no short-circuit around the readlane)
                in = in | (cj == ci);
            }
            if (tie) take = in;
        } else if (T > need) {
            // (argsort_stable) a tie entry is taken when fewer than `need` of them have a
            // smaller sorted index
            int rank = 0;
            if (E <= W) {
                for (int f = 0; f < T; ++f) rank += rdl(ci, less + f) < ci ? 1 : 0;
            } else {
                for (int f = 0; f < T; ++f) {
                    const int fp = f < c1 ? st1 + f : st2 + (f - c1);
                    rank += (int)(rec_load(PFS(P), gidx(P, fp, nf, __LINE__)).w >> 16) < ci ? 1 : 0;
                }
            }
            if (tie) take = rank < need;
        }
        if (take) {
            const GLOBAL_AS double *bsr = P.basis + (size_t)gidx(P, ci, P.n, __LINE__) * CCD_BASIS_STRIDE;
            double x[7];
#pragma unroll
            for (int c = 0; c < 7; ++c) x[c] = bsr[c];
            const unsigned qw[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if ((dm >> b) & 1u) {
                    const double *c = L->coef[b];
                    double pr = x[0] * c[0];
#pragma unroll
                    for (int jj = 1; jj < 7; ++jj) pr += x[jj] * c[jj];
                    pr += c[7];
                    const double y = (double)(int16_t)(qw[b >> 1] >> ((b & 1) * 16));
                    const double r = y - pr;
                    acc[b] += r * r;
                }
            }
        }
    }
    double sb[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) sb[b] = ((dm >> b) & 1u) ? wsum(acc[b]) : 0.0;
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        double v = 0.0;
#pragma unroll
        for (int b = 0; b < NB; ++b) v = bs[t] == b ? sb[b] : v;
        out[t] = t < nd ? sqrt(v) / 4.0 : 0.0;
    }
}

// comparison rmse of a fit window of <= 24 observations (all of them: find_closest_doy(...)[:24]
// takes every one) into L->comp, for every band
__device__ __forceinline__ void closest_doy_scan(Px &P, int fa, int fb) {
    Lds *L = &LDS();
    const int l = lane();
    const int nf = fb - fa;  // <= 24: every fit observation is among its "24 closest"
    const int bnd = l >> 3, osub = l & 7;  // band-major: a band's 8 partial sums share a DPP row
    // three fixed rounds of 8 observations, unrolled so the row / basis gathers of all three are
    // in flight together
    double e[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int s2 = osub + 8 * r;
        e[r] = (bnd < NB && s2 < nf) ? resid_at(P, bnd, fa + s2) : 0.0;
    }
    double ss = e[0] * e[0];
    ss += e[1] * e[1];
    ss += e[2] * e[2];
    ss = gsum8(ss);
    if (osub == 0 && bnd < NB) L->comp[bnd] = sqrt(ss) / 4.0;
    wsync();
}


// Residuals of the current models at compacted positions x0 .. x0 + 63 (lane = position) into
// the band-major ring PRES (same arithmetic as resid_at).
__device__ __forceinline__ void ring_rows(const Px &P, int x0) {
    Lds *L = &LDS();
    const int l = lane();
    const int j = x0 + l;
    double *R = PRES(L) + l;
    if (j < P.m) {
        const CRow cw = CROW(P, j);
        const GLOBAL_AS double *bs = P.basis + (size_t)cw.ci * CCD_BASIS_STRIDE;
        double x[7];
#pragma unroll
        for (int c = 0; c < 7; ++c) x[c] = bs[c];
#pragma unroll
        for (int bd = 0; bd < NB; ++bd) {
            const double *c = L->coef[bd];
            double pr = x[0] * c[0];
#pragma unroll
            for (int jj = 1; jj < 7; ++jj) pr += x[jj] * c[jj];
            pr += c[7];
            R[bd * PSTR] = (double)cw.v[bd] - pr;
        }
    }
    wsync();
}

// Entries of the fit window whose closest-DOY bin lies within circular distance d of bin u
// (L->hist2 = bin end positions after fit_bounds / build_buckets).
__device__ __forceinline__ int cnt_within(const Lds *L, int nf, int u, int d) {
    // bins [u - d, u + d] (circular; 2 d + 1 < 1461 so at most one end wraps)
    int lo = u - d;
    lo += lo < 0 ? 1461 : 0;
    int hi = u + d;
    hi -= hi > 1460 ? 1461 : 0;
    const int eh = bend(L, hi);
    const int el = bend(L, lo > 0 ? lo - 1 : 0);
    const int c = eh - (lo > 0 ? el : 0) + (lo > hi ? nf : 0);
    return d >= 730 ? nf : c;
}

// Upper bound of the closest-DOY comparison rmse of the step with reference date dref, per
// detection band (slot order of bs), from fit_bounds' bins and blocks (per lane, nf > 24): the 24
// closest entries lie within distance K of u (K: the smallest distance holding 24, from the bin
// ends), so within the blocks that bins [u - K, u + K] touch.  Their float block sums are each at
// most (n 2^-24) below the exact sum of the rounded-up terms, which bound the squares from above;
// inflated by 2^-9 they bound the exact -- and any computed -- sum of any 24 of them.
// (the slack below -- 2^-10 of the total for the float prefixes, 2^-9 for the float block sums of
// rounded-up terms -- covers at most 4096 terms per sum: CCDGPU_MAX_OBS)
static_assert(CCDGPU_MAX_OBS <= 4096, "comp_bound / fit_bounds float slack sized for <= 4096 fit observations");
__device__ __forceinline__ void comp_bound(int nf, int dref, const int (&bs)[NB], int nd, double (&cb)[NB]) {
    const Lds *L = &LDS();
    const int u = u1461(dref);
    int lo = 0, hi = 730;  // smallest K with cnt_within(K) >= 24
#pragma unroll
    for (int it = 0; it < 10; ++it) {
        const int mid = (lo + hi) >> 1;
        const bool ge = cnt_within(L, nf, u, mid) >= 24;
        const bool act = lo < hi;
        hi = act && ge ? mid : hi;
        lo = act && !ge ? mid + 1 : lo;
    }
    const int K = lo;
    // blocks of bins [u - K, u + K] (circular): one or two ascending block ranges
    int b0 = 0, b1 = 31, c0 = 1, c1 = 0;  // ranges [b0, b1] and [c0, c1] (c0 > c1: none)
    if (2 * K + 1 < 1461) {
        const int x0 = u - K, x1 = u + K;
        if (x0 < 0) {
            b0 = (x0 + 1461) / 46; b1 = 31; c0 = 0; c1 = x1 / 46;
        } else if (x1 > 1460) {
            b0 = x0 / 46; b1 = 31; c0 = 0; c1 = (x1 - 1461) / 46;
        } else {
            b0 = x0 / 46; b1 = x1 / 46;
        }
    }
    // L->blk holds per band the inclusive prefix over the blocks (fit_bounds): a range is two
    // reads; the prefixes' float rounding (< 2.5e-4 of the total for <= 4096 terms) is covered by
    // 2^-10 of the total
#pragma unroll
    for (int t = 0; t < NB; ++t) {
        double sd = 0.0;
        if (t < nd) {
            const int b = bs[t];
            const double tot = (double)L->blk[31][b];
            sd = (double)L->blk[b1][b] - (b0 > 0 ? (double)L->blk[b0 - 1][b] : 0.0);
            if (c0 <= c1) sd += (double)L->blk[c1][b] - (c0 > 0 ? (double)L->blk[c0 - 1][b] : 0.0);
            sd += 0x1p-10 * tot;
        }
        cb[t] = sqrt(sd * (1.0 + 0x1p-9)) / 4.0;
    }
}

// change.lookforward.  The first steps (no model yet, or fewer than 24 observations in the
// window) refit every step and run one at a time.  After that the model changes only at a refit
// (window span >= 1.33 x the fitted span), so the steps between refits are evaluated in batches,
// lane = step: a step at window start x uses the peek observations x .. x + k - 1 and the
// reference date of x + k - 1.  Only the first peek observation can be removed (outlier), so in
// the batch's own indexing every step's window is consecutive and the step sequence is fixed:
// step x removes x (outlier) or advances past it, and the batch ends at the first step that
// needs a refit (span test on the last kept observation before it) or detects a change.
// Removals are applied in one compaction pass per batch.
// ---- speculative early fits
// An early lookforward step (no model yet, or fewer than 24 observations in the window) refits
// the window [a, b) every step, and the next steps' windows are [a, b + 1), [a, b + 2), ... as
// long as no outlier is removed (removals are rare).  spec_fits fits up to 8 of these windows at
// once: lane = (window v, band), each lane one whole Lasso (models/lasso.py = sklearn 0.18
// coordinate descent, gradient form as in cd_lanes) on its own centred Gram held in registers,
// and its rmse from its own residuals (same arithmetic as resid_at).  The replay in lookforward
// then walks the steps one by one, installing window v's models when step v needs them.
constexpr int SPEC_PC = 5;  // design columns of a <= 6-coefficient model (windows < 24 obs)
struct SpecFit {
    double w[SPEC_PC];  // coefficients of t, cos wt, sin wt, cos 2wt, sin 2wt
    double c;           // intercept (original coordinates, sklearn: ym - xm . w)
    double rmse;
    int sweeps;
};

// index of (i, j), i <= j, in a row-major upper triangle of SPEC_PC columns
__host__ __device__ constexpr int ut(int i, int j) { return i * SPEC_PC - i * (i - 1) / 2 + (j - i); }

__device__ __forceinline__ void spec_fits(Px &P, int a, int nw0, int V, SpecFit &F) {
    const ccdgpu_params &p = ARGS().p;
    Lds *L = &LDS();
    const int l = lane();
    const int v = l >> 3, band = l & 7;
    const bool act = band < NB && v < V;
    const int nv = nw0 + v;       // rows of this lane's window
    const int R = nw0 + V - 1;    // rows staged (<= 23 < TR)
    const int t0 = CDRU(P, a);
    const CRow c0 = CROW(P, a);   // value shifts: the window's first observation
    if (l < R) {
        const CRow cw = CROW(P, a + l);
        const GLOBAL_AS double *bs = P.basis + (size_t)cw.ci * CCD_BASIS_STRIDE;
        double *r = L->row[l];
        r[0] = bs[0] - (double)t0;
#pragma unroll
        for (int c = 1; c < SPEC_PC; ++c) r[c] = bs[c];
#pragma unroll
        for (int bd = 0; bd < NB; ++bd) r[8 + bd] = (double)((int)cw.v[bd] - (int)c0.v[bd]);
    }
    wsync();
    const int yb = band < NB ? band : 0;
    const int y0 = (int)c0.v[yb];
    // raw sums of the lane's window in shifted coordinates (exact integer shifts)
    double sx[SPEC_PC], sxy[SPEC_PC], sxx[ut(SPEC_PC - 1, SPEC_PC - 1) + 1];
    double sy = 0.0, syy = 0.0;
#pragma unroll
    for (int i = 0; i < SPEC_PC; ++i) sx[i] = sxy[i] = 0.0;
#pragma unroll
    for (int e = 0; e < ut(SPEC_PC - 1, SPEC_PC - 1) + 1; ++e) sxx[e] = 0.0;
    const int nrow = act ? nv : 0;
    for (int r = 0; r < nrow; ++r) {
        const double *row = L->row[r];
        double x[SPEC_PC];
#pragma unroll
        for (int i = 0; i < SPEC_PC; ++i) x[i] = row[i];
        const double y = row[8 + yb];
        sy += y;
        syy += y * y;
#pragma unroll
        for (int i = 0; i < SPEC_PC; ++i) {
            sx[i] += x[i];
            sxy[i] += x[i] * y;
#pragma unroll
            for (int j = i; j < SPEC_PC; ++j) sxx[ut(i, j)] += x[i] * x[j];
        }
    }
    // centred Gram / X'y / y'y (sklearn centres X and y) and the coordinate descent
    const double n = act ? (double)nv : 1.0;
    double G[ut(SPEC_PC - 1, SPEC_PC - 1) + 1], q[SPEC_PC];
#pragma unroll
    for (int i = 0; i < SPEC_PC; ++i) {
        q[i] = sxy[i] - sx[i] * (sy / n);
#pragma unroll
        for (int j = i; j < SPEC_PC; ++j) G[ut(i, j)] = sxx[ut(i, j)] - sx[i] * (sx[j] / n);
    }
    const double yy = syy - sy * (sy / n);
    const int kc = num_coefs(p, nv);
    const int pc = kc - 1;
    const double alpha = p.lasso_alpha * (double)nv;
    const double tol = p.lasso_tol, tol_s = tol * yy;
    const int max_iter = p.lasso_max_iter;
    // h_i = g_i + G_ii w_i (sklearn's tmp for coordinate i), as in cd_coord: a change of w_i moves
    // every other h_m by -G_mi d and leaves h_i as it is
    double rg[SPEC_PC], w[SPEC_PC], h[SPEC_PC];
    bool can[SPEC_PC];
#pragma unroll
    for (int i = 0; i < SPEC_PC; ++i) {
        const double gd = G[ut(i, i)];
        rg[i] = gd != 0.0 ? 1.0 / gd : 0.0;
        can[i] = act && i < pc && gd != 0.0;  // sklearn skips zero-norm columns
        w[i] = 0.0;
        h[i] = q[i];
    }
    const bool any5 = bal(act && pc > 3) != 0ull;
    bool done = !act;
    int sweeps = max_iter;
#ifdef CCD_PHASE_TIMERS
    int wave_sweeps = max_iter;
#endif
    for (int it = 0; it < max_iter; ++it) {
        if (bal(!done) == 0ull) {
#ifdef CCD_PHASE_TIMERS
            wave_sweeps = it;
#endif
            break;
        }
        double dmax = 0.0;
#pragma unroll
        for (int i = 0; i < SPEC_PC; ++i) {
            if (i >= 3 && !any5) break;
            const double wn = copysign(fmax(fabs(h[i]) - alpha, 0.0), h[i]) * rg[i];
            const bool upd = !done && can[i];
            const double wnew = upd ? wn : w[i];
            const double d = wnew - w[i];
            w[i] = wnew;
            dmax = fmax(dmax, fabs(d));
#pragma unroll
            for (int m = 0; m < SPEC_PC; ++m)
                if (m != i) h[m] -= G[m < i ? ut(m, i) : ut(i, m)] * d;
        }
        double wmax = 0.0;
#pragma unroll
        for (int i = 0; i < SPEC_PC; ++i) wmax = fmax(wmax, fabs(w[i]));  // w = 0 past pc
        const bool ratio_lt = dmax / wmax < tol;  // (wmax = 0: the check's first clause)
        const bool check = !done && (wmax == 0.0 || ratio_lt || it == max_iter - 1);
        if (bal(check)) {
            double dual = 0.0, wq = 0.0, wxta = 0.0, l1 = 0.0;
#pragma unroll
            for (int i = 0; i < SPEC_PC; ++i) {
                const double g = h[i] - G[ut(i, i)] * w[i];  // X_i . R
                if (i < pc) dual = fmax(dual, fabs(g));
                wq += w[i] * q[i];
                wxta += w[i] * g;
                l1 += fabs(w[i]);
            }
            const double ry = yy - wq, rr = ry - wxta;
            double cst, gap;
            if (dual > alpha) {
                cst = alpha / dual;
                gap = 0.5 * (rr + rr * cst * cst);
            } else {
                cst = 1.0;
                gap = rr;
            }
            gap += alpha * l1 - cst * ry;
            if (check && gap < tol_s) {
                done = true;
                sweeps = it + 1;
            }
        }
    }
    // intercept in original coordinates (means as gram_finalize forms them) and the rmse
    double dot = (sx[0] + n * (double)t0) / n * w[0];
#pragma unroll
    for (int i = 1; i < SPEC_PC; ++i) dot += sx[i] / n * w[i];
    const double c = (sy + n * (double)y0) / n - dot;
    double ss = 0.0;
    for (int r = 0; r < nrow; ++r) {
        const double *row = L->row[r];
        double pr = (row[0] + (double)t0) * w[0];
#pragma unroll
        for (int i = 1; i < SPEC_PC; ++i) pr += row[i] * w[i];
        pr += c;
        const double res = (row[8 + yb] + (double)y0) - pr;
        ss += res * res;
    }
    wsync();  // the row tile is free again (the replay's peek residuals go there)
#ifdef CCD_PHASE_TIMERS
    {
        int ls = act ? sweeps : 0;  // lane sweeps summed over the active lanes
        for (int o = 32; o > 0; o >>= 1) ls += shfx(ls, o);
        PH_COUNT(P, 35, 1)
        PH_COUNT(P, 36, V)
        PH_COUNT(P, 38, wave_sweeps)
        PH_COUNT(P, 39, ls)
    }
#endif
#pragma unroll
    for (int i = 0; i < SPEC_PC; ++i) F.w[i] = w[i];
    F.c = c;
    F.rmse = sqrt(ss / (double)(nv - (p.rmse_dof ? kc : 0)));
    F.sweeps = sweeps;
}

// Models of speculative window s (lanes (s, band)) into the model slots of LDS; comp = rmse.
__device__ __forceinline__ void spec_install(Px &P, const SpecFit &F, int s, int nw, int kc) {
    Lds *L = &LDS();
    const int l = lane();
    const int v = l >> 3, band = l & 7;
    if (v == s && band < NB) {
#pragma unroll
        for (int i = 0; i < SPEC_PC; ++i) L->coef[band][i] = F.w[i];
        L->coef[band][5] = 0.0;
        L->coef[band][6] = 0.0;
        L->coef[band][7] = F.c;
        L->rmse[band] = F.rmse;
        L->comp[band] = F.rmse;
        stat_lane(ST_SWEEPS, (unsigned long long)F.sweeps);
        stat_lane(ST_FLOPS, (unsigned long long)F.sweeps * (unsigned long long)(2 * kc * kc + 6 * kc));
    }
    stat_uniform(ST_FITS, NB);
    stat_uniform(ST_FLOPS, (unsigned long long)nw * (unsigned long long)(kc * (kc + 1) + 14 * kc + 7 * (2 * kc + 3)));
    P.fit_k = 0;  // L->coef no longer describes the accumulated Gram window
    PH_COUNT(P, 19, 1)
    wsync();
}

// change_magnitude of the batched steps' peek observations (lane = step, ring PRES): allc =
// every peek observation's magnitude exceeds the change threshold, outj = the first one's exceeds
// the outlier threshold.  ND = number of detection bands read (5 for the default bands: the rows
// past them would add 0).  One peek observation per round: its ND ring reads go out together.
// The lane's ring address is re-derived every round (lane() is opaque), so no per-lane address
// stays live across the loop for the allocator to spill -- a spilled one cost a scratch reload
// and a full wait before every read.
template <int ND>
__device__ __forceinline__ void peek_mags(const int (&bs)[NB], const double (&irm)[NB], int k, bool &allc,
                                          bool &outj) {
    Lds *L = &LDS();
    allc = true;
    for (int j = 0; j < k; ++j) {
        const double *Rj = PRES(L) + lane() + j;
        double rv[ND];
#pragma unroll
        for (int t = 0; t < ND; ++t) rv[t] = Rj[bs[t] * PSTR];
        double mg = 0.0;
#pragma unroll
        for (int t = 0; t < ND; ++t) {
            const double v = rv[t] * irm[t];
            mg += v * v;
        }
        allc = allc && mg > L->chg;
        if (j == 0) outj = mg > ARGS().p.outlier_threshold;
        // the remaining peek observations decide nothing once no lane can still detect a change
        // (outj is fixed at j = 0; the ring keeps every residual for the medians)
        if (bal(allc) == 0ull) break;
    }
}

__device__ __forceinline__ void lookforward(Px &P, int &wa, int &wb) {
    const ccdgpu_params &p = ARGS().p;
    Lds *L = &LDS();
    const int l = lane();
    const int k = P.peek;
    const int B = W - (k - 1);  // steps per batch: windows x .. x + k - 1 stay inside the 64-row ring
    int a = wa, b = wb;
    int fa = a, fb = b;
    bool have = false;
    double change = 0.0;
    int nc = p.coef_min;
    int fit_span = CDRU(P, b - 1) - CDRU(P, a);  // days (wave-uniform)
    int peek_start = b;
    int moff = 0;            // ring offset of the last evaluated peek window
    int hfa = -1, hfb = -1;  // fit window the closest-DOY buckets describe
    int nc_fit = nc;         // coefficients of the current fit
    bool exiting = false;  // the loop ends at its top
    bool bnd_ok = false;   // fit_bounds' bins and blocks (L->hist2, L->blk) describe the current models
    // One fit_models site for the three refits of this loop (an early step, the long-peek span
    // refit, the batched span refit): a path that needs a fit records it in fmode and continues,
    // the fit runs at the top of the next iteration, and the early / long-peek steps then resume
    // with their single-step evaluation (ev), which they share.  One inlined copy of the Gram +
    // coordinate descent instead of three keeps the kernel body (and its instruction-cache
    // footprint) smaller; the order of operations is unchanged.
    int fmode = 0;  // pending fit: 1 early step, 2 long-peek span refit, 3 batched refit
    for (;;) {
        if (exiting) break;
        int ev = 0;  // single-step evaluation of this iteration: 1 early step, 2 long peek
        if (fmode) {
            // fmode 4: the current models' bounds only (a batch of more than 24 fit observations
            // whose fit was an early step's: the first of a lookforward whose initialize window
            // holds more than 24), then that batch again
            if (fmode != 4) {
            fit_models(P, fa, fb, nc_fit, fmode == 1 || fb - fa <= 24);  // rmse: from fit_bounds when it runs
            if (fmode == 1) {
                have = true;
                if (l < NB) L->comp[l] = L->rmse[l];  // early step: comparison rmse = model rmse
                wsync();
            }
            }
            // a span refit of more than 24 observations: its rmse and the batched steps'
            // comparison-rmse bounds from one pass over the window's residuals (the one site)
            bnd_ok = fmode == 4 || !(fmode == 1 || fb - fa <= 24);
            if (bnd_ok) {
                PH_BEGIN(fbd)
                fit_bounds(P, fa, fb, nc_fit);
                PH_END(P, fbd, 12)  // (with build_buckets: the "closest bucket build" slot)
            }
            ev = fmode == 3 || fmode == 4 ? 0 : fmode;
            fmode = 0;
        }
        if (!ev && !(b + k < P.m || !have)) {
            exiting = true;
            continue;
        }
        if (!ev && (!have || b - a < 24)) {
            // early steps: speculative fits of the next windows, then the steps one by one
            const int nw0 = b - a;
            int V = 24 - nw0;
            V = V > 8 ? 8 : V;
            V = V > P.m - b + 1 ? P.m - b + 1 : V;  // staged rows stay inside the period
            while (V > 1 && num_coefs(p, nw0 + V - 1) - 1 > SPEC_PC) --V;
            if (V >= 1 && num_coefs(p, nw0) - 1 <= SPEC_PC) {
                PH_BEGIN(sf)
                SpecFit F;
                spec_fits(P, a, nw0, V, F);
                PH_END(P, sf, 20)
                int sp = 0, valid = V - 1, installed = -1;
                bool brk = false;
                for (;;) {
                    if (!(b + k < P.m || !have)) break;
                    if (have && b - a >= 24) break;
                    if (sp > valid) break;
                    nc = num_coefs(p, b - a);
                    peek_start = b;
                    fa = a;
                    fb = b;
                    fit_span = CDRU(P, b - 1) - CDRU(P, a);
                    if (installed != sp) {
                        spec_install(P, F, sp, b - a, nc);
                        bnd_ok = false;
                        installed = sp;
                        PH_COUNT(P, 37, 1)
                    }
                    nc_fit = nc;
                    have = true;
                    double m0;
                    PH_BEGIN(ep)
                    const bool chg_now = eval_peek(P, k, b, 1, m0);
                    PH_END(P, ep, 8)
                    moff = 0;
                    if (chg_now) {
                        change = 1.0;
                        brk = true;
                        break;
                    }
                    if (m0 > p.outlier_threshold) {
                        const int rm = b;
                        compact_drop(P, rm, rm + 1, [&](int j) { return j == rm; });
                        valid = sp;  // later windows held the removed observation
                        continue;
                    }
                    b += 1;
                    sp += 1;
                }
                if (brk) exiting = true;
                continue;
            }
            // early step: refit every step (comparison rmse = model rmse), then evaluate it
            nc = num_coefs(p, b - a);
            peek_start = b;
            fa = a;
            fb = b;
            fit_span = CDRU(P, b - 1) - CDRU(P, a);
            nc_fit = nc;
            fmode = 1;
            continue;
        }
        if (!ev && k > W) {
            // A peek longer than the 64-row ring (adaptive peek > 64: median date gap < 1.5
            // days) runs one step at a time in change.lookforward's own order: refit on the span
            // test, comparison rmse from the 24 closest-DOY fit observations of the peek end.
            nc = num_coefs(p, b - a);
            peek_start = b;
            const int span = CDRU(P, b - 1) - CDRU(P, a);
            ev = 2;
            if ((double)span >= 1.33 * (double)fit_span) {
                fa = a;
                fb = b;
                fit_span = span;
                nc_fit = nc;
                fmode = 2;
                continue;
            }
        }
        if (ev) {
            if (ev == 2) {
                if (fb - fa > 24) {
                    // the exact comparison rmse of the step as a batched step's (coop_comp)
                    if (hfa != fa || hfb != fb) {
                        build_buckets(P, fa, fb);
                        hfa = fa;
                        hfb = fb;
                    }
                    const unsigned dm = det_mask();
                    const int nd = __builtin_popcount(dm);
                    int bs[NB];
                    unsigned rest = dm;
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        bs[t] = rest ? __builtin_ctz(rest) : 0;
                        rest &= rest - 1u;
                    }
                    double o[NB];
                    coop_comp(P, fa, fb - fa, CDR(P, b + k - 1), bs, nd, o);
#pragma unroll
                    for (int t = 0; t < NB; ++t)
                        if (t < nd && l == bs[t]) L->comp[l] = o[t];
                    wsync();
                } else {
                    closest_doy_scan(P, fa, fb);
                }
            }
            double m0;
            PH_BEGIN(ep)
            const bool chg_now = eval_peek(P, k, b, 1, m0);
            PH_END(P, ep, 8)
            moff = 0;
            if (chg_now) {
                change = 1.0;
                exiting = true;
                continue;
            }
            if (m0 > p.outlier_threshold) {
                const int rm = b;
                compact_drop(P, rm, rm + 1, [&](int j) { return j == rm; });
                continue;
            }
            b += 1;
            continue;
        }
        // ---- batch of up to B steps at window starts x0 .. x0 + B - 1 (model fixed)
        const int nf = fb - fa;
        if (nf > 24 && !bnd_ok) {
            fmode = 4;  // the bounds at the loop's top, then this batch
            continue;
        }
        if (nf <= 24) closest_doy_scan(P, fa, fb);  // every fit observation: one comp for all steps
        PH_BEGIN(cl)
        const int x0 = b, m0 = P.m;
        PH_BEGIN(rr)
        ring_rows(P, x0);
        PH_END(P, rr, 13)
        PH_COUNT(P, 17, 1)
        bool valid = l < B && x0 + l + k < m0;
        const int da = CDRU(P, a);
        const int dprev = CDRU(P, x0 - 1);
        const int dj = valid ? CDR(P, x0 + l) : 0;
        {
            // Steps past the first span-test refit are never executed.  Without removals step l's
            // last kept observation is x0 + l - 1; a removal only moves it earlier (the refit
            // later), so the first such step under that assumption bounds the batch from below:
            // lanes more than 2 steps past it are left out (with more removals before it the batch
            // ends there without a terminal step and the next one continues).
            const int dp = shf(dj, l > 0 ? l - 1 : 0);
            const bool t0 = valid && ((double)(l > 0 ? dp : dprev) - (double)da) >= 1.33 * (double)fit_span;
            const unsigned long long T0 = bal(t0);
            const int lim = T0 ? __ffsll((long long)T0) + 1 : W;  // first such step + 2
            valid = valid && l <= lim;
        }
        const unsigned long long V = bal(valid);
        bool allc = false, outj = false;
        if (nf > 24) {
            const unsigned dm = det_mask();
            const int nd = __builtin_popcount(dm);
            int bs[NB];
            unsigned rest = dm;
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                bs[t] = rest ? __builtin_ctz(rest) : 0;
                rest &= rest - 1u;
            }
            const int drf = valid ? CDR(P, x0 + l + k - 1) : 0;  // the step's reference date (peek end)
            // The magnitudes with the comparison rmse left out bound the true ones from above
            // (change_magnitude divides by max(vario, comp) >= vario; division, multiplication,
            // squares and sums are monotone under round-to-nearest): a step whose upper bound has
            // a peek magnitude <= the change threshold and a first one <= the outlier threshold
            // is a plain step, exactly as with its comp (~95 % of steps).  The others -- nearly
            // all true outliers -- get a lower bound too, from an upper bound of comp
            // (comp_bound: the squared residuals of the fit-window blocks around the step's day
            // of year, fit_bounds); a step whose two bounds agree on both tests is decided.  The
            // C3 tile mix leaves ~0.1 % of its steps to the exact comparison rmse below.
            bool und = false, au = false, ou = false;
            PH_BEGIN(mgu)
            if (valid) {
                double iu[NB];
                bool vz = false;  // a zero vario: 1 / vario is infinite (r = 0 would give NaN) -- no bound
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    const double vr = L->vario[bs[t]];
                    iu[t] = t < nd ? 1.0 / vr : 0.0;  // (a NaN vario: NaN, as with any comp)
                    vz = vz || (t < nd && vr == 0.0);
                }
                if (nd <= 5) peek_mags<5>(bs, iu, k, au, ou);
                else peek_mags<NB>(bs, iu, k, au, ou);
                und = vz || au || ou;
            }
            unsigned long long Um = bal(und);
            if (Um) {
                if (und) {
                    double cbv[NB];
                    comp_bound(nf, drf, bs, nd, cbv);
                    double il[NB];
                    bool vz = false;
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        const double vr = L->vario[bs[t]], cb = cbv[t];
                        const double rm = (vr != vr || cb != cb) ? __builtin_nan("") : (vr > cb ? vr : cb);
                        il[t] = t < nd ? 1.0 / rm : 0.0;
                        vz = vz || (t < nd && vr == 0.0);
                    }
                    bool al = false, ol = false;
                    if (nd <= 5) peek_mags<5>(bs, il, k, al, ol);
                    else peek_mags<NB>(bs, il, k, al, ol);
                    if (!vz && al == au && ol == ou) {
                        allc = au;
                        outj = ou;
                        und = false;
                    }
                }
                Um = bal(und);
            }
            PH_END(P, mgu, 15)
            if (Um) {
                // the undecided steps in order, each resolved exactly; once a step below the next
                // one is known to end the batch (change or span refit, from the steps below it,
                // all exact by then) the rest lie past the batch's first terminating step and
                // cannot change its outcome (left undecided as plain steps: allc = outj = false)
                PH_BEGIN(cmp)
                int nres = 0;  // (counted in the diagnostic build)
                (void)nres;
                for (unsigned long long mm = Um; mm; mm &= mm - 1ull) {
                    const int x = __builtin_ctzll(mm);
                    const unsigned long long Ok = bal(valid && outj);
                    const unsigned long long lw = (V & ~Ok) & ((1ull << l) - 1ull);
                    const int lkk = lw ? 63 - __clzll(lw) : 0;
                    const int dsh = shf(dj, lkk);
                    const int dlk = lw ? dsh : dprev;
                    const bool trg = valid && ((double)dlk - (double)da) >= 1.33 * (double)fit_span;
                    if (bal(l < x && (trg || allc))) break;
                    if (hfa != fa || hfb != fb) {
                        PH_BEGIN(hb)
                        build_buckets(P, fa, fb);
                        PH_END(P, hb, 12)
                        hfa = fa;
                        hfb = fb;
                    }
                    double o[NB];
                    coop_comp(P, fa, nf, rdl(drf, x), bs, nd, o);
                    ++nres;
                    if (l == x) {
                        double irm[NB];
#pragma unroll
                        for (int t = 0; t < NB; ++t) {
                            const double vr = L->vario[bs[t]], cr = o[t];
                            const double rm = (vr != vr || cr != cr) ? __builtin_nan("") : (vr > cr ? vr : cr);
                            irm[t] = t < nd ? 1.0 / rm : 0.0;
                        }
                        if (nd <= 5) peek_mags<5>(bs, irm, k, allc, outj);
                        else peek_mags<NB>(bs, irm, k, allc, outj);
                    }
                }
                PH_COUNT(P, 21, nres)  // exact comparison rmse evaluations
                PH_END(P, cmp, 14)
            }
        } else if (valid) {
            // comparison rmse per detection band: cs[s] for the s-th detection band bs[s]
            const unsigned dm = det_mask();
            const int nd = __builtin_popcount(dm);
            int bs[NB];
            unsigned rest = dm;
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                bs[t] = rest ? __builtin_ctz(rest) : 0;
                rest &= rest - 1u;
            }
            double cs[NB];
#pragma unroll
            for (int t = 0; t < NB; ++t) cs[t] = 0.0;
            // (nf <= 24: every fit observation, one comparison rmse for all steps: closest_doy_scan)
#pragma unroll
            for (int t = 0; t < NB; ++t) cs[t] = L->comp[bs[t]];
            PH_BEGIN(mg)
            // change_magnitude: (r / max(vario, comp))^2 summed over the detection bands (in band
            // order), with the division as a multiply by the band's reciprocal (one division per
            // band and step)
            double irm[NB];
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                const double vr = L->vario[bs[t]], cr = cs[t];
                const double rm = (vr != vr || cr != cr) ? __builtin_nan("") : (vr > cr ? vr : cr);
                irm[t] = t < nd ? 1.0 / rm : 0.0;
            }
            if (nd <= 5) peek_mags<5>(bs, irm, k, allc, outj);
            else peek_mags<NB>(bs, irm, k, allc, outj);
            PH_END(P, mg, 15)
        }
        const unsigned long long O = bal(valid && outj);
        const unsigned long long lower = (V & ~O) & ((1ull << l) - 1ull);
        const int lk = lower ? 63 - __clzll(lower) : 0;
        const int dsh = shf(dj, lk);
        const int dlk = lower ? dsh : dprev;  // date at position b - 1 when step l starts
        const bool trig = valid && ((double)dlk - (double)da) >= 1.33 * (double)fit_span;
        const unsigned long long TG = bal(trig);
        const unsigned long long Tm = bal(valid && (trig || allc));
        const int nv = popc(V);
        const int xs = Tm ? __ffsll((long long)Tm) - 1 : nv;  // first step not executed as a plain step
        const bool change_here = Tm && !((TG >> xs) & 1ull);
        // steps executed: 0 .. xs - 1 (plus xs itself when it detects the change)
        const int ne = change_here ? xs + 1 : xs;
        stat_uniform(ST_FLOPS, (unsigned long long)ne *
                ((unsigned long long)k * (7 * 2 * 8 + 5 * 3) + (unsigned long long)nf * 6 + 5 * 48));
        PH_COUNT(P, 16, ne)
#if !defined(CCD_CD_CYCLES) && !defined(CCD_CD_CHKSTAT)  // (slots 24-27 carry the coordinate-descent statistics there)
        PH_COUNT(P, 24, ne <= 16 ? 1 : 0)
        PH_COUNT(P, 25, ne <= 32 ? 1 : 0)
        PH_COUNT(P, 26, nv)
        PH_COUNT(P, 27, Tm ? 0 : 1)
#endif
        PH_END(P, cl, 7)
        const unsigned long long rem = xs >= 64 ? O : (O & ((1ull << xs) - 1ull));
        const int R = popc(rem);
        if (ne > 0) {
            const int last = ne - 1;  // last executed step
            peek_start = x0 + last - popc(rem & ((1ull << last) - 1ull));
            nc = num_coefs(p, peek_start - a);
            moff = last;
        }
        if (R) {
            PH_BEGIN(cp)
            compact_drop(P, x0, x0 + xs, [&](int j) { return ((rem >> (j - x0)) & 1ull) != 0ull; });
            PH_END(P, cp, 9)
        }
        if (change_here) {
            b = peek_start;
            change = 1.0;
            exiting = true;
            continue;
        }
        b = x0 + xs - R;
        if (Tm) {
            // refit at step xs (its evaluation runs in the next batch with the new model)
            nc = num_coefs(p, b - a);
            fa = a;
            fb = b;
            fit_span = CDRU(P, b - 1) - CDRU(P, a);
            nc_fit = nc;
            fmode = 3;  // the refit runs at the top of the loop
            PH_COUNT(P, 34, 1)
        }
    }
    PH_BEGIN(md)
    const double mag_lane = peek_medians(P, k, moff);
    emit(P, CDRU(P, a), CDRU(P, b - 1), CDRU(P, peek_start), b - a, change, nc, mag_lane);
    PH_END(P, md, 11)
    wa = a;
    wb = b;
}

// proc: the pixel's procedure.  The permanent-snow and insufficient-clear procedures
// (procedures.permanent_snow_procedure / insufficient_clear_procedure: one fit over every usable
// observation when there are at least meow_size of them) run through the same catch site.
__device__ __forceinline__ void standard_procedure(Px &P, int proc) {
    const ccdgpu_params &p = ARGS().p;
    const int meow = p.meow_size;
    int a = 0, b = meow, prev = 0, nres = 0;
    bool start = true;
    // ccd.procedures.standard_procedure's loop with its two catch() calls (the start segment
    // before a model, the end segment after the last one) run from one site (one inlined copy of
    // the fit): cmode 1 = the start catch, after which the iteration resumes; 2 = the end catch;
    // 3 = the whole-period segment of the other procedures.
    int cmode = 0, ca = 0, cb = 0, cq = 0;
    if (proc != CCDGPU_PROC_STANDARD) {
        if (P.m < meow) return;
        cmode = 3;
        cb = P.m;
        cq = proc == CCDGPU_PROC_PERMANENT_SNOW ? p.curve_qa_persist_snow : p.curve_qa_insuf_clear;
    } else {
        PH_BEGIN(vg)
        variogram(P);
        adjust_peek(P);
        wsync();  // LDS().chg written by lane 0
        PH_END(P, vg, 2)
    }
    for (;;) {
        bool resume = false;
        if (cmode) {
            catch_(P, ca, cb, cq, cmode == 3);
            if (cmode >= 2) break;
            cmode = 0;
            resume = true;
        }
        bool end = false;
        if (!resume) {
            if (!(b <= P.m - meow)) {
                end = true;
            } else {
                if (nres > 0) start = false;
                if (!initialize(P, a, b)) {
                    end = true;
                } else {
                    if (a > prev) lookback(P, a, b, prev);
                    if (a - prev > P.peek && start) {
                        ca = prev;
                        cb = a;
                        cq = p.curve_qa_start;
                        cmode = 1;
                        nres++;
                        start = false;
                        continue;
                    }
                }
            }
        }
        if (!end && b + P.peek > P.m) end = true;
        if (end) {
            if (!(prev + P.peek < P.m)) break;
            ca = prev;
            cb = P.m;
            cq = p.curve_qa_end;
            cmode = 2;
            continue;
        }
        lookforward(P, a, b);
        nres++;
        prev = b;
        a = b;
        b = b + meow;
    }
}

// ------------------------------------------------------------------ qa.py filters + compaction
// A pixel's inputs are read where they lie: the standard band-major layout (a plain upload, the
// chipmunk decoder), a raw section of a transport-encoded batch (the same layout at the section's
// own base pointers), or an encoded section (include/ccdgpu.h; ccd_encode.c) -- QA as 4-bit
// palette codes, band values sent only for observations without a drop bit, compacted per pixel.
// An encoded pixel is read in place, so the upload needs no decode pass (the standalone decoder
// ccd_decode_enc in ccd_pack.hip is the same mapping): pass 1 walks the code row in input order
// (class counts are order-free) and leaves, per 64 input observations, the bit mask of the
// observations whose bands were sent and the count before them in LDS; pass 2 gathers in date
// order, an observation's band values at its rank among the sent ones (-9999, the ARD fill value
// the encoder dropped, for the others).
// Returns the procedure, or -1 for an unsupported QA value.
__device__ __forceinline__ int px_setup(Px &P, int chip, int pix) {
    const CcdDetectArgs &A = ARGS();
    const ccdgpu_params &p = A.p;
    Lds *L = &LDS();
    const int l = lane();
    const int n = P.n;
    const int32_t *order = A.order + A.chip_obs_off[chip];
    const uint16_t *qa;
    const int16_t *sp;
    size_t bstride;
    const unsigned char *codes = nullptr;  // encoded: the pixel's code row
    int kcount = 0;                        // encoded: observations whose bands were sent
    unsigned drop = 0u;
    bool enc = false;
    if (A.enc) {
        const unsigned char *sec = A.enc + reinterpret_cast<const int64_t *>(A.enc)[1 + chip];
        const int32_t *h = reinterpret_cast<const int32_t *>(sec);
        const int64_t cpix = h[1];
        const int64_t plane = cpix * n;
        if (h[0] == 0) {
            qa = reinterpret_cast<const uint16_t *>(sec + 128) + (size_t)pix * n;
            sp = reinterpret_cast<const int16_t *>(sec + 128 + ((2 * plane + 15) & ~(int64_t)15)) + (size_t)pix * n;
            bstride = (size_t)plane;
        } else {
            enc = true;
            bstride = (size_t)reinterpret_cast<const int64_t *>(sec + 48)[2];
            const uint32_t *koff = reinterpret_cast<const uint32_t *>(sec + 128);
            const unsigned char *q4 = sec + 128 + ((4 * (cpix + 1) + 15) & ~(int64_t)15);
            const int64_t rowb = (n + 1) / 2;
            codes = q4 + (size_t)pix * rowb;
            const uint32_t k0 = koff[pix];
            kcount = (int)(koff[pix + 1] - k0);
            sp = reinterpret_cast<const int16_t *>(q4 + ((cpix * rowb + 15) & ~(int64_t)15)) + k0;
            qa = nullptr;
            drop = *reinterpret_cast<const uint32_t *>(sec + 80);
            if (l < 16) L->epal[l] = reinterpret_cast<const uint16_t *>(sec + 16)[l];
            wsync();
        }
    } else {
        const int64_t data_off = A.chip_data_off[chip];
        qa = A.qa + data_off + (size_t)pix * n;
        bstride = (size_t)(A.chip_pix_off[chip + 1] - A.chip_pix_off[chip]) * n;
        sp = A.spectra + (size_t)NB * data_off + (size_t)pix * n;
    }
    int c_clear = 0, c_water = 0, c_snow = 0, c_cloud = 0, c_fill = 0;
    bool bad = false;
    if (enc) {
        // input order: code bytes read contiguously (four chunks' loads together), palette in LDS
        constexpr int U = 4;
        int sent = 0;
        for (int base0 = 0; base0 < n; base0 += U * W) {
            unsigned cb[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = base0 + u * W + l;
                cb[u] = i < n ? (unsigned)codes[i >> 1] : 0u;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = base0 + u * W + l;
                const bool in = i < n;
                const unsigned q = L->epal[(cb[u] >> ((i & 1) * 4)) & 15u];
                const int cls = in ? (p.qa_bitpacked ? qabitval(p, q) : (int)q) : -2;
                c_clear += popc(bal(in && cls == p.qa_clear));
                c_water += popc(bal(in && cls == p.qa_water));
                c_snow += popc(bal(in && cls == p.qa_snow));
                c_cloud += popc(bal(in && cls == p.qa_cloud));
                c_fill += popc(bal(in && cls == p.qa_fill));
                if (bal(in && cls < 0)) bad = true;
                const unsigned long long km = bal(in && !(q & drop));
                if (l == 0 && base0 + u * W < n) {
                    L->ekm[(base0 >> 6) + u] = km;
                    L->ekp[(base0 >> 6) + u] = (uint16_t)sent;
                }
                sent += popc(km);
            }
        }
        wsync();
    } else {
    // (four 64-observation chunks per round, their dependent order -> qa loads issued together;
    // the next round's order loads go out with this round's qa loads)
    constexpr int U = 4;
    int on[U];
#pragma unroll
    for (int u = 0; u < U; ++u) on[u] = u * W + l < n ? order[u * W + l] : 0;
    for (int base0 = 0; base0 < n; base0 += U * W) {
        int o[U];
        unsigned q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) o[u] = on[u];
#pragma unroll
        for (int u = 0; u < U; ++u) q[u] = base0 + u * W + l < n ? (unsigned)qa[o[u]] : 0u;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base0 + (U + u) * W + l;
            on[u] = i < n ? order[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base0 + u * W + l;
            int cls = -2;
            if (i < n) cls = p.qa_bitpacked ? qabitval(p, q[u]) : (int)q[u];
            c_clear += popc(bal(i < n && cls == p.qa_clear));
            c_water += popc(bal(i < n && cls == p.qa_water));
            c_snow += popc(bal(i < n && cls == p.qa_snow));
            c_cloud += popc(bal(i < n && cls == p.qa_cloud));
            c_fill += popc(bal(i < n && cls == p.qa_fill));
            if (bal(i < n && cls < 0)) bad = true;
        }
    }
    }
    if (bad) return -1;
    const int total = n - c_fill;
    const int cw = c_clear + c_water;
    if (l == 0) {
        double *pr = A.probs + 3 * (size_t)P.gpix;
        pr[0] = (double)c_cloud / (double)total;
        pr[1] = (double)c_snow / ((double)(cw + c_snow) + 0.01);
        pr[2] = (double)c_water / ((double)(cw + c_snow) + 0.01);
    }
    int proc;
    if (!((double)cw / (double)total >= p.clear_pct_threshold))
        proc = ((double)c_snow / ((double)(cw + c_snow) + 0.01) >= p.snow_pct_threshold)
                   ? CCDGPU_PROC_PERMANENT_SNOW : CCDGPU_PROC_INSUFFICIENT_CLEAR;
    else
        proc = CCDGPU_PROC_STANDARD;
    const bool conv = proc == CCDGPU_PROC_STANDARD && p.kelvin_to_celsius;
    // processing mask: written straight into the pixel's output words (words past the chip's own
    // n are zero; the chunk loop below writes the rest)
    GLOBAL_AS unsigned *mk = pmask(P);
    for (int i = ((n + 31) >> 5) + l; i < A.mask_words; i += W) mk[i] = 0u;
    int m = 0;
    int carry = -1;  // date of the last kept observation (ordinals are >= 1)
    constexpr int U2 = 2;  // two chunks per round: their gathers (order -> qa, 7 bands, date) together,
                           // the next round's order loads with them
    int on2[U2];
#pragma unroll
    for (int u = 0; u < U2; ++u) on2[u] = u * W + l < n ? order[u * W + l] : 0;
    for (int base0 = 0; base0 < n; base0 += U2 * W) {
        int o2[U2], d2[U2];
        unsigned q2[U2];
        int16_t v2[U2][NB];
#pragma unroll
        for (int u = 0; u < U2; ++u) o2[u] = on2[u];
        if (enc) {
            unsigned cb[U2];
#pragma unroll
            for (int u = 0; u < U2; ++u) cb[u] = base0 + u * W + l < n ? (unsigned)codes[o2[u] >> 1] : 0u;
#pragma unroll
            for (int u = 0; u < U2; ++u) {
                const int i = base0 + u * W + l;
                const bool valid = i < n;
                const int o = o2[u];
                const unsigned q = L->epal[(cb[u] >> ((o & 1) * 4)) & 15u];
                q2[u] = valid ? q : 0u;
                const int w = o >> 6;
                const int r = (int)L->ekp[w] + popc(L->ekm[w] & ((1ull << (o & 63)) - 1ull));
                const bool have = valid && !(q & drop) && r < kcount;
#pragma unroll
                for (int b = 0; b < NB; ++b) v2[u][b] = valid ? (int16_t)-9999 : (int16_t)0;
                if (have) {
#pragma unroll
                    for (int b = 0; b < NB; ++b) v2[u][b] = sp[(size_t)b * bstride + r];
                }
                d2[u] = valid ? (int)P.sd[i] : 0;
            }
        } else {
#pragma unroll
        for (int u = 0; u < U2; ++u) {
            const int i = base0 + u * W + l;
            const bool valid = i < n;
            q2[u] = valid ? (unsigned)qa[o2[u]] : 0u;
#pragma unroll
            for (int b = 0; b < NB; ++b) v2[u][b] = valid ? sp[(size_t)b * bstride + o2[u]] : (int16_t)0;
            d2[u] = valid ? (int)P.sd[i] : 0;
        }
        }
#pragma unroll
        for (int u = 0; u < U2; ++u) {
            const int i = base0 + (U2 + u) * W + l;
            on2[u] = i < n ? order[i] : 0;
        }
#pragma unroll
        for (int u = 0; u < U2; ++u) {
        const int base = base0 + u * W;
        const int i = base + l;
        const bool valid = i < n;
        int cls = -2;
        const int d = d2[u];
        int16_t v[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) v[b] = v2[u][b];
        if (valid) {
            cls = p.qa_bitpacked ? qabitval(p, q2[u]) : (int)q2[u];
            if (conv) v[6] = (int16_t)((int)v[6] * 10 - 27315);
        }
        const bool cwi = cls == p.qa_clear || cls == p.qa_water;
        const bool th = v[6] > p.thermal_min && v[6] < p.thermal_max;
        bool sat = true;
#pragma unroll
        for (int b = 0; b < 6; ++b) sat = sat && v[b] > 0 && v[b] < 10000;
        bool keep = valid && cwi && th && sat;
        if (proc == CCDGPU_PROC_PERMANENT_SNOW) keep = keep || (valid && cls == p.qa_snow);
        const unsigned long long km = bal(keep);
        const unsigned long long lower = l ? (km & ((1ull << l) - 1ull)) : 0ull;
        const int pl = lower ? 63 - __clzll(lower) : l;
        const int pd = shf(d, pl);
        const int prevd = lower ? pd : carry;
        const bool keep2 = keep && d != prevd;
        if (km) carry = rdl(d, 63 - __clzll(km));
        const unsigned long long k2 = bal(keep2);
        if (keep2) {
            const int pos = gidx(P, m + below(k2), n, __LINE__);
            PCD(P)[pos] = d;
            CRow cw;
#pragma unroll
            for (int b = 0; b < NB; ++b) cw.v[b] = v[b];
            cw.ci = (uint16_t)i;
            PCR(P)[pos] = cw;
        }
        if (l == 0 && base < n) {
            mk[base >> 5] = (unsigned)k2;
            if (base + 32 < n) mk[(base >> 5) + 1] = (unsigned)(k2 >> 32);
        }
        m += popc(k2);
        }
    }
    P.m = m;
    P.gp = m;  // no gap yet: logical row = physical row
    P.gl = 0;
    psync();
    if (proc == CCDGPU_PROC_INSUFFICIENT_CLEAR && m > 0) {
        const CRow *g = PCR(P);
        auto gen = [&](int i, int &val) -> bool { val = (int)g[i].v[1] + 32768; return true; };
        const double med = median_u16(gen, m, m) - 32768.0 + (double)p.median_green_filter;
        compact_drop(P, 0, m, [&](int j) { return !((double)g[j].v[1] < med); });
    }
    return proc;
}

__device__ __forceinline__ void detect_body() {
    const CcdDetectArgs &A = ARGS();
    Lds &lds = LDS();
    const int l = lane();
    const int slot = blockIdx.x;
    const size_t nmax = (size_t)A.n_obs_max;  // per-slot scratch stride
    Px P;
    P.cd = A.s_date + (size_t)slot * nmax;
    P.cr = reinterpret_cast<CRow *>(A.s_row) + (size_t)slot * nmax;
    P.bad = 0;
    if (l < 4) lds.stat[l] = 0ull;
#ifdef CCD_PHASE_TIMERS
    if (l < CCD_NPHASE) lds.tph[l] = 0;
#endif
    // launch execution window on the device's constant-rate clock (first wave in, last wave out):
    // the kernel's own duration even when it queued behind another context's launch
    if (l == 0) atomicMin(&A.counters[5], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    for (;;) {
        unsigned long long job = 0;
        if (l == 0) job = atomicAdd(&A.counters[0], 1ull);
        job = uni(job);  // lane 0's
        if (job >= (unsigned long long)A.total_pix) break;
        // chip of this pixel: binary search of the chips' pixel offsets (wave-uniform)
        int lo = 0, hi = A.n_chips - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if ((unsigned long long)A.chip_pix_off[mid] <= job) lo = mid;
            else hi = mid - 1;
        }
        const int chip = lo;
        const int pix = (int)(job - (unsigned long long)A.chip_pix_off[chip]);
        const int64_t obs_off = A.chip_obs_off[chip];
        P.n = A.chip_nobs[chip];
        P.gpix = (int64_t)job;
        P.nseg = 0;
        P.acc_a = -1;
        P.acc_b = 0;
        P.fit_k = 0;
        P.basis = as_global(A.basis + (size_t)obs_off * CCD_BASIS_STRIDE);
        P.sd = A.sdates + obs_off;
#ifndef CCD_PHASE_TIMERS
        if (A.poison) {
            // test mode: no value may come from a previous pixel's (or wave's) LDS contents
            uint4 *w = reinterpret_cast<uint4 *>(&lds);
            for (int i = l; i < (int)(offsetof(Lds, stat) / 16); i += W) w[i] = uint4{~0u, ~0u, ~0u, ~0u};
            // ... nor from the slot's global scratch
            for (size_t i = l; i < CCD_SLOT_F64(nmax); i += W) PFS(P)[i] = __longlong_as_double(-1ll);
            for (size_t i = l; i < nmax; i += W) PBK(P)[i] = 0xFFFFu;
            for (size_t i = l; i < nmax; i += W) {
                P.cd[i] = -1;
                reinterpret_cast<uint4 *>(P.cr)[i] = uint4{~0u, ~0u, ~0u, ~0u};
            }
            gsync();
        }
#endif
        PH_BEGIN(tot)
        PH_BEGIN(su)
        const int proc = px_setup(P, chip, pix);
        PH_END(P, su, 1)
        if (proc < 0) {
            if (l == 0) {
                atomicMin(&A.counters[2], (unsigned long long)job);
                A.procedure[job] = -1;
                A.nseg[job] = 0;
            }
            for (int i = l; i < A.mask_words; i += W) A.mask_bits[(size_t)job * A.mask_words + i] = 0u;
            continue;
        }
        standard_procedure(P, proc);
        wsync();
        PH_END(P, tot, 0)
        if (l == 0) {
            A.procedure[job] = proc;
            A.nseg[job] = P.nseg;
        }
        wsync();
    }
    // index-guard report (first tripped line of any lane)
    {
        int bl = P.bad;
        for (int o = 32; o > 0; o >>= 1) {
            const int t = shfx(bl, o);
            bl = t > bl ? t : bl;
        }
        if (l == 0 && bl) atomicCAS(&A.counters[4], 0ull, (unsigned long long)bl);
    }
    // instrumentation
    if (l == 0) atomicMax(&A.counters[6], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    wsync();
    if (l == 0) {
        atomicAdd(&A.stats[0], lds.stat[ST_FITS]);
        atomicAdd(&A.stats[1], lds.stat[ST_SWEEPS]);
        atomicAdd(&A.stats[2], lds.stat[ST_FLOPS]);
#ifdef CCD_PHASE_TIMERS
        for (int i = 0; i < CCD_NPHASE; ++i) atomicAdd(&A.stats[8 + i], lds.tph[i]);
#endif
    }
}

// Four register budgets of the same body: 1 wave/SIMD (no spills), 2, 3 and 4 waves/SIMD (256,
// 168 and 128 VGPRs, spills growing).  The host picks one (CCDGPU_KERNEL=w1..w4; default w4, the
// fastest since round 5: C3 185.5 vs 193.0 ms per launch, C5 600 vs 614 ms -- its fourth wave hides
// more latency than its extra spills cost).
// (arg_slot: the c_args slot of the launching context, read by ARGS() from the kernarg segment)
__global__ __launch_bounds__(64) __attribute__((flatten)) void ccd_detect(int arg_slot) { detect_body(); }
__global__ __launch_bounds__(64, 2) __attribute__((flatten)) void ccd_detect_w2(int arg_slot) { detect_body(); }
__global__ __launch_bounds__(64, 3) __attribute__((flatten)) void ccd_detect_w3(int arg_slot) { detect_body(); }
__global__ __launch_bounds__(64, 4) __attribute__((flatten)) void ccd_detect_w4(int arg_slot) { detect_body(); }

// ------------------------------------------------------------------ per-chip preparation
// numpy's argsort (kind='quicksort', numpy < 1.17 aquicksort -- the pinned reference's; restated
// in oracle/ccd_oracle.c ccdoracle_np_argsort) of n <= CCDGPU_MAX_OBS keys in LDS, by one thread:
// ord holds 0 .. n-1 on entry and the argsort on return.  Only chips with repeated dates get here
// (without ties every sort gives the same order), so the sequential sort costs nothing elsewhere.
__device__ void np_aquicksort_lds(const int64_t *v, uint16_t *ord, int n) {
    int pl = 0, pr = n - 1;
    int stack[64];  // (pl, pr) pairs: the larger part is pushed, so <= 2 log2(n) entries
    int sp = 0;
    for (;;) {
        while (pr - pl > 15) {
            const int pm = pl + ((pr - pl) >> 1);
            uint16_t t;
            if (v[ord[pm]] < v[ord[pl]]) { t = ord[pm]; ord[pm] = ord[pl]; ord[pl] = t; }
            if (v[ord[pr]] < v[ord[pm]]) { t = ord[pr]; ord[pr] = ord[pm]; ord[pm] = t; }
            if (v[ord[pm]] < v[ord[pl]]) { t = ord[pm]; ord[pm] = ord[pl]; ord[pl] = t; }
            const int64_t vp = v[ord[pm]];
            int pi = pl, pj = pr - 1;
            t = ord[pm]; ord[pm] = ord[pj]; ord[pj] = t;
            for (;;) {
                do ++pi; while (v[ord[pi]] < vp);
                do --pj; while (vp < v[ord[pj]]);
                if (pi >= pj) break;
                t = ord[pi]; ord[pi] = ord[pj]; ord[pj] = t;
            }
            t = ord[pi]; ord[pi] = ord[pr - 1]; ord[pr - 1] = t;
            if (pi - pl < pr - pi) {
                stack[sp] = pi + 1; stack[sp + 1] = pr;
                pr = pi - 1;
            } else {
                stack[sp] = pl; stack[sp + 1] = pi - 1;
                pl = pi + 1;
            }
            sp = sp + 2 < 64 ? sp + 2 : 62;
        }
        for (int i = pl + 1; i <= pr; ++i) {  // insertion sort
            const uint16_t vi = ord[i];
            const int64_t vv = v[vi];
            int j = i;
            while (j > pl && vv < v[ord[j - 1]]) {
                ord[j] = ord[j - 1];
                --j;
            }
            ord[j] = vi;
        }
        if (sp == 0) break;
        sp -= 2;
        pl = stack[sp];
        pr = stack[sp + 1];
    }
}

// One 256-thread block per chip: the argsort of the dates (ccd/__init__.py detect: numpy's
// quicksort tie order, or with argsort_stable ties by input position), sorted dates, order, and
// the coefficient_matrix rows (w = 2 pi / avg_days_yr; cos/sin of w t, 2 w t, 3 w t exactly as
// models/lasso.coefficient_matrix forms them).  The stable rank of every date is computed in
// parallel; a chip whose dates repeat then takes numpy's order from np_aquicksort_lds.
__global__ __launch_bounds__(256) void ccd_prep(const int64_t *dates, const int32_t *chip_nobs,
                                                const int64_t *chip_obs_off, double avg_days_yr,
                                                int argsort_stable, int32_t *order, int64_t *sdates,
                                                double *basis) {
    const int chip = blockIdx.x;
    const int n = chip_nobs[chip];
    const int64_t off = chip_obs_off[chip];
    const int64_t *d = dates + off;
    int32_t *ord = order + off;
    int64_t *sd = sdates + off;
    double *bs = basis + (size_t)off * CCD_BASIS_STRIDE;
    __shared__ int64_t sdl[CCDGPU_MAX_OBS];
    __shared__ uint16_t perm[CCDGPU_MAX_OBS];  // sorted position -> input position
    __shared__ int dup;
    if (threadIdx.x == 0) dup = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) sdl[i] = d[i];
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const int64_t di = sdl[i];
        int rank = 0, eq = 0;
        for (int j = 0; j < n; ++j) {
            const int64_t dj = sdl[j];
            rank += (dj < di || (dj == di && j < i)) ? 1 : 0;
            eq += dj == di ? 1 : 0;
        }
        perm[rank] = (uint16_t)i;
        if (eq > 1) dup = 1;
    }
    __syncthreads();
    if (dup && !argsort_stable) {
        if (threadIdx.x == 0) {
            for (int i = 0; i < n; ++i) perm[i] = (uint16_t)i;
            np_aquicksort_lds(sdl, perm, n);
        }
        __syncthreads();
    }
    const double w = 2.0 * M_PI / avg_days_yr;
    for (int r = threadIdx.x; r < n; r += blockDim.x) {
        const int i = perm[r];
        const int64_t di = sdl[i];
        ord[r] = i;
        sd[r] = di;
        const double w12 = w * (double)di;
        const double w34 = 2.0 * w12;
        const double w56 = 3.0 * w12;
        double *row = bs + (size_t)r * CCD_BASIS_STRIDE;
        row[0] = (double)di;
        row[1] = cos(w12);
        row[2] = sin(w12);
        row[3] = cos(w34);
        row[4] = sin(w34);
        row[5] = cos(w56);
        row[6] = sin(w56);
        row[7] = 0.0;
    }
}

// Pool -> CSR: one wave per pooled segment, dwords copied lane-parallel.
__global__ __launch_bounds__(256) void ccd_scatter(const ccdgpu_segment *pool, const int32_t *seq, int64_t n_pool,
                                                   const int64_t *offsets, const int64_t *chip_pix_off,
                                                   int n_chips, ccdgpu_segment *out) {
    const int64_t s = (int64_t)blockIdx.x * (blockDim.x / W) + threadIdx.x / W;
    if (s >= n_pool) return;
    const int l = threadIdx.x % W;
    const int gp = pool[s].pixel;
    int lo = 0, hi = n_chips - 1;  // chip of the pixel
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (chip_pix_off[mid] <= gp) lo = mid;
        else hi = mid - 1;
    }
    const int64_t dst = offsets[gp] + seq[s];
    const uint32_t *src = reinterpret_cast<const uint32_t *>(pool + s);
    uint32_t *dd = reinterpret_cast<uint32_t *>(out + dst);
    constexpr int NW = (int)(sizeof(ccdgpu_segment) / 4);
    constexpr int PIXW = (int)(offsetof(ccdgpu_segment, pixel) / 4);
    for (int i = l; i < NW; i += W) dd[i] = (i == PIXW) ? (uint32_t)(gp - chip_pix_off[lo]) : src[i];
}

}  // namespace

extern "C" int ccdk_prep(const int64_t *dates, int32_t n_chips, const int32_t *chip_nobs, const int64_t *chip_obs_off,
                         double avg_days_yr, int32_t argsort_stable, int32_t *order, int64_t *sdates, double *basis,
                         void *stream) {
    hipLaunchKernelGGL(ccd_prep, dim3(n_chips), dim3(256), 0, (hipStream_t)stream, dates, chip_nobs,
                       chip_obs_off, avg_days_yr, (int)argsort_stable, order, sdates, basis);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ccdk_set_args(const CcdDetectArgs *host_args, int arg_slot, void *stream) {
    if (arg_slot < 0 || arg_slot >= CCD_ARG_SLOTS) return -1;
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_args), host_args, sizeof(CcdDetectArgs), sizeof(CcdDetectArgs) * (size_t)arg_slot,
                                  hipMemcpyHostToDevice, (hipStream_t)stream) == hipSuccess ? 0 : -1;
}

extern "C" size_t ccdk_lds_bytes(int32_t n_obs) {
    (void)n_obs;
    return sizeof(Lds);
}

static const void *detect_fn(int variant) {
    switch (variant) {
    case 1: return reinterpret_cast<const void *>(&ccd_detect);
    case 2: return reinterpret_cast<const void *>(&ccd_detect_w2);
    case 4: return reinterpret_cast<const void *>(&ccd_detect_w4);
    default: return reinterpret_cast<const void *>(&ccd_detect_w3);
    }
}

// resident waves per CU for this variant and period length (0 on error)
extern "C" int ccdk_occupancy(int variant, int32_t n_obs) {
    const size_t lds = ccdk_lds_bytes(n_obs);
    if (hipFuncSetAttribute(detect_fn(variant), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
        return 0;
    int blocks = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, detect_fn(variant), 64, lds) != hipSuccess) return 0;
    return blocks;
}

extern "C" int ccdk_detect(int32_t grid, int variant, int32_t n_obs, int arg_slot, void *stream) {
    const size_t lds = ccdk_lds_bytes(n_obs);
    if (arg_slot < 0 || arg_slot >= CCD_ARG_SLOTS) return -1;
    switch (variant) {
    case 1: hipLaunchKernelGGL(ccd_detect, dim3(grid), dim3(64), lds, (hipStream_t)stream, arg_slot); break;
    case 2: hipLaunchKernelGGL(ccd_detect_w2, dim3(grid), dim3(64), lds, (hipStream_t)stream, arg_slot); break;
    case 4: hipLaunchKernelGGL(ccd_detect_w4, dim3(grid), dim3(64), lds, (hipStream_t)stream, arg_slot); break;
    default: hipLaunchKernelGGL(ccd_detect_w3, dim3(grid), dim3(64), lds, (hipStream_t)stream, arg_slot); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ccdk_scatter(const ccdgpu_segment *pool, const int32_t *pool_seq, int64_t n_pool,
                            const int64_t *offsets, const int64_t *chip_pix_off, int32_t n_chips,
                            ccdgpu_segment *out, void *stream) {
    if (n_pool <= 0) return 0;
    const int per_block = 256 / W;
    const int64_t blocks = (n_pool + per_block - 1) / per_block;
    hipLaunchKernelGGL(ccd_scatter, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, pool,
                       pool_seq, n_pool, offsets, chip_pix_off, n_chips, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
