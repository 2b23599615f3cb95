// ccdgpu_api.cpp -- host side of the C-ABI declared in include/ccdgpu.h.
//
// Owns device memory and two HIP streams per context.  A detection call = H2D of the chip stacks
// (band-major, observation-contiguous, exactly the layout the Python packer hands over; chips of
// different observation counts packed back to back), the per-chip prep kernel, the persistent
// per-pixel detection kernel, an exclusive scan of the per-pixel segment counts (hipCUB) and the
// pool->CSR scatter, then D2H of the CSR result or of the device-packed table rows.
// Replaces the per-pixel ccd.detect call of ccdc/pyccd.py:168 (see include/ccdgpu.h).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <climits>
#include <cstdint>
#include <chrono>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ccdgpu.h"
#include "ccd_device.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                       \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return fail(CCDGPU_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

template <class T>
struct DevBuf {
    T *p = nullptr;
    size_t cap = 0;  // elements
    int ensure(size_t n) {
        if (n <= cap && p) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        if (hipMalloc(&p, sizeof(T) * (n ? n : 1)) != hipSuccess) {
            p = nullptr;
            return fail(CCDGPU_ENOMEM, "hipMalloc failed (" + std::to_string(sizeof(T) * n) + " bytes)");
        }
        cap = n;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// Page-locked host staging (hipHostMalloc), grown on demand: device-to-host copies into it run as
// one DMA at link speed instead of the runtime's chunked bounce through its own pinned buffers.
struct PinBuf {
    unsigned char *p = nullptr;
    size_t cap = 0;  // bytes
    int ensure(size_t n) {
        if (n <= cap && p) return 0;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        if (hipHostMalloc(reinterpret_cast<void **>(&p), n ? n : 1, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return fail(CCDGPU_ENOMEM, "hipHostMalloc failed (" + std::to_string(n) + " bytes)");
        }
        cap = n;
        return 0;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

double chi2_5_cdf(double x) {
    if (x <= 0) return 0.0;
    return std::erf(std::sqrt(x / 2.0)) - std::sqrt(2.0 * x / M_PI) * std::exp(-x / 2.0) * (1.0 + x / 3.0);
}

// inverse chi-square(5) cdf (change.adjustchgthresh uses scipy chi2.ppf(pt_cg, 5))
double chi2_5_ppf(double p) {
    double lo = 0.0, hi = 400.0;
    for (int i = 0; i < 200; ++i) {
        const double mid = 0.5 * (lo + hi);
        if (chi2_5_cdf(mid) < p) lo = mid;
        else hi = mid;
    }
    return 0.5 * (lo + hi);
}

// constant-memory launch-argument slots (CCD_ARG_SLOTS per process): one per live context
std::mutex g_slot_mu;
unsigned g_slots_used = 0;
int acquire_arg_slot() {
    std::lock_guard<std::mutex> g(g_slot_mu);
    for (int i = 0; i < CCD_ARG_SLOTS; ++i)
        if (!(g_slots_used & (1u << i))) {
            g_slots_used |= 1u << i;
            return i;
        }
    return -1;
}
void release_arg_slot(int i) {
    if (i < 0) return;
    std::lock_guard<std::mutex> g(g_slot_mu);
    g_slots_used &= ~(1u << i);
}

// Shape of a staged batch: per-chip pixel / observation counts and their prefix sums
// (ccd_device.h layout).
struct Shape {
    std::vector<int32_t> npix, nobs;
    std::vector<int64_t> obs_off, pix_off, data_off;  // [n_chips + 1]
    int32_t n_obs_max = 0;
    int n_chips() const { return (int)npix.size(); }
    int64_t total_obs() const { return obs_off.empty() ? 0 : obs_off.back(); }
    int64_t total_pix() const { return pix_off.empty() ? 0 : pix_off.back(); }
    int64_t total_data() const { return data_off.empty() ? 0 : data_off.back(); }
};

int make_shape(int32_t n_chips, const int32_t *n_pix, const int32_t *n_obs, Shape &s) {
    if (n_chips <= 0) return fail(CCDGPU_EINVAL, "n_chips must be > 0");
    if (!n_pix || !n_obs) return fail(CCDGPU_EINVAL, "NULL n_pix / n_obs array");
    s.npix.assign(n_pix, n_pix + n_chips);
    s.nobs.assign(n_obs, n_obs + n_chips);
    s.obs_off.assign(n_chips + 1, 0);
    s.pix_off.assign(n_chips + 1, 0);
    s.data_off.assign(n_chips + 1, 0);
    s.n_obs_max = 0;
    for (int c = 0; c < n_chips; ++c) {
        if (n_pix[c] <= 0) return fail(CCDGPU_EINVAL, "chip " + std::to_string(c) + ": n_pix must be > 0");
        if (n_obs[c] <= 0 || n_obs[c] > CCDGPU_MAX_OBS)
            return fail(CCDGPU_EINVAL, "chip " + std::to_string(c) + ": n_obs must be in [1, " + std::to_string(CCDGPU_MAX_OBS) + "]");
        s.obs_off[c + 1] = s.obs_off[c] + n_obs[c];
        s.pix_off[c + 1] = s.pix_off[c] + n_pix[c];
        s.data_off[c + 1] = s.data_off[c] + (int64_t)n_pix[c] * n_obs[c];
        s.n_obs_max = std::max(s.n_obs_max, n_obs[c]);
    }
    if (s.total_pix() >= (int64_t)1 << 31) return fail(CCDGPU_EINVAL, "more than 2^31 - 1 pixels in one batch");
    return 0;
}

// One upload stream per device shared by every context (unless CCDGPU_SHARED_UPLOADS=0):
// the host-to-device copies of all contexts then run one after another in the order they were
// staged -- the order their detections need them -- instead of side by side on separate DMA
// queues, where every upload in flight shares the link and each finishes late.  Created on first
// use, kept for the process's lifetime.
std::mutex g_up_mu;
hipStream_t g_up_stream[64] = {};
hipStream_t shared_upload_stream(int device) {
    if (device < 0 || device >= 64) return nullptr;
    std::lock_guard<std::mutex> g(g_up_mu);
    if (!g_up_stream[device] && hipStreamCreateWithFlags(&g_up_stream[device], hipStreamNonBlocking) != hipSuccess)
        g_up_stream[device] = nullptr;
    return g_up_stream[device];
}

}  // namespace

struct ccdgpu_ctx {
    int device = 0;
    int n_cu = 0;
    int slots_per_cu = 0;
    int variant = 4;  // detection kernel register budget: 1..4 waves/SIMD (CCDGPU_KERNEL=w1..w4)
    int poison = 0;   // CCDGPU_POISON=1: LDS and slot scratch filled with NaN bytes per pixel (test mode)
    int arg_slot = -1;  // this context's launch-argument slot in constant memory
    hipStream_t stream = nullptr;
    hipStream_t copy_stream = nullptr;  // uploads of ccdgpu_stage_slot (overlap a running detection)
    hipStream_t up_stream = nullptr;    // where the slot uploads go: copy_stream, or the device's shared one
    // every other kernel and copy of a launch (prep, CSR scan and scatter, row packing, small
    // copies): the detection stream itself, or -- with CUs reserved (ccdgpu_init_copy_cus) -- a
    // stream on the reserved CUs, so these short kernels never wait for wave slots behind
    // persistent detection waves; only the detection kernel then runs on `stream`
    hipStream_t aux = nullptr;
    bool aux_own = false;
    hipEvent_t uploaded[CCDGPU_UPLOAD_SLOTS] = {};
    // inputs the next detection reads: the single staged batch, or one of the two upload slots
    const int64_t *in_dates = nullptr;
    const int16_t *in_spectra = nullptr;
    const uint16_t *in_qa = nullptr;
    const unsigned char *in_enc = nullptr;  // a transport-encoded batch the kernel reads in place
    // decode encoded uploads into the standard layout first (CCDGPU_DECODE=1: the round-3 path, A/B)
    bool decode_enc = false;
    bool rows_fused = true;   // CCDGPU_ROWS_FUSED=0 (A/B): the separate scatter and per-chip row packing
    bool keep_slots = false;  // CCDGPU_KEEP_SLOTS=1 (measurement only, tools/overlap_test.py): a slot stays staged after its run
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    // the host waits for a detection through this event: blocking (the waiting thread sleeps on
    // the completion interrupt instead of polling), so the tile driver's waiting workers leave the
    // host's CPUs to its fetch / encode threads
    hipEvent_t done = nullptr;
    // staged batch
    bool staged = false, ran = false;
    ccdgpu_params params{};
    Shape shape;
    int32_t mask_words = 0, n_slots = 0;
    int64_t total_pix = 0, pool_cap = 0, n_pool = 0;
    // initial segment-pool room per pixel (CCDGPU_POOL_PER_PIXEL, test knob: a small pool makes
    // every change-dense batch take the overflow rerun) and the reruns of the last run
    int pool_per_pixel = 8;
    int64_t pool_reruns = 0;
    DevBuf<int64_t> dates, sdates, offsets;
    DevBuf<int16_t> spectra;
    DevBuf<uint16_t> qa;
    DevBuf<int32_t> order, procedure, nseg, pool_seq, chip_nobs;
    DevBuf<int64_t> chip_obs_off, chip_pix_off, chip_data_off;
    DevBuf<double> basis, probs, s_f64;
    DevBuf<unsigned long long> counters, stats;
    DevBuf<int32_t> s_date;
    DevBuf<uint16_t> s_row;
    DevBuf<uint16_t> s_bk;
    DevBuf<uint32_t> mask;
    DevBuf<ccdgpu_segment> pool, csr;
    DevBuf<unsigned char> cub_tmp;
    DevBuf<ccdgpu_row> rows;    // output writer scratch (ccdgpu_fetch_rows / ccdgpu_fetch_batch_rows)
    DevBuf<int64_t> row_off, seg_off1;
    DevBuf<int32_t> row_xy;     // per-chip (cx, cy) of a batch row fetch
    DevBuf<int8_t> mask8;
    PinBuf h_rows;              // pinned landing zone of a batch row fetch (rows, then mask words)
    // pinned staging of every launch's small host <-> device copies (initial counters, kernel
    // arguments, counters and statistics read back, CSR offsets): DMA from / to pinned memory,
    // where pageable memory would go through a runtime staging copy -- a blit kernel that has to
    // wait for free CUs while other contexts' detection kernels hold them all
    PinBuf h_small, h_off, h_tab, h_fo, h_xy;  // (h_tab: chip tables of a launch; h_fo: row-fetch offsets)
    DevBuf<int64_t> slot_dates[CCDGPU_UPLOAD_SLOTS];   // upload slots (ccdgpu_stage_slot / ccdgpu_run_slot)
    DevBuf<int16_t> slot_spectra[CCDGPU_UPLOAD_SLOTS];
    DevBuf<uint16_t> slot_qa[CCDGPU_UPLOAD_SLOTS];
    DevBuf<unsigned char> slot_enc[CCDGPU_UPLOAD_SLOTS];  // transport-encoded uploads (ccdgpu_stage_slot_encoded)
    Shape slot_shape[CCDGPU_UPLOAD_SLOTS];
    ccdgpu_params slot_params[CCDGPU_UPLOAD_SLOTS];
    bool slot_ready[CCDGPU_UPLOAD_SLOTS] = {};
    bool slot_encoded[CCDGPU_UPLOAD_SLOTS] = {};  // the slot holds an encoded batch read in place
    DevBuf<unsigned char> b64;  // chipmunk payload text of the last ccdgpu_stage_chipmunk
    DevBuf<int64_t> b64_off;
    std::vector<int64_t> h_offsets;
    ccdgpu_stats last{};
    unsigned long long diag[CCD_NSTATS] = {};
    // a detection launched by ccdgpu_run_slot_begin and not yet finished by ccdgpu_run_slot_end
    bool pending = false;
    int32_t pend_slot = -1;  // the upload slot that detection reads (not to be restaged until it ends)
    CcdDetectArgs pend_args{};
    // the batch chain of ccdgpu_run_slot_begin_rows: CSR, row packing and the copies of rows,
    // row offsets and mask words into the caller's (pinned) buffers, enqueued behind the
    // detection; `done_rows` marks the end of the chain
    bool rows_mode = false;
    int64_t *rq_offsets = nullptr, *rq_seg = nullptr;
    ccdgpu_row *rq_rows = nullptr;
    uint32_t *rq_mask = nullptr;
    int64_t rq_offsets_cap = 0, rq_rows_cap = 0, rq_mask_cap = 0;
    int32_t rq_width = 100;
    std::vector<int32_t> rq_cx, rq_cy;
    DevBuf<int64_t> rowcnt;
    hipEvent_t done_rows = nullptr;
    ~ccdgpu_ctx() {
        for (auto *b : {&dates, &sdates, &offsets, &chip_obs_off, &chip_pix_off, &chip_data_off, &row_off, &seg_off1, &b64_off})
            b->release();
        spectra.release();
        qa.release();
        for (auto *b : {&order, &procedure, &nseg, &pool_seq, &s_date, &chip_nobs, &row_xy}) b->release();
        for (auto *b : {&basis, &probs, &s_f64}) b->release();
        counters.release();
        stats.release();
        s_row.release();
        s_bk.release();
        mask.release();
        pool.release();
        csr.release();
        cub_tmp.release();
        b64.release();
        for (int i = 0; i < CCDGPU_UPLOAD_SLOTS; ++i) {
            slot_dates[i].release();
            slot_spectra[i].release();
            slot_qa[i].release();
            slot_enc[i].release();
            if (uploaded[i]) (void)hipEventDestroy(uploaded[i]);
        }
        if (copy_stream) (void)hipStreamDestroy(copy_stream);
        rows.release();
        mask8.release();
        h_rows.release();
        h_small.release();
        h_off.release();
        h_tab.release();
        h_fo.release();
        h_xy.release();
        if (aux_own && aux) (void)hipStreamDestroy(aux);
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        if (done) (void)hipEventDestroy(done);
        if (done_rows) (void)hipEventDestroy(done_rows);
        rowcnt.release();
        if (stream) (void)hipStreamDestroy(stream);
        release_arg_slot(arg_slot);
    }
};

extern "C" {

const char *ccdgpu_version(void) { return "ccdgpu 0.2.0 (gfx950; lcmap-pyccd:2018.03.12.dev-ncompare.b2 semantics)"; }

const char *ccdgpu_last_error(void) { return g_err.c_str(); }

void ccdgpu_params_default(ccdgpu_params *p) {
    std::memset(p, 0, sizeof(*p));
    p->meow_size = 12;
    p->peek_size = 6;
    p->day_delta = 365;
    p->coef_min = 4;
    p->coef_mid = 6;
    p->coef_max = 8;
    p->num_obs_factor = 3;
    p->detection_bands = 0x3E;
    p->tmask_bands = 0x12;
    p->lasso_max_iter = 1000;
    p->thermal_min = -9320;
    p->thermal_max = 7070;
    p->median_green_filter = 400;
    p->curve_qa_start = 14;
    p->curve_qa_end = 24;
    p->curve_qa_insuf_clear = 44;
    p->curve_qa_persist_snow = 54;
    p->qa_fill = 0;
    p->qa_clear = 1;
    p->qa_water = 2;
    p->qa_shadow = 3;
    p->qa_snow = 4;
    p->qa_cloud = 5;
    p->qa_cirrus1 = 8;
    p->qa_cirrus2 = 9;
    p->qa_occlusion = 10;
    p->qa_bitpacked = 1;
    p->adaptive_peek = 1;
    p->rmse_dof = 0;
    p->kelvin_to_celsius = 1;
    p->avg_days_yr = 365.2425;
    p->change_probability = 0.99;
    p->change_threshold = 15.086272469388987;
    p->outlier_threshold = 35.888186879610423;
    p->t_const = 4.42;
    p->lasso_alpha = 1.0;
    p->lasso_tol = 1e-4;
    p->clear_pct_threshold = 0.25;
    p->snow_pct_threshold = 0.75;
    p->argsort_stable = 0;  // numpy quicksort tie order (include/ccdgpu.h)
    p->reserved0 = 0;
}

int ccdgpu_device_count(int *count) {
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *count = 0;
        return fail(CCDGPU_EHIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *count = c;
    return 0;
}

int ccdgpu_device_numa_node(int device, int *node) {
    if (!node) return fail(CCDGPU_EINVAL, "node out pointer is NULL");
    *node = -1;
    char bus[64] = {0};
    HIPCHK(hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, device));
    for (char *q = bus; *q; ++q) *q = (char)std::tolower((unsigned char)*q);
    const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
    FILE *f = std::fopen(path.c_str(), "r");
    if (!f) return 0;  // not exposed: unknown
    int v = -1;
    if (std::fscanf(f, "%d", &v) != 1) v = -1;
    std::fclose(f);
    *node = v;
    return 0;
}

int ccdgpu_init(int device, ccdgpu_ctx **out) { return ccdgpu_init_copy_cus(device, 0, out); }

int ccdgpu_init_copy_cus(int device, int copy_cus, ccdgpu_ctx **out) {
    if (!out) return fail(CCDGPU_EINVAL, "ctx out pointer is NULL");
    if (copy_cus < 0) return fail(CCDGPU_EINVAL, "copy_cus must be >= 0");
    *out = nullptr;
    int count = 0;
    int rc = ccdgpu_device_count(&count);
    if (rc) return rc;
    if (device < 0 || device >= count)
        return fail(CCDGPU_EINVAL, "device " + std::to_string(device) + " out of range (" + std::to_string(count) + " visible)");
    HIPCHK(hipSetDevice(device));
    auto *c = new ccdgpu_ctx();
    c->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) {
        delete c;
        return fail(CCDGPU_EHIP, "hipGetDeviceProperties failed");
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        std::string arch = prop.gcnArchName;
        delete c;
        return fail(CCDGPU_EHIP, "device " + std::to_string(device) + " is " + arch + ", libccdgpu is built for gfx950 only");
    }
    c->n_cu = prop.multiProcessorCount;
    // copy_cus = k > 0: the copy stream (uploads' decode kernel, blits) gets k CUs of its own --
    // the same k for every context -- and the detection stream the rest, so a context's upload is
    // never starved of CUs by other contexts' persistent detection waves (which otherwise hold
    // every wave slot until their launch drains).  The mask bits are the last ceil(k / 8) of each
    // run of n_cu / 8.  The driver maps mask bit i to XCD i % 8 (the i / 8-th CU of that XCD,
    // shader engines interleaved; tools/probe/cu_mask.hip, profiles/r04/cu_mask_probe.txt), so for
    // k = 8 these are one shader engine of XCD 7: the detection stream runs on the other 248 CUs,
    // and the copy / aux streams -- whose masks are empty on XCDs 0-6, which the hardware treats
    // as unrestricted -- have those 8 CUs to themselves and share the rest.  The truly
    // interleaved reservation (ceil(k / 8) CUs on every XCD and nothing else for the copy
    // streams, CCDGPU_MASK_INTERLEAVED=1) measured slower: one context's detection 2.29M vs
    // 2.44M px/s (the same as with no reservation), four contexts with the batch chain 2.62M vs
    // 2.72M (profiles/r04/cu_layout_ab.txt).  CCDGPU_COPY_CUS overrides k (experiments).
    if (const char *e = std::getenv("CCDGPU_COPY_CUS")) copy_cus = std::max(0, std::atoi(e));
    const char *mi = std::getenv("CCDGPU_MASK_INTERLEAVED");
    const bool blocked = !(mi && std::atoi(mi) != 0);
    std::vector<uint32_t> mask_det, mask_copy;
    if (copy_cus > 0 && copy_cus < c->n_cu) {
        const int nw = (c->n_cu + 31) / 32, groups = 8, per = c->n_cu / groups;
        // at least one CU of every group stays with the detection stream, and at least one is reserved
        const int k = std::min((copy_cus + groups - 1) / groups, per - 1);
        if (per < 2 || k < 1) {
            const std::string msg = "copy_cus " + std::to_string(copy_cus) + " leaves no CU for detection or copies on " +
                                    std::to_string(c->n_cu) + " CUs";
            delete c;
            return fail(CCDGPU_EINVAL, msg);
        }
        mask_det.assign(nw, 0u);
        mask_copy.assign(nw, 0u);
        for (int cu = 0; cu < c->n_cu; ++cu) {
            const bool reserved = blocked ? (cu % per) >= per - k : cu >= c->n_cu - groups * k;
            (reserved ? mask_copy : mask_det)[cu / 32] |= 1u << (cu % 32);
        }
    }
    const bool masked = !mask_det.empty();
    if ((masked ? hipExtStreamCreateWithCUMask(&c->stream, (uint32_t)mask_det.size(), mask_det.data())
                : hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
        delete c;
        return fail(CCDGPU_EHIP, "hipStreamCreate failed");
    }
    for (auto &e : c->ev) (void)hipEventCreate(&e);
    (void)hipEventCreateWithFlags(&c->done, hipEventBlockingSync | hipEventDisableTiming);
    (void)hipEventCreateWithFlags(&c->done_rows, hipEventBlockingSync | hipEventDisableTiming);
    if ((masked ? hipExtStreamCreateWithCUMask(&c->copy_stream, (uint32_t)mask_copy.size(), mask_copy.data())
                : hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking)) != hipSuccess) {
        delete c;
        return fail(CCDGPU_EHIP, "hipStreamCreate failed");
    }
    for (auto &e : c->uploaded) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    // uploads in staging order on the device's shared stream (default; CCDGPU_SHARED_UPLOADS=0:
    // each context's own copy stream).  Tile leg A/B: 2.50 / 2.62M vs 2.42 / 2.50M px/s
    // (profiles/r04/tile_knobs.json).
    c->up_stream = c->copy_stream;
    {
        const char *v = std::getenv("CCDGPU_SHARED_UPLOADS");
        if (!v || std::atoi(v) != 0) {
            hipStream_t sh = shared_upload_stream(device);
            if (sh) c->up_stream = sh;
        }
    }
    c->aux = c->stream;
    if (masked) {
        if (hipExtStreamCreateWithCUMask(&c->aux, (uint32_t)mask_copy.size(), mask_copy.data()) != hipSuccess) {
            c->aux = nullptr;
            delete c;
            return fail(CCDGPU_EHIP, "hipStreamCreate failed");
        }
        c->aux_own = true;
    } else if (const char *v = std::getenv("CCDGPU_AUX_PRIORITY")) {
        // no CUs reserved: the launch's other kernels on a high-priority stream of their own, so the
        // dispatcher serves them ahead of waiting detection waves (experiment knob)
        if (std::atoi(v) != 0) {
            int lo = 0, hi = 0;
            if (hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess &&
                hipStreamCreateWithPriority(&c->aux, hipStreamNonBlocking, hi) == hipSuccess)
                c->aux_own = true;
            else
                c->aux = c->stream;
        }
    }
    c->arg_slot = acquire_arg_slot();
    if (c->arg_slot < 0) {
        delete c;
        return fail(CCDGPU_EINVAL, "more than " + std::to_string(CCD_ARG_SLOTS) + " live contexts in this process");
    }
    c->slots_per_cu = 16;
    c->variant = 4;
    if (const char *v = std::getenv("CCDGPU_KERNEL")) {
        if (v[0] == 'w' && v[1] >= '1' && v[1] <= '4' && v[2] == 0) c->variant = v[1] - '0';
    }
    if (const char *v = std::getenv("CCDGPU_SLOTS_PER_CU")) c->slots_per_cu = std::max(1, std::atoi(v));
    if (const char *v = std::getenv("CCDGPU_POISON")) c->poison = std::atoi(v) != 0;
    if (const char *v = std::getenv("CCDGPU_DECODE")) c->decode_enc = std::atoi(v) != 0;
    if (const char *v = std::getenv("CCDGPU_ROWS_FUSED")) c->rows_fused = std::atoi(v) != 0;
    if (const char *v = std::getenv("CCDGPU_KEEP_SLOTS")) c->keep_slots = std::atoi(v) != 0;
    if (const char *v = std::getenv("CCDGPU_POOL_PER_PIXEL")) c->pool_per_pixel = std::max(1, std::atoi(v));
    *out = c;
    return 0;
}

int ccdgpu_destroy(ccdgpu_ctx *ctx) {
    if (!ctx) return 0;
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamSynchronize(ctx->copy_stream);
    if (ctx->up_stream && ctx->up_stream != ctx->copy_stream) (void)hipStreamSynchronize(ctx->up_stream);
    if (ctx->aux) (void)hipStreamSynchronize(ctx->aux);
    delete ctx;
    return 0;
}

int ccdgpu_synchronize(ccdgpu_ctx *ctx) {
    if (!ctx) return fail(CCDGPU_EINVAL, "NULL ctx");
    HIPCHK(hipSetDevice(ctx->device));
    HIPCHK(hipDeviceSynchronize());
    return 0;
}

static int check_params(const ccdgpu_params *p) {
    if (!p) return fail(CCDGPU_EINVAL, "params is NULL");
    if (p->peek_size < 1 || p->peek_size > CCDGPU_MAX_PEEK)
        return fail(CCDGPU_EINVAL, "peek_size must be in [1, " + std::to_string(CCDGPU_MAX_PEEK) + "]");
    if (p->meow_size < 5) return fail(CCDGPU_EINVAL, "meow_size must be >= 5 (Tmask needs > 4 observations)");
    if (p->coef_min != 4 && p->coef_min != 6 && p->coef_min != 8)
        return fail(CCDGPU_EINVAL, "coefficient counts must be 4, 6 or 8");
    if ((p->coef_mid != 4 && p->coef_mid != 6 && p->coef_mid != 8) || (p->coef_max != 4 && p->coef_max != 6 && p->coef_max != 8))
        return fail(CCDGPU_EINVAL, "coefficient counts must be 4, 6 or 8");
    if (p->lasso_max_iter < 1) return fail(CCDGPU_EINVAL, "lasso_max_iter must be >= 1");
    if ((p->detection_bands & ~0x7Fu) || (p->tmask_bands & ~0x7Fu))
        return fail(CCDGPU_EINVAL, "band masks must only use bits 0..6");
    if (p->argsort_stable != 0 && p->argsort_stable != 1) return fail(CCDGPU_EINVAL, "argsort_stable must be 0 or 1");
    return 0;
}

// Device buffers of a staged batch (chip tables, per-slot scratch, outputs) and, with
// base_inputs, the input buffers plus the dates upload; the pixel data are filled by the caller
// (a plain upload or the chipmunk decoder).
static int stage_alloc(ccdgpu_ctx *c, const ccdgpu_params *params, const Shape &sh, const int64_t *dates,
                       bool base_inputs = true) {
    if (!c) return fail(CCDGPU_EINVAL, "NULL ctx");
    int rc = check_params(params);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    c->staged = false;
    c->params = *params;
    c->shape = sh;
    const int nc = sh.n_chips();
    c->mask_words = (sh.n_obs_max + 31) / 32;
    c->total_pix = sh.total_pix();
    const size_t tobs = (size_t)sh.total_obs(), tdata = (size_t)sh.total_data();
    if (base_inputs && ((rc = c->dates.ensure(tobs)) || (rc = c->spectra.ensure(7 * tdata)) || (rc = c->qa.ensure(tdata))))
        return rc;
    if ((rc = c->order.ensure(tobs)) || (rc = c->sdates.ensure(tobs)) || (rc = c->basis.ensure(tobs * CCD_BASIS_STRIDE)) ||
        (rc = c->chip_nobs.ensure(nc)) || (rc = c->chip_obs_off.ensure(nc + 1)) || (rc = c->chip_pix_off.ensure(nc + 1)) ||
        (rc = c->chip_data_off.ensure(nc + 1)) ||
        (rc = c->procedure.ensure(c->total_pix)) || (rc = c->nseg.ensure(c->total_pix)) ||
        (rc = c->probs.ensure(3 * c->total_pix)) || (rc = c->offsets.ensure(c->total_pix + 1)) ||
        (rc = c->mask.ensure((size_t)c->total_pix * c->mask_words)) || (rc = c->counters.ensure(8)) ||
        (rc = c->stats.ensure(CCD_NSTATS)))
        return rc;
    // persistent grid: one wave slot per resident wave (LDS / register occupancy), capped by
    // CCDGPU_SLOTS_PER_CU
    const int occ = ccdk_occupancy(c->variant, sh.n_obs_max);
    if (occ <= 0) return fail(CCDGPU_EHIP, "detection kernel cannot be resident with " + std::to_string(ccdk_lds_bytes(sh.n_obs_max)) + " B of LDS");
    c->n_slots = (int32_t)std::min<int64_t>(c->total_pix, (int64_t)c->n_cu * std::min(occ, c->slots_per_cu));
    const size_t ns = (size_t)c->n_slots, no = (size_t)sh.n_obs_max;
    const size_t nper = ns * no;  // the compacted periods (dates, 16-byte rows) per slot
    if ((rc = c->s_date.ensure(nper)) || (rc = c->s_row.ensure(nper * 8)) ||
        (rc = c->s_f64.ensure(ns * CCD_SLOT_F64(no))) || (rc = c->s_bk.ensure(ns * no)))
        return rc;
    if (c->pool_cap < c->total_pix * c->pool_per_pixel) c->pool_cap = c->total_pix * c->pool_per_pixel;
    c->pool_reruns = 0;
    if ((rc = c->pool.ensure(c->pool_cap)) || (rc = c->pool_seq.ensure(c->pool_cap))) return rc;
    // chip tables, through the context's pinned staging (DMA, no runtime staging copy), on the
    // aux stream that runs the launch's prep; the previous launch's table copies are done
    HIPCHK(hipStreamSynchronize(c->aux));
    const size_t t8 = 8 * ((size_t)nc + 1);
    if ((rc = c->h_tab.ensure(3 * t8 + 4 * (size_t)nc))) return rc;
    unsigned char *ht = c->h_tab.p;
    std::memcpy(ht, sh.obs_off.data(), t8);
    std::memcpy(ht + t8, sh.pix_off.data(), t8);
    std::memcpy(ht + 2 * t8, sh.data_off.data(), t8);
    std::memcpy(ht + 3 * t8, sh.nobs.data(), 4 * (size_t)nc);
    HIPCHK(hipMemcpyAsync(c->chip_obs_off.p, ht, t8, hipMemcpyHostToDevice, c->aux));
    HIPCHK(hipMemcpyAsync(c->chip_pix_off.p, ht + t8, t8, hipMemcpyHostToDevice, c->aux));
    HIPCHK(hipMemcpyAsync(c->chip_data_off.p, ht + 2 * t8, t8, hipMemcpyHostToDevice, c->aux));
    HIPCHK(hipMemcpyAsync(c->chip_nobs.p, ht + 3 * t8, 4 * (size_t)nc, hipMemcpyHostToDevice, c->aux));
    if (dates) HIPCHK(hipMemcpyAsync(c->dates.p, dates, sizeof(int64_t) * tobs, hipMemcpyHostToDevice, c->aux));
    c->in_dates = c->dates.p;
    c->in_spectra = c->spectra.p;
    c->in_qa = c->qa.p;
    c->in_enc = nullptr;
    return 0;
}

static void uniform(int32_t n_chips, int32_t n_pix, int32_t n_obs, std::vector<int32_t> &np, std::vector<int32_t> &no) {
    np.assign(n_chips > 0 ? n_chips : 0, n_pix);
    no.assign(n_chips > 0 ? n_chips : 0, n_obs);
}

int ccdgpu_stage_chips(ccdgpu_ctx *c, const ccdgpu_params *params, int32_t n_chips, const int32_t *n_pix,
                       const int32_t *n_obs, const int64_t *dates, const int16_t *spectra, const uint16_t *qa) {
    if (!dates || !spectra || !qa) return fail(CCDGPU_EINVAL, "NULL input buffer");
    Shape sh;
    int rc = make_shape(n_chips, n_pix, n_obs, sh);
    if (rc) return rc;
    if ((rc = stage_alloc(c, params, sh, dates))) return rc;
    const size_t tdata = (size_t)sh.total_data();
    HIPCHK(hipMemcpyAsync(c->spectra.p, spectra, sizeof(int16_t) * 7 * tdata, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->qa.p, qa, sizeof(uint16_t) * tdata, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->staged = true;
    c->ran = false;
    return 0;
}

int ccdgpu_stage(ccdgpu_ctx *c, const ccdgpu_params *params, int32_t n_chips, int32_t n_pix, int32_t n_obs,
                 const int64_t *dates, const int16_t *spectra, const uint16_t *qa) {
    std::vector<int32_t> np, no;
    uniform(n_chips, n_pix, n_obs, np, no);
    return ccdgpu_stage_chips(c, params, n_chips, np.data(), no.data(), dates, spectra, qa);
}

int ccdgpu_stage_chipmunk(ccdgpu_ctx *c, const ccdgpu_params *params, int32_t n_chips, int32_t n_pix, int32_t n_obs,
                          const int64_t *dates, const char *text, int64_t text_bytes, const int64_t *text_offsets,
                          double *unpack_seconds) {
    if (!dates || !text || !text_offsets || text_bytes < 0) return fail(CCDGPU_EINVAL, "NULL or empty chipmunk text");
    if (n_pix <= 0 || n_pix > (1 << 24)) return fail(CCDGPU_EINVAL, "n_pix out of range");
    if (n_chips <= 0 || n_obs <= 0) return fail(CCDGPU_EINVAL, "n_chips and n_obs must be > 0");
    // Every present payload is exactly the encoded length of n_pix 16-bit values ('=' padded):
    // it must lie inside the text and must not run into the next payload (a truncated payload
    // would otherwise decode its successor's characters as its own tail).
    const int64_t enc = 4 * (((int64_t)2 * n_pix + 2) / 3);
    const int64_t n_off = (int64_t)n_chips * n_obs * 8;
    std::vector<std::pair<int64_t, int64_t>> present;
    present.reserve((size_t)n_off);
    for (int64_t i = 0; i < n_off; ++i) {
        const int64_t o = text_offsets[i];
        if (o < 0) continue;
        if (o + enc > text_bytes)
            return fail(CCDGPU_EINVAL, "chipmunk payload " + std::to_string(i) + " runs past the end of the text");
        present.emplace_back(o, i);
    }
    std::sort(present.begin(), present.end());
    for (size_t k = 0; k + 1 < present.size(); ++k)
        if (present[k + 1].first - present[k].first < enc)
            return fail(CCDGPU_EINVAL, "chipmunk payload " + std::to_string(present[k].second) + " is shorter than " +
                                           std::to_string(enc) + " bytes (" + std::to_string(n_pix) + " values)");
    std::vector<int32_t> np, no;
    uniform(n_chips, n_pix, n_obs, np, no);
    Shape sh;
    int rc = make_shape(n_chips, np.data(), no.data(), sh);
    if (rc) return rc;
    if ((rc = stage_alloc(c, params, sh, dates))) return rc;
    if ((rc = c->b64.ensure((size_t)text_bytes + 8)) || (rc = c->b64_off.ensure((size_t)n_off))) return rc;
    HIPCHK(hipMemcpyAsync(c->b64.p, text, (size_t)text_bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(c->b64_off.p, text_offsets, sizeof(int64_t) * (size_t)n_off, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(c->counters.p, 0, sizeof(unsigned long long) * 8, c->stream));
    HIPCHK(hipEventRecord(c->ev[0], c->stream));
    if (ccdk_unpack_b64(c->b64.p, text_bytes, c->b64_off.p, n_chips, n_obs, n_pix, c->spectra.p, c->qa.p,
                        c->counters.p + 5, c->stream))
        return fail(CCDGPU_EHIP, std::string("unpack launch: ") + hipGetErrorString(hipGetLastError()));
    HIPCHK(hipEventRecord(c->ev[1], c->stream));
    unsigned long long err = 0;
    HIPCHK(hipMemcpyAsync(&err, c->counters.p + 5, sizeof(err), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, c->ev[0], c->ev[1]);
    if (unpack_seconds) *unpack_seconds = ms * 1e-3;
    if (err) return fail(CCDGPU_EINVAL, "chipmunk payload is not valid base64");
    c->staged = true;
    c->ran = false;
    return 0;
}

int ccdgpu_host_alloc(size_t bytes, void **ptr) {
    if (!ptr) return fail(CCDGPU_EINVAL, "NULL ptr");
    *ptr = nullptr;
    if (hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        *ptr = nullptr;
        return fail(CCDGPU_ENOMEM, "hipHostMalloc failed (" + std::to_string(bytes) + " bytes)");
    }
    return 0;
}

int ccdgpu_host_free(void *ptr) {
    if (ptr) HIPCHK(hipHostFree(ptr));
    return 0;
}

int ccdgpu_stage_slot_chips(ccdgpu_ctx *c, int32_t slot, const ccdgpu_params *params, int32_t n_chips,
                            const int32_t *n_pix, const int32_t *n_obs, const int64_t *dates, const int16_t *spectra,
                            const uint16_t *qa) {
    if (!c) return fail(CCDGPU_EINVAL, "NULL ctx");
    if (slot < 0 || slot >= CCDGPU_UPLOAD_SLOTS)
        return fail(CCDGPU_EINVAL, "slot must be in 0 .. " + std::to_string(CCDGPU_UPLOAD_SLOTS - 1));
    if (c->pending && slot == c->pend_slot)
        return fail(CCDGPU_EINVAL, "slot " + std::to_string(slot) + " is read by the detection begun with ccdgpu_run_slot_begin");
    if (!dates || !spectra || !qa) return fail(CCDGPU_EINVAL, "NULL input buffer");
    Shape sh;
    int rc = make_shape(n_chips, n_pix, n_obs, sh);
    if (rc || (rc = check_params(params))) return rc;
    HIPCHK(hipSetDevice(c->device));
    const size_t tobs = (size_t)sh.total_obs(), tdata = (size_t)sh.total_data();
    if ((rc = c->slot_dates[slot].ensure(tobs)) || (rc = c->slot_spectra[slot].ensure(7 * tdata)) ||
        (rc = c->slot_qa[slot].ensure(tdata)))
        return rc;
    // the slot's previous batch was detected by a ccdgpu_run_slot that has returned, so the
    // uploads may overwrite it; they run on the copy stream, concurrent with any detection
    HIPCHK(hipMemcpyAsync(c->slot_dates[slot].p, dates, sizeof(int64_t) * tobs, hipMemcpyHostToDevice, c->up_stream));
    HIPCHK(hipMemcpyAsync(c->slot_spectra[slot].p, spectra, sizeof(int16_t) * 7 * tdata, hipMemcpyHostToDevice, c->up_stream));
    HIPCHK(hipMemcpyAsync(c->slot_qa[slot].p, qa, sizeof(uint16_t) * tdata, hipMemcpyHostToDevice, c->up_stream));
    HIPCHK(hipEventRecord(c->uploaded[slot], c->up_stream));
    c->slot_shape[slot] = sh;
    c->slot_params[slot] = *params;  // each slot keeps its own parameters
    c->slot_ready[slot] = true;
    c->slot_encoded[slot] = false;
    return 0;
}

int ccdgpu_encoded_check(int32_t n_chips, const int32_t *n_pix, const int32_t *n_obs, const uint8_t *enc,
                         int64_t enc_bytes) {
    if (!enc || !n_pix || !n_obs || n_chips <= 0) return fail(CCDGPU_EINVAL, "NULL or empty encoded batch");
    // the encoded batch must describe exactly these chips (the decoder trusts its headers)
    const int64_t *tab = reinterpret_cast<const int64_t *>(enc);
    if (enc_bytes < (int64_t)(8 * (2 * (int64_t)n_chips + 3)) || tab[0] != n_chips)
        return fail(CCDGPU_EINVAL, "encoded batch: chip table does not match n_chips");
    const int64_t *off = tab + 1, *pixo = tab + 2 + n_chips;
    if (off[n_chips] > enc_bytes) return fail(CCDGPU_EINVAL, "encoded batch: longer than enc_bytes");
    int64_t pb = 0, db = 0;
    for (int32_t k = 0; k < n_chips; ++k) {
        if (n_pix[k] <= 0 || n_obs[k] <= 0 || n_obs[k] > CCDGPU_MAX_OBS)
            return fail(CCDGPU_EINVAL, "encoded batch: chip " + std::to_string(k) + " has no pixels / observations");
        if (off[k] < 0 || off[k] + 128 > off[k + 1] || pixo[k] != pb)
            return fail(CCDGPU_EINVAL, "encoded batch: bad chip table entry " + std::to_string(k));
        const int32_t *h = reinterpret_cast<const int32_t *>(enc + off[k]);
        const int64_t *h64 = reinterpret_cast<const int64_t *>(enc + off[k] + 48);
        if ((h[0] != 0 && h[0] != 1) || h[1] != n_pix[k] || h[2] != n_obs[k] || h64[1] != db ||
            (h[0] == 1 && (h[3] < 1 || h[3] > 16)))
            return fail(CCDGPU_EINVAL, "encoded batch: chip " + std::to_string(k) + " header does not match its shape");
        // the section holds everything its mode's layout addresses (the decoder trusts it)
        const int64_t np_ = n_pix[k], no_ = n_obs[k], plane = np_ * no_, sec = off[k + 1] - off[k];
        auto up_ = [](int64_t x, int64_t a) { return (x + a - 1) / a * a; };
        if (h[0] == 0) {
            if (sec < 128 + up_(2 * plane, 16) + 14 * plane)
                return fail(CCDGPU_EINVAL, "encoded batch: chip " + std::to_string(k) + " raw section is truncated");
        } else {
            const int64_t kept = h64[0], bstride = h64[2];
            const int64_t bands_at = 128 + up_(4 * (np_ + 1), 16) + up_(np_ * ((no_ + 1) / 2), 16);
            if (kept < 0 || kept > plane || bstride < kept || bstride % 8 != 0 || sec < bands_at + 14 * bstride)
                return fail(CCDGPU_EINVAL, "encoded batch: chip " + std::to_string(k) + " band columns do not fit its section");
            const uint32_t *koff = reinterpret_cast<const uint32_t *>(enc + off[k] + 128);
            if (koff[0] != 0 || (int64_t)koff[np_] != kept)
                return fail(CCDGPU_EINVAL, "encoded batch: chip " + std::to_string(k) + " kept-offset table does not end at kept");
            for (int64_t q = 0; q < np_; ++q)
                if (koff[q + 1] < koff[q] || (int64_t)(koff[q + 1] - koff[q]) > no_)
                    return fail(CCDGPU_EINVAL, "encoded batch: chip " + std::to_string(k) + " kept-offset table is not a run per pixel");
        }
        pb += n_pix[k];
        db += (int64_t)n_pix[k] * n_obs[k];
    }
    if (pixo[n_chips] != pb) return fail(CCDGPU_EINVAL, "encoded batch: pixel total does not match");
    return 0;
}

int ccdgpu_stage_slot_encoded(ccdgpu_ctx *c, int32_t slot, const ccdgpu_params *params, int32_t n_chips,
                              const int32_t *n_pix, const int32_t *n_obs, const int64_t *dates, const uint8_t *enc,
                              int64_t enc_bytes) {
    if (!c) return fail(CCDGPU_EINVAL, "NULL ctx");
    if (slot < 0 || slot >= CCDGPU_UPLOAD_SLOTS)
        return fail(CCDGPU_EINVAL, "slot must be in 0 .. " + std::to_string(CCDGPU_UPLOAD_SLOTS - 1));
    if (c->pending && slot == c->pend_slot)
        return fail(CCDGPU_EINVAL, "slot " + std::to_string(slot) + " is read by the detection begun with ccdgpu_run_slot_begin");
    if (!dates || !enc) return fail(CCDGPU_EINVAL, "NULL input buffer");
    Shape sh;
    int rc = make_shape(n_chips, n_pix, n_obs, sh);
    if (rc || (rc = check_params(params))) return rc;
    if ((rc = ccdgpu_encoded_check(n_chips, n_pix, n_obs, enc, enc_bytes))) return rc;
    const int64_t *off = reinterpret_cast<const int64_t *>(enc) + 1;
    const int64_t pb = sh.total_pix();
    HIPCHK(hipSetDevice(c->device));
    const size_t tobs = (size_t)sh.total_obs(), tdata = (size_t)sh.total_data();
    if ((rc = c->slot_dates[slot].ensure(tobs)) || (rc = c->slot_enc[slot].ensure((size_t)off[n_chips])))
        return rc;
    if (c->decode_enc && ((rc = c->slot_spectra[slot].ensure(7 * tdata)) || (rc = c->slot_qa[slot].ensure(tdata))))
        return rc;
    // upload on the copy stream; the detection kernel reads the encoded batch in place (no decode
    // pass: px_setup in ccd_kernels.hip), or -- CCDGPU_DECODE=1 -- it is decoded there into the
    // slot's standard buffers first.  run_slot waits for the copy stream through the slot's event.
    HIPCHK(hipMemcpyAsync(c->slot_dates[slot].p, dates, sizeof(int64_t) * tobs, hipMemcpyHostToDevice, c->up_stream));
    HIPCHK(hipMemcpyAsync(c->slot_enc[slot].p, enc, (size_t)off[n_chips], hipMemcpyHostToDevice, c->up_stream));
    HIPCHK(hipEventRecord(c->uploaded[slot], c->up_stream));
    if (c->decode_enc) {
        if (c->up_stream != c->copy_stream) HIPCHK(hipStreamWaitEvent(c->copy_stream, c->uploaded[slot], 0));
        if (ccdk_decode_enc(c->slot_enc[slot].p, pb, c->slot_spectra[slot].p, c->slot_qa[slot].p, c->copy_stream))
            return fail(CCDGPU_EHIP, "ccd_decode_enc launch failed");
        HIPCHK(hipEventRecord(c->uploaded[slot], c->copy_stream));
    }
    c->slot_shape[slot] = sh;
    c->slot_params[slot] = *params;
    c->slot_ready[slot] = true;
    c->slot_encoded[slot] = !c->decode_enc;
    return 0;
}

int ccdgpu_stage_slot(ccdgpu_ctx *c, int32_t slot, const ccdgpu_params *params, int32_t n_chips, int32_t n_pix,
                      int32_t n_obs, const int64_t *dates, const int16_t *spectra, const uint16_t *qa) {
    std::vector<int32_t> np, no;
    uniform(n_chips, n_pix, n_obs, np, no);
    return ccdgpu_stage_slot_chips(c, slot, params, n_chips, np.data(), no.data(), dates, spectra, qa);
}

static int slot_inputs(ccdgpu_ctx *c, int32_t slot) {
    if (!c) return fail(CCDGPU_EINVAL, "NULL ctx");
    if (c->pending) return fail(CCDGPU_EINVAL, "a detection begun with ccdgpu_run_slot_begin is not finished");
    if (slot < 0 || slot >= CCDGPU_UPLOAD_SLOTS || !c->slot_ready[slot]) return fail(CCDGPU_EINVAL, "slot has no staged batch");
    int rc = stage_alloc(c, &c->slot_params[slot], c->slot_shape[slot], nullptr, false);
    if (rc) return rc;
    HIPCHK(hipStreamWaitEvent(c->aux, c->uploaded[slot], 0));
    c->in_dates = c->slot_dates[slot].p;
    c->in_enc = c->slot_encoded[slot] ? c->slot_enc[slot].p : nullptr;
    c->in_spectra = c->slot_encoded[slot] ? nullptr : c->slot_spectra[slot].p;
    c->in_qa = c->slot_encoded[slot] ? nullptr : c->slot_qa[slot].p;
    c->staged = true;
    c->ran = false;
    if (!c->keep_slots) c->slot_ready[slot] = false;
    return 0;
}

int ccdgpu_run_slot(ccdgpu_ctx *c, int32_t slot, double *kernel_seconds) {
    int rc = slot_inputs(c, slot);
    return rc ? rc : ccdgpu_run_staged(c, kernel_seconds);
}

static void detect_args(ccdgpu_ctx *c, CcdDetectArgs &a);
static int launch(ccdgpu_ctx *c, CcdDetectArgs &a);
static int finish(ccdgpu_ctx *c, double *kernel_seconds, bool *again, bool chained = false);

int ccdgpu_run_slot_begin(ccdgpu_ctx *c, int32_t slot) {
    int rc = slot_inputs(c, slot);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    detect_args(c, c->pend_args);
    if ((rc = launch(c, c->pend_args))) return rc;
    c->pending = true;
    c->pend_slot = slot;
    return 0;
}

int ccdgpu_run_query(ccdgpu_ctx *c) {
    if (!c) return fail(CCDGPU_EINVAL, "NULL ctx");
    if (!c->pending) return 1;
    const hipError_t e = hipEventQuery(c->rows_mode ? c->done_rows : c->done);
    if (e == hipSuccess) return 1;
    if (e == hipErrorNotReady) return 0;
    return fail(CCDGPU_EHIP, std::string("hipEventQuery: ") + hipGetErrorString(e));
}

int ccdgpu_run_slot_end(ccdgpu_ctx *c, double *kernel_seconds) {
    if (!c) return fail(CCDGPU_EINVAL, "NULL ctx");
    if (!c->pending) return fail(CCDGPU_EINVAL, "no detection begun with ccdgpu_run_slot_begin");
    if (c->rows_mode) return fail(CCDGPU_EINVAL, "a detection begun with ccdgpu_run_slot_begin_rows ends with ccdgpu_run_slot_end_rows");
    HIPCHK(hipSetDevice(c->device));
    c->pending = false;
    c->pend_slot = -1;
    for (int attempt = 0; attempt < 4; ++attempt) {
        bool again = false;
        const int rc = finish(c, kernel_seconds, &again);
        if (!again) return rc;
        if (int rc2 = launch(c, c->pend_args)) return rc2;
    }
    return fail(CCDGPU_EOVERFLOW, "segment pool kept overflowing");
}

// An error after a detection was queued (the chain behind it could not be enqueued): wait for
// everything the context queued, so no kernel still reads the slot or writes the pool when the
// caller recovers and restages, then return the error.
static int drain_after_error(ccdgpu_ctx *c, int rc) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->aux);
    c->pending = false;
    c->rows_mode = false;
    c->pend_slot = -1;
    return rc;
}

// The rest of a batch behind its detection, all on the aux stream (which already waits for the
// detection's end): CSR offsets (scan), the closing entry and rows per pixel, row offsets
// (scan), pool -> CSR with the device's segment count, row packing per chip, then the copies of
// the CSR offsets (pinned staging), row offsets, rows (up to the caller's capacity) and mask
// words into the caller's buffers.  Capacities are sized for any segment count the pool holds.
static int enqueue_rows(ccdgpu_ctx *c) {
    const Shape &sh = c->shape;
    const int nc = sh.n_chips();
    const int64_t np = c->total_pix;
    hipStream_t ax = c->aux;
    int rc;
    const int64_t rows_dev = np + c->pool_cap;  // rows <= pixels + segments
    if ((rc = c->csr.ensure(c->pool_cap > 0 ? c->pool_cap : 1)) || (rc = c->rows.ensure((size_t)rows_dev)) ||
        (rc = c->row_off.ensure(np + 1)) || (rc = c->rowcnt.ensure(np + 1)) || (rc = c->offsets.ensure(np + 1)) ||
        (rc = c->h_off.ensure(sizeof(int64_t) * (size_t)(np + 1))))
        return rc;
    // temporary storage of both scans (their instantiations differ: int32 counts -> int64 offsets,
    // int64 row counts -> int64 row offsets), each called with its own size
    size_t tmp_seg = 0, tmp_row = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_seg, c->nseg.p, c->offsets.p, (int)np, ax));
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_row, c->rowcnt.p, c->row_off.p, (int)np + 1, ax));
    if ((rc = c->cub_tmp.ensure(std::max(tmp_seg, tmp_row)))) return rc;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->cub_tmp.p, tmp_seg, c->nseg.p, c->offsets.p, (int)np, ax));
    if (ccdk_row_counts(c->nseg.p, c->offsets.p, np, c->rowcnt.p, ax)) return fail(CCDGPU_EHIP, "row count launch failed");
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->cub_tmp.p, tmp_row, c->rowcnt.p, c->row_off.p, (int)np + 1, ax));
    // (on a pool overflow -- counters[3] -- the segment counts exceed what the pool holds: the scatter
    // and the row packing write nothing and ccdgpu_run_slot_end_rows reruns the batch)
    // the chips' (cx, cy) through pinned staging
    if ((rc = c->row_xy.ensure(2 * (size_t)nc)) || (rc = c->h_xy.ensure(sizeof(int32_t) * 2 * (size_t)nc))) return rc;
    int32_t *hxy = reinterpret_cast<int32_t *>(c->h_xy.p);
    for (int32_t ch = 0; ch < nc; ++ch) {
        hxy[2 * ch] = c->rq_cx[ch];
        hxy[2 * ch + 1] = c->rq_cy[ch];
    }
    HIPCHK(hipMemcpyAsync(c->row_xy.p, hxy, sizeof(int32_t) * 2 * (size_t)nc, hipMemcpyHostToDevice, ax));
    if (c->rows_fused) {
        // pool -> CSR and rows in one pass, then the default rows of pixels without a model
        if (ccdk_pool_rows(c->pool.p, c->pool_seq.p, c->counters.p + 1, 0, c->counters.p + 3, c->pool_cap, c->offsets.p,
                           c->chip_pix_off.p, nc, c->csr.p, c->row_off.p, c->row_xy.p,
                           c->rq_width, c->rows.p, rows_dev, 256, ax) ||
            ccdk_default_rows(c->nseg.p, np, c->counters.p + 3, c->chip_pix_off.p, nc, c->row_off.p, c->row_xy.p, c->rq_width,
                              c->rows.p, rows_dev, ax))
            return fail(CCDGPU_EHIP, "row packing launch failed");
    } else {
        if (ccdk_scatter_dev(c->pool.p, c->pool_seq.p, c->counters.p + 1, c->counters.p + 3, c->pool_cap, c->offsets.p,
                             c->chip_pix_off.p, nc, c->csr.p, ax))
            return fail(CCDGPU_EHIP, "scatter launch failed");
        for (int32_t ch = 0; ch < nc; ++ch) {
            const int64_t q = sh.pix_off[ch];
            if (ccdk_pack_rows(c->csr.p, c->offsets.p + q, c->row_off.p + q, c->mask.p + (size_t)q * c->mask_words,
                               c->mask_words, sh.npix[ch], sh.nobs[ch], c->rq_cx[ch], c->rq_cy[ch], c->rq_width, c->rows.p,
                               nullptr, c->counters.p + 3, c->pool_cap, rows_dev, ax))
                return fail(CCDGPU_EHIP, "row packing launch failed");
        }
    }
    const size_t ob = sizeof(int64_t) * (size_t)(np + 1);
    HIPCHK(hipMemcpyAsync(c->h_off.p, c->offsets.p, ob, hipMemcpyDeviceToHost, ax));
    HIPCHK(hipMemcpyAsync(c->rq_offsets, c->row_off.p, ob, hipMemcpyDeviceToHost, ax));
    const int64_t nrc = std::min<int64_t>(c->rq_rows_cap, rows_dev);
    if (nrc > 0) HIPCHK(hipMemcpyAsync(c->rq_rows, c->rows.p, sizeof(ccdgpu_row) * (size_t)nrc, hipMemcpyDeviceToHost, ax));
    const size_t nbits = (size_t)np * c->mask_words;
    if (nbits > 0) HIPCHK(hipMemcpyAsync(c->rq_mask, c->mask.p, sizeof(uint32_t) * nbits, hipMemcpyDeviceToHost, ax));
    HIPCHK(hipEventRecord(c->done_rows, ax));
    return 0;
}

int ccdgpu_run_slot_begin_rows(ccdgpu_ctx *c, int32_t slot, const int32_t *cx, const int32_t *cy, int32_t width,
                               int64_t *row_offsets, int64_t offsets_cap, ccdgpu_row *rows, int64_t rows_cap,
                               uint32_t *mask_bits, int64_t mask_cap) {
    if (!c || !cx || !cy || !row_offsets || !rows || !mask_bits) return fail(CCDGPU_EINVAL, "NULL argument");
    if (width <= 0) return fail(CCDGPU_EINVAL, "width must be > 0");
    if (c->pending) return fail(CCDGPU_EINVAL, "a detection begun with ccdgpu_run_slot_begin is not finished");
    if (slot < 0 || slot >= CCDGPU_UPLOAD_SLOTS || !c->slot_ready[slot]) return fail(CCDGPU_EINVAL, "slot has no staged batch");
    const Shape &ssh = c->slot_shape[slot];
    const int64_t np = ssh.total_pix();
    const int64_t words = (ssh.n_obs_max + 31) / 32;
    if (offsets_cap < np + 1 || mask_cap < np * words)
        return fail(CCDGPU_EINVAL, "run_slot_begin_rows: offsets / mask buffers too small (need " + std::to_string(np + 1) +
                                       " offsets, " + std::to_string(np * words) + " mask words)");
    int rc = slot_inputs(c, slot);
    if (rc) return rc;
    HIPCHK(hipSetDevice(c->device));
    c->rq_offsets = row_offsets;
    c->rq_offsets_cap = offsets_cap;
    c->rq_rows = rows;
    c->rq_rows_cap = rows_cap;
    c->rq_mask = mask_bits;
    c->rq_mask_cap = mask_cap;
    c->rq_width = width;
    const int nc = c->shape.n_chips();
    c->rq_cx.assign(cx, cx + nc);
    c->rq_cy.assign(cy, cy + nc);
    detect_args(c, c->pend_args);
    if ((rc = launch(c, c->pend_args))) return rc;
    if ((rc = enqueue_rows(c))) return drain_after_error(c, rc);
    c->pending = true;
    c->rows_mode = true;
    c->pend_slot = slot;
    return 0;
}

int ccdgpu_run_slot_end_rows(ccdgpu_ctx *c, double *kernel_seconds, int64_t *n_rows) {
    if (!c) return fail(CCDGPU_EINVAL, "NULL ctx");
    if (n_rows) *n_rows = 0;
    if (!c->pending || !c->rows_mode) return fail(CCDGPU_EINVAL, "no detection begun with ccdgpu_run_slot_begin_rows");
    HIPCHK(hipSetDevice(c->device));
    c->pending = false;
    c->rows_mode = false;
    c->pend_slot = -1;
    int rc = 0;
    for (int attempt = 0;; ++attempt) {
        HIPCHK(hipEventSynchronize(c->done_rows));
        bool again = false;
        rc = finish(c, kernel_seconds, &again, true);
        if (!again) break;
        if (attempt == 3) return fail(CCDGPU_EOVERFLOW, "segment pool kept overflowing");
        int rc2;
        if ((rc2 = launch(c, c->pend_args))) return rc2;
        if ((rc2 = enqueue_rows(c))) return drain_after_error(c, rc2);
    }
    if (rc && rc != CCDGPU_EQA) return rc;
    const int64_t nr = c->rq_offsets[c->total_pix];
    if (n_rows) *n_rows = nr;
    if (nr > c->rq_rows_cap) {
        // the run is complete (ccdgpu_fetch_batch_rows_into fetches it into larger buffers); an
        // unsupported QA value outranks the short buffer -- CCDGPU_EQA with *n_rows set, so the
        // caller both fetches every row and raises pyccd's ValueError
        if (rc == CCDGPU_EQA) return rc;
        return fail(CCDGPU_EOVERFLOW, "run_slot_end_rows: " + std::to_string(nr) + " rows, the buffer holds " +
                                          std::to_string(c->rq_rows_cap));
    }
    return rc;
}

int ccdgpu_staged_inputs(ccdgpu_ctx *c, int16_t *spectra, uint16_t *qa) {
    if (!c || !c->staged) return fail(CCDGPU_EINVAL, "nothing staged");
    HIPCHK(hipSetDevice(c->device));
    const size_t tdata = (size_t)c->shape.total_data();
    const int16_t *ins = c->in_spectra;
    const uint16_t *inq = c->in_qa;
    if (c->in_enc) {
        // an encoded batch read in place by the detection: decoded here (the standalone decoder,
        // the same mapping as px_setup's) into the context's standard buffers
        int rc;
        if ((rc = c->spectra.ensure(7 * tdata)) || (rc = c->qa.ensure(tdata))) return rc;
        if (ccdk_decode_enc(c->in_enc, c->shape.total_pix(), c->spectra.p, c->qa.p, c->stream))
            return fail(CCDGPU_EHIP, "ccd_decode_enc launch failed");
        ins = c->spectra.p;
        inq = c->qa.p;
    }
    if (spectra)
        HIPCHK(hipMemcpyAsync(spectra, ins, sizeof(int16_t) * 7 * tdata, hipMemcpyDeviceToHost, c->stream));
    if (qa) HIPCHK(hipMemcpyAsync(qa, inq, sizeof(uint16_t) * tdata, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

static void detect_args(ccdgpu_ctx *c, CcdDetectArgs &a) {
    const ccdgpu_params &p = c->params;
    const Shape &sh = c->shape;
    const int nc = sh.n_chips();
    std::memset(&a, 0, sizeof(a));
    a.p = p;
    a.n_chips = nc;
    a.n_obs_max = sh.n_obs_max;
    a.mask_words = c->mask_words;
    a.n_slots = c->n_slots;
    a.poison = c->poison;
    a.total_pix = c->total_pix;
    a.chip_nobs = c->chip_nobs.p;
    a.chip_obs_off = c->chip_obs_off.p;
    a.chip_pix_off = c->chip_pix_off.p;
    a.chip_data_off = c->chip_data_off.p;
    a.spectra = c->in_spectra;
    a.qa = c->in_qa;
    a.enc = c->in_enc;
    a.order = c->order.p;
    a.sdates = c->sdates.p;
    a.basis = c->basis.p;
    a.counters = c->counters.p;
    a.s_date = c->s_date.p;
    a.s_row = c->s_row.p;
    a.s_bk = c->s_bk.p;
    a.s_f64 = c->s_f64.p;
    a.mask_bits = c->mask.p;
    a.procedure = c->procedure.p;
    a.probs = c->probs.p;
    a.nseg = c->nseg.p;
    a.stats = c->stats.p;
    for (int k = 0; k <= CCDGPU_MAX_PEEK; ++k) {
        if (k <= p.peek_size) a.thr_table[k] = p.change_threshold;
        else a.thr_table[k] = chi2_5_ppf(1.0 - std::pow(1.0 - p.change_probability, (double)p.peek_size / k));
    }
}

static int launch(ccdgpu_ctx *c, CcdDetectArgs &a) {
    const ccdgpu_params &p = c->params;
    const Shape &sh = c->shape;
    const int nc = sh.n_chips();
    a.pool = c->pool.p;
    a.pool_seq = c->pool_seq.p;
    a.pool_cap = c->pool_cap;
    // h_small: [0, 64) initial counters, [64, 128) counters back, [128, 128 + 8 NSTATS) stats
    // back, then the kernel arguments (each launch waits for the previous one's copies)
    // [SM_ARGS + args, + 8 NSTATS) zeros for the statistics
    constexpr size_t SM_ARGS = 128 + 8 * CCD_NSTATS;
    constexpr size_t SM_ZERO = SM_ARGS + ((sizeof(CcdDetectArgs) + 63) & ~(size_t)63);
    if (int rc0 = c->h_small.ensure(SM_ZERO + 8 * CCD_NSTATS)) return rc0;
    unsigned long long *hinit = reinterpret_cast<unsigned long long *>(c->h_small.p);
    const unsigned long long init[8] = {0ull, 0ull, ~0ull, 0ull, 0ull, ~0ull, 0ull, ~0ull};
    std::memcpy(hinit, init, sizeof(init));
    std::memset(c->h_small.p + SM_ZERO, 0, 8 * CCD_NSTATS);
    hipStream_t ax = c->aux;
    HIPCHK(hipMemcpyAsync(c->counters.p, hinit, sizeof(init), hipMemcpyHostToDevice, ax));
    HIPCHK(hipMemcpyAsync(c->stats.p, c->h_small.p + SM_ZERO, 8 * CCD_NSTATS, hipMemcpyHostToDevice, ax));
    CcdDetectArgs *hargs = reinterpret_cast<CcdDetectArgs *>(c->h_small.p + SM_ARGS);
    std::memcpy(hargs, &a, sizeof(a));
    if (ccdk_set_args(hargs, c->arg_slot, ax)) return fail(CCDGPU_EHIP, "copying kernel arguments to constant memory failed");
    HIPCHK(hipEventRecord(c->ev[0], ax));
    if (ccdk_prep(c->in_dates, nc, c->chip_nobs.p, c->chip_obs_off.p, p.avg_days_yr, p.argsort_stable, c->order.p,
                  c->sdates.p, c->basis.p, ax))
        return fail(CCDGPU_EHIP, std::string("prep launch: ") + hipGetErrorString(hipGetLastError()));
    HIPCHK(hipEventRecord(c->ev[1], ax));
    if (ax != c->stream) HIPCHK(hipStreamWaitEvent(c->stream, c->ev[1], 0));
    if (ccdk_detect(c->n_slots, c->variant, sh.n_obs_max, c->arg_slot, c->stream))
        return fail(CCDGPU_EHIP, std::string("detect launch: ") + hipGetErrorString(hipGetLastError()));
    HIPCHK(hipEventRecord(c->ev[2], c->stream));
    if (ax != c->stream) HIPCHK(hipStreamWaitEvent(ax, c->ev[2], 0));
    // counters and statistics back into pinned memory; `done` marks their arrival (finish sleeps on it)
    unsigned long long *h = reinterpret_cast<unsigned long long *>(c->h_small.p + 64);
    unsigned long long *hst = reinterpret_cast<unsigned long long *>(c->h_small.p + 128);
    HIPCHK(hipMemcpyAsync(h, c->counters.p, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost, ax));
    HIPCHK(hipMemcpyAsync(hst, c->stats.p, sizeof(unsigned long long) * CCD_NSTATS, hipMemcpyDeviceToHost, ax));
    if (c->done) HIPCHK(hipEventRecord(c->done, ax));
    return 0;
}

static int finish(ccdgpu_ctx *c, double *kernel_seconds, bool *again, bool chained) {
    const ccdgpu_params &p = c->params;
    const Shape &sh = c->shape;
    const int nc = sh.n_chips();
    hipStream_t ax = c->aux;
    unsigned long long *h = reinterpret_cast<unsigned long long *>(c->h_small.p + 64);
    unsigned long long *hst = reinterpret_cast<unsigned long long *>(c->h_small.p + 128);
    *again = false;
    if (chained) {
        // the batch chain has completed (the caller waited for done_rows)
    } else if (c->done) {
        HIPCHK(hipEventSynchronize(c->done));
    } else {
        HIPCHK(hipStreamSynchronize(ax));
    }
    if (h[4] >= 100000) {
        // checking build: every call site that ran without a full EXEC, from the line bitmap
        // (bit = line / 2) in stats[8 ..]
        const unsigned long long *st = hst;
        std::string lines;
        for (int w = 8; w < CCD_NSTATS; ++w)
            for (int b = 0; b < 64; ++b)
                if ((st[w] >> b) & 1ull) {
                    const int l0 = 2 * (64 * (w - 8) + b);
                    lines += (lines.empty() ? "" : ", ") + std::to_string(l0) + "-" + std::to_string(l0 + 1);
                }
        return fail(CCDGPU_EHIP, "cross-lane primitive ran without a full EXEC at ccd_kernels.hip line " +
                                     std::to_string(h[4] - 100000) + " (all call sites: lines " + lines + ")");
    }
    if (h[4]) return fail(CCDGPU_EHIP, "kernel index guard tripped at ccd_kernels.hip line " + std::to_string(h[4]));
    if (h[3]) {  // pool overflow: grow and rerun
        c->pool_cap = (int64_t)(h[1] + h[1] / 4 + 1024);
        ++c->pool_reruns;
        int rc;
        if ((rc = c->pool.ensure(c->pool_cap)) || (rc = c->pool_seq.ensure(c->pool_cap))) return rc;
        *again = true;
        return 0;
    }
    c->n_pool = (int64_t)h[1];
    float ms_prep = 0.f, ms_det = 0.f;
    (void)hipEventElapsedTime(&ms_prep, c->ev[0], c->ev[1]);
    (void)hipEventElapsedTime(&ms_det, c->ev[1], c->ev[2]);
    const unsigned long long *st = hst;
    for (int i = 0; i < CCD_NSTATS; ++i) c->diag[i] = st[i];
    int rc;
    if (chained) {
        // CSR, offsets and rows were made by the chain (enqueue_rows); the offsets are in h_off
        c->h_offsets.resize(c->total_pix + 1);
        std::memcpy(c->h_offsets.data(), c->h_off.p, sizeof(int64_t) * (size_t)(c->total_pix + 1));
    } else {
    // CSR: exclusive scan of per-pixel counts, then scatter the pool
    if ((rc = c->csr.ensure(c->n_pool > 0 ? c->n_pool : 1))) return rc;
    size_t tmp_bytes = 0;
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, c->nseg.p, c->offsets.p, (int)c->total_pix + 1, ax));
    if ((rc = c->cub_tmp.ensure(tmp_bytes))) return rc;
    // nseg has total_pix entries; the scan over total_pix+1 needs a trailing zero
    HIPCHK(hipcub::DeviceScan::ExclusiveSum(c->cub_tmp.p, tmp_bytes, c->nseg.p, c->offsets.p, (int)c->total_pix, ax));
    c->h_offsets.resize(c->total_pix + 1);
    if ((rc = c->h_off.ensure(sizeof(int64_t) * (size_t)c->total_pix))) return rc;
    HIPCHK(hipMemcpyAsync(c->h_off.p, c->offsets.p, sizeof(int64_t) * c->total_pix, hipMemcpyDeviceToHost, ax));
    HIPCHK(hipStreamSynchronize(ax));
    std::memcpy(c->h_offsets.data(), c->h_off.p, sizeof(int64_t) * (size_t)c->total_pix);
    c->h_offsets[c->total_pix] = c->n_pool;
    if (c->rows_fused ? ccdk_pool_rows(c->pool.p, c->pool_seq.p, nullptr, c->n_pool, nullptr, c->n_pool, c->offsets.p,
                                       c->chip_pix_off.p, nc, c->csr.p, nullptr, nullptr, 1, nullptr, 0, 256, ax)
                      : ccdk_scatter(c->pool.p, c->pool_seq.p, c->n_pool, c->offsets.p, c->chip_pix_off.p, nc, c->csr.p, ax))
        return fail(CCDGPU_EHIP, "scatter launch failed");
    HIPCHK(hipEventRecord(c->ev[3], ax));
    HIPCHK(hipStreamSynchronize(ax));
    }
    c->last.detect_ms = ms_det;
    c->last.detect_ms_device = h[6] > h[5] ? (double)(h[6] - h[5]) / 1e5 : 0.0;  // 100 MHz clock
    c->last.prep_ms = ms_prep;
    c->last.pixels = c->total_pix;
    c->last.segments = c->n_pool;
    c->last.lasso_fits = (int64_t)st[0];
    c->last.cd_sweeps = (int64_t)st[1];
    c->last.flops = (int64_t)st[2];
    c->last.pool_reruns = c->pool_reruns;
    c->last.pool_cap = c->pool_cap;
    c->last.wave_slots = c->n_slots;
    c->last.n_cu = c->n_cu;
    const int64_t in_bytes = sh.total_data() * 16 + sh.total_obs() * 8;
    const int64_t out_bytes = c->n_pool * (int64_t)sizeof(ccdgpu_segment) + c->total_pix * ((int64_t)c->mask_words * 4 + 4 + 24 + 4);
    c->last.bytes = in_bytes + out_bytes;
    if (kernel_seconds) *kernel_seconds = (ms_prep + ms_det) * 1e-3;
    c->ran = true;
    if (h[7] != ~0ull)
        return fail(CCDGPU_EOVERFLOW, "adaptive peek of pixel " + std::to_string(h[7]) + " exceeds " +
                                          std::to_string(CCDGPU_MAX_PEEK) + " observations (PEEK_SIZE " +
                                          std::to_string(p.peek_size) + ")");
    if (h[2] != ~0ull) {
        g_err = "unsupported bit-packed QA value (pixel " + std::to_string(h[2]) + ")";
        return CCDGPU_EQA;
    }
    return 0;
}

int ccdgpu_run_staged(ccdgpu_ctx *c, double *kernel_seconds) {
    if (!c || !c->staged) return fail(CCDGPU_EINVAL, "nothing staged");
    if (c->pending) return fail(CCDGPU_EINVAL, "a detection begun with ccdgpu_run_slot_begin is not finished");
    HIPCHK(hipSetDevice(c->device));
    CcdDetectArgs a;
    detect_args(c, a);
    for (int attempt = 0; attempt < 4; ++attempt) {
        int rc = launch(c, a);
        if (rc) return rc;
        bool again = false;
        rc = finish(c, kernel_seconds, &again);
        if (!again) return rc;
    }
    return fail(CCDGPU_EOVERFLOW, "segment pool kept overflowing");
}

int ccdgpu_diag_counters(ccdgpu_ctx *c, uint64_t *out, int32_t n) {
    if (!c || !out || n < 0) return fail(CCDGPU_EINVAL, "bad argument");
    for (int i = 0; i < n && i < CCD_NSTATS; ++i) out[i] = c->diag[i];
    return 0;
}

int ccdgpu_last_stats(ccdgpu_ctx *c, ccdgpu_stats *s) {
    if (!c || !s) return fail(CCDGPU_EINVAL, "NULL argument");
    *s = c->last;
    return 0;
}

static int fetch_chip(ccdgpu_ctx *c, int32_t chip, ccdgpu_result *out) {
    std::memset(out, 0, sizeof(*out));
    if (!c->ran) return fail(CCDGPU_EINVAL, "no completed run to fetch");
    if (chip < 0 || chip >= c->shape.n_chips()) return fail(CCDGPU_EINVAL, "chip index out of range");
    HIPCHK(hipSetDevice(c->device));
    const int np = c->shape.npix[chip], no = c->shape.nobs[chip];
    const int64_t p0 = c->shape.pix_off[chip], o0 = c->shape.obs_off[chip];
    const int64_t s0 = c->h_offsets[p0], s1 = c->h_offsets[p0 + np];
    out->n_pix = np;
    out->n_obs = no;
    out->n_seg = s1 - s0;
    out->mask_words = c->mask_words;
    out->error_pixel = -1;
    out->seg_offsets = (int64_t *)std::malloc(sizeof(int64_t) * (np + 1));
    out->segments = (ccdgpu_segment *)std::malloc(sizeof(ccdgpu_segment) * (size_t)(out->n_seg + 1));
    out->mask_bits = (uint32_t *)std::malloc(sizeof(uint32_t) * (size_t)np * c->mask_words + 4);
    out->procedure = (int32_t *)std::malloc(sizeof(int32_t) * np);
    out->probs = (double *)std::malloc(sizeof(double) * 3 * np);
    out->sorted_dates = (int64_t *)std::malloc(sizeof(int64_t) * no);
    out->sort_index = (int32_t *)std::malloc(sizeof(int32_t) * no);
    if (!out->seg_offsets || !out->segments || !out->mask_bits || !out->procedure || !out->probs ||
        !out->sorted_dates || !out->sort_index) {
        ccdgpu_result_free(out);
        return fail(CCDGPU_ENOMEM, "host allocation failed");
    }
    for (int i = 0; i <= np; ++i) out->seg_offsets[i] = c->h_offsets[p0 + i] - s0;
    if (out->n_seg > 0)
        HIPCHK(hipMemcpyAsync(out->segments, c->csr.p + s0, sizeof(ccdgpu_segment) * out->n_seg, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(out->mask_bits, c->mask.p + (size_t)p0 * c->mask_words, sizeof(uint32_t) * (size_t)np * c->mask_words, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(out->procedure, c->procedure.p + p0, sizeof(int32_t) * np, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(out->probs, c->probs.p + 3 * p0, sizeof(double) * 3 * np, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(out->sorted_dates, c->sdates.p + o0, sizeof(int64_t) * no, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(out->sort_index, c->order.p + o0, sizeof(int32_t) * no, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < np; ++i)
        if (out->procedure[i] < 0) {
            out->error_pixel = i;
            break;
        }
    return 0;
}

// Rows of chips [c0, c1) of the last run, packed on the device and copied back in one piece:
// row offsets over the chips' pixels, rows pixel-major, and the masks either one byte per date
// (packed_mask false: chip c's block at data_off[c] - data_off[c0], [n_pix_c][n_obs_c]) or as the
// device's bit words ([pixels][mask_words]).
static int fetch_rows_range(ccdgpu_ctx *c, int32_t c0, int32_t c1, const int32_t *cx, const int32_t *cy, int32_t width,
                            ccdgpu_rows *out, bool packed_mask) {
    std::memset(out, 0, sizeof(*out));
    if (!c->ran) return fail(CCDGPU_EINVAL, "no completed run to fetch");
    if (width <= 0) return fail(CCDGPU_EINVAL, "width must be > 0");
    HIPCHK(hipSetDevice(c->device));
    const Shape &sh = c->shape;
    const int64_t p0 = sh.pix_off[c0], np = sh.pix_off[c1] - p0;
    const int64_t d0 = sh.data_off[c0], nd = sh.data_off[c1] - d0;
    const int64_t s0 = c->h_offsets[p0];
    // rows per pixel = max(1, segments): host prefix over the segment offsets already here
    std::vector<int64_t> soff((size_t)np + 1), roff((size_t)np + 1);
    roff[0] = 0;
    for (int64_t i = 0; i <= np; ++i) soff[i] = c->h_offsets[p0 + i] - s0;
    for (int64_t i = 0; i < np; ++i) roff[i + 1] = roff[i] + std::max<int64_t>(1, soff[i + 1] - soff[i]);
    const int64_t n_rows = roff[np];
    int rc;
    if ((rc = c->rows.ensure((size_t)n_rows)) || (rc = c->row_off.ensure(np + 1)) || (rc = c->seg_off1.ensure(np + 1)) ||
        (!packed_mask && (rc = c->mask8.ensure((size_t)nd))))
        return rc;
    // offsets through pinned staging, row packing and the copies back on the aux stream (the
    // reserved CUs when there are: other contexts' detections hold the rest)
    hipStream_t ax = c->aux;
    const size_t ob = sizeof(int64_t) * (size_t)(np + 1);
    if ((rc = c->h_fo.ensure(2 * ob))) return rc;
    std::memcpy(c->h_fo.p, soff.data(), ob);
    std::memcpy(c->h_fo.p + ob, roff.data(), ob);
    HIPCHK(hipMemcpyAsync(c->seg_off1.p, c->h_fo.p, ob, hipMemcpyHostToDevice, ax));
    HIPCHK(hipMemcpyAsync(c->row_off.p, c->h_fo.p + ob, ob, hipMemcpyHostToDevice, ax));
    for (int32_t ch = c0; ch < c1; ++ch) {
        const int64_t q = sh.pix_off[ch] - p0;
        if (ccdk_pack_rows(c->csr.p + s0, c->seg_off1.p + q, c->row_off.p + q, c->mask.p + (size_t)sh.pix_off[ch] * c->mask_words,
                           c->mask_words, sh.npix[ch], sh.nobs[ch], cx[ch - c0], cy[ch - c0], width, c->rows.p,
                           packed_mask ? nullptr : c->mask8.p + (sh.data_off[ch] - d0), nullptr, INT64_MAX, INT64_MAX, ax))
            return fail(CCDGPU_EHIP, "row packing launch failed");
    }
    out->n_pix = (int32_t)np;
    out->n_obs = c1 - c0 == 1 ? sh.nobs[c0] : 0;
    out->n_rows = n_rows;
    out->row_offsets = (int64_t *)std::malloc(sizeof(int64_t) * (np + 1));
    out->rows = (ccdgpu_row *)std::malloc(sizeof(ccdgpu_row) * (size_t)(n_rows > 0 ? n_rows : 1));
    const size_t nbits = (size_t)np * c->mask_words;
    if (packed_mask) {
        out->mask_words = c->mask_words;
        out->mask_bits = (uint32_t *)std::malloc(sizeof(uint32_t) * (nbits > 0 ? nbits : 1));
    } else {
        out->mask = (int8_t *)std::malloc((size_t)(nd > 0 ? nd : 1));
    }
    if (!out->row_offsets || !out->rows || (packed_mask ? !out->mask_bits : !out->mask)) {
        ccdgpu_rows_free(out);
        return fail(CCDGPU_ENOMEM, "host allocation failed");
    }
    std::memcpy(out->row_offsets, roff.data(), sizeof(int64_t) * (np + 1));
    const size_t row_bytes = sizeof(ccdgpu_row) * (size_t)n_rows;
    if (packed_mask) {
        // batch fetch: rows and mask words land in the context's pinned buffer by DMA (one copy
        // each at link speed), then go to the caller's buffers with a host memcpy
        const size_t bit_bytes = sizeof(uint32_t) * nbits;
        const size_t bit_at = (row_bytes + 255) & ~(size_t)255;
        if ((rc = c->h_rows.ensure(bit_at + bit_bytes))) {
            (void)hipStreamSynchronize(ax);
            ccdgpu_rows_free(out);
            return rc;
        }
        HIPCHK(hipMemcpyAsync(c->h_rows.p, c->rows.p, row_bytes, hipMemcpyDeviceToHost, ax));
        HIPCHK(hipMemcpyAsync(c->h_rows.p + bit_at, c->mask.p + (size_t)p0 * c->mask_words, bit_bytes,
                              hipMemcpyDeviceToHost, ax));
        HIPCHK(hipStreamSynchronize(ax));
        std::memcpy(out->rows, c->h_rows.p, row_bytes);
        std::memcpy(out->mask_bits, c->h_rows.p + bit_at, bit_bytes);
        return 0;
    }
    HIPCHK(hipMemcpyAsync(out->rows, c->rows.p, row_bytes, hipMemcpyDeviceToHost, ax));
    HIPCHK(hipMemcpyAsync(out->mask, c->mask8.p, (size_t)nd, hipMemcpyDeviceToHost, ax));
    HIPCHK(hipStreamSynchronize(ax));
    return 0;
}

int ccdgpu_fetch_rows(ccdgpu_ctx *c, int32_t chip, int32_t cx, int32_t cy, int32_t width, ccdgpu_rows *out) {
    if (!c || !out) return fail(CCDGPU_EINVAL, "NULL argument");
    if (chip < 0 || chip >= c->shape.n_chips()) {
        std::memset(out, 0, sizeof(*out));
        return fail(CCDGPU_EINVAL, "chip index out of range");
    }
    return fetch_rows_range(c, chip, chip + 1, &cx, &cy, width, out, false);
}

int ccdgpu_fetch_batch_rows(ccdgpu_ctx *c, const int32_t *cx, const int32_t *cy, int32_t width, ccdgpu_rows *out) {
    if (!c || !out || !cx || !cy) return fail(CCDGPU_EINVAL, "NULL argument");
    if (c->shape.n_chips() <= 0) {
        std::memset(out, 0, sizeof(*out));
        return fail(CCDGPU_EINVAL, "no completed run to fetch");
    }
    return fetch_rows_range(c, 0, c->shape.n_chips(), cx, cy, width, out, true);
}

int ccdgpu_fetch_batch_rows_into(ccdgpu_ctx *c, const int32_t *cx, const int32_t *cy, int32_t width, int64_t *row_offsets,
                                 int64_t offsets_cap, ccdgpu_row *rows, int64_t rows_cap, uint32_t *mask_bits,
                                 int64_t mask_cap, int64_t *n_rows) {
    if (!c || !cx || !cy || !row_offsets || !rows || !mask_bits || !n_rows) return fail(CCDGPU_EINVAL, "NULL argument");
    *n_rows = 0;
    if (!c->ran || c->shape.n_chips() <= 0) return fail(CCDGPU_EINVAL, "no completed run to fetch");
    if (width <= 0) return fail(CCDGPU_EINVAL, "width must be > 0");
    HIPCHK(hipSetDevice(c->device));
    const Shape &sh = c->shape;
    const int32_t nc = sh.n_chips();
    const int64_t np = sh.pix_off[nc];
    // rows per pixel = max(1, segments), from the segment offsets already on the host
    int64_t nr = 0;
    for (int64_t i = 0; i < np; ++i) nr += std::max<int64_t>(1, c->h_offsets[i + 1] - c->h_offsets[i]);
    *n_rows = nr;
    const size_t nbits = (size_t)np * c->mask_words;
    if (offsets_cap < np + 1 || rows_cap < nr || mask_cap < (int64_t)nbits)
        return fail(CCDGPU_EINVAL, "fetch_batch_rows_into: buffers too small (need " + std::to_string(np + 1) +
                                       " offsets, " + std::to_string(nr) + " rows, " + std::to_string(nbits) + " mask words)");
    int rc;
    if ((rc = c->rows.ensure((size_t)(nr > 0 ? nr : 1))) || (rc = c->row_off.ensure(np + 1)) || (rc = c->seg_off1.ensure(np + 1)))
        return rc;
    const size_t ob = sizeof(int64_t) * (size_t)(np + 1);
    if ((rc = c->h_fo.ensure(2 * ob))) return rc;
    int64_t *soff = reinterpret_cast<int64_t *>(c->h_fo.p), *roff = soff + (np + 1);
    const int64_t s0 = c->h_offsets[0];
    roff[0] = 0;
    for (int64_t i = 0; i <= np; ++i) soff[i] = c->h_offsets[i] - s0;
    for (int64_t i = 0; i < np; ++i) roff[i + 1] = roff[i] + std::max<int64_t>(1, soff[i + 1] - soff[i]);
    hipStream_t ax = c->aux;
    HIPCHK(hipMemcpyAsync(c->seg_off1.p, soff, ob, hipMemcpyHostToDevice, ax));
    HIPCHK(hipMemcpyAsync(c->row_off.p, roff, ob, hipMemcpyHostToDevice, ax));
    for (int32_t ch = 0; ch < nc; ++ch) {
        const int64_t q = sh.pix_off[ch];
        if (ccdk_pack_rows(c->csr.p + s0, c->seg_off1.p + q, c->row_off.p + q, c->mask.p + (size_t)q * c->mask_words,
                           c->mask_words, sh.npix[ch], sh.nobs[ch], cx[ch], cy[ch], width, c->rows.p, nullptr, nullptr,
                           INT64_MAX, INT64_MAX, ax))
            return fail(CCDGPU_EHIP, "row packing launch failed");
    }
    // straight into the caller's buffers (DMA when they are pinned: ccdgpu_host_alloc)
    if (nr > 0) HIPCHK(hipMemcpyAsync(rows, c->rows.p, sizeof(ccdgpu_row) * (size_t)nr, hipMemcpyDeviceToHost, ax));
    if (nbits > 0) HIPCHK(hipMemcpyAsync(mask_bits, c->mask.p, sizeof(uint32_t) * nbits, hipMemcpyDeviceToHost, ax));
    std::memcpy(row_offsets, roff, ob);
    HIPCHK(hipStreamSynchronize(ax));
    return 0;
}

void ccdgpu_rows_free(ccdgpu_rows *r) {
    if (!r) return;
    std::free(r->row_offsets);
    std::free(r->rows);
    std::free(r->mask);
    std::free(r->mask_bits);
    std::memset(r, 0, sizeof(*r));
}

int ccdgpu_fetch_staged(ccdgpu_ctx *c, int32_t chip, ccdgpu_result *out) {
    if (!c || !out) return fail(CCDGPU_EINVAL, "NULL argument");
    return fetch_chip(c, chip, out);
}

int ccdgpu_detect_batch(ccdgpu_ctx *c, const ccdgpu_params *params, int32_t n_pix, int32_t n_obs,
                        const int64_t *dates, const int16_t *spectra, const uint16_t *qa, ccdgpu_result *out) {
    if (!out) return fail(CCDGPU_EINVAL, "NULL result");
    std::memset(out, 0, sizeof(*out));
    auto t0 = std::chrono::steady_clock::now();
    int rc = ccdgpu_stage(c, params, 1, n_pix, n_obs, dates, spectra, qa);
    if (rc) return rc;
    double ks = 0;
    rc = ccdgpu_run_staged(c, &ks);
    if (rc && rc != CCDGPU_EQA) return rc;
    const int rc_qa = rc;
    const std::string qa_msg = g_err;
    rc = fetch_chip(c, 0, out);
    if (rc) return rc;
    out->seconds_kernel = ks;
    out->seconds_total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (rc_qa) g_err = qa_msg;
    return rc_qa;
}

void ccdgpu_result_free(ccdgpu_result *r) {
    if (!r) return;
    std::free(r->seg_offsets);
    std::free(r->segments);
    std::free(r->mask_bits);
    std::free(r->procedure);
    std::free(r->probs);
    std::free(r->sorted_dates);
    std::free(r->sort_index);
    std::memset(r, 0, sizeof(*r));
}

}  // extern "C"
