// demod_api.cpp — C ABI host layer of libfskdemod.so (include/demod.h).
//
// Handle lifecycle mirrors the Opus decoder the reference receiver drives
// (opus_decoder_create/destroy, hardware/src/playback.cpp:67-74); streaming
// intake mirrors the per-packet call at playback.cpp:115-122, where
// demodulate(pcm, nSamplesDecoded) would consume opus_decode's output.
// Errors are returned (no abort(), unlike OPUS_ERROR_CHECK playback.cpp:16-22).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/demod.h"
#include "demod_internal.h"
#include "plan.h"

using namespace fskd;

struct demod {
    demod_cfg_t cfg;
    int device = 0;
    int cus = 0;
    int log2g = 0;
    int detector = kDetGoertzel;
    hipStream_t stream = nullptr;
    float4 *d_rot = nullptr;    // [k][g]
    int slide_wt = 0;           // plain detector, SLIDE: windows per tile (0: off)
    float *d_tw512 = nullptr;   // FFT detector tables
    float *d_tw1024 = nullptr;
    int *d_bins = nullptr;
    int fft_bins[kMaxTones] = {};  // FFT detector: tone bins round(f n / fs)
    int fft_slot[kMaxTones] = {};  // FFT detector: where each tone bin's power sits (fft_quad_slot)
    unsigned fft_pmask = 0xFFu;    // tones only: the post-pass pair blocks holding a tone (fft_quad_pmask)
    // decision rescue (rescue.hip)
    bool rescue = false;        // K >= 2 and not switched off (FSKD_NO_RESCUE=1)
    bool rescue_launch = true;  // FSKD_NO_RESCUE=flags: flag only, no rescue launch (diagnostics)
    // large-output batches: one launch with L2 write-back bursts (default), or
    // the round-2 launch slices (FSKD_WB_BURSTS=0, measurement switch)
    bool wb_bursts = true;
    bool rescue_kernel_forced = false;  // FSKD_RESCUE_LAUNCH=1: the rescue launch everywhere (measurement)
    int wb_force = 0;  // FSKD_WB_BURSTS=<n >= 1>: n bursts on every hop = n batch (measurement)
    double tau = 0.0;           // decision rescue threshold factor (error_model.cpp)
    float amb_tq = 0.f;         // stage 1: amb_tq sqrt(P_max), the int16 worst-case energy
    float amb_floor = 0.f;
    float amb_t2e = 0.f;        // stage 2: threshold^2 = amb_t2e E P_max
    double rcoef[kMaxTones] = {};  // 2 cos(2 pi f_k / fs) in double, the caller's tone order
    double *d_rot64 = nullptr;  // in-kernel rescue, first step: [k][16][4] segment rotations in double
    double tau64 = 0.0;         // its threshold factor (error_model; 0: off)
    double t2e64 = 0.0;         // pass 0's margin test, threshold^2 = t2e64 E P_max
    float amb_d = 0.f;          // fold detector: the oracle's share of stage 2 (E_eff = (sqrt E + d)^2)
    double *d_rtw = nullptr;    // FFT: radix-2 twiddles (cos, sin)(-2 pi j / len), [n - 1]
    float coef[kMaxTones] = {};
    float sgn[kMaxTones] = {};  // plain detector, Reinsch form: sign of cos(w_k)
    bool reinsch = false;       // plain detector: Reinsch-modified recurrence
    int dcls = 0;               // residue detector: compile-time class pattern (residue.hip DC), slots permuted
    bool f16 = false;           // fold detector: fold by 16, slots permuted (Z0 tones, Z8 tones)
    int fold64 = 0;             // the rescue's pass 0 by the fold / residue fold (plan.h)
    unsigned long long perm = 0;  // DCLS: nibble s = tone index of kernel slot s
    int zcls[kMaxTones] = {};   // residue detector: class each tone reads
    // staging for host-pointer calls
    int16_t *d_in = nullptr;
    size_t d_in_cap = 0;        // samples
    uint8_t *d_sym = nullptr;
    float *d_mag = nullptr;
    size_t d_out_cap = 0;       // windows
    int16_t *h_in = nullptr;            // pinned staging for small host calls
    size_t h_in_cap = 0;                // samples
    uint8_t *h_sym = nullptr;           // pinned
    float *h_mag = nullptr;             // pinned [h_out_cap][k]
    size_t h_out_cap = 0;               // windows
    // packet-sized calls: the kernel reads the window samples from, and
    // writes its results to, mapped coherent host memory (no copies)
    int zc = 0;                         // 0: not set up, 1: ready, -1: unavailable
    int16_t *z_in = nullptr;            // host view [kZeroCopySamples]
    uint8_t *z_sym = nullptr;
    float *z_mag = nullptr;
    int16_t *zd_in = nullptr;           // device views of the same memory
    uint8_t *zd_sym = nullptr;
    float *zd_mag = nullptr;
    hipStream_t copy_stream = nullptr;  // H2D of large host-pointer calls
    hipEvent_t copied[2] = {};          // device slot b holds its chunk
    hipEvent_t consumed[2] = {};        // the kernel reading slot b has run
    // streaming carry (mono samples not yet consumed by a complete window)
    std::vector<int16_t> carry;
    std::vector<int16_t> scratch;
    // lead-in: mono frames still to drop at the start of the stream (cfg.lead_in
    // after demod_create / demod_reset)
    size_t skip = 0;
};

// Makes `dev` current for the scope of an entry point and restores the
// caller's current device on return (the ABI must not leave the calling
// thread on another device).
struct DeviceGuard {
    int prev = -1;
    hipError_t err = hipSuccess;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) {
            (void)hipGetLastError();
            prev = -1;
        }
        if (prev != dev) err = hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

#define HIP_TRY(x)                                                 \
    do {                                                           \
        hipError_t _e = (x);                                       \
        if (_e != hipSuccess) {                                    \
            std::fprintf(stderr, "fskdemod: %s failed: %s\n", #x,  \
                         hipGetErrorString(_e));                   \
            return DEMOD_DEVICE_ERROR;                             \
        }                                                          \
    } while (0)

extern "C" {

void demod_cfg_default(demod_cfg_t *cfg)
{
    if (!cfg) return;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->fs = 48000.0;
    cfg->n = 1024;
    cfg->hop = 1024;
    cfg->k = 2;
    cfg->channels = 1;
    cfg->channel_mode = DEMOD_CH_LEFT;
    cfg->device = 0;
    cfg->method = DEMOD_METHOD_AUTO;
    cfg->freqs[0] = 1500.0;
    cfg->freqs[1] = 3000.0;
}

static int validate(const demod_cfg_t *c) { return validate_cfg(c); }

static int init_device_state(demod_t *st)
{
    const demod_cfg_t &c = st->cfg;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return DEMOD_NO_DEVICE;
    }
    if (c.device < 0 || c.device >= ndev) return DEMOD_NO_DEVICE;
    if (c.device >= kMaxDevices) return DEMOD_BAD_ARG;
    HIP_TRY(hipSetDevice(c.device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, c.device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        std::fprintf(stderr, "fskdemod: device %d is %s, need gfx950 (MI355X)\n",
                     c.device, prop.gcnArchName);
        return DEMOD_NO_DEVICE;
    }
    st->device = c.device;
    st->cus = prop.multiProcessorCount;
    HIP_TRY(hipStreamCreateWithFlags(&st->stream, hipStreamNonBlocking));

    Plan pl;
    build_plan(c, pl);
    st->log2g = pl.log2g;
    st->detector = pl.detector;
    const bool slide = pl.slide;
    if (st->detector == kDetFft) {
        std::vector<float> t1(1024), t2(1024);
        for (int m = 0; m < 512; ++m) {
            t1[2 * m] = (float)std::cos(-2.0 * M_PI * m / 512.0);
            t1[2 * m + 1] = (float)std::sin(-2.0 * M_PI * m / 512.0);
            t2[2 * m] = (float)std::cos(-2.0 * M_PI * m / 1024.0);
            t2[2 * m + 1] = (float)std::sin(-2.0 * M_PI * m / 1024.0);
        }
        std::vector<int> bins(c.k);
        for (uint32_t k = 0; k < c.k; ++k) {
            bins[k] = pl.fft_bins[k];
            st->fft_bins[k] = pl.fft_bins[k];
            st->fft_slot[k] = pl.fft_slot[k];
        }
        // FSKD_FFT_PMASK=0 (measurement): the full post-pass on tones-only batches
        const char *pm_env = std::getenv("FSKD_FFT_PMASK");
        st->fft_pmask = pm_env && std::strcmp(pm_env, "0") == 0 ? 0xFFu : fft_quad_pmask(bins.data(), (int)c.k);
        // the rescue's radix-2 twiddles: stage len (2 .. n), j < len / 2 at
        // len / 2 - 1 + j, each the (cos, sin) of (-2 pi / len) j exactly as
        // the double FFT of the definition evaluates it (one libm sincos of
        // the same rounded argument)
        std::vector<double> rtw(2 * (size_t)(c.n - 1));
        for (uint32_t len = 2; len <= c.n; len <<= 1) {
            const double ang = -(2.0 * M_PI) / (double)len;
            for (uint32_t j = 0; j < len / 2; ++j) {
                double sn, cs;
                sincos(ang * (double)j, &sn, &cs);
                rtw[2 * (len / 2 - 1 + j)] = cs;
                rtw[2 * (len / 2 - 1 + j) + 1] = sn;
            }
        }
        HIP_TRY(hipMalloc(&st->d_rtw, rtw.size() * sizeof(double)));
        HIP_TRY(hipMemcpy(st->d_rtw, rtw.data(), rtw.size() * sizeof(double), hipMemcpyHostToDevice));
        HIP_TRY(hipMalloc(&st->d_tw512, t1.size() * sizeof(float)));
        HIP_TRY(hipMalloc(&st->d_tw1024, t2.size() * sizeof(float)));
        HIP_TRY(hipMalloc(&st->d_bins, bins.size() * sizeof(int)));
        HIP_TRY(hipMemcpy(st->d_tw512, t1.data(), t1.size() * sizeof(float), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(st->d_tw1024, t2.data(), t2.size() * sizeof(float), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(st->d_bins, bins.data(), bins.size() * sizeof(int), hipMemcpyHostToDevice));
    }
    // the tone plan's fp32 constants (error_model.cpp build_plan)
    st->reinsch = pl.reinsch;
    st->f16 = pl.f16;
    st->fold64 = pl.fold64;
    st->dcls = pl.dcls;
    st->perm = pl.perm;
    for (uint32_t k = 0; k < c.k; ++k) {
        st->coef[k] = pl.coef[k];
        st->sgn[k] = pl.sgn[k];
        st->zcls[k] = pl.zcls[k];
        st->rcoef[k] = pl.rcoef[k];
    }
    if (!pl.rot.empty()) {
        HIP_TRY(hipMalloc(&st->d_rot, pl.rot.size() * sizeof(float4)));
        HIP_TRY(hipMemcpy(st->d_rot, pl.rot.data(), pl.rot.size() * sizeof(float4), hipMemcpyHostToDevice));
    }
    // the in-kernel rescue's first pass (n = 1024): its tables (build_plan);
    // FSKD_RESCUE_SEG=0 (measurement switch) sends every flagged row to the
    // exact chain
    const char *seg_env = std::getenv("FSKD_RESCUE_SEG");
    const bool first_pass = !pl.rot64.empty() && !(seg_env && std::strcmp(seg_env, "0") == 0);
    if (!pl.rot64.empty()) {
        HIP_TRY(hipMalloc(&st->d_rot64, pl.rot64.size() * sizeof(double)));
        HIP_TRY(hipMemcpy(st->d_rot64, pl.rot64.data(), pl.rot64.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    // measurement switches: FSKD_NO_RESCUE=1 turns the rescue off, =flags
    // keeps the detectors' flags but skips the launch (the flagged windows'
    // symbols keep bit 7: counting them is how bench.py reports the rate)
    const char *no_rescue = std::getenv("FSKD_NO_RESCUE");
    st->rescue = c.k >= 2 && !(no_rescue && no_rescue[0] == '1');
    st->rescue_launch = !(no_rescue && std::strcmp(no_rescue, "flags") == 0);
    const char *rl_env = std::getenv("FSKD_RESCUE_LAUNCH");
    st->rescue_kernel_forced = rl_env && std::strcmp(rl_env, "1") == 0;
    const char *wb_env = std::getenv("FSKD_WB_BURSTS");
    st->wb_bursts = !(wb_env && std::strcmp(wb_env, "0") == 0);
    if (wb_env && std::atoi(wb_env) > 0) st->wb_force = std::min(std::atoi(wb_env), 64);
    if (st->rescue) {
        // Decision rescue thresholds, derived from the plan's
        // constants and the kernels' operation sequences (error_model.cpp):
        // stage 2 flags (P_1 - P_2)^2 < t2e E_eff P_1, stage 1 the same with
        // the int16 maximum of E_eff (tq, fl); pass 0 decides a flagged row
        // where its own margin clears t2e64 E P_max.
        ErrModel m;
        error_model(c, pl, first_pass, m);
        st->tau = m.tau;
        st->amb_tq = (float)m.tq;
        st->amb_floor = (float)m.fl;
        st->amb_t2e = (float)m.t2e;
        st->amb_d = (float)m.amb_d;
        st->tau64 = m.tau64;
        st->t2e64 = m.t2e64;
    }
    st->slide_wt = 0;
    if (slide && st->detector == kDetGoertzel)
        st->slide_wt = (64 - 16) / (int)(c.hop / 64) + 1;  // the last window's 16 segments end in the tile
    if (slide && st->detector == kDetFolded) {
        // 4 R windows (R per 16-lane group) whose 16 + (4R - 1) H segments fit the tile
        const int H = (int)(c.hop / 64);
        st->slide_wt = 4 * std::max(1, ((kFoldSlideSegs - 16) / H + 1) / 4);
    }
    return DEMOD_OK;
}

static void free_state(demod_t *st)
{
    if (st->stream) (void)hipStreamSynchronize(st->stream);
    if (st->d_rot) (void)hipFree(st->d_rot);
    if (st->d_rot64) (void)hipFree(st->d_rot64);
    if (st->d_tw512) (void)hipFree(st->d_tw512);
    if (st->d_tw1024) (void)hipFree(st->d_tw1024);
    if (st->d_bins) (void)hipFree(st->d_bins);
    if (st->d_rtw) (void)hipFree(st->d_rtw);
    if (st->d_in) (void)hipFree(st->d_in);
    if (st->d_sym) (void)hipFree(st->d_sym);
    if (st->d_mag) (void)hipFree(st->d_mag);
    if (st->h_in) (void)hipHostFree(st->h_in);
    if (st->h_sym) (void)hipHostFree(st->h_sym);
    if (st->h_mag) (void)hipHostFree(st->h_mag);
    if (st->z_in) (void)hipHostFree(st->z_in);
    if (st->z_sym) (void)hipHostFree(st->z_sym);
    if (st->z_mag) (void)hipHostFree(st->z_mag);
    if (st->copy_stream) (void)hipStreamSynchronize(st->copy_stream);
    for (int b = 0; b < 2; ++b) {
        if (st->copied[b]) (void)hipEventDestroy(st->copied[b]);
        if (st->consumed[b]) (void)hipEventDestroy(st->consumed[b]);
    }
    if (st->copy_stream) (void)hipStreamDestroy(st->copy_stream);
    if (st->stream) (void)hipStreamDestroy(st->stream);
}

demod_t *demod_create(const demod_cfg_t *cfg, int *error)
{
    int rc = validate(cfg);
    if (rc != DEMOD_OK) {
        if (error) *error = rc;
        return nullptr;
    }
    demod_t *st = new (std::nothrow) demod();
    if (!st) {
        if (error) *error = DEMOD_ALLOC_FAIL;
        return nullptr;
    }
    st->cfg = *cfg;
    DeviceGuard guard(cfg->device >= 0 ? cfg->device : 0);
    rc = init_device_state(st);
    if (rc != DEMOD_OK) {
        free_state(st);
        delete st;
        if (error) *error = rc;
        return nullptr;
    }
    st->carry.reserve(cfg->n);
    st->skip = cfg->lead_in;
    if (error) *error = DEMOD_OK;
    return st;
}

void demod_destroy(demod_t *st)
{
    if (!st) return;
    DeviceGuard guard(st->device);
    free_state(st);
    delete st;
}

int demod_reset(demod_t *st)
{
    if (!st) return DEMOD_BAD_ARG;
    st->carry.clear();
    st->skip = st->cfg.lead_in;
    return DEMOD_OK;
}

int demod_method(const demod_t *st)
{
    if (!st) return DEMOD_BAD_ARG;
    return st->detector == kDetFolded  ? DEMOD_METHOD_FOLDED
         : st->detector == kDetFft     ? DEMOD_METHOD_FFT
         : st->detector == kDetResidue ? DEMOD_METHOD_RESIDUE
                                       : DEMOD_METHOD_GOERTZEL;
}

int demod_slide_windows(const demod_t *st)
{
    if (!st) return DEMOD_BAD_ARG;
    return st->slide_wt;
}

int demod_pending(const demod_t *st)
{
    if (!st) return DEMOD_BAD_ARG;
    return (int)st->carry.size();
}

static size_t windows_for(const demod_t *st, size_t total)
{
    if (total < st->cfg.n) return 0;
    return (total - st->cfg.n) / st->cfg.hop + 1;
}

constexpr size_t kOutChunkBytes = 10u << 20;  // symbol + magnitude bytes per detector launch
constexpr size_t kBurstBytes = 5u << 20;      // output bytes per L2 write-back burst
constexpr size_t kBurstMinBytes = 4u << 20;   // smaller outputs: no bursts

// Windows per launch of a Goertzel-family batch (enqueue_batch): outputs
// beyond ~1 MiB per XCD L2 are written back to HBM while the input still
// streams in, and the read / write turnarounds cost ~1.3 us per MiB (8-FSK:
// 336.6 us with magnitudes vs 295.3 without); up to that size they stay dirty
// in L2 and go out in one burst at the kernel's end (2-FSK's 9 MiB: +1 us).
// So batches whose outputs exceed kOutChunkBytes run as equal slices of
// 64-window multiples (8-FSK: 4 launches, 322-325 us;
// scripts/split_launch_probe.py). Overlapping windows
// (hop < n) are bound by the recurrences and L2, not by HBM turnarounds, and
// only pay the extra launches there (2-FSK hop 128: 0.466 -> 0.494 ms), so
// they stay one launch, as does the VALU-bound FFT detector.
// Round 3: such a batch runs as ONE launch that writes each XCD's L2 back in
// bursts of ~kBurstBytes of output (wb_burst, demod_internal.h): no drain and
// ramp per slice (8-FSK 315-316 us against 331 us for the 4 slices and 337 us
// for one plain launch on one box, 309-310 / 324 / 316 us on another;
// scripts/mag_probe.hip wb). Batches from kBurstMinBytes up
// also take at least 4 bursts (2-FSK's 9 MiB: 0.3006 ms against 0.3058 ms
// with one write-back at the kernel's end, scripts/gpu_r3_wb2.sh).
// FSKD_WB_BURSTS=0 keeps the round-2 behaviour (slices, no bursts).
static size_t out_bytes(const demod_t *st, size_t n_windows, bool mags)
{
    return n_windows * (1 + (mags ? 4 * (size_t)st->cfg.k : 0));
}
static bool large_output(const demod_t *st, size_t n_windows, bool mags)
{
    return st->detector != kDetFft && st->cfg.hop >= st->cfg.n && n_windows &&
           out_bytes(st, n_windows, mags) > kOutChunkBytes;
}
static size_t launch_slice(const demod_t *st, size_t n_windows, bool mags)
{
    if (!large_output(st, n_windows, mags) || st->wb_bursts) return n_windows;
    const size_t parts = std::min<size_t>((out_bytes(st, n_windows, mags) + kOutChunkBytes - 1) / kOutChunkBytes, 16);
    const size_t per = (n_windows + parts - 1) / parts;
    return (per + 63) / 64 * 64;
}
static int burst_count(const demod_t *st, size_t n_windows, bool mags)
{
    if (st->wb_force && st->detector != kDetFft && st->cfg.hop >= st->cfg.n) return st->wb_force;
    if (!st->wb_bursts || st->detector == kDetFft || st->cfg.hop < st->cfg.n) return 0;
    const size_t out = out_bytes(st, n_windows, mags);
    if (out < kBurstMinBytes) return 0;
    return (int)std::min<size_t>(std::max<size_t>((out + kBurstBytes - 1) / kBurstBytes, 4), 64);
}

// The direct Goertzel-family kernels at n = 1024 (plain bank, fold, residue;
// any hop without segment sharing) re-decide their flagged windows inside the
// detector kernel (rescue_rows, demod_internal.h) from the tile they hold in
// LDS: no rescue launch. Segment-shared windows (SLIDE, fold_slide_kernel)
// and other window lengths keep rescue_kernel's launch; the FFT detector
// always rescues in its own kernel (rescue_fft.h).
static bool rescue_in_kernel(const demod_t *st)
{
    // the residue detector's plans take the rescue launch (round 5): its first
    // pass by the residue fold lives there (its per-lane class data would not
    // fit the residue kernels' registers). Worst case (every window a near
    // tie) 2.09 -> 1.59 ms per 2^20 8-FSK windows on bins 32 + 9i; the extra
    // launch costs the clean step 0.4-0.75 % (0.3446 vs 0.3420 ms,
    // profiles/round5/r5zg/, r5zh/)
    if (st->detector == kDetResidue && st->fold64 == 2) return false;
    return st->detector != kDetFft && st->log2g == 4 && st->slide_wt == 0 && !st->rescue_kernel_forced;
}

double demod_rescue_tau(const demod_t *st)
{
    if (!st || !st->rescue) return 0.0;
    return st->tau;
}

double demod_rescue_tau64(const demod_t *st)
{
    // every rescue at n = 1024 runs the first pass (round 5: the rescue launch
    // of segment-shared windows too, rescue.hip rescue_seg_kernel)
    if (!st || !st->rescue || !st->d_rot64) return 0.0;
    return st->tau64;
}

int demod_batch_launches(const demod_t *st, size_t n_windows, int with_mags)
{
    if (!st) return DEMOD_BAD_ARG;
    if (n_windows == 0) return 0;
    const size_t per = launch_slice(st, n_windows, with_mags != 0);
    // + the decision rescue's launch (the FFT detector rescues in the kernel)
    const size_t n = (n_windows + per - 1) / per +
                     (st->rescue && st->rescue_launch && st->detector != kDetFft &&
                              !rescue_in_kernel(st) ? 1 : 0);
    return n > 0x7FFFFFFF ? 0x7FFFFFFF : (int)n;
}

// The decision rescue over a batch's windows (rescue.hip), after its detector
// launches on the same stream.
static int enqueue_rescue(demod_t *st, const int16_t *d_pcm, size_t n_windows, uint8_t *d_sym,
                          float *d_mag, hipStream_t s)
{
    if (!st->rescue || !st->rescue_launch || n_windows == 0 || rescue_in_kernel(st)) return DEMOD_OK;
    RescueParams r;
    std::memset(&r, 0, sizeof(r));
    r.pcm = d_pcm;
    r.n_windows = (long long)n_windows;
    r.hop = st->cfg.hop;
    r.n = (int)st->cfg.n;
    r.k = (int)st->cfg.k;
    r.sym = d_sym;
    r.sym_aligned4 = ((uintptr_t)d_sym & 3) == 0;
    r.mag = d_mag;
    for (uint32_t k = 0; k < st->cfg.k; ++k) r.coef[k] = st->rcoef[k];
    // n = 1024: the segment-shared windows' rescue takes the first pass too
    // (the in-kernel rescue's tables and threshold, error_model.cpp)
    r.rot64 = st->d_rot64;
    r.t2e64 = st->d_rot64 ? st->t2e64 : 0.0;
    r.fold64 = st->fold64;
    HIP_TRY(launch_rescue(r, s));
    return DEMOD_OK;
}

int demod_max_symbols(const demod_t *st, size_t n_frames)
{
    if (!st) return DEMOD_BAD_ARG;
    const size_t fresh = n_frames > st->skip ? n_frames - st->skip : 0;
    size_t w = windows_for(st, st->carry.size() + fresh);
    return w > 0x7FFFFFFF ? 0x7FFFFFFF : (int)w;
}

static int enqueue_fft(demod_t *st, const int16_t *d_pcm, size_t n_windows, uint8_t *d_sym,
                       float *d_mag, float *d_spec, hipStream_t s)
{
    FftParams p;
    std::memset(&p, 0, sizeof(p));
    p.pcm = d_pcm;
    p.n_windows = (long long)n_windows;
    p.hop = st->cfg.hop;
    p.k = (int)st->cfg.k;
    p.xcd_swizzle = 1;  // neighbouring groups on one L2: shared input lines, whole output lines
    p.tw512 = st->d_tw512;
    p.tw1024 = st->d_tw1024;
    p.bins = st->d_bins;
    for (uint32_t k = 0; k < st->cfg.k; ++k) p.slot[k] = st->fft_slot[k];
    p.pmask = st->fft_pmask;
    p.sym = d_sym;
    p.mag = d_mag;
    p.spec = d_spec;
    p.amb_tq = st->amb_tq;
    p.amb_floor = st->amb_floor;
    p.amb_t2e = st->amb_t2e;
    // the FFT detector re-decides its flagged windows itself (rescue_fft.h):
    // one launch, no symbol scan
    p.rescue = st->rescue && st->rescue_launch ? 1 : 0;
    p.rtw = st->d_rtw;
    // the rescue's first pass (tones only; with the spectrum stored every
    // flagged window takes the double FFT, whose spectrum row is the oracle's)
    p.rot64 = st->d_rot64;
    p.t2e64 = st->t2e64;
    p.fold64 = st->fold64 == 1 ? 1 : 0;
    HIP_TRY(launch_fft_quad(p, s));
    return (int)n_windows;
}


// Enqueue the detector kernel on device-resident windows.
static int enqueue_batch(demod_t *st, const int16_t *d_pcm, size_t n_windows, uint8_t *d_sym,
                         float *d_mag, hipStream_t s)
{
    if (n_windows == 0) return 0;
    if (st->detector == kDetFft) return enqueue_fft(st, d_pcm, n_windows, d_sym, d_mag, nullptr, s);
    GoertzelParams p;
    std::memset(&p, 0, sizeof(p));
    p.pcm = d_pcm;
    p.n_windows = (long long)n_windows;
    p.hop = st->cfg.hop;
    p.log2g = st->log2g;
    p.k = (int)st->cfg.k;
    p.rot = st->d_rot;
    p.sym = d_sym;
    p.mag = d_mag;
    for (uint32_t k = 0; k < st->cfg.k; ++k) {
        p.coef[k] = st->coef[k];
        p.sgn[k] = st->sgn[k];
        p.zcls[k] = st->zcls[k];
    }
    p.reinsch = st->reinsch ? 1 : 0;
    p.dcls = st->dcls;
    p.f16 = st->f16 ? 1 : 0;
    p.perm = st->perm;
    p.slide_wt = st->slide_wt;
    // overlapping windows: neighbouring tiles share lines, keep them in L2
    p.cached = st->cfg.hop < st->cfg.n ? 1 : 0;
    // adjacent tiles on one XCD: their symbol / magnitude stores fill whole
    // lines in that XCD's L2 instead of eight L2s writing back pieces of the
    // same line (2-FSK: 0.325 -> 0.305 ms), and overlapping
    // windows find their shared lines there
    p.xcd_swizzle = 1;
    p.amb_tq = st->amb_tq;
    p.amb_floor = st->amb_floor;
    p.amb_t2e = st->amb_t2e;
    const size_t per = launch_slice(st, n_windows, d_mag != nullptr);
    p.wb_bursts = burst_count(st, n_windows, d_mag != nullptr);
    p.rescue_inline = st->rescue && st->rescue_launch && rescue_in_kernel(st) ? 1 : 0;
    for (uint32_t k = 0; k < st->cfg.k; ++k) p.rcoef[k] = st->rcoef[k];
    // the in-kernel rescue's tables; its first pass's threshold^2 = t2e64 E
    // P_max, E = sum x^2 (fp32 in the kernel; error_model's safety factor
    // covers its rounding), 0: the exact chain only
    p.rot64 = st->d_rot64;
    p.t2e64 = st->t2e64;
    p.fold64 = st->fold64 == 1 ? 1 : 0;  // rescue_rows: by the fold (the residue fold: the launch)
    p.amb_d = st->amb_d;
    for (size_t w0 = 0; w0 < n_windows; w0 += per) {
        const size_t cnt = std::min(per, n_windows - w0);
        p.pcm = d_pcm + w0 * st->cfg.hop;
        p.n_windows = (long long)cnt;
        p.sym = d_sym + w0;
        p.mag = d_mag ? d_mag + w0 * st->cfg.k : nullptr;
        HIP_TRY(launch_detector(st->detector, p, s));
    }
    const int rc = enqueue_rescue(st, d_pcm, n_windows, d_sym, d_mag, s);
    return rc < 0 ? rc : (int)n_windows;
}

static int ensure_dev(demod_t *st, size_t samples, size_t windows, bool mags)
{
    if (samples > st->d_in_cap) {
        if (st->d_in) (void)hipFree(st->d_in);
        st->d_in = nullptr;
        st->d_in_cap = 0;
        size_t cap = samples + samples / 4 + 64;
        HIP_TRY(hipMalloc(&st->d_in, cap * sizeof(int16_t)));
        st->d_in_cap = cap;
    }
    if (windows > st->d_out_cap || (mags && !st->d_mag)) {
        if (st->d_sym) (void)hipFree(st->d_sym);
        if (st->d_mag) (void)hipFree(st->d_mag);
        st->d_sym = nullptr;
        st->d_mag = nullptr;
        st->d_out_cap = 0;
        size_t cap = windows + windows / 4 + 16;
        HIP_TRY(hipMalloc(&st->d_sym, cap));
        HIP_TRY(hipMalloc(&st->d_mag, cap * st->cfg.k * sizeof(float)));
        st->d_out_cap = cap;
    }
    return DEMOD_OK;
}

static bool is_device_ptr(const void *p)
{
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Host samples [n_samples] -> device, kernel, results -> host (synchronous).
// The input goes to the device in chunks of kChunkWindows windows straight from
// the caller's (pageable) buffer — hipMemcpyAsync moves pageable memory at the
// PCIe rate (57 GB/s pinned vs 56.5 GB/s pageable measured), so a host-side
// staging copy would only add a memcpy — into two alternating device slots, so
// the kernel of chunk c runs while chunk c + 1 is in flight. Symbols and
// magnitudes land in device buffers and come back with one copy each.
static constexpr size_t kChunkWindows = 1 << 16;  // 128 MiB of input at n = hop = 1024

static constexpr size_t kSmallHostSamples = 1 << 21;  // 4 MiB: pinned-staging path
static constexpr size_t kPushThreads = 8;              // demod_streams_push staging threads

static int ensure_host(demod_t *st, size_t samples, size_t windows)
{
    if (samples > st->h_in_cap) {
        if (st->h_in) (void)hipHostFree(st->h_in);
        st->h_in = nullptr;
        st->h_in_cap = 0;
        HIP_TRY(hipHostMalloc(&st->h_in, samples * sizeof(int16_t), hipHostMallocDefault));
        st->h_in_cap = samples;
    }
    if (windows > st->h_out_cap) {
        if (st->h_sym) (void)hipHostFree(st->h_sym);
        if (st->h_mag) (void)hipHostFree(st->h_mag);
        st->h_sym = nullptr;
        st->h_mag = nullptr;
        st->h_out_cap = 0;
        HIP_TRY(hipHostMalloc(&st->h_sym, windows, hipHostMallocDefault));
        HIP_TRY(hipHostMalloc(&st->h_mag, windows * st->cfg.k * sizeof(float), hipHostMallocDefault));
        st->h_out_cap = windows;
    }
    return DEMOD_OK;
}

// Packet-sized calls (a 60 ms packet plus the carry is <= 3903 samples):
// mapped, coherent (uncached on the device) pinned buffers. The kernel's
// buffer loads read the samples over PCIe and its stores write the results
// back, so a call is one launch and one synchronize instead of an H2D copy, a
// launch, a D2H copy and the synchronize. The kernels' loads are bounded by
// the buffer descriptor's record count, so nothing past the call's samples is
// touched. If the runtime cannot map the memory the copy path below serves.
static constexpr size_t kZeroCopySamples = 1 << 14;   // 32 KiB: 16 windows at hop n

static int ensure_zero_copy(demod_t *st)
{
    if (st->zc) return st->zc;
    if (std::getenv("FSKD_NO_ZERO_COPY")) return st->zc = -1;  // measurement switch
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    const size_t wmax = kZeroCopySamples / 8;  // hop >= 8
    bool ok = hipHostMalloc(&st->z_in, kZeroCopySamples * sizeof(int16_t), fl) == hipSuccess &&
              hipHostMalloc(&st->z_sym, wmax, fl) == hipSuccess &&
              hipHostMalloc(&st->z_mag, wmax * st->cfg.k * sizeof(float), fl) == hipSuccess &&
              hipHostGetDevicePointer((void **)&st->zd_in, st->z_in, 0) == hipSuccess &&
              hipHostGetDevicePointer((void **)&st->zd_sym, st->z_sym, 0) == hipSuccess &&
              hipHostGetDevicePointer((void **)&st->zd_mag, st->z_mag, 0) == hipSuccess &&
              ((uintptr_t)st->zd_in & 15) == 0;
    if (!ok) (void)hipGetLastError();
    st->zc = ok ? 1 : -1;
    return st->zc;
}

static int run_host_zero_copy(demod_t *st, const int16_t *pcm, size_t n_samples, size_t n_windows,
                              uint8_t *symbols, float *mags)
{
    std::memcpy(st->z_in, pcm, n_samples * sizeof(int16_t));
    int rc = enqueue_batch(st, st->zd_in, n_windows, st->zd_sym, mags ? st->zd_mag : nullptr,
                           st->stream);
    if (rc < 0) return rc;
    HIP_TRY(hipStreamSynchronize(st->stream));
    std::memcpy(symbols, st->z_sym, n_windows);
    if (mags) std::memcpy(mags, st->z_mag, n_windows * st->cfg.k * sizeof(float));
    return (int)n_windows;
}

// Small calls: one pinned round trip on one stream — 20 us per packet,
// against ~50 us through the chunked path's pageable copies and cross-stream
// events.
static int run_host_small(demod_t *st, const int16_t *pcm, size_t n_samples, size_t n_windows,
                          uint8_t *symbols, float *mags)
{
    int rc;
    if (n_samples <= kZeroCopySamples && ensure_zero_copy(st) == 1)
        return run_host_zero_copy(st, pcm, n_samples, n_windows, symbols, mags);
    if ((rc = ensure_dev(st, n_samples, n_windows, mags != nullptr)) != DEMOD_OK) return rc;
    if ((rc = ensure_host(st, kSmallHostSamples, kSmallHostSamples / 8)) != DEMOD_OK) return rc;
    if (pcm != st->h_in) std::memcpy(st->h_in, pcm, n_samples * sizeof(int16_t));
    HIP_TRY(hipMemcpyAsync(st->d_in, st->h_in, n_samples * sizeof(int16_t), hipMemcpyHostToDevice,
                           st->stream));
    rc = enqueue_batch(st, st->d_in, n_windows, st->d_sym, mags ? st->d_mag : nullptr, st->stream);
    if (rc < 0) return rc;
    HIP_TRY(hipMemcpyAsync(st->h_sym, st->d_sym, n_windows, hipMemcpyDeviceToHost, st->stream));
    if (mags)
        HIP_TRY(hipMemcpyAsync(st->h_mag, st->d_mag, n_windows * st->cfg.k * sizeof(float),
                               hipMemcpyDeviceToHost, st->stream));
    HIP_TRY(hipStreamSynchronize(st->stream));
    std::memcpy(symbols, st->h_sym, n_windows);
    if (mags) std::memcpy(mags, st->h_mag, n_windows * st->cfg.k * sizeof(float));
    return (int)n_windows;
}

static int run_host(demod_t *st, const int16_t *pcm, size_t n_samples, size_t n_windows,
                    uint8_t *symbols, float *mags)
{
    // windows <= samples / 8 (hop >= 8), so the pinned outputs always fit
    if (n_samples <= kSmallHostSamples)
        return run_host_small(st, pcm, n_samples, n_windows, symbols, mags);
    const size_t hop = st->cfg.hop, n = st->cfg.n;
    const size_t cw = std::min(n_windows, kChunkWindows);
    const size_t slot = (cw - 1) * hop + n;  // samples per device slot
    int rc;
    if ((rc = ensure_dev(st, 2 * slot, n_windows, mags != nullptr)) != DEMOD_OK) return rc;
    if (!st->copy_stream) {
        HIP_TRY(hipStreamCreateWithFlags(&st->copy_stream, hipStreamNonBlocking));
        for (int b = 0; b < 2; ++b) {
            HIP_TRY(hipEventCreateWithFlags(&st->copied[b], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&st->consumed[b], hipEventDisableTiming));
        }
    }
    for (size_t w0 = 0, c = 0; w0 < n_windows; w0 += cw, ++c) {
        const int b = (int)(c & 1);
        const size_t nw = std::min(cw, n_windows - w0);
        const size_t ns = (nw - 1) * hop + n;
        int16_t *d = st->d_in + b * slot;
        if (c >= 2) HIP_TRY(hipStreamWaitEvent(st->copy_stream, st->consumed[b], 0));
        HIP_TRY(hipMemcpyAsync(d, pcm + w0 * hop, ns * sizeof(int16_t), hipMemcpyHostToDevice,
                               st->copy_stream));
        HIP_TRY(hipEventRecord(st->copied[b], st->copy_stream));
        HIP_TRY(hipStreamWaitEvent(st->stream, st->copied[b], 0));
        rc = enqueue_batch(st, d, nw, st->d_sym + w0, mags ? st->d_mag + w0 * st->cfg.k : nullptr,
                           st->stream);
        if (rc < 0) return rc;
        HIP_TRY(hipEventRecord(st->consumed[b], st->stream));
    }
    HIP_TRY(hipMemcpyAsync(symbols, st->d_sym, n_windows, hipMemcpyDeviceToHost, st->stream));
    if (mags)
        HIP_TRY(hipMemcpyAsync(mags, st->d_mag, n_windows * st->cfg.k * sizeof(float),
                               hipMemcpyDeviceToHost, st->stream));
    HIP_TRY(hipStreamSynchronize(st->stream));
    return (int)n_windows;
}

int demod_batch(demod_t *st, const int16_t *pcm, size_t n_windows, uint8_t *symbols, float *mags)
{
    if (!st || (!pcm && n_windows) || (!symbols && n_windows)) return DEMOD_BAD_ARG;
    if (n_windows > 0x7FFFFFFF) return DEMOD_BAD_ARG;
    if (n_windows == 0) return 0;
    if (((uintptr_t)pcm & 15) != 0) return DEMOD_BAD_ARG;
    DeviceGuard guard(st->device);
    HIP_TRY(guard.err);
    const size_t n_samples = (n_windows - 1) * st->cfg.hop + st->cfg.n;
    const bool din = is_device_ptr(pcm), dsym = is_device_ptr(symbols);
    const bool dmag = mags ? is_device_ptr(mags) : dsym;
    if (din && dsym && dmag) {
        int rc = enqueue_batch(st, pcm, n_windows, symbols, mags, st->stream);
        if (rc < 0) return rc;
        HIP_TRY(hipStreamSynchronize(st->stream));
        return rc;
    }
    if (!din && !dsym && !dmag) return run_host(st, pcm, n_samples, n_windows, symbols, mags);
    return DEMOD_BAD_ARG;  // mixed host/device pointers
}

int demod_batch_async(demod_t *st, const int16_t *d_pcm, size_t n_windows, uint8_t *d_symbols,
                      float *d_mags, void *stream)
{
    if (!st || (!d_pcm && n_windows) || (!d_symbols && n_windows)) return DEMOD_BAD_ARG;
    if (n_windows > 0x7FFFFFFF) return DEMOD_BAD_ARG;
    if (((uintptr_t)d_pcm & 15) != 0) return DEMOD_BAD_ARG;
    if (n_windows == 0) return 0;
    DeviceGuard guard(st->device);
    HIP_TRY(guard.err);
    return enqueue_batch(st, d_pcm, n_windows, d_symbols, d_mags, (hipStream_t)stream);
}

int demod_batch_spectrum_async(demod_t *st, const int16_t *d_pcm, size_t n_windows,
                               uint8_t *d_symbols, float *d_mags, float *d_spectrum, void *stream)
{
    if (!st || (!d_pcm && n_windows) || (!d_symbols && n_windows)) return DEMOD_BAD_ARG;
    if (st->detector != kDetFft) return DEMOD_UNIMPLEMENTED;
    if (n_windows > 0x7FFFFFFF) return DEMOD_BAD_ARG;
    if (((uintptr_t)d_pcm & 15) != 0) return DEMOD_BAD_ARG;
    if (n_windows == 0) return 0;
    DeviceGuard guard(st->device);
    HIP_TRY(guard.err);
    return enqueue_fft(st, d_pcm, n_windows, d_symbols, d_mags, d_spectrum, (hipStream_t)stream);
}

// The mono samples of n_frames frames (cfg.channels interleaved): the
// channel cfg.channel_mode selects, or (L + R) >> 1.
static void mono_frames(const demod_cfg_t &c, const int16_t *pcm, size_t n_frames, int16_t *dst)
{
    if (c.channels == 1) {
        if (n_frames) std::memcpy(dst, pcm, n_frames * sizeof(int16_t));
    } else if (c.channel_mode == DEMOD_CH_DOWNMIX) {
        for (size_t i = 0; i < n_frames; ++i)
            dst[i] = (int16_t)(((int32_t)pcm[2 * i] + (int32_t)pcm[2 * i + 1]) >> 1);
    } else {
        const int ch = c.channel_mode == DEMOD_CH_RIGHT ? 1 : 0;
        for (size_t i = 0; i < n_frames; ++i) dst[i] = pcm[2 * i + ch];
    }
}

int demodulate_mags(demod_t *st, const int16_t *pcm, size_t n_frames, uint8_t *symbols,
                    float *mags, size_t max_symbols)
{
    if (!st || (!pcm && n_frames)) return DEMOD_BAD_ARG;
    const demod_cfg_t &c = st->cfg;
    // lead-in (cfg.lead_in): the first frames of a stream are dropped, e.g. the
    // Opus decoder delay (OPUS_GET_LOOKAHEAD, 312 samples at 48 kHz for the
    // transmitter's settings, OpusEncoder.kt:65-67), so windows line up with
    // the transmitter's symbol boundaries
    const size_t drop = std::min(st->skip, n_frames);
    pcm += drop * c.channels;
    n_frames -= drop;
    const size_t have = st->carry.size();
    const size_t total = have + n_frames;
    const size_t W = windows_for(st, total);
    if (W > max_symbols) return DEMOD_BUFFER_TOO_SMALL;
    if (W && !symbols) return DEMOD_BAD_ARG;
    if (W > 0x7FFFFFFF) return DEMOD_BAD_ARG;
    DeviceGuard guard(st->device);
    HIP_TRY(guard.err);
    // Mono view: carried samples followed by the new frames' selected channel.
    // Packet-sized calls (the playback.cpp:118 position: 2880 frames) build it
    // straight in the pinned staging buffer the small-call path copies from.
    int16_t *m = nullptr;
    if (W && total <= kSmallHostSamples) {
        int rc = ensure_host(st, kSmallHostSamples, kSmallHostSamples / 8);
        if (rc != DEMOD_OK) return rc;
        m = st->h_in;
    } else {
        st->scratch.resize(total);
        m = st->scratch.data();
    }
    if (have) std::memcpy(m, st->carry.data(), have * sizeof(int16_t));
    mono_frames(c, pcm, n_frames, m + have);
    if (W) {
        const size_t used = (W - 1) * c.hop + c.n;
        int rc = run_host(st, m, used, W, symbols, mags);
        if (rc < 0) return rc;  // nothing consumed on failure
    }
    const size_t consumed = W * c.hop;
    st->carry.assign(m + consumed, m + total);
    st->skip -= drop;
    return (int)W;
}

int demodulate(demod_t *st, const int16_t *pcm, size_t n_frames, uint8_t *symbols,
               size_t max_symbols)
{
    return demodulate_mags(st, pcm, n_frames, symbols, nullptr, max_symbols);
}

}  // extern "C"

// Many streams behind one detector handle (mono, the streams' n and hop). A
// push lays the streams' runs of complete windows end to end in one batch,
// each run starting on a multiple of hop, so the batch is an ordinary
// hop-strided window sequence: stream s's windows are batch windows
// first[s] .. first[s] + W_s - 1, and the ceil(L_s / hop) - W_s windows that
// start inside its run but end past it (n / hop - 1 of them when hop divides
// n; none at hop = n) straddle into the next run and are computed and
// dropped. One H2D copy of each run (the overlapping samples once), one
// detector launch (at hop = 64 H the segment-shared kernels, as a per-stream
// handle would run) and one D2H copy serve all streams.
// Persistent staging threads of one streams handle (the
// first build spawned and joined up to 7 std::threads inside every push).
// Workers sleep on a condition variable between pushes; run() hands worker k
// the stream range [k per, (k + 1) per), does range 0 on the calling thread
// and waits for the rest. A worker that cannot be started leaves its range
// to the caller.
struct StagePool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable go, done;
    const std::function<void(size_t, size_t)> *job = nullptr;
    size_t per = 0, S = 0, active = 0, pending = 0;
    unsigned long long gen = 0;
    bool stop = false;

    ~StagePool()
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        go.notify_all();
        for (auto &t : th) t.join();
    }
    void worker(size_t k)
    {
        unsigned long long seen = 0;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            go.wait(lk, [&] { return stop || gen != seen; });
            if (stop) return;
            seen = gen;
            if (k >= active) continue;
            const size_t a = k * per, e = std::min(S, a + per);
            const auto *f = job;
            lk.unlock();
            if (a < e) (*f)(a, e);
            lk.lock();
            if (--pending == 0) done.notify_one();
        }
    }
    // f(a, e) stages streams [a, e); T ranges in all (T - 1 on workers)
    void run(size_t T, size_t n, const std::function<void(size_t, size_t)> &f)
    {
        while (th.size() + 1 < T) {
            try {
                const size_t k = th.size() + 1;
                th.emplace_back([this, k] { worker(k); });
            } catch (...) {
                break;
            }
        }
        T = std::min(T, th.size() + 1);
        const size_t pr = (n + T - 1) / T;
        {
            std::lock_guard<std::mutex> lk(mu);
            job = &f;
            per = pr;
            S = n;
            active = T;
            pending = T - 1;
            ++gen;
        }
        if (T > 1) go.notify_all();
        f(0, std::min(n, pr));
        std::unique_lock<std::mutex> lk(mu);
        done.wait(lk, [&] { return pending == 0; });
        job = nullptr;
    }
};

struct demod_streams {
    demod_cfg_t cfg;                      // the streams' configuration
    demod_t *st = nullptr;                // detector handle: same n, hop, tones; mono
    std::vector<std::vector<int16_t>> carry;
    std::vector<size_t> skip;             // lead-in frames still to drop per stream
    std::vector<size_t> first;            // per push: batch window of each stream's first
    std::vector<size_t> have;             // per push: carry lengths before it
    std::vector<uint8_t> sym;             // per push: batch symbols / magnitudes
    std::vector<float> mag;
    std::vector<int16_t> dec;             // push_packets: [stream][frame_size x channels] decoded PCM
    std::vector<size_t> dec_frames;
    std::vector<const int16_t *> dec_ptr;
    StagePool pool;                       // staging threads of large pushes
    // FSKD_STREAMS_MAPPED=1 (measurement switch, read at create): the push
    // stages into mapped pinned memory that the detector reads in place over
    // PCIe and writes its results back to, instead of one H2D copy of the
    // staging buffer and a D2H copy of the results
    bool mapped = false;
    int16_t *zm_in = nullptr, *zmd_in = nullptr;
    size_t zm_cap = 0;                    // samples
    uint8_t *zm_sym = nullptr, *zmd_sym = nullptr;
    float *zm_mag = nullptr, *zmd_mag = nullptr;
    size_t zm_wcap = 0;                   // windows
    ~demod_streams()
    {
        if (zm_in) (void)hipHostFree(zm_in);
        if (zm_sym) (void)hipHostFree(zm_sym);
        if (zm_mag) (void)hipHostFree(zm_mag);
    }
};

// Mapped staging of a push (demod_streams::mapped): samples and windows.
static int ensure_mapped(demod_streams_t *ms, size_t samples, size_t windows)
{
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    if (samples > ms->zm_cap) {
        if (ms->zm_in) (void)hipHostFree(ms->zm_in);
        ms->zm_in = ms->zmd_in = nullptr;
        ms->zm_cap = 0;
        const size_t cap = samples + samples / 4 + 4096;
        HIP_TRY(hipHostMalloc(&ms->zm_in, cap * sizeof(int16_t), fl));
        HIP_TRY(hipHostGetDevicePointer((void **)&ms->zmd_in, ms->zm_in, 0));
        ms->zm_cap = cap;
    }
    if (windows > ms->zm_wcap) {
        if (ms->zm_sym) (void)hipHostFree(ms->zm_sym);
        if (ms->zm_mag) (void)hipHostFree(ms->zm_mag);
        ms->zm_sym = ms->zmd_sym = nullptr;
        ms->zm_mag = ms->zmd_mag = nullptr;
        ms->zm_wcap = 0;
        const size_t cap = windows + windows / 4 + 64;
        HIP_TRY(hipHostMalloc(&ms->zm_sym, cap, fl));
        HIP_TRY(hipHostMalloc(&ms->zm_mag, cap * ms->cfg.k * sizeof(float), fl));
        HIP_TRY(hipHostGetDevicePointer((void **)&ms->zmd_sym, ms->zm_sym, 0));
        HIP_TRY(hipHostGetDevicePointer((void **)&ms->zmd_mag, ms->zm_mag, 0));
        ms->zm_wcap = cap;
    }
    return DEMOD_OK;
}

extern "C" {

demod_streams_t *demod_streams_create(const demod_cfg_t *cfg, size_t n_streams, int *error)
{
    int rc = validate(cfg);
    if (rc == DEMOD_OK && (n_streams < 1 || n_streams > ((size_t)1 << 24))) rc = DEMOD_BAD_ARG;
    if (rc != DEMOD_OK) {
        if (error) *error = rc;
        return nullptr;
    }
    demod_streams_t *ms = new (std::nothrow) demod_streams();
    if (!ms) {
        if (error) *error = DEMOD_ALLOC_FAIL;
        return nullptr;
    }
    ms->cfg = *cfg;
    demod_cfg_t dc = *cfg;
    dc.channels = 1;
    dc.channel_mode = DEMOD_CH_LEFT;
    dc.lead_in = 0;
    ms->st = demod_create(&dc, &rc);
    if (!ms->st) {
        delete ms;
        if (error) *error = rc;
        return nullptr;
    }
    const char *mp = std::getenv("FSKD_STREAMS_MAPPED");
    ms->mapped = mp && mp[0] == '1';
    try {
        ms->carry.resize(n_streams);
        ms->skip.assign(n_streams, cfg->lead_in);
        ms->first.assign(n_streams, 0);
    } catch (...) {
        demod_destroy(ms->st);
        delete ms;
        if (error) *error = DEMOD_ALLOC_FAIL;
        return nullptr;
    }
    if (error) *error = DEMOD_OK;
    return ms;
}

void demod_streams_destroy(demod_streams_t *ms)
{
    if (!ms) return;
    demod_destroy(ms->st);
    delete ms;
}

int demod_streams_reset(demod_streams_t *ms, size_t stream)
{
    if (!ms || stream >= ms->carry.size()) return DEMOD_BAD_ARG;
    ms->carry[stream].clear();
    ms->skip[stream] = ms->cfg.lead_in;
    return DEMOD_OK;
}

int demod_streams_pending(const demod_streams_t *ms, size_t stream)
{
    if (!ms || stream >= ms->carry.size()) return DEMOD_BAD_ARG;
    return (int)ms->carry[stream].size();
}

static size_t streams_windows(const demod_streams_t *ms, size_t s, size_t n_frames)
{
    const size_t fresh = n_frames > ms->skip[s] ? n_frames - ms->skip[s] : 0;
    const size_t total = ms->carry[s].size() + fresh;
    return total < ms->cfg.n ? 0 : (total - ms->cfg.n) / ms->cfg.hop + 1;
}

}  // extern "C"

// Every refusal demod_streams_push makes from its arguments and the handle's
// state, before anything is consumed (all but the caller's cap and symbols
// buffer), and the symbols each stream will emit (exactly what the push
// writes to counts; nullable). demod_group.cpp runs it on every rank before
// the first collective, so a refusal is agreed on rather than met mid-protocol.
// Returns the total, or the push's negative code.
long long fskd::streams_check(const demod_streams_t *ms, const int16_t *const *pcm, const size_t *n_frames,
                              uint32_t *counts)
{
    if (!ms || !n_frames) return DEMOD_BAD_ARG;
    const size_t S = ms->carry.size(), n = ms->cfg.n, hop = ms->cfg.hop;
    size_t W = 0, Wb = 0;
    for (size_t s = 0; s < S; ++s) {
        if (n_frames[s] && (!pcm || !pcm[s])) return DEMOD_BAD_ARG;
        if (n_frames[s] > ((size_t)1 << 40)) return DEMOD_BAD_ARG;
        const size_t w = streams_windows(ms, s, n_frames[s]);
        if (counts) counts[s] = (uint32_t)w;
        W += w;
        if (w) Wb += ((w - 1) * hop + n + hop - 1) / hop;  // ceil(L_s / hop): the batch slots
    }
    if (W > 0x7FFFFFFF || W * n > ((size_t)1 << 40)) return DEMOD_BAD_ARG;
    // the batch also counts the straddling windows that are computed and
    // dropped, up to ~W n / hop: it must still fit an int count
    if (Wb > 0x7FFFFFFF || Wb * hop > ((size_t)1 << 40)) return DEMOD_BAD_ARG;
    return (long long)W;
}

int fskd::streams_device(const demod_streams_t *ms) { return ms ? ms->st->device : -1; }

extern "C" {

long long demod_streams_max_symbols(const demod_streams_t *ms, const size_t *n_frames)
{
    if (!ms || !n_frames) return DEMOD_BAD_ARG;
    long long w = 0;
    for (size_t s = 0; s < ms->carry.size(); ++s) w += (long long)streams_windows(ms, s, n_frames[s]);
    return w;
}

int demod_streams_push(demod_streams_t *ms, const int16_t *const *pcm, const size_t *n_frames,
                       uint8_t *symbols, float *mags, size_t cap, uint32_t *counts)
{
    if (!ms || !n_frames || !counts) return DEMOD_BAD_ARG;
    const demod_cfg_t &c = ms->cfg;
    const size_t S = ms->carry.size(), n = c.n, hop = c.hop;
    const long long Wc = fskd::streams_check(ms, pcm, n_frames, nullptr);
    if (Wc < 0) return (int)Wc;
    const size_t W = (size_t)Wc;
    if (W > cap) return DEMOD_BUFFER_TOO_SMALL;
    if (W && !symbols) return DEMOD_BAD_ARG;
    demod_t *st = ms->st;
    DeviceGuard guard(st->device);
    HIP_TRY(guard.err);
    // every carry holds < n samples after a push: reserve n once so the
    // carry updates below never allocate
    std::vector<size_t> &have = ms->have;
    try {
        have.resize(S);
        for (size_t s = 0; s < S; ++s) {
            ms->carry[s].reserve(n);
            have[s] = ms->carry[s].size();
        }
    } catch (...) {
        return DEMOD_ALLOC_FAIL;
    }
    auto fresh = [&](size_t s) { return n_frames[s] - std::min(ms->skip[s], n_frames[s]); };
    auto windows = [&](size_t total) { return total < n ? (size_t)0 : (total - n) / hop + 1; };
    if (W) {
        // the streams' runs of complete windows end to end, each starting on a
        // multiple of hop, in the pinned staging buffer the host path copies
        // from. A stream writes its run's samples (carry, then its packet's
        // mono frames) there directly, one host copy of the packet, and only
        // within its own ceil(L / hop) hops, so streams are independent and
        // large pushes stage on several host threads; its new carry (the
        // samples past its last window's start + hop, < n) comes from its
        // old carry and packet.
        size_t Wb = 0;
        for (size_t s = 0; s < S; ++s) {
            const size_t w = windows(have[s] + fresh(s));
            ms->first[s] = Wb;
            if (w) Wb += ((w - 1) * hop + n + hop - 1) / hop;  // ceil(L_s / hop)
        }
        // (Wb, with the straddling windows, was bounded by streams_check)
        const size_t samples = (Wb - 1) * hop + n;  // the last run ends exactly here or earlier
        int rc = ms->mapped ? ensure_mapped(ms, Wb * hop + n, Wb)
                            : ensure_host(st, std::max(Wb * hop + n, kSmallHostSamples),
                                          kSmallHostSamples / 8);
        if (rc != DEMOD_OK) return rc;
        int16_t *const stage_base = ms->mapped ? ms->zm_in : st->h_in;
        try {
            ms->sym.resize(Wb);
            if (mags) ms->mag.resize(Wb * c.k);
        } catch (...) {
            return DEMOD_ALLOC_FAIL;
        }
        auto stage = [&](size_t s) {
            const size_t f = fresh(s), hv = have[s], total = hv + f, w = windows(total);
            if (!w) return;
            const size_t L = (w - 1) * hop + n, span = (L + hop - 1) / hop * hop;
            const size_t end = std::min(total, span);  // hv < n <= L <= end
            int16_t *b = stage_base + ms->first[s] * hop;
            const int16_t *src = pcm[s] + (n_frames[s] - f) * c.channels;
            std::vector<int16_t> &cs = ms->carry[s];
            if (hv) std::memcpy(b, cs.data(), hv * sizeof(int16_t));
            mono_frames(c, src, end - hv, b + hv);
            // the straddling windows read up to the next run's start: keep
            // the gap defined (their results are dropped)
            if (span > L) std::memset(b + L, 0, (span - L) * sizeof(int16_t));
            const size_t t0 = w * hop;  // new carry = samples [t0, total) of the run
            if (t0 >= hv) {
                cs.resize(total - t0);  // < n: within the reserved capacity
                mono_frames(c, src + (t0 - hv) * c.channels, total - t0, cs.data());
            } else {
                std::memmove(cs.data(), cs.data() + t0, (hv - t0) * sizeof(int16_t));
                cs.resize(total - t0);
                mono_frames(c, src, f, cs.data() + (hv - t0));
            }
        };
        // threads: ~1 per 2 MiB of staged samples, at most kPushThreads (1 per
        // MiB measured no better: 0.47 / 0.75 / 0.54-0.61 ms against 0.49-0.53 /
        // 0.67 / 0.55-0.59 for mono / stereo / hop 256 at 1024 streams); the
        // threads persist in the handle's pool between pushes
        size_t T = std::min<size_t>(kPushThreads, Wb * hop / (1u << 20));
        T = std::min(T, S);
        if (T >= 2) {
            const std::function<void(size_t, size_t)> range = [&stage](size_t a, size_t e) {
                for (size_t s = a; s < e; ++s) stage(s);
            };
            ms->pool.run(T, S, range);
        } else {
            for (size_t s = 0; s < S; ++s) stage(s);
        }
        if (ms->mapped) {
            // the detector reads the staged runs in place and writes the
            // results straight into mapped host memory: one launch (and the
            // rescue's), one synchronize
            rc = enqueue_batch(st, ms->zmd_in, Wb, ms->zmd_sym, mags ? ms->zmd_mag : nullptr,
                               st->stream);
            if (rc >= 0 && hipStreamSynchronize(st->stream) != hipSuccess) rc = DEMOD_DEVICE_ERROR;
            if (rc >= 0) {
                std::memcpy(ms->sym.data(), ms->zm_sym, Wb);
                if (mags) std::memcpy(ms->mag.data(), ms->zm_mag, Wb * c.k * sizeof(float));
            }
        } else {
            rc = run_host(st, st->h_in, samples, Wb, ms->sym.data(), mags ? ms->mag.data() : nullptr);
        }
        if (rc < 0) {
            // nothing consumed: the old carries are the runs' first samples
            // (have < n <= L, below the run's gap fill; no other run writes there)
            for (size_t s = 0; s < S; ++s)
                if (windows(have[s] + fresh(s))) {
                    const int16_t *b = stage_base + ms->first[s] * hop;
                    ms->carry[s].assign(b, b + have[s]);
                }
            return rc;
        }
    }
    uint8_t *so = symbols;
    float *mo = mags;
    for (size_t s = 0; s < S; ++s) {
        const size_t f = fresh(s), total = have[s] + f, w = windows(total);
        counts[s] = (uint32_t)w;
        if (w) {
            std::memcpy(so, ms->sym.data() + ms->first[s], w);
            so += w;
            if (mags) {
                std::memcpy(mo, ms->mag.data() + ms->first[s] * c.k, w * c.k * sizeof(float));
                mo += w * c.k;
            }
        } else if (f) {
            ms->carry[s].resize(total);  // < n: within the reserved capacity
            mono_frames(c, pcm[s] + (n_frames[s] - f) * c.channels, f, ms->carry[s].data() + have[s]);
        }
        ms->skip[s] -= std::min(ms->skip[s], n_frames[s]);
    }
    return (int)W;
}

int demod_streams_push_packets(demod_streams_t *ms, demod_decode_fn decode, void *const *decoders,
                               const uint8_t *const *packets, const int32_t *lens, int frame_size,
                               uint8_t *symbols, float *mags, size_t cap, uint32_t *counts)
{
    if (!ms || !decode || !decoders || !lens || !counts) return DEMOD_BAD_ARG;
    if (frame_size < 1 || frame_size > (1 << 20)) return DEMOD_BAD_ARG;
    const size_t S = ms->carry.size(), ch = ms->cfg.channels, per = (size_t)frame_size * ch;
    for (size_t s = 0; s < S; ++s)
        if (lens[s] < 0 || (lens[s] > 0 && (!packets || !packets[s]))) return DEMOD_BAD_ARG;
    try {
        ms->dec.resize(S * per);
        ms->dec_frames.assign(S, 0);
        ms->dec_ptr.assign(S, nullptr);
    } catch (...) {
        return DEMOD_ALLOC_FAIL;
    }
    // every stream's packet decoded by its own decoder (playback.cpp:118,
    // opus_decode into the PCM buffer), on the handle's staging threads: the
    // decoders are independent, so are the streams. A zero-length packet is
    // no packet (playback.cpp:105 skips it): the stream pushes 0 frames.
    std::vector<int> err(S, 0);
    auto dec_one = [&](size_t s) {
        if (lens[s] == 0) return;
        int16_t *out = ms->dec.data() + s * per;
        const int got = decode(decoders[s], packets[s], lens[s], out, frame_size, 0);
        if (got < 0) err[s] = got;
        else if (got > frame_size) err[s] = DEMOD_INTERNAL_ERROR;   // the decoder overran its frame_size
        else {
            ms->dec_frames[s] = (size_t)got;
            ms->dec_ptr[s] = out;
        }
    };
    size_t T = std::min<size_t>(kPushThreads, S);
    if (S < 8) T = 1;
    if (T >= 2) {
        const std::function<void(size_t, size_t)> range = [&dec_one](size_t a, size_t e) {
            for (size_t s = a; s < e; ++s) dec_one(s);
        };
        ms->pool.run(T, S, range);
    } else {
        for (size_t s = 0; s < S; ++s) dec_one(s);
    }
    // the lowest stream's decode error: nothing pushed, no carry consumed
    // (the decoders' own states have advanced, as the reference's on a
    // failed opus_decode)
    for (size_t s = 0; s < S; ++s)
        if (err[s]) return err[s];
    return demod_streams_push(ms, ms->dec_ptr.data(), ms->dec_frames.data(), symbols, mags, cap, counts);
}

int demod_synth_fsk(const demod_cfg_t *cfg, uint64_t seed, uint64_t w0, size_t n_windows,
                    int amplitude, int sigma, int16_t *d_pcm, uint8_t *d_symbols, void *stream)
{
    if (!cfg || cfg->k < 1 || cfg->k > DEMOD_MAX_TONES || cfg->n < 8 || (cfg->n % 8)) return DEMOD_BAD_ARG;
    if (!(cfg->fs > 0.0) || !d_pcm || ((uintptr_t)d_pcm & 15)) return DEMOD_BAD_ARG;
    if (amplitude < 0 || amplitude > 32767 || sigma < 0 || sigma > 32767) return DEMOD_BAD_ARG;
    if (n_windows == 0) return DEMOD_OK;
    if (cfg->device < 0 || cfg->device >= kMaxDevices) return DEMOD_BAD_ARG;
    DeviceGuard guard(cfg->device);
    HIP_TRY(guard.err);
    // the buffers must live on cfg->device (the launch goes there)
    for (const void *q : {(const void *)d_pcm, (const void *)d_symbols}) {
        if (!q) continue;
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            continue;  // not a runtime allocation: left to the caller
        }
        if (a.type == hipMemoryTypeDevice && a.device != cfg->device) return DEMOD_BAD_ARG;
    }
    HIP_TRY(synth_prepare());  // sine table on the current device (once, locked)
    SynthParams p;
    std::memset(&p, 0, sizeof(p));
    p.seed = seed;
    p.w0 = w0;
    p.n_windows = (long long)n_windows;
    p.n = (int)cfg->n;
    p.k = (int)cfg->k;
    p.amplitude = amplitude;
    p.sigma = sigma;
    p.pcm = d_pcm;
    p.sym = d_symbols;
    for (uint32_t t = 0; t < cfg->k; ++t)
        p.inc[t] = (uint32_t)((unsigned long long)std::llround(cfg->freqs[t] / cfg->fs * 4294967296.0) &
                              0xFFFFFFFFULL);
    HIP_TRY(launch_synth(p, (hipStream_t)stream));
    return DEMOD_OK;
}

long long demod_frame_symbols_size(size_t n, int bits, size_t max_payload)
{
    if (bits < 1 || bits > 8) return DEMOD_BAD_ARG;
    if (max_payload < 1 || max_payload > DEMOD_MAX_FRAME_PAYLOAD) return DEMOD_BAD_ARG;
    if (n > (size_t)1 << 40) return DEMOD_BAD_ARG;
    return frame_streams_size((long long)n, bits, (long long)max_payload, nullptr, nullptr, nullptr);
}

long long demod_frame_streams_async(const uint8_t *d_symbols, size_t n_streams, size_t n,
                                    int bits, size_t max_payload, uint8_t *d_out, void *stream)
{
    const long long stride = demod_frame_symbols_size(n, bits, max_payload);
    if (stride < 0) return stride;
    if (n_streams && n && (!d_symbols || !d_out)) return DEMOD_BAD_ARG;
    if (n_streams > (size_t)1 << 31) return DEMOD_BAD_ARG;
    if (n_streams == 0 || n == 0) return stride;
    HIP_TRY(launch_frame_streams(d_symbols, (long long)n_streams, (long long)n, bits,
                                 (long long)max_payload, d_out, (hipStream_t)stream));
    return stride;
}

const char *demod_strerror(int error)
{
    switch (error) {
    case DEMOD_OK: return "success";
    case DEMOD_BAD_ARG: return "invalid argument";
    case DEMOD_BUFFER_TOO_SMALL: return "buffer too small";
    case DEMOD_INTERNAL_ERROR: return "internal error";
    case DEMOD_INVALID_PACKET: return "corrupted frame";
    case DEMOD_UNIMPLEMENTED: return "request not implemented";
    case DEMOD_INVALID_STATE: return "invalid state";
    case DEMOD_ALLOC_FAIL: return "memory allocation failed";
    case DEMOD_DEVICE_ERROR: return "HIP device error";
    case DEMOD_NO_DEVICE: return "no gfx950 (MI355X) device available";
    case DEMOD_FRAME_TOO_LARGE: return "encoded frame exceeds max size";
    default: return "unknown error";
    }
}

int demod_read_ceiling_async(const void *d_buf, size_t n_bytes, void *stream)
{
    if (!d_buf || ((uintptr_t)d_buf & 15) || (n_bytes % 8192)) return DEMOD_BAD_ARG;
    if (n_bytes == 0) return DEMOD_OK;
    HIP_TRY(launch_read_ceiling((const int16_t *)d_buf, (long long)n_bytes, (hipStream_t)stream));
    return DEMOD_OK;
}

const char *demod_version_string(void) { return "fskdemod 0.1.0 (gfx950 HIP)"; }

}  // extern "C"
