// fft_probe.hip — interleaved A/B of FFT-detector kernel variants (config 4).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude scripts/fft_probe.hip -o scripts/bin/fft_probe
//   scripts/bin/fft_probe [hop=256] [rounds=6] [reps=10] [filter]
//
// One process, round-robin over variants on the same seeded 2^30-sample
// stream (cdna_hip_programming.md §5.4 rule 24): min / median kernel time from
// HIP events. Every variant's symbols and tone powers are compared with the
// shipped kernel's on all windows, and the full 513-bin spectra on a 4096-window
// sample (max |dP| relative to the window's peak bin, the 1e-5 bar).
#include "../audio-network_amd/csrc/fft_quad.hip"
#include "../audio-network_amd/csrc/synth.hip"
#include "fft_quad_r1b.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

using namespace fskd;

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,      \
                         hipGetErrorString(e_));                                \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

// the shipped kernel with decision-rescue strategy R (fft_quad.hip step 6)
template <int R>
hipError_t launch_rsc(const FftParams &p, hipStream_t s)
{
    const bool lin = p.spec && ((uintptr_t)p.spec & 15) == 0;
    if (p.hop < 1024)
        return lin ? launch_fft_quad_t<4, 4, 0, true, false, 0, 4, 0, 2, 0, 0, R>(p, s)
             : p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 0, 4, 0, 0, 0, 0, R>(p, s)
                      : launch_fft_quad_t<4, 4, 0, false, false, 0, 4, 0, 0, 0, 0, R>(p, s);
    return lin ? launch_fft_quad_t<4, 4, 0, true, false, 2, 4, 0, 2, 0, 0, R>(p, s)
         : p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 2, 4, 0, 0, 0, 0, R>(p, s)
                  : launch_fft_quad_t<4, 4, 0, false, false, 2, 4, 0, 0, 0, 0, R>(p, s);
}

struct Var {
    std::string name;
    std::function<hipError_t(const FftParams &, hipStream_t)> launch;
    std::vector<float> ms;
};

int main(int argc, char **argv)
{
    const int hop = argc > 1 ? std::atoi(argv[1]) : 256;
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 6;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 10;
    const char *filter = argc > 4 ? argv[4] : nullptr;
    // "spec": time with the full 513-bin spectrum stored (one shared buffer)
    const bool time_spec = argc > 5 && std::strcmp(argv[5], "spec") == 0;
    const long long src_windows = 1LL << 20;
    const long long n_samples = src_windows * 1024;
    const long long W = (n_samples - 1024) / hop + 1;
    const int K = 2;
    const double freqs[2] = {1500.0, 3000.0};

    int16_t *pcm;
    CK(hipMalloc(&pcm, n_samples * 2));
    CK(synth_prepare());
    SynthParams sp;
    std::memset(&sp, 0, sizeof sp);
    sp.seed = 0x2C5DA044;
    sp.n_windows = src_windows;
    sp.n = 1024;
    sp.k = K;
    sp.amplitude = 8000;
    sp.sigma = 400;
    sp.pcm = pcm;
    for (int t = 0; t < K; ++t)
        sp.inc[t] = (uint32_t)((unsigned long long)std::llround(freqs[t] / 48000.0 * 4294967296.0));
    CK(launch_synth(sp, nullptr));

    std::vector<float> t1(1024), t2(1024);
    for (int m = 0; m < 512; ++m) {
        t1[2 * m] = (float)std::cos(-2.0 * M_PI * m / 512.0);
        t1[2 * m + 1] = (float)std::sin(-2.0 * M_PI * m / 512.0);
        t2[2 * m] = (float)std::cos(-2.0 * M_PI * m / 1024.0);
        t2[2 * m + 1] = (float)std::sin(-2.0 * M_PI * m / 1024.0);
    }
    int bins[2] = {32, 64};
    float *d_t1, *d_t2;
    int *d_bins;
    CK(hipMalloc(&d_t1, 4096));
    CK(hipMalloc(&d_t2, 4096));
    CK(hipMalloc(&d_bins, 8));
    CK(hipMemcpy(d_t1, t1.data(), 4096, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_t2, t2.data(), 4096, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_bins, bins, 8, hipMemcpyHostToDevice));

    // the decision rescue's double radix-2 twiddles and thresholds, as
    // demod_api.cpp sets them for the FFT detector
    std::vector<double> rtw(2 * 1023);
    for (int len = 2; len <= 1024; len <<= 1) {
        const double ang = -(2.0 * M_PI) / (double)len;
        for (int j = 0; j < len / 2; ++j) {
            double sn, cs;
            sincos(ang * (double)j, &sn, &cs);
            rtw[2 * (len / 2 - 1 + j)] = cs;
            rtw[2 * (len / 2 - 1 + j) + 1] = sn;
        }
    }
    double *d_rtw;
    CK(hipMalloc(&d_rtw, rtw.size() * 8));
    CK(hipMemcpy(d_rtw, rtw.data(), rtw.size() * 8, hipMemcpyHostToDevice));
    const float amb_tq = (float)(12.0 * 2.64e-7 * 1024.0 * 32768.0);
    const float amb_floor = amb_tq * amb_tq / 16.0f;

    std::vector<Var> vs;
    // variant 0 is the reference every other variant is checked against
    vs.push_back({"quad r1 (round-1 shipped)", [](const FftParams &p, hipStream_t s) { return r1b::launch_fft_quad_r1_t<4, 0>(p, s); }, {}});
    vs.push_back({"separate DFT-4 / post-pass blocks", [](const FftParams &p, hipStream_t s) { return p.hop < 1024 ? (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 0, 0>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 0, 0>(p, s)) : (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 2, 0>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 2, 0>(p, s)); }, {}});
    vs.push_back({"quad shipped (fused, PF0 MINW4)", [](const FftParams &p, hipStream_t s) { return launch_fft_quad(p, s); }, {}});
    vs.push_back({"fused level 3", [](const FftParams &p, hipStream_t s) { return p.hop < 1024 ? (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 0, 3>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 0, 3>(p, s)) : (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 2, 3>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 2, 3>(p, s)); }, {}});
    vs.push_back({"fused level 2 (DFT-4 + post-pass)", [](const FftParams &p, hipStream_t s) { return p.hop < 1024 ? (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 0, 2>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 0, 2>(p, s)) : (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 2, 2>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 2, 2>(p, s)); }, {}});
    vs.push_back({"fused DFT-4 blocks", [](const FftParams &p, hipStream_t s) { return p.hop < 1024 ? (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 0, 1>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 0, 1>(p, s)) : (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 2, 1>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 2, 1>(p, s)); }, {}});
    vs.push_back({"aux1 (sc0)", [](const FftParams &p, hipStream_t s) { return p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 1>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 1>(p, s); }, {}});
    vs.push_back({"aux2 (nt, round-2 first ship)", [](const FftParams &p, hipStream_t s) { return p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 2>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 2>(p, s); }, {}});
    vs.push_back({"ds_read_b64 (no read2 pairing)", [](const FftParams &p, hipStream_t s) { return p.hop < 1024 ? (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 0, 4, 1>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 0, 4, 1>(p, s)) : (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 2, 4, 1>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 2, 4, 1>(p, s)); }, {}});
    vs.push_back({"ds_read_b64 + b128 tables", [](const FftParams &p, hipStream_t s) { return p.hop < 1024 ? (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 0, 4, 2>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 0, 4, 2>(p, s)) : (p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 2, 4, 2>(p, s) : launch_fft_quad_t<4, 4, 0, false, false, 2, 4, 2>(p, s)); }, {}});
    vs.push_back({"fused PF1 MINW0", [](const FftParams &p, hipStream_t s) { return p.spec ? launch_fft_quad_t<4, 0, 1, true>(p, s) : launch_fft_quad_t<4, 0, 1, false>(p, s); }, {}});
    // round 2, late: the next group's loads during the transpose (PF 1) with
    // the shipped fused kernel, at 3 and 4 waves per SIMD, and 3 waves alone
    vs.push_back({"pfx: fused4 PF1 MINW3", [](const FftParams &p, hipStream_t s) { return p.spec ? launch_fft_quad_t<4, 3, 1, true, false, 0, 4>(p, s) : launch_fft_quad_t<4, 3, 1, false, false, 0, 4>(p, s); }, {}});
    vs.push_back({"pfx: fused4 PF1 MINW4", [](const FftParams &p, hipStream_t s) { return p.spec ? launch_fft_quad_t<4, 4, 1, true, false, 0, 4>(p, s) : launch_fft_quad_t<4, 4, 1, false, false, 0, 4>(p, s); }, {}});
    vs.push_back({"pfx: fused4 PF0 MINW3", [](const FftParams &p, hipStream_t s) { return p.spec ? launch_fft_quad_t<4, 3, 0, true, false, 0, 4>(p, s) : launch_fft_quad_t<4, 3, 0, false, false, 0, 4>(p, s); }, {}});
    vs.push_back({"pfx: shipped", [](const FftParams &p, hipStream_t s) { return launch_fft_quad(p, s); }, {}});
    // round 3: round 1 of the transpose overlapped with column 0's DFT-16 (OVL)
    vs.push_back({"ovl: shipped", [](const FftParams &p, hipStream_t s) { return launch_fft_quad(p, s); }, {}});
    vs.push_back({"ovl: OVL1", [](const FftParams &p, hipStream_t s) {
        const bool lin = p.spec && ((uintptr_t)p.spec & 15) == 0;
        if (p.hop < 1024)
            return lin ? launch_fft_quad_t<4, 4, 0, true, false, 0, 4, 0, 2, 1>(p, s)
                 : p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 0, 4, 0, 0, 1>(p, s)
                          : launch_fft_quad_t<4, 4, 0, false, false, 0, 4, 0, 0, 1>(p, s);
        return lin ? launch_fft_quad_t<4, 4, 0, true, false, 2, 4, 0, 2, 1>(p, s)
             : p.spec ? launch_fft_quad_t<4, 4, 0, true, false, 2, 4, 0, 0, 1>(p, s)
                      : launch_fft_quad_t<4, 4, 0, false, false, 2, 4, 0, 0, 1>(p, s); }, {}});
    // spectrum: the next group's loads ahead of the spectrum stores (PF 2)
    vs.push_back({"spl: shipped", [](const FftParams &p, hipStream_t s) { return launch_fft_quad(p, s); }, {}});
    vs.push_back({"spl: PF2", [](const FftParams &p, hipStream_t s) {
        const bool lin = p.spec && ((uintptr_t)p.spec & 15) == 0;
        if (!lin) return launch_fft_quad(p, s);
        return p.hop < 1024 ? launch_fft_quad_t<4, 4, 2, true, false, 0, 4, 0, 2>(p, s)
                            : launch_fft_quad_t<4, 4, 2, true, false, 2, 4, 0, 2>(p, s); }, {}});
    // post-pass twiddles from registers (TW3R), tone-only and spectrum
    vs.push_back({"tw3: shipped", [](const FftParams &p, hipStream_t s) { return launch_fft_quad(p, s); }, {}});
    vs.push_back({"tw3: TW3R", [](const FftParams &p, hipStream_t s) {
        const bool lin = p.spec && ((uintptr_t)p.spec & 15) == 0;
        if (p.spec && !lin) return launch_fft_quad(p, s);
        if (p.hop < 1024)
            return lin ? launch_fft_quad_t<4, 4, 0, true, false, 0, 4, 0, 2, 0, 1>(p, s)
                       : launch_fft_quad_t<4, 4, 0, false, false, 0, 4, 0, 0, 0, 1>(p, s);
        return lin ? launch_fft_quad_t<4, 4, 0, true, false, 2, 4, 0, 2, 0, 1>(p, s)
                   : launch_fft_quad_t<4, 4, 0, false, false, 2, 4, 0, 0, 0, 1>(p, s); }, {}});
    vs.push_back({"tw3: TW3R OVL1", [](const FftParams &p, hipStream_t s) {
        if (p.spec) return launch_fft_quad(p, s);
        return p.hop < 1024 ? launch_fft_quad_t<4, 4, 0, false, false, 0, 4, 0, 0, 1, 1>(p, s)
                            : launch_fft_quad_t<4, 4, 0, false, false, 2, 4, 0, 0, 1, 1>(p, s); }, {}});
    vs.push_back({"ovl: OVL1 FMT", [](const FftParams &p, hipStream_t s) {
        if (p.spec) return launch_fft_quad(p, s);  // tone-only variant
        return p.hop < 1024 ? launch_fft_quad_t<4, 4, 0, false, true, 0, 4, 0, 0, 1>(p, s)
                            : launch_fft_quad_t<4, 4, 0, false, true, 2, 4, 0, 0, 1>(p, s); }, {}});
    // round 3: the decision rescue inside the detector (step 6): compiled out,
    // compiled in and off, flags only, per-wave and per-block rescue
    vs.push_back({"rsc0 no rescue code", [](const FftParams &p, hipStream_t s) { return launch_rsc<0>(p, s); }, {}});
    vs.push_back({"rsc1 compiled, off", [](const FftParams &p, hipStream_t s) { return launch_rsc<1>(p, s); }, {}});
    vs.push_back({"rsc1 flags only", [=](const FftParams &p, hipStream_t s) {
        FftParams q = p; q.amb_tq = amb_tq; q.amb_floor = amb_floor; return launch_rsc<1>(q, s); }, {}});
    vs.push_back({"rsc1 per-wave rescue", [=](const FftParams &p, hipStream_t s) {
        FftParams q = p; q.amb_tq = amb_tq; q.amb_floor = amb_floor; q.rescue = 1; q.rtw = d_rtw;
        return launch_rsc<1>(q, s); }, {}});
    vs.push_back({"rsc2 per-block rescue", [=](const FftParams &p, hipStream_t s) {
        FftParams q = p; q.amb_tq = amb_tq; q.amb_floor = amb_floor; q.rescue = 1; q.rtw = d_rtw;
        return launch_rsc<2>(q, s); }, {}});
    // round 3, late: the tone pick gathered by ds_bpermute (PICK 1) instead of
    // the per-tone register pick with per-lane best tracking
    vs.push_back({"pick: shipped", [](const FftParams &p, hipStream_t s) { return launch_fft_quad(p, s); }, {}});
    vs.push_back({"pick: PICK1", [](const FftParams &p, hipStream_t s) {
        if (p.spec) return launch_fft_quad(p, s);
        return p.hop < 1024 ? launch_fft_quad_t<4, 4, 0, false, false, 0, 4, 0, 0, 0, 0, 1, 1>(p, s)
                            : launch_fft_quad_t<4, 4, 0, false, false, 2, 4, 0, 0, 0, 0, 1, 1>(p, s); }, {}});
    // (round 3, late: lane 0's post-pass pairing through 32 exec-masked LDS
    // instructions instead of 32 v_cndmask, "l0: L0": -32 VALU per group but
    // +2.2 % at hop 256, +1.1 % at hop 1024, profiles/round3/r3t/; removed)
    // (round 3, late: the input as one wide read of the group's span staged
    // through the slab with a bank skew, "wl: WL": identical outputs but +4 %
    // at hop 256 with the spectrum, +4 % tones only, +2.7 % at hop 512 with
    // the spectrum, profiles/round3/r3w/; removed)
    if (filter) {
        std::vector<Var> keep;
        for (size_t i = 0; i < vs.size(); ++i)
            if (i == 0 || vs[i].name.find(filter) != std::string::npos) keep.push_back(vs[i]);
        vs.swap(keep);
    }

    FftParams base;
    std::memset(&base, 0, sizeof base);
    base.pcm = pcm;
    base.n_windows = W;
    base.hop = hop;
    base.k = K;
    base.xcd_swizzle = hop < 1024 ? 1 : 0;
    base.tw512 = d_t1;
    base.tw1024 = d_t2;
    base.bins = d_bins;
    for (int k = 0; k < K; ++k) base.slot[k] = fft_quad_slot(bins[k]);
    std::vector<uint8_t *> syms(vs.size());
    std::vector<float *> mags(vs.size()), specs(vs.size());
    const long long SW = 4096;
    for (size_t i = 0; i < vs.size(); ++i) {
        CK(hipMalloc(&syms[i], W));
        CK(hipMalloc(&mags[i], W * K * 4));
        CK(hipMalloc(&specs[i], SW * 513 * 4));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // correctness pass: all windows, symbols + tone powers; spectra on SW windows
    for (size_t i = 0; i < vs.size(); ++i) {
        FftParams p = base;
        p.sym = syms[i];
        p.mag = mags[i];
        CK(vs[i].launch(p, nullptr));
        FftParams ps = base;
        ps.n_windows = SW;
        ps.sym = syms[i];
        ps.spec = specs[i];
        CK(vs[i].launch(ps, nullptr));
        CK(vs[i].launch(p, nullptr));   // leave all-window symbols in syms
    }
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> s0(W), si(W);
    std::vector<float> m0(W * K), mi(W * K), sp0(SW * 513), spi(SW * 513);
    CK(hipMemcpy(s0.data(), syms[0], W, hipMemcpyDeviceToHost));
    CK(hipMemcpy(m0.data(), mags[0], W * K * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(sp0.data(), specs[0], SW * 513 * 4, hipMemcpyDeviceToHost));
    for (size_t i = 1; i < vs.size(); ++i) {
        CK(hipMemcpy(si.data(), syms[i], W, hipMemcpyDeviceToHost));
        CK(hipMemcpy(mi.data(), mags[i], W * K * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(spi.data(), specs[i], SW * 513 * 4, hipMemcpyDeviceToHost));
        long long mism = 0;
        double merr = 0, serr = 0;
        for (long long w = 0; w < W; ++w) {
            mism += s0[w] != si[w];
            double pk = std::max(m0[w * K], m0[w * K + 1]);
            for (int k = 0; k < K; ++k)
                merr = std::max(merr, std::fabs((double)mi[w * K + k] - m0[w * K + k]) / std::max(pk, 1e-30));
        }
        for (long long w = 0; w < SW; ++w) {
            double pk = 0;
            for (int b = 0; b < 513; ++b) pk = std::max(pk, (double)sp0[w * 513 + b]);
            for (int b = 0; b < 513; ++b)
                serr = std::max(serr, std::fabs((double)spi[w * 513 + b] - sp0[w * 513 + b]) / std::max(pk, 1e-30));
        }
        std::printf("check %-24s vs shipped: %lld symbol mismatches / %lld, max tone |dP|/peak %.2e, "
                    "spectrum (%lld windows) %.2e\n", vs[i].name.c_str(), mism, W, merr, SW, serr);
    }
    // timing: round-robin, symbols + tone powers (the bench's batch_async
    // shape), or with the full spectrum stored
    float *big_spec = nullptr;
    if (time_spec) CK(hipMalloc(&big_spec, (size_t)W * 513 * 4));
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            FftParams p = base;
            p.sym = syms[i];
            p.mag = mags[i];
            p.spec = big_spec;
            for (int w = 0; w < 3; ++w) CK(vs[i].launch(p, nullptr));
            for (int k = 0; k < reps; ++k) {
                CK(hipEventRecord(e0, nullptr));
                CK(vs[i].launch(p, nullptr));
                CK(hipEventRecord(e1, nullptr));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                vs[i].ms.push_back(ms);
            }
        }
    }
    const double fpw = 2.5 * 1024 * 10 + 3 * 513;
    for (auto &v : vs) {
        if (v.ms.empty()) continue;
        std::vector<float> m = v.ms;
        std::sort(m.begin(), m.end());
        const double med = m[m.size() / 2];
        std::printf("%-24s hop %d W %lld: min %.4f ms median %.4f ms  %.1f TF/s (%.1f %% of 157.3)\n",
                    v.name.c_str(), hop, W, m[0], med, fpw * W / (med * 1e-3) / 1e12,
                    100.0 * fpw * W / (med * 1e-3) / 1e12 / 157.3);
    }
    return 0;
}
