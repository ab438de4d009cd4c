// mag_probe.hip — what the 8-FSK magnitude stream (configs[2]: 32 MiB of
// |X_k|^2 beside 2 GiB of input) costs the fold-by-16 detector, by store
// policy and launch slicing.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude scripts/mag_probe.hip -o scripts/bin/mag_probe
//   scripts/bin/mag_probe [rounds=6] [reps=5] [loads|wb]
//
// Same kernel, grid and input as the shipped configs[2] path
// (fold_tile_kernel F16, 2-wave blocks, one tile per wave, XCD-swizzled);
// variants differ only in the magnitude store (window_sum.h mag_store: plain,
// non-temporal, buffer store with cache-policy bits) and in how many launches
// the 2^20 windows are split into (demod_api.cpp launch_slice ships 4 with
// plain stores).
// Round-robin over variants, HIP events around the whole batch, median per
// variant; every variant's symbols and magnitudes are checked against the
// shipped variant's (plain stores, one launch).
#include "../audio-network_amd/csrc/fold.hip"
#include "../audio-network_amd/csrc/synth.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

template <int MST, int LAUX = -1>
static const void *f16k()
{
    return reinterpret_cast<const void *>(
        &fold_tile_kernel<8, 4, true, kPlainWPB, false, false, true, false, true, true, MST, LAUX>);
}

struct Var {
    std::string name;
    const void *kern;
    int slices;
    bool mags;
    std::vector<float> ms;
    int bursts = 0;  // GoertzelParams::wb_bursts (round 3, late)
};

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 6;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const long long W = 1LL << 20;
    int16_t *pcm;
    uint8_t *truth;
    CK(hipMalloc(&pcm, W * 2048));
    CK(hipMalloc(&truth, W));
    {
        SynthParams sp{};
        sp.seed = 0x2C5DA044;
        sp.n_windows = W;
        sp.n = 1024;
        sp.k = 8;
        sp.amplitude = 8000;
        sp.sigma = 400;
        sp.pcm = pcm;
        sp.sym = truth;
        for (int i = 0; i < 8; ++i) sp.inc[i] = (unsigned)(32 + 8 * i) << 22;
        CK(launch_synth(sp, nullptr));
        CK(hipDeviceSynchronize());
    }
    // F16 plan as demod_api.cpp builds it for bins 32 + 8 i: slots 0-3 the
    // Z0 tones (32, 48, 64, 80), slots 4-7 the Z8 tones (40, 56, 72, 88)
    GoertzelParams p{};
    p.pcm = pcm;
    p.n_windows = W;
    p.hop = 1024;
    p.log2g = 4;
    p.k = 8;
    p.f16 = 1;
    p.perm = 0x75316420ull;
    p.xcd_swizzle = 1;
    {
        static const double b16[8] = {32, 48, 64, 80, 40, 56, 72, 88};
        std::vector<float4> rot(8 * 16);
        for (int k = 0; k < 8; ++k) {
            const double w = 2 * M_PI * b16[k] / 1024.0;
            p.coef[k] = (float)(2 * std::cos(w));
            for (int j = 0; j < 16; ++j) {
                const double a = -w * (8.0 * (j & 7) + 7), b = -w * (8.0 * (j & 7) + 8);
                rot[k * 16 + j] = make_float4(std::cos(a), std::sin(a), std::cos(b), std::sin(b));
            }
        }
        float4 *d;
        CK(hipMalloc(&d, rot.size() * sizeof(float4)));
        CK(hipMemcpy(d, rot.data(), rot.size() * sizeof(float4), hipMemcpyHostToDevice));
        p.rot = d;
    }
    uint8_t *sym, *sym_ref;
    float *mag, *mag_ref;
    CK(hipMalloc(&sym, W));
    CK(hipMalloc(&sym_ref, W));
    CK(hipMalloc(&mag, W * 8 * 4));
    CK(hipMalloc(&mag_ref, W * 8 * 4));

    std::vector<Var> vs;
    const bool loads = argc > 3 && std::strcmp(argv[3], "loads") == 0;
    const bool wb = argc > 3 && std::strcmp(argv[3], "wb") == 0;
    if (wb) {
        // round 3, late: L2 write-back bursts inside one launch (GoertzelParams::wb_bursts)
        // against the shipped 4 slices and no magnitudes
        for (int sl : {1, 4}) {
            vs.push_back({"no mags", f16k<-1>(), sl, false, {}});
            vs.push_back({"plain (shipped)", f16k<-1>(), sl, true, {}});
        }
        vs.push_back({"plain wbl2 x7", f16k<-1>(), 1, true, {}, 7});
        vs.push_back({"plain wbl2 x4", f16k<-1>(), 1, true, {}, 4});
        vs.push_back({"plain wbl2 x8", f16k<-1>(), 1, true, {}, 8});
        vs.push_back({"plain wbl2 x16", f16k<-1>(), 1, true, {}, 16});
        vs.push_back({"plain wbl2 x64", f16k<-1>(), 1, true, {}, 64});
        vs.push_back({"plain wbl2 x256", f16k<-1>(), 1, true, {}, 256});
        vs.push_back({"plain wbl2 x8", f16k<-1>(), 2, true, {}, 8});
        vs.push_back({"nontemporal wbl2 x8", f16k<1>(), 1, true, {}, 8});
    }
    for (int sl : {1, 2, 4}) {
        if (wb) break;
        vs.push_back({"no mags", f16k<-1>(), sl, false, {}});
        vs.push_back({"plain (shipped)", f16k<-1>(), sl, true, {}});
        if (loads) {
            // input load policy with plain magnitude stores (round 3, late)
            vs.push_back({"loads sc0 nt", f16k<-1, 3>(), sl, true, {}});
            vs.push_back({"loads sc1 nt", f16k<-1, 18>(), sl, true, {}});
            vs.push_back({"loads sc0 sc1", f16k<-1, 17>(), sl, true, {}});
            vs.push_back({"loads sc0 sc1 nt", f16k<-1, 19>(), sl, true, {}});
            vs.push_back({"loads plain", f16k<-1, 0>(), sl, true, {}});
            continue;
        }
        vs.push_back({"nontemporal", f16k<1>(), sl, true, {}});
        vs.push_back({"buffer nt", f16k<2 + 2>(), sl, true, {}});
        vs.push_back({"buffer sc1", f16k<2 + 16>(), sl, true, {}});
        vs.push_back({"buffer sc0 sc1", f16k<2 + 17>(), sl, true, {}});
        vs.push_back({"buffer sc0 sc1 nt", f16k<2 + 19>(), sl, true, {}});
    }
    auto run = [&](const Var &v, uint8_t *s_out, float *m_out) {
        const long long per = ((W + v.slices - 1) / v.slices + 63) / 64 * 64;
        for (long long w0 = 0; w0 < W; w0 += per) {
            GoertzelParams q = p;
            const long long cnt = std::min(per, W - w0);
            q.pcm = pcm + w0 * 1024;
            q.n_windows = cnt;
            q.sym = s_out + w0;
            q.mag = v.mags ? m_out + w0 * 8 : nullptr;
            q.wb_bursts = v.bursts;
            const long long tiles = (cnt + 3) / 4;
            const unsigned blocks = (unsigned)((tiles + kPlainWPB - 1) / kPlainWPB);
            void *args[] = {&q};
            CK(hipLaunchKernel(v.kern, dim3(blocks), dim3(64 * kPlainWPB), args, 0, nullptr));
        }
    };
    // reference outputs: plain stores, one launch
    run(vs[1], sym_ref, mag_ref);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> hs_ref(W), hs(W);
    std::vector<float> hm_ref(W * 8), hm(W * 8);
    CK(hipMemcpy(hs_ref.data(), sym_ref, W, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hm_ref.data(), mag_ref, W * 32, hipMemcpyDeviceToHost));

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r)
        for (auto &v : vs) {
            for (int k = 0; k < 2; ++k) run(v, sym, mag);
            for (int k = 0; k < reps; ++k) {
                CK(hipEventRecord(e0, nullptr));
                run(v, sym, mag);
                CK(hipEventRecord(e1, nullptr));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.ms.push_back(ms);
            }
            if (r == 0) {
                CK(hipMemcpy(hs.data(), sym, W, hipMemcpyDeviceToHost));
                bool ok = hs == hs_ref;
                if (v.mags) {
                    CK(hipMemcpy(hm.data(), mag, W * 32, hipMemcpyDeviceToHost));
                    ok = ok && std::memcmp(hm.data(), hm_ref.data(), W * 32) == 0;
                    CK(hipMemset(mag, 0, W * 32));
                }
                if (!ok) std::printf("MISMATCH: %s slices %d\n", v.name.c_str(), v.slices);
            }
        }
    CK(hipGetLastError());
    const double alg = (double)W * (2048 + 1 + 32);
    for (auto &v : vs) {
        std::vector<float> m = v.ms;
        std::sort(m.begin(), m.end());
        const double med = m[m.size() / 2];
        std::printf("%-20s slices %d  min %.1f us  median %.1f us  %.3f of 8 TB/s (alg. bytes with mags)\n",
                    v.name.c_str(), v.slices, m[0] * 1e3, med * 1e3, alg / (med * 1e-3) / 8e12);
    }
    return 0;
}
