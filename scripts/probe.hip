// probe.hip — interleaved A/B timing of Goertzel kernel variants and of a
// pure read-only HBM stream (the practical bandwidth ceiling of this box).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe.hip -o scripts/bin/probe
//   scripts/bin/probe [windows=1048576] [rounds=5] [reps=10]
//
// All variants run in one process, round-robin, on the same seeded input
// (cdna_hip_programming.md §5.4 rule 24); each reports min / median kernel
// time from HIP events and the algorithmic GB/s. Outputs are cross-checked
// against the default variant.
#include "../audio-network_amd/csrc/goertzel.hip"
#include "../audio-network_amd/csrc/synth.hip"
#include "../audio-network_amd/csrc/fold.hip"
#include "../audio-network_amd/csrc/residue.hip"
#include "fft_r0.hip"
#include "../audio-network_amd/csrc/fft_quad.hip"
#include "fft_quad_r1.hip"

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

template <bool NT, int U>
__global__ __launch_bounds__(256) void read_kernel(const u32x4 *__restrict__ p, long long n16,
                                                   unsigned *out)
{
    long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long stride = (long long)gridDim.x * 256;
    unsigned acc = 0;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = NT ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    for (; i < n16; i += stride) acc ^= p[i].x;
    if (acc == 0x9E3779B9u) out[0] = acc;
}

// The same one-shot access pattern as the tile kernels (each wave reads one
// contiguous 8 KiB tile with 8 coalesced 16 B/lane nt buffer loads) and no
// compute: the practical HBM read ceiling for this shape. L = loads per wave
// (8 KiB at L = 8), WPB = waves per block, AUX = buffer cache-policy bits.
template <int L, int WPB, int AUX>
__global__ __launch_bounds__(64 * WPB) void read_tile_kernel(const int16_t *p, long long n_tiles,
                                                             unsigned *out)
{
    const int lane = threadIdx.x & 63;
    const long long t = (long long)blockIdx.x * WPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (t >= n_tiles) return;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(p + t * 512 * L), (short)0, 1024 * L, 0x00020000);
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < L; ++i) {
        u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (64 * i + lane) * 16, 0, AUX);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) out[0] = acc;
}

struct Variant {
    std::string name;
    std::function<void(hipStream_t)> run;
    double bytes;
    std::vector<float> ms;
    uint8_t *sym = nullptr;
};

static void add_variant(std::vector<Variant> &vs, const void *f, int wpb, const char *label,
                        GoertzelParams p, int K, int cus, int tpw, size_t lds = 0,
                        const char *ksuffix = "")
{
    // tpw = 0: persistent grid (co-resident blocks); tpw >= 1: tiles per wave
    int per_cu = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, 64 * wpb, lds));
    const long long n_tiles = (p.n_windows + 3) / 4;
    long long blocks = tpw ? (n_tiles + (long long)wpb * tpw - 1) / ((long long)wpb * tpw)
                           : std::min<long long>((n_tiles + wpb - 1) / wpb, (long long)cus * per_cu);
    uint8_t *sym;
    CK(hipMalloc(&sym, p.n_windows));
    p.sym = sym;
    char name[200];
    std::snprintf(name, sizeof name, "%s K=%d%s WPB=%d %s%d grid=%lld (%d/CU)", label, K, ksuffix,
                  wpb, tpw ? "tpw=" : "persist", tpw, blocks, per_cu);
    Variant v;
    v.name = name;
    v.bytes = (double)p.n_windows * (2048 + 1 + (p.mag ? 4 * K : 0));
    v.sym = sym;
    v.run = [f, p, blocks, wpb, lds](hipStream_t s) {
        void *args[] = {const_cast<GoertzelParams *>(&p)};
        CK(hipLaunchKernel(f, dim3((unsigned)blocks), dim3(64 * wpb), args, lds, s));
    };
    vs.push_back(v);
}

#define GZ(K, PF, NT, WPB, DIRECT) \
    reinterpret_cast<const void *>(&goertzel_tile_kernel<K, 4, PF, NT, WPB, DIRECT>)
#define FD(K, WPB) reinterpret_cast<const void *>(&fold_tile_kernel<K, 4, true, WPB>)
#define FDL(K, WPB) reinterpret_cast<const void *>(&fold_tile_kernel<K, 4, true, WPB, true>)
#define FDS(K, WPB) reinterpret_cast<const void *>(&fold_tile_kernel<K, 4, true, WPB, false, true>)
#define GZS(K) reinterpret_cast<const void *>(&goertzel_tile_kernel<K, 4, 1, true, 4, false, true>)
#define GZP(K) reinterpret_cast<const void *>(&goertzel_tile_kernel<K, 4, 1, true, 4, false, false, true>)
#define GZPB(K) reinterpret_cast<const void *>(&goertzel_tile_kernel<K, 4, 1, true, 4, false, false, true, true>)
#define GZP2(K) reinterpret_cast<const void *>(&goertzel_tile_kernel<K, 4, 2, true, 4, false, false, true>)
#define GZB(K) reinterpret_cast<const void *>(&goertzel_tile_kernel<K, 4, 1, true, 4, false, false, false, true>)
#define GZW(K) reinterpret_cast<const void *>(&goertzel_tile_kernel<K, 4, 1, true, 4, false, false, (K >= 3), false, true>)
#define FDW(K) reinterpret_cast<const void *>(&fold_tile_kernel<K, 4, true, 4, false, false, true>)

int main(int argc, char **argv)
{
    const long long W = argc > 1 ? std::atoll(argv[1]) : (1LL << 20);
    const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
    const int reps = argc > 3 ? std::atoi(argv[3]) : 10;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    std::printf("device %s (%s), %d CUs, %lld windows (%.2f GiB)\n", prop.name, prop.gcnArchName,
                cus, W, W * 2048.0 / (1 << 30));

    // input: seeded FSK, identical to the product generator
    int16_t *pcm, *lut;
    CK(hipMalloc(&pcm, W * 2048));
    std::vector<int16_t> hl(16384);
    for (int i = 0; i < 16384; ++i) hl[i] = (int16_t)std::lrint(32767.0 * std::sin(2 * M_PI * i / 16384.0));
    CK(hipMalloc(&lut, 16384 * 2));
    CK(hipMemcpy(lut, hl.data(), 16384 * 2, hipMemcpyHostToDevice));
    float *mag;
    CK(hipMalloc(&mag, W * 8 * sizeof(float)));
    unsigned *sink;
    CK(hipMalloc(&sink, 64));

    std::vector<Variant> vs;
    // one input for all (2-FSK tones; the 8-FSK kernels read the same bytes)
    {
        SynthParams sp{};
        sp.seed = 0x2C5DA044;
        sp.n_windows = W;
        sp.n = 1024;
        sp.k = 2;
        sp.amplitude = 8000;
        sp.sigma = 400;
        sp.lut = lut;
        sp.pcm = pcm;
        sp.inc[0] = 32u << 22;
        sp.inc[1] = 64u << 22;
        CK(launch_synth(sp, nullptr));
        CK(hipDeviceSynchronize());
    }

    // rotation tables for K = 2 and 8 (freqs on bins 32.. as the bench)
    auto make_rot = [&](int K, const double *bins, GoertzelParams &p) {
        std::vector<float4> rot(K * 16);
        for (int k = 0; k < K; ++k) {
            const double w = 2 * M_PI * bins[k] / 1024.0;
            p.coef[k] = (float)(2 * std::cos(w));
            for (int j = 0; j < 16; ++j) {
                const double a = -w * (64.0 * j + 63), b = -w * (64.0 * j + 64);
                rot[k * 16 + j] = make_float4((float)std::cos(a), (float)std::sin(a),
                                              (float)std::cos(b), (float)std::sin(b));
            }
        }
        float4 *d;
        CK(hipMalloc(&d, rot.size() * sizeof(float4)));
        CK(hipMemcpy(d, rot.data(), rot.size() * sizeof(float4), hipMemcpyHostToDevice));
        p.rot = d;
    };
    const double b2[2] = {32, 64}, b8[8] = {32, 40, 48, 56, 64, 72, 80, 88};
    GoertzelParams p2{}, p8{};
    p2.pcm = p8.pcm = pcm;
    p2.n_windows = p8.n_windows = W;
    p2.hop = p8.hop = 1024;
    p2.log2g = p8.log2g = 4;
    p2.k = 2;
    p8.k = 8;
    p2.mag = p8.mag = mag;
    make_rot(2, b2, p2);
    make_rot(8, b8, p8);

    // fold rotation tables: lane j holds folded positions 8j..8j+7
    GoertzelParams f2 = p2, f8 = p8;
    auto make_fold_rot = [&](int K, const double *bins, GoertzelParams &p) {
        std::vector<float4> rot(K * 16);
        for (int k = 0; k < K; ++k) {
            const double w = 2 * M_PI * bins[k] / 1024.0;
            for (int j = 0; j < 16; ++j) {
                const double a = -w * (8.0 * j + 7), b = -w * (8.0 * j + 8);
                rot[k * 16 + j] = make_float4((float)std::cos(a), (float)std::sin(a),
                                              (float)std::cos(b), (float)std::sin(b));
            }
        }
        float4 *d;
        CK(hipMalloc(&d, rot.size() * sizeof(float4)));
        CK(hipMemcpy(d, rot.data(), rot.size() * sizeof(float4), hipMemcpyHostToDevice));
        p.rot = d;
    };
    make_fold_rot(2, b2, f2);
    make_fold_rot(8, b8, f8);

    GoertzelParams p2s = p2, f2s = f2, f8s = f8, p2n = p2, f8n = f8;
    p2s.xcd_swizzle = f2s.xcd_swizzle = f8s.xcd_swizzle = 1;
    p2n.mag = f8n.mag = nullptr;
    add_variant(vs, GZ(2, 1, true, 4, false), 4, "goertzel [default]", p2, 2, cus, 1);
    add_variant(vs, GZ(2, 1, true, 4, false), 4, "goertzel K2", p2, 2, cus, 2);
    add_variant(vs, GZ(2, 1, true, 4, false), 4, "goertzel K2", p2, 2, cus, 4);
    add_variant(vs, GZ(2, 1, true, 4, false), 4, "goertzel K2", p2, 2, cus, 8);
    add_variant(vs, GZ(2, 2, true, 4, false), 4, "goertzel K2 PF2", p2, 2, cus, 4);
    add_variant(vs, GZ(2, 1, true, 8, false), 8, "goertzel K2", p2, 2, cus, 1);
    add_variant(vs, GZ(2, 1, true, 2, false), 2, "goertzel K2", p2, 2, cus, 1);
    add_variant(vs, GZ(2, 1, true, 1, false), 1, "goertzel K2", p2, 2, cus, 1);
    add_variant(vs, GZP(4), 4, "goertzel PK [default]", p8, 4, cus, 1);
    add_variant(vs, GZP(8), 4, "goertzel PK [default]", p8, 8, cus, 1);
    add_variant(vs, GZP(8), 4, "goertzel PK", p8, 8, cus, 2);
    add_variant(vs, GZP(8), 4, "goertzel PK", p8, 8, cus, 4);
    add_variant(vs, GZP(8), 4, "goertzel PK", p8, 8, cus, 0);
    add_variant(vs, GZP2(8), 4, "goertzel PK PF2", p8, 8, cus, 0);
    add_variant(vs, GZP2(8), 4, "goertzel PK PF2", p8, 8, cus, 4);
    add_variant(vs, FD(2, 4), 4, "fold", f2, 2, cus, 1);
    add_variant(vs, FD(8, 4), 4, "fold", f8, 8, cus, 1);
    add_variant(vs, GZW(2), 4, "goertzel WS", p2, 2, cus, 1);
    add_variant(vs, GZW(4), 4, "goertzel PK WS", p8, 4, cus, 1);
    add_variant(vs, GZW(8), 4, "goertzel PK WS", p8, 8, cus, 1);
    add_variant(vs, FDW(2), 4, "fold WS", f2, 2, cus, 1);
    add_variant(vs, FDW(8), 4, "fold WS", f8, 8, cus, 1);
#define FDWB(K, B) reinterpret_cast<const void *>(&fold_tile_kernel<K, 4, true, B, false, false, true>)
#define FDWP(K, B) reinterpret_cast<const void *>(&fold_tile_kernel<K, 4, true, B, false, false, true, true>)
#define FDWT(K, B) reinterpret_cast<const void *>(&fold_tile_kernel<K, 4, true, B, false, false, true, false, true>)
#define GZWB(K, B) reinterpret_cast<const void *>(&goertzel_tile_kernel<K, 4, 1, true, B, false, false, true, false, true>)
    add_variant(vs, FDWB(8, 2), 2, "fold WS", f8, 8, cus, 1);
    add_variant(vs, FDWB(2, 2), 2, "fold WS", f2, 2, cus, 1);
    add_variant(vs, FDWB(2, 1), 1, "fold WS", f2, 2, cus, 1);
    add_variant(vs, FDWB(2, 8), 8, "fold WS", f2, 2, cus, 1);
    add_variant(vs, FDWB(8, 1), 1, "fold WS", f8, 8, cus, 1);
    add_variant(vs, FDWP(8, 2), 2, "fold WS PK", f8, 8, cus, 1);
    add_variant(vs, FDWP(8, 4), 4, "fold WS PK", f8, 8, cus, 1);
    add_variant(vs, FDWT(8, 2), 2, "fold WS LDST", f8, 8, cus, 1);
    add_variant(vs, FDWT(8, 4), 4, "fold WS LDST", f8, 8, cus, 1);
    add_variant(vs, FDWT(2, 2), 2, "fold WS LDST", f2, 2, cus, 1);
    {
        // F16 (survey 8-FSK plan: bins 32..88 step 8 -> slots: Z0 tones 32,48,64,80; Z8 tones 40,56,72,88)
        static GoertzelParams f16 = f8;
        static const double b16[8] = {32, 48, 64, 80, 40, 56, 72, 88};
        std::vector<float4> rot(8 * 16);
        for (int k = 0; k < 8; ++k) {
            const double w = 2 * M_PI * b16[k] / 1024.0;
            f16.coef[k] = (float)(2 * std::cos(w));
            for (int j = 0; j < 16; ++j) {
                const double a = -w * (8.0 * (j & 7) + 7), b = -w * (8.0 * (j & 7) + 8);
                rot[k * 16 + j] = make_float4(std::cos(a), std::sin(a), std::cos(b), std::sin(b));
            }
        }
        float4 *d;
        CK(hipMalloc(&d, rot.size() * sizeof(float4)));
        CK(hipMemcpy(d, rot.data(), rot.size() * sizeof(float4), hipMemcpyHostToDevice));
        f16.rot = d;
        f16.perm = 0x75316420ull;  // nibble s = tone index (bins 32 + 8 i) of slot s
#define FD16(B) reinterpret_cast<const void *>(&fold_tile_kernel<8, 4, true, B, false, false, true, false, true, true>)
        add_variant(vs, FD16(2), 2, "fold F16", f16, 8, cus, 1);
        add_variant(vs, FD16(2), 2, "fold F16", f16, 8, cus, 2);
        add_variant(vs, FD16(2), 2, "fold F16", f16, 8, cus, 4);
        GoertzelParams f16n = f16;
        f16n.mag = nullptr;
        add_variant(vs, FD16(2), 2, "fold F16 nomag", f16n, 8, cus, 1);
    }
    add_variant(vs, reinterpret_cast<const void *>(&fold_tile_kernel<8, 4, true, 2, false, false, true, true, true>),
                2, "fold WS PK LDST", f8, 8, cus, 1);
    add_variant(vs, GZWB(8, 2), 2, "goertzel PK WS", p8, 8, cus, 1);
    {
        // residue-class folding (residue.hip): rotation table as demod_api.cpp
        auto make_res = [&](int K, const double *bins, GoertzelParams &p) {
            static const int kCls[8] = {0, 1, 3, 2, 0, 2, 3, 1};
            static const double kGam[8] = {0, 1, -1, 1, 0, -1, 1, -1};
            std::vector<float4> rot(K * 16 * 2);
            for (int k = 0; k < K; ++k) {
                const double w = 2 * M_PI * bins[k] / 1024.0;
                const int rho = (int)bins[k] % 8;
                const double al = rho == 4 ? 0 : 1, be = rho == 4 ? 1 : 0, ga = kGam[rho];
                p.coef[k] = (float)(2 * std::cos(w));
                p.zcls[k] = kCls[rho];
                for (int j = 0; j < 16; ++j) {
                    const double a = -w * (8.0 * j + 7), b = -w * (8.0 * j + 8);
                    const double Ar = std::cos(a), Ai = std::sin(a), Br = std::cos(b), Bi = std::sin(b);
                    rot[(k * 16 + j) * 2] = make_float4(al * Ar, al * Ai, be * Ar - ga * Ai, be * Ai + ga * Ar);
                    rot[(k * 16 + j) * 2 + 1] =
                        make_float4(-al * Br, -al * Bi, -(be * Br - ga * Bi), -(be * Bi + ga * Br));
                }
            }
            float4 *d;
            CK(hipMalloc(&d, rot.size() * sizeof(float4)));
            CK(hipMemcpy(d, rot.data(), rot.size() * sizeof(float4), hipMemcpyHostToDevice));
            p.rot = d;
            p.k = K;
        };
#define RZ(K) reinterpret_cast<const void *>(&residue_tile_kernel<K, 4>)
#define RZC(K) reinterpret_cast<const void *>(&residue_tile_kernel<K, 4, 4, false, false>)
#define RZV(K) reinterpret_cast<const void *>(&residue_tile_kernel<K, 4, 4, true, true>)
#define RZW(K, W) reinterpret_cast<const void *>(&residue_tile_kernel<K, 4, 4, true, false, W>)
#define RZQ(K, W, Q, PF) reinterpret_cast<const void *>(&residue_tile_kernel<K, 4, 4, true, false, W, Q, PF>)
#define RZA(K) reinterpret_cast<const void *>(&residue_tile_kernel<K, 4, 4, true, false, (K <= 8 ? 4 : 0), 2, false, false>)
        static double bo[16];
        for (int i = 0; i < 16; ++i) bo[i] = 32 + 9 * i;  // every class mod 8
        // the same 8 bins permuted so slot pairs (2c, 2c+1) share class c (DCLS)
        static const double bp[8] = {32, 68, 41, 95, 59, 77, 50, 86};
        static GoertzelParams r8p = p8;
        make_res(8, bp, r8p);
        add_variant(vs, reinterpret_cast<const void *>(&residue_tile_kernel<8, 4>), 4,
                    "residue perm", r8p, 8, cus, 1, residue_lds_bytes(8, 4, 2), "o");
        add_variant(vs, reinterpret_cast<const void *>(
                        &residue_tile_kernel<8, 4, 4, true, false, 4, 2, false, true, false, true>),
                    4, "residue DCLS perm", r8p, 8, cus, 1, residue_lds_bytes(8, 4, 2), "o");
        add_variant(vs, reinterpret_cast<const void *>(
                        &residue_tile_kernel<8, 4, 4, true, false, 0, 2, false, true, false, true>),
                    4, "residue DCLS rotLDSonly perm", r8p, 8, cus, 1, 8 * 16 * 2 * 16, "o");
        add_variant(vs, reinterpret_cast<const void *>(&residue_tile_kernel<8, 4>), 4,
                    "residue perm", r8p, 8, cus, 1, residue_lds_bytes(8, 4, 2), "o");
        add_variant(vs, reinterpret_cast<const void *>(
                        &residue_tile_kernel<8, 4, 4, true, false, 4, 2, false, true, false, true>),
                    4, "residue DCLS perm", r8p, 8, cus, 1, residue_lds_bytes(8, 4, 2), "o");
        static GoertzelParams r8s = p8, r3 = p8, r4 = p8, r8 = p8, r16 = p8, g3 = p8, g4 = p8, g8 = p8;
        make_res(8, b8, r8s);
        make_res(3, bo, r3);
        make_res(4, bo, r4);
        make_res(8, bo, r8);
        make_res(16, bo, r16);
        static double be[8];
        for (int i = 0; i < 8; ++i) be[i] = 34 + 6 * i;  // even bins: classes 0 and 3 only
        static GoertzelParams r8e = p8, g8e = p8;
        make_res(8, be, r8e);
        make_rot(8, be, g8e);
        make_rot(3, bo, g3);
        make_rot(4, bo, g4);
        make_rot(8, bo, g8);
        g3.k = 3;
        g4.k = 4;
        float *mag16;
        CK(hipMalloc(&mag16, W * 16 * sizeof(float)));
        r16.mag = mag16;
        add_variant(vs, RZ(8), 4, "residue (survey plan)", r8s, 8, cus, 1, residue_lds_bytes(8, 4));
        add_variant(vs, GZP(3), 4, "goertzel PK", g3, 3, cus, 1, 0, "o");
        add_variant(vs, RZ(3), 4, "residue", r3, 3, cus, 1, residue_lds_bytes(3, 4), "o");
        add_variant(vs, GZP(4), 4, "goertzel PK", g4, 4, cus, 1, 0, "o");
        add_variant(vs, RZ(4), 4, "residue", r4, 4, cus, 1, residue_lds_bytes(4, 4), "o");
        add_variant(vs, GZP(8), 4, "goertzel PK", g8, 8, cus, 1, 0, "o");
        add_variant(vs, RZ(8), 4, "residue", r8, 8, cus, 1, residue_lds_bytes(8, 4), "o");
        add_variant(vs, RZA(8), 4, "residue allreduce-epilogue", r8, 8, cus, 1, residue_lds_bytes(8, 4), "o");
        add_variant(vs, reinterpret_cast<const void *>(&residue_tile_kernel<8, 4, 4, true, false, 4, 2, false, true, true>),
                    4, "residue LDST", r8, 8, cus, 1, residue_lds_bytes(8, 4), "o");
        add_variant(vs, reinterpret_cast<const void *>(&residue_tile_kernel<16, 4, 4, true, false, 0, 2, false, true, true>),
                    4, "residue LDST", r16, 16, cus, 1, residue_lds_bytes(16, 4), "o");
        add_variant(vs, reinterpret_cast<const void *>(&residue_tile_kernel<8, 4, 2>), 2, "residue", r8, 8, cus, 1,
                    (8 * 16 * 2 + 2 * 4 * 2 * 64) * 16, "o");
        add_variant(vs, reinterpret_cast<const void *>(&residue_tile_kernel<8, 4, 1>), 1, "residue", r8, 8, cus, 1,
                    (8 * 16 * 2 + 1 * 4 * 2 * 64) * 16, "o");
        add_variant(vs, RZA(16), 4, "residue allreduce-epilogue", r16, 16, cus, 1, residue_lds_bytes(16, 4), "o");
        add_variant(vs, RZC(8), 4, "residue C-butterfly", r8, 8, cus, 1, residue_lds_bytes(8, 4), "o");
        add_variant(vs, RZV(8), 4, "residue VGPR-rot", r8, 8, cus, 1, residue_lds_bytes(8, 4), "o");
        add_variant(vs, RZW(8, 4), 4, "residue MINW4", r8, 8, cus, 1, residue_lds_bytes(8, 4), "o");
        add_variant(vs, RZW(8, 5), 4, "residue MINW5", r8, 8, cus, 1, residue_lds_bytes(8, 4), "o");
        // measured, not shipped (profiles/round1/probe_residue.log): QP1 (4 KiB LDS
        // per wave) with MINW5/6 spills; QP4 halves occupancy; PF on 2-4 tiles
        // per wave and VGPR-resident rotations are slower
        add_variant(vs, RZQ(8, 4, 1, false), 4, "residue MINW4 QP1", r8, 8, cus, 1, residue_lds_bytes(8, 4, 1), "o");
        add_variant(vs, RZQ(8, 3, 2, true), 4, "residue MINW3 PF", r8, 8, cus, 4, residue_lds_bytes(8, 4, 2), "o");
        {
            static GoertzelParams r5 = p8, r6 = p8, g5 = p8, g6 = p8;
            make_res(5, bo, r5);
            make_res(6, bo, r6);
            make_rot(5, bo, g5);
            make_rot(6, bo, g6);
            g5.k = 5;
            g6.k = 6;
            add_variant(vs, GZP(5), 4, "goertzel PK", g5, 5, cus, 1, 0, "o");
            add_variant(vs, RZ(5), 4, "residue", r5, 5, cus, 1, residue_lds_bytes(5, 4), "o");
            add_variant(vs, GZP(6), 4, "goertzel PK", g6, 6, cus, 1, 0, "o");
            add_variant(vs, RZ(6), 4, "residue", r6, 6, cus, 1, residue_lds_bytes(6, 4), "o");
            static GoertzelParams g16 = p8;
            make_rot(16, bo, g16);
            g16.k = 16;
            g16.mag = mag16;
            add_variant(vs, GZP(16), 4, "goertzel PK", g16, 16, cus, 1, 0, "o");
        }
        add_variant(vs, RZ(16), 4, "residue", r16, 16, cus, 1, residue_lds_bytes(16, 4), "o");
        add_variant(vs, RZ(8), 4, "residue", r8e, 8, cus, 1, residue_lds_bytes(8, 4), "e");
        add_variant(vs, GZW(8), 4, "goertzel PK WS", g8e, 8, cus, 1, 0, "e");
        add_variant(vs, GZW(8), 4, "goertzel PK WS", g8, 8, cus, 1, 0, "o");
#undef RZ
#undef RZC
#undef RZV
#undef RZW
#undef RZQ
#undef RZA
    }
    {
        // FFT detector tables (2-FSK bins 32, 64)
        std::vector<float> t1(1024), t2(1024);
        for (int m = 0; m < 512; ++m) {
            t1[2 * m] = (float)std::cos(-2 * M_PI * m / 512.0);
            t1[2 * m + 1] = (float)std::sin(-2 * M_PI * m / 512.0);
            t2[2 * m] = (float)std::cos(-2 * M_PI * m / 1024.0);
            t2[2 * m + 1] = (float)std::sin(-2 * M_PI * m / 1024.0);
        }
        float *d1, *d2;
        int *db;
        int hb[2] = {32, 64};
        CK(hipMalloc(&d1, 4096));
        CK(hipMalloc(&d2, 4096));
        CK(hipMalloc(&db, 8));
        CK(hipMemcpy(d1, t1.data(), 4096, hipMemcpyHostToDevice));
        CK(hipMemcpy(d2, t2.data(), 4096, hipMemcpyHostToDevice));
        CK(hipMemcpy(db, hb, 8, hipMemcpyHostToDevice));
        for (int hop : {1024, 256}) {
            for (int swz : {4, 9, 4, 9}) {
                FftParams fp{};
                fp.pcm = pcm;
                fp.hop = hop;
                fp.n_windows = (W * 1024 - 1024) / hop + 1;
                fp.k = 2;
                fp.xcd_swizzle = swz == 5 ? 1 : 0;
                fp.tw512 = d1;
                fp.tw1024 = d2;
                fp.bins = db;
                CK(hipMalloc(&fp.sym, fp.n_windows));
                CK(hipMalloc(&fp.mag, fp.n_windows * 8));
                Variant v;
                v.name = "fft1024 K=2 hop=" + std::to_string(hop) + " swz=" + std::to_string(swz & 1) +
                         (swz == 2 || swz == 3 ? " QUAD-r1" : swz == 6 ? " QUAD-new-4w" :
                          swz == 7 ? " QUAD-split" : swz == 8 ? " QUAD-fuse" :
                          swz == 9 ? " QUAD-fmt" : " QUAD-new") +
                         " windows=" + std::to_string(fp.n_windows);
                v.bytes = (double)W * 2048 + fp.n_windows * 9.0;  // stream bytes read once
                if (hop == 1024) v.sym = fp.sym;  // same windows as the Goertzel K=2 variants
                if (swz == 2 || swz == 3)
                    v.run = [fp](hipStream_t s) { CK(r1::launch_fft_quad(fp, s)); };
                else if (swz == 6)
                    v.run = [fp](hipStream_t s) { CK((launch_fft_quad_t<4, 4>(fp, s))); };
                else if (swz == 7)
                    v.run = [fp](hipStream_t s) { CK((launch_fft_quad_t<4, 0, true>(fp, s))); };
                else if (swz == 8)
                    v.run = [fp](hipStream_t s) { CK((launch_fft_quad_t<4, 0, false, true>(fp, s))); };
                else if (swz == 9)
                    v.run = [fp](hipStream_t s) { CK((launch_fft_quad_t<4, 0, false, false, true>(fp, s))); };
                else
                    v.run = [fp](hipStream_t s) { CK(launch_fft_quad(fp, s)); };
                vs.push_back(v);
            }
        }
    }
    auto add_read = [&](const char *label, const void *f, int L, int wpb) {
        Variant v;
        v.name = label;
        v.bytes = (double)W * 2048;
        const long long nt = W * 2048 / (1024LL * L);
        const unsigned blocks = (unsigned)((nt + wpb - 1) / wpb);
        v.run = [=](hipStream_t s) {
            const int16_t *pp = pcm;
            long long ntt = nt;
            unsigned *sk = sink;
            void *args[] = {&pp, &ntt, &sk};
            CK(hipLaunchKernel(f, dim3(blocks), dim3(64 * wpb), args, 0, s));
        };
        vs.push_back(v);
    };
#define RT(L, WPB, AUX) reinterpret_cast<const void *>(&read_tile_kernel<L, WPB, AUX>), L, WPB
    add_read("read-only one-shot tile (8 KiB/wave, nt, 4 waves/WG)", RT(8, 4, 2));
    add_read("read-only one-shot tile (8 KiB/wave, plain, 4 waves/WG)", RT(8, 4, 0));
    add_read("read-only one-shot tile (8 KiB/wave, nt, 8 waves/WG)", RT(8, 8, 2));
    add_read("read-only one-shot tile (8 KiB/wave, nt, 2 waves/WG)", RT(8, 2, 2));
    add_read("read-only one-shot tile (8 KiB/wave, nt, 1 waves/WG)", RT(8, 1, 2));
    add_read("read-only one-shot tile (8 KiB/wave, nt, 16 waves/WG)", RT(8, 16, 2));
    add_read("read-only one-shot tile (4 KiB/wave, nt, 4 waves/WG)", RT(4, 4, 2));
    add_read("read-only one-shot tile (16 KiB/wave, nt, 4 waves/WG)", RT(16, 4, 2));
    add_read("read-only one-shot tile (16 KiB/wave, nt, 8 waves/WG)", RT(16, 8, 2));
    add_read("read-only one-shot tile (32 KiB/wave, nt, 4 waves/WG)", RT(32, 4, 2));
    add_read("read-only one-shot tile (8 KiB/wave, sc0|nt, 4 waves/WG)", RT(8, 4, 3));
    add_read("read-only one-shot tile (8 KiB/wave, sc1|nt, 4 waves/WG)", RT(8, 4, 18));
#undef RT
    {
        const long long n16 = W * 2048 / 16;
        for (int g : {2048, 4096, 8192}) {
            Variant v;
            v.name = "read-only dwordx4 nt U=4 grid=" + std::to_string(g);
            v.bytes = (double)W * 2048;
            v.run = [=](hipStream_t s) {
                hipLaunchKernelGGL((read_kernel<true, 4>), dim3(g), dim3(256), 0, s,
                                   (const u32x4 *)pcm, n16, sink);
            };
            vs.push_back(v);
        }
        Variant v;
        v.name = "read-only dwordx4 plain U=4 grid=4096";
        v.bytes = (double)W * 2048;
        v.run = [=](hipStream_t s) {
            hipLaunchKernelGGL((read_kernel<false, 4>), dim3(4096), dim3(256), 0, s,
                               (const u32x4 *)pcm, n16, sink);
        };
        vs.push_back(v);
    }

    // PROBE_FILTER=substr[|substr...] keeps only matching variants (e.g. for
    // rocprofv3 --pmc)
    if (const char *flt = std::getenv("PROBE_FILTER")) {
        std::vector<std::string> subs;
        for (std::string f = flt;;) {
            const size_t bar = f.find('|');
            subs.push_back(f.substr(0, bar));
            if (bar == std::string::npos) break;
            f = f.substr(bar + 1);
        }
        std::vector<Variant> keep;
        for (auto &v : vs)
            for (auto &sub : subs)
                if (v.name.find(sub) != std::string::npos) {
                    keep.push_back(v);
                    break;
                }
        vs.swap(keep);
        if (vs.empty()) return 0;
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // get past the power-management transient of sustained streaming
    // (~60 launches) before any variant is timed
    for (int i = 0; i < 200; ++i) vs[0].run(nullptr);
    for (auto &v : vs) v.run(nullptr);
    CK(hipDeviceSynchronize());
    // PROBE_B2B=1: each variant's reps launch back to back (events between
    // launches, one sync per batch), as bench.py runs them; default: a host
    // sync after every launch.
    const bool b2b = std::getenv("PROBE_B2B") != nullptr;
    std::vector<hipEvent_t> evs(reps + 1);
    for (auto &e : evs) CK(hipEventCreate(&e));
    for (int r = 0; r < rounds; ++r)
        for (auto &v : vs) {
            if (b2b) {
                CK(hipEventRecord(evs[0], nullptr));
                for (int i = 0; i < reps; ++i) {
                    v.run(nullptr);
                    CK(hipEventRecord(evs[i + 1], nullptr));
                }
                CK(hipEventSynchronize(evs[reps]));
                for (int i = 0; i < reps; ++i) {
                    float ms;
                    CK(hipEventElapsedTime(&ms, evs[i], evs[i + 1]));
                    v.ms.push_back(ms);
                }
                continue;
            }
            for (int i = 0; i < reps; ++i) {
                CK(hipEventRecord(a, nullptr));
                v.run(nullptr);
                CK(hipEventRecord(b, nullptr));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                v.ms.push_back(ms);
            }
        }
    // cross-check symbols of every variant against the first variant of the same K
    std::vector<std::pair<std::string, std::vector<uint8_t>>> refs;
    std::vector<uint8_t> cur(W);
    for (auto &v : vs) {
        if (!v.sym) continue;
        CK(hipMemcpy(cur.data(), v.sym, W, hipMemcpyDeviceToHost));
        const size_t kp = v.name.find(" K=");
        const std::string key = v.name.substr(kp, v.name.find(' ', kp + 1) - kp);
        auto it = std::find_if(refs.begin(), refs.end(), [&](auto &r) { return r.first == key; });
        if (it == refs.end()) {
            refs.push_back({key, cur});
            continue;
        }
        long long bad = 0;
        for (long long i = 0; i < W; ++i) bad += cur[i] != it->second[i];
        if (bad) std::printf("MISMATCH %s: %lld\n", v.name.c_str(), bad);
    }
    std::printf("%-72s %9s %9s %9s %7s\n", "variant", "min_us", "med_us", "GB/s(med)", "%peak");
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        const double mn = v.ms.front() * 1e3, md = v.ms[v.ms.size() / 2] * 1e3;
        const double gbs = v.bytes / (md * 1e-6) / 1e9;
        std::printf("%-72s %9.1f %9.1f %9.1f %6.1f%%\n", v.name.c_str(), mn, md, gbs, gbs / 80.0);
    }
    return 0;
}
