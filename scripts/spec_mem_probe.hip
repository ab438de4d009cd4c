// spec_mem_probe.hip — the memory floor of the full-spectrum FFT detector's
// traffic (config 4 with the spectrum stored, hop 256): the kernel's grid and
// access pattern with the arithmetic taken out.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude scripts/spec_mem_probe.hip -o scripts/bin/spec_mem_probe
//   scripts/bin/spec_mem_probe [rounds=6] [reps=5]
//
// Same persistent grid as fft1024_quad_kernel (4-wave blocks, 4 blocks per CU,
// XCD-swizzled group order), per 4-window group: the input loads of
// load_group (32 dword buffer loads per lane, 16 lanes per window, cached) and
// / or the linear-slab spectrum stores (9 x 16-byte stores per lane, the
// group's 4 x 513 floats as one contiguous run). Variants: read only, write
// only, read + write (nt / plain stores), read + write with the writes of a
// group issued before the next group's loads or after them. Round-robin over
// variants, HIP events, median per variant (cdna_hip_programming.md §5.4).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,      \
                         hipGetErrorString(e_));                                \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ long long tile_block_swz()
{
    const long long b = blockIdx.x, nb = gridDim.x;
    const long long per = nb / 8, full = per * 8;
    if (b >= full) return b;
    return (b % 8) * per + b / 8;
}

// R: read the group's input; W: 0 no writes, 1 nt stores, 2 plain stores,
// 3 buffer stores with cache-policy bits AUX; RUN: each wave takes a
// contiguous run of groups instead of every stride-th; RAUX: the loads'
// cache-policy bits
template <bool R, int W, int AUX = 0, bool RUN = false, int RAUX = 0, bool WIDE = false>
__global__ __launch_bounds__(256) void mem_kernel(const short *pcm, long long n_windows, long long hop,
                                                  float *spec, unsigned *sink)
{
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = lane >> 4, t = lane & 15;
    const long long n_groups = (n_windows + 3) >> 2;
    const long long n_waves = (long long)gridDim.x * 4;
    const long long wid = tile_block_swz() * 4 + wave;
    const long long per = (n_groups + n_waves - 1) / n_waves;
    const long long stride = RUN ? 1 : n_waves;
    const long long g_begin = RUN ? wid * per : wid;
    const long long g_end = RUN ? (g_begin + per < n_groups ? g_begin + per : n_groups) : n_groups;
    unsigned acc = 0;
    for (long long g = g_begin; g < g_end; g += stride) {
        if constexpr (R && WIDE) {
            // the group's 4 windows as one contiguous span (3 hops + 1024
            // samples), 16 B per lane: 4 wide loads per lane instead of 32 dwords
            const long long w0 = 4 * g;
            const long long left = n_windows - w0;
            long long bytes = (((left < 4 ? left : 4) - 1) * hop + 1024) * 2;
            __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(pcm + w0 * hop), (short)0, (int)bytes, 0x00020000);
            u4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * (64 * i + lane), 0, RAUX);
#pragma unroll
            for (int i = 0; i < 4; ++i) acc += (v[i].x ^ v[i].y ^ v[i].z ^ v[i].w) * (unsigned)(2 * i + 1);
        }
        if constexpr (R && !WIDE) {
            const long long w0 = 4 * g;
            const long long left = n_windows - w0;
            const long long wq = q < left ? q : left - 1;
            long long bytes = ((left - 1) * hop + 1024) * 2;
            if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
            __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                (void *)(pcm + w0 * hop), (short)0, (int)bytes, 0x00020000);
            const int voff = (int)(wq * hop * 2) + 4 * t;
            unsigned nx[32];
#pragma unroll
            for (int n1 = 0; n1 < 32; ++n1) nx[n1] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 64 * n1, 0, RAUX);
#pragma unroll
            for (int n1 = 0; n1 < 32; ++n1) acc += nx[n1] * (unsigned)(2 * n1 + 1);
        }
        if constexpr (W > 0) {
            const long long wg = 4 * g;
            const int L = 513 * (int)(n_windows - wg < 4 ? n_windows - wg : 4);
            float *dst = spec + wg * 513;
            const f4 v = {(float)acc, 1.f, 2.f, 3.f};
#pragma unroll
            for (int i = 0; i < 9; ++i) {
                const int f = 64 * i + lane;
                if (4 * f + 4 <= L) {
                    if constexpr (W == 1)
                        __builtin_nontemporal_store(v, reinterpret_cast<f4 *>(dst + 4 * f));
                    else if constexpr (W == 3) {
                        __amdgpu_buffer_rsrc_t ws = __builtin_amdgcn_make_buffer_rsrc(
                            (void *)dst, (short)0, L * 4, 0x00020000);
                        __builtin_amdgcn_raw_buffer_store_b128(
                            *reinterpret_cast<const __attribute__((ext_vector_type(4))) unsigned *>(&v),
                            ws, 16 * f, 0, AUX);
                    } else
                        *reinterpret_cast<f4 *>(dst + 4 * f) = v;
                } else if (4 * f < L) {
                    for (int e = 4 * f; e < L; ++e) dst[e] = v.x;
                }
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

struct Var {
    const char *name;
    void (*kern)(const short *, long long, long long, float *, unsigned *);
    std::vector<float> ms;
};

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 6;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const long long n_samples = 1LL << 30, hop = 256;
    const long long W = (n_samples - 1024) / hop + 1;
    short *pcm;
    float *spec;
    unsigned *sink;
    CK(hipMalloc(&pcm, n_samples * 2));
    CK(hipMalloc(&spec, W * 513 * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(pcm, 1, n_samples * 2));
    int dev = 0, cus = 256;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const unsigned blocks = (unsigned)cus * 4;
    std::vector<Var> vs = {
        {"read only (cached loads)", mem_kernel<true, 0>, {}},
        {"write only (nt 16 B)", mem_kernel<false, 1>, {}},
        {"write only (plain 16 B)", mem_kernel<false, 2>, {}},
        {"read + write (nt)", mem_kernel<true, 1>, {}},
        {"read + write (plain)", mem_kernel<true, 2>, {}},
        {"r+w buffer aux 1 (sc0)", mem_kernel<true, 3, 1>, {}},
        {"r+w buffer aux 2 (nt)", mem_kernel<true, 3, 2>, {}},
        {"r+w buffer aux 3 (sc0 nt)", mem_kernel<true, 3, 3>, {}},
        {"r+w buffer aux 16 (sc1)", mem_kernel<true, 3, 16>, {}},
        {"r+w buffer aux 18 (sc1 nt)", mem_kernel<true, 3, 18>, {}},
        {"r+w buffer aux 19 (sc0 sc1 nt)", mem_kernel<true, 3, 19>, {}},
        {"w only buffer aux 18", mem_kernel<false, 3, 18>, {}},
        {"w only buffer aux 19", mem_kernel<false, 3, 19>, {}},
        {"r+w nt, runs per wave", mem_kernel<true, 1, 0, true>, {}},
        {"w only nt, runs per wave", mem_kernel<false, 1, 0, true>, {}},
        {"w only plain, runs per wave", mem_kernel<false, 2, 0, true>, {}},
        {"r+w plain, runs per wave", mem_kernel<true, 2, 0, true>, {}},
        {"r(nt)+w nt", mem_kernel<true, 1, 0, false, 2>, {}},
        {"r(nt)+w plain", mem_kernel<true, 2, 0, false, 2>, {}},
        {"r(sc0)+w nt", mem_kernel<true, 1, 0, false, 1>, {}},
        {"r(nt)+w nt, runs per wave", mem_kernel<true, 1, 0, true, 2>, {}},
        {"r(nt)+w plain, runs per wave", mem_kernel<true, 2, 0, true, 2>, {}},
        {"r(sc0 nt)+w nt", mem_kernel<true, 1, 0, false, 3>, {}},
        // round 3, late: the group's span in 4 x 16 B per lane (each byte once per group)
        {"read only wide", mem_kernel<true, 0, 0, false, 0, true>, {}},
        {"r wide + w nt", mem_kernel<true, 1, 0, false, 0, true>, {}},
        {"r wide + w plain", mem_kernel<true, 2, 0, false, 0, true>, {}},
        {"r wide(nt) + w nt", mem_kernel<true, 1, 0, false, 2, true>, {}},
        {"r wide + w nt, runs per wave", mem_kernel<true, 1, 0, true, 0, true>, {}},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r)
        for (auto &v : vs) {
            for (int k = 0; k < 2; ++k)
                hipLaunchKernelGGL(v.kern, dim3(blocks), dim3(256), 0, nullptr, pcm, W, hop, spec, sink);
            for (int k = 0; k < reps; ++k) {
                CK(hipEventRecord(e0, nullptr));
                hipLaunchKernelGGL(v.kern, dim3(blocks), dim3(256), 0, nullptr, pcm, W, hop, spec, sink);
                CK(hipEventRecord(e1, nullptr));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.ms.push_back(ms);
            }
        }
    CK(hipGetLastError());
    const double rd = (double)n_samples * 2, wr = (double)W * 513 * 4;
    for (auto &v : vs) {
        std::vector<float> m = v.ms;
        std::sort(m.begin(), m.end());
        const double med = m[m.size() / 2];
        const bool R = v.name[0] == 'r';
        const bool Wr = v.kern != mem_kernel<true, 0> && v.kern != mem_kernel<true, 0, 0, false, 0, true>;
        const double bytes = (R ? rd : 0) + (Wr ? wr : 0);
        std::printf("%-28s W %lld: min %.4f ms median %.4f ms  %.2f TB/s (unique bytes %.2f GB)\n", v.name, W,
                    m[0], med, bytes / (med * 1e-3) / 1e12, bytes / 1e9);
    }
    return 0;
}
