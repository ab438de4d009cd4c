// fft_transpose_probe.hip — what the FFT detector's LDS transpose costs
// (configs[3], hop 256, 4 194 301 windows): the shipped
// kernel's grid, group loop, input loads and int16 -> fp32 converts, with the
// DFT arithmetic replaced by a synthetic packed-FMA stream of the same length,
// and the transpose (fft1024_quad_kernel's OVL order: round 0's 16 writes
// and column reads, then round 1's, per lane of a 16-lane window row, rows of
// 17 complex) either in or out. Results are deliberately meaningless.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/fft_transpose_probe.hip -o scripts/bin/fft_transpose_probe
//   scripts/bin/fft_transpose_probe [rounds=6] [reps=5] [valu=480]
//
// Variants (T: the transpose; V: `valu` packed FMAs per group, the shipped
// kernel's 540 VALU per group less its 64 converts is 476, rounded to 480):
//   ld          loads + converts only
//   ld+T        + the transpose
//   ld+V        + the FMA stream
//   ld+T+V      + both: the shipped kernel's shape
//   V, T+V      no loads (the converts of lane-computed words instead)
//   R:ld+T+V    two windows per row per iteration, the second reusing 24 of
//               the first's 32 loaded dwords (8 new loads, issued early)
// The transpose's marginal cost in the kernel's own shape is
// (ld+T+V) - (ld+V); in isolation (ld+T) - (ld). Round-robin over variants,
// HIP events, medians (cdna_hip_programming.md §5.4).
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

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kRow = 17, kWin = 16 * kRow, kSlab = 4 * kWin;

__device__ __forceinline__ long long tile_block_swz()
{
    const long long b = blockIdx.x, nb = gridDim.x;
    const long long per = nb / 8, full = per * 8;
    if (b >= full) return b;
    return (b % 8) * per + b / 8;
}

template <bool T, bool V, bool L = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void probe_kernel(
    const short *pcm, long long n_windows, long long hop, int valu, float *sink)
{
    __shared__ __attribute__((aligned(16))) f2 slab[4][kSlab];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = lane >> 4, t = lane & 15;
    const int k1b = t == 0 ? 16 : 32 - t;
    const long long n_groups = (n_windows + 3) >> 2;
    const long long stride = (long long)gridDim.x * 4;
    f2 acc = {0.f, 0.f};
    const f2 c1 = {1.0001f, 0.9999f}, c2 = {-0.5f, 0.25f};
    for (long long g = tile_block_swz() * 4 + wave; g < n_groups; g += stride) {
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
        for (int n1 = 0; n1 < 32; ++n1)
            nx[n1] = L ? __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 64 * n1, 0, 0)
                       : (unsigned)(voff + 64 * n1) * 0x9E3779B9u;   // L false: no loads
        f2 a[32];
#pragma unroll
        for (int n1 = 0; n1 < 32; ++n1) {
            a[n1] = (f2){(float)(int)(short)(nx[n1] & 0xFFFFu), (float)((int)nx[n1] >> 16)};
            asm("" : "+v"(a[n1]));
        }
        f2 b[32];
        if constexpr (T) {
            f2 *win = slab[wave] + q * kWin;
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int c = 0; c < 16; ++c) win[t * kRow + c] = a[c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int n2 = 0; n2 < 16; ++n2) b[n2] = win[n2 * kRow + t];
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int c = 0; c < 16; ++c) win[t * kRow + c] = a[16 + c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int n2 = 0; n2 < 16; ++n2) b[16 + n2] = win[n2 * kRow + k1b - 16];
        } else {
#pragma unroll
            for (int i = 0; i < 32; ++i) b[i] = a[i];
        }
        if constexpr (V) {
            // `valu` packed FMAs over 32 independent chains (the DFT's ILP)
            for (int r = 0; r < valu / 32; ++r) {
#pragma unroll
                for (int i = 0; i < 32; ++i) b[i] = __builtin_elementwise_fma(b[i], c1, c2);
            }
        }
#pragma unroll
        for (int i = 0; i < 32; ++i) acc += b[i];
    }
    if (acc.x == 1234.5f) sink[threadIdx.x] = acc.y;
}

// R: two windows per row per iteration (rows q handle windows 2q, 2q + 1 of
// an 8-window block), the second reusing 24 of the first's 32 loaded dwords
// (hop 256 = 8 n1 positions) and loading 8 new ones, issued right after the
// first window's loads so they are in flight during its transpose + FMAs
template <bool T, bool V>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void reuse_kernel(
    const short *pcm, long long n_windows, long long hop, int valu, float *sink)
{
    __shared__ __attribute__((aligned(16))) f2 slab[4][kSlab];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = lane >> 4, t = lane & 15;
    const int k1b = t == 0 ? 16 : 32 - t;
    const long long n_blocks = (n_windows + 7) >> 3;
    const long long stride = (long long)gridDim.x * 4;
    f2 acc = {0.f, 0.f};
    const f2 c1 = {1.0001f, 0.9999f}, c2 = {-0.5f, 0.25f};
    for (long long g = tile_block_swz() * 4 + wave; g < n_blocks; g += stride) {
        const long long w0 = 8 * g;
        const long long left = n_windows - w0;
        const long long wq = 2 * q < left ? 2 * q : left - 1;
        long long bytes = ((left - 1) * hop + 1024) * 2;
        if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(pcm + w0 * hop), (short)0, (int)bytes, 0x00020000);
        const int voff = (int)(wq * hop * 2) + 4 * t;
        unsigned nx[40];
#pragma unroll
        for (int n1 = 0; n1 < 32; ++n1) nx[n1] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 64 * n1, 0, 0);
#pragma unroll
        for (int n1 = 32; n1 < 40; ++n1) nx[n1] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 64 * n1, 0, 0);
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            f2 a[32];
#pragma unroll
            for (int n1 = 0; n1 < 32; ++n1) {
                const unsigned x = nx[n1 + 8 * pass];
                a[n1] = (f2){(float)(int)(short)(x & 0xFFFFu), (float)((int)x >> 16)};
                asm("" : "+v"(a[n1]));
            }
            f2 b[32];
            if constexpr (T) {
                f2 *win = slab[wave] + q * kWin;
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int c = 0; c < 16; ++c) win[t * kRow + c] = a[c];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int n2 = 0; n2 < 16; ++n2) b[n2] = win[n2 * kRow + t];
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int c = 0; c < 16; ++c) win[t * kRow + c] = a[16 + c];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int n2 = 0; n2 < 16; ++n2) b[16 + n2] = win[n2 * kRow + k1b - 16];
            } else {
#pragma unroll
                for (int i = 0; i < 32; ++i) b[i] = a[i];
            }
            if constexpr (V) {
                for (int r = 0; r < valu / 32; ++r) {
#pragma unroll
                    for (int i = 0; i < 32; ++i) b[i] = __builtin_elementwise_fma(b[i], c1, c2);
                }
            }
#pragma unroll
            for (int i = 0; i < 32; ++i) acc += b[i];
        }
    }
    if (acc.x == 1234.5f) sink[threadIdx.x] = acc.y;
}

struct Var {
    const char *name;
    void (*kern)(const short *, long long, long long, int, float *);
    std::vector<float> ms;
};

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? std::atoi(argv[1]) : 6;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const int valu = argc > 3 ? std::atoi(argv[3]) : 480;
    const long long n_samples = 1LL << 30, hop = 256;
    const long long W = (n_samples - 1024) / hop + 1;
    short *pcm;
    float *sink;
    CK(hipMalloc(&pcm, n_samples * 2));
    CK(hipMalloc(&sink, 4096));
    CK(hipMemset(pcm, 1, n_samples * 2));
    int dev = 0, cus = 256;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const unsigned blocks = (unsigned)cus * 4;
    std::vector<Var> vs = {
        {"ld", probe_kernel<false, false>, {}},
        {"ld+T", probe_kernel<true, false>, {}},
        {"ld+V", probe_kernel<false, true>, {}},
        {"ld+T+V", probe_kernel<true, true>, {}},
        {"V", probe_kernel<false, true, false>, {}},
        {"T+V", probe_kernel<true, true, false>, {}},
        {"R:ld+T+V", reuse_kernel<true, true>, {}},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r)
        for (auto &v : vs) {
            for (int k = 0; k < 2; ++k)
                hipLaunchKernelGGL(v.kern, dim3(blocks), dim3(256), 0, nullptr, pcm, W, hop, valu, sink);
            for (int k = 0; k < reps; ++k) {
                CK(hipEventRecord(e0, nullptr));
                hipLaunchKernelGGL(v.kern, dim3(blocks), dim3(256), 0, nullptr, pcm, W, hop, valu, sink);
                CK(hipEventRecord(e1, nullptr));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.ms.push_back(ms);
            }
        }
    CK(hipGetLastError());
    std::vector<double> med;
    for (auto &v : vs) {
        std::vector<float> m = v.ms;
        std::sort(m.begin(), m.end());
        med.push_back(m[m.size() / 2]);
        std::printf("%-8s W %lld valu %d: min %.4f ms median %.4f ms\n", v.name, W, valu, m.front(), med.back());
    }
    std::printf("transpose in isolation (ld+T - ld): %.4f ms; in the kernel's shape (ld+T+V - ld+V): %.4f ms\n",
                med[1] - med[0], med[3] - med[2]);
    std::printf("loads + converts in the kernel's shape (ld+T+V - T+V): %.4f ms; VALU stream alone (V): %.4f ms\n",
                med[3] - med[5], med[4]);
    std::printf("two windows per row reusing 24 of 32 loads (R:ld+T+V): %.4f ms against ld+T+V %.4f ms\n",
                med[6], med[3]);
    return 0;
}
