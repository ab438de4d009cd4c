// fmt_probe.hip — does a typed buffer load (16_16 SSCALED) convert int16 pairs
// to fp32 in the texture path, and at what rate against raw dword loads plus
// VALU converts? Experiment for the FFT detector's 64 converts per group.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/fmt_probe.hip -o scripts/bin/fmt_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef float f2 __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

// word3: DST_SEL x,y,z,w = 4,5,6,7; NUM_FORMAT 3 (SSCALED); DATA_FORMAT 5 (16_16)
constexpr int kFmtWord3 = 0xFAC | (3 << 12) | (5 << 15);

__device__ __forceinline__ f2 load_fmt(__amdgpu_buffer_rsrc_t rs, int voff)
{
    f2 v;
    asm volatile("buffer_load_format_xy %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(rs));
    return v;
}

__global__ void check_kernel(const short *p, f2 *out, int n_pairs)
{
    int i = blockIdx.x * 256 + threadIdx.x;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, n_pairs * 4, kFmtWord3);
    f2 v = load_fmt(rs, i * 4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (i < n_pairs) out[i] = v;
}

// Each wave reads one 8 KiB tile as 32 loads of 64 lanes x 4 B and sums.
template <bool FMT>
__global__ __launch_bounds__(256) void rate_kernel(const short *p, long long n_tiles, float *out)
{
    const int lane = threadIdx.x & 63;
    const long long t = (long long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (t >= n_tiles) return;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(p + t * 4096), (short)0, 8192, FMT ? kFmtWord3 : 0x00020000);
    f2 acc = {0.f, 0.f};
    if (FMT) {
        f2 v[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = load_fmt(rs, (64 * i + lane) * 4);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < 32; ++i) acc += v[i];
    } else {
        unsigned v[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, (64 * i + lane) * 4, 0, 2);
#pragma unroll
        for (int i = 0; i < 32; ++i)
            acc += f2{(float)(int)(short)(v[i] & 0xFFFFu), (float)((int)v[i] >> 16)};
    }
    if (acc.x == 1234.5f) out[0] = acc.y;
}

int main()
{
    // 1. conversion check
    const int np = 1 << 16;
    std::vector<short> h(2 * np);
    for (int i = 0; i < 2 * np; ++i) h[i] = (short)((i * 2654435761u) >> 7);
    h[0] = -32768; h[1] = 32767; h[2] = -1; h[3] = 0;
    short *d; f2 *o;
    CK(hipMalloc(&d, h.size() * 2)); CK(hipMalloc(&o, np * sizeof(f2)));
    CK(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(check_kernel, dim3(np / 256), dim3(256), 0, 0, d, o, np);
    CK(hipDeviceSynchronize());
    std::vector<f2> r(np);
    CK(hipMemcpy(r.data(), o, np * sizeof(f2), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < np; ++i)
        if (r[i].x != (float)h[2 * i] || r[i].y != (float)h[2 * i + 1]) {
            if (bad < 5) std::printf("mismatch %d: %d %d -> %g %g\n", i, h[2 * i], h[2 * i + 1], r[i].x, r[i].y);
            ++bad;
        }
    std::printf("format 16_16 SSCALED check: %d / %d pairs wrong\n", bad, np);
    // 2. rate
    const long long bytes = 2LL << 30, tiles = bytes / 8192;
    short *big; float *dummy;
    CK(hipMalloc(&big, bytes)); CK(hipMalloc(&dummy, 4));
    CK(hipMemset(big, 1, bytes));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    std::vector<float> ts[2];
    for (int rep = 0; rep < 12; ++rep)
        for (int f = 0; f < 2; ++f) {
            CK(hipEventRecord(a));
            if (f) hipLaunchKernelGGL(rate_kernel<true>, dim3(tiles / 4), dim3(256), 0, 0, big, tiles, dummy);
            else hipLaunchKernelGGL(rate_kernel<false>, dim3(tiles / 4), dim3(256), 0, 0, big, tiles, dummy);
            CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b));
            if (rep >= 2) ts[f].push_back(ms);
        }
    for (int f = 0; f < 2; ++f) {
        std::sort(ts[f].begin(), ts[f].end());
        float med = ts[f][ts[f].size() / 2];
        std::printf("%s: median %.1f us, %.0f GB/s\n", f ? "format_xy (SSCALED)" : "b32 + 2 cvt",
                    med * 1e3, bytes / (med * 1e-3) / 1e9);
    }
    return bad != 0;
}
