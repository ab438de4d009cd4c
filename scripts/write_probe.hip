// write_probe.hip — why a 1.5 % magnitude write stream costs ~13 % in
// back-to-back launches: read 2 GiB in 8 KiB tiles (nt
// buffer loads, as the tone-bank kernels do) and write 128 B per tile
// (32 MiB, the 8-FSK magnitudes), with different write schedules:
//   A  one tile per wave, its 128 B written right away (the shipped pattern)
//   C  persistent waves over contiguous tile ranges, writes right away
//   B  persistent waves, 128 B per tile staged in LDS, flushed every 32 tiles
//      as one 4 KiB burst per wave
// and each without writes. Launches back to back, HIP events in between.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/write_probe.hip -o scripts/bin/write_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <functional>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__device__ __forceinline__ unsigned tile_value(const short *p, long long t, int lane)
{
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)(p + t * 4096), (short)0, 8192, 0x00020000);
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, (64 * i + lane) * 16, 0, 2);
        acc += v.x ^ v.y ^ v.z ^ v.w;
    }
    // fold the upper half-wave into the lower one, so every lane's loads stay
    // live when only lanes 0-31 store
    return acc ^ (unsigned)__shfl_xor((int)acc, 32);
}

// W: 0 = no write, 1 = 128 B per tile (8-FSK magnitudes), 2 = 32 B per tile
// (2-FSK magnitudes), 3 = 4 B per tile (the symbols of its 4 windows)
template <int W>
__global__ __launch_bounds__(128) void kA(const short *p, long long n_tiles, unsigned *out)
{
    const int lane = threadIdx.x & 63;
    const long long t = (long long)blockIdx.x * 2 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (t >= n_tiles) return;
    unsigned v = tile_value(p, t, lane);
    if (W == 1) {
        if (lane < 32) out[t * 32 + lane] = v;
    } else if (W == 2) {
        v ^= (unsigned)__shfl_xor((int)v, 8) ^ (unsigned)__shfl_xor((int)v, 16);
        if (lane < 8) out[t * 8 + lane] = v;
    } else if (W == 3) {
        v ^= (unsigned)__shfl_xor((int)v, 1) ^ (unsigned)__shfl_xor((int)v, 2) ^ (unsigned)__shfl_xor((int)v, 4) ^
             (unsigned)__shfl_xor((int)v, 8) ^ (unsigned)__shfl_xor((int)v, 16);
        if (lane == 0) out[t] = v;
    } else if (v == 0x9E3779B9u) out[0] = v;
}

// 2-FSK pattern: per tile 4 B of symbols + 32 B of magnitudes into two arrays.
// S16: blocks of 16 waves stage both in LDS and write them as one 64 B and one
// 512 B contiguous store after a block barrier; S1: every wave writes its own.
template <bool STAGE>
__global__ __launch_bounds__(1024) void kS(const short *p, long long n_tiles, unsigned *sym, unsigned *mag)
{
    __shared__ unsigned ss[16], sm[16 * 8];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long t = (long long)blockIdx.x * 16 + wv;
    unsigned v = t < n_tiles ? tile_value(p, t, lane) : 0u;
    v ^= (unsigned)__shfl_xor((int)v, 8) ^ (unsigned)__shfl_xor((int)v, 16);
    if (!STAGE) {
        if (t < n_tiles) {
            if (lane < 8) mag[t * 8 + lane] = v;
            if (lane == 0) sym[t] = v >> 3;
        }
        return;
    }
    if (lane < 8) sm[wv * 8 + lane] = v;
    if (lane == 0) ss[wv] = v >> 3;
    __syncthreads();
    const long long t0 = (long long)blockIdx.x * 16;
    if (wv == 0) {
        if (lane < 16 && t0 + lane < n_tiles) sym[t0 + lane] = ss[lane];
    } else if (wv == 1) {
        for (int i = lane; i < 128; i += 64)
            if (t0 + i / 8 < n_tiles) mag[t0 * 8 + i] = sm[i];
    }
}

// A4: as A, the 128 B written by 8 lanes as dwordx4
__global__ __launch_bounds__(128) void kA4(const short *p, long long n_tiles, unsigned *out)
{
    const int lane = threadIdx.x & 63;
    const long long t = (long long)blockIdx.x * 2 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (t >= n_tiles) return;
    unsigned v = tile_value(p, t, lane);
    v ^= (unsigned)__shfl_xor((int)v, 8) ^ (unsigned)__shfl_xor((int)v, 16);
    if (lane < 8) reinterpret_cast<u32x4 *>(out)[t * 8 + lane] = u32x4{v, v + 1, v + 2, v + 3};
}

// persistent: wave g of G handles tiles [g T, (g + 1) T)
template <bool W, bool STAGE>
__global__ __launch_bounds__(256) void kP(const short *p, long long n_tiles, long long T, unsigned *out)
{
    __shared__ unsigned st[4][32 * 32];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long g = (long long)blockIdx.x * 4 + wv;
    const long long t0 = g * T, t1 = std::min(t0 + T, n_tiles);
    unsigned sink = 0;
    for (long long t = t0; t < t1; ++t) {
        const unsigned v = tile_value(p, t, lane);
        if (!W) { sink ^= v; continue; }
        if (!STAGE) {
            if (lane < 32) out[t * 32 + lane] = v;
            continue;
        }
        const int slot = (int)((t - t0) & 31);
        if (lane < 32) st[wv][slot * 32 + lane] = v;
        if (slot == 31 || t + 1 == t1) {
            __builtin_amdgcn_wave_barrier();
            const long long base = (t - slot) * 32;  // first staged tile's words
            const int words = (slot + 1) * 32;
            for (int i = lane; i < words; i += 64) out[base + i] = st[wv][i];
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (!W && sink == 0x9E3779B9u) out[0] = sink;
}

// D: persistent, every tile's 128 B staged in LDS (T <= 64 tiles per wave,
// 8 KiB), the whole range written at the end of the wave
__global__ __launch_bounds__(256) void kD(const short *p, long long n_tiles, long long T, unsigned *out)
{
    __shared__ unsigned st[4][64 * 32];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long long g = (long long)blockIdx.x * 4 + wv;
    const long long t0 = g * T, t1 = std::min(t0 + T, n_tiles);
    for (long long t = t0; t < t1; ++t) {
        const unsigned v = tile_value(p, t, lane);
        if (lane < 32) st[wv][(t - t0) * 32 + lane] = v;
    }
    __builtin_amdgcn_wave_barrier();
    const int words = (int)(t1 - t0) * 32;
    for (int i = lane; i < words; i += 64) out[t0 * 32 + i] = st[wv][i];
}

// E: writes only, 128 B per wave (the magnitude pattern without the reads)
__global__ __launch_bounds__(128) void kE(long long n_tiles, unsigned *out)
{
    const int lane = threadIdx.x & 63;
    const long long t = (long long)blockIdx.x * 2 + (threadIdx.x >> 6);
    if (t < n_tiles && lane < 32) out[t * 32 + lane] = (unsigned)t ^ lane;
}
// F: writes only, 1 KiB per wave instruction (dwordx4 from all 64 lanes)
__global__ __launch_bounds__(256) void kF(long long n16, u32x4 *out)
{
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) out[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

int main()
{
    const long long bytes = 2LL << 30, n_tiles = bytes / 8192;
    short *in; unsigned *out;
    CK(hipMalloc(&in, bytes)); CK(hipMalloc(&out, n_tiles * 128));
    CK(hipMemset(in, 3, bytes));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const long long waves = (long long)cus * 4 * 4;  // 4 blocks of 4 waves per CU
    const long long T = (n_tiles + waves - 1) / waves;
    struct V { const char *name; std::function<void()> run; std::vector<float> ms; };
    std::vector<V> vs;
    vs.push_back({"A one tile/wave, no write", [&] { hipLaunchKernelGGL(kA<0>, dim3(n_tiles / 2), dim3(128), 0, 0, in, n_tiles, out); }, {}});
    vs.push_back({"A one tile/wave, 128 B write", [&] { hipLaunchKernelGGL(kA<1>, dim3(n_tiles / 2), dim3(128), 0, 0, in, n_tiles, out); }, {}});
    vs.push_back({"A one tile/wave, 32 B write", [&] { hipLaunchKernelGGL(kA<2>, dim3(n_tiles / 2), dim3(128), 0, 0, in, n_tiles, out); }, {}});
    vs.push_back({"A one tile/wave, 4 B write", [&] { hipLaunchKernelGGL(kA<3>, dim3(n_tiles / 2), dim3(128), 0, 0, in, n_tiles, out); }, {}});
    unsigned *sym2;
    CK(hipMalloc(&sym2, n_tiles * 4));
    vs.push_back({"S1 2-FSK pattern, each wave its 4 B + 32 B", [&] { hipLaunchKernelGGL(kS<false>, dim3(n_tiles / 16), dim3(1024), 0, 0, in, n_tiles, sym2, out); }, {}});
    vs.push_back({"S16 2-FSK pattern, 16-wave block stages, 64 B + 512 B", [&] { hipLaunchKernelGGL(kS<true>, dim3(n_tiles / 16), dim3(1024), 0, 0, in, n_tiles, sym2, out); }, {}});
    vs.push_back({"A4 one tile/wave, 128 B as 8 x dwordx4", [&] { hipLaunchKernelGGL(kA4, dim3(n_tiles / 2), dim3(128), 0, 0, in, n_tiles, out); }, {}});
    vs.push_back({"P persistent, no write", [&] { hipLaunchKernelGGL((kP<false, false>), dim3(waves / 4), dim3(256), 0, 0, in, n_tiles, T, out); }, {}});
    vs.push_back({"C persistent, 128 B write per tile", [&] { hipLaunchKernelGGL((kP<true, false>), dim3(waves / 4), dim3(256), 0, 0, in, n_tiles, T, out); }, {}});
    vs.push_back({"B persistent, 4 KiB burst per 32 tiles", [&] { hipLaunchKernelGGL((kP<true, true>), dim3(waves / 4), dim3(256), 0, 0, in, n_tiles, T, out); }, {}});
    if (T <= 64)
        vs.push_back({"D persistent, all writes at the wave's end", [&] { hipLaunchKernelGGL(kD, dim3(waves / 4), dim3(256), 0, 0, in, n_tiles, T, out); }, {}});
    vs.push_back({"E writes only, 128 B per wave (32 MiB)", [&] { hipLaunchKernelGGL(kE, dim3(n_tiles / 2), dim3(128), 0, 0, n_tiles, out); }, {}});
    vs.push_back({"F writes only, dwordx4 (32 MiB)", [&] { hipLaunchKernelGGL(kF, dim3(n_tiles * 8 / 256), dim3(256), 0, 0, n_tiles * 8, (u32x4 *)out); }, {}});
    const int reps = 40;
    std::vector<hipEvent_t> ev(reps + 1);
    for (auto &e : ev) CK(hipEventCreate(&e));
    for (int i = 0; i < 100; ++i) vs[1].run();
    for (int r = 0; r < 3; ++r)
        for (auto &v : vs) {
            CK(hipEventRecord(ev[0]));
            for (int i = 0; i < reps; ++i) { v.run(); CK(hipEventRecord(ev[i + 1])); }
            CK(hipEventSynchronize(ev[reps]));
            for (int i = 0; i < reps; ++i) { float ms; CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1])); v.ms.push_back(ms); }
        }
    for (auto &v : vs) {
        std::sort(v.ms.begin(), v.ms.end());
        std::printf("%-44s median %7.1f us  min %7.1f us\n", v.name, v.ms[v.ms.size() / 2] * 1e3, v.ms[0] * 1e3);
    }
    return 0;
}
