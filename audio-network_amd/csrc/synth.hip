// synth.hip — device generator of the seeded FSK test signal.
//
// Same integer-exact function as oracle/fsk_oracle.c:oracle_synth_fsk
// (DESIGN.md §Synthetic input), evaluated 8 samples per thread: splitmix64 is
// counter-based, so any sample is generated independently and the bytes are
// identical to the CPU generator's (tests/test_gpu_parity.py checks this).
#include <cmath>
#include <mutex>
#include <vector>

#include "demod_internal.h"

namespace fskd {

// Module-scope device tables: one copy per device, owned (and freed) by the
// HIP runtime with the code object, so the library keeps no process-global
// heap allocations. The sine table is filled once per device under a lock
// (synth_prepare); the sink only keeps the read-ceiling loads alive.
__device__ int16_t g_sine_lut[16384];
__device__ unsigned g_ceiling_sink[16];

hipError_t synth_prepare()
{
    static std::mutex mu;
    static bool ready[kMaxDevices] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
    std::lock_guard<std::mutex> lock(mu);
    if (ready[dev]) return hipSuccess;
    // the Q15 sine table of oracle/fsk_oracle.c:oracle_sine_lut
    std::vector<int16_t> lut(16384);
    for (int i = 0; i < 16384; ++i)
        lut[i] = (int16_t)std::lrint(32767.0 * std::sin(2.0 * M_PI * (double)i / 16384.0));
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_sine_lut), lut.data(), lut.size() * sizeof(int16_t), 0,
                          hipMemcpyHostToDevice);
    if (e == hipSuccess) ready[dev] = true;
    return e;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void synth_kernel(SynthParams p)
{
    const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long total8 = p.n_windows * (long long)p.n / 8;
    if (gid >= total8) return;
    const long long base = gid * 8;
    const long long w = base / p.n;
    const int s0 = (int)(base - w * p.n);
    const uint64_t gamma = 0x9E3779B97F4A7C15ULL;
    const uint64_t rw = mix64(p.seed + (p.w0 + (uint64_t)w + 1) * gamma);
    const uint32_t sym = (uint32_t)(((rw >> 32) * (uint64_t)p.k) >> 32);
    const uint32_t phase0 = (uint32_t)rw;
    const uint64_t ns = mix64(rw ^ 0xA0761D6478BD642FULL);
    uint32_t inc = 0;
#pragma unroll
    for (int t = 0; t < kMaxTones; ++t)
        if ((uint32_t)t == sym) inc = p.inc[t];

    int16_t out[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        const uint32_t s = (uint32_t)(s0 + r);
        const uint32_t ph = phase0 + s * inc;
        const int32_t tone = (p.amplitude * (int32_t)g_sine_lut[ph >> 18] + 16384) >> 15;
        const uint64_t d = mix64(ns + ((uint64_t)s + 1) * gamma);
        const int64_t u = (int64_t)((d & 0xFFFF) + ((d >> 16) & 0xFFFF) +
                                    ((d >> 32) & 0xFFFF) + (d >> 48));
        const int64_t noise = ((u - 131070) * (int64_t)p.sigma * 113512) >> 32;
        int64_t v = (int64_t)tone + noise;
        v = v > 32767 ? 32767 : (v < -32768 ? -32768 : v);
        out[r] = (int16_t)v;
    }
    uint4 pk;
    pk.x = (uint16_t)out[0] | ((uint32_t)(uint16_t)out[1] << 16);
    pk.y = (uint16_t)out[2] | ((uint32_t)(uint16_t)out[3] << 16);
    pk.z = (uint16_t)out[4] | ((uint32_t)(uint16_t)out[5] << 16);
    pk.w = (uint16_t)out[6] | ((uint32_t)(uint16_t)out[7] << 16);
    *reinterpret_cast<uint4 *>(p.pcm + base) = pk;
    if (s0 == 0 && p.sym) p.sym[w] = (uint8_t)sym;
}

hipError_t launch_synth(const SynthParams &p, hipStream_t s)
{
    const long long total8 = p.n_windows * (long long)p.n / 8;
    const long long blocks = (total8 + 255) / 256;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p);
    return hipGetLastError();
}

}  // namespace fskd

namespace fskd {

typedef unsigned int u32x4s __attribute__((ext_vector_type(4)));

// Read-only reference stream for bench.py (demod_read_ceiling_async): each
// wave reads one contiguous 8 KiB tile with 8 coalesced 16 B/lane
// non-temporal buffer loads and discards it, i.e. the tile kernels' access
// pattern (2-wave blocks, XCD-swizzled tiles) with no compute and no stores.
// Its bandwidth on the box at hand is the practical ceiling the detector
// kernels are compared with.
__global__ __launch_bounds__(64 * kPlainWPB) void read_ceiling_kernel(const int16_t *p, long long n_tiles)
{
    const int lane = threadIdx.x & 63;
    const long long t = tile_block(1) * kPlainWPB + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (t >= n_tiles) return;
    __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(p + t * 4096), (short)0, 8192, 0x00020000);
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const u32x4s v = __builtin_amdgcn_raw_buffer_load_b128(rs, (64 * i + lane) * 16, 0, 2);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x9E3779B9u) g_ceiling_sink[lane & 15] = acc;  // keeps the loads; practically never stores
}

hipError_t launch_read_ceiling(const int16_t *p, long long n_bytes, hipStream_t s)
{
    const long long n_tiles = n_bytes / 8192;
    if (n_tiles <= 0) return hipSuccess;
    const long long blocks = (n_tiles + kPlainWPB - 1) / kPlainWPB;
    if (blocks > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(read_ceiling_kernel, dim3((unsigned)blocks), dim3(64 * kPlainWPB), 0, s, p,
                       n_tiles);
    return hipGetLastError();
}

}  // namespace fskd
