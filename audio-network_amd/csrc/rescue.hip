// rescue.hip — the decision rescue.
//
// The detectors decide in fp32. A window whose fp32 top-2 margin is within the
// powers' error bound (demod_internal.h amb_margin) may have a different
// exact argmax, so its symbol leaves the detector with kSymAmbiguous set.
// This kernel, launched after a Goertzel detector on the same stream, finds
// those windows and decides them again with the definition's arithmetic in
// double precision, operation for operation as the specification states it
// (SURVEY.md §8 a3-a5): per tone, the sequential recurrence s = x + c s1 - s2
// over the window's n samples, P = s1^2 + s2^2 - c s1 s2, argmax with ties to
// the lowest tone. Every rounding step is the same as in oracle/fsk_oracle.c
// (goertzel_window_d: no contraction, same order, the same libm coefficients
// computed on the host), so a rescued window's powers are bit-identical to the
// oracle's and so is its symbol. The rescued powers are written (rounded to
// fp32) over the window's magnitudes. (The FFT detector rescues its windows
// inside its own kernel: rescue_fft.h.)
//
// Layout: one wave per 512 consecutive windows (round 3: 4096; with every
// window of a chunk flagged a wave served them one group after another, so
// eight times more waves bound the worst case eight times lower). It first reads
// their symbol bytes (dword loads, all in flight at once) and exits if none is
// flagged — the common case: one short pass over 1 byte per window. Otherwise
// it compacts the flagged windows, in order, into an LDS list. Goertzel:
// groups of up to 64 / K flagged windows are staged whole into LDS (stride
// 2 n + 16 bytes: conflict-free 16-byte reads across windows), then lane
// f K + t runs tone t of window f (K chains per window in parallel, the
// dependent fp64 chain of n steps per lane); lane f K decides.
#include "demod_internal.h"

namespace fskd {

// windows whose symbols one wave scans
constexpr int kRescueChunk = 512;
constexpr int kRescueLdsBytes = 32768;    // Goertzel: staged samples per group

typedef unsigned int u32x4q __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(64) void rescue_kernel(RescueParams p)
{
#pragma clang fp contract(off)
    __shared__ unsigned short idx[kRescueChunk];
    __shared__ __attribute__((aligned(16))) unsigned char smp[kRescueLdsBytes];
    __shared__ double pd[64];
    const int lane = threadIdx.x;
    // the chunk the detector's XCD-swizzled tiles wrote from this block's XCD
    // (tile_block): its symbol lines are still in this XCD's L2
    const long long base = tile_block(1) * kRescueChunk;
    const int span = (int)min((long long)kRescueChunk, p.n_windows - base);

    // 1. any flagged window in the chunk? (buffer loads bounded by the
    // chunk's record count: nothing past the last window is read)
    __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(p.sym + base), (short)0, span, 0x00020000);
    unsigned any = 0;
    if (p.sym_aligned4) {
#pragma unroll
        for (int c = 0; c < kRescueChunk / 256; ++c)
            any |= __builtin_amdgcn_raw_buffer_load_b32(rs, (64 * c + lane) * 4, 0, 0) & 0x80808080u;
        // a last dword cut by the record count reads as 0: its bytes one by one
        if (lane < (span & 3)) any |= __builtin_amdgcn_raw_buffer_load_b8(rs, (span & ~3) + lane, 0, 0) & 0x80u;
    } else {
        for (int c = 0; c < kRescueChunk / 64; ++c)
            any |= __builtin_amdgcn_raw_buffer_load_b8(rs, 64 * c + lane, 0, 0) & 0x80u;
    }
    if (__ballot(any != 0) == 0) return;

    // 2. the chunk's flagged windows, in order, into idx[0 .. T)
    int T = 0;
    for (int i = 0; i < kRescueChunk / 64; ++i) {
        const int o = 64 * i + lane;
        const bool f = o < span && (p.sym[base + o] & kSymAmbiguous);
        const unsigned long long b = __ballot(f);
        if (f) idx[T + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(b >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b, 0u))] =
            (unsigned short)o;
        T += __popcll(b);
    }
    __syncthreads();

    {
        // 3. Goertzel: groups of wpw windows, lane f K + t = tone t of window f
        const int K = p.k, n = p.n;
        const int stride = 2 * n + 16;
        int wpw = 64 / K;
        if (wpw * stride > kRescueLdsBytes) wpw = kRescueLdsBytes / stride;
        const int f = lane / K, t = lane - (lane / K) * K;
        for (int g0 = 0; g0 < T; g0 += wpw) {
            const int cnt = min(wpw, T - g0);
            const int chunks = n / 8;  // 16-byte chunks per window
            // 16-byte chunks, eight loads per lane in flight at a time (a
            // plain loop left one L2 round trip per chunk on the critical path)
            for (int c0 = 0; c0 < cnt * chunks; c0 += 8 * 64) {
                u32x4q v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int c = c0 + 64 * u + lane;
                    if (c < cnt * chunks) {
                        const int ff = c / chunks, q = c - ff * chunks;
                        const long long w = base + idx[g0 + ff];
                        v[u] = reinterpret_cast<const u32x4q *>(p.pcm + w * p.hop)[q];
                    }
                }
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int c = c0 + 64 * u + lane;
                    if (c < cnt * chunks) {
                        const int ff = c / chunks, q = c - ff * chunks;
                        *reinterpret_cast<u32x4q *>(smp + ff * stride + 16 * q) = v[u];
                    }
                }
            }
            __syncthreads();
            const bool act = f < cnt;
            double P = 0.0;
            if (act) {
                const double c = p.coef[t];
                double s1 = 0.0, s2 = 0.0;
                const u32x4q *xs = reinterpret_cast<const u32x4q *>(smp + f * stride);
#pragma unroll 4
                for (int q = 0; q < chunks; ++q) {
                    const u32x4q d = xs[q];
                    const unsigned d4[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const double x = (double)(short)((d4[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
                        double s = x + c * s1;
                        s = s - s2;
                        s2 = s1;
                        s1 = s;
                    }
                }
                const double a = s1 * s1 + s2 * s2;
                const double b = c * s1;
                P = a - b * s2;
                pd[lane] = P;
            }
            __syncthreads();
            if (act) {
                const long long w = base + idx[g0 + f];
                if (p.mag) p.mag[w * K + t] = (float)P;
                if (t == 0) {
                    double best = -1.0;
                    int arg = 0;
                    for (int k = 0; k < K; ++k)
                        if (pd[f * K + k] > best) {
                            best = pd[f * K + k];
                            arg = k;
                        }
                    p.sym[w] = (uint8_t)arg;
                }
            }
            __syncthreads();
        }
    }
}

hipError_t launch_rescue(const RescueParams &p, hipStream_t s)
{
    if (p.n_windows <= 0) return hipSuccess;
    if (p.k < 2 || p.k > kMaxTones) return hipErrorInvalidValue;
    if (p.n < 64 || (p.n % 8) || 2 * p.n + 16 > kRescueLdsBytes) return hipErrorInvalidValue;
    const long long blocks = (p.n_windows + kRescueChunk - 1) / kRescueChunk;
    if (blocks > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(rescue_kernel, dim3((unsigned)blocks), dim3(64), 0, s, p);
    return hipGetLastError();
}

}  // namespace fskd
