// rescue.hip — the decision rescue.
//
// The detectors decide in fp32. A window whose fp32 top-2 margin is within the
// powers' error bound (demod_internal.h amb_margin) may have a different
// exact argmax, so its symbol leaves the detector with kSymAmbiguous set.
// This kernel, launched after the detector on the same stream, finds those
// windows and decides them again with the definition's arithmetic in double
// precision, operation for operation as the specification states it:
//   * Goertzel detectors: per tone, the sequential
//     recurrence s = x + c s1 - s2 over the window's n samples,
//     P = s1^2 + s2^2 - c s1 s2, argmax with ties to the lowest tone;
//   * the FFT detector (a6): an iterative radix-2 DIT FFT of the window
//     (bit-reversed input, stages len = 2 .. n, twiddles cos / sin of
//     -2 pi j / len from a host table), P[b] = re^2 + im^2 at the tone bins.
// Every rounding step is the same as in oracle/fsk_oracle.c
// (goertzel_window_d, oracle_fft_power: no contraction, same order, the same
// libm coefficients and twiddles computed on the host), so a rescued window's
// powers are bit-identical to the oracle's and so is its symbol. The
// rescued powers are written (rounded to fp32) over the window's magnitudes
// and, for the FFT, its whole spectrum.
//
// Layout: one wave per 4096 consecutive windows (FFT: 1024). It first reads
// their symbol bytes (dword loads, all in flight at once) and exits if none is
// flagged — the common case: one short pass over 1 byte per window. Otherwise
// it compacts the flagged windows, in order, into an LDS list. Goertzel:
// groups of up to 64 / K flagged windows are staged whole into LDS (stride
// 2 n + 16 bytes: conflict-free 16-byte reads across windows), then lane
// f K + t runs tone t of window f (K chains per window in parallel, the
// dependent fp64 chain of n steps per lane); lane f K decides. FFT: one
// window at a time, 16 KiB of double re / im and the 16 KiB twiddle table in
// LDS, 8 butterflies per lane per stage.
#include "demod_internal.h"

namespace fskd {

// windows whose symbols one wave scans: Goertzel 4096; FFT 1024 (each
// flagged window is a whole FFT for the wave, so more waves share them)
constexpr int kRescueChunkG = 4096;
constexpr int kRescueChunkF = 1024;
constexpr int kRescueLdsBytes = 32768;    // Goertzel: staged samples per group (FFT: 16 KiB)

typedef unsigned int u32x4q __attribute__((ext_vector_type(4)));

__device__ __forceinline__ unsigned bitrev10(unsigned i)
{
    return __builtin_bitreverse32(i) >> 22;
}

template <bool FFT>
__global__ __launch_bounds__(64) void rescue_kernel(RescueParams p)
{
#pragma clang fp contract(off)
    constexpr int kRescueChunk = FFT ? kRescueChunkF : kRescueChunkG;
    __shared__ unsigned short idx[kRescueChunk];
    __shared__ __attribute__((aligned(16))) unsigned char smp[FFT ? 16384 : kRescueLdsBytes];
    __shared__ double pd[64];
    const int lane = threadIdx.x;
    const long long base = (long long)blockIdx.x * kRescueChunk;
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

    if constexpr (!FFT) {
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
    } else {
        // 3. FFT: one window at a time; the twiddle table is staged into LDS
        // once (a global read per butterfly put an L2 round trip into each
        // of the ten dependent stages)
        double *re = reinterpret_cast<double *>(smp);
        double *im = re + 1024;
        __shared__ double2 tw[1023];
        const double2 *gtw = reinterpret_cast<const double2 *>(p.tw);
        for (int i = lane; i < 1023; i += 64) tw[i] = gtw[i];
        for (int g0 = 0; g0 < T; ++g0) {
            const long long w = base + idx[g0];
            // lane l loads samples 16 l .. 16 l + 15 (two 16-byte loads, the
            // window start is 16-byte aligned) and scatters them bit-reversed
            const u32x4q *x = reinterpret_cast<const u32x4q *>(p.pcm + w * p.hop) + 2 * lane;
            const u32x4q x0 = x[0], x1 = x[1];
            const unsigned xs[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const unsigned r = bitrev10((unsigned)(16 * lane + e));
                re[r] = (double)(short)((xs[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
                im[r] = 0.0;
            }
            __syncthreads();
#pragma unroll
            for (int half = 1; half < 1024; half <<= 1) {
                const int len = 2 * half;
#pragma unroll
                for (int q = lane; q < 512; q += 64) {
                    const int j = q & (half - 1);
                    const int a = (q / half) * len + j, b = a + half;
                    const double2 wv = tw[half - 1 + j];
                    const double wr = wv.x, wi = wv.y;
                    const double tr = re[b] * wr - im[b] * wi;
                    const double ti = re[b] * wi + im[b] * wr;
                    const double ra = re[a], ia = im[a];
                    re[b] = ra - tr;
                    im[b] = ia - ti;
                    re[a] = ra + tr;
                    im[a] = ia + ti;
                }
                __syncthreads();
            }
            if (p.spec)
                for (int b = lane; b <= 512; b += 64)
                    p.spec[w * 513 + b] = (float)(re[b] * re[b] + im[b] * im[b]);
            if (lane < p.k) {
                const int b = p.bins[lane];
                const double P = re[b] * re[b] + im[b] * im[b];
                pd[lane] = P;
                if (p.mag) p.mag[w * p.k + lane] = (float)P;
            }
            __syncthreads();
            if (lane == 0) {
                double best = -1.0;
                int arg = 0;
                for (int k = 0; k < p.k; ++k)
                    if (pd[k] > best) {
                        best = pd[k];
                        arg = k;
                    }
                p.sym[w] = (uint8_t)arg;
            }
            __syncthreads();
        }
    }
}

hipError_t launch_rescue(const RescueParams &p, hipStream_t s)
{
    if (p.n_windows <= 0) return hipSuccess;
    if (p.k < 2 || p.k > kMaxTones) return hipErrorInvalidValue;
    if (p.fft ? (p.n != 1024 || !p.tw) : (p.n < 64 || (p.n % 8) || 2 * p.n + 16 > kRescueLdsBytes))
        return hipErrorInvalidValue;
    const int chunk = p.fft ? kRescueChunkF : kRescueChunkG;
    const long long blocks = (p.n_windows + chunk - 1) / chunk;
    if (blocks > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    if (p.fft)
        hipLaunchKernelGGL(rescue_kernel<true>, dim3((unsigned)blocks), dim3(64), 0, s, p);
    else
        hipLaunchKernelGGL(rescue_kernel<false>, dim3((unsigned)blocks), dim3(64), 0, s, p);
    return hipGetLastError();
}

}  // namespace fskd
