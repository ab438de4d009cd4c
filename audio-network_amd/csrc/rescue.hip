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
// Two kernels share the scan and compaction below: rescue_kernel (n != 1024,
// or the first pass switched off: the exact chains only) and
// rescue_seg_kernel (n = 1024, round 5: the first pass, then the exact
// chains of what it leaves).
//
// Layout (rescue_kernel): one wave per 512 consecutive windows (round 3:
// 4096; with every window of a chunk flagged a wave served them one group
// after another, so eight times more waves bound the worst case eight times
// lower; rescue_seg_kernel runs 4 waves per chunk, below). It first reads
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
// rescue_seg_kernel: waves per chunk's block. A chunk of 512 near ties is ~2 ms
// of one wave's work; 2048 chunks per 2^20 windows at one wave each are 2
// waves per SIMD, too few to hide the double chains' latency (and 4 x the
// blocks of one wave each cost ~2.5 us of dispatch per launch)
constexpr int kRescueSplit = 4;
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

// n = 1024 with the first pass (round 5): the rescue of
// segment-shared windows (SLIDE, fold-slide), which every window of a stream
// of near ties reaches. rescue_kernel stages each group of 64 / K windows in
// 32 KiB of LDS for K lanes per window's exact chains: one wave per SIMD and
// 1 024 dependent double steps per lane (6.1 ms for 4.19 M windows of two
// equal tones at hop 256, 12x the detector). Here the flagged windows take
// rescue_rows' pass 0 (demod_internal.h): every tone's double recurrence over
// each of the window's 16 segments of 64 samples, rotated into the window's
// phase (rot64), summed over the segments in a 16-lane row (DPP, the xor
// butterfly's tree);
// where the top-2 margin clears t2e64 E P_max (the derived bound,
// error_model.cpp) the window is decided (symbol, powers rounded to fp32).
// A segment's recurrence starts from zero at the segment, so at hop = 64 H
// (H < 16) the windows of a run share their segments' end states bit for bit:
//  dense runs: R consecutive windows holding enough flagged ones run each of
//    their (R - 1) H + 16 segments' chains once (lane per segment and tone
//    pair, 128 contiguous bytes per lane), the end states and fp32 sums x^2
//    go to LDS, and each flagged window's row rotates and sums its 16 (at
//    hop 256: a quarter of the chains);
//  sparse windows: the row runs its window's 16 segments itself;
//  fold plans (plan.h fold64; p.fold64): every window's pass 0 by the fold
//    (rescue_rows_fold0's arithmetic: lane j's folded samples 8j .. 8j + 7,
//    8-step chains), no runs;
//  pass 1: the windows pass 0 leaves (exact ties) take the exact chain, lane
//    f K + t on tone t of window f, its 1 024 samples read from L2 directly:
//    every rounding step of oracle/fsk_oracle.c, bit-identical powers and
//    symbol.
// LDS end states per dense run: segments x K (256: 4 waves per SIMD with the
// 4-wave chunk blocks; 512 held them at 3 by LDS and measured 2 % slower on
// the 2-FSK hop-256 worst case, profiles/round5/r5zx/)
constexpr int kSegStates = 256;

#ifdef FSKD_BOUNDS_DEBUG
// debug builds only (a bounds probe): report an out-of-range index and clamp it
#define RS_CHECK(v, lim, tag)                                                                  \
    do {                                                                                      \
        if ((long long)(v) < 0 || (long long)(v) >= (long long)(lim)) {                       \
            printf("RS_CHECK %s: %lld not in [0, %lld) block %d lane %d\n", tag, (long long)(v), \
                   (long long)(lim), (int)blockIdx.x, (int)threadIdx.x);                      \
            v = 0;                                                                            \
        }                                                                                     \
    } while (0)
#else
#define RS_CHECK(v, lim, tag) \
    do {                      \
    } while (0)
#endif

// Tones c0, c1's recurrences over one segment's 64 samples (8 chunks of 8),
// from zero: rescue_rows' pass-0 arithmetic, operation for operation.
// v is made opaque first: the extractions are not shared with an earlier use
// (seg_energy64's were kept live, 64 VGPRs, for these).
__device__ __forceinline__ void seg_pair(u32x4q (&v)[8], double c0, double c1, double &a1,
                                         double &a2, double &b1, double &b2)
{
#pragma clang fp contract(off)
#pragma unroll
    for (int q = 0; q < 8; ++q) asm volatile("" : "+v"(v[q]));
    a1 = a2 = b1 = b2 = 0.0;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const unsigned d4[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const double x = (double)(short)((d4[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
            double sa = x + c0 * a1;
            sa = sa - a2;
            a2 = a1;
            a1 = sa;
            double sb = x + c1 * b1;
            sb = sb - b2;
            b2 = b1;
            b1 = sb;
        }
        // a chunk's conversions stay with its steps (scheduled early, the 64
        // doubles took 128 VGPRs)
        __builtin_amdgcn_sched_barrier(0);
    }
}

// A lane's sum x^2 over its 64 samples (8 x 16 bytes): per dword the exact
// x_lo^2 + x_hi^2 by one v_dot2_i32_i16 (clamped: only (-32768, -32768)
// reaches 2^31, read as 2^31 - 1), converted and summed in fp32 — 3
// instructions per 2 samples instead of 4, relative error < 36 u for the 32
// non-negative terms (error_model.cpp's E allows 100 u)
typedef short rs_short2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float seg_energy64(const u32x4q (&v)[8])
{
    float e = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const unsigned d4[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const rs_short2 s = __builtin_bit_cast(rs_short2, d4[c]);
            e += (float)__builtin_amdgcn_sdot2(s, s, 0, true);
        }
    }
    return e;
}

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One tone of a row's pass-0 decision: rotation of the lane's segment state
// (s1, s2) into the window's phase, the 16-lane sums, the power and the
// running argmax (rescue_rows' pass 0, operation for operation).
__device__ __forceinline__ void seg_tone_step(const RescueParams &p, int t, int seg, double s1,
                                              double s2, double &best, double &second, double &mine,
                                              int &arg)
{
#pragma clang fp contract(off)
    const double *r = p.rot64 + 4 * (t * 16 + seg);
    double re = r[0] * s1, im = r[1] * s1;
    re = re - r[2] * s2;
    im = im - r[3] * s2;
    re = row_sum16d(re);
    im = row_sum16d(im);
    const double pk = re * re + im * im;
    if (pk > best) {
        second = best;
        best = pk;
        arg = t;
    } else if (pk > second) {
        second = pk;
    }
    if (t == seg) mine = pk;
}

// The row's margin test on its K powers (e: the lane's fp32 sum x^2); decided
// live rows write their symbol and powers. Returns "still ambiguous".
__device__ __forceinline__ bool seg_finish(const RescueParams &p, long long w, bool live, int seg,
                                           float e, double best, double second, double mine, int arg)
{
#pragma clang fp contract(off)
    const int K = p.k;
    const double cth = p.t2e64 * (double)row_sum16(e), dm = best - second;
    const bool still = !(best > 0.0) || dm * dm < cth * best || 16.0 * best < cth;
    if (live && !still) {
        if (seg == 0) p.sym[w] = (uint8_t)arg;
        if (p.mag && seg < K) p.mag[w * K + seg] = (float)mine;
    }
    return still;
}

// Row (16 lanes) decision of window w from its lane's segment state per tone
// (st(t) -> {s1, s2}) and the lane's fp32 sum x^2 e: rescue_rows' pass-0
// rotation, butterfly, argmax and margin test. Returns "still ambiguous";
// decided live rows write their symbol and powers.
template <typename St>
__device__ __forceinline__ bool seg_decide(const RescueParams &p, long long w, bool live, int seg,
                                           float e, St st)
{
    double best = -1.0, second = -1.0, mine = 0.0;
    int arg = 0;
#pragma unroll 1
    for (int t = 0; t < p.k; ++t) {
        const double2 s = st(t);
        seg_tone_step(p, t, seg, s.x, s.y, best, second, mine, arg);
    }
    return seg_finish(p, w, live, seg, e, best, second, mine, arg);
}

// Pass 0 of window w by the residue fold (plan.h fold64 = 2; the residue
// detector's plans, every tone on an integer bin b, residue rho = b mod 8):
// lane seg reads the window's samples 128 m + 8 seg + i (m, i < 8), forms per
// position i, once per window, the exact butterflies a_m = x_m + x_{m+4},
// d_m = x_m - x_{m+4} and the class values every residue needs (six exact
// integers and c u, c v in double, c = sqrt(2) / 2); per tone Y_rho = sum_m
// x_m e^{-2 pi i rho m / 8} (rho 0 / 4 real, 2 / 6 complex integers, odd rho
// d0 +- c u, +-d2 +- c v), its real and imaginary 8-step chains at the exact
// bin, the complex rotation into the window's phase and the row sums. Every
// operation as error_model.cpp first_pass_residue_rho analyses it
// (contraction off; tests/test_rescue_model64.py pass0_residue_powers
// restates it). Returns "still ambiguous"; decided live rows write their
// symbol and powers. 128 VGPRs (occupancy 4) with the class data as integers
// converted per use; as doubles (16 fewer converts per odd tone) 192.
__device__ __forceinline__ bool seg_residue_window(const RescueParams &p, long long w, bool live,
                                                   int seg)
{
#pragma clang fp contract(off)
    const int K = p.k;
    const int16_t *xs = p.pcm + w * p.hop + 8 * seg;
    u32x4q v[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) v[m] = *reinterpret_cast<const u32x4q *>(xs + 128 * m);
    auto smp = [&](int m, int i) {
        const unsigned d4[4] = {v[m].x, v[m].y, v[m].z, v[m].w};
        return (int)(short)((d4[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
    };
    // per position: its 8 samples, the lane's sum x^2 (any order: E only
    // scales the threshold, within error_model's safety factor), the exact
    // butterflies and the class values every residue's Y is formed from, in
    // double once per window (shared by the tones): Y_0 = (a0 + a2) + (a1 +
    // a3), Y_4 = (a0 + a2) - (a1 + a3), P = a0 - a2, Q = a1 - a3 (Y_2 = P -
    // i Q, Y_6 = P + i Q), d0, d2, c u, c v (u = d1 - d3, v = d1 + d3)
    const double kC = 0.70710678118654752440;
    // class values as exact integers, pair (m, m + 4) by pair (the pair's
    // samples die with it), then converted position by position
    float e = seg_energy64(v);
    int q[8][8];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int xl = smp(m, i), xh = smp(m + 4, i);
            const int am = xl + xh, dm = xl - xh;
            int *c = q[i];
            if (m == 0) {
                c[0] = am; c[1] = am; c[2] = am; c[4] = dm;
            } else if (m == 1) {
                c[0] += am; c[1] -= am; c[3] = am; c[6] = dm; c[7] = dm;
            } else if (m == 2) {
                c[0] += am; c[1] += am; c[2] -= am; c[5] = dm;
            } else {
                c[0] += am; c[1] -= am; c[3] -= am; c[6] -= dm; c[7] += dm;
            }
        }
    }
    // (e is done here: not sunk past the tone loop with the samples held)
    asm volatile("" : "+v"(e));
    // c u, c v in double (rounded once, shared by the odd residues); the
    // exact integer classes converted where a tone uses them
    double cw[8][2];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        cw[i][0] = kC * (double)q[i][6];
        cw[i][1] = kC * (double)q[i][7];
        __builtin_amdgcn_sched_barrier(0);
    }
    double best = -1.0, second = -1.0, mine = 0.0;
    int arg = 0;
#pragma unroll 1
    for (int t = 0; t < K; ++t) {
        // wave-uniform (an SGPR): the residue's branches below are uniform
        const int rho = __builtin_amdgcn_readfirstlane((int)p.rot64[66 * K + t]);
        const double c0 = p.rot64[64 * K + t];
        const bool cplx = (rho & 3) != 0;
        // opaque per tone: the odd residues' sums (d0 +- c u ...) are formed
        // per tone, not hoisted out of the tone loop (64 more VGPRs)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
#pragma unroll
            for (int c = 0; c < 6; ++c) asm volatile("" : "+v"(q[i][c]));
            asm volatile("" : "+v"(cw[i][0]), "+v"(cw[i][1]));
        }
        auto yv = [&](int i, int c) { return c < 6 ? (double)q[i][c] : cw[i][c - 6]; };
        double a1 = 0.0, a2 = 0.0, b1 = 0.0, b2 = 0.0;
        auto step = [&](double yr, double yi) {
            double sa = yr + c0 * a1;
            sa = sa - a2;
            a2 = a1;
            a1 = sa;
            double sb = yi + c0 * b1;
            sb = sb - b2;
            b2 = b1;
            b1 = sb;
        };
        // (negations are exact and rounding is sign-symmetric: -(D2 + CV) is
        // the bits of (-d2) - c v)
        auto real = [&](int qc) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                double sa = yv(i, qc) + c0 * a1;
                sa = sa - a2;
                a2 = a1;
                a1 = sa;
            }
        };
        if (rho == 0) {
            real(0);
        } else if (rho == 4) {
            real(1);
        } else if (rho == 2) {
#pragma unroll
            for (int i = 0; i < 8; ++i) step(yv(i, 2), -yv(i, 3));
        } else if (rho == 6) {
#pragma unroll
            for (int i = 0; i < 8; ++i) step(yv(i, 2), yv(i, 3));
        } else if (rho == 1) {
#pragma unroll
            for (int i = 0; i < 8; ++i) step(yv(i, 4) + yv(i, 6), -(yv(i, 5) + yv(i, 7)));
        } else if (rho == 3) {
#pragma unroll
            for (int i = 0; i < 8; ++i) step(yv(i, 4) - yv(i, 6), yv(i, 5) - yv(i, 7));
        } else if (rho == 5) {
#pragma unroll
            for (int i = 0; i < 8; ++i) step(yv(i, 4) - yv(i, 6), -(yv(i, 5) - yv(i, 7)));
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) step(yv(i, 4) + yv(i, 6), yv(i, 5) + yv(i, 7));
        }
        const double *r = p.rot64 + 4 * (t * 16 + seg);
        double re, im;
        if (cplx) {
            const double t1 = r[0] * a1 - r[1] * b1, t2 = r[2] * a2 - r[3] * b2;
            re = t1 - t2;
            const double t3 = r[0] * b1 + r[1] * a1, t4 = r[2] * b2 + r[3] * a2;
            im = t3 - t4;
        } else {
            re = r[0] * a1;
            im = r[1] * a1;
            re = re - r[2] * a2;
            im = im - r[3] * a2;
        }
        re = row_sum16d(re);
        im = row_sum16d(im);
        const double pk = re * re + im * im;
        if (pk > best) {
            second = best;
            best = pk;
            arg = t;
        } else if (pk > second) {
            second = pk;
        }
        if (t == seg) mine = pk;
    }
    return seg_finish(p, w, live, seg, e, best, second, mine, arg);
}

// MODE = p.fold64 (0: by segments, dense runs at hop 64 H; 1: by the fold;
// 2: by the residue fold), a template argument so that each form's registers
// stay in its own kernel (by segments 109 VGPRs, by the fold 85, by the
// residue fold 128)
template <int MODE>
__global__ __launch_bounds__(64 * kRescueSplit) __attribute__((amdgpu_waves_per_eu(4)))
void rescue_seg_kernel(RescueParams p)
{
#pragma clang fp contract(off)
    // per wave: its flagged windows (offsets from base), in order, and pass
    // 1's list; dense runs (MODE 0): [segment][tone] {s1, s2} and [segment]
    // fp32 sum x^2
    constexpr int kL = MODE == 0 ? kRescueChunk : kRescueChunk / kRescueSplit;
    constexpr int kD = MODE == 0 ? kSegStates : 1;
    __shared__ unsigned short idx_w[kRescueSplit][kL];
    __shared__ unsigned short left_w[kRescueSplit][kL];
    __shared__ double2 sst_w[kRescueSplit][kD];
    __shared__ float sen_w[kRescueSplit][(kD + 1) / 2];
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    unsigned short *idx = idx_w[wv], *left = left_w[wv];
    double2 *sst = sst_w[wv];
    float *sen = sen_w[wv];
    // a block per 512-window chunk, kRescueSplit waves. With dense runs (hop =
    // 64 H, H < 16) every wave scans the whole chunk (512 symbol bytes from
    // L2) and takes every S-th run; otherwise each scans and works on its own
    // 512 / S windows of it
    constexpr int S = kRescueSplit;
    const int sub = wv;
    const int H = (MODE == 0 && p.hop % 64 == 0 && p.hop < 1024) ? (int)(p.hop / 64) : 0;
    const int len = H > 0 ? kRescueChunk : kRescueChunk / S;
    const long long base = tile_block(1) * kRescueChunk + (H > 0 ? 0 : sub * len);
    if (base >= p.n_windows) return;
    const int span = (int)min((long long)len, p.n_windows - base);
    // (buffer loads bounded by span: nothing past the last window is read,
    // a last dword cut by the bound reads as 0, its bytes one by one)
    __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)(p.sym + base), (short)0, span, 0x00020000);
    unsigned any = 0;
    if (p.sym_aligned4) {
#pragma unroll 1
        for (int c = 0; 256 * c < len; ++c)
            any |= __builtin_amdgcn_raw_buffer_load_b32(rs, (64 * c + lane) * 4, 0, 0) & 0x80808080u;
        if (lane < (span & 3)) any |= __builtin_amdgcn_raw_buffer_load_b8(rs, (span & ~3) + lane, 0, 0) & 0x80u;
    } else {
#pragma unroll 1
        for (int c = 0; 64 * c < len; ++c)
            any |= __builtin_amdgcn_raw_buffer_load_b8(rs, 64 * c + lane, 0, 0) & 0x80u;
    }
    if (__ballot(any != 0) == 0) return;
    int T = 0;
    for (int i = 0; 64 * i < len; ++i) {
        const int o = 64 * i + lane;
        const bool f = o < span && (p.sym[base + o] & kSymAmbiguous);
        const unsigned long long b = __ballot(f);
        if (f) idx[T + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(b >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)b, 0u))] =
            (unsigned short)o;
        T += __popcll(b);
    }
    wave_sync();
    const int K = p.k;
    const int row = lane >> 4, seg = lane & 15;
    int Tl = 0;  // left[0 .. Tl)

    // dense runs (hop = 64 H, H < 16): runs of R windows, ((R - 1) H + 16) K
    // end states in LDS
    // (by the fold every window's pass 0 is 8 steps per lane and tone: no runs)
    int Ts = T;  // windows for the per-window pass: idx[0 .. Ts)
    if (H > 0) {
        // the run length with the most windows per lane pass of the segment
        // loop (hop 256, K = 2: 29 windows, 128 segments = 2 full passes)
        const int pairs = (K + 1) >> 1;
        int R = 1, Ri = 1;
        for (int r = 1; r <= 64 && ((r - 1) * H + 16) * K <= kSegStates; ++r) {
            const int it = (((r - 1) * H + 16) * pairs + 63) >> 6;
            if (r * Ri > R * it) {
                R = r;
                Ri = it;
            }
        }
        Ts = 0;
        int i = 0, run = 0;
#pragma unroll 1
        while (i < T) {
            const int rb = (idx[i] / R) * R;
            // (past the list: a sentinel no run reaches; rb + R may pass the
            // chunk's end when R does not divide it)
            const int my = i + lane < T ? (int)idx[i + lane] : 0x7FFFFFFF;
            const int cnt = __popcll(__ballot(lane < R && my < rb + R));
            const int nw = min(R, span - rb);
            const int segs = (nw - 1) * H + 16;
#ifdef FSKD_BOUNDS_DEBUG
            {
                int c2 = cnt, n2 = nw, t2 = T;
                RS_CHECK(c2, 65, "cnt");
                RS_CHECK(n2, 65, "nw");
                RS_CHECK(t2, kRescueChunk + 1, "T");
                if (cnt == 0) printf("RS cnt 0 at i %d T %d rb %d R %d\n", i, T, rb, R);
            }
#endif
            // run run % S is this sub-block's (the others skip it)
            if (run++ % S != sub) {
                i += cnt;
                continue;
            }
            if (cnt * 16 <= segs) {
                // sparse: to the per-window pass (Ts <= i: the read is done
                // before the write)
                if (lane < cnt) idx[Ts + lane] = (unsigned short)my;
                Ts += cnt;
                i += cnt;
                wave_sync();
                continue;
            }
            const int16_t *s0 = p.pcm + (base + rb) * p.hop;
#pragma unroll 1
            for (int it = lane; it < segs * pairs; it += 64) {
                const int pp = it / segs;
                int s = it - pp * segs;
#ifdef FSKD_BOUNDS_DEBUG
                {
                    long long smp = (base + rb) * p.hop + 64LL * s + 64;
                    RS_CHECK(smp, (p.n_windows - 1) * p.hop + 1025, "dense samples");
                    int ss = s;
                    RS_CHECK(ss, kSegStates / 2, "sen");
                    int si = s * K + 1;
                    RS_CHECK(si, kSegStates, "sst");
                }
#endif
                const u32x4q *src = reinterpret_cast<const u32x4q *>(s0 + 64 * s);
                u32x4q v[8];
#pragma unroll
                for (int q = 0; q < 8; ++q) v[q] = src[q];
                if (pp == 0) sen[s] = seg_energy64(v);
                const int t0 = 2 * pp, t1 = t0 + 1 < K ? t0 + 1 : t0;
                double a1, a2, b1, b2;
                seg_pair(v, p.rot64[64 * K + t0], p.rot64[64 * K + t1], a1, a2, b1, b2);
                // unconditional (t1 == t0: the same bits twice); under the
                // condition the compiler ran b's chain after a's, the 64
                // converted samples live in between
                sst[s * K + t0] = make_double2(a1, a2);
                sst[s * K + t1] = make_double2(b1, b2);
            }
            wave_sync();
#pragma unroll 1
            for (int j = 0; j < cnt; j += 4) {
                const bool live = j + row < cnt;
                int ii = i + (live ? j + row : j);
                RS_CHECK(ii, kRescueChunk, "idx combine");
                const int o = idx[ii];
                int sb = (o - rb) * H + seg;
                RS_CHECK(sb, segs, "sb");
                const bool still = seg_decide(p, base + o, live, seg, sen[sb],
                                              [&](int t) { return sst[sb * K + t]; });
                const unsigned long long lb = __ballot(live && still && seg == 0);
                if (live && still && seg == 0) left[Tl + __popcll(lb & ((1ull << lane) - 1))] = (unsigned short)o;
                Tl += __popcll(lb);
            }
            i += cnt;
            wave_sync();
        }
    }

    // per-window pass: rows of 16 lanes, one window each, its segments' chains
    // run by the row
#pragma unroll 1
    for (int g0 = 0; g0 < Ts; g0 += 4) {
        const bool live = g0 + row < Ts;
        const int o = idx[live ? g0 + row : g0];
        long long w = base + o;
        RS_CHECK(w, p.n_windows, "per-window w");
        bool still;
        if constexpr (MODE == 2) {
            still = seg_residue_window(p, w, live, seg);
            const unsigned long long lb = __ballot(live && still && seg == 0);
            if (live && still && seg == 0) left[Tl + __popcll(lb & ((1ull << lane) - 1))] = (unsigned short)o;
            Tl += __popcll(lb);
            continue;
        }
        if constexpr (MODE == 1) {
            // rescue_rows_fold0's arithmetic: lane seg's folded samples
            // 8 seg .. + 7 (samples 128 m + 8 seg + i, m < 8), 8-step chains
            const int16_t *xs = p.pcm + w * p.hop + 8 * seg;
            u32x4q v[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) v[m] = *reinterpret_cast<const u32x4q *>(xs + 128 * m);
            int xf[8];
            float e = seg_energy64(v);
#pragma unroll
            for (int i = 0; i < 8; ++i) xf[i] = 0;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const unsigned d4[4] = {v[m].x, v[m].y, v[m].z, v[m].w};
#pragma unroll
                for (int i = 0; i < 8; ++i) xf[i] += (int)(short)((d4[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
            }
            // the folded samples converted once (exact); the tones' chains two
            // at a time (independent chains interleaved), then each tone's
            // rotation, sums and argmax step exactly as seg_decide's
            asm volatile("" : "+v"(e));  // done here, not sunk past the tone loop
            double xd[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) xd[i] = (double)xf[i];
            double best = -1.0, second = -1.0, mine = 0.0;
            int arg = 0;
#pragma unroll 1
            for (int t0 = 0; t0 < K; t0 += 2) {
                const int t1 = t0 + 1 < K ? t0 + 1 : t0;
                const double c0 = p.rot64[64 * K + t0], c1 = p.rot64[64 * K + t1];
                double a1 = 0.0, a2 = 0.0, b1 = 0.0, b2 = 0.0;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    double sa = xd[i] + c0 * a1;
                    sa = sa - a2;
                    a2 = a1;
                    a1 = sa;
                    double sb = xd[i] + c1 * b1;
                    sb = sb - b2;
                    b2 = b1;
                    b1 = sb;
                }
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    if (h && t1 == t0) break;
                    const int t = h ? t1 : t0;
                    const double s1 = h ? b1 : a1, s2 = h ? b2 : a2;
                    seg_tone_step(p, t, seg, s1, s2, best, second, mine, arg);
                }
            }
            still = seg_finish(p, w, live, seg, e, best, second, mine, arg);
            const unsigned long long lb = __ballot(live && still && seg == 0);
            if (live && still && seg == 0) left[Tl + __popcll(lb & ((1ull << lane) - 1))] = (unsigned short)o;
            Tl += __popcll(lb);
            continue;
        }
        const u32x4q *src = reinterpret_cast<const u32x4q *>(p.pcm + w * p.hop + 64 * seg);
        u32x4q v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = src[q];
        const float e = seg_energy64(v);
        double2 sp[2];
        if (K <= 2) {
            seg_pair(v, p.rot64[64 * K], p.rot64[64 * K + K - 1], sp[0].x, sp[0].y, sp[1].x, sp[1].y);
            still = seg_decide(p, w, live, seg, e, [&](int t) { return t ? sp[1] : sp[0]; });
        } else {
            // K > 2: each tone's chain where seg_decide asks for it (one pass
            // over the samples per tone; v opaque per pass so its conversions
            // are not hoisted out of the tone loop as 64 doubles)
            still = seg_decide(p, w, live, seg, e, [&](int t) {
                const double c = p.rot64[64 * K + t];
                double2 r, u;
                seg_pair(v, c, c, r.x, r.y, u.x, u.y);
                return r;
            });
        }
        const unsigned long long lb = __ballot(live && still && seg == 0);
        if (live && still && seg == 0) left[Tl + __popcll(lb & ((1ull << lane) - 1))] = (unsigned short)o;
        Tl += __popcll(lb);
    }
    wave_sync();

    // pass 1: the exact chains of what is left, straight from L2
    const int wpw = 64 / K;
    const int f = lane / K, t = lane - (lane / K) * K;
#pragma unroll 1
    for (int g0 = 0; g0 < Tl; g0 += wpw) {
        const bool act = f < wpw && g0 + f < Tl;
        long long w = base + left[act ? g0 + f : g0];
        RS_CHECK(w, p.n_windows, "pass1 w");
        double P = 0.0;
        if (act) {
            const double c = p.coef[t];
            double s1 = 0.0, s2 = 0.0;
            const u32x4q *xs = reinterpret_cast<const u32x4q *>(p.pcm + w * p.hop);
            u32x4q nx = xs[0];
#pragma unroll 1
            for (int q = 0; q < 128; ++q) {
                const u32x4q d = nx;
                if (q + 1 < 128) nx = xs[q + 1];
                const unsigned d4[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
                for (int e2 = 0; e2 < 8; ++e2) {
                    const double x = (double)(short)((d4[e2 >> 1] >> (16 * (e2 & 1))) & 0xFFFFu);
                    double s = x + c * s1;
                    s = s - s2;
                    s2 = s1;
                    s1 = s;
                }
            }
            const double a = s1 * s1 + s2 * s2;
            const double b = c * s1;
            P = a - b * s2;
            if (p.mag) p.mag[w * K + t] = (float)P;
        }
        // the window's argmax across its K lanes (ties to the lowest tone)
        double bestx = -1.0;
        int argx = 0;
        for (int k = 0; k < K; ++k) {
            const double pk = __shfl(P, (f * K + k) & 63);
            if (pk > bestx) {
                bestx = pk;
                argx = k;
            }
        }
        if (act && t == 0) p.sym[w] = (uint8_t)argx;
    }
}

hipError_t launch_rescue(const RescueParams &p, hipStream_t s)
{
    if (p.n_windows <= 0) return hipSuccess;
    if (p.k < 2 || p.k > kMaxTones) return hipErrorInvalidValue;
    if (p.n < 64 || (p.n % 8) || 2 * p.n + 16 > kRescueLdsBytes) return hipErrorInvalidValue;
    const long long blocks = (p.n_windows + kRescueChunk - 1) / kRescueChunk;
    if (blocks > 0x7FFFFFFFLL) return hipErrorInvalidValue;
    if (p.n == 1024 && p.rot64 && p.t2e64 > 0.0)
    {
        const dim3 grid((unsigned)blocks), block(64 * kRescueSplit);
        if (p.fold64 == 2)
            hipLaunchKernelGGL(rescue_seg_kernel<2>, grid, block, 0, s, p);
        else if (p.fold64 == 1)
            hipLaunchKernelGGL(rescue_seg_kernel<1>, grid, block, 0, s, p);
        else
            hipLaunchKernelGGL(rescue_seg_kernel<0>, grid, block, 0, s, p);
    }
    else
        hipLaunchKernelGGL(rescue_kernel, dim3((unsigned)blocks), dim3(64), 0, s, p);
    return hipGetLastError();
}

}  // namespace fskd
