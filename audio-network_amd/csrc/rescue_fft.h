// rescue_fft.h — the FFT detector's decision rescue, run inside the detector
// (DESIGN.md §2a).
//
// A window whose fp32 top-2 tone margin is within the powers' error bound is
// decided again with the definition's arithmetic in double precision: the
// iterative radix-2 DIT FFT of oracle/fsk_oracle.c:oracle_fft_power
// (bit-reversed input, stages len = 2 .. 1024, w = (cos, sin)(-2 pi j / len)
// from the host's table, t = w b, b' = a - t, a' = a + t, every product and
// sum rounded on its own), P[b] = re^2 + im^2, argmax over the tone bins with
// ties to the lowest tone. Every butterfly runs on the same operands in the
// same order as the oracle's, so the rescued powers and symbol are the
// oracle's bit for bit; only where the values wait between stages differs.
//
// After its group loop, each wave reads back the symbol bytes of the groups
// it decided (fft_quad.hip, step 6) and runs this, in a wave-uniform branch,
// with all 64 lanes on one flagged window: the ten stages in three register passes of
// 16 points per lane — positions 16 l + e of the bit-reversed array (stages
// len 2 .. 16 inside the lane), then (l & 15) + 16 m + 256 (l >> 4) (len 32 ..
// 256), then l + 64 q + 256 m (len 512, 1024) — with two exchanges through
// the wave's own 1088-double LDS slab (re, then im). Flagged windows are rare
// (0.04 % of the hop-256 bench stream), so the cost spreads over the
// detector's grid: no second launch. (Round 4: a first pass by segments,
// rescue_fft_seg below, takes the tone-only batches' flagged groups first.)
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "demod_internal.h"

namespace fskd {

typedef __attribute__((address_space(3))) double lds_double;

// LDS slot of FFT position q: one pad double per 16 (1088 slots)
__device__ __forceinline__ int rfslot(int q) { return q + (q >> 4); }

__device__ __forceinline__ void rf_wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// the definition's radix-2 butterfly on (a, b) with twiddle (wr, wi)
__device__ __forceinline__ void rf_bfly(double &ar, double &ai, double &br, double &bi, double wr, double wi)
{
#pragma clang fp contract(off)
    const double tr = br * wr - bi * wi;
    const double ti = br * wi + bi * wr;
    const double xr = ar, xi = ai;
    br = xr - tr;
    bi = xi - ti;
    ar = xr + tr;
    ai = xi + ti;
}

// The same butterfly with w = (cos 0, sin 0) = (1, -0): t = b exactly (up to
// the sign of a zero), so the products are skipped. Zeros of either sign add
// and square alike, so every power stays bit-identical to the oracle's.
__device__ __forceinline__ void rf_bfly0(double &ar, double &ai, double &br, double &bi)
{
#pragma clang fp contract(off)
    const double xr = ar, xi = ai;
    ar = xr + br;
    ai = xi + bi;
    br = xr - br;
    bi = xi - bi;
}

// One window (n = 1024) at x, the whole wave. xs: the wave's LDS slab (>= 1088
// doubles, free on entry, free on return). rtw: [1023] (cos, sin), stage len
// at len / 2 - 1 + j. bins: the k tone bins. Writes the symbol, and the tone
// powers / full spectrum (rounded to fp32) where the rows are given.
__device__ __attribute__((always_inline)) inline void rescue_fft_window(const int16_t *__restrict__ x, lds_double *xs,
                                                            const double2 *__restrict__ rtw,
                                                            const int *__restrict__ bins, int k,
                                                            uint8_t *sym, float *mag, float *spec)
{
#pragma clang fp contract(off)
    const int lane = (int)__lane_id();
    const int lo = lane & 15, hi = lane >> 4;
    const int brl = (int)(__builtin_bitreverse32((unsigned)lane) >> 26);  // bitrev6(lane)
    double ar[16], ai[16];
    // pass A: position 16 l + e holds sample bitrev10(16 l + e) = 64 bitrev4(e) + bitrev6(l)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
        const int b4 = (int)(__builtin_bitreverse32((unsigned)e) >> 28);
        ar[e] = (double)x[64 * b4 + brl];
        ai[e] = 0.0;
    }
#pragma unroll
    for (int h = 1; h <= 8; h <<= 1)
#pragma unroll
        for (int e = 0; e < 16; ++e)
            if (!(e & h)) {
                if ((e & (h - 1)) == 0) {
                    rf_bfly0(ar[e], ai[e], ar[e + h], ai[e + h]);
                } else {
                    const double2 t = rtw[h - 1 + (e & (h - 1))];
                    rf_bfly(ar[e], ai[e], ar[e + h], ai[e + h], t.x, t.y);
                }
            }
    // exchange A -> B: lane l takes positions lo + 16 m + 256 hi
#pragma unroll
    for (int e = 0; e < 16; ++e) xs[rfslot(16 * lane + e)] = ar[e];
    rf_wave_sync();
#pragma unroll
    for (int m = 0; m < 16; ++m) ar[m] = xs[rfslot(lo + 16 * m + 256 * hi)];
    rf_wave_sync();
#pragma unroll
    for (int e = 0; e < 16; ++e) xs[rfslot(16 * lane + e)] = ai[e];
    rf_wave_sync();
#pragma unroll
    for (int m = 0; m < 16; ++m) ai[m] = xs[rfslot(lo + 16 * m + 256 * hi)];
    // pass B: stages len 32 .. 256 (half 16 h), j = lo + 16 (m & (h - 1))
#pragma unroll
    for (int h = 1; h <= 8; h <<= 1)
#pragma unroll
        for (int m = 0; m < 16; ++m)
            if (!(m & h)) {
                const double2 t = rtw[16 * h - 1 + lo + 16 * (m & (h - 1))];
                rf_bfly(ar[m], ai[m], ar[m + h], ai[m + h], t.x, t.y);
            }
    // exchange B -> C: lane l takes positions l + 64 q + 256 m (slot 4 q + m)
    rf_wave_sync();
#pragma unroll
    for (int m = 0; m < 16; ++m) xs[rfslot(lo + 16 * m + 256 * hi)] = ar[m];
    rf_wave_sync();
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int m = 0; m < 4; ++m) ar[4 * q + m] = xs[rfslot(lane + 64 * q + 256 * m)];
    rf_wave_sync();
#pragma unroll
    for (int m = 0; m < 16; ++m) xs[rfslot(lo + 16 * m + 256 * hi)] = ai[m];
    rf_wave_sync();
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int m = 0; m < 4; ++m) ai[4 * q + m] = xs[rfslot(lane + 64 * q + 256 * m)];
    // pass C: stage len 512 (pairs m, m + 1; j = g) and 1024 (pairs m, m + 2; j = g + 256 m)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int g = lane + 64 * q;
        const double2 t1 = rtw[255 + g], t2 = rtw[511 + g], t3 = rtw[767 + g];
        rf_bfly(ar[4 * q], ai[4 * q], ar[4 * q + 1], ai[4 * q + 1], t1.x, t1.y);
        rf_bfly(ar[4 * q + 2], ai[4 * q + 2], ar[4 * q + 3], ai[4 * q + 3], t1.x, t1.y);
        rf_bfly(ar[4 * q], ai[4 * q], ar[4 * q + 2], ai[4 * q + 2], t2.x, t2.y);
        rf_bfly(ar[4 * q + 1], ai[4 * q + 1], ar[4 * q + 3], ai[4 * q + 3], t3.x, t3.y);
    }
    // natural order now: slot 4 q + m holds bin g + 256 m. P = re^2 + im^2 for
    // bins 0 .. 512 into the slab (reads done above), the spectrum row as fp32
    rf_wave_sync();
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            const int b = lane + 64 * q + 256 * m;
            const double P = ar[4 * q + m] * ar[4 * q + m] + ai[4 * q + m] * ai[4 * q + m];
            xs[b] = P;
            if (spec) spec[b] = (float)P;
        }
    if (lane == 0) {
        const double P = ar[2] * ar[2] + ai[2] * ai[2];
        xs[512] = P;
        if (spec) spec[512] = (float)P;
    }
    rf_wave_sync();
    // argmax over the tones (ties to the lowest), as the oracle's loop
    double best = -1.0;
    int arg = 0;
    for (int i = 0; i < k; ++i) {
        const double P = xs[bins[i]];
        if (mag && lane == i) mag[i] = (float)P;
        if (P > best) {
            best = P;
            arg = i;
        }
    }
    if (lane == 0) *sym = (uint8_t)arg;
    rf_wave_sync();
}

// The FFT rescue's first pass (round 4, tones only): the
// Goertzel family's pass 0 (demod_internal.h rescue_rows) for the four
// windows of a flagged group, one per 16-lane row as the detector holds them:
// lane seg runs each tone bin's recurrence in double over its own 64 samples
// (read once from global memory / L2 into 32 VGPRs: the group loop's
// registers are dead here), rotates its end state into the window's phase
// and the row sums. The bins' sqrt powers come within rho_first sqrt(E) of the
// oracle's double FFT's (both errors, derived by error_model.cpp), so where
// their top-2 margin satisfies margin^2 >= t2e64 E P_max the row is decided
// here (symbol; tone powers rounded to fp32, within that bound of the oracle's).
// Returns the lane's row verdict: still ambiguous (for rescue_fft_window).
// x: the row's window (valid where amb_row); k tones at runtime.
// fold (every tone bin a multiple of 8; round 5): the lane reads samples
// 128 m + 8 seg .. + 7 (m < 8) instead and runs rescue_rows_fold0's 8-step
// chains over their integer sums (the window folded to 128), rot64 then
// holding the fold tables (plan.h fold64).
__device__ __forceinline__ bool rescue_fft_seg(const int16_t *__restrict__ x, const double *__restrict__ rot64,
                                               double t2e64, int k, int seg, bool amb_row, uint8_t *sym,
                                               float *mag, bool fold)
{
#pragma clang fp contract(off)
    unsigned v[32];
    const unsigned *src = reinterpret_cast<const unsigned *>(x + (fold ? 8 : 64) * seg);
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = amb_row ? src[fold ? 64 * (i >> 2) + (i & 3) : i] : 0u;
    int xf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        int a = 0;
        if (fold) {
#pragma unroll
            for (int m = 0; m < 8; ++m) a += (int)(short)((v[4 * m + (i >> 1)] >> (16 * (i & 1))) & 0xFFFFu);
        }
        xf[i] = a;
    }
    float e = 0.f;
#pragma unroll
    for (int i = 0; i < 64; ++i) {
        const float xf = (float)(short)((v[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
        e = __builtin_fmaf(xf, xf, e);
    }
    double best = -1.0, second = -1.0, mine = 0.0;
    int arg = 0;
#pragma unroll 1
    for (int t = 0; t < k; ++t) {
        const double c = rot64[64 * k + t];
        double s1 = 0.0, s2 = 0.0;
        if (fold) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                double s = (double)xf[i] + c * s1;
                s = s - s2;
                s2 = s1;
                s1 = s;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 64; ++i) {
                const double xd = (double)(short)((v[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
                double s = xd + c * s1;
                s = s - s2;
                s2 = s1;
                s1 = s;
            }
        }
        const double *r = rot64 + 4 * (t * 16 + seg);
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
    const double cth = t2e64 * (double)row_sum16(e), dm = best - second;
    const bool still = !(best > 0.0) || dm * dm < cth * best || 16.0 * best < cth;
    if (amb_row && !still) {
        if (seg == 0) *sym = (uint8_t)arg;
        if (mag && seg < k) mag[seg] = (float)mine;
    }
    return amb_row && still;
}

}  // namespace fskd
