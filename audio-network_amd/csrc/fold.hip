// fold.hip — Goertzel tone bank on the period-folded window (integer-bin tones).
//
// Identity (exact): for tone bins b_k that are all multiples of 8,
// e^{-j 2 pi b_k (n + N/8) / N} = e^{-j 2 pi b_k n / N}, so
//     X_k = sum_{n<N} x[n] W^{b_k n} = sum_{r<N/8} xf[r] W^{b_k r},
//     xf[r] = sum_{m<8} x[r + m N/8]           (integer sums, exact).
// The Goertzel recurrence then runs over the N/8 folded samples instead of N;
// P_k and the argmax are the same quantities the plain tone bank computes
// (oracle/fsk_oracle.c:goertzel_window_d), to fp32 rounding.
//
// Layout: a window of N = 64 G samples = 8 G chunks of 8 samples; lane j of
// the window's G-lane group loads chunks j + G m (m = 0..7) — per wave
// instruction each window contributes G consecutive 16-byte chunks, i.e. whole
// 128-byte lines, so the loads are coalesced without any LDS transpose —
// folds them into xf[8j .. 8j+7], runs the K recurrences over those 8 values,
// rotates into window phase (A = e^{-jw(8j+7)}, B = e^{-jw(8j+8)}) and sums
// over the group with DPP, exactly as goertzel.hip does for 64-sample segments.
// VALU per sample drops from ~(1 + 2K) to ~(1 + 2K/8 + epilogue), which makes
// 8-FSK HBM-bound.
#include "demod_internal.h"
#include "window_sum.h"

namespace fskd {

typedef unsigned int u32x4f __attribute__((ext_vector_type(4)));
typedef float f32x2f __attribute__((ext_vector_type(2)));

template <int CTRL>
__device__ __forceinline__ float dppf_(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

__device__ __forceinline__ float group_sum_f(float v, int log2g)
{
    if (log2g > 0) v += dppf_<0xB1>(v);
    if (log2g > 1) v += dppf_<0x4E>(v);
    if (log2g > 2) v += dppf_<0x141>(v);
    if (log2g > 3) v += dppf_<0x140>(v);
    if (log2g > 4) v += __shfl_xor(v, 16);
    if (log2g > 5) v += __shfl_xor(v, 32);
    return v;
}

// The energy stage 2 compares against: the folded window's, E_f = sum xf^2.
// Where it is 0 (every folded sum zero, so every fp32 tone power is too) the
// row is a candidate only if the window itself is not digital silence:
// rawfn() (called by every lane, only when some live row of the wave has E_f
// == 0) returns the raw window's sum x^2, which the P_max == 0 test of
// demod_internal.h amb_energy then reads (> 0: ambiguous). A window with
// E_f > 0 has raw energy too, so only its threshold scale matters.
// Round 5: the threshold carries the double oracle's own error too, which
// scales with the raw window (error_model.cpp): E_eff = (sqrt(E_f) + d)^2,
// d = p.amb_d in units of sqrt(E_f); a row with E_f == 0 gets d^2 (> 0: a
// candidate) unless its raw window is digital silence.
template <typename RawFn>
__device__ __forceinline__ float fold_energy(float ef, bool live, float d, RawFn rawfn)
{
    if (__ballot(live && ef == 0.f) != 0) {
        const float er = rawfn();
        if (ef == 0.f) return er > 0.f ? fmaxf(d * d, 1e-30f) : 0.f;
    }
    const float s = __builtin_amdgcn_sqrtf(ef) + d;
    return s * s;
}

// The decision of one window at n = 1024 from this lane's folded integer sums
// acc[0..7] (lane j of the window: positions 8j .. 8j + 7 of the N/8 fold,
// i.e. the even-segment half of positions 8(j & 7).. for j < 8 and the odd
// half for j >= 8): the int -> fp32 converts, the K recurrences over the 8
// folded samples, the rotation into window phase and the window_sum.h
// epilogue. F16: c16 / r hold this lane's four slots (fold_tile_kernel F16).
// fold_tile_kernel and fold_slide_kernel both end here, so a window's result
// does not depend on which of them formed its sums.
// Stage 2 of the ambiguity test uses the energy of the folded window the
// detector transforms, E = sum xf^2 over its N/8 positions (the lanes' acc;
// amb_t2e = tau^2 N/8): the fold itself is exact, so the fp32 error scales with
// the folded window, and E <= 8 sum x^2. defer: flagged rows are left to the
// kernel's rescue_rows. Returns the row's ambiguity verdict.
template <int K, bool F16, int MST = -1, typename RawFn>
__device__ __forceinline__ bool fold_decide(const int (&acc)[8], const float4 *r,
                                            const float (&c16)[4], int lane, long long w,
                                            bool live, const GoertzelParams &p, bool defer,
                                            RawFn rawfn)
{
    float xf[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) xf[q] = (float)acc[q];
    auto efn = [&]() {
        f32x2f a = {0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 8; q += 2)
            a = __builtin_elementwise_fma(f32x2f{xf[q], xf[q + 1]}, f32x2f{xf[q], xf[q + 1]}, a);
        return fold_energy(row_sum16(a.x + a.y), live, p.amb_d, rawfn);
    };
    const AmbTest at{p.amb_tq, p.amb_floor, p.amb_t2e, defer};
    if constexpr (F16) {
        const float sg = (lane & 8) ? -1.f : 1.f;
        float y[8];
#pragma unroll
        for (int q = 0; q < 8; ++q)  // lanes < 8: E + O = Z0; lanes >= 8: E - O = Z8
            y[q] = fmaf(sg, xf[q], dppf_<0x128>(xf[q]));
        float xr[4], xi[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // tone pairs in packed fp32 (2 ops per pair-sample)
            const f32x2f c2 = f32x2f{c16[2 * h], c16[2 * h + 1]};
            f32x2f a1 = f32x2f{0.f, 0.f}, a2 = f32x2f{0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const f32x2f a = __builtin_elementwise_fma(c2, a1, f32x2f{y[q], y[q]} - a2);
                a2 = a1;
                a1 = a;
            }
            // rotation as packed (re, im) pairs: X = (A s1) - (B s2), 2 ops per tone
            const f32x2f X0 = __builtin_elementwise_fma(
                f32x2f{-r[2 * h].z, -r[2 * h].w}, f32x2f{a2.x, a2.x},
                f32x2f{r[2 * h].x, r[2 * h].y} * f32x2f{a1.x, a1.x});
            const f32x2f X1 = __builtin_elementwise_fma(
                f32x2f{-r[2 * h + 1].z, -r[2 * h + 1].w}, f32x2f{a2.y, a2.y},
                f32x2f{r[2 * h + 1].x, r[2 * h + 1].y} * f32x2f{a1.y, a1.y});
            xr[2 * h] = X0.x;
            xi[2 * h] = X0.y;
            xr[2 * h + 1] = X1.x;
            xi[2 * h + 1] = X1.y;
        }
        return window_sum_decide_split8<true, MST>(xr, xi, lane, w, live, p.sym, p.mag, p.perm, at, efn);
    } else {
        float xr[K], xi[K];
        constexpr int HP = K / 2;  // packed tone pairs; an odd last tone runs scalar
#pragma unroll
        for (int h = 0; h < HP; ++h) {
            const f32x2f c2 = f32x2f{p.coef[2 * h], p.coef[2 * h + 1]};
            f32x2f a1 = f32x2f{0.f, 0.f}, a2 = f32x2f{0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const f32x2f a = __builtin_elementwise_fma(c2, a1, f32x2f{xf[q], xf[q]} - a2);
                a2 = a1;
                a1 = a;
            }
            // explicit fma: the rounding does not depend on the compiler's
            // contraction (error_model.cpp, tests/fp32emu.py)
            xr[2 * h] = fmaf(r[2 * h].x, a1.x, -(r[2 * h].z * a2.x));
            xi[2 * h] = fmaf(r[2 * h].y, a1.x, -(r[2 * h].w * a2.x));
            xr[2 * h + 1] = fmaf(r[2 * h + 1].x, a1.y, -(r[2 * h + 1].z * a2.y));
            xi[2 * h + 1] = fmaf(r[2 * h + 1].y, a1.y, -(r[2 * h + 1].w * a2.y));
        }
        if constexpr (K & 1) {
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const float a = fmaf(p.coef[K - 1], s1, xf[q] - s2);
                s2 = s1;
                s1 = a;
            }
            xr[K - 1] = fmaf(r[K - 1].x, s1, -(r[K - 1].z * s2));
            xi[K - 1] = fmaf(r[K - 1].y, s1, -(r[K - 1].w * s2));
        }
        return window_sum_decide<K, false, MST>(xr, xi, lane, w, live, p.sym, p.mag, 0, at, efn);
    }
}

//   ROTLDS: keep the per-lane rotation constants in a block LDS table instead
//           of 4K VGPRs (raises occupancy for large K).
//   NTS: non-temporal output stores.
//   LAUX: (probe) the input loads' cache-policy bits; -1: nt when NT, else plain.
//   WS: window_sum.h epilogue (reduce-scatter, packed-key argmax) at n = 1024.
//   PK: (with WS) tone pairs in packed fp32, one v_pk_add_f32 + v_pk_fma_f32
//       per pair per folded sample instead of 2 scalar instructions per tone.
//   LDST: (n = 1024) load the tile as the plain bank does, 1 KiB contiguous per
//       wave instruction, and regroup it through an 8 KiB wave-private LDS
//       slice (linear: chunk q at 16 q, conflict-free for both the 64-chunk
//       writes and the j + 16 m reads), instead of the direct per-lane
//       layout whose instructions each touch four 256-byte pieces.
//   F16: (K = 8, n = 1024, LDST) fold by 16. Tones on multiples of 16 bins
//       read Z0[r] = sum_{m<16} x[r + 64 m], tones on odd multiples of 8 read
//       Z8[r] = sum (-1)^m x[r + 64 m] (W^{64 b} = +1 / -1). Lane j < 8 of a
//       window holds the even-m half E of folded positions 8(j & 7) .. +7,
//       lane j + 8 the odd half O, so one DPP row_ror:8 gives both lanes
//       E + O (lanes < 8) and E - O (lanes >= 8); the host permutes the plan
//       so slots 0-3 are Z0 tones and 4-7 Z8 tones (4 each), and lanes < 8
//       run slots 0-3, lanes >= 8 slots 4-7: half the recurrences and
//       rotations per lane, and the first reduce-scatter stage is already done
//       (window_sum_decide_split8; perm maps slots back to the caller's tones).
template <int K, int LOG2G, bool NT = true, int WPB = 4, bool ROTLDS = false, bool NTS = false,
          bool WS = false, bool PK = false, bool LDST = false, bool F16 = false, int MST = -1,
          int LAUX = -1>
__global__ __launch_bounds__(64 * WPB) void fold_tile_kernel(GoertzelParams p)
{
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: tile bases stay in SGPRs (no waterfall loop per buffer load)
    const int log2g = LOG2G >= 0 ? LOG2G : p.log2g;
    const int g = 1 << log2g;
    const int n = 64 << log2g;
    const int j = lane & (g - 1);
    const int win_in_tile = lane >> log2g;
    const long long wins_per_tile = 64 >> log2g;
    const long long n_tiles = (p.n_windows + wins_per_tile - 1) / wins_per_tile;

    static_assert(!F16 || (K == 8 && LOG2G == 4 && LDST && WS && !ROTLDS), "F16: K = 8, n = 1024");
    float4 r[ROTLDS ? 1 : K];
    __shared__ float4 rot_lds[ROTLDS ? K * 64 : 1];
    float c16[4];
    if constexpr (F16) {
        // lane j runs slots 4 * (j >= 8) + s; rotation rows are per slot and lane
        const bool up = (lane & 8) != 0;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            c16[s4] = up ? p.coef[4 + s4] : p.coef[s4];
            r[s4] = p.rot[(s4 + (up ? 4 : 0)) * 16 + (lane & 15)];
        }
    } else if (ROTLDS) {
        for (int i = threadIdx.x; i < K * g; i += 64 * WPB) rot_lds[i] = p.rot[i];
        __syncthreads();
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = p.rot[k * g + j];
    }
    static_assert(!LDST || LOG2G == 4, "LDST regrouping is written for n = 1024");
    __shared__ __attribute__((aligned(16))) unsigned char lds_t[LDST ? WPB * 8192 : 16];
    u32x4f *wl = reinterpret_cast<u32x4f *>(lds_t + (LDST ? wave * 8192 : 0));
    int goff[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        if (LDST) {
            const int q = 64 * m + lane;  // chunk q of the tile: window q / 128, chunk q % 128
            goff[m] = (int)(((long long)(q >> 7) * p.hop + (long long)(q & 127) * 8) * 2);
        } else {
            goff[m] = (int)(((long long)win_in_tile * p.hop + (long long)(j + g * m) * 8) * 2);
        }
    }

    const long long stride = (long long)gridDim.x * WPB;
    // one tile's loads (a buffer resource clamped to the batch's bytes)
    auto load_tile = [&](long long tt, u32x4f (&v)[8]) {
        const long long wb = tt * wins_per_tile;
        long long bytes = ((p.n_windows - wb - 1) * p.hop + n) * 2;
        if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.pcm + wb * p.hop), (short)0, (int)bytes, 0x00020000);
#pragma unroll
        for (int m = 0; m < 8; ++m)
            v[m] = __builtin_amdgcn_raw_buffer_load_b128(rs, goff[m], 0, LAUX >= 0 ? LAUX : NT ? 2 : 0);
    };
    // PFN (LDST, K <= 2): the next tile's loads are issued as soon as this
    // tile is in LDS, so they are in flight during this tile's arithmetic (as
    // goertzel.hip's do_tile) when a wave takes more than one tile. With the
    // shipped one-tile-per-wave grid (tile_grid) it never issues; what it
    // changes there is the register allocation (114 VGPRs, 4 waves/SIMD,
    // instead of 84 / 5), measured 0.5 % faster at K = 2 (0.3033 vs 0.3048 ms,
    // interleaved; the plain bank 0.2967; profiles/round6/fold_k2_ab.log)
    constexpr bool PFN = LDST && K <= 2 && !F16;
    u32x4f v[8];
    const long long t_first = tile_block(p.xcd_swizzle) * WPB + wave;
    if (PFN && t_first < n_tiles) load_tile(t_first, v);
    for (long long t = t_first; t < n_tiles; t += stride) {
        const long long wbase = t * wins_per_tile;
        // the raw window's sum x^2 (fold_energy's fallback: rows whose folded
        // sums are all zero), from the tile in LDS (LDST) or L2
        auto rawfn = [&]() {
            float e;
            if constexpr (LDST) {
                e = seg_energy([&](int m) { return wl[128 * win_in_tile + 16 * m + j]; });
            } else {
                const long long w = wbase + win_in_tile;
                const int16_t *sp = p.pcm + w * p.hop + 8 * j;
                const bool live = w < p.n_windows;
                e = seg_energy_serial([&](int m) {
                    return live ? *reinterpret_cast<const u32x4f *>(sp + 8 * g * m) : u32x4f{0u, 0u, 0u, 0u};
                });
            }
            return group_sum_f(e, log2g);
        };
        if (!PFN) load_tile(t, v);
        if (LDST) {
#pragma unroll
            for (int m = 0; m < 8; ++m) wl[64 * m + lane] = v[m];
            if (PFN && t + stride < n_tiles) load_tile(t + stride, v);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        u32x4f cur[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) cur[m] = LDST ? wl[128 * win_in_tile + 16 * m + j] : v[m];
        if (LDST) {
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }

        int acc[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) acc[q] = 0;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t d4[4] = {cur[m].x, cur[m].y, cur[m].z, cur[m].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                acc[2 * q] += (int)(short)(d4[q] & 0xFFFFu);
                acc[2 * q + 1] += (int)d4[q] >> 16;
            }
        }
        if constexpr (F16 || (WS && LOG2G == 4 && !PK && !ROTLDS)) {
            const long long w = wbase + win_in_tile;
            const bool live = w < p.n_windows;
            // in-kernel decision rescue (LDST: the tile is still in the wave's
            // LDS slice, window u's chunks at 128 u ..)
            constexpr bool kInline = LDST && K >= 2;
            const bool defer = kInline && p.rescue_inline;
            const bool amb = fold_decide<K, F16, MST>(acc, r, c16, lane, w, live, p, defer, rawfn);
            if constexpr (kInline) {
                if (defer && __ballot(amb && live) != 0)
                    rescue_rows<K, (K <= kFold64MaxK) ? 1 : 0>(p, w, j, lane, amb && live, [&](int q) { return wl[128 * win_in_tile + q]; });
            }
            continue;
        }
        float xf[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) xf[q] = (float)acc[q];

        if constexpr (WS && LOG2G == 4) {
            float xr[K], xi[K];
            float t1[K], t2[K];
            constexpr int H = PK ? K / 2 : 0;  // packed tone pairs; the rest scalar
#pragma unroll
            for (int h = 0; h < H; ++h) {
                const f32x2f c2 = f32x2f{p.coef[2 * h], p.coef[2 * h + 1]};
                f32x2f a1 = f32x2f{0.f, 0.f}, a2 = f32x2f{0.f, 0.f};
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const f32x2f a = __builtin_elementwise_fma(c2, a1, f32x2f{xf[q], xf[q]} - a2);
                    a2 = a1;
                    a1 = a;
                }
                t1[2 * h] = a1.x;
                t1[2 * h + 1] = a1.y;
                t2[2 * h] = a2.x;
                t2[2 * h + 1] = a2.y;
            }
#pragma unroll
            for (int k = 2 * H; k < K; ++k) {
                float s1 = 0.f, s2 = 0.f;
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const float a = fmaf(p.coef[k], s1, xf[q] - s2);
                    s2 = s1;
                    s1 = a;
                }
                t1[k] = s1;
                t2[k] = s2;
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const float4 rk = ROTLDS ? rot_lds[k * g + j] : r[ROTLDS ? 0 : k];
                xr[k] = fmaf(rk.x, t1[k], -(rk.z * t2[k]));
                xi[k] = fmaf(rk.y, t1[k], -(rk.w * t2[k]));
            }
            const long long w = wbase + win_in_tile;
            auto efn = [&]() {
                float e = 0.f;
#pragma unroll
                for (int q = 0; q < 8; ++q) e = fmaf(xf[q], xf[q], e);
                return fold_energy(row_sum16(e), w < p.n_windows, p.amb_d, rawfn);
            };
            window_sum_decide<K, false, MST>(xr, xi, lane, w, w < p.n_windows, p.sym, p.mag, 0,
                                             AmbTest{p.amb_tq, p.amb_floor, p.amb_t2e, false}, efn);
            continue;
        }
        float P[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float s1 = 0.f, s2 = 0.f;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const float a = fmaf(p.coef[k], s1, xf[q] - s2);
                s2 = s1;
                s1 = a;
            }
            const float4 rk = ROTLDS ? rot_lds[k * g + j] : r[ROTLDS ? 0 : k];
            float re = fmaf(rk.x, s1, -(rk.z * s2));  // explicit, as fold_decide
            float im = fmaf(rk.y, s1, -(rk.w * s2));
            re = group_sum_f(re, log2g);
            im = group_sum_f(im, log2g);
            P[k] = fmaf(re, re, im * im);
        }

        const long long w = wbase + win_in_tile;
        auto efn = [&]() {
            float e = 0.f;
#pragma unroll
            for (int q = 0; q < 8; ++q) e = fmaf(xf[q], xf[q], e);
            return fold_energy(group_sum_f(e, log2g), w < p.n_windows, p.amb_d, rawfn);
        };
        bool amb;
        const int arg = chain_decide<K>(P, w < p.n_windows, p.amb_tq, p.amb_floor, p.amb_t2e, efn, amb);
        if (w < p.n_windows) {
            if (j == 0) out_store<NTS>(p.sym + w, (uint8_t)(arg | (amb ? kSymAmbiguous : 0)));
            if (p.mag) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if ((k & (g - 1)) == j) out_store<NTS>(p.mag + w * K + k, P[k]);
            }
        }
    }
    wb_burst(p.wb_bursts);
}

// acc (lo, hi) += the sign-extended int16 halves of n, minus those of o: four
// SDWA integer ops (the extraction is the operand select; hipcc reaches the
// same count from C here, but not for the first window's sums in
// fold_slide_kernel, where it built bfe / ashr extracts plus v_add3: 9 more
// VALU per tile).
__device__ __forceinline__ void slide_add_sub(int &lo, int &hi, uint32_t n, uint32_t o)
{
    asm("v_add_u32_sdwa %0, sext(%2), %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD\n\t"
        "v_add_u32_sdwa %1, sext(%2), %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD\n\t"
        "v_sub_u32_sdwa %0, %0, sext(%3) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0\n\t"
        "v_sub_u32_sdwa %1, %1, sext(%3) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
        : "+v"(lo), "+v"(hi)
        : "v"(n), "v"(o));
}
// acc (lo, hi) += the sign-extended int16 halves of n (two SDWA adds)
__device__ __forceinline__ void slide_add(int &lo, int &hi, uint32_t n)
{
    asm("v_add_u32_sdwa %0, sext(%2), %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD\n\t"
        "v_add_u32_sdwa %1, sext(%2), %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
        : "+v"(lo), "+v"(hi)
        : "v"(n));
}

// Overlapping windows (n = 1024, hop = 64 H < n) for fold-eligible plans:
// the folded sums of a window are sums of its 64-sample segments. With
// seg_s the segments of the stream and window u starting at segment uH,
// lane j of the window holds (fold_tile_kernel's LDST layout)
//     E_u = sum_{m even < 16} seg_{uH + m}   (j < 8)
//     O_u = sum_{m odd  < 16} seg_{uH + m}   (j >= 8)
// over positions 8 (j & 7) .. + 7. The window H segments later shares all but
// H of them: with pp = (parity + H) mod 2, the lane's sums of window u are
// the previous window's parity-pp sums minus its parity-pp segments m < H and
// plus its parity-pp segments 16 <= m < 16 + H (for odd H the E and O roles
// swap between the lane and its partner j ^ 8: one DPP row_ror:8). Integer
// sums, so every window's sums equal direct folding bit for bit, and the
// decision is the same fold_decide: the output is bit-identical to
// fold_tile_kernel on that window alone. Per window a lane reads H segment
// chunks instead of 8 (hop 256: 32 instead of 64 integer adds) and the tile
// streams from HBM once, where the direct kernel re-reads every window.
//   Tile: Wt = 4 R windows (p.slide_wt; host: the largest R whose
//   16 + (4R - 1) H segments fit kFoldSlideSegs = 80, i.e. 10 KiB), loaded
//   contiguously (16 B/lane, 10 instructions) into a wave-private LDS slice
//   (chunk c of segment s at 16 (8 s + c)); each 16-lane group takes R
//   consecutive windows, running the sums forward from its first. Every
//   group has R windows, so no pass of the epilogue idles (a 64-segment tile
//   at hop 256 holds 13 windows: 4 passes for 13).
template <int K, bool F16>
__global__ __launch_bounds__(64 * kPlainWPB) void fold_slide_kernel(GoertzelParams p)
{
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = lane & 15;
    const int par = j >> 3;      // 0: even segments of the window, 1: odd
    const int chunk = j & 7;     // positions 8 chunk .. + 7 of a segment
    const int H = (int)(p.hop >> 6);
    const int wt = p.slide_wt;
    const int R = wt >> 2;
    const int u0 = (lane >> 4) * R;
    const long long n_tiles = (p.n_windows + wt - 1) / wt;

    float4 r[K];
    float c16[4];
    if constexpr (F16) {
        const bool up = (lane & 8) != 0;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
            c16[s4] = up ? p.coef[4 + s4] : p.coef[s4];
            r[s4] = p.rot[(s4 + (up ? 4 : 0)) * 16 + j];
        }
    } else {
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = p.rot[k * 16 + j];
    }
    constexpr int kChunks = kFoldSlideSegs * 8;  // 16-byte chunks per tile
    __shared__ __attribute__((aligned(16))) u32x4f lds_s[kPlainWPB * kChunks];
    u32x4f *wl = lds_s + wave * kChunks;

    const long long stride = (long long)gridDim.x * kPlainWPB;
    for (long long t = tile_block(p.xcd_swizzle) * kPlainWPB + wave; t < n_tiles; t += stride) {
        const long long wbase = t * wt;
        long long bytes = ((p.n_windows - wbase - 1) * p.hop + 1024) * 2;
        if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.pcm + wbase * p.hop), (short)0, (int)bytes, 0x00020000);
        u32x4f v[kChunks / 64];
#pragma unroll
        for (int i = 0; i < kChunks / 64; ++i)  // cached: neighbouring tiles share their edge segments
            v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, (64 * i + lane) * 16, 0, 0);
#pragma unroll
        for (int i = 0; i < kChunks / 64; ++i) wl[64 * i + lane] = v[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        int acc[8];
        for (int i = 0; i < R; ++i) {
            const int u = u0 + i;
            if (i == 0) {
#pragma unroll
                for (int q = 0; q < 8; ++q) acc[q] = 0;
#pragma unroll
                for (int m2 = 0; m2 < 8; ++m2) {
                    const u32x4f d = wl[8 * (u * H + 2 * m2 + par) + chunk];
                    const uint32_t d4[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) slide_add(acc[2 * q], acc[2 * q + 1], d4[q]);
                }
            } else {
                if (H & 1) {
#pragma unroll
                    for (int q = 0; q < 8; ++q)
                        acc[q] = __builtin_amdgcn_mov_dpp(acc[q], 0x128, 0xF, 0xF, true);
                }
                const int pp = (par + H) & 1;
                const int base = (u - 1) * H;
                for (int m2 = 0; 2 * m2 < H; ++m2) {
                    const int mm = 2 * m2 + pp;
                    if (mm < H) {
                        const u32x4f o = wl[8 * (base + mm) + chunk];
                        const u32x4f nw = wl[8 * (base + 16 + mm) + chunk];
                        const uint32_t o4[4] = {o.x, o.y, o.z, o.w};
                        const uint32_t n4[4] = {nw.x, nw.y, nw.z, nw.w};
#pragma unroll
                        for (int q = 0; q < 4; ++q) slide_add_sub(acc[2 * q], acc[2 * q + 1], n4[q], o4[q]);
                    }
                }
            }
            const long long w = wbase + u;
            // the raw window's sum x^2 (fold_energy's fallback): segment j of
            // window u from the tile in LDS
            auto rawfn = [&]() {
                return row_sum16(seg_energy([&](int c) { return wl[8 * (u * H + j) + c]; }));
            };
            fold_decide<K, F16>(acc, r, c16, lane, w, w < p.n_windows, p, false, rawfn);
        }
        // the next tile's samples overwrite this one's
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

template <int K, bool NT>
static const void *fold_kernel_for_t(int log2g, bool f16)
{
    if constexpr (K == 8)
        if (log2g == 4 && f16)
            return reinterpret_cast<const void *>(
                &fold_tile_kernel<8, 4, NT, kPlainWPB, false, false, true, false, true, true>);
    // n = 1024: window_sum.h epilogue (K = 8: 352 -> 347 us, K = 2: 335 -> 329 us)
    // and LDS regrouping of contiguous loads (K = 8: 345.8 -> 339.9 us, K = 2:
    // 338.5 -> 319.9 us; profiles/round1/probe_ldst.log)
    if (log2g == 4)
        return reinterpret_cast<const void *>(
            &fold_tile_kernel<K, 4, NT, kPlainWPB, false, false, true, false, true>);
    return reinterpret_cast<const void *>(&fold_tile_kernel<K, -1, NT, kPlainWPB>);
}

// nt: hop = n (each byte read once); overlapping windows keep their lines in L2
template <int K>
static const void *fold_kernel_for(int log2g, bool f16, bool nt)
{
    return nt ? fold_kernel_for_t<K, true>(log2g, f16) : fold_kernel_for_t<K, false>(log2g, f16);
}

template <int K>
static const void *fold_slide_kernel_for(bool f16)
{
    if constexpr (K == 8)
        if (f16) return reinterpret_cast<const void *>(&fold_slide_kernel<8, true>);
    return reinterpret_cast<const void *>(&fold_slide_kernel<K, false>);
}

const void *fold_kernel_ptr(int k, int log2g, bool f16, bool nt, bool slide)
{
    if (slide && log2g != 4) return nullptr;
    switch (k) {
#define FSKD_CASE(K) case K: return slide ? fold_slide_kernel_for<K>(f16) : fold_kernel_for<K>(log2g, f16, nt);
        FSKD_CASE(1) FSKD_CASE(2) FSKD_CASE(3) FSKD_CASE(4)
        FSKD_CASE(5) FSKD_CASE(6) FSKD_CASE(7) FSKD_CASE(8)
        FSKD_CASE(9) FSKD_CASE(10) FSKD_CASE(11) FSKD_CASE(12)
        FSKD_CASE(13) FSKD_CASE(14) FSKD_CASE(15) FSKD_CASE(16)
#undef FSKD_CASE
    default: return nullptr;
    }
}

}  // namespace fskd
