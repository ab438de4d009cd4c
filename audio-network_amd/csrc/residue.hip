// residue.hip — Goertzel tone bank on the window folded per residue class
// mod 8: any tone plan whose tones sit on integer bins (the usual FSK choice:
// integer bins are what makes the tones orthogonal over a window).
//
// Identity (exact): with P = N/8, r < P and m < 8, a tone on integer bin
// b = 8 beta + rho has
//     W^{b (r + m P)} = W^{b r} e^{-j 2 pi rho m / 8},
// so
//     X_b = sum_{r<P} W^{b r} Z_rho[r],   Z_rho[r] = sum_{m<8} x[r + m P] w8^{rho m},
// i.e. Z_rho is bin rho of an 8-point DFT over the eight samples spaced P
// apart. For real x, Z_{8-rho} = conj Z_rho, so four classes cover all eight
// residues:
//     class 0: (Z0, Z4)       both real, carried as one pair
//     class 1: Z1             (rho 7 = conj)
//     class 2: Z3             (rho 5 = conj)
//     class 3: (e1, e3) = Z6  (rho 2 = conj)
// fold.hip is the rho = 0 special case (every tone a multiple of 8 bins). The
// Goertzel recurrence s = z + c s1 - s2 is linear with a real coefficient, so
// it runs on the complex z as one packed fp32 pair (re, im) per tone, over 8
// folded samples per lane instead of 64 raw ones. The class a tone reads is a
// run-time uniform value: the four class pairs of each folded sample go
// through a wave-private LDS slice and each tone reads its class at a uniform
// offset (an SGPR-indexed register file; no per-tone branches, so the K
// chains stay interleaved). The conjugation, and for class 0 the choice of
// Z0 or Z4, is folded into the per-lane rotation constants on the host:
//     X = s1.lo C1 + s1.hi C2 + s2.lo C3 + s2.hi C4   (C* complex, demod_api.cpp).
//
// Oracle: the same quantities as oracle/fsk_oracle.c:goertzel_window_d (the
// plain sequential recurrence over all N samples), to fp32 rounding; the
// 8-point butterflies are exact integer sums in fp32 except the two products
// by 1/sqrt 2.
//
// Layout: as fold.hip — lane j of a window's G-lane group loads chunks
// j + G m (m = 0..7), whole 128-byte lines per wave instruction, so folded
// samples r = 8j .. 8j+7 of all eight spacings m arrive in the lane that
// folds them. VALU per sample ~ 2.3 for the butterflies + K/4 for the
// recurrences (vs ~ 1 + K for the plain bank), so K = 8 stays HBM-bound.
#include "demod_internal.h"
#include "window_sum.h"

namespace fskd {

typedef unsigned int u32x4r __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

template <int CTRL>
__device__ __forceinline__ float dppr_(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

__device__ __forceinline__ float group_sum_r(float v, int log2g)
{
    if (log2g > 0) v += dppr_<0xB1>(v);
    if (log2g > 1) v += dppr_<0x4E>(v);
    if (log2g > 2) v += dppr_<0x141>(v);
    if (log2g > 3) v += dppr_<0x140>(v);
    if (log2g > 4) v += __shfl_xor(v, 16);
    if (log2g > 5) v += __shfl_xor(v, 32);
    return v;
}

// Class pairs of one folded sample from its eight spaced samples x[m].
//   a_m = x_m + x_{m+4}, d_m = x_m - x_{m+4}           (m < 4)
//   e0 = a0 + a2, e1 = a0 - a2, e2 = a1 + a3, e3 = a1 - a3
//   Z0 = e0 + e2, Z4 = e0 - e2, Z2 = e1 - j e3 (class 3 stores (e1, e3) = Z6)
//   u = d1 - d3, v = d1 + d3
//   Z1 = (d0 + u/sqrt2) - j (d2 + v/sqrt2),  Z3 = (d0 - u/sqrt2) + j (d2 - v/sqrt2)
__device__ __forceinline__ void residue_classes(const float x[8], f2 &z04, f2 &z1, f2 &z3, f2 &z6)
{
    const float kr = 0.70710678118654752f;
    const f2 a02 = f2{x[0], x[2]} + f2{x[4], x[6]};
    const f2 d02 = f2{x[0], x[2]} - f2{x[4], x[6]};
    const f2 a13 = f2{x[1], x[3]} + f2{x[5], x[7]};
    const f2 d13 = f2{x[1], x[3]} - f2{x[5], x[7]};
    const f2 e01 = f2{a02.x, a02.x} + f2{a02.y, -a02.y};
    const f2 e23 = f2{a13.x, a13.x} + f2{a13.y, -a13.y};
    z04 = f2{e01.x, e01.x} + f2{e23.x, -e23.x};
    z6 = f2{e01.y, e23.y};
    const f2 uv = f2{d13.x, d13.x} + f2{-d13.y, d13.y};
    z1 = __builtin_elementwise_fma(uv, f2{kr, -kr}, f2{d02.x, -d02.y});
    z3 = __builtin_elementwise_fma(uv, f2{-kr, -kr}, d02);
}

// The same butterflies as one asm block with the op_sel / neg modifiers
// spelled out: hipcc builds per-half negations and half swaps from v_xor +
// v_mov. Inputs are the pairs (x0, x2), (x4, x6), (x1, x3), (x5, x7); kk =
// (1/sqrt2, 1/sqrt2). The sums are formed in place ((a0, a2) -> (e0, e1),
// (a1, a3) -> (e2, e3), (d1, d3) -> (u, v)) to keep the register footprint at
// 4 scratch pairs, and every packed result is read no earlier than two
// instructions after it is written (gfx950 needs one wait state after a
// packed-fp32 write), so the block needs no s_nop.
__device__ __forceinline__ void residue_classes_asm(f2 p02, f2 p46, f2 p13, f2 p57, f2 kk,
                                                   f2 &z04, f2 &z1, f2 &z3, f2 &z6)
{
    f2 t02, d02, t13, t_d13;
    asm("v_pk_add_f32 %[t02], %[p02], %[p46]\n\t"                                    // (a0, a2)
        "v_pk_add_f32 %[d02], %[p02], %[p46] neg_lo:[0,1] neg_hi:[0,1]\n\t"          // (d0, d2)
        "v_pk_add_f32 %[t13], %[p13], %[p57]\n\t"                                    // (a1, a3)
        "v_pk_add_f32 %[d13], %[p13], %[p57] neg_lo:[0,1] neg_hi:[0,1]\n\t"          // (d1, d3)
        "v_pk_add_f32 %[t02], %[t02], %[t02] op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]\n\t"  // (e0, e1)
        "v_pk_add_f32 %[t13], %[t13], %[t13] op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]\n\t"  // (e2, e3)
        "v_pk_add_f32 %[d13], %[d13], %[d13] op_sel:[0,1] op_sel_hi:[0,1] neg_lo:[0,1]\n\t"  // (u, v)
        "v_pk_add_f32 %[z04], %[t02], %[t13] op_sel_hi:[0,0] neg_hi:[0,1]\n\t"       // (Z0, Z4)
        "v_pk_mov_b32 %[z6], %[t02], %[t13] op_sel:[1,1]\n\t"                         // (e1, e3)
        "v_pk_fma_f32 %[z1], %[d13], %[kk], %[d02] neg_hi:[0,1,1]\n\t"               // Z1
        "v_pk_fma_f32 %[z3], %[d13], %[kk], %[d02] neg_lo:[0,1,0] neg_hi:[0,1,0]"       // Z3
        : [t02] "=&v"(t02), [d02] "=&v"(d02), [t13] "=&v"(t13), [d13] "=&v"(t_d13),
          [z04] "=v"(z04), [z1] "=v"(z1), [z3] "=v"(z3), [z6] "=v"(z6)
        : [p02] "v"(p02), [p46] "v"(p46), [p13] "v"(p13), [p57] "v"(p57), [kk] "s"(kk));
}

// Only classes 0 and / or 3 (every tone bin even: residues 0, 2, 4, 6), for
// two folded samples at once (e = 0, 1 interleaved, so every packed result
// is read two or more instructions after it is written): 5 packed ops per
// sample for one class, 6 for both, against 11 for all four (the odd
// residues' d terms and 1/sqrt2 products are not formed).
//   Z03 = 2: (Z0, Z4) and (e1, e3);  1: (Z0, Z4) only;  3: (e1, e3) only.
template <int Z03>
__device__ __forceinline__ void residue_even_classes_asm(const f2 (&p02)[2], const f2 (&p46)[2],
                                                         const f2 (&p13)[2], const f2 (&p57)[2],
                                                         f2 (&z04)[2], f2 (&z6)[2])
{
    f2 a0, b0, a1, b1;
    asm("v_pk_add_f32 %[a0], %[p02a], %[p46a]\n\t"                                    // (a0, a2)
        "v_pk_add_f32 %[b0], %[p13a], %[p57a]\n\t"                                    // (a1, a3)
        "v_pk_add_f32 %[a1], %[p02b], %[p46b]\n\t"
        "v_pk_add_f32 %[b1], %[p13b], %[p57b]\n\t"
        "v_pk_add_f32 %[a0], %[a0], %[a0] op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]\n\t"  // (e0, e1)
        "v_pk_add_f32 %[b0], %[b0], %[b0] op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]\n\t"  // (e2, e3)
        "v_pk_add_f32 %[a1], %[a1], %[a1] op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %[b1], %[b1], %[b1] op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]"
        : [a0] "=&v"(a0), [b0] "=&v"(b0), [a1] "=&v"(a1), [b1] "=&v"(b1)
        : [p02a] "v"(p02[0]), [p46a] "v"(p46[0]), [p13a] "v"(p13[0]), [p57a] "v"(p57[0]),
          [p02b] "v"(p02[1]), [p46b] "v"(p46[1]), [p13b] "v"(p13[1]), [p57b] "v"(p57[1]));
    if constexpr (Z03 != 3)
        asm("v_pk_add_f32 %[z0], %[a0], %[b0] op_sel_hi:[0,0] neg_hi:[0,1]\n\t"      // (Z0, Z4)
            "v_pk_add_f32 %[z1], %[a1], %[b1] op_sel_hi:[0,0] neg_hi:[0,1]"
            : [z0] "=&v"(z04[0]), [z1] "=v"(z04[1])
            : [a0] "v"(a0), [b0] "v"(b0), [a1] "v"(a1), [b1] "v"(b1));
    if constexpr (Z03 != 1)
        asm("v_pk_mov_b32 %[z0], %[a0], %[b0] op_sel:[1,1]\n\t"                      // (e1, e3)
            "v_pk_mov_b32 %[z1], %[a1], %[b1] op_sel:[1,1]"
            : [z0] "=&v"(z6[0]), [z1] "=v"(z6[1])
            : [a0] "v"(a0), [b0] "v"(b0), [a1] "v"(a1), [b1] "v"(b1));
}

// Dynamic LDS: [K][G][2] float4 rotation constants (block), then per wave
// [4 classes][QP sample pairs][64 lanes] float4 (4 QP KiB).
constexpr int kResidueQP = 2;  // shipped: two sample pairs per LDS round

// Tunables (defaults = shipped, chosen with scripts/probe.hip, in git history at 8b49018):
//   ASM   butterflies as residue_classes_asm (else the plain-C residue_classes),
//   ROTV  rotation constants in VGPRs (8 per tone) instead of the LDS table,
//   MINW  > 0: ask for MINW waves per SIMD (VGPR budget 512 / MINW),
//   QP    sample pairs per LDS round (1, 2 or 4): 4 QP KiB of LDS per wave,
//   PF    prefetch the wave's next tile before computing the current one
//         (only matters on grids with more than one tile per wave),
//   WS    window_sum.h epilogue (reduce-scatter, packed-key argmax) at n = 1024,
//   LDST  (n = 1024, QP = 2) load the tile 1 KiB contiguous per wave
//         instruction, as the plain bank does, and regroup it through the
//         wave's LDS slice (linear chunk q at 16 q; the class pairs reuse the
//         slice afterwards) instead of the direct per-lane layout.
//   DC    compile-time classes: tone slot k reads its class straight from
//         registers (no LDS class file), for plans the host has permuted
//         into a fixed slot -> class pattern (window_sum maps slots back):
//         1 = class (k / 2) % 4 (K / 4 tones per class: every residue once at
//         K = 8, e.g. any odd bin spacing); 2 = slots < K / 2 class 0, the
//         rest class 3 (even bins, half on residues 0 / 4 and half on 2 / 6:
//         spacings 2 and 6); 3 = every slot class 0 (residues 0 / 4 only,
//         e.g. spacing 4 or 12 from an odd multiple of 4); 4 = every slot
//         class 3 (residues 2 / 6). Modes 2-4 form only the classes they read
//         (residue_even_classes_asm). 0 = the LDS class file (any plan).
template <int K, int LOG2G, int WPB = kWavesPerBlock, bool ASM = true, bool ROTV = false,
          int MINW = (K <= 8 ? 4 : 0), int QP = kResidueQP, bool PF = false, bool WS = true,
          bool LDST = false, int DC = 0, bool NT = true>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MINW > 0 ? MINW : 1)))
void residue_tile_kernel(GoertzelParams p)
{
    constexpr bool DCLS = DC > 0;
    extern __shared__ f4 lds_r[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int log2g = LOG2G >= 0 ? LOG2G : p.log2g;
    const int g = 1 << log2g;
    const int n = 64 << log2g;
    const int j = lane & (g - 1);
    const int win_in_tile = lane >> log2g;
    const long long wins_per_tile = 64 >> log2g;
    const long long n_tiles = (p.n_windows + wins_per_tile - 1) / wins_per_tile;

    f4 *rot = lds_r;
    f4 *zw = lds_r + K * g * 2 + wave * (4 * QP * 64) + lane;
    const f4 *grot = reinterpret_cast<const f4 *>(p.rot);
    static_assert(!LDST || (LOG2G == 4 && QP == 2), "LDST regrouping: n = 1024, 8 KiB slice");
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
    auto load_tile = [&](long long tt, u32x4r v[8]) {
        const long long wbase = tt * wins_per_tile;
        long long bytes = ((p.n_windows - wbase - 1) * p.hop + n) * 2;
        if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.pcm + wbase * p.hop), (short)0, (int)bytes, 0x00020000);
#pragma unroll
        for (int m = 0; m < 8; ++m)
            v[m] = __builtin_amdgcn_raw_buffer_load_b128(rs, goff[m], 0, NT ? 2 : 0);
    };

    const long long stride = (long long)gridDim.x * WPB;
    long long t = tile_block(p.xcd_swizzle) * WPB + wave;
    // The first tile's loads go out before the rotation table is staged and
    // the block barrier, so the two latencies overlap: with one tile per wave
    // (the usual grid) this prologue is on every wave's critical path.
    u32x4r v[8];
    if (t < n_tiles) load_tile(t, v);
    f4 rv[ROTV ? 2 * K : 1];
    if (ROTV) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            rv[2 * k] = grot[(k * g + j) * 2];
            rv[2 * k + 1] = grot[(k * g + j) * 2 + 1];
        }
    } else {
        for (int i = threadIdx.x; i < K * g * 2; i += 64 * WPB) rot[i] = grot[i];
        __syncthreads();
    }
    const f2 kk = f2{0.70710678118654752f, 0.70710678118654752f};

    for (bool first = true; t < n_tiles; t += stride, first = false) {
        const long long wbase = t * wins_per_tile;
        u32x4r cur[8];
        if (PF) {
#pragma unroll
            for (int m = 0; m < 8; ++m) cur[m] = v[m];
            if (t + stride < n_tiles) load_tile(t + stride, v);
        } else {
            if (!first) load_tile(t, v);
#pragma unroll
            for (int m = 0; m < 8; ++m) cur[m] = v[m];
        }
        if (LDST) {
            u32x4r *wl = reinterpret_cast<u32x4r *>(zw - lane);  // the wave's 8 KiB slice
#pragma unroll
            for (int m = 0; m < 8; ++m) wl[64 * m + lane] = cur[m];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int m = 0; m < 8; ++m) cur[m] = wl[128 * win_in_tile + 16 * m + j];
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }

        f2 s1[K], s2[K];
#pragma unroll
        for (int k = 0; k < K; ++k) { s1[k] = f2{0.f, 0.f}; s2[k] = f2{0.f, 0.f}; }

        // 4 / QP rounds of 2 QP folded samples: classes -> LDS, then every
        // tone advances 2 QP steps reading its class
#pragma unroll
        for (int h = 0; h < 4 / QP; ++h) {
#pragma unroll
            for (int qp = 0; qp < QP; ++qp) {
                const int d = QP * h + qp;  // dword d of each chunk = samples 2d, 2d+1
                f2 c[2][4];
                float x[2][8];
#pragma unroll
                for (int e = 0; e < 2; ++e)
#pragma unroll
                    for (int m = 0; m < 8; ++m) {
                        const uint32_t w = cur[m][d];
                        x[e][m] = e ? (float)((int)w >> 16) : (float)(int)(short)(w & 0xFFFFu);
                    }
                if constexpr (DC >= 2) {
                    const f2 p02[2] = {f2{x[0][0], x[0][2]}, f2{x[1][0], x[1][2]}};
                    const f2 p46[2] = {f2{x[0][4], x[0][6]}, f2{x[1][4], x[1][6]}};
                    const f2 p13[2] = {f2{x[0][1], x[0][3]}, f2{x[1][1], x[1][3]}};
                    const f2 p57[2] = {f2{x[0][5], x[0][7]}, f2{x[1][5], x[1][7]}};
                    f2 z04[2], z6[2];
                    residue_even_classes_asm<DC == 2 ? 2 : DC == 3 ? 1 : 3>(p02, p46, p13, p57, z04, z6);
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        if constexpr (DC != 4) c[e][0] = z04[e];
                        if constexpr (DC != 3) c[e][3] = z6[e];
                    }
                } else if (ASM) {
#pragma unroll
                    for (int e = 0; e < 2; ++e)
                        residue_classes_asm(f2{x[e][0], x[e][2]}, f2{x[e][4], x[e][6]},
                                            f2{x[e][1], x[e][3]}, f2{x[e][5], x[e][7]}, kk,
                                            c[e][0], c[e][1], c[e][2], c[e][3]);
                } else {
                    residue_classes(x[0], c[0][0], c[0][1], c[0][2], c[0][3]);
                    residue_classes(x[1], c[1][0], c[1][1], c[1][2], c[1][3]);
                }
                if constexpr (DCLS) {
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const int cl = DC == 1 ? (k / 2) % 4 : DC == 2 ? (k < K / 2 ? 0 : 3)
                                     : DC == 3 ? 0 : 3;
                        const f2 cc = f2{p.coef[k], p.coef[k]};
                        f2 a = __builtin_elementwise_fma(cc, s1[k], c[0][cl] - s2[k]);
                        s2[k] = s1[k];
                        s1[k] = a;
                        a = __builtin_elementwise_fma(cc, s1[k], c[1][cl] - s2[k]);
                        s2[k] = s1[k];
                        s1[k] = a;
                    }
                    continue;
                }
#pragma unroll
                for (int cl = 0; cl < 4; ++cl)
                    zw[(cl * QP + qp) * 64] = f4{c[0][cl].x, c[0][cl].y, c[1][cl].x, c[1][cl].y};
            }
            if (DCLS) continue;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const f4 *zk = zw + p.zcls[k] * (QP * 64);
                const f2 cc = f2{p.coef[k], p.coef[k]};
#pragma unroll
                for (int qp = 0; qp < QP; ++qp) {
                    const f4 z = zk[qp * 64];
                    f2 a = __builtin_elementwise_fma(cc, s1[k], f2{z.x, z.y} - s2[k]);
                    s2[k] = s1[k];
                    s1[k] = a;
                    a = __builtin_elementwise_fma(cc, s1[k], f2{z.z, z.w} - s2[k]);
                    s2[k] = s1[k];
                    s1[k] = a;
                }
            }
        }

        float xr[K], xi[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const f4 c12 = ROTV ? rv[2 * k] : rot[(k * g + j) * 2];
            const f4 c34 = ROTV ? rv[2 * k + 1] : rot[(k * g + j) * 2 + 1];
            f2 X = f2{c12.x, c12.y} * s1[k].x;
            X = __builtin_elementwise_fma(f2{c12.z, c12.w}, f2{s1[k].y, s1[k].y}, X);
            X = __builtin_elementwise_fma(f2{c34.x, c34.y}, f2{s2[k].x, s2[k].x}, X);
            X = __builtin_elementwise_fma(f2{c34.z, c34.w}, f2{s2[k].y, s2[k].y}, X);
            xr[k] = X.x;
            xi[k] = X.y;
        }
        const long long w = wbase + win_in_tile;
        const bool live = w < p.n_windows;
        if constexpr (WS && LOG2G == 4) {
            // Stage 2 of the ambiguity test and the in-kernel rescue both need
            // the raw samples, which only lived in registers: the tile is read
            // again (L2 / HBM), only by waves with a stage-1 flag, into the
            // wave's LDS slice (the class file is dead by now) in the linear
            // layout (window u's chunks at 128 u ..); lane j of a row sums
            // chunks 8 j .. 8 j + 7 of its window.
            u32x4r *wl = reinterpret_cast<u32x4r *>(zw - lane);
            auto efn = [&]() {
                long long bytes = ((p.n_windows - wbase - 1) * p.hop + n) * 2;
                if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
                __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    (void *)(p.pcm + wbase * p.hop), (short)0, (int)bytes, 0x00020000);
                u32x4r v2[8];
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const int q = 64 * m + lane;
                    v2[m] = __builtin_amdgcn_raw_buffer_load_b128(
                        rs, (int)(((long long)(q >> 7) * p.hop + (long long)(q & 127) * 8) * 2), 0, 0);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int m = 0; m < 8; ++m) wl[64 * m + lane] = v2[m];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                return row_sum16(seg_energy([&](int i) { return wl[128 * win_in_tile + 8 * j + i]; }));
            };
            const bool defer = K >= 2 && p.rescue_inline;
            const bool amb = window_sum_decide<K, DCLS>(xr, xi, lane, w, live, p.sym, p.mag, p.perm,
                                                        AmbTest{p.amb_tq, p.amb_floor, p.amb_t2e, defer},
                                                        efn);
            if constexpr (K >= 2) {
                if (defer && __ballot(amb && live) != 0)
                    rescue_rows<K>(p, w, j, lane, amb && live, [&](int q) { return wl[128 * win_in_tile + q]; });
            }
            // the next tile's class file overwrites the slice
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        static_assert(!DCLS || (WS && LOG2G == 4), "DCLS un-permutes in the window_sum epilogue");
        float P[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const float re = group_sum_r(xr[k], log2g);
            const float im = group_sum_r(xi[k], log2g);
            P[k] = fmaf(re, re, im * im);
        }
        // stage 2: the lane's chunks again (L2 / HBM), only on flagged waves
        auto efn = [&]() {
            u32x4r v2[8];
            load_tile(t, v2);
            return group_sum_r(seg_energy([&](int i) { return v2[i]; }), log2g);
        };
        bool amb;
        const int arg = chain_decide<K>(P, live, p.amb_tq, p.amb_floor, p.amb_t2e, efn, amb);
        if (live) {
            if (j == 0) p.sym[w] = (uint8_t)(arg | (amb ? kSymAmbiguous : 0));
            if (p.mag) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if ((k & (g - 1)) == j) p.mag[w * K + k] = P[k];
            }
        }
    }
    wb_burst(p.wb_bursts);
}

size_t residue_lds_bytes(int k, int log2g, int qp)
{
    return ((size_t)k * (1u << log2g) * 2 + (size_t)kWavesPerBlock * 4 * qp * 64) * sizeof(f4);
}

// DC (K = 8, 16 at n = 1024, host-permuted plans): mode 1 (K / 4 tones per
// class) 356-362 -> 312 us at K = 8 on bins 32 + 9i, the box's read ceiling
// (profiles/round1/probe_dcls.log); modes 2-4 for even-bin plans.
template <int K, int DC, bool NT>
static const void *residue_dc_kernel()
{
    return reinterpret_cast<const void *>(
        &residue_tile_kernel<K, 4, kWavesPerBlock, true, false, (K <= 8 ? 4 : 0), kResidueQP, false,
                             true, false, DC, NT>);
}

template <int K, bool NT>
static const void *residue_kernel_for_t(int log2g, int dcls)
{
    if (log2g == 4) {
        if constexpr (K == 8 || K == 16) {
            switch (dcls) {
            case 1: return residue_dc_kernel<K, 1, NT>();
            case 2: return residue_dc_kernel<K, 2, NT>();
            case 3: return residue_dc_kernel<K, 3, NT>();
            case 4: return residue_dc_kernel<K, 4, NT>();
            default: break;
            }
        }
        return residue_dc_kernel<K, 0, NT>();
    }
    return reinterpret_cast<const void *>(
        &residue_tile_kernel<K, -1, kWavesPerBlock, true, false, (K <= 8 ? 4 : 0), kResidueQP, false,
                             true, false, 0, NT>);
}

// nt: hop = n (each byte read once); overlapping windows keep their lines in L2
template <int K>
static const void *residue_kernel_for(int log2g, int dcls, bool nt)
{
    return nt ? residue_kernel_for_t<K, true>(log2g, dcls) : residue_kernel_for_t<K, false>(log2g, dcls);
}

const void *residue_kernel_ptr(int k, int log2g, int dcls, bool nt)
{
    switch (k) {
#define FSKD_CASE(K) case K: return residue_kernel_for<K>(log2g, dcls, nt);
        FSKD_CASE(1) FSKD_CASE(2) FSKD_CASE(3) FSKD_CASE(4)
        FSKD_CASE(5) FSKD_CASE(6) FSKD_CASE(7) FSKD_CASE(8)
        FSKD_CASE(9) FSKD_CASE(10) FSKD_CASE(11) FSKD_CASE(12)
        FSKD_CASE(13) FSKD_CASE(14) FSKD_CASE(15) FSKD_CASE(16)
#undef FSKD_CASE
    default: return nullptr;
    }
}

}  // namespace fskd
