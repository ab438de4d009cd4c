// fft_quad.hip — the full-spectrum detector laid
// out as 16 lanes per window, 4 windows per wave: per window a 1024-point real
// FFT, |X[b]|^2 for b = 0..512, symbol = argmax over the tone bins (ties ->
// lowest k). Oracle: oracle/fsk_oracle.c:oracle_fft_demod.
//
// z[n] = x[2n] + i x[2n+1] (n < 512) is a 512-point complex FFT, split 32 x 16:
//   n = t + 16 n1 (t = lane % 16, n1 < 32),   k = k1 + 32 k2 (k1 < 32, k2 < 16)
//   Z[k1 + 32 k2] = sum_t W16^{t k2} W512^{t k1} sum_n1 z[t + 16 n1] W32^{n1 k1}
//   1. lane t loads its 32 dwords z[t + 16 n1] (16 lanes = 64 contiguous bytes
//      per instruction) and runs a DFT-32 in registers;
//   2. ONE transpose through LDS: row t -> columns. Lane t' takes the column
//      pair {k1, 32 - k1} (lane 0: {0, 16}) and runs, per column, the DFT-16
//      of the W512^{t k1}-twiddled column in registers;
//   3. the real-FFT post-pass pairs Z[k] with conj Z[512 - k]. With the column
//      pairing above that mirror lives in the same lane, so it needs no
//      exchange: per pair one twiddle product gives both |X[k]|^2 and
//      |X[512 - k]|^2.
// LDS traffic per window: 4 KiB written + 4 KiB read for the transpose (plus
// 2 KiB of bin powers when the full spectrum is stored) — against 12 + 12 KiB
// for a 64-lane radix-8 Stockham layout (scripts/fft_r0.hip, in git history
// at 8b49018), whose LDS writes
// bound it (guide: ds_write aggregates 38-51 TB/s). Every twiddle product is
// fused into the butterfly that consumes it (fft1024_quad_kernel below); the
// round-1 kernel with separate products is scripts/fft_quad_r1b.hip (git
// history, 8b49018).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "demod_internal.h"
#include "rescue_fft.h"
#include "window_sum.h"

namespace fskd {
namespace quad {

// A complex number as a packed fp32 pair: complex add/sub is one v_pk_add_f32,
// a complex product two packed ops. CDNA4 runs a packed op at the same flop
// rate as two plain ones, but one wave issues half as many instructions — and
// this kernel is issue-bound (one wave/SIMD issues a VALU op every 4 cycles).
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

// a * w (w in VGPRs): lo = a.x w.x - a.y w.y, hi = a.x w.y + a.y w.x
__device__ __forceinline__ f2 cmul(f2 a, f2 w)
{
    f2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "v"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(a), "v"(w), "v"(t));
    return r;
}
// a * w with w a compile-time constant (SGPR pair)
__device__ __forceinline__ f2 cmulk(f2 a, f2 w)
{
    f2 t, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[1,0]" : "=v"(t) : "v"(a), "s"(w));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(a), "s"(w), "v"(t));
    return r;
}
// Two independent complex products in one block, ordered mul0 mul1 fma0 fma1.
// gfx950 needs a wait state between a packed-fp32 VGPR write and an
// immediately dependent packed read: the compiler pads every single cmul
// (mul -> dependent fma) with an s_nop, which this ordering avoids.
__device__ __forceinline__ void cmul2(f2 &r0, f2 a0, f2 w0, f2 &r1, f2 a1, f2 w1)
{
    f2 t0, t1;
    asm("v_pk_mul_f32 %2, %4, %5 op_sel:[1,1] op_sel_hi:[1,0]\n\t"
        "v_pk_mul_f32 %3, %6, %7 op_sel:[1,1] op_sel_hi:[1,0]\n\t"
        "v_pk_fma_f32 %0, %4, %5, %2 op_sel_hi:[0,1,1] neg_lo:[0,0,1]\n\t"
        "v_pk_fma_f32 %1, %6, %7, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]"
        : "=&v"(r0), "=&v"(r1), "=&v"(t0), "=&v"(t1)
        : "v"(a0), "v"(w0), "v"(a1), "v"(w1));
}
// the same with both twiddles compile-time constants (SGPR pairs)
__device__ __forceinline__ void cmulk2(f2 &r0, f2 a0, f2 w0, f2 &r1, f2 a1, f2 w1)
{
    f2 t0, t1;
    asm("v_pk_mul_f32 %2, %4, %5 op_sel:[1,1] op_sel_hi:[1,0]\n\t"
        "v_pk_mul_f32 %3, %6, %7 op_sel:[1,1] op_sel_hi:[1,0]\n\t"
        "v_pk_fma_f32 %0, %4, %5, %2 op_sel_hi:[0,1,1] neg_lo:[0,0,1]\n\t"
        "v_pk_fma_f32 %1, %6, %7, %3 op_sel_hi:[0,1,1] neg_lo:[0,0,1]"
        : "=&v"(r0), "=&v"(r1), "=&v"(t0), "=&v"(t1)
        : "v"(a0), "s"(w0), "v"(a1), "s"(w1));
}
// (|u|^2 of two pairs): p = (re.x^2 + im.x^2, re.y^2 + im.y^2) for two
// independent (re, im), interleaved like cmul2
__device__ __forceinline__ void pwr2(f2 &p0, f2 re0, f2 im0, f2 &p1, f2 re1, f2 im1)
{
    f2 t0, t1;
    asm("v_pk_mul_f32 %2, %5, %5\n\t"
        "v_pk_mul_f32 %3, %7, %7\n\t"
        "v_pk_fma_f32 %0, %4, %4, %2\n\t"
        "v_pk_fma_f32 %1, %6, %6, %3"
        : "=&v"(p0), "=&v"(p1), "=&v"(t0), "=&v"(t1)
        : "v"(re0), "v"(im0), "v"(re1), "v"(im1));
}
// x + (-i) y = (x.x + y.y, x.y - y.x)
__device__ __forceinline__ f2 add_mj(f2 x, f2 y)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
// x - (-i) y = (x.x - y.y, x.y + y.x)
__device__ __forceinline__ f2 sub_mj(f2 x, f2 y)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(x), "v"(y));
    return r;
}
// (-i) a = (a.y, -a.x), as a * (1, -1) with the halves swapped
__device__ __forceinline__ f2 mj(f2 a)
{
    f2 r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(a), "s"((f2){1.0f, -1.0f}));
    return r;
}

// Real-FFT post-pass pieces (fft1024_quad_kernel step 3), one packed op each:
// S = P + conj Q
__device__ __forceinline__ f2 pp_s(f2 P, f2 Q)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(r) : "v"(P), "v"(Q));
    return r;
}
// D = -i (P - conj Q) = (P.y + Q.y, Q.x - P.x)
__device__ __forceinline__ f2 pp_d(f2 P, f2 Q)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]" : "=v"(r) : "v"(P), "v"(Q));
    return r;
}
// (S.x + T.x, S.x - T.x) and (S.y + T.y, S.y - T.y): the real / imaginary
// parts of U = S + T and V = S - T side by side
__device__ __forceinline__ f2 pp_re(f2 S, f2 T)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel_hi:[0,0] neg_hi:[0,1]" : "=v"(r) : "v"(S), "v"(T));
    return r;
}
__device__ __forceinline__ f2 pp_im(f2 S, f2 T)
{
    f2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[1,1] neg_hi:[0,1]" : "=v"(r) : "v"(S), "v"(T));
    return r;
}


// lane % 16 == 0 ? a : b (lanes 0, 16, 32, 48 of the wave)
__device__ __forceinline__ f2 sel_l0(f2 a, f2 b)
{
    f2 r;
    // %0 %1 = r; %2 a.x, %3 b.x, %4 mask, %5 a.y, %6 b.y; dst = mask ? src1 : src0
    asm("v_cndmask_b32 %0, %3, %2, %4\n\tv_cndmask_b32 %1, %6, %5, %4"
        : "=&v"(r.x), "=v"(r.y)
        : "v"(a.x), "v"(b.x), "s"(0x0001000100010001ull), "v"(a.y), "v"(b.y));
    return r;
}

// W32^j = e^{-2 pi i j / 32}: real and imaginary parts.
constexpr float kW32r[32] = {
    1.0f, 0.98078528040323043f, 0.92387953251128674f, 0.83146961230254524f,
    0.70710678118654752f, 0.55557023301960218f, 0.38268343236508977f, 0.19509032201612827f,
    0.0f, -0.19509032201612827f, -0.38268343236508977f, -0.55557023301960218f,
    -0.70710678118654752f, -0.83146961230254524f, -0.92387953251128674f, -0.98078528040323043f,
    -1.0f, -0.98078528040323043f, -0.92387953251128674f, -0.83146961230254524f,
    -0.70710678118654752f, -0.55557023301960218f, -0.38268343236508977f, -0.19509032201612827f,
    0.0f, 0.19509032201612827f, 0.38268343236508977f, 0.55557023301960218f,
    0.70710678118654752f, 0.83146961230254524f, 0.92387953251128674f, 0.98078528040323043f};
constexpr float kW32i[32] = {
    0.0f, -0.19509032201612827f, -0.38268343236508977f, -0.55557023301960218f,
    -0.70710678118654752f, -0.83146961230254524f, -0.92387953251128674f, -0.98078528040323043f,
    -1.0f, -0.98078528040323043f, -0.92387953251128674f, -0.83146961230254524f,
    -0.70710678118654752f, -0.55557023301960218f, -0.38268343236508977f, -0.19509032201612827f,
    0.0f, 0.19509032201612827f, 0.38268343236508977f, 0.55557023301960218f,
    0.70710678118654752f, 0.83146961230254524f, 0.92387953251128674f, 0.98078528040323043f,
    1.0f, 0.98078528040323043f, 0.92387953251128674f, 0.83146961230254524f,
    0.70710678118654752f, 0.55557023301960218f, 0.38268343236508977f, 0.19509032201612827f};

// a * W32^J; the half and quarter turns are sign/swap operations.
template <int J>
__device__ __forceinline__ f2 w32(f2 a)
{
    constexpr int j = ((J % 32) + 32) % 32;
    if constexpr (j == 0) return a;
    else if constexpr (j == 8) return mj(a);
    else if constexpr (j == 16) return -a;
    else if constexpr (j == 24) return -mj(a);
    else return cmulk(a, (f2){kW32r[j], kW32i[j]});
}

template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (I < N) {
        f(std::integral_constant<int, I>{});
        static_for<I + 1, N>(f);
    }
}

// The non-trivial twiddles W_N^{i2 k1} (not a multiple of a quarter turn) of
// one dft<N> level: slot i2 + N2 k1 and the W32 exponent.
template <int N>
struct TwList {
    static constexpr int N1 = (N == 32) ? 8 : 4, N2 = N / N1;
    int slot[N];
    int j[N];
    int n;
    constexpr TwList() : slot(), j(), n(0)
    {
        for (int i2 = 0; i2 < N2; ++i2)
            for (int k1 = 1; k1 < N1; ++k1) {
                const int jj = ((i2 * k1) * (32 / N)) % 32;
                if (jj % 8) {
                    slot[n] = i2 + N2 * k1;
                    j[n] = jj;
                    ++n;
                }
            }
    }
};

// In-register DFT of x[0], x[S], ..., x[(N-1) S] (N = 2, 4, 8, 16, 32), result
// in natural order in the same slots. Mixed radix N = N1 x N2 (N1 = 4 or 8):
//   X[k1 + N1 k2] = sum_i2 W_N^{i2 k1} W_N2^{i2 k2} sum_i1 x[N2 i1 + i2] W_N1^{i1 k1}
template <int N, int S = 1>
__device__ __forceinline__ void dft(f2 *x)
{
    if constexpr (N == 2) {
        const f2 a = x[0], b = x[S];
        x[0] = a + b;
        x[S] = a - b;
    } else if constexpr (N == 4) {
        const f2 a0 = x[0] + x[2 * S], a1 = x[0] - x[2 * S];
        const f2 b0 = x[S] + x[3 * S], b1 = x[S] - x[3 * S];
        x[0] = a0 + b0;
        x[2 * S] = a0 - b0;
        x[S] = add_mj(a1, b1);
        x[3 * S] = sub_mj(a1, b1);
    } else {
        constexpr int N1 = (N == 32) ? 8 : 4;
        constexpr int N2 = N / N1;
        // DFT-N1 over i1 for every i2 (stride N2 S), then twiddle W_N^{i2 k1}:
        // the quarter turns in place, the rest two at a time (cmulk2)
        static_for<0, N2>([&](auto c) {
            constexpr int i2 = decltype(c)::value;
            dft<N1, N2 * S>(x + i2 * S);
            static_for<1, N1>([&](auto d) {
                constexpr int k1 = decltype(d)::value;
                if constexpr (((i2 * k1) * (32 / N)) % 8 == 0)
                    x[(i2 + N2 * k1) * S] = w32<(i2 * k1) * (32 / N)>(x[(i2 + N2 * k1) * S]);
            });
        });
        constexpr TwList<N> L{};
        static_for<0, (L.n + 1) / 2>([&](auto pc) {
            constexpr int i0 = 2 * decltype(pc)::value, i1 = i0 + 1;
            constexpr int s0 = L.slot[i0] * S, j0 = L.j[i0];
            if constexpr (i1 < L.n) {
                constexpr int s1 = L.slot[i1] * S, j1 = L.j[i1];
                cmulk2(x[s0], x[s0], (f2){kW32r[j0], kW32i[j0]},
                       x[s1], x[s1], (f2){kW32r[j1], kW32i[j1]});
            } else {
                x[s0] = cmulk(x[s0], (f2){kW32r[j0], kW32i[j0]});
            }
        });
        // DFT-N2 over i2 for every k1 (contiguous run of N2 at N2 k1)
        static_for<0, N1>([&](auto d) {
            constexpr int k1 = decltype(d)::value;
            dft<N2, S>(x + N2 * k1 * S);
        });
        // slot (N2 k1 + k2) S holds X[k1 + N1 k2]: rename to natural order
        f2 t[N];
        static_for<0, N>([&](auto e) {
            constexpr int m = decltype(e)::value;  // m = N2 k1 + k2
            t[(m / N2) + N1 * (m % N2)] = x[m * S];
        });
        static_for<0, N>([&](auto e) {
            constexpr int m = decltype(e)::value;
            x[m * S] = t[m];
        });
    }
}

// ---- fused twiddle butterflies (fft1024_quad_kernel) ----------------------
// A twiddled radix-2 butterfly (u, v) = (x + w y, x - w y) in three packed
// FMAs instead of a complex product (2) and two complex adds (2):
//   t = fma(y, w.xx, x)                    = (x.x + w.x y.x, x.y + w.x y.y)
//   u = fma(y.yx, (-w.y, w.y), t)          = x + w y
//   v = fma(x, 2, -u)                      = x - w y
// (v is 2x - u: one extra rounding of u, far inside the 1e-5 bar.) The -j w
// of a radix-4 butterfly's second output pair is the same register read with
// other op_sel / neg modifiers (-j w = (w.y, -w.x)), so it needs no table.
// Two independent pairs per asm block, interleaved so no packed result feeds
// the next instruction (gfx950 packed-fp32 write -> dependent read hazard).
#define QTB_T(U, Y, W, X) "v_pk_fma_f32 " U ", " Y ", " W ", " X " op_sel_hi:[1,0,1]\n\t"
#define QTB_U(U, Y, W) "v_pk_fma_f32 " U ", " Y ", " W ", " U " op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]\n\t"
#define QTB_TM(U, Y, W, X) "v_pk_fma_f32 " U ", " Y ", " W ", " X " op_sel:[0,1,0] op_sel_hi:[1,1,1]\n\t"
#define QTB_UM(U, Y, W) "v_pk_fma_f32 " U ", " Y ", " W ", " U " op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_hi:[0,1,0]\n\t"
#define QTB_V(V, X, TWO, U) "v_pk_fma_f32 " V ", " X ", " TWO ", " U " neg_lo:[0,0,1] neg_hi:[0,0,1]"

// pair 0 with w0, pair 1 with w1 (both SGPR pairs: compile-time constants)
__device__ __forceinline__ void tbk2(f2 &u0, f2 &v0, f2 x0, f2 y0, f2 w0, f2 &u1, f2 &v1, f2 x1,
                                     f2 y1, f2 w1)
{
    asm(QTB_T("%0", "%5", "%6", "%4") QTB_T("%2", "%8", "%9", "%7")
        QTB_U("%0", "%5", "%6") QTB_U("%2", "%8", "%9")
        QTB_V("%1", "%4", "%10", "%0") "\n\t" QTB_V("%3", "%7", "%10", "%2")
        : "=&v"(u0), "=&v"(v0), "=&v"(u1), "=&v"(v1)
        : "v"(x0), "v"(y0), "s"(w0), "v"(x1), "v"(y1), "s"(w1), "s"((f2){2.0f, 2.0f}));
}
// pair 0 with w, pair 1 with -j w (MJ1) or w (!MJ1); w a VGPR pair (per-lane table)
template <bool MJ1>
__device__ __forceinline__ void tbv2(f2 &u0, f2 &v0, f2 x0, f2 y0, f2 &u1, f2 &v1, f2 x1, f2 y1,
                                     f2 w)
{
    if constexpr (MJ1)
        asm(QTB_T("%0", "%5", "%8", "%4") QTB_TM("%2", "%7", "%8", "%6")
            QTB_U("%0", "%5", "%8") QTB_UM("%2", "%7", "%8")
            QTB_V("%1", "%4", "%9", "%0") "\n\t" QTB_V("%3", "%6", "%9", "%2")
            : "=&v"(u0), "=&v"(v0), "=&v"(u1), "=&v"(v1)
            : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(w), "s"((f2){2.0f, 2.0f}));
    else
        asm(QTB_T("%0", "%5", "%8", "%4") QTB_T("%2", "%7", "%8", "%6")
            QTB_U("%0", "%5", "%8") QTB_U("%2", "%7", "%8")
            QTB_V("%1", "%4", "%9", "%0") "\n\t" QTB_V("%3", "%6", "%9", "%2")
            : "=&v"(u0), "=&v"(v0), "=&v"(u1), "=&v"(v1)
            : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(w), "s"((f2){2.0f, 2.0f}));
}

// W32^E trivial (a quarter turn)?
constexpr bool w32_trivial(int e) { return (((e % 32) + 32) % 32) % 8 == 0; }
template <int E>
__device__ __forceinline__ f2 w32c()
{
    constexpr int j = ((E % 32) + 32) % 32;
    return (f2){kW32r[j], kW32i[j]};
}
// (u, v) = (x + W32^E y, x - W32^E y) for a quarter-turn E
template <int E>
__device__ __forceinline__ void tb_triv(f2 &u, f2 &v, f2 x, f2 y)
{
    constexpr int j = ((E % 32) + 32) % 32;
    static_assert(j % 8 == 0, "quarter turn");
    if constexpr (j == 0) { u = x + y; v = x - y; }
    else if constexpr (j == 16) { u = x - y; v = x + y; }
    else if constexpr (j == 8) { u = add_mj(x, y); v = sub_mj(x, y); }   // w = -j
    else { u = sub_mj(x, y); v = add_mj(x, y); }                          // w = +j
}
// two pairs, W32^E0 and W32^E1, both trivial or both not
template <int E0, int E1>
__device__ __forceinline__ void tbk2c(f2 &u0, f2 &v0, f2 x0, f2 y0, f2 &u1, f2 &v1, f2 x1, f2 y1)
{
    static_assert(w32_trivial(E0) == w32_trivial(E1), "pair kinds");
    if constexpr (w32_trivial(E0)) {
        tb_triv<E0>(u0, v0, x0, y0);
        tb_triv<E1>(u1, v1, x1, y1);
    } else {
        tbk2(u0, v0, x0, y0, w32c<E0>(), u1, v1, x1, y1, w32c<E1>());
    }
}

// DFT-4 of (y0, w y1, w^2 y2, w^3 y3) at x[0], x[S], x[2S], x[3S] (natural
// order out), w = W32^E: four fused butterflies,
//   a = y0 +- w^2 y2, c = y1 +- w^2 y3, X0/X2 = a0 +- w c0, X1/X3 = a1 +- (-j w) c1.
template <int E, int S>
__device__ __forceinline__ void dft4_geo_k(f2 *x)
{
    f2 a0, a1, c0, c1;
    tbk2c<2 * E, 2 * E>(a0, a1, x[0], x[2 * S], c0, c1, x[S], x[3 * S]);
    f2 X0, X1, X2, X3;
    tbk2c<E, E + 8>(X0, X2, a0, c0, X1, X3, a1, c1);
    x[0] = X0;
    x[S] = X1;
    x[2 * S] = X2;
    x[3 * S] = X3;
}
// the same with a per-lane w (VGPRs) and its square w2
template <int S>
__device__ __forceinline__ void dft4_geo_v(f2 *x, f2 w, f2 w2)
{
    f2 a0, a1, c0, c1;
    tbv2<false>(a0, a1, x[0], x[2 * S], c0, c1, x[S], x[3 * S], w2);
    f2 X0, X1, X2, X3;
    tbv2<true>(X0, X2, a0, c0, X1, X3, a1, c1, w);
    x[0] = X0;
    x[S] = X1;
    x[2 * S] = X2;
    x[3 * S] = X3;
}

// The same two butterfly stages as ONE asm block (12 packed FMAs): every
// result is read two or more instructions after it is written, so the block
// needs none of the packed-write s_nops the two separate blocks cost at their
// seam (the second block's first pairs read the first block's last results).
// Operands: %0-%3 X0..X3 (out), %4-%7 a0 a1 c0 c1 (scratch), %8-%11 x0..x3,
// %12 w (second stage; the -j w pair by modifiers), %13 w^2 (first stage),
// %14 (2, 2).
#define QF_STAGES(WA, WB, TMB, UMB)                                                        \
    QTB_T("%4", "%10", WA, "%8") QTB_T("%6", "%11", WA, "%9")                              \
    QTB_U("%4", "%10", WA) QTB_U("%6", "%11", WA)                                          \
    QTB_V("%5", "%8", "%14", "%4") "\n\t" QTB_V("%7", "%9", "%14", "%6") "\n\t"         \
    QTB_T("%0", "%6", WB, "%4") TMB("%1", "%7", WB, "%5")                                   \
    QTB_U("%0", "%6", WB) UMB("%1", "%7", WB)                                               \
    QTB_V("%2", "%4", "%14", "%0") "\n\t" QTB_V("%3", "%5", "%14", "%1")
template <int S>
__device__ __forceinline__ void dft4_fused_v(f2 *x, f2 w, f2 w2)
{
    f2 X0, X1, X2, X3, a0, a1, c0, c1;
    asm(QF_STAGES("%13", "%12", QTB_TM, QTB_UM)
        : "=&v"(X0), "=&v"(X1), "=&v"(X2), "=&v"(X3), "=&v"(a0), "=&v"(a1), "=&v"(c0), "=&v"(c1)
        : "v"(x[0]), "v"(x[S]), "v"(x[2 * S]), "v"(x[3 * S]), "v"(w), "v"(w2),
          "s"((f2){2.0f, 2.0f}));
    x[0] = X0;
    x[S] = X1;
    x[2 * S] = X2;
    x[3 * S] = X3;
}

// Two independent dft4_fused_v, interleaved instruction by instruction
// (dependent results four instructions apart) and updated in place (the
// first stage's inputs are dead once it has run): %0-%3 / %4-%7 the two
// DFT-4s' x0..x3 (in / out), %8-%15 scratch a0 a1 c0 c1 of each, %16 / %17
// w / w^2 of the first, %18 / %19 of the second, %20 (2, 2).
template <int S>
__device__ __forceinline__ void dft4x2_fused_v(f2 *xa, f2 *xb, f2 wa, f2 w2a, f2 wb, f2 w2b)
{
    f2 a0, a1, c0, c1, b0, b1, d0, d1;
    asm(// first stage: a = x0 +- w^2 x2, c = x1 +- w^2 x3 (both DFT-4s)
        QTB_T("%8", "%2", "%17", "%0") QTB_T("%10", "%3", "%17", "%1")
        QTB_T("%12", "%6", "%19", "%4") QTB_T("%14", "%7", "%19", "%5")
        QTB_U("%8", "%2", "%17") QTB_U("%10", "%3", "%17")
        QTB_U("%12", "%6", "%19") QTB_U("%14", "%7", "%19")
        QTB_V("%9", "%0", "%20", "%8") "\n\t" QTB_V("%11", "%1", "%20", "%10") "\n\t"
        QTB_V("%13", "%4", "%20", "%12") "\n\t" QTB_V("%15", "%5", "%20", "%14") "\n\t"
        // second stage into x: X0/X2 = a0 +- w c0, X1/X3 = a1 +- (-j w) c1
        QTB_T("%0", "%10", "%16", "%8") QTB_TM("%1", "%11", "%16", "%9")
        QTB_T("%4", "%14", "%18", "%12") QTB_TM("%5", "%15", "%18", "%13")
        QTB_U("%0", "%10", "%16") QTB_UM("%1", "%11", "%16")
        QTB_U("%4", "%14", "%18") QTB_UM("%5", "%15", "%18")
        QTB_V("%2", "%8", "%20", "%0") "\n\t" QTB_V("%3", "%9", "%20", "%1") "\n\t"
        QTB_V("%6", "%12", "%20", "%4") "\n\t" QTB_V("%7", "%13", "%20", "%5")
        : "+v"(xa[0]), "+v"(xa[S]), "+v"(xa[2 * S]), "+v"(xa[3 * S]),
          "+v"(xb[0]), "+v"(xb[S]), "+v"(xb[2 * S]), "+v"(xb[3 * S]),
          "=&v"(a0), "=&v"(a1), "=&v"(c0), "=&v"(c1), "=&v"(b0), "=&v"(b1), "=&v"(d0), "=&v"(d1)
        : "v"(wa), "v"(w2a), "v"(wb), "v"(w2b), "s"((f2){2.0f, 2.0f}));
}

// dft4_geo_k<E, S> as one block when neither w^2 = W32^{2E} nor w is a
// quarter turn: first stage both pairs with w^2, second stage w and -j w =
// W32^{E+8}, all SGPR constants (%12 w, %13 w^2, %15 -j w).
#define QF_STAGES_K                                                                         \
    QTB_T("%4", "%10", "%13", "%8") QTB_T("%6", "%11", "%13", "%9")                        \
    QTB_U("%4", "%10", "%13") QTB_U("%6", "%11", "%13")                                    \
    QTB_V("%5", "%8", "%14", "%4") "\n\t" QTB_V("%7", "%9", "%14", "%6") "\n\t"         \
    QTB_T("%0", "%6", "%12", "%4") QTB_T("%1", "%7", "%15", "%5")                           \
    QTB_U("%0", "%6", "%12") QTB_U("%1", "%7", "%15")                                       \
    QTB_V("%2", "%4", "%14", "%0") "\n\t" QTB_V("%3", "%5", "%14", "%1")
template <int E, int S>
__device__ __forceinline__ void dft4_fused_k(f2 *x)
{
    f2 X0, X1, X2, X3, a0, a1, c0, c1;
    asm(QF_STAGES_K
        : "=&v"(X0), "=&v"(X1), "=&v"(X2), "=&v"(X3), "=&v"(a0), "=&v"(a1), "=&v"(c0), "=&v"(c1)
        : "v"(x[0]), "v"(x[S]), "v"(x[2 * S]), "v"(x[3 * S]), "s"(w32c<E>()), "s"(w32c<2 * E>()),
          "s"((f2){2.0f, 2.0f}), "s"(w32c<E + 8>()));
    x[0] = X0;
    x[S] = X1;
    x[2 * S] = X2;
    x[3 * S] = X3;
}

// FUSED 3: the trivial-twiddle pieces of the DFT-32 as single blocks too.
// x + (-j) y and x - (-j) y as instruction text (add_mj / sub_mj)
#define QA_MJ(R, X, Y) "v_pk_add_f32 " R ", " X ", " Y " op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]\n\t"
#define QS_MJ(R, X, Y) "v_pk_add_f32 " R ", " X ", " Y " op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]\n\t"
#define QADD(R, X, Y) "v_pk_add_f32 " R ", " X ", " Y "\n\t"
#define QSUB(R, X, Y) "v_pk_add_f32 " R ", " X ", " Y " neg_lo:[0,1] neg_hi:[0,1]\n\t"
// DFT-4 with no twiddles (dft4_geo_k<0>): 8 packed adds.
// %0-%3 X0..X3, %4-%7 a0 a1 c0 c1, %8-%11 x0..x3
template <int S>
__device__ __forceinline__ void dft4_triv(f2 *x)
{
    f2 X0, X1, X2, X3, a0, a1, c0, c1;
    asm(QADD("%4", "%8", "%10") QSUB("%5", "%8", "%10") QADD("%6", "%9", "%11") QSUB("%7", "%9", "%11")
        QADD("%0", "%4", "%6") QSUB("%2", "%4", "%6") QA_MJ("%1", "%5", "%7")
        "v_pk_add_f32 %3, %5, %7 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]"
        : "=&v"(X0), "=&v"(X1), "=&v"(X2), "=&v"(X3), "=&v"(a0), "=&v"(a1), "=&v"(c0), "=&v"(c1)
        : "v"(x[0]), "v"(x[S]), "v"(x[2 * S]), "v"(x[3 * S]));
    x[0] = X0;
    x[S] = X1;
    x[2 * S] = X2;
    x[3 * S] = X3;
}
// dft4_geo_k<E> with w^2 = -j (E = 4): first stage add_mj / sub_mj, second
// stage w = W32^E and -j w = W32^{E+8} (%12, %13 SGPR pairs, %14 (2, 2)).
template <int E, int S>
__device__ __forceinline__ void dft4_fused_kq(f2 *x)
{
    static_assert(((2 * E) % 32 + 32) % 32 == 8, "w^2 = -j");
    f2 X0, X1, X2, X3, a0, a1, c0, c1;
    asm(QA_MJ("%4", "%8", "%10") QA_MJ("%6", "%9", "%11") QS_MJ("%5", "%8", "%10") QS_MJ("%7", "%9", "%11")
        QTB_T("%0", "%6", "%12", "%4") QTB_T("%1", "%7", "%13", "%5")
        QTB_U("%0", "%6", "%12") QTB_U("%1", "%7", "%13")
        QTB_V("%2", "%4", "%14", "%0") "\n\t" QTB_V("%3", "%5", "%14", "%1")
        : "=&v"(X0), "=&v"(X1), "=&v"(X2), "=&v"(X3), "=&v"(a0), "=&v"(a1), "=&v"(c0), "=&v"(c1)
        : "v"(x[0]), "v"(x[S]), "v"(x[2 * S]), "v"(x[3 * S]), "s"(w32c<E>()), "s"(w32c<E + 8>()),
          "s"((f2){2.0f, 2.0f}));
    x[0] = X0;
    x[S] = X1;
    x[2 * S] = X2;
    x[3 * S] = X3;
}
// The DFT-8's last stage (dftf<8>): pairs (slot 2k1, 2k1 + 1) with W8^k1:
// k1 = 0 trivial, 2 is -j, 1 and 3 general (W32^4, W32^12), interleaved.
// %0-%7 out slots 0..7 (u0 u1 u2 u3 v0 v1 v2 v3), %8-%15 in, %16 W32^4,
// %17 W32^12, %18 (2, 2)
template <int S>
__device__ __forceinline__ void dft8_last(f2 *x)
{
    f2 u0, u1, u2, u3, v0, v1, v2, v3;
    asm(QTB_T("%1", "%11", "%16", "%10") QTB_T("%3", "%15", "%17", "%14")
        QADD("%0", "%8", "%9") QSUB("%4", "%8", "%9")
        QTB_U("%1", "%11", "%16") QTB_U("%3", "%15", "%17")
        QA_MJ("%2", "%12", "%13") QS_MJ("%6", "%12", "%13")
        QTB_V("%5", "%10", "%18", "%1") "\n\t" QTB_V("%7", "%14", "%18", "%3")
        : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3), "=&v"(v0), "=&v"(v1), "=&v"(v2), "=&v"(v3)
        : "v"(x[0]), "v"(x[S]), "v"(x[2 * S]), "v"(x[3 * S]), "v"(x[4 * S]), "v"(x[5 * S]),
          "v"(x[6 * S]), "v"(x[7 * S]), "s"(w32c<4>()), "s"(w32c<12>()), "s"((f2){2.0f, 2.0f}));
    x[0] = u0; x[S] = u1; x[2 * S] = u2; x[3 * S] = u3;
    x[4 * S] = v0; x[5 * S] = v1; x[6 * S] = v2; x[7 * S] = v3;
}

// In-register DFT of x[0], x[S], .., x[(N-1) S] (N = 4, 8, 16, 32), natural
// order out, every twiddle fused into the butterfly that consumes it.
// Mixed radix N = N1 x N2 (N2 = 4, or 2 at N = 8): DFT-N1 over i1 for each i2,
// then per k1 a DFT-N2 over i2 of the twiddled column, which is geometric in
// w = W_N^{k1} (dft4_geo_k).
// L (FUSED level): >= 1 both-nontrivial DFT-4s as one block, >= 3 the
// trivial pieces too.
template <int N, int S = 1, int L = 0>
__device__ __forceinline__ void dftf(f2 *x)
{
    if constexpr (N == 4) {
        if constexpr (L >= 3)
            dft4_triv<S>(x);
        else
            dft4_geo_k<0, S>(x);
    } else if constexpr (N == 8) {
        dftf<4, 2 * S, L>(x);       // i2 = 0: X[k1] at slot 2 k1
        dftf<4, 2 * S, L>(x + S);   // i2 = 1: X[k1] at slot 2 k1 + 1
        // per k1: (slot 2k1, slot 2k1+1) -> X[k1], X[k1 + 4], twiddle W8^k1 = W32^{4 k1}
        if constexpr (L >= 3) {
            dft8_last<S>(x);
            return;
        }
        f2 u0, v0, u1, v1, u2, v2, u3, v3;
        tb_triv<0>(u0, v0, x[0], x[S]);
        tb_triv<8>(u2, v2, x[4 * S], x[5 * S]);
        tbk2c<4, 12>(u1, v1, x[2 * S], x[3 * S], u3, v3, x[6 * S], x[7 * S]);
        x[0] = u0; x[S] = u1; x[2 * S] = u2; x[3 * S] = u3;
        x[4 * S] = v0; x[5 * S] = v1; x[6 * S] = v2; x[7 * S] = v3;
    } else {
        constexpr int N1 = N / 4;   // 8 (N = 32) or 4 (N = 16)
        static_for<0, 4>([&](auto c) {
            constexpr int i2 = decltype(c)::value;
            dftf<N1, 4 * S, L>(x + i2 * S);   // X[k1] of column i2 at slot i2 + 4 k1
        });
        static_for<0, N1>([&](auto d) {
            constexpr int k1 = decltype(d)::value;
            constexpr int E = k1 * (32 / N);
            if constexpr (L >= 1 && !w32_trivial(E) && !w32_trivial(2 * E))
                dft4_fused_k<E, S>(x + 4 * k1 * S);
            else if constexpr (L >= 3 && ((E % 32) + 32) % 32 == 0)
                dft4_triv<S>(x + 4 * k1 * S);
            else if constexpr (L >= 3 && !w32_trivial(E) && ((2 * E) % 32 + 32) % 32 == 8)
                dft4_fused_kq<E, S>(x + 4 * k1 * S);
            else
                dft4_geo_k<E, S>(x + 4 * k1 * S);   // slot 4 k1 + k2 = X[k1 + N1 k2]
        });
        f2 t[N];
        static_for<0, N>([&](auto e) {
            constexpr int m = decltype(e)::value;  // m = 4 k1 + k2
            t[(m / 4) + N1 * (m % 4)] = x[m * S];
        });
        static_for<0, N>([&](auto e) {
            constexpr int m = decltype(e)::value;
            x[m * S] = t[m];
        });
    }
}

// Real post-pass with the 1/2 of X = (S + W D)/2 folded into two FMAs (T
// carries W/2): (S.x/2 + T.x, S.x/2 - T.x) and (S.y/2 + T.y, S.y/2 - T.y)
__device__ __forceinline__ f2 pp_re_h(f2 S, f2 T)
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %3, %2 op_sel_hi:[0,1,0] neg_hi:[0,0,1]"
        : "=v"(r) : "v"(S), "v"(T), "s"((f2){0.5f, 0.5f}));
    return r;
}
__device__ __forceinline__ f2 pp_im_h(f2 S, f2 T)
{
    f2 r;
    asm("v_pk_fma_f32 %0, %1, %3, %2 op_sel:[1,0,1] neg_hi:[0,0,1]"
        : "=v"(r) : "v"(S), "v"(T), "s"((f2){0.5f, 0.5f}));
    return r;
}

// Two mirror pairs of the real post-pass as one block (16 packed ops):
// S = P + conj Q, D = -i (P - conj Q), T = D (W / 2), (re, im) of X[kP] and
// X[512 - kP] side by side, powers (|X[kP]|^2, |X[512 - kP]|^2). Interleaved
// so every result is read two instructions after it is written.
// Operands: %0 %1 pw0 pw1 (out), %2-%9 scratch S0 S1 D0 D1 T0 T1 R0 R1,
// %10 P0, %11 Q0, %12 W0, %13 P1, %14 Q1, %15 W1, %16 (1/2, 1/2).
__device__ __forceinline__ void postpair2(f2 &pw0, f2 P0, f2 Q0, f2 W0, f2 &pw1, f2 P1, f2 Q1, f2 W1)
{
    f2 S0, S1, D0, D1, T0, T1, R0, R1;
    asm("v_pk_add_f32 %2, %10, %11 neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %3, %13, %14 neg_hi:[0,1]\n\t"
        "v_pk_add_f32 %4, %10, %11 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]\n\t"
        "v_pk_add_f32 %5, %13, %14 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]\n\t"
        "v_pk_mul_f32 %6, %4, %12 op_sel:[1,1] op_sel_hi:[1,0]\n\t"
        "v_pk_mul_f32 %7, %5, %15 op_sel:[1,1] op_sel_hi:[1,0]\n\t"
        "v_pk_fma_f32 %6, %4, %12, %6 op_sel_hi:[0,1,1] neg_lo:[0,0,1]\n\t"
        "v_pk_fma_f32 %7, %5, %15, %7 op_sel_hi:[0,1,1] neg_lo:[0,0,1]\n\t"
        "v_pk_fma_f32 %8, %2, %16, %6 op_sel_hi:[0,1,0] neg_hi:[0,0,1]\n\t"
        "v_pk_fma_f32 %9, %3, %16, %7 op_sel_hi:[0,1,0] neg_hi:[0,0,1]\n\t"
        "v_pk_fma_f32 %4, %2, %16, %6 op_sel:[1,0,1] neg_hi:[0,0,1]\n\t"
        "v_pk_fma_f32 %5, %3, %16, %7 op_sel:[1,0,1] neg_hi:[0,0,1]\n\t"
        "v_pk_mul_f32 %6, %4, %4\n\t"
        "v_pk_mul_f32 %7, %5, %5\n\t"
        "v_pk_fma_f32 %0, %8, %8, %6\n\t"
        "v_pk_fma_f32 %1, %9, %9, %7"
        : "=&v"(pw0), "=&v"(pw1), "=&v"(S0), "=&v"(S1), "=&v"(D0), "=&v"(D1), "=&v"(T0), "=&v"(T1),
          "=&v"(R0), "=&v"(R1)
        : "v"(P0), "v"(Q0), "v"(W0), "v"(P1), "v"(Q1), "v"(W1), "s"((f2){0.5f, 0.5f}));
}

}  // namespace quad

// Per-wave LDS: 4 windows x 16 rows x 17 complex (8704 B). The transpose
// moves half the columns per round (k1 < 16, then k1 >= 16), so only half of
// the DFT-32 output and half of the DFT-16 input are live at once. Row stride
// 34 words: the 16 lanes of a row write (ds_write_b64) cover 32 banks; the
// window stride 544 words = 32 mod 64 puts odd windows on the other 32, so a
// 32-lane pass of writes or column reads is conflict-free. Reused for the bin
// powers (4 x 513 floats).
// Bin powers after step 3, per window (stride kQPow floats): pair j of lane t
// stores (|X[kP]|^2, |X[512 - kP]|^2) as one f2 at slot 16 j + t; lane 0's
// |X[0]|^2, |X[512]|^2 sit at floats 512, 513. quad_slot(b) is the float
// index of bin b.
constexpr int kQPow = 544;  // floats per window: 8-byte aligned, odd windows on the other 32 banks
__host__ __device__ constexpr int quad_slot(int b)
{
    const int u = b & 31, v = b >> 5;
    // lane 0: pairs j < 8 hold kP = 16 + 32 j, pair 8 |X[256]|^2 twice,
    // pairs j > 8 kP = 32 j; |X[0]|^2 and |X[512]|^2 at floats 512, 513
    if (b == 0 || b == 512) return 512 + (b >> 9);
    if (u == 0) return v > 8 ? 2 * (16 * v) : v == 8 ? 256 : 2 * (16 * (16 - v)) + 1;
    if (u == 16) return v < 8 ? 2 * (16 * v) : 2 * (16 * (15 - v)) + 1;
    if (u < 16) return 2 * (16 * v + u);                 // kP = t + 32 j
    return 2 * (16 * (15 - v) + (32 - u)) + 1;           // mirror 512 - kP
}

constexpr int kQRow = 17;            // complex per row (16 + 1 pad)
constexpr int kQWin = 16 * kQRow;    // complex per window
constexpr int kQSlab = 4 * kQWin;    // complex per wave
static_assert(4 * kQPow <= 2 * kQSlab, "bin powers of 4 windows must fit the slab");

// Typed (format) buffer loads, for the FMT variant below.
namespace quad {
typedef int i4 __attribute__((ext_vector_type(4)));
__device__ f2 raw_buffer_load_format_v2f32(i4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.format.v2f32");
// buffer descriptor word 3: DST_SEL x,y,z,w = 4,5,6,7; NUM_FORMAT 3 (SSCALED);
// DATA_FORMAT 5 (16_16)
constexpr int kFmtWord3 = 0xFAC | (3 << 12) | (5 << 15);
}  // namespace quad

// fft1024_quad_kernel (round 2): the quad layout with every twiddle fused into the
// butterfly that consumes it (dftf, dft4_geo_*), the stage-1 twiddle moved
// behind the transpose and the 1/2 of the real split folded into the
// post-pass FMAs:
//   * stage 1: DFT-32 over n1 (compile-time twiddles fused), transposed raw;
//   * stage 2: lane t' runs, per column col in {t', k1b}, the DFT-16 over rows
//     t of A_t[col] W512^{t col}. With t = i2 + 4 i1 the twiddle factors as
//     W512^{i2 col} W128^{i1 col}: the inner DFT-4 over i1 is geometric in
//     v = W128^col, and W512^{i2 col} moves onto its outputs, where it joins
//     W16^{i2 k1} into the outer DFT-4's ratio g_k1 = W512^{col + 32 k1}; per
//     lane and column v, v^2, g_k1, g_k1^2 come from a 2.5 KiB LDS table
//     (tw2), -j w by operand modifiers;
//   * post-pass: T = (W/2) D (tw3 holds W1024^kP / 2), (re, im) pairs by FMA
//     with 1/2 (pp_re_h / pp_im_h).
// 514 instead of 575 packed instructions per group of 4 windows.
// PF: 1 = the next group's 32 loads go out during the transpose (32 VGPRs live
// across stage 2 and the post-pass), 0 = each group loads at the top of its
// iteration and the co-resident waves cover the latency (4 waves/SIMD at
// MINW = 4 without spills: 104-116 VGPRs), 2 (SPEC + SPL) = the next group's
// loads go out after the post-pass, ahead of the spectrum stores.
// SPEC: false = symbols (+ tone powers) only: the tone powers are picked
// from the registers of the lanes that hold them (p.slot, a wave-uniform
// index: s_set_gpr_idx) instead of going through the 2 KiB per-window power
// slab in LDS; true = the slab, for the full-spectrum store.
// PICK (SPEC false): 0 = each lane keeps the best and second tone it owns
// (per tone: a compare chain, selects and an exec-masked magnitude store),
// then the row argmax; 1 = tone i's power is gathered into lane i of its row
// by one ds_bpermute, so lanes t < K hold tone t like the slab pick leaves
// them (4 VALU per tone instead of ~27, one coalesced magnitude store).
// AUX: the loads' cache-policy bits (2 = nt, 1 = sc0, 0 = plain; launch_fft_quad).
// FUSED: 1 = each DFT-4's two butterfly stages as one asm block
// (dft4_fused_v / _k), 2 = also the post-pass pairs (postpair2), 3 = also
// the DFT-32's trivial-twiddle DFT-4s and DFT-8 stages (dft4_triv,
// dft4_fused_kq, dft8_last), 4 = stage 2's DFT-4s two per block,
// interleaved (dft4x2_fused_v); the separate blocks cost an s_nop and a
// scheduling barrier at every seam.
// FMT (PF = 0 only): typed buffer loads (16_16 SSCALED) convert both int16
// halves to fp32 in the texture path instead of 64 VALU converts per group
// (measured neutral).
// SPL (with SPEC): 1 = the bin powers go to the slab as the output's own
// layout (4 windows x 513 floats, contiguous, bin b of window q at float
// 513 q + b; each lane's pair j lands at its bins by immediate offsets), and
// the group's live windows leave as one contiguous run of 16-byte stores
// (9 ds_read_b128 + 9 dwordx4 stores per lane, 1 KiB per wave instruction);
// 2 = the same with non-temporal stores (the spectrum is written once);
// 0 = the quad_slot layout, 33 scattered dword stores per lane.
// OVL (FUSED 4): round 1 of the transpose overlaps column 0's DFT-16. Column
// 0's twiddles are read right behind round 0's column reads, round 1's writes
// and reads follow, and column 0's DFT-16 runs while they are in flight (the
// waits land on the first use of round 1's data, not before column 0's
// math); the next group's round-0 writes are ordered behind them.
// TW3R: the post-pass twiddles W1024^kP / 2 from registers instead of the
// LDS table tw3: kP = te + 32 j, so the twiddle is a per-lane base
// W1024^te / 2 (te = t, or 16 for lane 0's pairs j < 8) times the
// compile-time W32^j — one packed complex product (29 VALU per group) in
// place of 8 ds_read2_b64.
template <int WPB = 4, int MINW = 4, int PF = 0, bool SPEC = true, bool FMT = false, int AUX = 2,
          int FUSED = 0, int RD = 0, int SPL = 0, int OVL = 0, int TW3R = 0, int RSC = 1, int PICK = 0>
__device__ __attribute__((always_inline)) inline void fft1024_quad_body(const FftParams &p)
{
    static_assert(!OVL || (FUSED >= 4 && PF != 1), "OVL: the FUSED 4 column DFT-16");
    static_assert(PF != 2 || (SPEC && SPL), "PF 2: ahead of the linear-slab spectrum stores");
    static_assert(!SPL || SPEC, "SPL: the linear power slab of the spectrum store");
    using namespace quad;
    __shared__ __attribute__((aligned(16))) f2 slab[WPB][kQSlab];
    // RD < 2: tw2 [column slot][v, v2, g0, g0^2, .., g3, g3^2][t], tw3 [j][t];
    // RD 2: lane-major, [slot][t][m] and [t][j] (row padded to 18), so each
    // pair used together is one 16-byte read; the row strides (20 and 36
    // dwords) put a ds_read_b128 group's 16 addresses on distinct banks
    constexpr int kT3 = RD >= 2 ? 18 : 16;
    __shared__ __attribute__((aligned(16))) f2 tw2[2 * 10 * 16];
    __shared__ __attribute__((aligned(16))) f2 tw3[16 * kT3];
    auto tw2_at = [](int sl, int m, int tt) { return RD >= 2 ? sl * 160 + tt * 10 + m : sl * 160 + m * 16 + tt; };
    auto tw3_at = [](int j, int tt) { return RD >= 2 ? tt * kT3 + j : j * 16 + tt; };
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int q = lane >> 4;   // window of the wave
    const int t = lane & 15;   // row / column-pair index
    const f2 *t512 = reinterpret_cast<const f2 *>(p.tw512);
    const f2 *t1024 = reinterpret_cast<const f2 *>(p.tw1024);
    for (int i = threadIdx.x; i < 2 * 10 * 16; i += 64 * WPB) {
        const int tt = i & 15, m = (i >> 4) % 10, sl = i / 160;
        const int col = sl == 0 ? tt : (tt == 0 ? 16 : 32 - tt);
        int e;  // exponent of W512
        if (m == 0) e = 4 * col;                          // v = W128^col
        else if (m == 1) e = 8 * col;                     // v^2
        else {
            const int k1 = (m - 2) >> 1;
            e = (col + 32 * k1) * (((m - 2) & 1) ? 2 : 1);   // g_k1, g_k1^2
        }
        tw2[tw2_at(sl, m, tt)] = t512[e & 511];
    }
    for (int i = threadIdx.x; i < 16 * 16; i += 64 * WPB) {
        const int tt = i & 15, j = i >> 4;
        tw3[tw3_at(j, tt)] = 0.5f * t1024[(tt == 0 && j < 8) ? 16 + 32 * j : tt + 32 * j];
    }
    const int k1b = t == 0 ? 16 : 32 - t;
    const int mybin = t < p.k ? p.bins[t] : 0;
    const int myslot = SPL ? q * 513 + mybin : quad_slot(mybin);
    float *pw = reinterpret_cast<float *>(slab[wave]);
    // TW3R: this lane's post-pass twiddle bases (pairs j < 8 and j >= 8)
    f2 tb_lo = (f2){0.f, 0.f}, tb_hi = (f2){0.f, 0.f};
    if constexpr (TW3R) {
        tb_lo = 0.5f * t1024[t == 0 ? 16 : t];
        tb_hi = 0.5f * t1024[t];
    }
    const int rowaddr = (lane & 48) * 4;  // byte address of this window row's lane 0 (ds_bpermute)
    __syncthreads();

    const long long n_groups = (p.n_windows + 3) >> 2;
    const long long stride = (long long)gridDim.x * WPB;
    long long g = tile_block(p.xcd_swizzle) * WPB + wave;
    const long long g_first = g;
    static_assert(!FMT || PF == 0, "FMT loads straight into a[]");
    uint32_t nx[FMT ? 1 : 32];
    f2 nxf[FMT ? 32 : 1];
    // One buffer descriptor per group (wave-uniform base = its first window);
    // the lane offset is the window's start + 4 t bytes, and z[t + 16 n1] is
    // the immediate offset 64 n1 (< 4 KiB). Windows past the end are clamped
    // to the last (never stored).
    auto load_group = [&](long long gg) {
        const long long w0 = 4 * gg;
        const long long left = p.n_windows - w0;  // >= 1
        const long long wq = q < left ? q : left - 1;
        long long bytes = ((left - 1) * p.hop + 1024) * 2;
        if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.pcm + w0 * p.hop), (short)0, (int)bytes, 0x00020000);
        const int voff = (int)(wq * p.hop * 2) + 4 * t;
        if constexpr (FMT) {
            const unsigned long long base = (unsigned long long)(p.pcm + w0 * p.hop);
            const i4 rf = {(int)(unsigned)base, (int)((base >> 32) & 0xFFFF), (int)bytes, kFmtWord3};
#pragma unroll
            for (int n1 = 0; n1 < 32; ++n1)
                nxf[n1] = raw_buffer_load_format_v2f32(rf, voff + 64 * n1, 0, AUX);
        } else {
#pragma unroll
            for (int n1 = 0; n1 < 32; ++n1)
                nx[n1] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 64 * n1, 0, AUX);
        }
    };
    if (PF && g < n_groups) load_group(g);
    for (; g < n_groups; g += stride) {
        const long long w = 4 * g + q;
        if (!PF) load_group(g);
        f2 a[32];
#pragma unroll
        for (int n1 = 0; n1 < 32; ++n1) {
            if constexpr (FMT) {
                a[n1] = nxf[n1];
                continue;
            }
            a[n1] = (f2){(float)(int)(short)(nx[FMT ? 0 : n1] & 0xFFFFu),
                         (float)((int)nx[FMT ? 0 : n1] >> 16)};
            asm("" : "+v"(a[n1]));  // opaque: keep (float)a + (float)b a packed add
        }

        // 1. DFT-32 over n1 (fused twiddles), no stage-1 twiddle here
        dftf<32, 1, FUSED>(a);

        // 2. transpose in two column rounds; lane (q, t') gets columns
        //    k1 = t' (round 0) and k1b (round 1) of its window
        f2 b[32];  // b[n2] = A_n2[t'], b[16 + n2] = A_n2[k1b]
        f2 *win = slab[wave] + q * kQWin;
        // twp(sl, m): the pair (m, m + 1) of slot sl, m even
        auto twp = [&](int sl, int m, f2 &lo, f2 &hi) {
            if constexpr (RD >= 2) {
                const f4 x = *reinterpret_cast<const f4 *>(&tw2[tw2_at(sl, m, t)]);
                lo = (f2){x.x, x.y};
                hi = (f2){x.z, x.w};
            } else {
                lo = tw2[tw2_at(sl, m, t)];
                hi = tw2[tw2_at(sl, m + 1, t)];
            }
        };
        auto twv = [&](int sl, int m) -> f2 { return tw2[tw2_at(sl, m, t)]; };
        // one column's DFT-16 (FUSED 4) with its ten twiddles given
        auto col16 = [&](f2 *bb, f2 v, f2 v2, f2 g0, f2 g0s, f2 g1, f2 g1s, f2 g2, f2 g2s, f2 g3,
                         f2 g3s) {
            dft4x2_fused_v<4>(bb + 0, bb + 1, v, v2, v, v2);
            dft4x2_fused_v<4>(bb + 2, bb + 3, v, v2, v, v2);
            dft4x2_fused_v<1>(bb + 0, bb + 4, g0, g0s, g1, g1s);
            dft4x2_fused_v<1>(bb + 8, bb + 12, g2, g2s, g3, g3s);
            f2 tt[16];
            static_for<0, 16>([&](auto e) {
                constexpr int m = decltype(e)::value;  // m = 4 k1 + k2 holds Z[col + 32 (k1 + 4 k2)]
                tt[(m / 4) + 4 * (m % 4)] = bb[m];
            });
            static_for<0, 16>([&](auto e) {
                constexpr int m = decltype(e)::value;
                bb[m] = tt[m];
            });
        };
        if constexpr (OVL) {
            // the previous group's round-1 reads stay ahead of these writes
            // (LDS executes one wave's operations in order)
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int c = 0; c < 16; ++c) win[t * kQRow + c] = a[c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int n2 = 0; n2 < 16; ++n2) b[n2] = win[n2 * kQRow + t];
            f2 v, v2, g0, g0s, g1, g1s, g2, g2s, g3, g3s;
            twp(0, 0, v, v2);
            twp(0, 2, g0, g0s);
            twp(0, 4, g1, g1s);
            twp(0, 6, g2, g2s);
            twp(0, 8, g3, g3s);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int c = 0; c < 16; ++c) win[t * kQRow + c] = a[16 + c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int n2 = 0; n2 < 16; ++n2) b[16 + n2] = win[n2 * kQRow + k1b - 16];
            col16(b, v, v2, g0, g0s, g1, g1s, g2, g2s, g3, g3s);
            twp(1, 0, v, v2);
            twp(1, 2, g0, g0s);
            twp(1, 4, g1, g1s);
            twp(1, 6, g2, g2s);
            twp(1, 8, g3, g3s);
            col16(b + 16, v, v2, g0, g0s, g1, g1s, g2, g2s, g3, g3s);
        }
#pragma unroll
        for (int r = 0; r < (OVL ? 0 : 2); ++r) {
#pragma unroll
            for (int c = 0; c < 16; ++c) win[t * kQRow + c] = a[16 * r + c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (PF == 1 && r == 0) load_group(g + stride < n_groups ? g + stride : g);
            const int col = r == 0 ? t : k1b - 16;
#pragma unroll
            for (int n2 = 0; n2 < 16; ++n2) b[16 * r + n2] = win[n2 * kQRow + col];
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        // 3. per column: DFT-16 over t of A_t[col] W512^{t col}, twiddles fused
#pragma unroll
        for (int sl = 0; sl < (OVL ? 0 : 2); ++sl) {
            f2 *bb = b + 16 * sl;
            f2 v, v2;
            twp(sl, 0, v, v2);
            if constexpr (FUSED >= 4) {
                dft4x2_fused_v<4>(bb + 0, bb + 1, v, v2, v, v2);
                dft4x2_fused_v<4>(bb + 2, bb + 3, v, v2, v, v2);
                f2 g0, g0s, g1, g1s, g2, g2s, g3, g3s;
                twp(sl, 2, g0, g0s);
                twp(sl, 4, g1, g1s);
                twp(sl, 6, g2, g2s);
                twp(sl, 8, g3, g3s);
                dft4x2_fused_v<1>(bb + 0, bb + 4, g0, g0s, g1, g1s);
                dft4x2_fused_v<1>(bb + 8, bb + 12, g2, g2s, g3, g3s);
            } else {
            static_for<0, 4>([&](auto c) {
                constexpr int i2 = decltype(c)::value;
                if constexpr (FUSED >= 1)
                    dft4_fused_v<4>(bb + i2, v, v2);
                else
                    dft4_geo_v<4>(bb + i2, v, v2);   // column i2's X[k1] at slot i2 + 4 k1
            });
            static_for<0, 4>([&](auto d) {
                constexpr int k1 = decltype(d)::value;
                if constexpr (FUSED >= 1)
                    dft4_fused_v<1>(bb + 4 * k1, twv(sl, 2 + 2 * k1), twv(sl, 3 + 2 * k1));
                else
                    dft4_geo_v<1>(bb + 4 * k1, twv(sl, 2 + 2 * k1), twv(sl, 3 + 2 * k1));
            });
            }
            f2 tt[16];
            static_for<0, 16>([&](auto e) {
                constexpr int m = decltype(e)::value;  // m = 4 k1 + k2 holds Z[col + 32 (k1 + 4 k2)]
                tt[(m / 4) + 4 * (m % 4)] = bb[m];
            });
            static_for<0, 16>([&](auto e) {
                constexpr int m = decltype(e)::value;
                bb[m] = tt[m];
            });
        }
        // b[k2] = Z[t + 32 k2], b[16 + k2] = Z[k1b + 32 k2] (unscaled)

        // 4. real post-pass over 16 mirror pairs, as fft1024_quad_kernel step 3
        //    with X[kP] = S/2 + (W/2) D and the powers of both mirrors per pair
        const bool l0 = (t == 0);
        float *pq = pw + q * kQPow;
        // SPL: float index of (|X[kP]|^2, |X[512 - kP]|^2) of pair j, as row
        // base + 32 j and mirror base + 32 (15 - j): lane t has kP = t + 32 j;
        // lane 0 has kP = 16 + 32 j for j < 8 (like t = 16) and 32 j for
        // j >= 8. Formed here from the lane id, fenced from hoisting, so the
        // four bases do not stay live across the group loop (with them the
        // kernel hit 128 VGPRs and spilled 20 B per lane).
        int tl = (int)(threadIdx.x & 63);
        if constexpr (SPL) asm volatile("" : "+v"(tl));
        const int tt = tl & 15, rowb = (tl >> 4) * 513;
        const int te_lo = tt == 0 ? 16 : tt;
        const int spl_a_lo = rowb + te_lo, spl_m_lo = rowb + 32 - te_lo;
        const int spl_a_hi = rowb + tt, spl_m_hi = rowb + 32 - tt;
        f2 *const ps = reinterpret_cast<f2 *>(pq) + t;  // slot (j, t) at ps[16 j]
        // !SPEC: this lane's powers, pv[2 j + half], one 32-register tuple so a
        // uniform index reads it with v_movrels (no scratch, no select chain)
        typedef float f32x32 __attribute__((ext_vector_type(32)));
        f32x32 pv;
        static_for<0, 8>([&](auto jc) {
            constexpr int j0 = 2 * decltype(jc)::value, j1 = j0 + 1;
            f2 pw0, pw1;  // (|X[kP]|^2, |X[512-kP]|^2)
            // PICK 2: only the pair blocks holding a tone bin (p.pmask,
            // wave-uniform: a scalar branch per block; the skipped blocks'
            // powers are undefined and never read, and only their values,
            // not the power tuple, merge at the branch). The empty asm
            // defines them without an instruction (left undefined, the
            // compiler zeroed them: 4 v_mov per block, executed or not)
            if constexpr (!SPEC && PICK == 2) asm volatile("" : "=v"(pw0), "=v"(pw1));
            const bool need = SPEC || PICK != 2 || ((p.pmask >> decltype(jc)::value) & 1u);
            if (need) {
            f2 P0 = b[j0], Q0 = b[16 + 15 - j0];
            f2 P1 = b[j1], Q1 = b[16 + 15 - j1];
            // lane 0 (columns 0 and 16): pairs j < 8 are column 16's
            // (Z[16 + 32 j], mirror in the default Q slot), pairs j >= 8
            // column 0's (Z[32 j] with Z[32 (16 - j)]; j = 8 is Z[256] with
            // itself): 16 selects instead of 24 for the layout before
            if constexpr (j0 < 8) {
                P0 = sel_l0(b[16 + j0], P0);
                P1 = sel_l0(b[16 + j1], P1);
            } else {
                Q0 = sel_l0(b[16 - j0], Q0);
                Q1 = sel_l0(b[16 - j1], Q1);
            }
            f2 w0, w1;
            if constexpr (RD >= 2) {
                const f4 x = *reinterpret_cast<const f4 *>(&tw3[tw3_at(j0, t)]);
                w0 = (f2){x.x, x.y};
                w1 = (f2){x.z, x.w};
            } else if constexpr (TW3R) {
                // W1024^kP / 2 = base x W32^j (j0 = 0 and j0 + 1 = 8 ... cheap cases)
                const f2 b0 = j0 < 8 ? tb_lo : tb_hi, b1 = j1 < 8 ? tb_lo : tb_hi;
                if constexpr (j0 == 0) {
                    w0 = b0;
                    w1 = cmulk(b1, w32c<j1>());
                } else if constexpr (j0 == 8) {
                    w0 = mj(b0);
                    w1 = cmulk(b1, w32c<j1>());
                } else {
                    cmulk2(w0, b0, w32c<j0>(), w1, b1, w32c<j1>());
                }
            } else {
                w0 = tw3[tw3_at(j0, t)];
                w1 = tw3[tw3_at(j1, t)];
            }
            if constexpr (FUSED >= 2) {
                postpair2(pw0, P0, Q0, w0, pw1, P1, Q1, w1);
            } else {
                const f2 S0 = pp_s(P0, Q0), S1 = pp_s(P1, Q1);
                const f2 D0 = pp_d(P0, Q0), D1 = pp_d(P1, Q1);
                f2 T0, T1;
                cmul2(T0, D0, w0, T1, D1, w1);
                const f2 re0 = pp_re_h(S0, T0), re1 = pp_re_h(S1, T1);
                const f2 im0 = pp_im_h(S0, T0), im1 = pp_im_h(S1, T1);
                pwr2(pw0, re0, im0, pw1, re1, im1);
            }
            }
            if constexpr (SPEC && SPL) {
                const int a = j0 < 8 ? spl_a_lo : spl_a_hi, m = j0 < 8 ? spl_m_lo : spl_m_hi;
                pw[a + 32 * j0] = pw0.x;
                pw[m + 32 * (15 - j0)] = pw0.y;
                pw[a + 32 * j1] = pw1.x;
                pw[m + 32 * (15 - j1)] = pw1.y;
            } else if constexpr (SPEC) {
                ps[16 * j0] = pw0;
                ps[16 * j1] = pw1;
            } else {
                pv[2 * j0] = pw0.x;
                pv[2 * j0 + 1] = pw0.y;
                pv[2 * j1] = pw1.x;
                pv[2 * j1 + 1] = pw1.y;
            }
        });
        // lane 0's X[0] = Re Z[0] + Im Z[0] and X[512] = Re Z[0] - Im Z[0]
        f2 px;
        asm("v_pk_add_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(px) : "v"(b[0]));
        px = px * px;
        const bool live = w < p.n_windows;
        float pk = -1.f, pk2 = -1.f;  // the best (and runner-up) tone power this lane holds
        int arg = t < p.k ? t : kMaxTones;  // kMaxTones: this lane holds no tone
        if constexpr (SPEC) {
            if (l0) {
                if constexpr (SPL) {
                    pw[rowb] = px.x;
                    pw[rowb + 512] = px.y;
                } else {
                    pq[512] = px.x;
                    pq[513] = px.y;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // 5. tone pick (as fft1024_quad_kernel step 4)
            if (t < p.k) pk = SPL ? pw[rowb + mybin] : pq[myslot];
            // SPL: the fenced lane id again, so the store address is formed
            // here rather than held across the loop
            if (live && t < p.k && p.mag) p.mag[w * p.k + (SPL ? tt : t)] = pk;
        } else if constexpr (PICK == 1 || PICK == 2) {
            // 5. tone pick, gathered: tone i's power (register slot and lane
            //    from its uniform slot, as below) is read across the row with
            //    one ds_bpermute into lane t = i, so lanes t < K end holding
            //    tone t's power, as the slab pick of the spectrum path leaves
            //    them: one coalesced magnitude store and the same row argmax
            float mine = -1.f;
#pragma nounroll
            for (int i = 0; i < p.k; ++i) {
                const int f = p.slot[i];
                const float v = f >= 512 ? (f == 512 ? px.x : px.y) : pv[((f >> 5) << 1) | (f & 1)];
                const int src = f >= 512 ? 0 : ((f >> 1) & 15);
                const float got = __int_as_float(
                    __builtin_amdgcn_ds_bpermute(rowaddr + 4 * src, __float_as_int(v)));
                mine = t == i ? got : mine;
            }
            pk = mine;
            if (live && t < p.k && p.mag) p.mag[w * p.k + t] = pk;
        } else {
            // 5. tone pick from registers: tone i's power sits in lane
            //    (slot >> 1) & 15 of each window row at pv[slot >> 5 | half]
            //    (uniform index); each lane keeps the best tone it owns (first
            //    index on ties), then the row argmax below
            arg = kMaxTones;
#pragma unroll
            for (int i = 0; i < kMaxTones; ++i) {
                if (i >= p.k) break;
                const int f = p.slot[i];
                const bool own = f >= 512 ? l0 : t == ((f >> 1) & 15);
                const float val = f >= 512 ? (f == 512 ? px.x : px.y) : pv[((f >> 5) << 1) | (f & 1)];
                if (own && live && p.mag) p.mag[w * p.k + i] = val;
                if (own && val > pk) {
                    pk2 = pk;
                    pk = val;
                    arg = i;
                } else if (own && val > pk2) {
                    pk2 = val;
                }
            }
        }
        // row argmax, ties to the lowest tone: the two DPP max passes of
        // window_sum.h (powers >= 0, so their bits order as unsigned)
        const bool owns = arg < kMaxTones;
        float mx;
        arg = (int)ws_argmax_m<false>(__float_as_uint(pk), owns, arg, 0u, false, 0, mx);
        // decision rescue: a runner-up within the threshold
        // decision rescue, two stages: the int16 worst case,
        // then (only waves with a stage-1 flag) the window's energy by
        // Parseval, E = 2 x the sum of its 513 bin powers >= n sum x^2 (the
        // row's lanes hold every bin once, bin 256 twice in the register
        // tuple: an upper bound either way)
        auto efn = [&]() {
            float e = 0.f;
            if constexpr (SPEC && SPL) {
                // the fenced lane id again (as the stores below): the row
                // base is not kept live from the post-pass
                int tl2 = (int)(threadIdx.x & 63);
                asm volatile("" : "+v"(tl2));
                const float *row = pw + (tl2 >> 4) * 513;
                for (int i = tl2 & 15; i < 513; i += 16) e += row[i];
            } else if constexpr (SPEC) {
                for (int i = t; i < 513; i += 16) e += pq[quad_slot(i)];
            } else if constexpr (PICK == 2) {
                // not every bin's power exists here: n sum x^2 from the
                // window's samples, read again (L2; only waves stage 1
                // flagged), lane t's 64 (dwords t + 16 n1)
                if (live) {
                    const uint32_t *src = reinterpret_cast<const uint32_t *>(p.pcm + w * p.hop) + t;
#pragma unroll
                    for (int n1 = 0; n1 < 32; ++n1) {
                        const uint32_t d = src[16 * n1];
                        const float lo = (float)(int16_t)(d & 0xFFFFu), hi = (float)(int16_t)(d >> 16);
                        e = __builtin_fmaf(lo, lo, e);
                        e = __builtin_fmaf(hi, hi, e);
                    }
                }
                return 1024.f * row_sum16(e);
            } else {
                f2 a = {0.f, 0.f};
#pragma unroll
                for (int i = 0; i < 32; i += 2) a = a + f2{pv[i], pv[i + 1]};
                e = (a.x + a.y) + (l0 ? px.x + px.y : 0.f);
            }
            return 2.f * row_sum16(e);
        };
        const bool amb = p.k >= 2 && ws_amb_two_stage(mx, pk, owns, pk2, pk2 >= 0.f, live, p.amb_tq,
                                                      p.amb_floor, p.amb_t2e, efn);
        if (live && t == 0) p.sym[w] = (uint8_t)(arg | (amb ? kSymAmbiguous : 0));
        if constexpr (SPEC && SPL) {
            if constexpr (PF == 2) {
                // the next group's loads go out ahead of this group's spectrum
                // stores: vmcnt retires in order, so waiting for those loads
                // no longer waits for these stores to be acknowledged
                __builtin_amdgcn_sched_barrier(0);
                load_group(g + stride < n_groups ? g + stride : g);
                __builtin_amdgcn_sched_barrier(0);
            }
            if (p.spec) {
                // the group's live windows: floats [0, L) of the slab = the
                // output run from window 4 g (16-byte aligned: 4 g x 513 x 4 B)
                const long long wg = 4 * g;
                const int L = 513 * (int)(p.n_windows - wg < 4 ? p.n_windows - wg : 4);
                float *dst = p.spec + wg * 513;
                const f4 *src4 = reinterpret_cast<const f4 *>(pw);
#pragma unroll
                for (int i = 0; i < 9; ++i) {
                    const int f = 64 * i + lane;
                    if (4 * f + 4 <= L) {
                        if constexpr (SPL == 2)
                            __builtin_nontemporal_store(src4[f], reinterpret_cast<f4 *>(dst + 4 * f));
                        else
                            *reinterpret_cast<f4 *>(dst + 4 * f) = src4[f];
                    } else if (4 * f < L) {
                        for (int e = 4 * f; e < L; ++e) dst[e] = pw[e];
                    }
                }
            }
        } else if constexpr (SPEC) {
            if (p.spec && live) {
                float *so = p.spec + w * 513;
                for (int i = t; i < 513; i += 16) so[i] = pq[quad_slot(i)];
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
    }

    // 6. decision rescue (rescue_fft.h), after the group loop
    //    (no code inside it, whose registers stay as they were): the symbol
    //    bytes of the groups are read back (one byte per window, plain loads:
    //    the bytes were written by this wave or its block) and every
    //    flagged window is decided again in double, one window per wave at a
    //    time through the wave's slab.
    //    RSC 1: each wave its own groups' windows.
    //    RSC 2: the block's flagged windows dealt round-robin to its waves, 64
    //    groups per wave at a time; every wave reads a chunk's bytes before
    //    any rescue rewrites them (the barrier), so all deal the same list.
    //    RSC 0: no rescue code (probe A/B).
    auto rescue_one = [&](long long ww, lds_double *xs) {
        rescue_fft_window(p.pcm + ww * p.hop, xs, reinterpret_cast<const double2 *>(p.rtw), p.bins, p.k,
                          p.sym + ww, p.mag ? p.mag + ww * p.k : nullptr, p.spec ? p.spec + ww * 513 : nullptr);
    };
    auto flags4 = [&](long long gl) {  // bit q: window 4 gl + q is flagged
        unsigned f = 0;
        if (gl < n_groups) {
#pragma unroll
            for (int q0 = 0; q0 < 4; ++q0) {
                const long long ww = 4 * gl + q0;
                if (ww < p.n_windows && (p.sym[ww] & kSymAmbiguous)) f |= 1u << q0;
            }
        }
        return f;
    };
    if constexpr (RSC == 1) {
        if (p.rescue) {
            // this wave's symbol stores have landed (in this XCD's L2, where
            // the plain loads below find them) and are ordered before the loads
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
            lds_double *xs = (lds_double *)(slab[wave]);
            bool rescan = true;  // the double FFTs' scan (below) has work
            if (p.t2e64 > 0.0 && !p.spec) {
                // first pass over each flagged group's windows, one per row
                // (rescue_fft_seg), where it is cheaper than their double
                // FFTs: it costs ~k x 200 double operations per lane for the
                // whole group, a double FFT ~800 per flagged window (at k = 8
                // and ~1.8 flagged windows per group both cost the same,
                // profiles/round4/r4l/). It clears the flag of every window
                // it decides; the loop below then finds only what it left.
                // (A separate loop: folded into the one below it made that
                // loop's double FFTs 30 % slower, profiles/round4/r4n/.)
                // (a wave that finds no flagged window here, nearly all of
                // them, skips the second scan of its symbol bytes)
                bool any = false;
                for (long long gb = g_first; gb < n_groups; gb += 64 * stride) {
                    const unsigned f = flags4(gb + (long long)lane * stride);
                    unsigned long long m = __ballot(f != 0);
                    any = any || m != 0;
                    while (m) {
                        const int src = __builtin_ctzll(m);
                        m &= m - 1;
                        const unsigned fs = (unsigned)__builtin_amdgcn_readlane((int)f, src);
                        if (p.k > 4 * __builtin_popcount(fs)) continue;
                        const long long gs = gb + (long long)src * stride;
                        const int row = lane >> 4;
                        const long long ww = 4 * gs + row;
                        const bool amb = (fs >> row) & 1u;
                        (void)rescue_fft_seg(p.pcm + (amb ? ww : 0) * p.hop, p.rot64, p.t2e64, p.k, lane & 15,
                                             amb, p.sym + ww, p.mag ? p.mag + ww * p.k : nullptr, p.fold64 != 0);
                    }
                }
                __builtin_amdgcn_s_waitcnt(0);
                __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
                rescan = any;
            }
            for (long long gb = g_first; rescan && gb < n_groups; gb += 64 * stride) {
                const unsigned f = flags4(gb + (long long)lane * stride);
                unsigned long long m = __ballot(f != 0);
                while (m) {
                    const int src = __builtin_ctzll(m);
                    m &= m - 1;
                    const unsigned fs = (unsigned)__builtin_amdgcn_readlane((int)f, src);
                    const long long gs = gb + (long long)src * stride;
                    for (int q0 = 0; q0 < 4; ++q0)
                        if ((fs >> q0) & 1u) rescue_one(4 * gs + q0, xs);
                }
            }
        }
    } else if constexpr (RSC == 2) {
        if (p.rescue) {
            __builtin_amdgcn_s_waitcnt(0);  // this wave's symbol stores have landed
            __syncthreads();                // ... and every wave's of the block (a workgroup fence)
            lds_double *xs = (lds_double *)(slab[wave]);
            int seen = 0;                   // flagged windows dealt so far (wave-uniform)
            for (long long gb0 = g_first - wave; gb0 < n_groups; gb0 += 64 * stride) {
                unsigned f[WPB];
#pragma unroll
                for (int wv = 0; wv < WPB; ++wv) f[wv] = flags4(gb0 + wv + (long long)lane * stride);
                __syncthreads();
#pragma unroll
                for (int wv = 0; wv < WPB; ++wv) {
                    unsigned long long m = __ballot(f[wv] != 0);
                    while (m) {
                        const int src = __builtin_ctzll(m);
                        m &= m - 1;
                        const unsigned fs = (unsigned)__builtin_amdgcn_readlane((int)f[wv], src);
                        const long long gs = gb0 + wv + (long long)src * stride;
                        for (int q0 = 0; q0 < 4; ++q0)
                            if ((fs >> q0) & 1u) {
                                if (seen++ % WPB != wave) continue;
                                rescue_one(4 * gs + q0, xs);
                            }
                    }
                }
            }
        }
    }
}

template <int WPB = 4, int MINW = 4, int PF = 0, bool SPEC = true, bool FMT = false, int AUX = 2,
          int FUSED = 0, int SPL = 0, int OVL = 0, int TW3R = 0, int RSC = 1, int PICK = 0>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MINW > 0 ? MINW : 1)))
void fft1024_quad_kernel(FftParams p)
{
    fft1024_quad_body<WPB, MINW, PF, SPEC, FMT, AUX, FUSED, 0, SPL, OVL, TW3R, RSC, PICK>(p);
}

// (a device-code attribute: the host pass of hipcc does not know the feature)
#if defined(__HIP_DEVICE_COMPILE__)
#define FSKD_NO_LDS_PAIRING __attribute__((target("no-load-store-opt")))
#else
#define FSKD_NO_LDS_PAIRING
#endif
// The same kernel without the backend's LDS-access pairing: the transpose's
// column reads and the twiddle-table reads stay ds_read_b64 (2 LDS cycles per
// wave, 256 B/clk) instead of being merged into ds_read2_b64 (8 cycles for
// twice the bytes, 128 B/clk; MI355X_MICROARCH.md §LDS). RD 2: also the
// twiddle tables lane-major, one ds_read_b128 (4 cycles) per twiddle pair.
template <int WPB = 4, int MINW = 4, int PF = 0, bool SPEC = true, bool FMT = false, int AUX = 2,
          int FUSED = 0, int RD = 1>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MINW > 0 ? MINW : 1)))
FSKD_NO_LDS_PAIRING void fft1024_quad_kernel_r64(FftParams p)
{
    fft1024_quad_body<WPB, MINW, PF, SPEC, FMT, AUX, FUSED, RD>(p);
}

// Persistent grid: as many blocks as fit the chip, each wave strides over
// groups of 4 windows (the LDS twiddle tables are built once per block).
template <int WPB, int MINW, int PF, bool SPEC, bool FMT = false, int AUX = 2, int FUSED = 0, int RD = 0,
          int SPL = 0, int OVL = 0, int TW3R = 0, int RSC = 1, int PICK = 0>
hipError_t launch_fft_quad_t(const FftParams &p, hipStream_t s)
{
    void (*kern)(FftParams);
    static_assert(!(RD > 0 && (SPL > 0 || OVL > 0 || TW3R > 0)), "SPL / OVL / TW3R: fft1024_quad_kernel only");
    if constexpr (RD > 0)
        kern = fft1024_quad_kernel_r64<WPB, MINW, PF, SPEC, FMT, AUX, FUSED, RD>;
    else
        kern = fft1024_quad_kernel<WPB, MINW, PF, SPEC, FMT, AUX, FUSED, SPL, OVL, TW3R, RSC, PICK>;
    int dev = 0, cus = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64 * WPB, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const long long groups = (p.n_windows + 3) / 4;
    long long blocks = (groups + WPB - 1) / WPB;
    blocks = std::min<long long>(blocks, (long long)cus * per_cu);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64 * WPB), 0, s, p);
    return hipGetLastError();
}

// Shipped: 4-wave blocks, 4 waves/SIMD, loads at the top of each group, the
// register tone pick unless the full spectrum is asked for
// (scripts/fft_probe.hip, profiles/round2/fft/). Load policy: windows that
// overlap (hop < n) are read by up to n / hop groups, so their loads keep the
// lines in L2 (plain cached loads, AUX 0: FETCH 1.06x the stream at hop 256,
// 3-6 % faster; sc0 measured the same or slower); disjoint windows stream
// through with nt (AUX 2; nt at hop 256 re-fetches 1.55x the stream).
// FUSED 4: the DFT-4 stages (stage 2: two interleaved per block), the
// DFT-32's trivial pieces and the post-pass pairs as single asm blocks
// (-3 to -4.5 % at hop 256, -2 to -4 % at hop 1024 against separate blocks;
// scripts/fft_probe.hip, profiles/round2/fft_fused/).
// The full-spectrum store (p.spec) goes through the linear slab with
// non-temporal 16-byte stores (SPL 2) when the output is 16-byte aligned,
// else through the quad_slot slab. Hop 256, 4.19 M windows, 8.6 GB of
// spectrum: quad_slot slab 4.00-4.12 ms, linear slab 2.85-2.89 ms, + nt
// 2.73 ms; a write-only fill of the same buffer 1.45 ms, the detector
// without the spectrum 1.71-1.80 ms (scripts/spectrum_probe.py,
// profiles/round2/spec_lin/).
// Tones only: the gathered tone pick (PICK 1), -1.8 % at hop 256 and -1.7 %
// at hop 1024 against the per-lane register pick, identical outputs
// (profiles/round3/r3s/); round 5: only the post-pass blocks holding a tone
// bin (PICK 2, -13 %), with round 1 of the transpose overlapping column 0's
// DFT-16 (OVL: within +-0.5 % on the full post-pass, -2.7 % once the VALU
// stream had shrunk; the twiddles from registers, TW3R, another -1 % but
// other bits than the table's, not taken; profiles/round5/r5zp/).
hipError_t launch_fft_quad(const FftParams &p, hipStream_t s)
{
    const bool lin = p.spec && ((uintptr_t)p.spec & 15) == 0;
    if (p.hop < 1024) {
        if (lin) return launch_fft_quad_t<4, 4, 0, true, false, 0, 4, 0, 2>(p, s);
        if (p.spec) return launch_fft_quad_t<4, 4, 0, true, false, 0, 4>(p, s);
        return p.pmask == 0xFFu ? launch_fft_quad_t<4, 4, 0, false, false, 0, 4, 0, 0, 0, 0, 1, 1>(p, s)
                                : launch_fft_quad_t<4, 4, 0, false, false, 0, 4, 0, 0, 1, 0, 1, 2>(p, s);
    }
    if (lin) return launch_fft_quad_t<4, 4, 0, true, false, 2, 4, 0, 2>(p, s);
    if (p.spec) return launch_fft_quad_t<4, 4, 0, true, false, 2, 4>(p, s);
    return p.pmask == 0xFFu ? launch_fft_quad_t<4, 4, 0, false, false, 2, 4, 0, 0, 0, 0, 1, 1>(p, s)
                            : launch_fft_quad_t<4, 4, 0, false, false, 2, 4, 0, 0, 1, 0, 1, 2>(p, s);
}

int fft_quad_slot(int bin) { return quad_slot(bin); }

// The post-pass pair blocks (pairs 2 jb, 2 jb + 1) the tone bins sit in
// (quad_slot: pair j = slot >> 5; bins 0 and 512 come from Z[0] on the side)
unsigned fft_quad_pmask(const int *bins, int k)
{
    unsigned m = 0;
    for (int i = 0; i < k; ++i) {
        const int f = quad_slot(bins[i]);
        if (f < 512) m |= 1u << ((f >> 5) >> 1);
    }
    return m;
}

}  // namespace fskd
