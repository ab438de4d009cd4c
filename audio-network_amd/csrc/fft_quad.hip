// fft_quad.hip — the full-spectrum detector laid
// out as 16 lanes per window, 4 windows per wave. Same contract as
// fft1024_kernel (fft.hip): per window a 1024-point real FFT, |X[b]|^2 for
// b = 0..512, symbol = argmax over the tone bins (ties -> lowest k). Oracle:
// oracle/fsk_oracle.c:oracle_fft_demod.
//
// z[n] = x[2n] + i x[2n+1] (n < 512) is a 512-point complex FFT, split 32 x 16:
//   n = t + 16 n1 (t = lane % 16, n1 < 32),   k = k1 + 32 k2 (k1 < 32, k2 < 16)
//   Z[k1 + 32 k2] = sum_t W16^{t k2} W512^{t k1} sum_n1 z[t + 16 n1] W32^{n1 k1}
//   1. lane t loads its 32 dwords z[t + 16 n1] (16 lanes = 64 contiguous bytes
//      per instruction) and runs a DFT-32 in registers, then multiplies by
//      W512^{t k1} (block LDS table, broadcast across the 4 windows);
//   2. ONE transpose through LDS: row t -> columns. Lane t' takes the column
//      pair {k1, 32 - k1} (lane 0: {0, 16}) and runs two DFT-16 in registers;
//   3. the real-FFT post-pass pairs Z[k] with conj Z[512 - k]. With the column
//      pairing above that mirror lives in the same lane, so it needs no
//      exchange: per pair one twiddle product gives both |X[k]|^2 and
//      |X[512 - k]|^2.
// LDS traffic per window: 4 KiB written + 4 KiB read for the transpose, plus
// 2 KiB of bin powers for the tone pick — against 12 + 12 KiB for the
// 64-lane radix-8 Stockham layout (fft.hip), whose LDS writes bound it (guide:
// ds_write aggregates 38-51 TB/s).
#include <algorithm>
#include <type_traits>

#include "demod_internal.h"

namespace fskd {
namespace quad {

// A complex number as a packed fp32 pair: complex add/sub is one v_pk_add_f32,
// a complex product two packed ops. CDNA4 runs a packed op at the same flop
// rate as two plain ones, but one wave issues half as many instructions — and
// this kernel is issue-bound (one wave/SIMD issues a VALU op every 4 cycles).
typedef float f2 __attribute__((ext_vector_type(2)));

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

// The real post-pass of two mirror pairs in one block (step 3 of the kernel):
// S = P + conj Q, D = -i (P - conj Q), T = W D, then
// pw = (|S + T|^2, |S - T|^2 with the imaginary part of S - T conjugated), i.e.
// (|X[kP]|^2, |X[512 - kP]|^2). Sixteen packed ops, ordered so that no result
// feeds the next instruction: one asm block, because the compiler pads every
// asm boundary whose last write is read next with an s_nop (gfx950 packed-fp32
// write -> dependent read hazard), and a chain of small blocks is all
// boundaries.
__device__ __forceinline__ void post_pair2(f2 &pw0, f2 P0, f2 Q0, f2 W0, f2 &pw1, f2 P1, f2 Q1,
                                           f2 W1)
{
    f2 S0, S1, D0, D1, T0, T1, R0, R1, I0, I1;
    asm("v_pk_add_f32 %2, %12, %13 neg_hi:[0,1]\n\t"                              // S0
        "v_pk_add_f32 %3, %15, %16 neg_hi:[0,1]\n\t"                              // S1
        "v_pk_add_f32 %4, %12, %13 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]\n\t" // D0
        "v_pk_add_f32 %5, %15, %16 op_sel:[1,1] op_sel_hi:[0,0] neg_hi:[1,0]\n\t" // D1
        "v_pk_mul_f32 %6, %4, %14 op_sel:[1,1] op_sel_hi:[1,0]\n\t"               // t0
        "v_pk_mul_f32 %7, %5, %17 op_sel:[1,1] op_sel_hi:[1,0]\n\t"               // t1
        "v_pk_fma_f32 %6, %4, %14, %6 op_sel_hi:[0,1,1] neg_lo:[0,0,1]\n\t"       // T0 = W0 D0
        "v_pk_fma_f32 %7, %5, %17, %7 op_sel_hi:[0,1,1] neg_lo:[0,0,1]\n\t"       // T1
        "v_pk_add_f32 %8, %2, %6 op_sel_hi:[0,0] neg_hi:[0,1]\n\t"                // re pair 0
        "v_pk_add_f32 %9, %3, %7 op_sel_hi:[0,0] neg_hi:[0,1]\n\t"                // re pair 1
        "v_pk_add_f32 %10, %2, %6 op_sel:[1,1] neg_hi:[0,1]\n\t"                  // im pair 0
        "v_pk_add_f32 %11, %3, %7 op_sel:[1,1] neg_hi:[0,1]\n\t"                  // im pair 1
        "v_pk_mul_f32 %4, %10, %10\n\t"                                            // im0^2
        "v_pk_mul_f32 %5, %11, %11\n\t"                                            // im1^2
        "v_pk_fma_f32 %0, %8, %8, %4\n\t"                                          // pw0
        "v_pk_fma_f32 %1, %9, %9, %5"                                                // pw1
        : "=&v"(pw0), "=&v"(pw1), "=&v"(S0), "=&v"(S1), "=&v"(D0), "=&v"(D1), "=&v"(T0),
          "=&v"(T1), "=&v"(R0), "=&v"(R1), "=&v"(I0), "=&v"(I1)
        : "v"(P0), "v"(Q0), "v"(W0), "v"(P1), "v"(Q1), "v"(W1));
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

}  // namespace quad

// Per-wave LDS: 4 windows x 16 rows x 17 complex (8704 B). The transpose
// moves half the columns per round (k1 < 16, then k1 >= 16), so only half of
// the DFT-32 output and half of the DFT-16 input are live at once. Row stride
// 34 words: the 16 lanes of a row write (ds_write_b64) cover 32 banks; the
// window stride 544 words = 32 mod 64 puts odd windows on the other 32, so a
// 32-lane pass of writes or column reads is conflict-free. Reused for the bin
// powers (4 x 513 floats).
// Bin powers after step 3, per window (stride kQPow floats): pair j of lane t
// stores (|X[kP]|^2, |X[512 - kP]|^2) as one f2 at slot 16 j + t; |X[256]|^2
// sits at float 512. quad_slot(b) is the float index of bin b.
constexpr int kQPow = 544;  // floats per window: 8-byte aligned, odd windows on the other 32 banks
__host__ __device__ constexpr int quad_slot(int b)
{
    if (b == 256) return 512;
    const int u = b & 31, v = b >> 5;
    if (u == 0) return v < 8 ? 2 * (16 * v) : 2 * (16 * (16 - v)) + 1;  // lane 0: kP = 32 j
    if (u == 16) return v < 8 ? 2 * (16 * (v + 8)) : 2 * (16 * (23 - v)) + 1;  // lane 0, j >= 8
    if (u < 16) return 2 * (16 * v + u);                 // kP = t + 32 j
    return 2 * (16 * (15 - v) + (32 - u)) + 1;           // mirror 512 - kP
}

constexpr int kQRow = 17;            // complex per row (16 + 1 pad)
constexpr int kQWin = 16 * kQRow;    // complex per window
constexpr int kQSlab = 4 * kQWin;    // complex per wave
static_assert(4 * kQPow <= 2 * kQSlab, "bin powers of 4 windows must fit the slab");

// MINW > 0 asks the compiler for MINW waves per SIMD (VGPR budget 512 / MINW).
// SPLIT: the next group's 32 loads go out in two halves — the 16 dwords the
// first two DFT-8 columns of stage 1 need (n1 % 4 < 2) during the transpose,
// the rest after the post-pass — so only 16 prefetch VGPRs are live across
// the DFT-16 and post-pass.
// FUSE: step 3 as one asm block per two pairs (post_pair2) instead of the
// cmul2 / pwr2 pieces: 23 -> 8 hazard nops but 142 -> 160 VGPRs, and the same
// time (interleaved A/B, profiles/round1/probe_fft_fuse.log), so off.
// FMT: load z[t + 16 n1] with a typed buffer load (DATA_FORMAT 16_16,
// NUM_FORMAT SSCALED): the texture path converts both int16 halves to fp32,
// replacing the 64 VALU converts per group (exact for every int16).
namespace quad {
typedef int i4 __attribute__((ext_vector_type(4)));
__device__ f2 raw_buffer_load_format_v2f32(i4 rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.format.v2f32");
// buffer descriptor word 3: DST_SEL x,y,z,w = 4,5,6,7; NUM_FORMAT 3 (SSCALED);
// DATA_FORMAT 5 (16_16)
constexpr int kFmtWord3 = 0xFAC | (3 << 12) | (5 << 15);
}  // namespace quad

template <int WPB = 4, int MINW = 0, bool SPLIT = false, bool FUSE = false, bool FMT = false>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MINW > 0 ? MINW : 1)))
void fft1024_quad_kernel(FftParams p)
{
    using namespace quad;
    __shared__ __attribute__((aligned(16))) f2 slab[WPB][kQSlab];
    __shared__ f2 tw1[31 * 16];  // W512^{t k1} / 2 at [k1 - 1][t]
    __shared__ f2 tw3[16 * 16];  // post-pass W1024^{kP(t, j)} at [j][t]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: tile bases stay in SGPRs (no waterfall loop per buffer load)
    const int q = lane >> 4;   // window of the wave
    const int t = lane & 15;   // row / column-pair index
    const f2 *t512 = reinterpret_cast<const f2 *>(p.tw512);
    const f2 *t1024 = reinterpret_cast<const f2 *>(p.tw1024);
    // The real split X = (S + W D)/2 needs Z/2: the 1/2 rides on the stage-1
    // twiddles (and column 0), exact in binary floating point.
    for (int i = threadIdx.x; i < 31 * 16; i += 64 * WPB)
        tw1[i] = 0.5f * t512[((i & 15) * ((i >> 4) + 1)) & 511];
    // post-pass twiddles W1024^kP for bin kP(t, j) (step 3): t + 32 j, and
    // for t = 0, j >= 8: 16 + 32 (j - 8)
    for (int i = threadIdx.x; i < 16 * 16; i += 64 * WPB) {
        const int tt = i & 15, j = i >> 4;
        tw3[i] = t1024[(tt == 0 && j >= 8) ? 16 + 32 * (j - 8) : tt + 32 * j];
    }
    const int k1b = t == 0 ? 16 : 32 - t;
    const int myslot = quad_slot(t < p.k ? p.bins[t] : 0);
    float *pw = reinterpret_cast<float *>(slab[wave]);
    __syncthreads();

    const long long n_groups = (p.n_windows + 3) >> 2;
    const long long stride = (long long)gridDim.x * WPB;
    long long g = tile_block(p.xcd_swizzle) * WPB + wave;
    uint32_t nx[FMT ? 1 : 32];
    f2 nxf[FMT ? 32 : 1];
    // One buffer descriptor per group (wave-uniform base = its first window);
    // the lane offset is the window's start + 4 t bytes, and z[t + 16 n1] is
    // the immediate offset 64 n1 (< 4 KiB), so the 32 loads need no address
    // arithmetic. Windows past the end are clamped to the last (never stored).
    auto load_group = [&](long long gg, int half) {  // half: 0 / 1 of SPLIT, 2 = all
        const long long w0 = 4 * gg;
        const long long left = p.n_windows - w0;  // >= 1
        const int wq = q < left ? q : (int)left - 1;
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
                if (half == 2 || ((n1 & 3) < 2) == (half == 0))
                    nxf[n1] = raw_buffer_load_format_v2f32(rf, voff + 64 * n1, 0, 2);
        } else {
#pragma unroll
            for (int n1 = 0; n1 < 32; ++n1)
                if (half == 2 || ((n1 & 3) < 2) == (half == 0))
                    nx[n1] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff + 64 * n1, 0, 2);
        }
    };
    if (g < n_groups) load_group(g, 2);
    for (; g < n_groups; g += stride) {
        const long long w = 4 * g + q;
        f2 a[32];
#pragma unroll
        for (int n1 = 0; n1 < 32; ++n1) {
            if constexpr (FMT) {
                a[n1] = nxf[n1];
                continue;
            }
            a[n1] = (f2){(float)(int)(short)(nx[FMT ? 0 : n1] & 0xFFFFu), (float)((int)nx[FMT ? 0 : n1] >> 16)};
            // opaque: otherwise the compiler rewrites (float)a + (float)b as
            // (float)(a + b) and the first butterflies become 2 integer ops +
            // 2 converts each instead of one packed add
            asm("" : "+v"(a[n1]));
        }

        // 1. DFT-32 over n1, twiddle W512^{t k1} (and the 1/2 of the real split)
        dft<32>(a);
        a[0] *= 0.5f;
#pragma unroll
        for (int k1 = 1; k1 < 31; k1 += 2)
            cmul2(a[k1], a[k1], tw1[16 * (k1 - 1) + t], a[k1 + 1], a[k1 + 1], tw1[16 * k1 + t]);
        a[31] = cmul(a[31], tw1[16 * 30 + t]);

        // 2. transpose in two column rounds; lane (q, t') gets columns
        //    k1 = t' (round 0) and k1b (round 1) of its window
        f2 b[32];  // b[n2] = Y[n2][t'], b[16 + n2] = Y[n2][k1b]
        f2 *win = slab[wave] + q * kQWin;
#pragma unroll
        for (int r = 0; r < 2; ++r) {
#pragma unroll
            for (int c = 0; c < 16; ++c) win[t * kQRow + c] = a[16 * r + c];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (r == 0) {
                // prefetch the next group here, where half of the DFT-32 output
                // is already in LDS (unconditional, clamped: one basic block)
                load_group(g + stride < n_groups ? g + stride : g, SPLIT ? 0 : 2);
            }
            const int col = r == 0 ? t : k1b - 16;
#pragma unroll
            for (int n2 = 0; n2 < 16; ++n2) b[16 * r + n2] = win[n2 * kQRow + col];
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        dft<16>(b);
        dft<16>(b + 16);
        // b[k2] = Z[t + 32 k2], b[16 + k2] = Z[k1b + 32 k2]

        // 3. real post-pass over 16 mirror pairs (P_j, Q_j = Z[512 - kP]):
        //    t > 0:  P = Za[j], Q = Zb[15 - j], kP = t + 32 j
        //    t = 0:  j < 8: P = Za[j], Q = Za[(16 - j) % 16], kP = 32 j
        //            j >= 8: P = Zb[j - 8], Q = Zb[23 - j], kP = 16 + 32 (j - 8)
        //    X[kP] = (S + W D)/2, X[512 - kP] = conj(S - W D)/2 with
        //    S = P + conj Q, D = -i (P - conj Q), W = W1024^kP (b holds Z/2,
        //    so S + W D is X itself).
        const bool l0 = (t == 0);
        float *pq = pw + q * kQPow;
        f2 *const ps = reinterpret_cast<f2 *>(pq) + t;  // slot (j, t) at ps[16 j]
        // two pairs at a time (j, j + 1), so no packed result feeds the very
        // next instruction (cmul2 / pwr2)
        static_for<0, 8>([&](auto jc) {
            constexpr int j0 = 2 * decltype(jc)::value, j1 = j0 + 1;
            // lane 0's pairing, selected per lane with v_cndmask on a constant
            // lane mask (a C++ select of two b[] elements becomes a runtime
            // index into b, which sends b to scratch)
            f2 P0 = b[j0], Q0 = b[16 + 15 - j0];
            f2 P1 = b[j1], Q1 = b[16 + 15 - j1];
            if constexpr (j0 >= 8) {
                P0 = sel_l0(b[16 + j0 - 8], P0);
                P1 = sel_l0(b[16 + j1 - 8], P1);
            }
            if constexpr (j0 < 8) {
                Q0 = sel_l0(b[(16 - j0) & 15], Q0);
                Q1 = sel_l0(b[(16 - j1) & 15], Q1);
            } else {
                Q0 = sel_l0(b[16 + 23 - j0], Q0);
                Q1 = sel_l0(b[16 + 23 - j1], Q1);
            }
            f2 pw0, pw1;  // (|X[kP]|^2, |X[512-kP]|^2)
            if constexpr (FUSE) {
                post_pair2(pw0, P0, Q0, tw3[16 * j0 + t], pw1, P1, Q1, tw3[16 * j1 + t]);
            } else {
                const f2 S0 = pp_s(P0, Q0), S1 = pp_s(P1, Q1);
                const f2 D0 = pp_d(P0, Q0), D1 = pp_d(P1, Q1);
                f2 T0, T1;
                cmul2(T0, D0, tw3[16 * j0 + t], T1, D1, tw3[16 * j1 + t]);
                const f2 re0 = pp_re(S0, T0), re1 = pp_re(S1, T1);
                const f2 im0 = pp_im(S0, T0), im1 = pp_im(S1, T1);
                pwr2(pw0, re0, im0, pw1, re1, im1);
            }
            ps[16 * j0] = pw0;
            ps[16 * j1] = pw1;
        });
        // Z[256] is its own mirror: |X[256]|^2 = |Z[256]|^2 = 4 |b[8]|^2
        if (l0) pq[512] = 4.f * fmaf(b[8].x, b[8].x, b[8].y * b[8].y);
        if (SPLIT) load_group(g + stride < n_groups ? g + stride : g, 1);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // 4. tone pick: lane (q, i < K) reads bin power i, argmax over the
        //    16-lane row (ties -> lowest i), lane (q, 0) stores the symbol.
        const bool live = w < p.n_windows;
        float pk = -1.f;
        int arg = t;
        if (t < p.k) pk = pq[myslot];
        if (live && t < p.k && p.mag) p.mag[w * p.k + t] = pk;
        // row_ror:1,2,4,8 within the 16-lane row: every lane sees the whole row
        static_for<0, 4>([&](auto sc) {
            constexpr int ctrl = 0x120 + (1 << decltype(sc)::value);
            const float po = __int_as_float(
                __builtin_amdgcn_update_dpp(0, __float_as_int(pk), ctrl, 0xF, 0xF, false));
            const int ao = __builtin_amdgcn_update_dpp(0, arg, ctrl, 0xF, 0xF, false);
            const bool take = (po > pk) | ((po == pk) & (ao < arg));  // branch-free
            pk = take ? po : pk;
            arg = take ? ao : arg;
        });
        if (live && t == 0) p.sym[w] = (uint8_t)arg;
        if (p.spec && live) {
            float *so = p.spec + w * 513;
            for (int i = t; i < 513; i += 16) so[i] = pq[quad_slot(i)];
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// Persistent grid: as many blocks as fit the chip, each wave strides over
// groups of 4 windows (the LDS twiddle tables are built once per block).
template <int WPB, int MINW, bool SPLIT = false, bool FUSE = false, bool FMT = false>
hipError_t launch_fft_quad_t(const FftParams &p, hipStream_t s)
{
    int dev = 0, cus = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fft1024_quad_kernel<WPB, MINW, SPLIT, FUSE, FMT>,
                                                     64 * WPB, 0) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    const long long groups = (p.n_windows + 3) / 4;
    long long blocks = (groups + WPB - 1) / WPB;
    blocks = std::min<long long>(blocks, (long long)cus * per_cu);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL((fft1024_quad_kernel<WPB, MINW, SPLIT, FUSE, FMT>), dim3((unsigned)blocks), dim3(64 * WPB), 0,
                       s, p);
    return hipGetLastError();
}

hipError_t launch_fft_quad(const FftParams &p, hipStream_t s)
{
    return launch_fft_quad_t<4, 0>(p, s);
}

}  // namespace fskd
