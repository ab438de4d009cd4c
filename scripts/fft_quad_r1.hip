// fft_quad.hip — the full-spectrum detector laid
// out as 16 lanes per window, 4 windows per wave. Same contract as
// fft1024_kernel (scripts/fft_r0.hip): per window a 1024-point real FFT, |X[b]|^2 for
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
// 64-lane radix-8 Stockham layout (scripts/fft_r0.hip), whose LDS writes bound it (guide:
// ds_write aggregates 38-51 TB/s).
#include <algorithm>
#include <type_traits>

#include "../audio-network_amd/csrc/demod_internal.h"

namespace fskd { namespace r1 {
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
        // DFT-N1 over i1 for every i2 (stride N2 S), then twiddle W_N^{i2 k1}
        static_for<0, N2>([&](auto c) {
            constexpr int i2 = decltype(c)::value;
            dft<N1, N2 * S>(x + i2 * S);
            static_for<1, N1>([&](auto d) {
                constexpr int k1 = decltype(d)::value;
                x[(i2 + N2 * k1) * S] = w32<(i2 * k1) * (32 / N)>(x[(i2 + N2 * k1) * S]);
            });
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
constexpr int kQRow = 17;            // complex per row (16 + 1 pad)
constexpr int kQWin = 16 * kQRow;    // complex per window
constexpr int kQSlab = 4 * kQWin;    // complex per wave
static_assert(4 * 513 <= 2 * kQSlab, "bin powers of 4 windows must fit the slab");

template <int WPB = 4>
__global__ __launch_bounds__(64 * WPB) void fft1024_quad_kernel(FftParams p)
{
    using namespace quad;
    __shared__ __attribute__((aligned(16))) f2 slab[WPB][kQSlab];
    __shared__ f2 tw1[31 * 16];  // W512^{t k1} / 2 at [k1 - 1][t]
    __shared__ f2 tw3[16 * 16];  // post-pass W1024^{kP(t, j)} at [j][t]
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
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
    const int mybin = t < p.k ? p.bins[t] : 0;
    float *pw = reinterpret_cast<float *>(slab[wave]);
    __syncthreads();

    const long long n_groups = (p.n_windows + 3) >> 2;
    const long long stride = (long long)gridDim.x * WPB;
    long long g = tile_block(p.xcd_swizzle) * WPB + wave;
    uint32_t nx[32];
    auto load_group = [&](long long gg) {
        long long w = 4 * gg + q;
        if (w >= p.n_windows) w = p.n_windows - 1;  // clamped, never stored
        const uint32_t *xw = reinterpret_cast<const uint32_t *>(p.pcm + w * p.hop) + t;
#pragma unroll
        for (int n1 = 0; n1 < 32; ++n1) nx[n1] = __builtin_nontemporal_load(xw + 16 * n1);
    };
    if (g < n_groups) load_group(g);
    for (; g < n_groups; g += stride) {
        const long long w = 4 * g + q;
        f2 a[32];
#pragma unroll
        for (int n1 = 0; n1 < 32; ++n1) {
            a[n1] = (f2){(float)(int)(short)(nx[n1] & 0xFFFFu), (float)((int)nx[n1] >> 16)};
            // opaque: otherwise the compiler rewrites (float)a + (float)b as
            // (float)(a + b) and the first butterflies become 2 integer ops +
            // 2 converts each instead of one packed add
            asm("" : "+v"(a[n1]));
        }

        // 1. DFT-32 over n1, twiddle W512^{t k1} (and the 1/2 of the real split)
        dft<32>(a);
        a[0] *= 0.5f;
#pragma unroll
        for (int k1 = 1; k1 < 32; ++k1) a[k1] = cmul(a[k1], tw1[16 * (k1 - 1) + t]);

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
                load_group(g + stride < n_groups ? g + stride : g);
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
        float *pq = pw + q * 513;
        // bin kP = t + 32 j (lane 0, j >= 8: t + 32 j - 240); mirror 512 - kP
        float *const pA = pq + t, *const pB = pA - (l0 ? 240 : 0);
        float *const mA = pq + 32 - t, *const mB = mA + (l0 ? 240 : 0);
        static_for<0, 16>([&](auto jc) {
            constexpr int j = decltype(jc)::value;
            // lane 0's pairing, selected per lane with v_cndmask on a constant
            // lane mask (a C++ select of two b[] elements becomes a runtime
            // index into b, which sends b to scratch)
            f2 P = b[j], Q = b[16 + 15 - j];
            if constexpr (j >= 8) P = sel_l0(b[16 + j - 8], P);
            Q = sel_l0((j < 8) ? b[(16 - j) & 15] : b[16 + 23 - j], Q);
            const f2 S = pp_s(P, Q);
            const f2 D = pp_d(P, Q);
            const f2 T = cmul(D, tw3[16 * j + t]);
            const f2 re = pp_re(S, T), im = pp_im(S, T);
            const f2 pwr = __builtin_elementwise_fma(re, re, im * im);  // (|X[kP]|^2, |X[512-kP]|^2)
            ((j < 8) ? pA : pB)[32 * j] = pwr.x;
            ((j < 8) ? mA : mB)[32 * (15 - j)] = pwr.y;
        });
        // Z[256] is its own mirror: |X[256]|^2 = |Z[256]|^2 = 4 |b[8]|^2
        if (l0) pq[256] = 4.f * fmaf(b[8].x, b[8].x, b[8].y * b[8].y);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // 4. tone pick: lane (q, i < K) reads bin power i, argmax over the
        //    16-lane row (ties -> lowest i), lane (q, 0) stores the symbol.
        const bool live = w < p.n_windows;
        float pk = -1.f;
        int arg = t;
        if (t < p.k) pk = pq[mybin];
        if (live && t < p.k && p.mag) p.mag[w * p.k + t] = pk;
        // row_ror:1,2,4,8 within the 16-lane row: every lane sees the whole row
        static_for<0, 4>([&](auto sc) {
            constexpr int ctrl = 0x120 + (1 << decltype(sc)::value);
            const float po = __int_as_float(
                __builtin_amdgcn_update_dpp(0, __float_as_int(pk), ctrl, 0xF, 0xF, false));
            const int ao = __builtin_amdgcn_update_dpp(0, arg, ctrl, 0xF, 0xF, false);
            if (po > pk || (po == pk && ao < arg)) { pk = po; arg = ao; }
        });
        if (live && t == 0) p.sym[w] = (uint8_t)arg;
        if (p.spec && live) {
            float *so = p.spec + w * 513;
            for (int i = t; i < 513; i += 16) so[i] = pq[i];
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

hipError_t launch_fft_quad(const FftParams &p, hipStream_t s)
{
    constexpr int WPB = 4;
    int dev = 0, cus = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fft1024_quad_kernel<WPB>, 64 * WPB, 0) !=
            hipSuccess || per_cu < 1)
        per_cu = 1;
    const long long groups = (p.n_windows + 3) / 4;
    long long blocks = (groups + WPB - 1) / WPB;
    blocks = std::min<long long>(blocks, (long long)cus * per_cu);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL((fft1024_quad_kernel<WPB>), dim3((unsigned)blocks), dim3(64 * WPB), 0, s, p);
    return hipGetLastError();
}

}  } // namespace fskd::r1
