// fft_quad_r1b.hip — the round-1 shipped FFT detector kernel, kept (outside
// the library) as the A/B baseline of scripts/fft_probe.hip. Include after
// audio-network_amd/csrc/fft_quad.hip (it uses that file's quad:: helpers).
// Round 2 replaced it in the library with the fused-twiddle kernel
// (DESIGN.md §4.4).
namespace fskd {
namespace quad {
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
}  // namespace quad
namespace r1b {
// the round-1 lane-0 pairing: pairs j < 8 hold kP = 32 j, j >= 8 kP = 16 + 32 (j - 8),
// |X[256]|^2 at float 512
constexpr int quad_slot_r1(int b)
{
    if (b == 256) return 512;
    const int u = b & 31, v = b >> 5;
    if (u == 0) return v < 8 ? 2 * (16 * v) : 2 * (16 * (16 - v)) + 1;
    if (u == 16) return v < 8 ? 2 * (16 * (v + 8)) : 2 * (16 * (23 - v)) + 1;
    if (u < 16) return 2 * (16 * v + u);
    return 2 * (16 * (15 - v) + (32 - u)) + 1;
}
using namespace quad;
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
template <int WPB = 4, int MINW = 0, bool SPLIT = false, bool FUSE = false, bool FMT = false>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(MINW > 0 ? MINW : 1)))
void fft1024_quad_r1_kernel(FftParams p)
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
    const int myslot = quad_slot_r1(t < p.k ? p.bins[t] : 0);
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
            for (int i = t; i < 513; i += 16) so[i] = pq[quad_slot_r1(i)];
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// Persistent grid: as many blocks as fit the chip, each wave strides over
// groups of 4 windows (the LDS twiddle tables are built once per block).
template <int WPB, int MINW, bool SPLIT = false, bool FUSE = false, bool FMT = false>
hipError_t launch_fft_quad_r1_t(const FftParams &p, hipStream_t s)
{
    int dev = 0, cus = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fft1024_quad_r1_kernel<WPB, MINW, SPLIT, FUSE, FMT>,
                                                     64 * WPB, 0) != hipSuccess ||
        per_cu < 1)
        per_cu = 1;
    const long long groups = (p.n_windows + 3) / 4;
    long long blocks = (groups + WPB - 1) / WPB;
    blocks = std::min<long long>(blocks, (long long)cus * per_cu);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL((fft1024_quad_r1_kernel<WPB, MINW, SPLIT, FUSE, FMT>), dim3((unsigned)blocks), dim3(64 * WPB), 0,
                       s, p);
    return hipGetLastError();
}

}  // namespace r1b
}  // namespace fskd
