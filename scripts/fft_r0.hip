// fft_r0.hip — FIRST LAYOUT of the full-spectrum detector, kept for the
// interleaved A/B in scripts/probe.hip only (not built into libfskdemod.so;
// the shipped detector is audio-network_amd/csrc/fft_quad.hip). Full-spectrum detector: per window a
// 1024-point real FFT, |X[b]|^2 for b = 0..512, symbol = argmax over the tone
// bins b_k = round(f_k N / fs) (ties -> lowest k). Oracle:
// oracle/fsk_oracle.c:oracle_fft_demod (double radix-2 FFT).
//
// One wave per window, everything in registers + a wave-private LDS slice:
//   * real -> complex packing z[n] = x[2n] + i x[2n+1] (n < 512); lane j loads
//     z[j + 64 r], r = 0..7 — one coalesced 256-byte dword load per r, which is
//     exactly the input layout of the first Stockham stage;
//   * 512-point complex FFT as three radix-8 Stockham stages (Ns = 1, 8, 64;
//     lane j = butterfly j), DFT-8 in registers, per-lane stage twiddles held
//     in registers, LDS exchange between stages (in place: one wave's LDS
//     operations complete in order);
//   * real-FFT post-pass: X[k] = Xe + W_1024^k Xo, X[k+512] = Xe - W_1024^k Xo
//     with Xe/Xo from Z[k] and conj(Z[512-k]) (mirror read from LDS);
//   * |X|^2 stays in registers: tone bins are read lane-to-scalar (readlane),
//     argmax in scalars; optional full-spectrum store straight from registers.
// Cost ~350 VALU + ~60 LDS ops per lane per window: compute-bound.
#include <algorithm>

#include "../audio-network_amd/csrc/demod_internal.h"

namespace fskd {

struct cf {
    float x, y;
};

__device__ __forceinline__ cf cadd(cf a, cf b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ cf csub(cf a, cf b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ cf cmul(cf a, cf w)
{
    return {fmaf(a.x, w.x, -a.y * w.y), fmaf(a.x, w.y, a.y * w.x)};
}
__device__ __forceinline__ cf mul_mj(cf a) { return {a.y, -a.x}; }  // * (-i)
__device__ __forceinline__ cf mul_pj(cf a) { return {-a.y, a.x}; }  // * (+i)

// In-register forward DFT-8: X[k] = sum_n v[n] e^{-2 pi i n k / 8}.
__device__ __forceinline__ void dft8(cf v[8])
{
    const float h = 0.70710678118654752f;
    // DFT-4 of evens (v0, v2, v4, v6) and odds (v1, v3, v5, v7)
    cf e0 = cadd(v[0], v[4]), e1 = csub(v[0], v[4]), e2 = cadd(v[2], v[6]), e3 = csub(v[2], v[6]);
    cf E0 = cadd(e0, e2), E2 = csub(e0, e2), E1 = cadd(e1, mul_mj(e3)), E3 = csub(e1, mul_mj(e3));
    cf o0 = cadd(v[1], v[5]), o1 = csub(v[1], v[5]), o2 = cadd(v[3], v[7]), o3 = csub(v[3], v[7]);
    cf O0 = cadd(o0, o2), O2 = csub(o0, o2), O1 = cadd(o1, mul_mj(o3)), O3 = csub(o1, mul_mj(o3));
    // twiddles W8^k on the odd half: W8^1 = h(1 - i), W8^2 = -i, W8^3 = h(-1 - i)
    cf T1 = {h * (O1.x + O1.y), h * (O1.y - O1.x)};
    cf T2 = mul_mj(O2);
    cf T3 = {h * (O3.y - O3.x), -h * (O3.x + O3.y)};
    v[0] = cadd(E0, O0);
    v[4] = csub(E0, O0);
    v[1] = cadd(E1, T1);
    v[5] = csub(E1, T1);
    v[2] = cadd(E2, T2);
    v[6] = csub(E2, T2);
    v[3] = cadd(E3, T3);
    v[7] = csub(E3, T3);
}

// Physical LDS slot of logical element e of the 512-point exchange buffer:
// XOR-swizzle the pair index inside each 8-element block with bits 4-5 of e
// (stage-0 ds_write_b128: lanes 64 B apart -> 8 distinct 16-byte bank slots)
// and pad each 64-element row by 8 elements (stage-1 ds_write_b64: lanes 512 B
// apart land on the other half of the banks). Measured before: 537M bank
// conflict cycles per 4M-window dispatch (SQ_LDS_BANK_CONFLICT), more than the
// 399M active LDS cycles.
__device__ __forceinline__ int zi(int e)
{
    return 8 * (e >> 6) + ((e & ~7) | ((((e >> 1) & 3) ^ ((e >> 4) & 3)) << 1) | (e & 1));
}

// Persistent waves: the twiddles a lane needs depend only on its lane index
// (stage 1: W_512^{8 (j%8) r}, stage 2: W_512^{j r}, post-pass: W_1024^{j+64r}),
// so they are loaded once into registers and the LDS carries only the data
// exchange; the next window's 8 input dwords are prefetched during the current
// window's FFT.
// TWLDS: stage-1 and post-pass twiddles from block LDS tables instead of
// registers (-30 VGPRs: more waves per SIMD to hide the LDS round trips).
template <int WPB = 4, bool TWLDS = false>
__global__ __launch_bounds__(64 * WPB) void fft1024_kernel(FftParams p)
{
    __shared__ __attribute__((aligned(16))) cf zbuf[WPB][576];   // per-wave exchange slice (padded)
    __shared__ cf tws1[TWLDS ? 64 : 1];                            // W_512^{8 a b}, a,b < 8
    __shared__ cf tws3[TWLDS ? 512 : 1];                           // W_1024^k
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: tile bases stay in SGPRs (no waterfall loop per buffer load)
    cf *z = zbuf[wave];
    const cf *t512 = reinterpret_cast<const cf *>(p.tw512);
    const cf *t1024 = reinterpret_cast<const cf *>(p.tw1024);
    cf ta[TWLDS ? 1 : 8], tb[8], tc[TWLDS ? 1 : 8];
    if (TWLDS) {
        for (int i = threadIdx.x; i < 512; i += 64 * WPB) {
            tws3[i] = t1024[i];
            if (i < 64) tws1[i] = t512[(8 * (i >> 3) * (i & 7)) & 511];
        }
        __syncthreads();
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
        if (!TWLDS) ta[TWLDS ? 0 : r] = t512[(8 * (lane & 7) * r) & 511];
        tb[r] = t512[(lane * r) & 511];
        if (!TWLDS) tc[TWLDS ? 0 : r] = t1024[lane + 64 * r];
    }

    const long long stride = (long long)gridDim.x * WPB;
    long long w = tile_block(p.xcd_swizzle) * WPB + wave;
    uint32_t nx[8];
    auto load_win = [&](long long ww) {
        const uint32_t *xw = reinterpret_cast<const uint32_t *>(p.pcm + ww * p.hop);
#pragma unroll
        for (int r = 0; r < 8; ++r) nx[r] = __builtin_nontemporal_load(xw + lane + 64 * r);
    };
    if (w < p.n_windows) load_win(w);
    // zi() of every access, as a few per-lane bases plus immediates (the
    // swizzle only touches bits 1-2 within a 72-element padded row):
    //   zi(j + 64 r)         = zl + 72 r
    //   zi(8 j + 2 r)        = 72 (j/8) + 8 (j%8) + 2 (r ^ s)       s = (j/2)%4
    //   zi(64(j/8)+j%8+8r)   = 72 (j/8) + j%2 + 8 r + 2 (s ^ r/2)
    //   zi((512-j-64r)%512)  = zm0 + 72 (7 - r)   (j = 0, r = 0: slot 0)
    const int sw = (lane >> 1) & 3;
    const int zl = zi(lane);
    const int row0 = 72 * (lane >> 3) + 8 * (lane & 7);
    const int row1 = 72 * (lane >> 3) + (lane & 1);
    const int zm0 = zi(64 - lane);
    for (; w < p.n_windows; w += stride) {
        // stage-0 operands: z[j + 64 r] = (x[2(j+64r)], x[2(j+64r)+1])
        cf v[8];
#pragma unroll
        for (int r = 0; r < 8; ++r)
            v[r] = {(float)(int)(short)(nx[r] & 0xFFFFu), (float)((int)nx[r] >> 16)};
        if (w + stride < p.n_windows) load_win(w + stride);
        // stage 0 (Ns = 1): no twiddles; out[8 j + r] (64 contiguous bytes per lane)
        dft8(v);
#pragma unroll
        for (int r = 0; r < 4; ++r)
            *reinterpret_cast<float4 *>(z + row0 + 2 * (r ^ sw)) =
                make_float4(v[2 * r].x, v[2 * r].y, v[2 * r + 1].x, v[2 * r + 1].y);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // stage 1 (Ns = 8): in[j + 64 r] * W_512^{8 (j%8) r}; out[(j/8) 64 + j%8 + 8 r]
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = z[zl + 72 * r];
#pragma unroll
        for (int r = 1; r < 8; ++r)
            v[r] = cmul(v[r], TWLDS ? tws1[8 * (lane & 7) + r] : ta[TWLDS ? 0 : r]);
        dft8(v);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < 8; ++r) z[row1 + 8 * r + 2 * (sw ^ (r >> 1))] = v[r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // stage 2 (Ns = 64): in[j + 64 r] * W_512^{j r}; result Z[j + 64 r] stays in v
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] = z[zl + 72 * r];
#pragma unroll
        for (int r = 1; r < 8; ++r) v[r] = cmul(v[r], tb[r]);
        dft8(v);
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < 8; ++r) z[zl + 72 * r] = v[r];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // real post-pass: k = j + 64 r; Zm = conj(Z[(512 - k) mod 512])
        float pr[8];
        float p512 = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int k = lane + 64 * r;
            const cf zm = z[r == 0 ? (lane == 0 ? 0 : zm0 + 504) : zm0 + 72 * (7 - r)];
            const cf xe = {0.5f * (v[r].x + zm.x), 0.5f * (v[r].y - zm.y)};
            const cf d = {0.5f * (v[r].x - zm.x), 0.5f * (v[r].y + zm.y)};
            const cf t = cmul(mul_mj(d), TWLDS ? tws3[k] : tc[TWLDS ? 0 : r]);  // W_1024^k (Z - conj Zm) / (2i)
            const cf X = cadd(xe, t);
            pr[r] = fmaf(X.x, X.x, X.y * X.y);
            if (r == 0) {
                const cf X512 = csub(xe, t);  // meaningful in lane 0 (k = 0)
                p512 = fmaf(X512.x, X512.x, X512.y * X512.y);
            }
        }
        if (p.spec) {
            float *so = p.spec + w * 513;
#pragma unroll
            for (int r = 0; r < 8; ++r) so[lane + 64 * r] = pr[r];
            if (lane == 0) so[512] = p512;
        }
        // Tone-bin powers: bin b lives in lane b & 63, register b >> 6 (bin
        // 512 in lane 0's p512); read them into scalars, argmax (ties -> lowest).
        float best = -1.f;
        int arg = 0;
        for (int i = 0; i < p.k; ++i) {
            const int b = __builtin_amdgcn_readfirstlane(p.bins[i]);
            float sel = p512;
            const int rr = b >> 6;
#pragma unroll
            for (int r = 0; r < 8; ++r)
                if (rr == r) sel = pr[r];
            const float pk = __int_as_float(
                __builtin_amdgcn_readlane(__float_as_int(sel), b == 512 ? 0 : (b & 63)));
            if (p.mag && lane == i) p.mag[w * p.k + i] = pk;
            if (pk > best) { best = pk; arg = i; }
        }
        if (lane == 0) p.sym[w] = (uint8_t)arg;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

template <int WPB, bool TWLDS>
hipError_t launch_fft_variant(const FftParams &p, hipStream_t s);

hipError_t launch_fft(const FftParams &p, hipStream_t s);  // 64 lanes / window (first layout)
hipError_t launch_fft(const FftParams &p, hipStream_t s)
{
    return launch_fft_variant<4, false>(p, s);
}

template <int WPB, bool TWLDS>
hipError_t launch_fft_variant(const FftParams &p, hipStream_t s)
{
    int dev = 0, cus = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fft1024_kernel<WPB, TWLDS>, 64 * WPB, 0) !=
            hipSuccess || per_cu < 1)
        per_cu = 1;
    long long blocks = (p.n_windows + WPB - 1) / WPB;
    blocks = std::min<long long>(blocks, (long long)cus * per_cu);
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL((fft1024_kernel<WPB, TWLDS>), dim3((unsigned)blocks), dim3(64 * WPB), 0, s, p);
    return hipGetLastError();
}

}  // namespace fskd
