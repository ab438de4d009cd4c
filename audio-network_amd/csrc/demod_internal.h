// demod_internal.h — shared between the C-ABI host layer and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace fskd {

constexpr int kSeg = 64;              // samples per lane segment
constexpr int kTileSamples = 64 * kSeg;  // samples one wave owns per tile (8 KiB)
constexpr int kWavesPerBlock = 4;  // residue kernel: 4-wave blocks share the rotation table
// Plain and fold kernels: 2-wave blocks. Same 16 waves per CU as 4-wave blocks
// (LDS-limited for the plain bank), but a block's LDS and slots free up as
// soon as its 2 waves finish: K = 2 330.7 -> 322.8 us, plain K = 8 461.7 ->
// 450.0 us, fold K = 8 350.6 -> 346.5 us (profiles/round1/probe_wpb.log).
constexpr int kPlainWPB = 2;
constexpr int kLdsSegStride = 144;    // bytes: 128 B segment + 16 B pad (conflict-free b128 reads)
constexpr int kLdsWaveBytes = 64 * kLdsSegStride;
constexpr int kMaxTones = 16;
constexpr int kFoldSlideSegs = 80;    // fold.hip fold_slide_kernel: segments per tile (10 KiB)
constexpr int kMaxDevices = 64;       // device ordinals the module tables cover

// Uniform per-launch parameters (kernarg -> SGPRs).
struct GoertzelParams {
    const int16_t *pcm;      // window w starts at pcm + w*hop
    long long n_windows;
    long long hop;           // samples, multiple of 8
    int log2g;               // lanes per window = 2^log2g = n / 64
    int k;                   // tones
    const float4 *rot;       // [k][g] {Ar, Ai, Br, Bi} rotation of each lane segment
    uint8_t *sym;            // [n_windows]
    float *mag;              // [n_windows][k] or nullptr
    float coef[kMaxTones];   // 2 cos(w_k); reinsch: lambda_k = 2 cos(w_k) - 2 sgn_k
    float sgn[kMaxTones];    // reinsch: sign of cos(w_k) (+1 / -1)
    int reinsch;             // goertzel.hip: Reinsch-modified recurrence (tones near 0 / fs/2)
    int dcls;                // residue.hip: compile-time slot -> class pattern (DC, 0 = LDS class file)
    unsigned long long perm; // DCLS / F16: nibble s = the host's index of tone slot s
    int f16;                 // fold.hip: fold by 16 (K = 8, four tones each on Z0 / Z8)
    int zcls[kMaxTones];     // residue.hip: residue class (0..3) tone k reads
    int xcd_swizzle;         // 1: blocks b, b+8, b+16.. (one XCD) take adjacent tiles
    // goertzel.hip SLIDE (n = 1024, hop = 64 H < n): a tile is 64 contiguous
    // segments shared by slide_wt windows (0: off)
    int slide_wt;
    // 1: overlapping windows (hop < n) share lines between tiles, so the loads
    // keep them in L2 (plain policy); 0: each byte is read once (nt)
    int cached;
    // write-back bursts (wb_burst): 0 = none, else the number of bursts per
    // XCD in this launch
    int wb_bursts;
    // in-kernel decision rescue (goertzel.hip, n = 1024, K <= 2 chain path):
    // flagged windows are re-decided by their own row instead of a rescue
    // launch; rcoef = 2 cos(2 pi f_k / fs) in double, the caller's tone order
    int rescue_inline;
    double rcoef[kMaxTones];
    // decision rescue (rescue.hip): ambiguity test constants
    float amb_tq;            // threshold = amb_tq * sqrt(P_max); 0: no flagging
    float amb_floor;         // 0 < P_max < amb_floor: always ambiguous
};

// Decision rescue. A detector's fp32 powers carry an error
// |dP_k| <= r sqrt(P_max NE), NE = n sum x^2 <= Q = n^2 2^30 for int16 input
// (r measured per detector, scripts/precision_probe.py). Where the fp32 top-2
// margin is below amb_tq sqrt(P_max) (amb_tq = tau sqrt(Q), tau = 12 r), or
// P_max is so small that the second-order term could dominate, the fp32
// argmax may differ from the exact one: the detector sets kSymAmbiguous on
// the window's symbol and rescue_kernel re-decides it with the definition's
// double-precision arithmetic (bit-identical to oracle/fsk_oracle.c).
// P_max == 0 (every tone power exactly zero: silence) is decided as a tie
// (tone 0) without a rescue.
constexpr uint8_t kSymAmbiguous = 0x80;

__device__ __forceinline__ bool amb_margin(float p1, float p2, float tq, float fl)
{
    return tq > 0.f && p1 > 0.f && (p1 - p2 < tq * __builtin_amdgcn_sqrtf(p1) || p1 < fl);
}

// Sequential argmax (ties to the lowest k) that also keeps the runner-up, for
// the detectors' K-tone chains where every lane holds every P_k.
template <int K>
__device__ __forceinline__ int chain_argmax(const float (&P)[K], float &p1, float &p2)
{
    float best = -1.f, second = -1.f;
    int arg = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (P[k] > best) {
            second = best;
            best = P[k];
            arg = k;
        } else if (P[k] > second) {
            second = P[k];
        }
    }
    p1 = best;
    p2 = second;
    return arg;
}

// The symbol byte a chain decision stores (K >= 2: ambiguous windows flagged).
template <int K>
__device__ __forceinline__ uint8_t chain_symbol(const float (&P)[K], float tq, float fl)
{
    float p1, p2;
    const int arg = chain_argmax<K>(P, p1, p2);
    const bool amb = K >= 2 && amb_margin(p1, p2, tq, fl);
    return (uint8_t)(arg | (amb ? kSymAmbiguous : 0));
}

// Output store; NTS = non-temporal (streamed once, never re-read by the kernel).
template <bool NTS, typename T>
__device__ __forceinline__ void out_store(T *ptr, T v)
{
    if (NTS)
        __builtin_nontemporal_store(v, ptr);
    else
        *ptr = v;
}

// Tile-group index of this block. Blocks are dealt round-robin to the 8 XCDs
// (MI355X_MICROARCH.md §Workgroup dispatch), so with the swizzle each XCD
// walks one contiguous 1/8 of the tiles and every output line is written by a
// single XCD's L2. Placement only affects speed, never correctness.
__device__ __forceinline__ long long tile_block(int swz)
{
    const long long b = blockIdx.x, nb = gridDim.x;
    if (!swz) return b;
    const long long per = nb / 8, full = per * 8;
    if (b >= full) return b;
    return (b % 8) * per + b / 8;
}

// Write-back bursts (round 3), at the end of a Goertzel-family
// tile kernel. A batch whose outputs are more than the XCDs' L2s hold dirty
// (8-FSK: 33 MiB) runs as one launch in which the last block of every
// 1/wb_bursts of an XCD's swizzled blocks (its wave 0, after its stores)
// writes that XCD's L2 back with an agent-scope release, so the output lines
// leave in a few bursts instead of trickling out between the input's reads;
// the launch slices this replaces paid a drain and a ramp per slice.
// In-kernel decision rescue of one window by its 16-lane row (round 3, late;
// goertzel.hip K <= 2 at n = 1024): lane seg < K runs tone seg's recurrence
// in double over the window's n samples with exactly rescue_kernel's
// operations and order (so exactly oracle/fsk_oracle.c's), the row's argmax
// (ties to the lowest tone) replaces the flagged symbol, and the powers
// (rounded to fp32) the magnitudes. Every lane of the wave calls it (the
// shuffles); rows with amb_row false change nothing.
template <int K>
__device__ __forceinline__ void rescue_row(const GoertzelParams &p, long long w, int seg, int lane,
                                           bool amb_row, int n)
{
#pragma clang fp contract(off)
    typedef unsigned int u32x4r __attribute__((ext_vector_type(4)));
    double P = 0.0;
    if (amb_row && seg < K) {
        const double c = p.rcoef[seg];
        double s1 = 0.0, s2 = 0.0;
        const u32x4r *xs = reinterpret_cast<const u32x4r *>(p.pcm + w * p.hop);
        for (int q = 0; q < n / 8; ++q) {
            const u32x4r d = xs[q];
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
    }
    double best = -1.0;
    int arg = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const double pk = __shfl(P, (lane & 48) + k);
        if (pk > best) {
            best = pk;
            arg = k;
        }
    }
    if (amb_row) {
        if (seg == 0) p.sym[w] = (uint8_t)arg;
        if (p.mag && seg < K) p.mag[w * K + seg] = (float)P;
    }
}

__device__ __forceinline__ void wb_burst(int wb_bursts)
{
    if (wb_bursts <= 0 || threadIdx.x >= 64) return;
    const long long b = blockIdx.x, per = gridDim.x / 8, seg = per / wb_bursts;
    if (seg > 0 && b < per * 8 && (b / 8) % seg == seg - 1)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

// Full-spectrum detector (fft.hip), n = 1024.
struct FftParams {
    const int16_t *pcm;
    long long n_windows;
    long long hop;           // samples, even
    int k;
    int xcd_swizzle;
    const float *tw512;      // [512][2]  e^{-2 pi i m / 512}
    const float *tw1024;     // [512][2]  e^{-2 pi i k / 1024}
    const int *bins;         // [k] tone bins round(f n / fs), device
    int slot[kMaxTones];     // fft_quad_slot(bin) of each tone (quad2 register pick)
    uint8_t *sym;
    float *mag;              // [n_windows][k] or nullptr
    float *spec;             // [n_windows][513] or nullptr
    float amb_tq;            // decision rescue, as GoertzelParams
    float amb_floor;
    int rescue;              // 1: flagged windows are re-decided in the kernel (rescue_fft.h)
    const double *rtw;       // rescue: [1023] (cos, sin), stage len at len / 2 - 1 + j
};

// rescue.hip: re-decides every window whose symbol carries kSymAmbiguous.
struct RescueParams {
    const int16_t *pcm;      // window w at pcm + w * hop (the batch's first window)
    long long n_windows;
    long long hop;
    int n;
    int k;
    uint8_t *sym;
    int sym_aligned4;        // sym is 4-byte aligned: dword scans
    float *mag;              // [n_windows][k] or nullptr
    double coef[kMaxTones];  // Goertzel: 2 cos(2 pi f_k / fs), the caller's tone order
};
hipError_t launch_rescue(const RescueParams &p, hipStream_t s);

struct SynthParams {
    uint64_t seed;
    uint64_t w0;             // index of the first generated window in the stream
    long long n_windows;
    int n;                   // samples per window (multiple of 8)
    int k;
    int amplitude;
    int sigma;
    int16_t *pcm;
    uint8_t *sym;
    uint32_t inc[kMaxTones];  // phase increment per sample, 2^32 / cycle
};

// Detectors (the kernels behind DEMOD_METHOD_*).
constexpr int kDetGoertzel = 1;  // goertzel.hip: 64-sample lane segments
constexpr int kDetFft = 2;       // fft.hip: 1024-point real FFT, argmax over tone bins
constexpr int kDetFolded = 3;    // fold.hip: Goertzel on the N/8-folded window
constexpr int kDetResidue = 4;   // residue.hip: per-residue-class folding (any integer bins)

hipError_t launch_detector(int detector, const GoertzelParams &p, hipStream_t s);
// residue.hip: rotation table is [k][g][2] float4 {C1, C2}, {C3, C4}
const void *residue_kernel_ptr(int k, int log2g, int dcls = 0, bool nt = true);
size_t residue_lds_bytes(int k, int log2g, int qp = 2);
int tile_grid(long long n_windows, int log2g, int wpb = kWavesPerBlock, int wins_per_tile = 0);
hipError_t synth_prepare();  // upload the sine table to the current device (once, locked)
hipError_t launch_synth(const SynthParams &p, hipStream_t s);
hipError_t launch_read_ceiling(const int16_t *p, long long n_bytes, hipStream_t s);
hipError_t launch_fft_quad(const FftParams &p, hipStream_t s);  // 16 lanes / window (fft_quad.hip)
int fft_quad_slot(int bin);  // where fft_quad keeps |X[bin]|^2: 2 (16 j + t) + half, or 512 / 513 (bins 0 / 512)
// ip.proto framing of [n_streams][n] symbols, one frame run per stream (frame_gpu.hip)
long long frame_streams_size(long long n, int bits, long long max_payload, unsigned *per,
                             unsigned *full, int *frames);
hipError_t launch_frame_streams(const uint8_t *d_sym, long long n_streams, long long n, int bits,
                                long long max_payload, uint8_t *d_out, hipStream_t s);

}  // namespace fskd
