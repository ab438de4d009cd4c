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
constexpr int kMaxDevices = 64;
// the rescue's pass 0 by the fold (plan.h fold64) for fold plans up to this K
// (above, its code cost the fold kernels an occupancy step: K = 14, 4 -> 3)
constexpr int kFold64MaxK = 12;       // device ordinals the module tables cover

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
    // in-kernel decision rescue (the direct Goertzel-family kernels at n =
    // 1024): flagged windows are re-decided by their own row instead of a
    // rescue launch; rcoef = 2 cos(2 pi f_k / fs) in double, the caller's tone
    // order
    int rescue_inline;
    double rcoef[kMaxTones];
    // rescue_rows' pass 0 by the fold (plan.h fold64; plain-bank plans on
    // multiples of 8 bins read it at run time)
    int fold64;
    // rescue_rows' tables: rot64 = [k][16][4] {Ar, Ai, Br, Bi} in double (the
    // caller's tone order), pass 0's chain coefficients c[k] (= rcoef[k]
    // except by the fold, plan.h fold64), then rcoef[k] again (the exact
    // chains', read with a per-lane index);
    // pass 0 leaves a row to the exact chain when margin^2 < t2e64 E P_max;
    // t2e64 = 0: every flagged row takes the exact chain
    const double *rot64;
    double t2e64;
    // decision rescue (rescue.hip): ambiguity test constants.
    // Stage 1 (every window, no per-sample work): the int16 worst case
    // Q >= NE, threshold amb_tq sqrt(P_max), amb_tq = tau sqrt(Q); 0: no
    // flagging. Stage 2 (only rows stage 1 flags): the window's own energy,
    // threshold^2 = amb_t2e E P_max with E the detector's energy sum (plain
    // bank / residue: sum x^2, amb_t2e = tau^2 n; fold: sum xf^2 of the folded
    // window, tau^2 n / 8), floor amb_t2e E / 16.
    float amb_tq;
    float amb_floor;         // stage 1: 0 < P_max < amb_floor is ambiguous
    float amb_t2e;
    // fold detector: stage 2's energy is E_eff = (sqrt(sum xf^2) + amb_d)^2,
    // amb_d the double oracle's own error (which scales with the RAW window)
    // in units of the folded window's norm (error_model.cpp)
    float amb_d;
};

// Decision rescue. A detector's fp32 tone powers carry an
// error that error_model.cpp BOUNDS, from the kernel's own operation sequence
// and fp32 constants (round 5; no measured constant):
// |sqrt(P_k) - |X_k|| <= rho_det sqrt(E), and the double oracle's
// |sigma(P_ref,k) - |X_k|| <= rho_ref sqrt(sum x^2). A window whose fp32
// top-2 margin satisfies (P_max - P_2nd)^2 >= t2e E_eff P_max (t2e = 16
// (bound)^2) has sqrt P_max - sqrt P_2nd above twice both bounds, so its fp32
// argmax is the oracle's; every other window (and P_max == 0 with energy) is
// marked ambiguous and the rescue (rescue_rows in the detector, or
// rescue_kernel) re-decides it with the definition's double-precision
// arithmetic (bit-identical to oracle/fsk_oracle.c). The test runs in two
// stages: E_eff <= E_max for int16 input, so a window whose margin clears
// the threshold at E_max clears the exact test too and no per-sample work is
// spent on it (stage 1, amb_tq / amb_floor); only rows stage 1 flags compute
// their energy (stage 2), so quiet input (dithered silence, idle-channel
// noise) is not flagged wholesale.
// P_max == 0 (every fp32 tone power exactly zero) is a stage-1 candidate and
// ambiguous when the window's energy is not zero: input with no energy at the
// tones (a fold detector's folded window that cancels to a constant, say)
// leaves the oracle's double powers at its own rounding noise, whose argmax
// only its own arithmetic reproduces (round 4: tests/test_gpu_error_model.py
// test_rescued_decisions_every_window found one such window of clipped
// square waves on the fold-slide path). Digital silence (zero energy) is
// decided as a tie (tone 0) without a rescue, as the oracle's exact zeros are.
constexpr uint8_t kSymAmbiguous = 0x80;

// stage 1: margin within tau sqrt(Q P_max) (amb_tq = tau sqrt(Q)), or
// P_max == 0 (a candidate: stage 2 asks for energy)
__device__ __forceinline__ bool amb_margin(float p1, float p2, float tq, float fl)
{
    return tq > 0.f && (p1 == 0.f || p1 - p2 < tq * __builtin_amdgcn_sqrtf(p1) || p1 < fl);
}

// stage 2: (p1 - p2)^2 < t2e E p1, or p1 below the floor t2e E / 16, or p1 ==
// 0 with E > 0
__device__ __forceinline__ bool amb_energy(float p1, float p2, float e, float t2e)
{
    const float c = t2e * e, d = p1 - p2;
    return p1 > 0.f ? (d * d < c * p1 || 16.f * p1 < c) : c > 0.f;
}

// The two stages over a wave: `amb1` is this lane's stage-1 verdict (false for
// lanes without a real window); efn() returns the lane's row energy E and is
// called by every lane (it may shuffle), only when some lane of the wave has
// amb1 set (a wave-uniform branch: nothing is spent on unflagged waves).
template <typename EFn>
__device__ __forceinline__ bool amb_two_stage(bool amb1, float p1, float p2, float t2e, EFn efn)
{
    if (__ballot(amb1) == 0) return false;
    const float e = efn();
    return amb1 && amb_energy(p1, p2, e, t2e);
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

// A chain decision (K >= 2 flags ambiguous windows): the argmax, and the
// two-stage ambiguity verdict (stage 2 via efn, see amb_two_stage; `live` =
// the lane's window exists).
template <int K, typename EFn>
__device__ __forceinline__ int chain_decide(const float (&P)[K], bool live, float tq, float fl, float t2e,
                                            EFn efn, bool &amb)
{
    float p1, p2;
    const int arg = chain_argmax<K>(P, p1, p2);
    amb = K >= 2 && amb_two_stage(live && amb_margin(p1, p2, tq, fl), p1, p2, t2e, efn);
    return arg;
}

// Sum of squares of the 64 int16 samples of one lane segment, 16-byte chunks
// read by `chunk(i)` (i < 8), as fp32 (each square and partial sum rounded:
// relative error < 100 u, covered by error_model.cpp's safety factor in
// amb_t2e).
typedef unsigned int u32x4e __attribute__((ext_vector_type(4)));
typedef float f32x2e __attribute__((ext_vector_type(2)));
template <typename Chunk>
__device__ __forceinline__ float seg_energy(Chunk chunk)
{
    f32x2e a = {0.f, 0.f}, b = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const u32x4e d = chunk(i);
        const unsigned d4[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x2e x = {(float)(int)(short)(d4[q] & 0xFFFFu), (float)((int)d4[q] >> 16)};
            if (q & 1) b = __builtin_elementwise_fma(x, x, b);
            else a = __builtin_elementwise_fma(x, x, a);
        }
    }
    return (a.x + a.y) + (b.x + b.y);
}

// seg_energy's arithmetic, bit for bit, U chunks in flight at a time
template <int U, typename Chunk>
__device__ __forceinline__ float seg_energy_lowreg(Chunk chunk)
{
    f32x2e a = {0.f, 0.f}, b = {0.f, 0.f};
#pragma unroll U
    for (int i = 0; i < 8; ++i) {
        const u32x4e d = chunk(i);
        const unsigned d4[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x2e x = {(float)(int)(short)(d4[q] & 0xFFFFu), (float)((int)d4[q] >> 16)};
            if (q & 1) b = __builtin_elementwise_fma(x, x, b);
            else a = __builtin_elementwise_fma(x, x, a);
        }
    }
    return (a.x + a.y) + (b.x + b.y);
}

// A serial sum one chunk at a time (4 VGPRs of samples live instead of 32:
// for rare paths inside kernels at their VGPR limit)
template <typename Chunk>
__device__ __forceinline__ float seg_energy_serial(Chunk chunk)
{
    float e = 0.f;
#pragma unroll 1
    for (int i = 0; i < 8; ++i) {
        const u32x4e d = chunk(i);
        const unsigned d4[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const float x = (float)(short)((d4[q >> 1] >> (16 * (q & 1))) & 0xFFFFu);
            e = __builtin_fmaf(x, x, e);
        }
    }
    return e;
}

// Sum over the 16 lanes of a row (n = 1024 windows), every lane the same total.
__device__ __forceinline__ float row_sum16(float v)
{
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true));
    v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, true));
    return v;
}

// The same tree in double (the rescue's pass 0): each stage's partner by DPP
// (two 32-bit moves) instead of __shfl_xor's ds_bpermute round trips through
// the LDS crossbar. Bit-identical to the xor butterfly: after each stage the
// lanes of a group hold one value (a + b == b + a), so any lane of the
// partner group is the partner.
template <int C>
__device__ __forceinline__ double dpp_d(double v)
{
    const unsigned long long b = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)b, C, 0xF, 0xF, true);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(b >> 32), C, 0xF, 0xF, true);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ double row_sum16d(double v)
{
    v += dpp_d<0xB1>(v);
    v += dpp_d<0x4E>(v);
    v += dpp_d<0x141>(v);
    v += dpp_d<0x140>(v);
    return v;
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
// In-kernel decision rescue of a wave's flagged windows, each by its 16-lane
// row (n = 1024; round 3 for the 2-FSK plain bank, round 4 every direct
// Goertzel-family kernel at n = 1024). Two passes of one loop (one copy of
// the code, so the detector's VGPR budget pays for one):
//  pass 0 (round 4, when t2e64 > 0): the row's K powers in double, computed
//    the way the fp32 plain bank computes them — lane seg runs every tone's
//    recurrence over its own 64 samples, rotates its end state into the
//    window's phase (rot64) and the row sums — K x 64 double steps per lane
//    on all 16 lanes, instead of one 1024-step chain per tone on K lanes
//    (~10x fewer wave instructions at K = 2). These powers are not the
//    oracle's bits, but |sqrt P_0 - sigma P_ref| <= rho_first sqrt(E) (its own
//    rounding and the oracle's, derived by error_model.cpp from both
//    operation sequences; checked by tests/test_rescue_model64.py), so where
//    their top-2 margin satisfies margin^2 >= t2e64 E P_max (t2e64 = 16
//    rho_first^2) the argmax is the oracle's and the row is decided here (its
//    magnitudes: these powers rounded to fp32, within the bound of the
//    oracle's). Rows inside that band (exact ties; margins within ~1e-10 of
//    P_max) go on to
//  pass 1: lane seg < K runs tone seg's recurrence in double over the
//    window's 1024 samples with exactly rescue_kernel's operations and order
//    (so exactly oracle/fsk_oracle.c's: contraction off); the row's argmax
//    (ties to the lowest tone) replaces the symbol, and the powers (rounded
//    to fp32) the magnitudes, bit-identical to the oracle's.
// chunk(q) returns the window's 16-byte chunk q (samples 8q .. 8q + 7) from
// wherever the kernel holds the tile (its LDS slice: no global round trip).
// Every lane of the wave calls it (the shuffles); rows with amb_row false
// change nothing. The detector leaves the symbol and magnitudes of a flagged
// row to this function (no second store).
// Pass 0 by the fold (FOLD: fold detector plans, every tone on a multiple of
// 8 bins; round 5): lane seg sums the window's samples
// 128 m + 8 seg + i over m < 8 (exact integers: the folded samples 8 seg ..
// 8 seg + 7 of the window folded to 128), then per tone an 8-step double
// chain at the exact bin, the rotation (rot64: the fold tables, plan.h
// fold64), the row sum and the power; the margin test as pass 0 above (t2e64
// derived for this sequence, error_model.cpp first_pass_fold_rho). 8x fewer
// double steps than 64 raw samples per lane per tone. Returns amb_row after
// it (the rows left to the exact chains).
// x_lo^2 + x_hi^2 of 4 dwords (8 int16 samples): exact per dword by
// v_dot2_i32_i16 (clamped, only (-32768, -32768) saturates, to 2^31 - 1),
// converted and summed in fp32 (pass 0's energy: error_model.cpp allows E
// 100 u, this is < 36 u over a lane's 64 samples)
typedef short i16x2_dot __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float dot_energy4(const unsigned (&d4)[4])
{
    float e = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const i16x2_dot s = __builtin_bit_cast(i16x2_dot, d4[c]);
        e += (float)__builtin_amdgcn_sdot2(s, s, 0, true);
    }
    return e;
}

template <int K, typename Chunk>
__device__ __forceinline__ bool rescue_rows_fold0(const GoertzelParams &p, long long w, int seg,
                                                  bool amb_row, Chunk chunk)
{
#pragma clang fp contract(off)
    // opaque here: no address built from seg is hoisted into the detector's
    // loop (where it would hold VGPRs across every tile)
    asm volatile("" : "+v"(seg));
    int xf[8];
    float e = 0.f;  // the lane's 64 raw samples' sum x^2 (any partition of the window)
#pragma unroll
    for (int i = 0; i < 8; ++i) xf[i] = 0;
#pragma unroll 1
    for (int m = 0; m < 8; ++m) {
        const u32x4e d = chunk(16 * m + seg);
        const unsigned d4[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) xf[i] += (int)(short)((d4[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
        e += dot_energy4(d4);
    }
    double best = -1.0, second = -1.0;
    int arg = 0;
#pragma unroll 1
    for (int k = 0; k < K; ++k) {
        int ci = 64 * K + k;
        asm volatile("" : "+v"(ci));  // a vector load (as scalar, SGPR spills at large K)
        const double c = p.rot64[ci];
        double s1 = 0.0, s2 = 0.0;
        // each sample converted at its step (scheduled together, the 8
        // doubles raised the fold kernels' VGPR peak)
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            double s = (double)xf[i] + c * s1;
            s = s - s2;
            s2 = s1;
            s1 = s;
            __builtin_amdgcn_sched_barrier(0);
        }
        const double2 A = *reinterpret_cast<const double2 *>(p.rot64 + 4 * (k * 16 + seg));
        const double2 B = *reinterpret_cast<const double2 *>(p.rot64 + 4 * (k * 16 + seg) + 2);
        double re = A.x * s1, im = A.y * s1;
        re = re - B.x * s2;
        im = im - B.y * s2;
        re = row_sum16d(re);
        im = row_sum16d(im);
        const double pk = re * re + im * im;
        if (pk > best) {
            second = best;
            best = pk;
            arg = k;
        } else if (pk > second) {
            second = pk;
        }
        if (k == seg && amb_row && p.mag) p.mag[w * K + seg] = (float)pk;
    }
    const double cth = p.t2e64 * (double)row_sum16(e), dm = best - second;
    const bool still = !(best > 0.0) || dm * dm < cth * best || 16.0 * best < cth;
    if (amb_row && !still && seg == 0) p.sym[w] = (uint8_t)arg;
    return amb_row && still;
}

// FOLD: 0 = pass 0 by segments, 1 = by the fold (fold kernels), 2 = as the
// plan says at run time (p.fold64: plain-bank plans on multiples of 8 bins)
template <int K, int FOLD = 0, typename Chunk>
__device__ __forceinline__ void rescue_rows(const GoertzelParams &p, long long w, int seg, int lane,
                                            bool amb_row, Chunk chunk)
{
#pragma clang fp contract(off)
    int first = p.t2e64 > 0.0 ? 0 : 1;
    if constexpr (FOLD != 0) {
        if (first == 0 && (FOLD == 1 || p.fold64)) {
            amb_row = rescue_rows_fold0<K>(p, w, seg, amb_row, chunk);
            if (__ballot(amb_row) == 0) return;
            first = 1;
        }
    }
#pragma unroll 1
    for (int pass = first; pass < 2; ++pass) {
        const bool exact = pass == 1;
        const bool run = exact ? amb_row && seg < K : true;  // lanes that run chains
        const int q0 = exact ? 0 : 8 * seg, q1 = exact ? 128 : 8 * seg + 8;
        double best = -1.0, second = -1.0, mine = 0.0;
        float e = 0.f;  // pass 0: the lane's sum x^2
        int arg = 0;
#pragma unroll 1
        for (int t = 0; t < (exact ? 1 : K); ++t) {
            const int k = exact ? seg : t;
            // pass 0's coefficient, or the oracle's rcoef[k] (exact), per lane
            const double c = p.rot64[(exact ? 65 : 64) * K + (k < K ? k : 0)];
            double s1 = 0.0, s2 = 0.0;
            if (run) {
#pragma unroll 1
                for (int q = q0; q < q1; ++q) {
                    const u32x4e d = chunk(q);
                    const unsigned d4[4] = {d.x, d.y, d.z, d.w};
                    if (!exact && t == 0) e += dot_energy4(d4);
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const double x = (double)(short)((d4[i >> 1] >> (16 * (i & 1))) & 0xFFFFu);
                        double s = x + c * s1;
                        s = s - s2;
                        s2 = s1;
                        s1 = s;
                    }
                }
            }
            if (exact) {
                const double a = s1 * s1 + s2 * s2;
                const double b = c * s1;
                mine = run ? a - b * s2 : 0.0;
            } else {
                // the rotation's loads after the chain (an offset that depends
                // on its result): hoisted above it they hold 8 VGPRs through it
                // (and B's after A's products: 4 VGPRs of table live at a time)
                int ro = 4 * (k * 16 + seg);
                asm volatile("" : "+v"(ro) : "v"(s1));
                const double2 A = *reinterpret_cast<const double2 *>(p.rot64 + ro);
                double re = A.x * s1, im = A.y * s1;
                asm volatile("" : "+v"(ro) : "v"(re), "v"(im));
                const double2 B = *reinterpret_cast<const double2 *>(p.rot64 + ro + 2);
                re = re - B.x * s2;
                im = im - B.y * s2;
                re = row_sum16d(re);
                im = row_sum16d(im);
                const double pk = re * re + im * im;
                if (pk > best) {
                    second = best;
                    best = pk;
                    arg = k;
                } else if (pk > second) {
                    second = pk;
                }
                // the row's magnitudes now (pass 1 rewrites those of the rows
                // it takes over): no register holds them across the loop
                if (k == seg && amb_row && p.mag) p.mag[w * K + seg] = (float)pk;
            }
        }
        bool still = false;
        if (exact) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const double pk = __shfl(mine, (lane & 48) + k);
                if (pk > best) {
                    best = pk;
                    arg = k;
                }
            }
        } else {
            // stage threshold^2 = t2e64 E P_max, E the row's sum x^2 (fp32,
            // within 1e-5: the host's t2e64 carries (1 + 1e-3))
            const double cth = p.t2e64 * (double)row_sum16(e), dm = best - second;
            still = !(best > 0.0) || dm * dm < cth * best || 16.0 * best < cth;
        }
        if (amb_row && !still) {
            if (seg == 0) p.sym[w] = (uint8_t)arg;
            if (exact && p.mag && seg < K) p.mag[w * K + seg] = (float)mine;
        }
        amb_row = amb_row && still;
        if (__ballot(amb_row) == 0) break;
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
    // tones only: bit jb set = the post-pass pair block jb (pairs 2 jb and
    // 2 jb + 1 of every lane) holds some tone bin; 0xFF: every block (the
    // full post-pass, stage 2's energy by Parseval of the bin powers), else
    // only those blocks (PICK 2) and stage 2's energy n sum x^2 from the
    // samples (fft_quad_pmask; FSKD_FFT_PMASK=0: every block, measurement)
    unsigned pmask;
    uint8_t *sym;
    float *mag;              // [n_windows][k] or nullptr
    float *spec;             // [n_windows][513] or nullptr
    float amb_tq;            // decision rescue, as GoertzelParams (stage 2:
    float amb_floor;         // E = 2 x the window's 513 bin powers >= n sum x^2,
    float amb_t2e;           // Parseval, amb_t2e = tau^2)
    int rescue;            // 1: flagged windows are re-decided in the kernel (rescue_fft.h)
    const double *rtw;       // rescue: [1023] (cos, sin), stage len at len / 2 - 1 + j
    // the rescue's first pass (rescue_fft_seg, tones only): the tone bins'
    // powers in double by segments, rot64 = [k][16][4] {Ar, Ai, Br, Bi} at the
    // bins' frequencies, then 2 cos(2 pi b_k / n); t2e64 = 0: every flagged
    // window takes the double FFT
    const double *rot64;
    double t2e64;
    int fold64;              // rot64 by the fold (plan.h; every tone bin a multiple of 8)
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
    // n = 1024 (round 5): the first pass by segments (rescue_rows pass 0's
    // arithmetic and tables) before the exact chains; t2e64 = 0: exact only;
    // fold64: 1 = by the fold (rescue_rows_fold0's arithmetic), 2 = by the
    // residue fold (rescue.hip seg_residue_window; plan.h)
    const double *rot64;
    double t2e64;
    int fold64;
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
unsigned fft_quad_pmask(const int *bins, int k);  // FftParams::pmask of a tone plan
int fft_quad_slot(int bin);  // where fft_quad keeps |X[bin]|^2: 2 (16 j + t) + half, or 512 / 513 (bins 0 / 512)
// ip.proto framing of [n_streams][n] symbols, one frame run per stream (frame_gpu.hip)
long long frame_streams_size(long long n, int bits, long long max_payload, unsigned *per,
                             unsigned *full, int *frames);
hipError_t launch_frame_streams(const uint8_t *d_sym, long long n_streams, long long n, int bits,
                                long long max_payload, uint8_t *d_out, hipStream_t s);

}  // namespace fskd
