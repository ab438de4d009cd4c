// window_sum.h — epilogue shared by the tone-bank kernels for 16-lane
// windows (n = 1024): sum every lane's partial X_k = (re, im) over the
// window's 16 lanes, |X_k|^2, the argmax decision and the stores.
//
// The all-reduce it replaces adds all 2K partials at each of the 4 DPP
// stages (8K adds) and leaves every lane with every X_k, then decides
// tone by tone and stores one magnitude per instruction. Here the 2K values
// are reduce-SCATTERED instead: at each stage a lane keeps the half of its
// list selected by its lane bit, adds its partner's copy of that half (the
// partner sends the other half), and the list halves. For 2K = 16 that is
// 8 + 4 + 2 + 1 pairs x (2 selects + 1 DPP add) = 45 instructions instead of
// 64, and lane l ends with the window total of value l (re_k in lane 2k, im_k
// in lane 2k + 1): |X_k|^2 is one square plus one DPP add for all tones, the
// magnitudes go out as one coalesced store, and the argmax is two passes of
// 4 DPP max steps (ws_argmax).
//
// Decision (ws_argmax): the exact argmax of the fp32 powers the kernel
// stores, ties to the lowest tone index — the same rule as the K <= 2 path's
// sequential `P > best` and the oracle's (oracle/fsk_oracle.c
// goertzel_window_d). Two DPP max passes over the 16-lane row: the largest
// power's IEEE bits (P >= 0, so unsigned order is numeric order), then the
// lowest tone among the lanes holding exactly that power. (Round 1 packed
// both into one key by overwriting the low 4 mantissa bits with the tone, which
// resolved powers within 2^-19 relative to the lower tone even when the
// higher one was strictly larger.)
#pragma once
#include "demod_internal.h"

namespace fskd {

// Magnitude store policy. 0 plain, 1 non-temporal, 2 + a: raw buffer store
// with cache-policy bits a (probe only, 32-bit offsets). The default (-1,
// kMagStore<K>) is plain for every K. Non-temporal stores at K = 8 (a wave's
// 4 windows fill one whole 128-byte line) measured box-dependent against the
// shipped plain stores in 4 launch slices (demod_api.cpp launch_slice): one
// launch 310 vs 327 us on one box, 331 vs 324 us on the next, the
// no-magnitude floor 307 / 298 us (scripts/mag_probe.hip,
// profiles/round3/r3q/, r3r/); no policy was better on both.
template <int K>
constexpr int kMagStore = 0;

template <int MST>
__device__ __forceinline__ void mag_store(float *mag, long long idx, float v)
{
    if constexpr (MST == 0) {
        mag[idx] = v;
    } else if constexpr (MST == 1) {
        __builtin_nontemporal_store(v, mag + idx);
    } else {
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(mag, (short)0, 0x7FFFFFF0, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)(4 * idx), 0, MST - 2);
    }
}

template <int CTRL>
__device__ __forceinline__ float ws_dpp(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ unsigned ws_dpp_u(unsigned v)
{
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}

// DPP partner of lane bit B inside a 16-lane row: bit 3 row_mirror (i <-> 15 - i),
// bit 2 row_half_mirror (i <-> 7 - i within 8), bit 1 quad_perm [2,3,0,1],
// bit 0 quad_perm [1,0,3,2]. Each pairs lanes that differ in bit B (and in the
// lower bits for the mirrors, which the halving never looks at).
template <int B> struct WsCtrl;
template <> struct WsCtrl<3> { static constexpr int v = 0x140; };
template <> struct WsCtrl<2> { static constexpr int v = 0x141; };
template <> struct WsCtrl<1> { static constexpr int v = 0x4E; };
template <> struct WsCtrl<0> { static constexpr int v = 0xB1; };

// Per-lane select on lane bit B: (lane bit B set) ? b : a, as one v_cndmask
// on a constant lane mask. Written as asm: as C selects, hipcc folds
// `hi ? v[f] : v[e]` into a lane-dependent index into v and lowers that to
// compare-and-select chains over the whole list (3800 VALU per tile at K = 8).
template <int B>
__device__ __forceinline__ float ws_sel(float a, float b)
{
    constexpr unsigned long long m = B == 0 ? 0xAAAAAAAAAAAAAAAAull
                                   : B == 1 ? 0xCCCCCCCCCCCCCCCCull
                                   : B == 2 ? 0xF0F0F0F0F0F0F0F0ull
                                            : 0xFF00FF00FF00FF00ull;
    float r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(m));
    return r;
}

// One stage on lane bit B over a list of V values (value index bit B is
// split if B < log2(min(V, 16)), else the stage all-reduces).
template <int B, int V>
__device__ __forceinline__ void ws_stage(float (&v)[V], int lane)
{
    constexpr int C = WsCtrl<B>::v;
    constexpr int VS = V > 16 ? 16 : V;  // values a 16-lane group can scatter
    if constexpr ((1 << B) >= VS) {
#pragma unroll
        for (int e = 0; e < V; ++e) v[e] += ws_dpp<C>(v[e]);
    } else {
#pragma unroll
        for (int e = 0; e < V; ++e) {
            if (e & (1 << B)) continue;
            const int f = e | (1 << B);
            const float keep = ws_sel<B>(v[e], v[f]);
            const float send = ws_sel<B>(v[f], v[e]);
            v[e] = keep + ws_dpp<C>(send);
        }
    }
}

// Exact argmax over a 16-lane row (one window): lane candidates (bits of a
// power P >= 0, ok, tone index o); a second candidate per lane when TWO (K > 8).
// Returns the winning tone in every lane of the row: the largest P, and among
// equal P the lowest o. `mx` receives the row's largest power.
template <bool TWO>
__device__ __forceinline__ unsigned ws_argmax_m(unsigned pb0, bool ok0, int o0, unsigned pb1,
                                                bool ok1, int o1, float &mx)
{
    unsigned m = ok0 ? pb0 : 0u;
    if constexpr (TWO) m = max(m, ok1 ? pb1 : 0u);
    m = max(m, ws_dpp_u<0xB1>(m));
    m = max(m, ws_dpp_u<0x4E>(m));
    m = max(m, ws_dpp_u<0x141>(m));
    m = max(m, ws_dpp_u<0x140>(m));
    mx = __uint_as_float(m);
    // every lane now holds the row's max; key 16 - o marks the lanes holding it
    unsigned key = (ok0 && pb0 == m) ? (unsigned)(16 - o0) : 0u;
    if constexpr (TWO) key = max(key, (ok1 && pb1 == m) ? (unsigned)(16 - o1) : 0u);
    key = max(key, ws_dpp_u<0xB1>(key));
    key = max(key, ws_dpp_u<0x4E>(key));
    key = max(key, ws_dpp_u<0x141>(key));
    key = max(key, ws_dpp_u<0x140>(key));
    return 16u - key;
}

template <bool TWO>
__device__ __forceinline__ unsigned ws_argmax(unsigned pb0, bool ok0, int o0, unsigned pb1 = 0u,
                                              bool ok1 = false, int o1 = 0)
{
    float mx;
    return ws_argmax_m<TWO>(pb0, ok0, o0, pb1, ok1, o1, mx);
}

// Decision-rescue test over a row (demod_internal.h
// amb_margin): the window is ambiguous when a second tone's power lies within
// the threshold of the row's max mx (the max's own lane counts once), or mx is
// below the floor; mx == 0 is a stage-1 candidate and ambiguous in stage 2
// when the row's energy is not zero (t2c > 0; digital silence is decided
// without a rescue). Every lane of the row gets the same answer.
// Squared form, (mx - a)^2 < tq^2 mx (mx >= a >= 0; no square root), and
// the row count from two ballots: a row is ambiguous when two of its lanes
// hold a near tone (two bits in its 16-bit field) or one lane holds two; the
// per-row answer goes back to the lanes as a lane mask (inverse ballot), so
// the count costs scalar instructions instead of a 16-lane DPP reduction
// (FFT detector: ~8 VALU fewer per 4-window group).
// Threshold^2 = t2c mx, floor flc (stage 1: t2c = tq^2, flc = fl; stage 2:
// t2c = t2e E, flc = t2e E / 16, E the row's energy; demod_internal.h).
__device__ __forceinline__ bool ws_ambiguous_t(float mx, float a0, bool ok0, float a1, bool ok1,
                                               float t2c, float flc)
{
    const float t2 = t2c * mx;
    const float d0 = mx - a0, d1 = mx - a1;
    const bool n0 = ok0 && d0 * d0 < t2, n1 = ok1 && d1 * d1 < t2;
    const unsigned long long any = __ballot(n0 || n1), two = __ballot(n0 && n1);
    unsigned long long rows = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const unsigned f = (unsigned)(any >> (16 * r)) & 0xFFFFu;
        if ((f & (f - 1u)) != 0u || ((two >> (16 * r)) & 0xFFFFull) != 0) rows |= 0xFFFFull << (16 * r);
    }
    return mx > 0.f ? (__builtin_amdgcn_inverse_ballot_w64(rows) || mx < flc) : t2c > 0.f;
}

__device__ __forceinline__ bool ws_ambiguous(float mx, float a0, bool ok0, float a1, bool ok1,
                                             float tq, float fl)
{
    if (!(tq > 0.f)) return false;
    return ws_ambiguous_t(mx, a0, ok0, a1, ok1, tq * tq, fl);
}

// Both stages over the wave (demod_internal.h amb_two_stage): stage 1 with
// the int16 worst case, stage 2 only if some live row of the wave is flagged
// (efn: the row energy, called by every lane). Row-uniform result.
template <typename EFn>
__device__ __forceinline__ bool ws_amb_two_stage(float mx, float a0, bool ok0, float a1, bool ok1,
                                                 bool live, float tq, float fl, float t2e, EFn efn)
{
    const bool amb1 = ws_ambiguous(mx, a0, ok0, a1, ok1, tq, fl) && live;
    if (__ballot(amb1) == 0) return false;
    const float c = t2e * efn();
    const bool amb2 = ws_ambiguous_t(mx, a0, ok0, a1, ok1, c, c * 0.0625f);  // every lane: ballots inside
    return amb1 && amb2;
}

// The decision rescue's ambiguity test in an epilogue (demod_internal.h):
// stage-1 tq / fl (tq = 0: off), stage-2 t2e, and `defer`: the kernel
// re-decides flagged rows itself (rescue_rows), so their symbol and magnitudes
// are left to it; otherwise a flagged symbol leaves with kSymAmbiguous set
// (rescue_kernel, or FSKD_NO_RESCUE=flags).
struct AmbTest {
    float tq, fl, t2e;
    bool defer;
};

// X[k] = this lane's partial (re, im) of tone k. Writes the symbol of window
// w (lane j == 0) and, if mag, its K magnitudes; `live` = w is a real window.
// PERM: the kernel's tone slot s holds the host's tone (perm >> 4 s) & 15
// (residue.hip DCLS); magnitudes, the tie rule and the symbol use that index.
// efn: the row's energy for stage 2 of the ambiguity test (called by every
// lane, only when stage 1 flags some live row of the wave). Returns whether
// the row is ambiguous (row-uniform).
template <int K, bool PERM = false, int MST = -1, typename EFn>
__device__ __forceinline__ bool window_sum_decide(const float (&re)[K], const float (&im)[K],
                                                  int lane, long long w, bool live,
                                                  uint8_t *sym, float *mag,
                                                  unsigned long long perm, const AmbTest &at, EFn efn)
{
    static_assert(K >= 1 && K <= 16, "tones");
    constexpr int KP = K <= 1 ? 1 : K <= 2 ? 2 : K <= 4 ? 4 : K <= 8 ? 8 : 16;
    constexpr int V = 2 * KP;
    float v[V];
#pragma unroll
    for (int k = 0; k < KP; ++k) {
        v[2 * k] = k < K ? re[k] : 0.f;
        v[2 * k + 1] = k < K ? im[k] : 0.f;
    }
    ws_stage<3>(v, lane);
    ws_stage<2>(v, lane);
    ws_stage<1>(v, lane);
    ws_stage<0>(v, lane);
    // lane j holds value (j mod VS) in v[0] (and value 16 + j in v[16] if V = 32)
    constexpr int VS = V > 16 ? 16 : V;
    const int j = lane & 15;
    const int idx = j & (VS - 1);
    const bool re_lane = (idx & 1) == 0 && j < VS;
    const int t0 = idx >> 1;
    // re^2 + im^2 in the re lane as fma(re, re, im^2): explicit, so the
    // rounding does not depend on the compiler's contraction (the error
    // bound and tests/fp32emu.py follow this operation sequence)
    float sq = v[0] * v[0];
    const float P0 = __builtin_fmaf(v[0], v[0], ws_dpp<0xB1>(sq));
    float P1 = 0.f;
    if constexpr (V > 16) {
        sq = v[16] * v[16];
        P1 = __builtin_fmaf(v[16], v[16], ws_dpp<0xB1>(sq));
    }
    const bool ok0 = re_lane && t0 < K;
    const bool ok1 = V > 16 && re_lane && t0 + 8 < K;
    const int o0 = PERM ? (int)((perm >> (4 * t0)) & 15u) : t0;
    const int o1 = PERM ? (int)((perm >> (4 * ((t0 + 8) & 15))) & 15u) : t0 + 8;
    float mx;
    const unsigned arg = ws_argmax_m<(V > 16)>(__float_as_uint(P0), ok0, o0, __float_as_uint(P1),
                                               ok1, o1, mx);
    const bool amb = K >= 2 && ws_amb_two_stage(mx, P0, ok0, P1, ok1, live, at.tq, at.fl, at.t2e, efn);
    constexpr int MS = MST >= 0 ? MST : kMagStore<K>;
    if (live && !(amb && at.defer)) {
        if (mag) {
            if (ok0) mag_store<MS>(mag, w * K + o0, P0);
            if (ok1) mag_store<MS>(mag, w * K + o1, P1);
        }
        if (j == 0) sym[w] = (uint8_t)(arg | (amb ? kSymAmbiguous : 0u));
    }
    return amb;
}

// The same epilogue for K = 8 when the kernel has already split the tones by
// lane bit 3 (fold.hip F16: lanes 0-7 of a window hold tones 0-3, lanes 8-15
// tones 4-7, each over the whole window): that is the state after the first
// reduce-scatter stage, so only stages 2, 1, 0 run (21 instead of 45
// instructions). re/im = this lane's 4 tones (slots 4 * bit3 + s).
template <bool PERM = false, int MST = -1, typename EFn>
__device__ __forceinline__ bool window_sum_decide_split8(const float (&re)[4], const float (&im)[4],
                                                         int lane, long long w, bool live,
                                                         uint8_t *sym, float *mag,
                                                         unsigned long long perm, const AmbTest &at,
                                                         EFn efn)
{
    constexpr int K = 8;
    float v[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[2 * k] = re[k];
        v[2 * k + 1] = im[k];
    }
    ws_stage<2>(v, lane);
    ws_stage<1>(v, lane);
    ws_stage<0>(v, lane);
    // lane j holds value (j & 15) of the 16-value list: re_t in lane 2t, im_t in 2t + 1
    const int j = lane & 15;
    const bool re_lane = (j & 1) == 0;
    const int t0 = j >> 1;
    const float sq = v[0] * v[0];
    const float P0 = __builtin_fmaf(v[0], v[0], ws_dpp<0xB1>(sq));  // as window_sum_decide
    const int o0 = PERM ? (int)((perm >> (4 * t0)) & 15u) : t0;
    float mx;
    const unsigned arg = ws_argmax_m<false>(__float_as_uint(P0), re_lane, o0, 0u, false, 0, mx);
    const bool amb = ws_amb_two_stage(mx, P0, re_lane, 0.f, false, live, at.tq, at.fl, at.t2e, efn);
    constexpr int MS = MST >= 0 ? MST : kMagStore<K>;
    if (live && !(amb && at.defer)) {
        if (mag && re_lane) mag_store<MS>(mag, w * K + o0, P0);
        if (j == 0) sym[w] = (uint8_t)(arg | (amb ? kSymAmbiguous : 0u));
    }
    return amb;
}

}  // namespace fskd
