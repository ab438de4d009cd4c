// goertzel.hip — per-window Goertzel tone bank, |X_k|^2 and argmax on gfx950.
//
// The north-star hot path. The reference has no such
// kernel; the math restates the textbook recurrence that
// oracle/fsk_oracle.c:goertzel_window_d evaluates sequentially in double.
//
// Work decomposition:
//   * a wave owns a TILE of 64 lane-segments x 64 samples (8 KiB of int16);
//     a window of n = 64*G samples spans G consecutive lanes, so one tile
//     holds 64/G windows (4 at n = 1024);
//   * the tile is read from HBM with coalesced 16 B/lane non-temporal buffer
//     loads (8 x 1 KiB per wave; the per-tile descriptor's record count
//     bounds the last tile), prefetched one tile ahead in registers, then
//     transposed through a wave-private LDS slice (segment stride 144 B, so
//     every ds_read_b128 lane group hits 16 distinct bank slots);
//   * each lane runs the Goertzel recurrence over its own 64 contiguous
//     samples for all K tones (K independent chains interleave in the VALU);
//   * the segment's partial DFT is rotated into window phase,
//       X_k += A_seg s1 - B_seg s2,  A = e^{-jw(n0+63)}, B = e^{-jw(n0+64)},
//     and summed over the G lanes of the window with DPP row operations;
//   * every lane of the window then holds X_k; P_k = Re^2 + Im^2, argmax with
//     ties to the lowest k, one lane stores the symbol, lanes store P_k.
// 64-sample chains keep the fp32 error <= ~3e-6 of max_k P (a single
// 1024-sample chain reaches ~2e-5, over the 1e-5 bar).
#include "demod_internal.h"

#ifndef FSKD_SLIDE_EU
#define FSKD_SLIDE_EU 4
#endif
#include "window_sum.h"

namespace fskd {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v)
{
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}

// Sum over aligned groups of 2^log2g lanes; every lane of a group gets the
// bit-identical total (each step adds the same two operands in both lanes).
__device__ __forceinline__ float group_sum(float v, int log2g)
{
    if (log2g > 0) v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
    if (log2g > 1) v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
    if (log2g > 2) v += dpp_f<0x141>(v);  // row_half_mirror: other quad of the 8
    if (log2g > 3) v += dpp_f<0x140>(v);  // row_mirror: other half of the row
    if (log2g > 4) v += __shfl_xor(v, 16);
    if (log2g > 5) v += __shfl_xor(v, 32);
    return v;
}

// 16-byte chunk i of the samples at sp (plain load: the lines were just
// streamed in, L2 may still hold them)
__device__ __forceinline__ u32x4 global_chunk(const int16_t *sp, int i)
{
    return reinterpret_cast<const u32x4 *>(sp)[i];
}

// LOG2G >= 0: lane-group size fixed at compile time (4 <=> n = 1024);
// LOG2G == -1: taken from p.log2g at run time.
// Tunables (defaults are the shipped configuration, chosen by scripts/probe):
//   PF  tiles prefetched per wave in registers (1 or 2),
//   NT  non-temporal loads (the PCM is read exactly once),
//   WPB waves per block (each wave owns a private LDS slice).
//   DIRECT  no LDS: each lane loads its own 128-byte segment (8 x 16 B;
//           per instruction 64 lines, each fully consumed over the 8).
//   NTS     non-temporal output stores.
//   PK      pair tones into packed fp32 (v_pk_fma_f32 / v_pk_add_f32).
//   SB      sched_barrier after every sample's K-tone step, so the K independent
//           recurrences stay interleaved (hipcc otherwise serialises one tone's
//           whole chain after another: issue-stall bound at large K).
//   WS      window_sum.h epilogue (reduce-scatter, packed-key argmax, one
//           coalesced magnitude store) at n = 1024.
//   SLIDE   overlapping windows at n = 1024, hop = 64 H < n: a
//           window's 16 segments are shared with the windows around it, so a
//           tile is 64 CONTIGUOUS segments whose recurrence states (s1, s2)
//           are computed once and kept in LDS; each of the
//           Wt = (64 - 16) / H + 1 windows u whose segments all lie in the tile
//           then rotates and sums segments uH .. uH + 15 exactly as the direct
//           path does (4 windows per pass of the 16-lane epilogue), so its
//           result is bit-identical to evaluating that window alone. Direct
//           evaluation recomputes every sample n / hop times and re-reads it
//           as often.
//   RS      Reinsch-modified recurrence for tone plans with a tone near 0 or
//           fs/2, where the fp32 coefficient 2cos(w) cannot resolve w (a tone
//           at bin 3 of 1024 misses the 1e-5 bar by 4x). With sgn = sign(cos w),
//           lambda = 2cos(w) - 2 sgn = -4 sin^2(w/2) or 4 cos^2(w/2) (full
//           relative precision) and d[n] = s[n] - sgn s[n-1]:
//             d[n] = x[n] + lambda s[n-1] + sgn d[n-1],  s[n] = sgn s[n-1] + d[n]
//           (3 ops per sample-tone instead of 2). The kernel keeps s in s1 and
//           d in s2; the host folds s2 = sgn (s1 - d) into the rotation
//           constants: X += (A - sgn B) s1 + sgn B d.
template <int K, int LOG2G, int PF = 1, bool NT = true, int WPB = kWavesPerBlock,
          bool DIRECT = false, bool NTS = false, bool PK = false, bool SB = false,
          bool WS = false, bool RS = false, bool SLIDE = false>
__global__ __launch_bounds__(64 * WPB) void goertzel_tile_kernel(GoertzelParams p)
{
    static_assert(PF == 1 || PF == 2, "prefetch depth");
    static_assert(!SLIDE || (LOG2G == 4 && !DIRECT && PF == 1), "SLIDE: n = 1024");
    static_assert(!SLIDE || K * 64 * 8 + 64 * 4 <= kLdsWaveBytes, "SLIDE: states + energies in the slice");
    __shared__ __attribute__((aligned(16))) unsigned char lds[DIRECT ? 16 : WPB * kLdsWaveBytes];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: tile bases stay in SGPRs (no waterfall loop per buffer load)
    unsigned char *wl = lds + wave * kLdsWaveBytes;
    const int log2g = LOG2G >= 0 ? LOG2G : p.log2g;
    const int g = 1 << log2g;
    const int n = 64 << log2g;
    const int seg = lane & (g - 1);          // segment index inside the window
    const int win_in_tile = lane >> log2g;
    const long long wins_per_tile = SLIDE ? (long long)p.slide_wt : 64 >> log2g;
    const long long n_tiles = (p.n_windows + wins_per_tile - 1) / wins_per_tile;

    float4 r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) r[k] = p.rot[k * g + seg];

    // Byte offset (from the tile's first window) of this lane's 16-byte chunk
    // i: chunk q = 64 i + lane is chunk (q mod 8G) of tile window q / 8G
    // (SLIDE: the tile's samples are contiguous, i.e. the same with hop = n).
    const int cpw_log2 = 3 + log2g;
    const long long lhop = SLIDE ? (long long)n : p.hop;
    int goff[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const int q = 64 * i + lane;
        if (DIRECT)
            goff[i] = (int)(((long long)win_in_tile * p.hop + seg * 64 + 8 * i) * 2);
        else
            goff[i] = (int)(((long long)(q >> cpw_log2) * lhop +
                             (long long)(q & ((1 << cpw_log2) - 1)) * 8) * 2);
    }
    // LDS write slot of chunk i: segment 8i + lane/8, chunk lane%8
    const int wr_off = (lane >> 3) * kLdsSegStride + (lane & 7) * 16;
    const int rd_off = lane * kLdsSegStride;

    const long long stride = (long long)gridDim.x * WPB;
    long long t = tile_block(p.xcd_swizzle) * WPB + wave;

    auto load_tile = [&](long long tt, u32x4 v[8]) {
        const long long wbase = tt * wins_per_tile;
        const long long left = p.n_windows - wbase;  // >= 1
        long long bytes = ((left - 1) * p.hop + n) * 2;
        if (bytes > 0x7FFFFFF0LL) bytes = 0x7FFFFFF0LL;
        __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)(p.pcm + wbase * p.hop), (short)0, (int)bytes, 0x00020000);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            v[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, goff[i], 0, NT ? 2 : 0);
    };

    // One tile: stage v through LDS, refill v with tile `next`, then run the
    // recurrences, the rotation + lane-group reduction and the decision.
    auto do_tile = [&](long long tt, u32x4 v[8], long long next) {
        u32x4 cur[8];
        if (DIRECT) {
#pragma unroll
            for (int i = 0; i < 8; ++i) cur[i] = v[i];
            if (next < n_tiles) load_tile(next, v);
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i)
                *reinterpret_cast<u32x4 *>(wl + wr_off + i * 8 * kLdsSegStride) = v[i];
            if (next < n_tiles) load_tile(next, v);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }

        float s1[K], s2[K];
#pragma unroll
        for (int k = 0; k < K; ++k) { s1[k] = 0.f; s2[k] = 0.f; }

        if constexpr (PK && K >= 2) {
            // tone pairs in packed fp32 (v_pk_add_f32 + v_pk_fma_f32 per sample
            // per pair); an odd last tone runs as a scalar chain
            constexpr int H = K / 2;
            f32x2 c2[H], sg2[H], a1[H], a2[H];
            float cs = 0.f, ss = 0.f, b1 = 0.f, b2 = 0.f;
#pragma unroll
            for (int h = 0; h < H; ++h) {
                c2[h] = f32x2{p.coef[2 * h], p.coef[2 * h + 1]};
                if (RS) sg2[h] = f32x2{p.sgn[2 * h], p.sgn[2 * h + 1]};
                a1[h] = f32x2{0.f, 0.f};
                a2[h] = f32x2{0.f, 0.f};
            }
            if (K & 1) {
                cs = p.coef[K - 1];
                if (RS) ss = p.sgn[K - 1];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const u32x4 sj = DIRECT ? cur[j] : *reinterpret_cast<const u32x4 *>(wl + rd_off + j * 16);
                const uint32_t d4[4] = {sj.x, sj.y, sj.z, sj.w};
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const uint32_t d = d4[q >> 1];
                    const float x = (q & 1) ? (float)((int)d >> 16) : (float)(int)(short)(d & 0xFFFFu);
                    const f32x2 xx = f32x2{x, x};
#pragma unroll
                    for (int h = 0; h < H; ++h) {
                        if constexpr (RS) {  // a1 = s, a2 = d
                            const f32x2 d = __builtin_elementwise_fma(
                                c2[h], a1[h], __builtin_elementwise_fma(sg2[h], a2[h], xx));
                            a1[h] = __builtin_elementwise_fma(sg2[h], a1[h], d);
                            a2[h] = d;
                        } else {
                            const f32x2 a = __builtin_elementwise_fma(c2[h], a1[h], xx - a2[h]);
                            a2[h] = a1[h];
                            a1[h] = a;
                        }
                    }
                    if (K & 1) {
                        if constexpr (RS) {
                            const float d = fmaf(cs, b1, fmaf(ss, b2, x));
                            b1 = fmaf(ss, b1, d);
                            b2 = d;
                        } else {
                            const float a = fmaf(cs, b1, x - b2);
                            b2 = b1;
                            b1 = a;
                        }
                    }
                    if (SB) __builtin_amdgcn_sched_barrier(0);
                }
            }
#pragma unroll
            for (int h = 0; h < H; ++h) {
                s1[2 * h] = a1[h].x;
                s1[2 * h + 1] = a1[h].y;
                s2[2 * h] = a2[h].x;
                s2[2 * h + 1] = a2[h].y;
            }
            if (K & 1) {
                s1[K - 1] = b1;
                s2[K - 1] = b2;
            }
        } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const u32x4 sj = DIRECT ? cur[j] : *reinterpret_cast<const u32x4 *>(wl + rd_off + j * 16);
            const uint32_t d4[4] = {sj.x, sj.y, sj.z, sj.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t d = d4[q];
                const float x0 = (float)(int)(short)(d & 0xFFFFu);
                const float x1 = (float)((int)d >> 16);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const float x = h ? x1 : x0;
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        if constexpr (RS) {  // s1 = s, s2 = d
                            const float dd = fmaf(p.coef[k], s1[k], fmaf(p.sgn[k], s2[k], x));
                            s1[k] = fmaf(p.sgn[k], s1[k], dd);
                            s2[k] = dd;
                        } else {
                            const float a = fmaf(p.coef[k], s1[k], x - s2[k]);
                            s2[k] = s1[k];
                            s1[k] = a;
                        }
                    }
                }
                if (SB) __builtin_amdgcn_sched_barrier(0);
            }
        }
        }

        if constexpr (SLIDE) {
            // segment states -> LDS (the samples are consumed)
            float2 *lz = reinterpret_cast<float2 *>(wl);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int k = 0; k < K; ++k) lz[k * 64 + lane] = make_float2(s1[k], s2[k]);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const int H = (int)(p.hop >> 6);
            const int wt = (int)wins_per_tile;
            // stage 2's energies: the tile's segments' fp32 sums x^2, computed
            // once per tile (lane = segment, re-read from L2) into LDS after
            // the states, when a window of the tile first needs one (round 5:
            // per window, 16 lanes re-read its 2 KiB, which at hop 256 with
            // every window a candidate cost the detector 0.7 ms more)
            float *le = reinterpret_cast<float *>(wl + K * 64 * sizeof(float2));
            bool have_e = false;  // wave-uniform (efn runs on every lane)
            for (int u0 = 0; u0 < wt; u0 += 4) {
                const int u = u0 + win_in_tile;                 // window of the tile
                const int sg = (u < wt ? u * H : 0) + seg;      // its segment j = seg
                const long long w = tt * wins_per_tile + u;
                const bool live = u < wt && w < p.n_windows;
                float xr[K], xi[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const float2 z = lz[k * 64 + sg];   // (s1, s2) of segment j of window u
                    if constexpr (WS) {
                        // packed (re, im): (A s1) - (B s2), as the direct WS path below
                        const f32x2 X = __builtin_elementwise_fma(
                            f32x2{-r[k].z, -r[k].w}, f32x2{z.y, z.y},
                            f32x2{r[k].x, r[k].y} * f32x2{z.x, z.x});
                        xr[k] = X.x;
                        xi[k] = X.y;
                    } else {  // as the direct K <= 2 path below
                        // explicit fma (as the direct path): the SLIDE and direct
                        // kernels must round alike whatever the contraction
                        xr[k] = fmaf(r[k].x, z.x, -(r[k].z * z.y));
                        xi[k] = fmaf(r[k].y, z.x, -(r[k].w * z.y));
                    }
                }
                // stage 2 of the ambiguity test: the window's energy from its
                // segments, re-read from L2 (the samples in LDS are gone)
                auto efn = [&]() {
                    if (!have_e) {
                        // the tile's segments of real windows: (nlive - 1) H + 16
                        const long long nlive = min((long long)wt, p.n_windows - tt * wins_per_tile);
                        const bool real = lane < (int)((nlive - 1) * H + 16);
                        const int16_t *sp = p.pcm + tt * wins_per_tile * p.hop + 64 * lane;
                        le[lane] = seg_energy_lowreg<FSKD_SLIDE_EU>([&](int i) {
                            return real ? global_chunk(sp, i) : u32x4{0u, 0u, 0u, 0u};
                        });
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        have_e = true;
                    }
                    return group_sum(live ? le[sg] : 0.f, 4);
                };
                if constexpr (WS) {
                    window_sum_decide<K>(xr, xi, lane, w, live, p.sym, p.mag, 0,
                                         AmbTest{p.amb_tq, p.amb_floor, p.amb_t2e, false}, efn);
                } else {
                    float P[K];
#pragma unroll
                    for (int k = 0; k < K; ++k) {
                        const float re = group_sum(xr[k], 4), im = group_sum(xi[k], 4);
                        P[k] = fmaf(re, re, im * im);
                    }
                    bool amb;
                    const int arg = chain_decide<K>(P, live, p.amb_tq, p.amb_floor, p.amb_t2e, efn, amb);
                    if (live) {
                        if (seg == 0) out_store<NTS>(p.sym + w, (uint8_t)(arg | (amb ? kSymAmbiguous : 0)));
                        if (p.mag) {
#pragma unroll
                            for (int k = 0; k < K; ++k)
                                if ((k & 15) == seg) out_store<NTS>(p.mag + w * K + k, P[k]);
                        }
                    }
                }
            }
            // the next tile's samples overwrite the partials
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            return;
        }
        const long long w = tt * wins_per_tile + win_in_tile;
        const bool live = w < p.n_windows;
        // stage 2 of the ambiguity test (demod_internal.h): this lane's 64
        // samples again (the tile is still in the wave's LDS slice, or from
        // L2 for DIRECT), summed over the window's lanes
        auto efn = [&]() {
            float e;
            if constexpr (DIRECT) {
                const int16_t *sp = p.pcm + w * p.hop + 64 * seg;
                e = seg_energy([&](int i) { return live ? global_chunk(sp, i) : u32x4{0u, 0u, 0u, 0u}; });
            } else {
                // an opaque offset: the recurrence read the same LDS bytes,
                // and reusing those values would keep 32 VGPRs live across it
                int off = rd_off;
                asm volatile("" : "+v"(off));
                e = seg_energy([&](int i) { return *reinterpret_cast<const u32x4 *>(wl + off + 16 * i); });
            }
            return group_sum(e, log2g);
        };
        // in-kernel rescue (n = 1024, tile in LDS): the window's chunk q
        auto chunk = [&](int q) {
            return *reinterpret_cast<const u32x4 *>(wl + (16 * win_in_tile + (q >> 3)) * kLdsSegStride +
                                                    (q & 7) * 16);
        };
        constexpr bool kInline = LOG2G == 4 && !DIRECT && K >= 2 && K <= 16;
        const bool defer = kInline && p.rescue_inline;
        if constexpr (WS && LOG2G == 4) {
            float xr[K], xi[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                // packed (re, im): (A s1) - (B s2), 2 ops per tone
                const f32x2 X = __builtin_elementwise_fma(f32x2{-r[k].z, -r[k].w},
                                                          f32x2{s2[k], s2[k]},
                                                          f32x2{r[k].x, r[k].y} * f32x2{s1[k], s1[k]});
                xr[k] = X.x;
                xi[k] = X.y;
            }
            const bool amb = window_sum_decide<K>(xr, xi, lane, w, live, p.sym, p.mag, 0,
                                                  AmbTest{p.amb_tq, p.amb_floor, p.amb_t2e, defer}, efn);
            if constexpr (kInline) {
                if (defer && __ballot(amb && live) != 0) rescue_rows<K, (K <= 2 ? 2 : 0)>(p, w, seg, lane, amb && live, chunk);
            }
            return;
        }
        float P[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            float re = fmaf(r[k].x, s1[k], -(r[k].z * s2[k]));  // explicit: SLIDE rounds alike
            float im = fmaf(r[k].y, s1[k], -(r[k].w * s2[k]));
            re = group_sum(re, log2g);
            im = group_sum(im, log2g);
            P[k] = fmaf(re, re, im * im);
        }

        bool amb;
        const int arg = chain_decide<K>(P, live, p.amb_tq, p.amb_floor, p.amb_t2e, efn, amb);
        if (live && !(amb && defer)) {
            if (seg == 0) out_store<NTS>(p.sym + w, (uint8_t)(arg | (amb ? kSymAmbiguous : 0)));
            if (p.mag) {
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if ((k & (g - 1)) == seg) out_store<NTS>(p.mag + w * K + k, P[k]);
            }
        }
        if constexpr (kInline) {
            // decision rescue in the kernel (demod_internal.h rescue_rows); every
            // lane of a row holds the same all-reduced powers, so the same verdict
            if (defer && __ballot(amb && live) != 0) rescue_rows<K, (K <= 2 ? 2 : 0)>(p, w, seg, lane, amb && live, chunk);
        }
    };

    if (PF == 1) {
        u32x4 v[8];
        if (t < n_tiles) load_tile(t, v);
        for (; t < n_tiles; t += stride) do_tile(t, v, t + stride);
    } else {
        u32x4 va[8], vb[8];
        if (t < n_tiles) load_tile(t, va);
        if (t + stride < n_tiles) load_tile(t + stride, vb);
        for (; t < n_tiles; t += 2 * stride) {
            do_tile(t, va, t + 2 * stride);
            if (t + stride >= n_tiles) break;
            do_tile(t + stride, vb, t + 3 * stride);
        }
    }
    wb_burst(p.wb_bursts);
}

// Shipped configuration: packed tone pairs for K >= 3 (K = 4: 407 -> 336 us,
// K = 8: 657 -> 506 us on 2^20 windows; K = 2 is HBM-bound either way) and the
// window_sum.h epilogue for K >= 3 (K = 8: 484 -> 456 us; neutral at K <= 4,
// profiles/round1/probe_window_sum.log).
// RS (Reinsch form) only for plans with a tone near 0 or fs/2 (the host's
// kReinschSin test): elsewhere the plain form is within the bar at 2 ops.
template <int K, bool NT>
static const void *kernel_for_t(int log2g, bool rs)
{
    constexpr bool PK = K >= 3;
    if (log2g == 4)
        return rs ? reinterpret_cast<const void *>(
                        &goertzel_tile_kernel<K, 4, 1, NT, kPlainWPB, false, false, PK, false,
                                              K >= 3, true>)
                  : reinterpret_cast<const void *>(
                        &goertzel_tile_kernel<K, 4, 1, NT, kPlainWPB, false, false, PK, false,
                                              K >= 3>);
    return rs ? reinterpret_cast<const void *>(
                    &goertzel_tile_kernel<K, -1, 1, NT, kPlainWPB, false, false, PK, false,
                                          false, true>)
              : reinterpret_cast<const void *>(
                    &goertzel_tile_kernel<K, -1, 1, NT, kPlainWPB, false, false, PK>);
}

// nt: the PCM is read once (hop = n); overlapping windows (hop < n) load with
// the plain cache policy so neighbouring tiles find their shared lines in L2.
template <int K>
static const void *kernel_for(int log2g, bool rs, bool slide, bool nt)
{
    constexpr bool PK = K >= 3;
    if (slide)  // cached loads: neighbouring tiles share their edge segments
        return rs ? reinterpret_cast<const void *>(
                        &goertzel_tile_kernel<K, 4, 1, false, kPlainWPB, false, false, PK, false,
                                              K >= 3, true, true>)
                  : reinterpret_cast<const void *>(
                        &goertzel_tile_kernel<K, 4, 1, false, kPlainWPB, false, false, PK, false,
                                              K >= 3, false, true>);
    return nt ? kernel_for_t<K, true>(log2g, rs) : kernel_for_t<K, false>(log2g, rs);
}

static const void *kernel_ptr(int k, int log2g, bool rs, bool slide, bool nt)
{
    switch (k) {
#define FSKD_CASE(K) case K: return kernel_for<K>(log2g, rs, slide, nt);
        FSKD_CASE(1) FSKD_CASE(2) FSKD_CASE(3) FSKD_CASE(4)
        FSKD_CASE(5) FSKD_CASE(6) FSKD_CASE(7) FSKD_CASE(8)
        FSKD_CASE(9) FSKD_CASE(10) FSKD_CASE(11) FSKD_CASE(12)
        FSKD_CASE(13) FSKD_CASE(14) FSKD_CASE(15) FSKD_CASE(16)
#undef FSKD_CASE
    default: return nullptr;
    }
}

// One tile per wave (grid = tiles / waves-per-block): measured 317 us vs
// 363 us for a persistent grid-stride grid on 2^20 windows (profiles/,
// DESIGN.md §Tuning) — the dispatcher keeps every CU fed to the last tile.
int tile_grid(long long n_windows, int log2g, int wpb, int wins_per_tile_override)
{
    const long long wins_per_tile = wins_per_tile_override > 0 ? wins_per_tile_override : 64 >> log2g;
    const long long n_tiles = (n_windows + wins_per_tile - 1) / wins_per_tile;
    long long blocks = (n_tiles + wpb - 1) / wpb;
    if (blocks > 0x7FFFFFFFLL) blocks = 0x7FFFFFFFLL;  // kernels grid-stride beyond
    if (blocks < 1) blocks = 1;
    return (int)blocks;
}

const void *fold_kernel_ptr(int k, int log2g, bool f16, bool nt, bool slide);

hipError_t launch_detector(int detector, const GoertzelParams &p, hipStream_t s)
{
    const bool nt = p.cached == 0;
    const void *f = detector == kDetFolded    ? fold_kernel_ptr(p.k, p.log2g, p.f16 != 0, nt, p.slide_wt > 0)
                  : detector == kDetResidue ? residue_kernel_ptr(p.k, p.log2g, p.dcls, nt)
                                            : kernel_ptr(p.k, p.log2g, p.reinsch != 0, p.slide_wt > 0, nt);
    if (!f) return hipErrorInvalidValue;
    // a tile must hold every segment of its windows (fold: 4 R windows in
    // kFoldSlideSegs segments; plain bank: 64 segments)
    if (p.slide_wt > 0 && (detector == kDetResidue || p.log2g != 4 || p.hop % 64 || p.hop < 64 ||
                           (p.slide_wt - 1) * (p.hop / 64) + 16 >
                               (detector == kDetFolded ? kFoldSlideSegs : 64) ||
                           (detector == kDetFolded && p.slide_wt % 4)))
        return hipErrorInvalidValue;
    const size_t lds = detector == kDetResidue ? residue_lds_bytes(p.k, p.log2g) : 0;
    const int wpb = detector == kDetResidue ? kWavesPerBlock : kPlainWPB;
    void *args[] = {const_cast<GoertzelParams *>(&p)};
    return hipLaunchKernel(f, dim3(tile_grid(p.n_windows, p.log2g, wpb, p.slide_wt)), dim3(64 * wpb),
                           args, lds, s);
}

}  // namespace fskd
