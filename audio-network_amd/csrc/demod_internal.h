// demod_internal.h — shared between the C-ABI host layer and the kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace fskd {

constexpr int kSeg = 64;              // samples per lane segment
constexpr int kTileSamples = 64 * kSeg;  // samples one wave owns per tile (8 KiB)
constexpr int kWavesPerBlock = 4;
constexpr int kLdsSegStride = 144;    // bytes: 128 B segment + 16 B pad (conflict-free b128 reads)
constexpr int kLdsWaveBytes = 64 * kLdsSegStride;
constexpr int kMaxTones = 16;

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
    float coef[kMaxTones];   // 2 cos(w_k)
};

struct SynthParams {
    uint64_t seed;
    uint64_t w0;             // index of the first generated window in the stream
    long long n_windows;
    int n;                   // samples per window (multiple of 8)
    int k;
    int amplitude;
    int sigma;
    const int16_t *lut;      // 16384-entry Q15 sine table (device)
    int16_t *pcm;
    uint8_t *sym;
    uint32_t inc[kMaxTones];  // phase increment per sample, 2^32 / cycle
};

hipError_t launch_goertzel(const GoertzelParams &p, int grid, hipStream_t s);
int goertzel_grid(int k, long long n_windows, int log2g, int device, int device_cus);
hipError_t launch_synth(const SynthParams &p, hipStream_t s);

}  // namespace fskd
