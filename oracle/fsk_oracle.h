/*
 * fsk_oracle.h — TEST INFRASTRUCTURE ONLY (not shipped, never on the product
 * path). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load liboracle.so, and only as the checker / CPU baseline.
 *
 * Scalar CPU restatement of the north-star path.
 *
 * PARITY STATUS: the reference (tmarsteel/audio-network) contains no
 * Goertzel / FSK demodulator at all, so the decision has
 * no reference counterpart. The spectral values are pinned to the
 * reference's own FFT, opus_fft_c (libopus celt/kiss_fft.c:569-589, built in
 * place by oracle/ref.mk; golden tests/golden/ref_kissfft.npz), to its Q15
 * precision, and to independent known answers (tests/test_oracle.py):
 * numpy.fft bins, a direct double DFT at non-integer frequencies, closed-form
 * pure-tone magnitudes, and the committed golden vectors in tests/golden/.
 */
#ifndef FSK_ORACLE_H
#define FSK_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Seeded FSK test signal (DESIGN.md §Synthetic input). Integer-exact. */
void oracle_sine_lut(int16_t lut[16384]);
void oracle_synth_fsk(double fs, uint32_t n, uint32_t k, const double *freqs,
                      uint64_t seed, size_t w0, size_t n_windows,
                      int amplitude, int sigma, int16_t *pcm, uint8_t *syms);

/* Goertzel tone bank in double, sequential recurrence.
 * Window w = x[w*hop .. w*hop+n). P may be NULL. */
void oracle_goertzel(const int16_t *x, size_t n_windows, size_t hop,
                     uint32_t n, uint32_t k, const double *freqs, double fs,
                     uint8_t *sym, double *P);

/* Same with an OpenMP parallel-for over windows (CPU baseline). */
void oracle_goertzel_omp(const int16_t *x, size_t n_windows, size_t hop,
                         uint32_t n, uint32_t k, const double *freqs,
                         double fs, uint8_t *sym, double *P, int threads);

/* fp32 sequential variant (diagnostic only: shows the single-chain error). */
void oracle_goertzel_f32(const int16_t *x, size_t n_windows, size_t hop,
                         uint32_t n, uint32_t k, const double *freqs,
                         double fs, uint8_t *sym, float *P);

/* Direct DFT power |sum x[n] e^{-j w n}|^2 in double (independent check). */
void oracle_dft_power(const int16_t *x, uint32_t n, uint32_t k,
                      const double *freqs, double fs, double *P);

/* Full-spectrum power |X[b]|^2, b = 0..n/2, by an iterative radix-2 FFT in
 * double (n a power of two), for the FFT detector. */
int oracle_fft_power(const int16_t *x, uint32_t n, double *P);

/* FFT detector: symbol = argmax over tone bins b_i = round(f_i*n/fs). */
int oracle_fft_demod(const int16_t *x, size_t n_windows, size_t hop,
                     uint32_t n, uint32_t k, const double *freqs, double fs,
                     uint8_t *sym, double *P);

int oracle_fft_demod_omp(const int16_t *x, size_t n_windows, size_t hop,
                         uint32_t n, uint32_t k, const double *freqs, double fs,
                         uint8_t *sym, double *P, int threads);

/* Streaming restatement of demodulate(pcm, n). */
typedef struct oracle_stream oracle_stream_t;
oracle_stream_t *oracle_stream_create(uint32_t n, uint32_t hop,
                                      uint32_t channels, int channel_mode,
                                      uint32_t k, const double *freqs,
                                      double fs);
void oracle_stream_destroy(oracle_stream_t *st);
/* returns symbols emitted (written to sym / P[k*i]) */
long oracle_stream_push(oracle_stream_t *st, const int16_t *pcm,
                        size_t n_frames, uint8_t *sym, double *P,
                        size_t cap);
int oracle_stream_pending(const oracle_stream_t *st);
/* Drop the next `frames` input frames before any window is formed (the
 * demod_cfg_t.lead_in contract: e.g. the 312-sample Opus decoder delay). */
void oracle_stream_set_lead_in(oracle_stream_t *st, uint32_t frames);

#ifdef __cplusplus
}
#endif
#endif
