/*
 * fsk_oracle.c — TEST INFRASTRUCTURE ONLY. See fsk_oracle.h for who may use
 * it and for its parity status (spectra pinned to the reference's own FFT and
 * to independent known answers; the decision itself has no reference
 * counterpart, since the reference has no demodulator).
 *
 * Plain scalar C, double precision, written for clarity, not speed.
 */
#include "fsk_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TWO_PI 6.283185307179586476925286766559

/* ------------------------------------------------------------------------ */
/* Synthetic signal (DESIGN.md §Synthetic input).                             */
/* splitmix64 (Steele, Lea, Flood 2014): counter-based, so any sample can be  */
/* generated independently — the GPU generator evaluates the same function.  */
/* ------------------------------------------------------------------------ */
#define SM_GAMMA 0x9E3779B97F4A7C15ULL

static uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void oracle_sine_lut(int16_t lut[16384])
{
    for (int i = 0; i < 16384; ++i)
        lut[i] = (int16_t)lrint(32767.0 * sin(TWO_PI * (double)i / 16384.0));
}

void oracle_synth_fsk(double fs, uint32_t n, uint32_t k, const double *freqs,
                      uint64_t seed, size_t w0, size_t n_windows,
                      int amplitude, int sigma, int16_t *pcm, uint8_t *syms)
{
    int16_t lut[16384];
    uint32_t inc[64];
    oracle_sine_lut(lut);
    for (uint32_t t = 0; t < k; ++t)
        inc[t] = (uint32_t)((uint64_t)llround(freqs[t] / fs * 4294967296.0) &
                            0xFFFFFFFFULL);
    for (size_t i = 0; i < n_windows; ++i) {
        uint64_t w = (uint64_t)(w0 + i);
        uint64_t rw = mix64(seed + (w + 1) * SM_GAMMA);
        uint32_t sym = (uint32_t)(((rw >> 32) * (uint64_t)k) >> 32);
        uint32_t phase0 = (uint32_t)rw;
        uint64_t ns = mix64(rw ^ 0xA0761D6478BD642FULL);
        if (syms) syms[i] = (uint8_t)sym;
        for (uint32_t s = 0; s < n; ++s) {
            uint32_t ph = phase0 + s * inc[sym];
            int32_t tone = (amplitude * (int32_t)lut[ph >> 18] + 16384) >> 15;
            uint64_t d = mix64(ns + ((uint64_t)s + 1) * SM_GAMMA);
            int64_t u = (int64_t)((d & 0xFFFF) + ((d >> 16) & 0xFFFF) +
                                  ((d >> 32) & 0xFFFF) + (d >> 48));
            int64_t noise = ((u - 131070) * (int64_t)sigma * 113512) >> 32;
            int64_t v = (int64_t)tone + noise;
            if (v > 32767) v = 32767;
            if (v < -32768) v = -32768;
            pcm[i * (size_t)n + s] = (int16_t)v;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* Goertzel tone bank — SURVEY.md §8(a3) recurrence, (a4) magnitude, (a5)    */
/* argmax with ties to the lowest tone index.                               */
/*   c_k = 2 cos(2 pi f_k / fs)                                             */
/*   s[n] = x[n] + c_k s[n-1] - s[n-2],  s[-1] = s[-2] = 0                  */
/*   P_k  = s1^2 + s2^2 - c_k s1 s2  (= |sum x[n] e^{-j w n}|^2)            */
/* ------------------------------------------------------------------------ */
static uint8_t goertzel_window_d(const int16_t *x, uint32_t n, uint32_t k,
                                 const double *c, double *P)
{
    double best = -1.0;
    uint8_t arg = 0;
    for (uint32_t t = 0; t < k; ++t) {
        double s1 = 0.0, s2 = 0.0;
        for (uint32_t i = 0; i < n; ++i) {
            double s = (double)x[i] + c[t] * s1 - s2;
            s2 = s1;
            s1 = s;
        }
        double p = s1 * s1 + s2 * s2 - c[t] * s1 * s2;
        if (P) P[t] = p;
        if (p > best) { best = p; arg = (uint8_t)t; }
    }
    return arg;
}

static void coefs(uint32_t k, const double *freqs, double fs, double *c)
{
    for (uint32_t t = 0; t < k; ++t) c[t] = 2.0 * cos(TWO_PI * freqs[t] / fs);
}

void oracle_goertzel(const int16_t *x, size_t n_windows, size_t hop,
                     uint32_t n, uint32_t k, const double *freqs, double fs,
                     uint8_t *sym, double *P)
{
    double c[64];
    coefs(k, freqs, fs, c);
    for (size_t w = 0; w < n_windows; ++w) {
        uint8_t s = goertzel_window_d(x + w * hop, n, k, c, P ? P + w * k : NULL);
        if (sym) sym[w] = s;
    }
}

void oracle_goertzel_omp(const int16_t *x, size_t n_windows, size_t hop,
                         uint32_t n, uint32_t k, const double *freqs,
                         double fs, uint8_t *sym, double *P, int threads)
{
    double c[64];
    coefs(k, freqs, fs, c);
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static)
#endif
    for (long w = 0; w < (long)n_windows; ++w) {
        uint8_t s = goertzel_window_d(x + (size_t)w * hop, n, k, c,
                                      P ? P + (size_t)w * k : NULL);
        if (sym) sym[w] = s;
    }
    (void)threads;
}

void oracle_goertzel_f32(const int16_t *x, size_t n_windows, size_t hop,
                         uint32_t n, uint32_t k, const double *freqs,
                         double fs, uint8_t *sym, float *P)
{
    double cd[64];
    coefs(k, freqs, fs, cd);
    for (size_t w = 0; w < n_windows; ++w) {
        const int16_t *xw = x + w * hop;
        float best = -1.0f;
        uint8_t arg = 0;
        for (uint32_t t = 0; t < k; ++t) {
            float c = (float)cd[t], s1 = 0.f, s2 = 0.f;
            for (uint32_t i = 0; i < n; ++i) {
                float s = (float)xw[i] + c * s1 - s2;
                s2 = s1;
                s1 = s;
            }
            float p = s1 * s1 + s2 * s2 - c * s1 * s2;
            if (P) P[w * k + t] = p;
            if (p > best) { best = p; arg = (uint8_t)t; }
        }
        if (sym) sym[w] = arg;
    }
}

void oracle_dft_power(const int16_t *x, uint32_t n, uint32_t k,
                      const double *freqs, double fs, double *P)
{
    for (uint32_t t = 0; t < k; ++t) {
        double w = TWO_PI * freqs[t] / fs, re = 0.0, im = 0.0;
        for (uint32_t i = 0; i < n; ++i) {
            re += (double)x[i] * cos(w * (double)i);
            im -= (double)x[i] * sin(w * (double)i);
        }
        P[t] = re * re + im * im;
    }
}

/* ------------------------------------------------------------------------ */
/* Full-spectrum detector: iterative radix-2 DIT FFT, double. */
/* ------------------------------------------------------------------------ */
int oracle_fft_power(const int16_t *x, uint32_t n, double *P)
{
    if (n < 2 || (n & (n - 1))) return -1;
    double *re = (double *)malloc(sizeof(double) * n);
    double *im = (double *)malloc(sizeof(double) * n);
    if (!re || !im) { free(re); free(im); return -7; }
    uint32_t bits = 0;
    while ((1u << bits) < n) ++bits;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t r = 0;
        for (uint32_t b = 0; b < bits; ++b) r |= ((i >> b) & 1u) << (bits - 1 - b);
        re[r] = (double)x[i];
        im[r] = 0.0;
    }
    for (uint32_t len = 2; len <= n; len <<= 1) {
        double ang = -TWO_PI / (double)len;
        for (uint32_t i = 0; i < n; i += len) {
            for (uint32_t j = 0; j < len / 2; ++j) {
                double wr = cos(ang * j), wi = sin(ang * j);
                uint32_t a = i + j, b = i + j + len / 2;
                double tr = re[b] * wr - im[b] * wi;
                double ti = re[b] * wi + im[b] * wr;
                re[b] = re[a] - tr; im[b] = im[a] - ti;
                re[a] += tr;        im[a] += ti;
            }
        }
    }
    for (uint32_t b = 0; b <= n / 2; ++b) P[b] = re[b] * re[b] + im[b] * im[b];
    free(re);
    free(im);
    return 0;
}

int oracle_fft_demod(const int16_t *x, size_t n_windows, size_t hop,
                     uint32_t n, uint32_t k, const double *freqs, double fs,
                     uint8_t *sym, double *P)
{
    double *spec = (double *)malloc(sizeof(double) * (n / 2 + 1));
    if (!spec) return -7;
    for (size_t w = 0; w < n_windows; ++w) {
        int rc = oracle_fft_power(x + w * hop, n, spec);
        if (rc) { free(spec); return rc; }
        double best = -1.0;
        uint8_t arg = 0;
        for (uint32_t t = 0; t < k; ++t) {
            long b = lround(freqs[t] * (double)n / fs);
            if (b < 0) b = 0;
            if (b > (long)(n / 2)) b = (long)(n / 2);
            double p = spec[b];
            if (P) P[w * k + t] = p;
            if (p > best) { best = p; arg = (uint8_t)t; }
        }
        if (sym) sym[w] = arg;
    }
    free(spec);
    return 0;
}

int oracle_fft_demod_omp(const int16_t *x, size_t n_windows, size_t hop,
                         uint32_t n, uint32_t k, const double *freqs, double fs,
                         uint8_t *sym, double *P, int threads)
{
    int rc = 0;
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(static) reduction(| : rc)
#endif
    for (long w = 0; w < (long)n_windows; ++w)
        rc |= oracle_fft_demod(x + (size_t)w * hop, 1, hop, n, k, freqs, fs,
                               sym ? sym + w : NULL, P ? P + (size_t)w * k : NULL);
    (void)threads;
    return rc;
}

/* ------------------------------------------------------------------------ */
/* Streaming demodulate(pcm, n): carry buffer of mono samples, one symbol per */
/* complete window, advance by hop (the carry mirrors the   */
/* transmitter's ring-buffer framing, OpusEncoder.kt:133-150).              */
/* ------------------------------------------------------------------------ */
struct oracle_stream {
    uint32_t n, hop, channels, k;
    int mode;
    double fs;
    double freqs[64];
    double c[64];
    int16_t *buf;
    uint32_t fill;
    uint32_t skip;  /* lead-in frames still to drop */
};

oracle_stream_t *oracle_stream_create(uint32_t n, uint32_t hop,
                                      uint32_t channels, int channel_mode,
                                      uint32_t k, const double *freqs,
                                      double fs)
{
    oracle_stream_t *st = (oracle_stream_t *)calloc(1, sizeof(*st));
    if (!st) return NULL;
    st->n = n; st->hop = hop; st->channels = channels; st->k = k;
    st->mode = channel_mode; st->fs = fs;
    memcpy(st->freqs, freqs, sizeof(double) * k);
    coefs(k, freqs, fs, st->c);
    st->buf = (int16_t *)malloc(sizeof(int16_t) * n);
    if (!st->buf) { free(st); return NULL; }
    return st;
}

void oracle_stream_destroy(oracle_stream_t *st)
{
    if (!st) return;
    free(st->buf);
    free(st);
}

int oracle_stream_pending(const oracle_stream_t *st) { return (int)st->fill; }

void oracle_stream_set_lead_in(oracle_stream_t *st, uint32_t frames) { st->skip = frames; }

static int16_t channel_sample(const oracle_stream_t *st, const int16_t *f)
{
    if (st->channels == 1) return f[0];
    if (st->mode == 0) return f[0];
    if (st->mode == 1) return f[1];
    return (int16_t)(((int32_t)f[0] + (int32_t)f[1]) >> 1);
}

long oracle_stream_push(oracle_stream_t *st, const int16_t *pcm,
                        size_t n_frames, uint8_t *sym, double *P, size_t cap)
{
    long out = 0;
    for (size_t i = 0; i < n_frames; ++i) {
        if (st->skip) {
            --st->skip;
            continue;
        }
        st->buf[st->fill++] = channel_sample(st, pcm + i * st->channels);
        if (st->fill == st->n) {
            if ((size_t)out >= cap) return -2;
            sym[out] = goertzel_window_d(st->buf, st->n, st->k, st->c,
                                         P ? P + (size_t)out * st->k : NULL);
            ++out;
            uint32_t keep = st->n - st->hop;
            memmove(st->buf, st->buf + st->hop, sizeof(int16_t) * keep);
            st->fill = keep;
        }
    }
    return out;
}
