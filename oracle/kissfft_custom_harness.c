/*
 * kissfft_custom_harness.c — TEST INFRASTRUCTURE ONLY.
 *
 * The reference's own FFT (hardware/lib/libopus/src/celt/kiss_fft.c) at the
 * north-star window size N = 1024. The static modes (kissfft_ref_harness.c)
 * only hold nfft = 480/240/120/60; kiss_fft.c allocates any other size
 * (radix 2/3/4/5 factorisation, kf_factor / compute_twiddles /
 * opus_fft_alloc_twiddles, kiss_fft.c:315-519) when it is compiled with the
 * libopus configure option CUSTOM_MODES, which the reference's config.h
 * leaves off (config.h:11, "#undef CUSTOM_MODES" commented). oracle/ref.mk
 * therefore compiles kiss_fft.c and mathops.c a second time, in place, with
 * the reference's own config.h plus -DCUSTOM_MODES (a build flag of the
 * reference's own source, no stand-in header), into
 * oracle/_ref/libkissfft_custom.so. FIXED_POINT stays on: twiddles are Q15
 * (kf_cexp2 of celt_cos_norm), nfft = 1024 = 4^5 runs five radix-4 stages,
 * and opus_fft_c divides the input by nfft before them (scale = Q15ONE,
 * scale_shift = 10 for a power of two, kiss_fft.c:578-584).
 */
#include <stdint.h>
#include <stdlib.h>

#include "config.h"
#include "kiss_fft.h"

#define MAX_NFFT 4096

/* opus_fft_c of one real frame x[0..nfft) (imaginary parts 0) with a state
 * allocated for nfft by opus_fft_alloc; outputs (X/nfft in the input's scale)
 * go to re/im as doubles. Returns nfft, -1 if the reference cannot allocate
 * that size, -2 on a bad argument. */
int ref_fft_custom32(int nfft, const int32_t *x, double *re, double *im)
{
    if (nfft <= 0 || nfft > MAX_NFFT || !x || !re || !im) return -2;
    kiss_fft_state *st = opus_fft_alloc(nfft, 0, 0, 0);
    if (!st) return -1;
    kiss_fft_cpx *in = malloc(sizeof(kiss_fft_cpx) * (size_t)nfft);
    kiss_fft_cpx *out = malloc(sizeof(kiss_fft_cpx) * (size_t)nfft);
    if (!in || !out) {
        free(in);
        free(out);
        opus_fft_free(st, 0);
        return -2;
    }
    for (int i = 0; i < nfft; ++i) {
        in[i].r = (kiss_fft_scalar)x[i];
        in[i].i = 0;
    }
    opus_fft_c(st, in, out);
    for (int i = 0; i < nfft; ++i) {
        re[i] = (double)out[i].r;
        im[i] = (double)out[i].i;
    }
    free(in);
    free(out);
    opus_fft_free(st, 0);
    return nfft;
}
