/*
 * kissfft_ref_harness.c — TEST INFRASTRUCTURE ONLY.
 *
 * Exposes the reference's own FFT, opus_fft_c (hardware/lib/libopus/src/
 * celt/kiss_fft.c:569-589; SURVEY.md §8 a6 names it as the reference code
 * nearest to the full-spectrum detector), to the tests, so the oracle's
 * spectral restatement can be pinned to reference code. oracle/ref.mk
 * compiles kiss_fft.c, celt/modes.c (static mode tables,
 * static_modes_fixed.h) and celt/mathops.c in place from /root/reference
 * with the reference's own config.h (FIXED_POINT, no CUSTOM_MODES); output
 * only into oracle/_ref/. With CUSTOM_MODES off the only FFT states are the
 * static ones of the 48 kHz / 960-sample mode: nfft = 480, 240, 120, 60
 * (mdct.kfft[0..3]). opus_fft_c scales its output by 1/nfft in Q15 fixed
 * point (kiss_fft.c:578-584); it is built for Q31-range inputs (the CELT MDCT
 * feeds it pre-shifted data), so callers pre-scale int16 samples (<< 14).
 */
#include <stdint.h>

/* The reference's own build configuration (FIXED_POINT etc.): every
 * reference translation unit includes it, so the harness must see the same
 * kiss_fft_scalar and CELTMode layout. */
#include "config.h"
#include "kiss_fft.h"
#include "modes.h"

static const kiss_fft_state *static_state(int which)
{
    int err = 0;
    const CELTMode *m = opus_custom_mode_create(48000, 960, &err);
    if (!m || which < 0 || which > 3) return 0;
    return m->mdct.kfft[which];
}

/* nfft of static state kfft[which] (which = 0..3), or -1. */
int ref_fft_static_size(int which)
{
    const kiss_fft_state *st = static_state(which);
    return st ? st->nfft : -1;
}

/* opus_fft_c of one real frame x[0..n_in) (n_in must equal the state's nfft)
 * with static state kfft[which]; the reference's fixed-point outputs (X/nfft
 * scaled as the input) go to re/im as doubles. Returns nfft or a negative
 * code. */
int ref_fft_static32(int which, const int32_t *x, int n_in, double *re, double *im)
{
    const kiss_fft_state *st = static_state(which);
    if (!st || st->nfft != n_in || n_in > 480) return -2;
    kiss_fft_cpx in[480], out[480];
    for (int i = 0; i < n_in; ++i) {
        in[i].r = (kiss_fft_scalar)x[i];
        in[i].i = 0;
    }
    opus_fft_c(st, in, out);
    for (int i = 0; i < n_in; ++i) {
        re[i] = (double)out[i].r;
        im[i] = (double)out[i].i;
    }
    return n_in;
}
