"""Pinning the oracle before trusting it (CPU only).

The reference has no demodulator, so the Goertzel
restatement has no reference counterpart to be compared with directly. Its
spectral values are pinned to the reference's OWN FFT code (opus_fft_c,
libopus celt/kiss_fft.c:569-589, fixed point, static sizes 480/240/120/60;
golden fixture tests/golden/ref_kissfft.npz, regenerated and checked live
when oracle/_ref is built) to the reference's Q15 precision, and to
independent known answers (numpy.fft at integer bins, a direct double DFT at
arbitrary frequencies, closed-form pure tone magnitudes, Parseval) at 1e-9;
plus the committed golden vectors.
"""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FS = 48000.0


def test_goertzel_equals_numpy_fft_at_integer_bins(O):
    for n, bins in ((1024, (32, 64)), (1024, tuple(32 + 8 * i for i in range(8))), (256, (3, 17, 100))):
        freqs = tuple(b * FS / n for b in bins)
        pcm, _ = O.synth_fsk(freqs, n, 50, 3, 8000, 2000)
        _, P = O.goertzel(pcm, freqs, n)
        X = np.fft.rfft(pcm.astype(np.float64), axis=1)
        Pf = np.abs(X[:, list(bins)]) ** 2
        assert np.abs(P - Pf).max() <= 1e-9 * Pf.max()


def test_goertzel_equals_direct_dft_noninteger(O):
    rng = np.random.default_rng(0)
    freqs = (433.3, 1777.7, 5012.9, 11111.1, 23999.0)
    for _ in range(5):
        x = rng.integers(-32768, 32768, 777).astype(np.int16)
        _, P = O.goertzel(x, freqs, 777)
        Pd = O.dft_power(x, freqs)
        n = np.arange(777)
        Pn = np.array([np.abs((x * np.exp(-2j * np.pi * f / FS * n)).sum()) ** 2 for f in freqs])
        assert np.allclose(P[0], Pd, rtol=1e-9, atol=1e-3)
        assert np.allclose(P[0], Pn, rtol=1e-9, atol=1e-3)


def test_pure_tone_closed_form(O):
    n, k, A_ = 1024, 48, 10000
    t = np.arange(n)
    x = np.round(A_ * np.cos(2 * np.pi * k * t / n)).astype(np.int16)
    _, P = O.goertzel(x, (k * FS / n, (k + 5) * FS / n), n)
    X = (x.astype(np.float64) * np.exp(-2j * np.pi * k * t / n)).sum()
    assert abs(P[0, 0] - abs(X) ** 2) <= 1e-9 * abs(X) ** 2
    assert abs(np.sqrt(P[0, 0]) - A_ * n / 2) < 0.5 * n      # |X| = A N / 2 up to rounding
    assert P[0, 1] < 1e-6 * P[0, 0]                          # orthogonal bin


def test_impulse_and_dc(O):
    n = 64
    x = np.zeros(n, np.int16)
    x[5] = 1000
    _, P = O.goertzel(x, (750.0, 3000.0, 10000.0), n)
    assert np.allclose(P[0], 1e6, rtol=1e-12)                # |X| = 1000 at every freq
    x = np.full(n, 7, np.int16)
    _, P = O.goertzel(x, (0.0,), n)
    assert np.isclose(P[0, 0], (7 * n) ** 2)


def test_argmax_ties_go_to_lowest_index(O):
    x = np.zeros((3, 64), np.int16)
    sym, P = O.goertzel(x, (750.0, 1500.0, 2250.0), 64)
    assert (sym == 0).all() and (P == 0).all()


def test_fft_oracle_matches_numpy(O):
    rng = np.random.default_rng(2)
    for n in (8, 64, 1024):
        x = rng.integers(-32768, 32768, n).astype(np.int16)
        P = O.fft_power(x)
        Pn = np.abs(np.fft.rfft(x.astype(np.float64))) ** 2
        assert np.allclose(P, Pn, rtol=1e-9, atol=1e-3 * n)
        # Parseval
        full = np.abs(np.fft.fft(x.astype(np.float64))) ** 2
        assert np.isclose(full.sum(), n * (x.astype(np.float64) ** 2).sum())


def test_fft_demod_equals_goertzel_at_integer_bins(O):
    freqs = tuple(1500.0 + 375.0 * i for i in range(8))
    pcm, truth = O.synth_fsk(freqs, 1024, 40, 4)
    s1, P1 = O.goertzel(pcm, freqs, 1024)
    s2, P2 = O.fft_demod(pcm, freqs, 1024)
    assert (s1 == s2).all() and (s1 == truth).all()
    assert np.allclose(P1, P2, rtol=1e-9)


def test_fp32_single_chain_error_is_why_segments_exist(O):
    """The sequential fp32 recurrence over 1024 samples misses the 1e-5 bar on
    some windows — the reason the GPU kernel runs 64-sample lane segments."""
    freqs = tuple(1500.0 + 375.0 * i for i in range(8))
    pcm, _ = O.synth_fsk(freqs, 1024, 2000, 6)
    _, P = O.goertzel(pcm, freqs, 1024)
    _, P32 = O.goertzel_f32(pcm, freqs, 1024)
    err = (np.abs(P32 - P).max(1) / P.max(1)).max()
    assert err > 1e-6


def test_omp_equals_serial(O):
    pcm, _ = O.synth_fsk((1500.0, 3000.0), 1024, 300, 8)
    a = O.goertzel(pcm, (1500.0, 3000.0), 1024)
    b = O.goertzel(pcm, (1500.0, 3000.0), 1024, threads=4)
    assert (a[0] == b[0]).all() and (a[1] == b[1]).all()


def test_generator_properties(O):
    freqs = (1500.0, 3000.0)
    pcm, sym = O.synth_fsk(freqs, 1024, 4000, 0x2C5DA044)
    assert pcm.dtype == np.int16 and np.abs(pcm.astype(np.int32)).max() <= 8000 + 4 * 400
    assert abs(sym.mean() - 0.5) < 0.03
    # w0 offsets address the same stream
    p2, s2 = O.synth_fsk(freqs, 1024, 10, 0x2C5DA044, w0=100)
    assert (p2 == pcm[100:110]).all() and (s2 == sym[100:110]).all()
    lut = O.sine_lut()
    assert lut[0] == 0 and lut[4096] == 32767 and lut[12288] == -32767


@pytest.mark.parametrize("name", ["fsk2_n1024", "fsk8_n1024", "k5_nonint_n512", "fsk2_hop256",
                                  "fsk4_n256_lowsnr"])
def test_oracle_reproduces_golden(O, name):
    g = np.load(os.path.join(HERE, "golden", name + ".npz"), allow_pickle=False)
    n, hop = int(g["n"]), int(g["hop"])
    sym, P = O.goertzel(g["pcm"], tuple(g["freqs"]), n, hop)
    assert (sym == g["sym"]).all()
    assert np.array_equal(P, g["P"])
    # regenerate the input from its seed
    W = g["pcm"].size // n
    pcm, truth = O.synth_fsk(tuple(g["freqs"]), n, W, int(g["seed"]), int(g["amplitude"]),
                             int(g["sigma"]))
    assert (pcm.reshape(-1) == g["pcm"]).all() and (truth == g["truth"]).all()


def test_stream_oracle_golden_and_batch_equivalence(O):
    g = np.load(os.path.join(HERE, "golden", "stereo_stream.npz"), allow_pickle=False)
    inter, n = g["pcm"], int(g["n"])
    freqs = tuple(g["freqs"])
    for mode in (0, 1, 2):
        L = inter[0::2].astype(np.int32)
        R = inter[1::2].astype(np.int32)
        mono = {0: L, 1: R, 2: (L + R) >> 1}[mode].astype(np.int16)
        sym, P = O.goertzel(mono, freqs, n)
        assert (sym == g[f"sym_mode{mode}"]).all()
        assert np.array_equal(P, g[f"P_mode{mode}"])
        assert int(g[f"pending_mode{mode}"]) == mono.size % n


def test_stream_oracle_sliding(O):
    pcm, _ = O.synth_fsk((1500.0, 3000.0), 1024, 6, 10)
    flat = pcm.reshape(-1)
    st = O.Stream((1500.0, 3000.0), n=1024, hop=256)
    got = np.concatenate([st.push(flat[i:i + 700])[0] for i in range(0, flat.size, 700)])
    want, _ = O.goertzel(flat, (1500.0, 3000.0), 1024, 256)
    assert (got == want).all()


def test_fft_demod_omp_equals_serial(O):
    pcm, _ = O.synth_fsk((1500.0, 3000.0), 1024, 20, 12)
    a = O.fft_demod(pcm, (1500.0, 3000.0), 1024, 256)
    b = O.fft_demod(pcm, (1500.0, 3000.0), 1024, 256, threads=4)
    assert (a[0] == b[0]).all() and np.array_equal(a[1], b[1])


# ---- the reference's own FFT (opus_fft_c) ------------------------------------
# Tolerance: opus_fft_c is fixed point (Q15 twiddles, 1/N scale in Q15,
# kiss_fft.c:578-584); its |X|^2 errors scale with the frame's energy, so the
# bar is relative to the Parseval total N * sum(x^2) (measured <= 1.7e-4, at
# DC; <= 3.5e-5 elsewhere).
REF_FFT_TOL = 3e-4


def _ref_kissfft_golden():
    return np.load(os.path.join(HERE, "golden", "ref_kissfft.npz"), allow_pickle=False)


def _ref_powers(g, n):
    Y = (g[f"re{n}"] + 1j * g[f"im{n}"]) * n / 2.0 ** int(g["preshift"])
    return np.abs(Y[:, : n // 2 + 1]) ** 2


@pytest.mark.parametrize("n", [1024, 480, 240, 120, 60])
def test_oracle_goertzel_pinned_to_reference_fft(O, n):
    """Oracle Goertzel powers at every bin of the n-point frame equal the
    reference opus_fft_c's |X|^2 (golden outputs) to the reference's Q15
    precision; at n = 480, where the 2-FSK tones are bins 15 and 30, the
    oracle's symbol is the argmax of the reference spectrum at those bins.
    n = 1024 (the north-star window) is the CUSTOM_MODES build of the same
    kiss_fft.c; there the oracle's 2-FSK (bins 32, 64) and 8-FSK (bins
    32 + 8 i) symbols are the argmax of the reference spectrum."""
    g = _ref_kissfft_golden()
    x = g[f"x{n}"]
    Pr = _ref_powers(g, n)
    freqs = [k * FS / n for k in range(n // 2 + 1)]
    for i, row in enumerate(x):
        P = np.concatenate([O.goertzel(row, freqs[c:c + 16], n)[1][0]
                            for c in range(0, len(freqs), 16)])
        energy = n * float((row.astype(np.float64) ** 2).sum())
        assert np.abs(P - Pr[i]).max() <= REF_FFT_TOL * max(energy, 1.0), (n, i)
    if n == 480:
        sym, _ = O.goertzel(x[:4], (1500.0, 3000.0), n)
        assert (sym == np.argmax(Pr[:4][:, [15, 30]], axis=1)).all()
    if n == 1024:
        sym, _ = O.goertzel(x[:4], (1500.0, 3000.0), n)
        assert (sym == np.argmax(Pr[:4][:, [32, 64]], axis=1)).all()
        f8 = tuple(1500.0 + 375.0 * i for i in range(8))
        sym, _ = O.goertzel(x[4:8], f8, n)
        assert (sym == np.argmax(Pr[4:8][:, [32 + 8 * i for i in range(8)]], axis=1)).all()
        # and the FFT oracle's full spectrum against the reference's
        for i, row in enumerate(x):
            Pf = O.fft_power(row)
            energy = n * float((row.astype(np.float64) ** 2).sum())
            assert np.abs(Pf - Pr[i]).max() <= REF_FFT_TOL * max(energy, 1.0), i


def test_reference_fft_golden_is_live_reference_output(O):
    """The committed golden outputs are what the reference's opus_fft_c
    (oracle/_ref/libkissfft_ref.so, built from /root/reference) computes."""
    if O.ref_kissfft() is None:
        pytest.skip("oracle/_ref/libkissfft_ref.so not built (needs /root/reference)")
    g = _ref_kissfft_golden()
    assert int(g["preshift"]) == O.KISSFFT_PRESHIFT
    for which in range(4):
        n = O.ref_kissfft().ref_fft_static_size(which)
        y = np.stack([O.ref_fft_static(which, row) for row in g[f"x{n}"]])
        assert np.array_equal(y.real, g[f"re{n}"]) and np.array_equal(y.imag, g[f"im{n}"])


def test_reference_fft1024_golden_is_live_reference_output(O):
    """The committed N = 1024 outputs are what the reference's kiss_fft.c,
    compiled with CUSTOM_MODES (oracle/_ref/libkissfft_custom.so), computes;
    at the static sizes that build agrees with the static states bit for bit."""
    if O.ref_kissfft_custom() is None:
        pytest.skip("oracle/_ref/libkissfft_custom.so not built (needs /root/reference)")
    g = _ref_kissfft_golden()
    y = np.stack([O.ref_fft_custom(row) for row in g["x1024"]])
    assert np.array_equal(y.real, g["re1024"]) and np.array_equal(y.imag, g["im1024"])
    for n in (480, 240):
        y = np.stack([O.ref_fft_custom(row) for row in g[f"x{n}"][:3]])
        assert np.array_equal(y.real, g[f"re{n}"][:3]) and np.array_equal(y.imag, g[f"im{n}"][:3])


def test_oracle_rejects_too_many_tones(O):
    with pytest.raises(ValueError):
        O.goertzel(np.zeros(64, np.int16), [100.0] * 65, 64)


def test_stream_lead_in_drops_frames(O):
    """oracle.Stream(lead_in=L) equals the plain stream over pcm[L:] (the
    demod_cfg_t.lead_in contract), whatever the packet sizes."""
    import numpy as np
    pcm, _ = O.synth_fsk((1500.0, 3000.0), 1024, 12, 99)
    x = pcm.reshape(-1)
    for L in (0, 1, 312, 1024, 5000):
        s = O.Stream((1500.0, 3000.0), lead_in=L)
        got = np.concatenate([s.push(x[i:i + 2880])[0] for i in range(0, x.size, 2880)])
        want, _ = O.goertzel(x[L:], (1500.0, 3000.0), 1024)
        assert np.array_equal(got, want)
        assert s.pending() == (x.size - L) % 1024
    st = np.empty(2 * x.size, np.int16)
    st[0::2], st[1::2] = x, -x
    s = O.Stream((1500.0, 3000.0), channels=2, channel_mode=1, lead_in=312)
    got = np.concatenate([s.push(st[i:i + 5760])[0] for i in range(0, st.size, 5760)])
    want, _ = O.goertzel(-x[312:], (1500.0, 3000.0), 1024)
    assert np.array_equal(got, want)
