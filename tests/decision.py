"""The decision rule every detector must follow, checked on every window.

Rule (oracle/fsk_oracle.c goertzel_window_d): symbol =
argmax_k P_k with ties to the lowest k. The GPU evaluates it exactly on the
fp32 powers it returns (window_sum.h ws_argmax, the K <= 2 `P > best` chain,
the FFT pick), so:

1. every symbol equals np.argmax of the returned magnitudes (numpy's argmax
   also takes the first of equal maxima) — bit-exact, no tolerance;
2. against the double-precision oracle the symbol is the oracle's wherever
   the oracle's top-2 margin exceeds the fp32 error band (4 x the 1e-5
   magnitude bar, relative to the window's normaliser); inside the band the
   GPU's pick must still be a tone the oracle puts within the band of its
   maximum (a near-tie of the two top tones, decided by fp32 rounding).

No window is exempt.
"""
import numpy as np

MAG_TOL = 1e-5
BAND = 4 * MAG_TOL


def check_decisions(sym, mag, ref_sym, ref_P, denom=None):
    """Assert the rule above; returns the number of windows inside the band."""
    sym = np.asarray(sym)
    ref_P = np.asarray(ref_P, dtype=np.float64)
    if denom is None:
        denom = np.maximum(ref_P.max(axis=1), 1e-30)
    if mag is not None:
        mag = np.asarray(mag)
        own = np.argmax(mag, axis=1)
        bad = np.flatnonzero(own != sym)
        assert bad.size == 0, ("symbol is not the argmax of the returned powers",
                               bad[:8], sym[bad[:8]], mag[bad[:8]])
    if ref_P.shape[1] < 2:
        assert (sym == 0).all()
        return 0
    Ps = np.sort(ref_P, axis=1)
    margin = (Ps[:, -1] - Ps[:, -2]) / denom
    posed = margin > BAND
    bad = np.flatnonzero(posed & (sym != ref_sym))
    assert bad.size == 0, ("decision differs from the oracle outside the fp32 band", bad[:8])
    picked = ref_P[np.arange(sym.size), sym.astype(np.int64)]
    far = np.flatnonzero(picked < Ps[:, -1] - BAND * denom)
    assert far.size == 0, ("picked a tone the oracle puts outside the band of its max", far[:8])
    return int((~posed).sum())
