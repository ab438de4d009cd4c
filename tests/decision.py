"""The decision rule every detector must follow, checked on every window.

Rule (oracle/fsk_oracle.c goertzel_window_d and
oracle_fft_demod): symbol = argmax_k P_k of the double-precision powers, ties
to the lowest k. The GPU decides in fp32, flags every window whose fp32 top-2
margin is within the powers' error bound, and re-decides the flagged windows
in double with the oracle's own arithmetic (rescue.hip). So:

1. every symbol equals the oracle's, bit for bit, on every window (no band,
   no tolerance);
2. the returned magnitudes agree with it: the symbol's power is a maximum of
   the returned fp32 powers (a rescued window's powers are the double ones
   rounded to fp32, so rounding can tie them, never reverse them);
3. no symbol still carries the detector's "ambiguous" bit (0x80).

The one exemption: a window whose fp32 tone powers are all exactly 0 is
decided as tone 0 without a rescue (silence). Where its oracle powers are not
all 0 they are double rounding noise of an exactly-zero tone content (e.g. a
constant window against integer-bin tones); such a window is accepted only if
the caller passes the window's energy scale `denom` and the oracle's largest
power is below 1e-9 of it.
"""
import numpy as np

MAG_TOL = 1e-5
BAND = 4 * MAG_TOL  # fp32 band (reported only): oracle margins below it need the rescue


def check_decisions(sym, mag, ref_sym, ref_P, denom=None):
    """Assert the rule above; returns the number of windows whose oracle
    top-2 margin lies inside the fp32 band (decided there by the rescue)."""
    sym = np.asarray(sym)
    ref_sym = np.asarray(ref_sym)
    ref_P = np.asarray(ref_P, dtype=np.float64)
    assert (sym & 0x80).sum() == 0, "a symbol still carries the ambiguous flag"
    if denom is None:
        denom = np.maximum(ref_P.max(axis=1), 1e-30)
    bad = sym != ref_sym
    if mag is not None:
        mag = np.asarray(mag)
        silent = (mag == 0).all(axis=1) & (ref_P.max(axis=1) <= 1e-9 * denom) & (sym == 0)
        bad &= ~silent
        picked = mag[np.arange(sym.size), sym.astype(np.int64)]
        notmax = np.flatnonzero(picked < mag.max(axis=1))
        assert notmax.size == 0, ("symbol's power is not a maximum of the returned powers",
                                  notmax[:8], sym[notmax[:8]], mag[notmax[:8]])
    bad = np.flatnonzero(bad)
    assert bad.size == 0, ("decision differs from the double oracle", bad[:8], sym[bad[:8]],
                           ref_sym[bad[:8]])
    if ref_P.shape[1] < 2:
        return 0
    Ps = np.sort(ref_P, axis=1)
    return int(((Ps[:, -1] - Ps[:, -2]) <= BAND * denom).sum())
