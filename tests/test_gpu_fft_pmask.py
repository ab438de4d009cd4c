"""Tones-only FFT batches run the real split's post-pass only in the pair
blocks that hold a tone bin (fft_quad.hip PICK 2, FftParams::pmask; round 5):
the 512-point complex FFT is computed in full, and each tone's pair is the
same operation sequence as in the full post-pass, so every tone power is the
full post-pass's bit for bit (FSKD_FFT_PMASK=0 runs every block, the kernel
of round 4). Stage 2 of the flag test takes E = n sum x^2 from the samples
instead of Parseval over all 513 bin powers; the flags it sets are checked
against the stated threshold by test_gpu_error_model.py (fft cases).
"""
import os

import numpy as np
import pytest

import error_model as EM

pytestmark = pytest.mark.gpu
N = 1024


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def quad_slot(b):
    """fft_quad.hip quad_slot, restated."""
    u, v = b & 31, b >> 5
    if b in (0, 512):
        return 512 + (b >> 9)
    if u == 0:
        return 2 * (16 * v) if v > 8 else 256 if v == 8 else 2 * (16 * (16 - v)) + 1
    if u == 16:
        return 2 * (16 * v) if v < 8 else 2 * (16 * (15 - v)) + 1
    if u < 16:
        return 2 * (16 * v + u)
    return 2 * (16 * (15 - v) + (32 - u)) + 1


def pmask(bins):
    m = 0
    for b in bins:
        f = quad_slot(b)
        if f < 512:
            m |= 1 << ((f >> 5) >> 1)
    return m


PLANS = {
    "fsk2": [32, 64],
    "fsk8": [32 + 8 * i for i in range(8)],
    "edges": [0, 16, 256, 512],          # Z[0] side bins, lane 0's column 16, X[256]
    "lane0": [32, 48, 288, 304, 480],    # columns 0 and 16 on both sides of 256
    "mirror": [17, 47, 300, 495, 511],   # bins on the mirror side of their pair
    "all": [3 + 31 * i for i in range(16)],
}


def run(A, freqs, hop, x, W, env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        d = A.Demodulator(A.make_cfg(n=N, hop=hop, freqs=freqs, method=A.METHOD_FFT))
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    with d:
        return d.batch(x, n_windows=W, mags=True)


@pytest.mark.parametrize("hop", [1024, 256])
@pytest.mark.parametrize("plan", sorted(PLANS))
def test_pair_blocks_equal_full_post_pass(A, O, torch, plan, hop):
    bins = PLANS[plan]
    freqs = tuple(EM.BIN * b for b in bins)
    info = A.plan_info(A.make_cfg(n=N, hop=hop, freqs=freqs, method=A.METHOD_FFT))
    assert info["fft_pmask"] == pmask(bins)
    W = 1536 + 5
    blocks = -(-((W - 1) * hop + N) // N)
    rng = np.random.default_rng(len(bins) + hop)
    fam = ("fsk_s400", "two_tone_equal", "random_full")[rng.integers(0, 3)]
    x = EM.family(fam, freqs, N, blocks, 5)[:(W - 1) * hop + N]
    s_full, m_full = run(A, freqs, hop, x, W, {"FSKD_NO_RESCUE": "flags", "FSKD_FFT_PMASK": "0"})
    s_pair, m_pair = run(A, freqs, hop, x, W, {"FSKD_NO_RESCUE": "flags"})
    assert np.array_equal(m_full.view(np.uint32), m_pair.view(np.uint32))
    assert np.array_equal(s_full & 0x7F, s_pair & 0x7F)
    # shipped (rescue on): every symbol the oracle's
    sym, _ = run(A, freqs, hop, x, W, {})
    rs, _ = O.fft_demod(x, freqs, N, hop=hop, fs=EM.FS, threads=16)
    assert not (sym & 0x80).any()
    assert np.array_equal(sym, rs[:W])
