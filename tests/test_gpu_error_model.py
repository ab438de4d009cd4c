"""The decision rescue's derived error bounds, asserted on every window
(tests/error_model.py): for every detector path and tone
plan of error_model.CASES (plain bank at the Reinsch edge, near Nyquist,
n = 256 / 4096, segment-shared; fold incl. F16, edge bins, n = 256 / 4096,
fold-slide; residue with compile-time and LDS classes, n = 256 / 4096; FFT at
hop 1024 / 256) and every adversarial signal family (FSK at sigma 0 / 400,
full scale with clipping, full-scale clipped square waves, DC offset + tone,
uniform full-scale int16, dithered silence, two tones at equal power, a tone
cancelling itself, a near-Nyquist tone beside a plan tone):
  * every fp32 tone power is within the derived bound of the oracle's
    (|sqrt P_gpu - sigma P_oracle| <= rho_det sqrt E_det + rho_ref sqrt E);
  * the kernel flags exactly the windows the stated threshold selects;
  * every window it leaves unflagged already carries the oracle's symbol;
  * quiet input is not flagged wholesale (the round-3 threshold
    used the int16 worst-case energy and flagged every window of dithered
    silence).
And the kernels' fp32 powers equal tests/fp32emu.py's operation-for-operation
emulation bit for bit (test_kernels_equal_emulation), which ties the CPU
check of the bounds (tests/test_error_bound.py) to the shipped code.
"""
import json
import math
import os

import pytest

import error_model as EM

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


@pytest.mark.parametrize("case", EM.CASES, ids=[c[0] for c in EM.CASES])
def test_error_model_every_window(A, O, torch, case):
    rows = []
    out = os.environ.get("FSKD_ERROR_MODEL_OUT")  # optional: the rows as JSON lines (profiles)
    for fam in EM.FAMILIES:
        r = EM.evaluate(A, O, case, fam, W=4096)
        rows.append(r)
        print(json.dumps({k: v for k, v in r.items()}))
        if out:
            with open(out, "a") as f:
                f.write(json.dumps(r) + "\n")
    for r in rows:
        assert r["tau"] > 0
        assert r["flag_missed"] == 0 and r["flag_extra"] == 0, r
        assert r["unflagged_wrong"] == 0, r
        assert r["worst_ratio_to_model"] <= 1.0, r
        if r["family"] == "quiet_s3":
            assert r["flagged"] <= 0.03 * r["windows"], r
    worst = max(rows, key=lambda r: r["worst_err_frac_of_tau"])
    print("worst error as a fraction of tau:", worst["case"], worst["family"],
          worst["worst_err_frac_of_tau"])


@pytest.mark.parametrize("case", EM.CASES, ids=[c[0] for c in EM.CASES])
def test_rescued_decisions_every_window(A, O, torch, case):
    """The same paths with the rescue on (shipped): on the families that flag
    the most windows (two tones at equal power: every window; clipped square
    waves; a near-Nyquist tone beside a plan tone; dithered silence) every
    window's symbol is the oracle's and no flag bit is left — through the
    in-kernel rescue's first pass by segments and its exact chain, the
    rescue launch (segment-shared windows, n != 1024) and the FFT's."""
    import numpy as np
    name, freqs, n, hop, method = case
    W = 4096
    seed0 = int(os.environ.get("FSKD_SWEEP_SEED", "7"))
    fams = (EM.FAMILIES if os.environ.get("FSKD_SWEEP_ALL") else
            ("two_tone_equal", "clipped_square", "near_nyquist_tone", "quiet_s3"))
    for fi, fam in enumerate(fams):
        blocks = -(-((W - 1) * hop + n) // n)
        x = EM.family(fam, freqs, n, blocks, seed0 + fi)[:(W - 1) * hop + n]
        with A.Demodulator(A.make_cfg(n=n, hop=hop, freqs=freqs, method=method)) as d:
            fft = int(d.method) == 2
            sym = d.batch(x, n_windows=W)
        rs, _ = (O.fft_demod if fft else O.goertzel)(x, freqs, n, hop=hop, fs=EM.FS, threads=16)
        assert not (sym & 0x80).any(), (name, fam)
        bad = np.flatnonzero(sym != rs[:W])
        assert bad.size == 0, (name, fam, bad[:8].tolist())


@pytest.mark.parametrize("plan", ["fsk2", "fsk8"])
@pytest.mark.parametrize("hop", [128, 256, 384])
def test_rescue_launch_equals_in_kernel_rescue(A, O, torch, monkeypatch, plan, hop):
    """The rescue launch of segment-shared windows (rescue.hip
    rescue_seg_kernel: pass 0 by shared segment states in dense runs, per
    window otherwise, by the fold for fold plans; then the exact chain) runs
    the in-kernel rescue's arithmetic (demod_internal.h rescue_rows), so on
    two tones at equal power (every window flagged and rescued) every
    segment-shared window that starts at a multiple of n carries the same
    symbol and magnitude bits as the direct kernel's window at hop = n, with
    pass 0 on both sides (round 5), and every symbol is the oracle's. (The
    2-FSK plain bank takes pass 0 by the fold at hop = n and by shared
    segments at hop < n: FSKD_PASS0_FOLD=0 puts both on segments here.)"""
    import numpy as np
    freqs = A.FSK2_FREQS if plan == "fsk2" else A.FSK8_FREQS
    n, blocks = 1024, 96
    x = EM.family("two_tone_equal", freqs, n, blocks, 11)
    if plan == "fsk2":
        monkeypatch.setenv("FSKD_PASS0_FOLD", "0")
    with A.Demodulator(A.make_cfg(n=n, hop=n, freqs=freqs)) as d:
        sym_d, mag_d = d.batch(x, mags=True)
    W = (x.size - n) // hop + 1
    with A.Demodulator(A.make_cfg(n=n, hop=hop, freqs=freqs)) as d:
        assert d.slide_windows > 0
        sym_s, mag_s = d.batch(x, n_windows=W, mags=True)
    rs, _ = O.goertzel(x, freqs, n, hop=hop, fs=EM.FS, threads=16)
    assert not (sym_s & 0x80).any()
    assert np.array_equal(sym_s, rs[:W])
    # the segment-shared windows that start at a multiple of n
    w = np.arange(0, W, n // math.gcd(n, hop))
    dw = w * hop // n
    keep = dw < sym_d.size
    w, dw = w[keep], dw[keep]
    assert w.size > 8
    assert np.array_equal(sym_s[w], sym_d[dw])
    assert np.array_equal(mag_s[w].view(np.uint32), mag_d[dw].view(np.uint32))


# the direct kernels of each path (the segment-shared ones are bit-identical
# to them: test_gpu_slide.py, test_gpu_fold_slide.py)
EMU_CASES = [c for c in EM.CASES if c[2] == c[3] and c[4] != 2] + [
    ("plain_k16_n4096", tuple(700.0 + 1234.5 * i for i in range(16)), 4096, 4096, 1),
    ("residue_k16", tuple(EM.BIN * (20 + 7 * i) for i in range(16)), 1024, 1024, 4),
    ("plain_k3_ws", (1500.0, 2250.0, 3000.0), 1024, 1024, 1),
]


@pytest.mark.parametrize("case", EMU_CASES, ids=[c[0] for c in EMU_CASES])
def test_kernels_equal_emulation(A, O, torch, case):
    """The detector's fp32 tone powers (rescue off: FSKD_NO_RESCUE=1) equal
    fp32emu.detector_powers bit for bit on adversarial families."""
    import numpy as np
    import fp32emu as E
    name, freqs, n, hop, method = case
    W = 512
    cfg = A.make_cfg(n=n, hop=hop, freqs=freqs, method=method)
    info = A.plan_info(cfg)
    old = os.environ.get("FSKD_NO_RESCUE")
    os.environ["FSKD_NO_RESCUE"] = "1"
    try:
        d = A.Demodulator(cfg)
    finally:
        if old is None:
            del os.environ["FSKD_NO_RESCUE"]
        else:
            os.environ["FSKD_NO_RESCUE"] = old
    with d:
        for fi, fam in enumerate(("fsk_s400", "two_tone_equal", "random_full", "near_nyquist_tone")):
            x = EM.family(fam, freqs, n, W, 300 + fi)[:W * n]
            _, mag = d.batch(x, n_windows=W, mags=True)
            emu = E.detector_powers(info, x, n, n, W, len(freqs))
            diff = np.flatnonzero((mag != emu).any(axis=1))
            assert diff.size == 0, (name, fam, diff.size, diff[:4].tolist(),
                                    mag[diff[:1]].tolist(), emu[diff[:1]].tolist())


def test_fft_kernel_equals_emulation(A, O, torch):
    """The FFT detector's full 513-bin spectrum equals fp32emu.fft_spectrum bit
    for bit (rescue off), at hop 1024 and hop 256."""
    import numpy as np
    import fp32emu as E
    old = os.environ.get("FSKD_NO_RESCUE")
    os.environ["FSKD_NO_RESCUE"] = "1"
    try:
        for hop in (1024, 256):
            d = A.Demodulator(A.make_cfg(hop=hop, freqs=A.FSK8_FREQS, method=A.METHOD_FFT))
            with d:
                for fi, fam in enumerate(("fsk_s400", "random_full", "near_nyquist_tone")):
                    W = 256
                    blocks = -(-((W - 1) * hop + 1024) // 1024)
                    x = EM.family(fam, A.FSK8_FREQS, 1024, blocks, 400 + fi)[:(W - 1) * hop + 1024]
                    xt = torch.from_numpy(x).cuda()
                    sym = torch.empty(W, dtype=torch.uint8, device="cuda")
                    spec = torch.empty(W * 513, dtype=torch.float32, device="cuda")
                    d.batch_spectrum_async(xt, W, sym, None, spec)
                    torch.cuda.synchronize()
                    got = spec.cpu().numpy().reshape(W, 513)
                    emu = E.fft_spectrum(x, hop, W)
                    diff = np.flatnonzero((got != emu).any(axis=1))
                    assert diff.size == 0, (hop, fam, diff.size, diff[:4].tolist())
    finally:
        if old is None:
            del os.environ["FSKD_NO_RESCUE"]
        else:
            os.environ["FSKD_NO_RESCUE"] = old


FFT_TONE_PLANS = {
    "fsk2": [32, 64],
    "fsk8": [32 + 8 * i for i in range(8)],
    "all": [3 + 31 * i for i in range(16)],
}


@pytest.mark.parametrize("hop", [1024, 256])
@pytest.mark.parametrize("plan", sorted(FFT_TONE_PLANS))
def test_fft_tones_only_kernel_equals_emulation(A, O, torch, plan, hop):
    """the SHIPPED tones-only FFT instantiation (the device
    batch with magnitudes and no spectrum: PICK 2, the pair-block post-pass
    mask fft_pmask, OVL at hop < n; the configs[3] kernel) equals
    fp32emu.fft_spectrum at the plan's tone bins bit for bit (rescue off), so
    the CPU proof of the FFT bound (tests/test_error_bound.py over the
    emulation) covers the code the bench times. Nearest reference FFT:
    kiss_fft.c:569-589 (tests/test_gpu_parity.py pins the spectrum to it)."""
    import numpy as np
    import fp32emu as E
    bins = FFT_TONE_PLANS[plan]
    freqs = tuple(EM.BIN * b for b in bins)
    cfg = A.make_cfg(hop=hop, freqs=freqs, method=A.METHOD_FFT)
    info = A.plan_info(cfg)
    if plan != "all":
        assert bin(info["fft_pmask"] & 0xFF).count("1") < 8   # the post-pass is masked
    old = os.environ.get("FSKD_NO_RESCUE")
    os.environ["FSKD_NO_RESCUE"] = "1"
    try:
        d = A.Demodulator(cfg)
    finally:
        if old is None:
            del os.environ["FSKD_NO_RESCUE"]
        else:
            os.environ["FSKD_NO_RESCUE"] = old
    with d:
        for fi, fam in enumerate(("fsk_s400", "two_tone_equal", "random_full", "near_nyquist_tone")):
            W = 1024 + 3
            blocks = -(-((W - 1) * hop + 1024) // 1024)
            x = EM.family(fam, freqs, 1024, blocks, 500 + fi)[:(W - 1) * hop + 1024]
            xt = torch.from_numpy(x).cuda()
            sym = torch.empty(W, dtype=torch.uint8, device="cuda")
            mag = torch.empty((W, len(bins)), dtype=torch.float32, device="cuda")
            d.batch_async(xt, W, sym, mag)
            torch.cuda.synchronize()
            got = mag.cpu().numpy()
            emu = E.fft_spectrum(x, hop, W)[:, bins]
            diff = np.flatnonzero((got.view(np.uint32) != emu.astype(np.float32).view(np.uint32)).any(axis=1))
            assert diff.size == 0, (plan, hop, fam, diff.size, diff[:4].tolist(), got[diff[:1]].tolist(),
                                    emu[diff[:1]].tolist())
