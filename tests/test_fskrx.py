"""The C host receiver (audio-network_amd/host/fskrx.c): raw int16 PCM on
stdin -> demodulate() -> delimited ToReceiver frames on stdout."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FSKRX = os.path.join(ROOT, "audio-network_amd", "fskrx")


def _gpu_visible() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="module")
def fskrx():
    subprocess.run(["make", "-C", os.path.join(ROOT, "audio-network_amd", "csrc"), "-s"],
                   check=True, capture_output=True)
    assert os.path.exists(FSKRX)
    return FSKRX


def _run(binary, pcm: np.ndarray, *args):
    return subprocess.run([binary, *args], input=pcm.astype("<i2").tobytes(),
                          capture_output=True, timeout=120)


def _symbols(A, frames: bytes, n: int, bits: int) -> np.ndarray:
    per = A.DEMOD_MAX_FRAME_PAYLOAD * 8 // bits
    out, got = [], 0
    for payload in A.iter_frames(frames):
        cnt = min(per, n - got)
        out.append(A.unpack_symbols(payload, cnt, bits))
        got += cnt
    return np.concatenate(out) if out else np.zeros(0, np.uint8)


def test_usage_errors(fskrx):
    assert subprocess.run([fskrx, "-x"], capture_output=True).returncode == 2
    assert subprocess.run([fskrx, "-f"], capture_output=True).returncode == 2
    assert subprocess.run([fskrx, "-M", "bogus", "-c", "1"], capture_output=True).returncode == 2


def test_no_device_fails_loudly(fskrx):
    if _gpu_visible():
        pytest.skip("a GPU is visible")
    r = _run(fskrx, np.zeros(4096, np.int16))
    assert r.returncode == 3
    assert b"no gfx950" in r.stderr
    assert r.stdout == b""


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [["-p", "2880"], ["-p", "1000"], ["-p", "100000"], ["-b"]])
@pytest.mark.parametrize("k", [2, 8])
def test_stereo_pcm_to_frames(A, O, fskrx, mode, k):
    """Left channel carries the FSK signal, right is noise; the emitted frames
    carry exactly the oracle's symbols of every complete window."""
    if not _gpu_visible():
        pytest.skip("no GPU visible")
    freqs = A.FSK8_FREQS if k == 8 else A.FSK2_FREQS
    W = 40000 if k == 2 else 3000   # 2-FSK crosses the 32768-symbol frame payload
    pcm, _ = O.synth_fsk(freqs, 1024, W, 77 + k, 8000, 400)
    mono = np.concatenate([pcm.reshape(-1), pcm.reshape(-1)[:333]])  # ragged tail
    right = np.random.default_rng(k).integers(-2000, 2000, mono.size).astype(np.int16)
    st = np.empty(2 * mono.size, np.int16)
    st[0::2], st[1::2] = mono, right
    r = _run(fskrx, st, "-c", "2", "-m", "left", "-f", ",".join(str(f) for f in freqs), *mode)
    assert r.returncode == 0, r.stderr.decode()
    bits = A.bits_per_symbol(k)
    got = _symbols(A, r.stdout, W, bits)
    ref, _ = O.goertzel(mono, freqs, 1024)
    assert got.size == W and ref.size == W
    assert np.array_equal(got, ref)
    assert b"333 samples pending" in r.stderr
