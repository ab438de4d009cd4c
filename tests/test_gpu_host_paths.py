"""The three ways host-pointer calls reach the kernels (demod_api.cpp
run_host): packet-sized calls (<= 16 Ki samples) through mapped coherent
pinned memory with no copies, small calls (<= 2 Mi samples) through one pinned
round trip, and larger ones chunked and double-buffered from pageable memory.
Every path must return exactly what the device-pointer call returns on the
same samples (symbols and magnitude bits), for every detector and at hop < n,
including the sizes either side of each boundary.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ZERO_COPY_SAMPLES = 1 << 14
SMALL_SAMPLES = 1 << 21
K8_ODD = tuple(46.875 * (32 + 9 * i) for i in range(8))   # residue detector


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def windows_for(samples, n, hop):
    return (samples - n) // hop + 1


def host_vs_device(A, torch, freqs, method, hop, samples, seed):
    n = 1024
    rng = np.random.default_rng(seed)
    flat = rng.integers(-12000, 12000, size=samples).astype(np.int16)
    W = windows_for(samples, n, hop)
    with A.Demodulator(freqs=freqs, hop=hop, method=method) as d:
        sym, mag = d.batch(flat, n_windows=W, mags=True)
        d_pcm = torch.from_numpy(flat).cuda()
        d_sym = torch.empty(W, dtype=torch.uint8, device="cuda")
        d_mag = torch.empty((W, len(freqs)), dtype=torch.float32, device="cuda")
        d.batch_device(d_pcm, W, d_sym, d_mag)
        torch.cuda.synchronize()
        assert np.array_equal(sym, d_sym.cpu().numpy())
        assert np.array_equal(mag.view(np.uint32), d_mag.cpu().numpy().view(np.uint32))
    return W


@pytest.mark.parametrize("samples", [1024, 3903, ZERO_COPY_SAMPLES - 1, ZERO_COPY_SAMPLES,
                                     ZERO_COPY_SAMPLES + 1, SMALL_SAMPLES, SMALL_SAMPLES + 1024])
@pytest.mark.parametrize("method,plan", [(1, "FSK2_FREQS"), (3, "FSK8_FREQS"), (4, "K8_ODD"),
                                         (2, "FSK8_FREQS")])   # plain, fold, residue, FFT
def test_host_paths_equal_device(A, torch, method, plan, samples):
    freqs = getattr(A, plan) if hasattr(A, plan) else globals()[plan]
    assert host_vs_device(A, torch, freqs, method, 1024, samples, seed=samples + method) >= 1


@pytest.mark.parametrize("hop", [256, 200, 64])
@pytest.mark.parametrize("samples", [3903, ZERO_COPY_SAMPLES, ZERO_COPY_SAMPLES + 8])
def test_host_paths_overlapping(A, torch, hop, samples):
    """hop < n: the zero-copy kernels read each sample several times over
    PCIe (segment-shared and direct kernels alike)."""
    for freqs in (A.FSK2_FREQS, A.FSK8_FREQS):
        host_vs_device(A, torch, freqs, 0, hop, samples, seed=hop + samples)


def test_packets_back_to_back_reuse_buffers(A, O, torch):
    """Consecutive packet calls reuse the same mapped buffers: every call's
    result must be its own (no stale samples or results from the call
    before), against the oracle's stream."""
    n = 1024
    pcm, _ = O.synth_fsk(A.FSK8_FREQS, n, 60, 11, 8000, 400)
    flat = pcm.reshape(-1)
    ref = O.Stream(A.FSK8_FREQS, n=n)
    with A.Demodulator(freqs=A.FSK8_FREQS) as d:
        pos, got, want = 0, [], []
        rng = np.random.default_rng(2)
        while pos < flat.size:
            step = int(rng.choice([1, 500, 1024, 2880, 4096, 9000]))
            chunk = flat[pos:pos + step]
            pos += step
            got.append(d.demodulate(chunk))
            want.append(ref.push(chunk)[0])
    assert np.array_equal(np.concatenate(got), np.concatenate(want))
