"""Re-entrancy across handles (include/demod.h, DESIGN.md §1: "re-entrant
across handles, not within one handle"): several host threads, each with its
own handle, detector and plan, run batch and streaming calls at the same time
(ctypes releases the GIL around every foreign call, so the library really runs
concurrently); every thread's results must equal the oracle's."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def test_concurrent_handles(A, O, torch):
    odd8 = tuple(46.875 * (32 + 9 * i) for i in range(8))
    jobs = [
        dict(freqs=A.FSK2_FREQS, method=A.METHOD_GOERTZEL, hop=1024, channels=1),
        dict(freqs=A.FSK8_FREQS, method=A.METHOD_FOLDED, hop=512, channels=1),
        dict(freqs=odd8, method=A.METHOD_RESIDUE, hop=1024, channels=2),
        dict(freqs=A.FSK2_FREQS, method=A.METHOD_FFT, hop=256, channels=1),
        dict(freqs=(300.0, 1234.5, 5000.0), method=A.METHOD_GOERTZEL, hop=1024, channels=2),
        dict(freqs=A.FSK8_FREQS, method=A.METHOD_AUTO, hop=1024, channels=1),
    ]
    W, n = 400, 1024
    inputs, expect = [], []
    for i, j in enumerate(jobs):
        L, _ = O.synth_fsk(j["freqs"], n, W, 900 + i, 8000, 400)
        x = L.reshape(-1)
        if j["channels"] == 2:
            R, _ = O.synth_fsk(j["freqs"], n, W, 950 + i, 8000, 400)
            stream = np.stack([x, R.reshape(-1)], axis=1).reshape(-1)
        else:
            stream = x
        Wh = (x.size - n) // j["hop"] + 1
        demod = O.fft_demod if j["method"] == A.METHOD_FFT else O.goertzel
        ref_sym, _ = demod(x, j["freqs"], n, j["hop"]) if j["method"] == A.METHOD_FFT \
            else demod(x, j["freqs"], n, j["hop"], Wh)
        inputs.append((x, stream, Wh))
        expect.append(ref_sym)

    errors = []

    def worker(i):
        try:
            j = jobs[i]
            x, stream, Wh = inputs[i]
            with A.Demodulator(freqs=j["freqs"], method=j["method"], hop=j["hop"],
                               channels=j["channels"]) as d:
                for rep in range(6):
                    sym = d.batch(x, n_windows=Wh)
                    if not (sym == expect[i]).all():
                        errors.append((i, rep, "batch", int((sym != expect[i]).sum())))
                    d.reset()
                    got, pos, ch = [], 0, j["channels"]
                    sizes = [2880, 1, 4999, 1024, 7]
                    k = 0
                    while pos < stream.size // ch:
                        fr = sizes[k % len(sizes)]
                        k += 1
                        got.append(d.demodulate(stream[pos * ch:(pos + fr) * ch]))
                        pos += fr
                    s = np.concatenate(got)
                    if not (s.size == expect[i].size and (s == expect[i]).all()):
                        errors.append((i, rep, "stream", s.size))
        except Exception as e:  # surfaced below
            errors.append((i, "exception", repr(e)))

    # the handle-less entry points too: demod_synth_fsk (module sine table,
    # filled once per device under a lock) and demod_read_ceiling_async, from
    # several threads at once, each into its own buffers
    synth_ref = O.synth_fsk(A.FSK8_FREQS, n, 300, 4242, 8000, 400)

    def synth_worker(i):
        try:
            cfg = A.make_cfg(freqs=A.FSK8_FREQS)
            for rep in range(6):
                d_pcm = torch.empty((300, n), dtype=torch.int16, device="cuda")
                d_sym = torch.empty(300, dtype=torch.uint8, device="cuda")
                s = torch.cuda.Stream()
                A.synth_fsk(cfg, 4242, 300, 8000, 400, d_pcm, d_sym, stream=s.cuda_stream)
                A.read_ceiling_async(d_pcm, 300 * n * 2 // 8192 * 8192, stream=s.cuda_stream)
                s.synchronize()
                if not (np.array_equal(d_pcm.cpu().numpy(), synth_ref[0])
                        and np.array_equal(d_sym.cpu().numpy(), synth_ref[1])):
                    errors.append((i, rep, "synth"))
        except Exception as e:
            errors.append((i, "synth exception", repr(e)))

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(len(jobs))]
    threads += [threading.Thread(target=synth_worker, args=(100 + i,)) for i in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in threads)
    assert not errors, errors[:5]
