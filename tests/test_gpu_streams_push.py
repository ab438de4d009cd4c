"""Many streams behind one detector (demod_streams_push, include/demod.h):
each stream must behave exactly like its own demod_t from the same cfg fed
the same packets — same symbols, same magnitudes (bits: every window is
evaluated alone in both cases), same pending count — and match the oracle's
streaming restatement (oracle.Stream), while all streams' windows go through
one batch per push.
"""
import numpy as np
import pytest

from decision import check_decisions

pytestmark = pytest.mark.gpu

MAG_TOL = 1e-5


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU visible")
    return t


def streams_vs_single(A, O, n_streams, freqs, hop, channels=1, mode=0, lead_in=0, method=0,
                      rounds=12, seed=0, max_frames=4000, mapped=False):
    n = 1024
    rng = np.random.default_rng(seed)
    # each stream its own seeded signal, long enough for the rounds
    per = rounds * max_frames // n + 2
    sig = []
    for s in range(n_streams):
        L, _ = O.synth_fsk(freqs, n, per, 1000 * seed + s, 8000, 400)
        if channels == 2:
            R, _ = O.synth_fsk(freqs, n, per, 1000 * seed + s + 500, 8000, 400)
            sig.append(np.stack([L.reshape(-1), R.reshape(-1)], axis=1).reshape(-1))
        else:
            sig.append(L.reshape(-1))
    pos = [0] * n_streams
    kw = dict(freqs=freqs, hop=hop, channels=channels, channel_mode=mode, lead_in=lead_in,
              method=method)
    singles = [A.Demodulator(**kw) for _ in range(n_streams)]
    refs = [O.Stream(freqs, n=n, hop=hop, channels=channels, channel_mode=mode, lead_in=lead_in)
            for _ in range(n_streams)]
    total = 0
    import os
    if mapped:  # measurement switch: stage into mapped memory the detector reads in place
        os.environ["FSKD_STREAMS_MAPPED"] = "1"
    try:
        ms_h = A.Streams(n_streams, **kw)
    finally:
        os.environ.pop("FSKD_STREAMS_MAPPED", None)
    with ms_h as ms:
        for r in range(rounds):
            pkts = []
            for s in range(n_streams):
                f = int(rng.choice([0, 1, 7, 2880, int(rng.integers(1, max_frames))]))
                if rng.random() < 0.15:
                    pkts.append(None)
                    continue
                a = sig[s][pos[s] * channels:(pos[s] + f) * channels]
                pos[s] += f
                pkts.append(a)
            got_s, got_m = ms.push(pkts, mags=True)
            for s in range(n_streams):
                a = pkts[s] if pkts[s] is not None else np.zeros(0, np.int16)
                one_s, one_m = singles[s].demodulate(a, mags=True)
                ref_s, ref_P = refs[s].push(a)
                assert np.array_equal(got_s[s], one_s), (r, s)
                assert np.array_equal(got_m[s].view(np.uint32), one_m.view(np.uint32)), (r, s)
                assert got_s[s].size == ref_s.size, (r, s)
                if ref_s.size:
                    err = (np.abs(got_m[s].astype(np.float64) - ref_P).max(axis=1) /
                           np.maximum(ref_P.max(axis=1), 1e-30)).max()
                    if hop == n:
                        assert err <= MAG_TOL, (r, s, err)
                        check_decisions(got_s[s], got_m[s], ref_s, ref_P)
                    else:
                        # straddling windows too: the decision rescue makes every
                        # symbol the oracle's
                        assert np.array_equal(got_s[s], ref_s), (r, s)
                assert ms.pending(s) == singles[s].pending() == refs[s].pending(), (r, s)
                total += got_s[s].size
    for d in singles:
        d.close()
    assert total > 0


@pytest.mark.parametrize("n_streams", [1, 3, 64])
def test_mono_hop_n(A, O, torch, n_streams):
    streams_vs_single(A, O, n_streams, A.FSK2_FREQS, 1024, seed=n_streams)


@pytest.mark.parametrize("hop", [256, 512, 1000, 64])
def test_overlapping_windows(A, O, torch, hop):
    """hop < n: each window's n samples are copied into the batch; the
    per-stream handles run the segment-shared kernels (bit-identical)."""
    streams_vs_single(A, O, 9, A.FSK8_FREQS, hop, seed=hop)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_stereo_and_lead_in(A, O, torch, mode):
    streams_vs_single(A, O, 7, A.FSK8_FREQS, 1024, channels=2, mode=mode,
                      lead_in=A.DEMOD_OPUS_LOOKAHEAD, seed=10 + mode)


@pytest.mark.parametrize("method", [2, 4, 1])
def test_other_detectors(A, O, torch, method):
    f = A.FSK2_FREQS if method != 4 else tuple(46.875 * (32 + 9 * i) for i in range(8))
    streams_vs_single(A, O, 5, f, 1024, method=method, seed=20 + method, rounds=6)


def test_reset_buffer_too_small_and_errors(A, O, torch):
    """reset drops one stream's carry and re-arms its lead-in; a cap below
    the push's window count consumes nothing."""
    n = 1024
    pcm, _ = O.synth_fsk(A.FSK2_FREQS, n, 8, 5, 8000, 400)
    flat = pcm.reshape(-1)
    with A.Streams(2, freqs=A.FSK2_FREQS, lead_in=100) as ms:
        with pytest.raises(A.DemodError) as e:
            ms.push([flat[:3000], flat[:3000]], cap=3)
        assert e.value.code == A.DEMOD_BUFFER_TOO_SMALL
        assert ms.pending(0) == 0 and ms.pending(1) == 0
        out = ms.push([flat[:3000], flat[:500]])
        assert [o.size for o in out] == [2, 0]
        assert ms.pending(0) == 3000 - 100 - 2048 and ms.pending(1) == 400
        ms.reset(1)
        assert ms.pending(1) == 0
        out = ms.push([None, flat[:1124]])
        assert [o.size for o in out] == [0, 1]      # lead-in of 100 re-armed
        with pytest.raises(A.DemodError):
            ms.push([flat[:10]])                     # one packet per stream
        with pytest.raises(A.DemodError):
            ms.reset(2)
    with pytest.raises(A.DemodError):
        A.Streams(0, freqs=A.FSK2_FREQS)


def test_many_streams_one_push(A, O, torch):
    """1024 streams x one 60 ms packet (2880 frames) per push, as a receiver
    of config 5's streams would call it: symbols equal the oracle's stream of
    every stream."""
    n, S = 1024, 1024
    pcm, _ = O.synth_fsk(A.FSK2_FREQS, n, 3 * S, 77, 8000, 400)
    flat = pcm.reshape(S, -1)
    refs = [O.Stream(A.FSK2_FREQS, n=n) for _ in range(S)]
    with A.Streams(S, freqs=A.FSK2_FREQS) as ms:
        for r in range(2):
            pk = [flat[s, r * 1440:(r + 1) * 1440] for s in range(S)]
            got = ms.push(pk)
            for s in range(S):
                assert np.array_equal(got[s], refs[s].push(pk[s])[0]), (r, s)


@pytest.mark.parametrize("channels", [1, 2])
def test_rows_of_one_array(A, O, torch, channels):
    """A 2-D array of packets (rows = streams, here column slices of a longer
    recording, so rows are not adjacent in memory) gives the same symbols and
    magnitudes as the same packets passed as a list."""
    S, F, n = 33, 2880, 1024
    pcm, _ = O.synth_fsk(A.FSK8_FREQS, n, 9 * S * channels, 3, 8000, 400)
    rec = pcm.reshape(S, -1)                       # each row one stream's recording (>= 3 F frames)
    kw = dict(freqs=A.FSK8_FREQS, channels=channels)
    with A.Streams(S, **kw) as a, A.Streams(S, **kw) as b:
        for r in range(3):
            block = rec[:, r * F * channels:(r + 1) * F * channels]
            assert not block.flags.c_contiguous
            s1, m1 = a.push(block, mags=True)
            s2, m2 = b.push([np.array(x) for x in block], mags=True)
            for s in range(S):
                assert np.array_equal(s1[s], s2[s])
                assert np.array_equal(m1[s].view(np.uint32), m2[s].view(np.uint32))
                assert a.pending(s) == b.pending(s)
        with pytest.raises(A.DemodError):
            a.push(rec[:S - 1, :F * channels])
        if channels == 2:
            with pytest.raises(A.DemodError):
                a.push(rec[:, :3])


@pytest.mark.parametrize("hop,channels", [(1024, 1), (1024, 2), (256, 1)])
def test_threaded_staging(A, O, torch, hop, channels):
    """Pushes big enough to stage on several host threads (>= 4 MiB of run
    samples: 1024 streams x ~4000 frames), ragged and empty packets so the
    thread ranges hold streams with and without windows: every stream's
    symbols equal the oracle's stream, and a sample of 24 streams equals its
    own single handle bit for bit (symbols, magnitudes, carry). At hop < n
    the oracle bar is agreement on >= 99.9 % of the windows."""
    n, S, R = 1024, 1024, 3
    rng = np.random.default_rng(hop + channels)
    pcm, _ = O.synth_fsk(A.FSK8_FREQS, n, 16 * S * channels, 40 + hop, 8000, 400)
    rec = pcm.reshape(S, -1)                      # 16 * channels windows per stream
    kw = dict(freqs=A.FSK8_FREQS, hop=hop, channels=channels)
    probe = sorted(rng.choice(S, 24, replace=False).tolist())
    singles = {s: A.Demodulator(**kw) for s in probe}
    refs = [O.Stream(A.FSK8_FREQS, n=n, hop=hop, channels=channels) for _ in range(S)]
    pos = np.zeros(S, dtype=np.int64)
    staged = 0
    try:
        with A.Streams(S, **kw) as ms:
            for r in range(R):
                pk = []
                for s in range(S):
                    f = 0 if rng.random() < 0.05 else int(rng.integers(2000, 6000))
                    pk.append(rec[s, pos[s] * channels:(pos[s] + f) * channels])
                    pos[s] += f
                staged += sum(p.size // channels for p in pk)
                got_s, got_m = ms.push(pk, mags=True)
                same = total = 0
                for s in range(S):
                    ref_s, _ = refs[s].push(pk[s])
                    assert got_s[s].size == ref_s.size, (r, s)
                    if hop == n:
                        assert np.array_equal(got_s[s], ref_s), (r, s)
                    same += int((got_s[s] == ref_s).sum())
                    total += ref_s.size
                    assert ms.pending(s) == refs[s].pending(), (r, s)
                # windows straddling a symbol boundary can be near-ties (§4.8)
                assert same >= 0.999 * total, (r, same, total)
                for s in probe:
                    one_s, one_m = singles[s].demodulate(pk[s], mags=True)
                    assert np.array_equal(got_s[s], one_s), (r, s)
                    assert np.array_equal(got_m[s].view(np.uint32), one_m.view(np.uint32)), (r, s)
                    assert ms.pending(s) == singles[s].pending(), (r, s)
    finally:
        for d in singles.values():
            d.close()
    assert staged / R > 2 * (1 << 20)            # several threads per push (one per 2 MiB)


@pytest.mark.parametrize("channels,hop,n_streams", [(1, 1024, 300), (2, 1024, 64), (1, 256, 200),
                                                   (1, 1000, 50)])
def test_mapped_staging_variant(A, O, torch, channels, hop, n_streams):
    """FSKD_STREAMS_MAPPED=1 (the push stages into mapped pinned memory that
    the detector reads in place): the same per-stream
    results as per-stream handles, bit for bit."""
    streams_vs_single(A, O, n_streams, A.FSK2_FREQS, hop, channels=channels, rounds=6,
                      seed=91 + hop + channels, mapped=True)


def test_group_push_and_bucket_world1(A):
    """demod_group (the C ABI's RCCL group) at world 1 on
    the box: pushes equal demod_streams_push symbol for symbol (stereo,
    lead-in, ragged packets), both as one rank of a multi-process group and
    as a one-device local group; the device bucket's gathered frames equal
    demod_frame_streams_async of the same symbols byte for byte."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    S = 7
    cfg = A.make_cfg(channels=2, channel_mode=A.CH_DOWNMIX, lead_in=312)
    rng = np.random.default_rng(5)
    ms = A.Streams(S, cfg)
    with A.Group(cfg, S) as g, A.Group(cfg, S, devices=[0]) as gl:
        assert g.world == 1 and gl.world == 1 and g.shard(0) == (0, 0, S)
        for rnd in range(5):
            packets = [rng.integers(-20000, 20000, 2 * (2880 - 131 * s - 17 * rnd)).astype(np.int16)
                       for s in range(S)]
            per = ms.push(packets)
            sa = np.concatenate(per)
            ca = np.array([len(p) for p in per], np.uint32)
            sb, cb = g.push(packets)
            sc, cc = gl.push(packets)
            assert np.array_equal(ca, cb) and np.array_equal(ca, cc)
            assert np.array_equal(sa, sb) and np.array_equal(sa, sc)
    ms.close()
    # the bucket: 16 steps, ring 4, 3 streams x 64 windows, vs the torch path's framing
    cfg1 = A.make_cfg()
    S, wps, steps, ring = 3, 64, 16, 4
    dev = torch.device("cuda", 0)
    d_pcm = torch.empty((S * wps, 1024), dtype=torch.int16, device=dev)
    tru = torch.empty(S * wps, dtype=torch.uint8, device=dev)
    A.synth_fsk(cfg1, A.BENCH_SEED, S * wps, 8000, 400, d_pcm, tru)
    ringbuf = torch.stack([d_pcm] * ring).contiguous()
    bits = A.bits_per_symbol(2)
    with A.Group(cfg1, S) as g:
        block = A.group_block_bytes(S, 1, steps, wps, bits)
        d_all = torch.zeros(block, dtype=torch.uint8, device=dev)
        got = g.bucket_async([ringbuf], ring, wps, steps, [d_all],
                             [torch.cuda.current_stream().cuda_stream])
        torch.cuda.synchronize()
        assert got == block
    with A.Demodulator(cfg1) as d:
        sym = torch.empty(S * wps, dtype=torch.uint8, device=dev)
        d.batch_async(d_pcm, S * wps, sym, None)
        stride = A.frame_symbols_size(wps, bits)
        fr = torch.empty(S * stride, dtype=torch.uint8, device=dev)
        A.frame_streams_async(sym, S, wps, bits, fr)
        torch.cuda.synchronize()
    one = fr.cpu().numpy()
    allf = d_all.cpu().numpy()
    for s in range(steps):
        assert np.array_equal(allf[s * S * stride:(s + 1) * S * stride], one), s
    assert (sym == tru).all()


def _group_with_env(A, monkeypatch, value, cfg, S, **kw):
    monkeypatch.setenv("FSKD_GROUP_FAIL", value)   # read by demod_group_create*
    try:
        return A.Group(cfg, S, **kw)
    finally:
        monkeypatch.delenv("FSKD_GROUP_FAIL")


@pytest.mark.parametrize("local", [False, True])
def test_group_injected_failures_world1(A, monkeypatch, local):
    """Injected failures (FSKD_GROUP_FAIL) through the real
    RCCL group at world 1, both group kinds: a refusal before the push
    returns its code and leaves the group alive with nothing consumed; a
    failed push returns its code, kills the group (demod_group_status), and
    every later call is refused with DEMOD_INVALID_STATE; a bucket whose rank
    fails still posts its gathers and demod_group_wait returns the code."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    kw = {"devices": [0]} if local else {}
    cfg = A.make_cfg()
    S = 3
    rng = np.random.default_rng(11)
    packets = [rng.integers(-20000, 20000, 2880 + 100 * s).astype(np.int16) for s in range(S)]
    ms = A.Streams(S, cfg)
    ref = [ms.push(packets) for _ in range(2)]
    ms.close()
    # refusal before the push: nothing consumed, the group stays usable
    g = _group_with_env(A, monkeypatch, "check:0", cfg, S, **kw)
    with pytest.raises(A.DemodError) as e:
        g.push(packets)
    assert e.value.code == A.DEMOD_INTERNAL_ERROR and g.status() == A.DEMOD_OK
    g.close()
    g = A.Group(cfg, S, **kw)
    assert g.device(0) == 0 and g.status() == A.DEMOD_OK
    for want in ref:   # the same symbols as demod_streams_push, push after push
        sym, cnt = g.push(packets)
        assert np.array_equal(sym, np.concatenate(want))
    g.close()
    # a failed push kills the group
    g = _group_with_env(A, monkeypatch, "push:0", cfg, S, **kw)
    with pytest.raises(A.DemodError) as e:
        g.push(packets)
    assert e.value.code == A.DEMOD_DEVICE_ERROR and g.status() == A.DEMOD_DEVICE_ERROR
    with pytest.raises(A.DemodError) as e:
        g.push(packets)
    assert e.value.code == A.DEMOD_INVALID_STATE
    dev = torch.device("cuda", 0)
    d_pcm = torch.zeros((S * 4, 1024), dtype=torch.int16, device=dev)
    block = A.group_block_bytes(S, 1, 2, 4, A.bits_per_symbol(2))
    d_all = torch.zeros(block, dtype=torch.uint8, device=dev)
    with pytest.raises(A.DemodError) as e:
        g.bucket_async([d_pcm], 1, 4, 2, [d_all])
    assert e.value.code == A.DEMOD_INVALID_STATE
    g.close()
    # a failing rank's bucket: its code returned, its gathers still posted,
    # demod_group_wait reports it; the group stays alive
    g = _group_with_env(A, monkeypatch, "bucket:0", cfg, S, **kw)
    with pytest.raises(A.DemodError) as e:
        g.bucket_async([d_pcm], 1, 4, 2, [d_all])
    assert e.value.code == A.DEMOD_INTERNAL_ERROR
    with pytest.raises(A.DemodError) as e:
        g.wait()
    assert e.value.code == A.DEMOD_INTERNAL_ERROR and g.status() == A.DEMOD_OK
    g.close()
    # a NULL gather target on a rank: refused, posted into the group's sink
    with A.Group(cfg, S, **kw) as g:
        assert g.bucket_async([d_pcm], 1, 4, 2, [d_all]) == block
        g.wait()
        with pytest.raises(A.DemodError) as e:
            g.bucket_async([d_pcm], 1, 4, 2, [None])
        assert e.value.code == A.DEMOD_BAD_ARG
        with pytest.raises(A.DemodError) as e:
            g.wait()
        assert e.value.code == A.DEMOD_BAD_ARG
        assert g.bucket_async([d_pcm], 1, 4, 2, [d_all]) == block   # alive: the next bucket is fine
        g.wait()


def _passthrough(A, channels, fail_on=None, calls=None):
    """A PCM pass-through demod_decode_fn (opus_decode's signature): the
    packet's bytes are interleaved int16 frames."""
    import ctypes

    def dec(state, data, ln, pcm, frame_size, fec):
        if calls is not None:
            calls.append(int(state or 0))
        if fail_on is not None and int(state or 0) == fail_on:
            return A.DEMOD_INVALID_PACKET
        frames = ln // (2 * channels)
        if frames > frame_size:
            return A.DEMOD_BUFFER_TOO_SMALL
        ctypes.memmove(pcm, data, frames * 2 * channels)
        return frames
    return A.DECODE_FN(dec)


@pytest.mark.parametrize("channels", [1, 2])
def test_push_packets_passthrough_equals_push(A, torch, channels):
    """demod_streams_push_packets with a PCM pass-through
    decoder (opus_decode's signature) equals demod_streams_push byte for byte
    over rounds of ragged packets with lead-in, empty packets (no packet, as
    playback.cpp:105) and 12 streams (staging threads decode concurrently);
    a decoder error returns its code with nothing consumed."""
    import numpy as np
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    S = 12
    cfg = A.make_cfg(channels=channels, channel_mode=A.CH_DOWNMIX if channels == 2 else A.CH_LEFT,
                     lead_in=312)
    rng = np.random.default_rng(40 + channels)
    a, b = A.Streams(S, cfg), A.Streams(S, cfg)
    fn = _passthrough(A, channels)
    for rnd in range(6):
        pk = [rng.integers(-20000, 20000, channels * (2880 - 97 * s - 13 * rnd)).astype(np.int16)
              for s in range(S)]
        pk[(rnd * 5) % S] = np.zeros(0, np.int16)          # no packet for one stream
        want = a.push(pk, mags=True)
        got = A.push_packets(b, fn, [1 + s for s in range(S)], [p.tobytes() for p in pk], 2880,
                             mags=True)
        for s in range(S):
            assert np.array_equal(want[0][s], got[0][s]), (rnd, s)
            assert np.array_equal(want[1][s].view(np.uint32), got[1][s].view(np.uint32)), (rnd, s)
    pend = [b.pending(s) for s in range(S)]
    bad = _passthrough(A, channels, fail_on=1 + 7)
    pk = [rng.integers(-20000, 20000, channels * 2880).astype(np.int16).tobytes() for _ in range(S)]
    with pytest.raises(A.DemodError) as e:
        A.push_packets(b, bad, [1 + s for s in range(S)], pk, 2880)
    assert e.value.code == A.DEMOD_INVALID_PACKET
    assert [b.pending(s) for s in range(S)] == pend        # nothing consumed
    a.close()
    b.close()


def test_push_packets_argument_and_decoder_errors(A, torch):
    """demod_streams_push_packets' refusals: a negative length, a NULL
    packet with a length, frame_size outside [1, 2^20], a decoder that
    claims more frames than frame_size (DEMOD_INTERNAL_ERROR) — each with
    nothing consumed; every packet empty (no decode call) pushes nothing."""
    import ctypes
    import numpy as np
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    S = 3
    ms = A.Streams(S, A.make_cfg())
    lib = ms._lib
    calls = []
    ok = _passthrough(A, 1, calls=calls)
    decs = (ctypes.c_void_p * S)(1, 2, 3)
    counts = np.zeros(S, np.uint32)
    sym = np.zeros(64, np.uint8)
    buf = (ctypes.c_uint8 * 64)()
    pk = (ctypes.c_void_p * S)(ctypes.addressof(buf), None, ctypes.addressof(buf))

    def push(lens, frame_size=2880, fn=ok, packets=pk):
        ln = (ctypes.c_int32 * S)(*lens)
        return lib.demod_streams_push_packets(ms._h, ctypes.cast(fn, ctypes.c_void_p), decs, packets, ln,
                                              frame_size, sym.ctypes.data, None, sym.size,
                                              counts.ctypes.data)
    assert push([4, -1, 0]) == A.DEMOD_BAD_ARG
    assert push([4, 4, 0]) == A.DEMOD_BAD_ARG          # stream 1 has no packet pointer
    assert push([4, 0, 0], frame_size=0) == A.DEMOD_BAD_ARG
    assert push([4, 0, 0], frame_size=(1 << 20) + 1) == A.DEMOD_BAD_ARG
    assert calls == []                                   # refused before any decode

    def liar(state, data, ln, pcm, frame_size, fec):
        return frame_size + 1
    bad = A.DECODE_FN(liar)
    assert push([4, 0, 4], frame_size=2, fn=bad) == A.DEMOD_INTERNAL_ERROR
    assert [ms.pending(s) for s in range(S)] == [0, 0, 0]
    assert push([0, 0, 0], packets=None) == 0 and calls == [] and counts.sum() == 0
    assert push([64, 0, 64]) == 0 and sorted(calls) == [1, 3]     # 32 frames each: no window yet
    assert [ms.pending(s) for s in range(S)] == [32, 0, 32]
    ms.close()
