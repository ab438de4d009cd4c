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


@pytest.mark.gpu
def test_batch_many_payloads_and_lead_in(A, O, fskrx):
    """-b with more than 3 payloads' worth of symbols in one demodulate() call
    (hop 8: 3 x 32768 + 1000 windows from 0.8 MB of PCM): every payload is
    framed on its own; and -L drops the stream's lead-in before windowing."""
    if not _gpu_visible():
        pytest.skip("no GPU visible")
    freqs = A.FSK2_FREQS
    W = 3 * 32768 + 1000
    n_samp = (W - 1) * 8 + 1024
    pcm, _ = O.synth_fsk(freqs, 1024, n_samp // 1024 + 2, 5150, 8000, 400)
    mono = pcm.reshape(-1)[:n_samp + 312]
    r = _run(fskrx, mono, "-H", "8", "-b", "-L", "312")
    assert r.returncode == 0, r.stderr.decode()
    got = _symbols(A, r.stdout, W, 1)
    ref, _ = O.goertzel(mono[312:], freqs, 1024, 8)
    assert ref.size == W and np.array_equal(got, ref)
    assert b"4 ToReceiver frames" in r.stderr


def test_network_usage_errors(fskrx):
    # discovery, -1 or -r without a TCP listener, and a device name over 127 bytes
    assert subprocess.run([fskrx, "-u", "0"], capture_output=True).returncode == 2
    assert subprocess.run([fskrx, "-1"], capture_output=True).returncode == 2
    assert subprocess.run([fskrx, "-r"], capture_output=True).returncode == 2
    assert subprocess.run([fskrx, "-l", "0", "-N", "x" * 128], capture_output=True).returncode == 2


def _start_listener(fskrx, *args):
    import re
    p = subprocess.Popen([fskrx, "-l", "0", "-u", "0", "-a", "127.0.0.1", "-1", *args],
                         stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    line = p.stderr.readline().decode()
    m = re.search(r"listening tcp (\d+) udp (\d+)", line)
    assert m, line
    return p, int(m.group(1)), int(m.group(2))


@pytest.mark.gpu
@pytest.mark.parametrize("channels", [1, 2])
def test_network_receiver_session(A, O, fskrx, channels):
    """fskrx -l: UDP discovery answer (network.cpp:473-492), the ToTransmitter
    hello on connect (network.cpp:380-403), then AudioData frames of PCM ->
    symbol frames on stdout equal to the oracle's; a frame nanopb rejects ends
    the stream (network.cpp:411-421)."""
    import socket
    if not _gpu_visible():
        pytest.skip("no GPU visible")
    freqs = A.FSK2_FREQS
    W = 600
    pcm, _ = O.synth_fsk(freqs, 1024, W, 91 + channels, 8000, 400)
    mono = np.concatenate([pcm.reshape(-1), pcm.reshape(-1)[:100]])
    if channels == 2:
        inter = np.empty(2 * mono.size, np.int16)
        inter[0::2] = mono
        inter[1::2] = np.random.default_rng(3).integers(-900, 900, mono.size).astype(np.int16)
    else:
        inter = mono
    p, tport, uport = _start_listener(fskrx, "-r", "-c", str(channels), "-m", "left", "-N",
                                      "bench-rx")
    try:
        u = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        u.settimeout(0.5)
        u.sendto(bytes.fromhex("08c5c0f6e2021001"), ("127.0.0.1", uport))   # wrong magic
        u.sendto(A.broadcast_request_encode(), ("127.0.0.1", uport))
        which, magic, d = A.broadcast_decode(u.recvfrom(1024)[0])
        assert (which, magic) == (A.DEMOD_MSG_DISCOVERY_RESPONSE, A.DEMOD_BROADCAST_MAGIC)
        assert d["device_name"] == b"bench-rx" and d["protocol_version"] == 1
        assert d["opus_version"] == A.version_string().encode() and not d["currently_streaming"]
        with pytest.raises(socket.timeout):
            u.recvfrom(1024)                     # the wrong-magic datagram got no answer
        t = socket.create_connection(("127.0.0.1", tport), timeout=30)
        hello = b""
        while True:
            hello += t.recv(4096)
            try:
                which, info, used = A.to_transmitter_decode(hello)
                break
            except A.DemodError as e:
                assert e.code == A.DEMOD_BUFFER_TOO_SMALL
        assert which == A.DEMOD_MSG_RECEIVER_INFORMATION and used == len(hello)
        assert info["max_encoded_frame_size"] == 4096 and info["max_decoded_frame_size"] == 11520
        # while streaming, discovery reports it
        u.sendto(A.broadcast_request_encode(), ("127.0.0.1", uport))
        assert A.broadcast_decode(u.recvfrom(1024)[0])[2]["currently_streaming"]
        raw = inter.astype("<i2").tobytes()
        rng = np.random.default_rng(channels)
        off, wire = 0, b""
        fb = 2 * channels
        while off < len(raw):                    # ragged payloads of whole PCM frames
            n = fb * int(rng.integers(1, 4096 // fb + 1))
            wire += A.frame_encode(raw[off:off + n])
            off += n
        for i in range(0, len(wire), 1500):      # TCP segments that cut frames
            t.sendall(wire[i:i + 1500])
        t.sendall(bytes.fromhex("05") + b"\x0a\x03\x08\x01\x00")  # AudioData without bytes
        out, err = p.communicate(timeout=60)
        t.close()
        u.close()
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    assert p.returncode == 0, err.decode()
    assert b"bad frame" in err and b"1 transmitter(s) served" in err
    got = _symbols(A, out, W, 1)
    ref, _ = O.goertzel(mono, freqs, 1024)
    assert got.size == W and np.array_equal(got, ref)


def _hello(A, t):
    buf = b""
    while True:
        buf += t.recv(4096)
        try:
            return A.to_transmitter_decode(buf)
        except A.DemodError as e:
            assert e.code == A.DEMOD_BUFFER_TOO_SMALL


@pytest.mark.gpu
@pytest.mark.parametrize("raw,payload", [(False, 4 * 1000), (False, 693), (True, 693),
                                         (True, 6)])
def test_network_refuses_non_pcm_audio(A, fskrx, raw, payload):
    """A reference transmitter sends Opus packets in AudioData
    (MulticastAudioOutput.kt:124-130); this receiver does not decode Opus, so
    without -r any AudioData, and with -r a payload that is not whole PCM frames
    (stereo: 4 B), is refused: ToTransmitter{error{audio_decode_error}}, the
    connection closed, exit status 4 — never demodulated as noise."""
    import socket
    if not _gpu_visible():
        pytest.skip("no GPU visible")
    args = ["-c", "2"] + (["-r"] if raw else [])
    p, tport, _ = _start_listener(fskrx, *args)
    try:
        t = socket.create_connection(("127.0.0.1", tport), timeout=30)
        which, _, _ = _hello(A, t)
        assert which == A.DEMOD_MSG_RECEIVER_INFORMATION
        t.sendall(A.frame_encode(bytes(range(256)) * (payload // 256) + bytes(payload % 256)))
        reply = b""
        while True:
            chunk = t.recv(4096)
            if not chunk:
                break
            reply += chunk
        out, err = p.communicate(timeout=60)
        t.close()
    finally:
        if p.poll() is None:
            p.kill()
            p.wait()
    assert p.returncode == 4, err.decode()
    which, fields, used = A.to_transmitter_decode(reply)
    assert which == A.DEMOD_MSG_RECEIVER_ERROR and used == len(reply)
    assert fields == {"audio_underflow": False, "audio_decode_error": True}
    assert b"1 refused" in err and out == b""


@pytest.mark.gpu
def test_group_mode_matches_single_streams(fskrx, tmp_path, A, O):
    """fskrx -g 1 -S 3: three packet-interleaved streams through a one-GPU
    RCCL group (demod_group_create_local + demod_group_push); each stream's
    frames are byte-identical to fskrx run on that stream alone, and decode
    to the oracle's symbols."""
    S, per = 3, 2880
    streams = []
    for s in range(S):
        pcm, _ = O.synth_fsk(A.FSK2_FREQS, 1024, 40 + 7 * s, 77 + s)
        streams.append(pcm.reshape(-1))
    L = max(x.size for x in streams)
    rounds = -(-L // per)
    # whole rounds (zero-padded streams), so every stream sees the same packets
    full = [np.concatenate([streams[s], np.zeros(rounds * per - streams[s].size, np.int16)])
            for s in range(S)]
    inter = np.concatenate([full[s][r * per:(r + 1) * per] for r in range(rounds) for s in range(S)])
    prefix = str(tmp_path / "s")
    r = _run(fskrx, inter, "-g", "1", "-S", str(S), "-o", prefix, "-p", str(per))
    assert r.returncode == 0, r.stderr.decode()
    for s in range(S):
        alone = _run(fskrx, full[s], "-p", str(per))
        assert alone.returncode == 0
        got = open(f"{prefix}{s}.bin", "rb").read()
        assert got == alone.stdout, s
        n = full[s].size // 1024
        sym = _symbols(A, got, n, 1)
        ref, _ = O.goertzel(full[s][:n * 1024], A.FSK2_FREQS, 1024)
        assert np.array_equal(sym, ref)
