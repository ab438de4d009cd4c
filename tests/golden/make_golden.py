#!/usr/bin/env python3
"""Regenerate the committed golden fixtures in tests/golden/.

    python tests/golden/make_golden.py      (from the repo root, this container)

Demodulation vectors: inputs from the seeded generator, expected symbols and
P_k from the double-precision oracle (oracle/fsk_oracle.c) — which is itself
pinned to the reference's own FFT (opus_fft_c, tests/golden/ref_kissfft.npz)
and to numpy.fft / direct-DFT known answers (tests/test_oracle.py); the
reference has no demodulator, so these are oracle outputs, not reference
outputs.

Frame vectors: ToReceiver frames encoded and decode verdicts given by the
reference's OWN nanopb 0.4.5 + generated ip.pb.c, compiled in place from
/root/reference by oracle/ref.mk (oracle/_ref/libnanopb_ref.so).

Everything is stored as .npz (plain arrays, loadable with allow_pickle=False)
or JSON.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

SEED = 0x2C5DA044
FSK2 = (1500.0, 3000.0)
FSK8 = tuple(1500.0 + 375.0 * i for i in range(8))


def demod_case(name, freqs, n, W, seed, amplitude=8000, sigma=400, hop=None):
    pcm, truth = O.synth_fsk(freqs, n, W, seed, amplitude, sigma)
    flat = pcm.reshape(-1)
    hop = n if hop is None else hop
    sym, P = O.goertzel(flat, freqs, n, hop)
    np.savez(os.path.join(HERE, name + ".npz"), pcm=flat, n=np.int64(n), hop=np.int64(hop),
             freqs=np.array(freqs, np.float64), fs=np.float64(48000.0), seed=np.uint64(seed),
             amplitude=np.int64(amplitude), sigma=np.int64(sigma), truth=truth, sym=sym, P=P)
    print(name, flat.size, "samples", sym.size, "windows")


def stream_case():
    n = 1024
    L, _ = O.synth_fsk(FSK2, n, 12, 21)
    R, _ = O.synth_fsk(FSK2, n, 12, 22)
    inter = np.stack([L.reshape(-1), R.reshape(-1)], axis=1).reshape(-1)
    # 60 ms Opus packets as decoded at playback.cpp:118 (2880 stereo frames)
    out = {}
    for mode in (0, 1, 2):
        st = O.Stream(FSK2, n=n, channels=2, channel_mode=mode)
        syms, Ps = [], []
        for i in range(0, inter.size // 2, 2880):
            s, P = st.push(inter[2 * i:2 * (i + 2880)])
            syms.append(s)
            Ps.append(P)
        out[f"sym_mode{mode}"] = np.concatenate(syms)
        out[f"P_mode{mode}"] = np.concatenate(Ps)
        out[f"pending_mode{mode}"] = np.int64(st.pending())
    np.savez(os.path.join(HERE, "stereo_stream.npz"), pcm=inter, n=np.int64(n),
             freqs=np.array(FSK2), packet_frames=np.int64(2880), **out)
    print("stereo_stream", inter.size, "samples")


def vi(n):
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def tag(num, wire):
    return vi((num << 3) | wire)


def ld(num, data):
    return tag(num, 2) + vi(len(data)) + data


def delim(msg):
    return vi(len(msg)) + msg


def crafted_frames():
    """Malformed / unusual ToReceiver frames (delimited), built by hand."""
    audio = lambda *fields: ld(1, b"".join(fields))  # ToReceiver.audio_data
    pl = lambda b: ld(1, b)                           # AudioData.opus_encoded_frame
    c = {
        "ok_small": delim(audio(pl(b"\x01\x02"))),
        "empty_payload": delim(audio(pl(b""))),
        "empty_message": delim(b""),
        "audio_data_empty": delim(audio()),
        "audio_data_unknown_only": delim(audio(tag(2, 0) + vi(5))),
        "unknown_varint_then_audio": delim(tag(3, 0) + vi(1) + audio(pl(b"\x01\x02"))),
        "unknown_ld_then_audio": delim(ld(5, b"abc") + audio(pl(b"\x09"))),
        "unknown_fixed64_fixed32": delim(tag(6, 1) + bytes(8) + tag(7, 5) + bytes(4) + audio(pl(b"\x07"))),
        "unknown_group_field": delim(tag(2, 3) + audio(pl(b"\x01"))),
        "unknown_wire6": delim(tag(2, 6) + audio(pl(b"\x01"))),
        "unknown_varint_11_bytes": delim(tag(4, 0) + b"\x80" * 10 + b"\x01" + audio(pl(b"\x05"))),
        "trailing_unknown_varint": delim(audio(pl(b"\x01\x02")) + tag(3, 0) + vi(1)),
        "unknown_inside_audio": delim(audio(tag(9, 0) + vi(300) + pl(b"\xaa") + ld(8, b"zz"))),
        "bytes_as_varint": delim(audio(tag(1, 0) + vi(0))),
        "bytes_as_varint_multibyte": delim(audio(tag(1, 0) + vi(150))),
        "bytes_as_varint_10_bytes": delim(audio(tag(1, 0) + b"\xff" * 9 + b"\x01")),
        "bytes_as_varint_11_bytes": delim(audio(tag(1, 0) + b"\xff" * 10 + b"\x01")),
        "bytes_as_fixed32": delim(audio(tag(1, 5) + b"\x01\x02\x03\x04")),
        "bytes_as_fixed64": delim(audio(tag(1, 1) + bytes(range(8)))),
        "bytes_as_group": delim(audio(tag(1, 3))),
        "audio_as_varint": delim(tag(1, 0) + vi(3)),
        "audio_as_fixed32": delim(tag(1, 5) + bytes(4)),
        "zero_tag_in_message": delim(b"\x00" + audio(pl(b"\x01"))),
        "zero_tag_after_audio": delim(audio(pl(b"\x01")) + b"\x00\x00"),
        "zero_tag_in_audio": delim(audio(pl(b"\x01") + b"\x00")),
        "field0_wire2_tag": delim(b"\x02\x00" + audio(pl(b"\x01"))),
        "tag_overlong_5_bytes": delim(b"\x8a\x80\x80\x80\x00" + vi(4) + pl(b"\x01\x02")),
        "tag_overlong_6_bytes": delim(b"\x8a\x80\x80\x80\x80\x00" + vi(4) + pl(b"\x01\x02")),
        "tag_5th_byte_high_bits": delim(b"\x8a\x80\x80\x80\x10" + vi(4) + pl(b"\x01\x02")),
        "tag_sign_extended": delim(b"\x8a\x80\x80\x80\x8f\xff\xff\xff\xff\x01" + audio(pl(b"\x01"))),
        "tag_too_long_11_bytes": delim(b"\x8a" + b"\x80" * 9 + b"\x00" + audio(pl(b"\x01"))),
        "prefix_overlong": b"\x84\x80\x00" + audio(pl(b"\x01\x02"))[:0] + audio(pl(b"\x01\x02")),
        "payload_len_noncanonical": delim(ld(1, tag(1, 2) + b"\x82\x00" + b"\x0c\x0d")),
        "two_audio_data_merge": delim(audio(pl(b"\x01\x02")) + audio(pl(b"\x03\x04"))),
        "second_audio_data_empty": delim(audio(pl(b"\x01\x02")) + audio()),
        "bytes_twice_in_one_audio": delim(audio(pl(b"\xaa") + pl(b"\xbb\xcc"))),
        "truncated_payload": bytes.fromhex("140a120a10") + b"\xab" * 8,
        "length_overrun_inner": delim(ld(1, tag(1, 2) + vi(5) + b"\xff")),
        "audio_len_overrun": delim(tag(1, 2) + vi(9) + pl(b"\x01")),
        "payload_4096": delim(audio(pl(bytes(4096)))),
        "payload_4097": delim(audio(pl(bytes(4097)))),
        "trailing_next_frame": delim(audio(pl(b"\x01"))) + delim(audio(pl(b"\x02"))),
    }
    return c


def frame_cases():
    R = O.ref_nanopb()
    if R is None:
        raise SystemExit("oracle/_ref/libnanopb_ref.so missing: make -f oracle/ref.mk")
    frames = []
    for size in (0, 1, 2, 16, 127, 128, 129, 300, 1000, 4095, 4096):
        payload = bytes((i * 37 + 11) & 0xFF for i in range(size))
        enc = O.ref_encode(payload)
        rc, dec, used = O.ref_decode(enc)
        assert rc == 0 and dec == payload and used == len(enc)
        frames.append({"payload_len": size, "frame_hex": enc.hex()})
    # decode verdicts of the reference nanopb on crafted inputs
    verdicts = []
    for name, buf in crafted_frames().items():
        rc, dec, used = O.ref_decode(buf)
        verdicts.append({"name": name, "frame_hex": buf.hex(), "nanopb_rc": rc,
                         "payload_hex": dec.hex() if rc == 0 else None,
                         "consumed": used if rc == 0 else None})
    json.dump({"source": "reference nanopb 0.4.5 + hardware/src/protogen/ip.pb.c via oracle/ref.mk",
               "payload_rule": "byte i = (i*37 + 11) & 0xFF",
               "frames": frames, "decode_verdicts": verdicts},
              open(os.path.join(HERE, "frames_golden.json"), "w"), indent=1)
    print("frames_golden.json", len(frames), "frames", len(verdicts), "verdicts")


if __name__ == "__main__":
    demod_case("fsk2_n1024", FSK2, 1024, 64, SEED)
    demod_case("fsk8_n1024", FSK8, 1024, 64, SEED + 1)
    demod_case("k5_nonint_n512", (612.3, 2471.9, 5003.3, 9100.0, 15777.7), 512, 48, 7, sigma=2000)
    demod_case("fsk2_hop256", FSK2, 1024, 16, 9, hop=256)
    demod_case("fsk4_n256_lowsnr", (1500.0, 3000.0, 4500.0, 6000.0), 256, 96, 13,
               amplitude=600, sigma=400)
    stream_case()
    frame_cases()
