"""ip.proto framing (host C, libfskdemod.so) against the reference's nanopb.

Golden frames and decode verdicts in tests/golden/frames_golden.json were
produced by the reference's own nanopb 0.4.5 + ip.pb.c (oracle/ref.mk); when
oracle/_ref is present the same checks also run live against it. The
transmitter side (protobuf-java writeDelimitedTo, protobuf_async.kt:110-114)
is cross-checked with the official Python protobuf runtime on a descriptor
built from protocol/ip.proto's ToReceiver/AudioData definitions.
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "frames_golden.json")))


def payload_of(n):
    return bytes((i * 37 + 11) & 0xFF for i in range(n))


@pytest.mark.parametrize("case", GOLD["frames"], ids=lambda c: str(c["payload_len"]))
def test_encode_matches_reference_nanopb_golden(A, case):
    pl = payload_of(case["payload_len"])
    enc = A.frame_encode(pl)
    assert enc.hex() == case["frame_hex"]
    assert len(enc) == A.frame_size(len(pl))
    dec, used = A.frame_decode(enc)
    assert dec == pl and used == len(enc)


@pytest.mark.parametrize("v", GOLD["decode_verdicts"], ids=lambda v: v["name"])
def test_decode_verdict_matches_reference_nanopb(A, v):
    buf = bytes.fromhex(v["frame_hex"])
    try:
        dec, used = A.frame_decode(buf)
        rc = 0
    except A.DemodError as e:
        rc = e.code
    if v["nanopb_rc"] == 0:
        assert rc == 0
        assert dec.hex() == v["payload_hex"] and used == v["consumed"]
    else:
        assert rc != 0
        if v["nanopb_rc"] == -10:       # payload > MAX_ENCODED_FRAME_SIZE
            assert rc == A.DEMOD_FRAME_TOO_LARGE
        else:                            # truncated input: "read more"; else corrupt
            assert rc in (A.DEMOD_INVALID_PACKET, A.DEMOD_BUFFER_TOO_SMALL)


def test_live_reference_nanopb_roundtrip(A, O):
    if O.ref_nanopb() is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    rng = np.random.default_rng(0)
    for n in list(range(0, 300)) + [4000, 4095, 4096]:
        pl = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        enc = A.frame_encode(pl)
        assert enc == O.ref_encode(pl)
        rc, dec, used = O.ref_decode(enc)
        assert rc == 0 and dec == pl and used == len(enc)


def test_live_reference_nanopb_fuzz_verdicts(A, O):
    """Random mutations of valid frames: accept/reject and payload agree."""
    if O.ref_nanopb() is None:
        pytest.skip("oracle/_ref not built")
    rng = np.random.default_rng(1)
    base = [A.frame_encode(payload_of(n)) for n in (0, 1, 5, 130)]
    for it in range(3000):
        b = bytearray(base[it % len(base)])
        for _ in range(int(rng.integers(1, 4))):
            op = rng.integers(0, 3)
            if op == 0 and len(b):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            elif op == 1:
                b.insert(int(rng.integers(0, len(b) + 1)), int(rng.integers(0, 256)))
            elif len(b) > 1:
                del b[int(rng.integers(0, len(b)))]
        buf = bytes(b)
        rc_ref, dec_ref, used_ref = O.ref_decode(buf)
        try:
            dec, used = A.frame_decode(buf)
            rc = 0
        except A.DemodError as e:
            rc = e.code
        assert (rc == 0) == (rc_ref == 0), (buf.hex(), rc, rc_ref)
        if rc == 0:
            assert dec == dec_ref and used == used_ref


def _python_protobuf_classes():
    pytest.importorskip("google.protobuf")
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    fdp = descriptor_pb2.FileDescriptorProto(name="ip_test.proto", package="t", syntax="proto2")
    ad = fdp.message_type.add(name="AudioData")
    ad.field.add(name="opus_encoded_frame", number=1, label=2, type=12)  # required bytes
    tr = fdp.message_type.add(name="ToReceiver")
    tr.oneof_decl.add(name="message")
    tr.field.add(name="audio_data", number=1, label=1, type=11, type_name=".t.AudioData",
                 oneof_index=0)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = getattr(message_factory, "GetMessageClass", None)
    to_recv = pool.FindMessageTypeByName("t.ToReceiver")
    cls = get(to_recv) if get else message_factory.MessageFactory(pool).GetPrototype(to_recv)
    return cls


def _varint(n):
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def test_matches_protobuf_writeDelimitedTo(A):
    """Transmitter framing: writeVarUInt32(size) + toByteArray()."""
    ToReceiver = _python_protobuf_classes()
    for n in (0, 1, 127, 128, 2000, 4096):
        pl = payload_of(n)
        m = ToReceiver()
        m.audio_data.opus_encoded_frame = pl
        body = m.SerializeToString()
        assert A.frame_encode(pl) == _varint(len(body)) + body
        dec, _ = A.frame_decode(_varint(len(body)) + body)
        parsed = ToReceiver()
        parsed.ParseFromString(body)
        assert parsed.audio_data.opus_encoded_frame == dec == pl


def test_incomplete_frames_ask_for_more(A):
    enc = A.frame_encode(payload_of(300))
    for cut in (0, 1, 2, 5, len(enc) - 1):
        with pytest.raises(A.DemodError) as e:
            A.frame_decode(enc[:cut])
        assert e.value.code == A.DEMOD_BUFFER_TOO_SMALL


def test_encode_limits(A):
    with pytest.raises(A.DemodError) as e:
        A.frame_encode(bytes(4097))
    assert e.value.code == A.DEMOD_FRAME_TOO_LARGE


@pytest.mark.parametrize("bits", range(1, 9))
def test_pack_unpack_roundtrip(A, bits):
    rng = np.random.default_rng(bits)
    for n in (0, 1, 7, 8, 9, 1000):
        s = rng.integers(0, 1 << bits, n, dtype=np.uint8)
        packed = A.pack_symbols(s, bits)
        assert len(packed) == (n * bits + 7) // 8
        assert (A.unpack_symbols(packed, n, bits) == s).all()
        # MSB-first reference packing
        bitstr = "".join(format(int(v), f"0{bits}b") for v in s)
        bitstr += "0" * (-len(bitstr) % 8)
        ref = bytes(int(bitstr[i:i + 8], 2) for i in range(0, len(bitstr), 8))
        assert packed == ref


def test_bits_per_symbol(A):
    assert [A.bits_per_symbol(k) for k in (1, 2, 3, 4, 5, 8, 9, 16)] == [1, 1, 2, 2, 3, 3, 4, 4]


def test_frame_symbols_stream(A):
    rng = np.random.default_rng(5)
    for k, n, maxp in ((2, 100000, 4096), (8, 33333, 4096), (16, 5000, 100), (2, 0, 4096)):
        bits = A.bits_per_symbol(k)
        s = rng.integers(0, k, n, dtype=np.uint8)
        stream = A.frame_symbols(s, bits, maxp)
        payloads = list(A.iter_frames(stream))
        assert all(len(p) <= maxp for p in payloads)
        per = maxp * 8 // bits
        got = np.concatenate([A.unpack_symbols(p, min(per, n - i * per), bits)
                              for i, p in enumerate(payloads)]) if payloads else np.zeros(0, np.uint8)
        assert (got == s).all()


@pytest.mark.parametrize("n,bits", [(0, 1), (1, 1), (7, 1), (8, 1), (2048, 1), (32768, 1),
                                    (32769, 1), (100000, 1), (5, 3), (10923, 3), (40000, 3),
                                    (16384, 2), (8193, 4), (3, 8), (4097, 8)])
def test_frame_symbols_size_matches_host_framing(A, n, bits):
    """demod_frame_symbols_size == len(demod_frame_symbols output)."""
    sym = np.random.default_rng(n + bits).integers(0, 1 << bits, n, dtype=np.uint8)
    assert A.frame_symbols_size(n, bits) == len(A.frame_symbols(sym, bits))
    for mp in (1, 17, 256):
        assert A.frame_symbols_size(n, bits, mp) == len(A.frame_symbols(sym, bits, mp))
