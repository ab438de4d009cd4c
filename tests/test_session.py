"""ip.proto session messages (host C, libfskdemod.so demod_session.c) against
the reference's nanopb.

Golden bytes and decode verdicts in tests/golden/session_golden.json come
from the reference's own nanopb 0.4.5 + ip.pb.c (oracle/ref.mk, generator
tests/golden/make_session_golden.py); when oracle/_ref is present the same
checks also run live, over more seeded mutations. The transmitter side
(protobuf-java toByteArray / parseFrom / readSingleDelimited, discovery.kt:44-84,
RemoteAudioReceiver.kt:60) is cross-checked with the Python protobuf runtime on
a descriptor built from protocol/ip.proto.
"""
import json
import os

import pytest

import session_cases as C

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "session_golden.json")))


def _d(j):
    return {k: (bytes.fromhex(v) if k in ("device_name", "opus_version") else v)
            for k, v in j.items()}


def _fields(j):
    if j is None or "discovery_data" not in j:
        return j
    return dict(j, discovery_data=_d(j["discovery_data"]))


def _ours_broadcast(A, buf):
    try:
        which, magic, d = A.broadcast_decode(buf)
        return 0, which, magic, d
    except A.DemodError as e:
        assert e.code == A.DEMOD_INVALID_PACKET
        return -1, None, None, None


def _ours_to_transmitter(A, buf):
    try:
        which, f, used = A.to_transmitter_decode(buf)
        return 0, which, f, used
    except A.DemodError as e:
        assert e.code in (A.DEMOD_INVALID_PACKET, A.DEMOD_BUFFER_TOO_SMALL)
        return -1, None, None, None


def test_request_matches_reference(A):
    assert A.broadcast_request_encode().hex() == GOLD["request_hex"]
    assert A.broadcast_request_encode() == bytes.fromhex("08c4c0f6e2021001")


@pytest.mark.parametrize("i", range(len(GOLD["encodings"])))
def test_response_and_hello_match_reference(A, i):
    g = GOLD["encodings"][i]
    d = _d(g["discovery"])
    assert A.broadcast_response_encode(d).hex() == g["response_hex"]
    info = {"discovery_data": d, "max_encoded_frame_size": g["max_encoded_frame_size"],
            "max_decoded_frame_size": g["max_decoded_frame_size"]}
    hello = A.hello_encode(info)
    assert hello.hex() == g["hello_hex"]
    assert A.broadcast_decode(A.broadcast_response_encode(d)) == (
        A.DEMOD_MSG_DISCOVERY_RESPONSE, A.DEMOD_BROADCAST_MAGIC, d)
    assert A.to_transmitter_decode(hello) == (A.DEMOD_MSG_RECEIVER_INFORMATION, info, len(hello))


@pytest.mark.parametrize("g", GOLD["errors"], ids=lambda g: g["hex"])
def test_receiver_error_matches_reference(A, g):
    enc = A.receiver_error_encode(g["audio_underflow"], g["audio_decode_error"])
    assert enc.hex() == g["hex"]
    assert A.to_transmitter_decode(enc) == (
        A.DEMOD_MSG_RECEIVER_ERROR, {"audio_underflow": g["audio_underflow"],
                                     "audio_decode_error": g["audio_decode_error"]}, len(enc))


def test_broadcast_verdicts_match_reference(A):
    bad = []
    for v in GOLD["broadcast_verdicts"]:
        rc, which, magic, d = _ours_broadcast(A, bytes.fromhex(v["hex"]))
        if v["rc"] != 0:
            ok = rc != 0
        else:
            ok = (rc == 0 and which == v["which"] and magic == v["magic"] and
                  d == (None if v["discovery"] is None else _d(v["discovery"])))
        if not ok:
            bad.append(v["name"])
    assert not bad, bad
    names = {v["name"]: v["rc"] for v in GOLD["broadcast_verdicts"]}
    # the edge cases are what the crafted list says they are
    assert names["request"] == 0 and names["response_twice_merge"] == 0
    assert names["response_name_128"] != 0 and names["magic_overflow"] != 0


def test_to_transmitter_verdicts_match_reference(A):
    bad = []
    for v in GOLD["to_transmitter_verdicts"]:
        rc, which, f, used = _ours_to_transmitter(A, bytes.fromhex(v["hex"]))
        if v["rc"] != 0:
            ok = rc != 0
        else:
            ok = (rc == 0 and which == v["which"] and f == _fields(v["fields"]) and
                  used == v["consumed"])
        if not ok:
            bad.append(v["name"])
    assert not bad, bad


def test_discovery_answer_rule(A):
    """network.cpp:473-485: answer iff decoded, magic matches, member is the request."""
    def answers(buf):
        rc, which, magic, _ = _ours_broadcast(A, buf)
        return rc == 0 and magic == A.DEMOD_BROADCAST_MAGIC and which == A.DEMOD_MSG_DISCOVERY_REQUEST

    cases = dict(C.crafted_broadcast())
    assert answers(cases["request"]) and answers(cases["request_false"])
    assert answers(cases["response_then_request"]) and answers(cases["request_before_magic"])
    assert not answers(cases["request_wrong_magic"])
    assert not answers(cases["request_no_magic"])
    assert not answers(cases["response"])
    assert not answers(cases["magic_only"])


def test_partial_hello_asks_for_more(A):
    hello = A.hello_encode({"discovery_data": C.STRUCTS[0]})
    for cut in range(len(hello)):
        with pytest.raises(A.DemodError) as e:
            A.to_transmitter_decode(hello[:cut])
        assert e.value.code == A.DEMOD_BUFFER_TOO_SMALL
    which, _, used = A.to_transmitter_decode(hello + b"\x07trailing")
    assert which == A.DEMOD_MSG_RECEIVER_INFORMATION and used == len(hello)


def test_encode_errors(A):
    import ctypes
    lib = A.load_library()
    d = A._discovery_struct(C.STRUCTS[0])
    ctypes.memmove(ctypes.addressof(d) + A.DemodDiscovery.device_name.offset, b"y" * 128, 128)
    out = (ctypes.c_uint8 * 512)()
    assert lib.demod_broadcast_response_encode(ctypes.byref(d), out, 512) == A.DEMOD_BAD_ARG
    d = A._discovery_struct(C.STRUCTS[2])
    need = len(A.broadcast_response_encode(C.STRUCTS[2]))
    assert lib.demod_broadcast_response_encode(ctypes.byref(d), out, need - 1) == \
        A.DEMOD_BUFFER_TOO_SMALL
    assert lib.demod_broadcast_response_encode(ctypes.byref(d), out, need) == need
    assert lib.demod_broadcast_request_encode(out, 7) == A.DEMOD_BUFFER_TOO_SMALL
    info = A.DemodReceiverInfo()
    info.discovery_data = d
    hneed = lib.demod_hello_encode(ctypes.byref(info), out, 512)
    assert hneed > 0
    assert lib.demod_hello_encode(ctypes.byref(info), out, hneed - 1) == A.DEMOD_BUFFER_TOO_SMALL
    err = A.DemodReceiverError(1, 1)
    assert lib.demod_receiver_error_encode(ctypes.byref(err), out, 6) == A.DEMOD_BUFFER_TOO_SMALL


def test_live_reference_session_fuzz(A, O):
    """More seeded mutations, verdicts and values against the live reference."""
    if O.ref_nanopb() is None:
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    for name, buf in C.mutations(C.broadcast_bases(), 3000, seed=101):
        ref = O.ref_broadcast_decode(buf)
        ours = _ours_broadcast(A, buf)
        assert (ours[0] == 0) == (ref[0] == 0), (name, buf.hex())
        if ref[0] == 0:
            assert ours[1:] == ref[1:], (name, buf.hex())
    for name, buf in C.mutations(C.to_transmitter_bases(), 3000, seed=102):
        ref = O.ref_to_transmitter_decode(buf)
        ours = _ours_to_transmitter(A, buf)
        assert (ours[0] == 0) == (ref[0] == 0), (name, buf.hex())
        if ref[0] == 0:
            assert ours[1:] == ref[1:], (name, buf.hex())
    for i, d in enumerate(C.STRUCTS):
        info = {"discovery_data": d, "max_encoded_frame_size": C.MAXES[i][0],
                "max_decoded_frame_size": C.MAXES[i][1]}
        assert A.hello_encode(info) == O.ref_to_transmitter_encode(1, info)
        assert A.broadcast_response_encode(d) == O.ref_broadcast_encode(3, C.MAGIC, d=d)


def _pb_classes():
    pytest.importorskip("google.protobuf")
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    f = descriptor_pb2.FileDescriptorProto(name="ip_session_test.proto", package="s",
                                           syntax="proto2")
    dr = f.message_type.add(name="DiscoveryResponse")
    for name, num, typ in (("protocol_version", 1, 13), ("mac_address", 2, 4),
                           ("device_name", 3, 9), ("currently_streaming", 4, 8),
                           ("opus_version", 5, 9)):
        dr.field.add(name=name, number=num, label=2, type=typ)
    b = f.message_type.add(name="BroadcastMessage")
    b.oneof_decl.add(name="message")
    b.field.add(name="magic_word", number=1, label=2, type=13)
    b.field.add(name="discovery_request", number=2, label=1, type=8, oneof_index=0)
    b.field.add(name="discovery_response", number=3, label=1, type=11,
                type_name=".s.DiscoveryResponse", oneof_index=0)
    ri = f.message_type.add(name="ReceiverInformation")
    ri.field.add(name="discovery_data", number=1, label=2, type=11,
                 type_name=".s.DiscoveryResponse")
    ri.field.add(name="max_encoded_frame_size", number=2, label=2, type=13)
    ri.field.add(name="max_decoded_frame_size", number=3, label=2, type=13)
    re_ = f.message_type.add(name="ReceiverError")
    re_.field.add(name="audio_underflow", number=1, label=2, type=8)
    re_.field.add(name="audio_decode_error", number=2, label=2, type=8)
    tt = f.message_type.add(name="ToTransmitter")
    tt.oneof_decl.add(name="message")
    tt.field.add(name="receiver_information", number=1, label=1, type=11,
                 type_name=".s.ReceiverInformation", oneof_index=0)
    tt.field.add(name="error", number=2, label=1, type=11, type_name=".s.ReceiverError",
                 oneof_index=0)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(f)
    get = getattr(message_factory, "GetMessageClass", None)

    def cls(n):
        d = pool.FindMessageTypeByName("s." + n)
        return get(d) if get else message_factory.MessageFactory(pool).GetPrototype(d)
    return cls("BroadcastMessage"), cls("ToTransmitter")


def test_transmitter_side_protobuf(A):
    """discovery.kt:44-48 request bytes; discovery.kt:84 / RemoteAudioReceiver.kt:60
    parse what this receiver sends."""
    Broadcast, ToTransmitter = _pb_classes()
    req = Broadcast(magic_word=C.MAGIC, discovery_request=True)
    assert req.SerializeToString() == A.broadcast_request_encode()
    rc, _, magic, _ = _ours_broadcast(A, req.SerializeToString())
    assert rc == 0 and magic == C.MAGIC
    for i, d in enumerate(C.STRUCTS):
        resp = Broadcast()
        resp.ParseFromString(A.broadcast_response_encode(d))
        assert resp.WhichOneof("message") == "discovery_response"
        r = resp.discovery_response
        assert (r.protocol_version, r.mac_address, r.device_name.encode(),
                r.currently_streaming, r.opus_version.encode()) == (
            d["protocol_version"], d["mac_address"], d["device_name"],
            d["currently_streaming"], d["opus_version"])
        info = {"discovery_data": d, "max_encoded_frame_size": C.MAXES[i][0],
                "max_decoded_frame_size": C.MAXES[i][1]}
        hello = A.hello_encode(info)
        n, p = 0, 0
        while True:  # readVarUInt32 prefix (protobuf_async.kt:42-67)
            byte = hello[p]
            n |= (byte & 0x7F) << (7 * p)
            p += 1
            if not byte & 0x80:
                break
        t = ToTransmitter()
        t.ParseFromString(hello[p:p + n])
        assert p + n == len(hello)
        assert t.WhichOneof("message") == "receiver_information"
        assert t.receiver_information.max_encoded_frame_size == C.MAXES[i][0]
        assert t.receiver_information.max_decoded_frame_size == C.MAXES[i][1]
        assert t.receiver_information.discovery_data.SerializeToString() == \
            r.SerializeToString()
