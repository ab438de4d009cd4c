"""Test-case builders for the ip.proto session messages (tests/test_session.py,
tests/golden/make_session_golden.py): structs to encode, crafted decode edge
cases written as raw protobuf bytes, and seeded mutations of valid messages.
Deterministic, pure Python (no reference code)."""
import numpy as np

MAGIC = 0x2C5DA044

STRUCTS = [
    # what the firmware announces (network.cpp:356-378): empty device name
    {"protocol_version": 1, "mac_address": 0x0000F6E5D4C3B2A1, "device_name": b"",
     "currently_streaming": False, "opus_version": b"libopus 1.3.1-fixed"},
    {"protocol_version": 0, "mac_address": 0, "device_name": b"", "currently_streaming": False,
     "opus_version": b""},
    {"protocol_version": 0xFFFFFFFF, "mac_address": 0xFFFFFFFFFFFFFFFF,
     "device_name": b"x" * 127, "currently_streaming": True, "opus_version": b"v" * 127},
    {"protocol_version": 127, "mac_address": 128, "device_name": b"living room",
     "currently_streaming": True, "opus_version": b"fskdemod 0.1.0 (gfx950 HIP)"},
    {"protocol_version": 128, "mac_address": 1 << 63, "device_name": "Küche".encode(),
     "currently_streaming": False, "opus_version": b"a" * 126},
]
MAXES = [(4096, 11520), (0, 0), (0xFFFFFFFF, 0xFFFFFFFF), (127, 128), (16384, 1)]


def varint(n):
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def tag(field, wire):
    return varint(field << 3 | wire)


def ld(field, body):
    return tag(field, 2) + varint(len(body)) + body


def vf(field, v):
    return tag(field, 0) + varint(v)


def disc(pv=1, mac=0xA1B2, name=b"n", streaming=0, ver=b"v", drop=None, extra=b""):
    parts = {1: vf(1, pv), 2: vf(2, mac), 3: ld(3, name), 4: vf(4, streaming), 5: ld(5, ver)}
    return b"".join(p for f, p in parts.items() if f != drop) + extra


def bm(*parts):
    return b"".join(parts)


def delim(body):
    return varint(len(body)) + body


def rinfo(d=None, me=4096, md=11520, drop=None, extra=b""):
    parts = {1: ld(1, disc() if d is None else d), 2: vf(2, me), 3: vf(3, md)}
    return b"".join(p for f, p in parts.items() if f != drop) + extra


def rerr(u=1, e=0, drop=None):
    parts = {1: vf(1, u), 2: vf(2, e)}
    return b"".join(p for f, p in parts.items() if f != drop)


def crafted_broadcast():
    m = vf(1, MAGIC)
    req = vf(2, 1)
    resp = ld(3, disc())
    over = tag(1, 0) + b"\xc4\xc0\xf6\xe2\x12"          # 5-byte varint > 2^32
    cases = [
        ("empty", b""),
        ("magic_only", m),
        ("request", m + req),
        ("request_false", m + vf(2, 0)),
        ("request_no_magic", req),
        ("request_wrong_magic", vf(1, 0x2C5DA045) + req),
        ("request_bool_10byte", m + tag(2, 0) + b"\x81\x80\x80\x80\x80\x80\x80\x80\x80\x01"),
        ("request_bool_bad_sign", m + tag(2, 0) + b"\x81\x80\x80\x80\x80\x80\x80\x80\x80\x02"),
        ("request_wire2", m + ld(2, b"\x01")),
        ("magic_overflow", over + req),
        ("magic_fixed32", tag(1, 5) + b"\x44\xa0\x5d\x2c" + req),
        ("magic_twice_last_wins", vf(1, 7) + m + req),
        ("request_before_magic", req + m),
        ("response", m + resp),
        ("response_then_request", m + resp + req),
        ("request_then_response", m + req + resp),
        ("response_twice_merge", m + ld(3, disc(name=b"a")) + ld(3, disc(name=b"bb", pv=9))),
        ("response_missing_pv", m + ld(3, disc(drop=1))),
        ("response_missing_mac", m + ld(3, disc(drop=2))),
        ("response_missing_name", m + ld(3, disc(drop=3))),
        ("response_missing_stream", m + ld(3, disc(drop=4))),
        ("response_missing_ver", m + ld(3, disc(drop=5))),
        ("response_missing_then_full", m + ld(3, disc(drop=3)) + resp),
        ("response_name_127", m + ld(3, disc(name=b"n" * 127))),
        ("response_name_128", m + ld(3, disc(name=b"n" * 128))),
        ("response_ver_128", m + ld(3, disc(ver=b"v" * 128))),
        ("response_name_nul", m + ld(3, disc(name=b"ab\x00cd"))),
        ("response_pv_overflow", m + ld(3, disc(pv=1 << 32))),
        ("response_mac_max", m + ld(3, disc(mac=(1 << 64) - 1))),
        ("response_mac_11byte", m + ld(3, disc(drop=2, extra=tag(2, 0) + b"\xff" * 10 + b"\x01"))),
        ("response_mac_10byte_hi", m + ld(3, disc(drop=2, extra=tag(2, 0) + b"\xff" * 9 + b"\x7f"))),
        ("response_stream_2", m + ld(3, disc(streaming=2))),
        ("response_name_wire0", m + ld(3, disc(drop=3, extra=vf(3, 5)))),
        ("response_unknown_fields", m + ld(3, disc(extra=vf(9, 1) + ld(10, b"xyz") +
                                                 tag(11, 1) + b"\0" * 8 + tag(12, 5) + b"\0" * 4))),
        ("response_group_field", m + ld(3, disc(extra=tag(9, 3)))),
        ("response_zero_tag", m + ld(3, disc() + b"\x00")),
        ("response_truncated", m + ld(3, disc())[:-2]),
        ("response_len_past_end", m + tag(3, 2) + varint(200) + disc()),
        ("response_wire0", m + vf(3, 1)),
        ("unknown_top_fields", m + vf(4, 3) + ld(15, b"\x01\x02") + req),
        ("top_zero_tag", m + req + b"\x00"),
        ("top_wire6", m + tag(5, 6) + req),
        ("top_wire7", m + tag(5, 7)),
        ("top_skip_varint_unterminated", m + tag(5, 0) + b"\x80\x80"),
        ("top_ld_truncated", m + tag(5, 2) + varint(5) + b"ab"),
        ("top_fixed64_truncated", m + tag(5, 1) + b"\0" * 7),
        ("top_tag_overlong", m + b"\x90\x80\x80\x80\x00" + b"\x01"),
        ("top_tag_6byte", m + b"\x90\x80\x80\x80\x80\x00\x01"),
        ("top_tag_5th_high_bits", m + b"\x90\x80\x80\x80\x10\x01"),
    ]
    return cases


def crafted_to_transmitter():
    ri = ld(1, rinfo())
    er = ld(2, rerr())
    cases = [
        ("empty_message", delim(b"")),
        ("empty_input", b""),
        ("hello", delim(ri)),
        ("error", delim(er)),
        ("error_all_false", delim(ld(2, rerr(0, 0)))),
        ("hello_then_error", delim(ri + er)),
        ("error_then_hello", delim(er + ri)),
        ("hello_twice", delim(ld(1, rinfo(me=1)) + ld(1, rinfo(md=2)))),
        ("hello_missing_disc", delim(ld(1, rinfo(drop=1)))),
        ("hello_missing_maxenc", delim(ld(1, rinfo(drop=2)))),
        ("hello_missing_maxdec", delim(ld(1, rinfo(drop=3)))),
        ("hello_disc_missing_field", delim(ld(1, rinfo(d=disc(drop=4))))),
        ("hello_disc_twice", delim(ld(1, rinfo(extra=ld(1, disc(name=b"second", pv=5)))))),
        ("hello_disc_twice_partial", delim(ld(1, rinfo(extra=ld(1, disc(drop=1)))))),
        ("hello_maxenc_overflow", delim(ld(1, rinfo(me=1 << 33)))),
        ("hello_maxenc_wire5", delim(ld(1, rinfo(drop=2, extra=tag(2, 5) + b"\0\x10\0\0")))),
        ("hello_disc_wire0", delim(ld(1, rinfo(drop=1, extra=vf(1, 3))))),
        ("error_missing_decode", delim(ld(2, rerr(drop=2)))),
        ("error_missing_underflow", delim(ld(2, rerr(drop=1)))),
        ("error_bool_overlong", delim(ld(2, tag(1, 0) + b"\x80\x80\x80\x80\x80\x80\x01" +
                                         vf(2, 1)))),
        ("error_wire2", delim(ld(2, ld(1, b"\x01") + vf(2, 0)))),
        ("member_wire0", delim(vf(1, 1))),
        ("unknown_top", delim(vf(3, 1) + ld(4, b"zz") + ri)),
        ("zero_tag", delim(ri + b"\x00")),
        ("truncated_prefix_only", varint(len(ri))),
        ("truncated_body", delim(ri)[:-3]),
        ("trailing_bytes", delim(ri) + b"\x05garbage"),
        ("prefix_overlong", b"\x80\x80\x80\x80\x80\x80\x80\x80\x80\x80\x00"),
        ("inner_len_past_end", delim(tag(1, 2) + varint(200) + rinfo())),
    ]
    return cases


def broadcast_bases():
    return [vf(1, MAGIC) + vf(2, 1), vf(1, MAGIC) + ld(3, disc(name=b"dev", ver=b"libopus")),
            vf(1, MAGIC) + ld(3, disc(mac=(1 << 48) - 3))]


def to_transmitter_bases():
    return [delim(ld(1, rinfo())), delim(ld(2, rerr(1, 1))),
            delim(ld(1, rinfo(d=disc(name=b"", ver=b"libopus 1.3.1-fixed"))))]


def mutations(bases, count, seed):
    """Seeded byte flips / inserts / deletes of valid messages."""
    rng = np.random.default_rng(seed)
    out = []
    for it in range(count):
        b = bytearray(bases[it % len(bases)])
        for _ in range(int(rng.integers(1, 4))):
            op = int(rng.integers(0, 3))
            if op == 0 and len(b):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            elif op == 1:
                b.insert(int(rng.integers(0, len(b) + 1)), int(rng.integers(0, 256)))
            elif len(b) > 1:
                del b[int(rng.integers(0, len(b)))]
        out.append((f"mut{seed}_{it}", bytes(b)))
    return out
