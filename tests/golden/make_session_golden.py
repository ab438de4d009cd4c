#!/usr/bin/env python3
"""Regenerate tests/golden/session_golden.json (this container only).

    python tests/golden/make_session_golden.py      (from the repo root)

Session messages of ip.proto encoded, and decode
verdicts + decoded values given, by the reference's OWN nanopb 0.4.5 +
generated ip.pb.c compiled in place from /root/reference by oracle/ref.mk
(oracle/_ref/libnanopb_ref.so, harness oracle/nanopb_ref_harness.c):

- "encodings": BroadcastMessage (discovery request / response, pb_encode as
  network.cpp:486-492) and delimited ToTransmitter (hello /
  error, pb_encode_delimited as network.cpp:388-403) for the structs in
  session_cases.STRUCTS;
- "broadcast_verdicts" / "to_transmitter_verdicts": pb_decode /
  pb_decode_delimited of crafted edge cases (session_cases.crafted_*) and
  seeded mutations of valid messages (session_cases.mutations).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))
from oracle import oracle as O  # noqa: E402
import session_cases as C  # noqa: E402


def jd(d):
    """discovery dict -> JSON (bytes as hex)."""
    if d is None:
        return None
    return {k: (v.hex() if isinstance(v, bytes) else v) for k, v in d.items()}


def jfields(f):
    if f is None:
        return None
    if "discovery_data" in f:
        f = dict(f, discovery_data=jd(f["discovery_data"]))
    return f


def main():
    if O.ref_nanopb() is None:
        sys.exit("oracle/_ref/libnanopb_ref.so missing: make -f oracle/ref.mk")
    enc = []
    for i, d in enumerate(C.STRUCTS):
        info = {"discovery_data": d, "max_encoded_frame_size": C.MAXES[i % len(C.MAXES)][0],
                "max_decoded_frame_size": C.MAXES[i % len(C.MAXES)][1]}
        enc.append({"discovery": jd(d), "max_encoded_frame_size": info["max_encoded_frame_size"],
                    "max_decoded_frame_size": info["max_decoded_frame_size"],
                    "response_hex": O.ref_broadcast_encode(3, C.MAGIC, d=d).hex(),
                    "hello_hex": O.ref_to_transmitter_encode(1, info).hex()})
    errors = [{"audio_underflow": u, "audio_decode_error": e,
               "hex": O.ref_to_transmitter_encode(2, underflow=u, decode_error=e).hex()}
              for u in (False, True) for e in (False, True)]
    request_hex = O.ref_broadcast_encode(2, C.MAGIC, True).hex()

    bv = []
    for name, buf in C.crafted_broadcast() + C.mutations(C.broadcast_bases(), 400, seed=7):
        rc, which, magic, d = O.ref_broadcast_decode(buf)
        bv.append({"name": name, "hex": buf.hex(), "rc": rc, "which": which, "magic": magic,
                   "discovery": jd(d)})
    tv = []
    for name, buf in C.crafted_to_transmitter() + C.mutations(C.to_transmitter_bases(), 400,
                                                               seed=8):
        rc, which, f, used = O.ref_to_transmitter_decode(buf)
        tv.append({"name": name, "hex": buf.hex(), "rc": rc, "which": which,
                   "fields": jfields(f), "consumed": used if rc == 0 else None})
    out = {"generator": "tests/golden/make_session_golden.py (reference nanopb 0.4.5, oracle/_ref)",
           "request_hex": request_hex, "encodings": enc, "errors": errors,
           "broadcast_verdicts": bv, "to_transmitter_verdicts": tv}
    json.dump(out, open(os.path.join(HERE, "session_golden.json"), "w"), indent=0)
    print("session_golden.json:", len(enc), "structs,", len(bv), "broadcast and", len(tv),
          "to_transmitter verdicts,", sum(v["rc"] == 0 for v in bv + tv), "accepted")


if __name__ == "__main__":
    main()
