/*
 * demod_frame.c — ip.proto framing of decoded symbols.
 *
 * Own minimal protobuf wire codec for exactly one message shape,
 *   ToReceiver { oneof message { AudioData audio_data = 1; } }
 *   AudioData  { required bytes opus_encoded_frame = 1; }
 * (protocol/ip.proto:32-36,63-65), length-delimited with a varint32 prefix as
 * nanopb pb_encode_delimited / pb_decode_delimited do on the receiver
 * (hardware/src/network.cpp:389-403,411) and protobuf-java writeDelimitedTo /
 * readSingleDelimited do on the transmitter (protobuf_async.kt:42-114).
 * Byte-for-byte parity with the reference's nanopb is checked against golden
 * frames minted by oracle/_ref (tests/test_frame.py).
 *
 * Decode rules follow nanopb's behaviour for this schema: unknown fields are
 * skipped, the last occurrence of a bytes field wins, a missing required
 * opus_encoded_frame or a missing audio_data is an error, payloads above
 * MAX_ENCODED_FRAME_SIZE (network.cpp:24,223-227) are rejected.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/demod.h"
#include "pbwire.h"

size_t demod_frame_size(size_t payload_len)
{
    size_t inner = 1 + varint_len(payload_len) + payload_len;   /* AudioData */
    size_t msg = 1 + varint_len(inner) + inner;                  /* ToReceiver */
    return varint_len(msg) + msg;
}

int demod_frame_encode(const uint8_t *payload, size_t len, uint8_t *out, size_t cap)
{
    if ((!payload && len) || !out) return DEMOD_BAD_ARG;
    if (len > DEMOD_MAX_FRAME_PAYLOAD) return DEMOD_FRAME_TOO_LARGE;
    size_t need = demod_frame_size(len);
    if (need > cap) return DEMOD_BUFFER_TOO_SMALL;
    size_t inner = 1 + varint_len(len) + len;
    size_t msg = 1 + varint_len(inner) + inner;
    size_t p = put_varint(out, msg);
    out[p++] = 0x0A; /* ToReceiver.audio_data: field 1, wire type 2 */
    p += put_varint(out + p, inner);
    out[p++] = 0x0A; /* AudioData.opus_encoded_frame: field 1, wire type 2 */
    p += put_varint(out + p, len);
    if (len) memcpy(out + p, payload, len);
    return (int)(p + len);
}

/* Parse one AudioData occurrence in [start, end). Its required
 * opus_encoded_frame must be present in THIS occurrence (nanopb checks
 * required fields per submessage decode). A field of a non-length-delimited
 * wire type hands its raw value bytes to the callback, as nanopb's
 * decode_callback_field/read_raw_value do (pb_decode.c:743-784,320-353). */
static int parse_audio_data(const uint8_t *in, size_t start, size_t end, const uint8_t **payload,
                            size_t *payload_len)
{
    size_t pos = start;
    int have = 0;
    while (pos < end) {
        uint32_t tag;
        if (get_varint32(in, end, &pos, &tag) != 0) return DEMOD_INVALID_PACKET;
        unsigned field = tag >> 3, wire = tag & 7;
        if (field == 0) return DEMOD_INVALID_PACKET; /* "zero tag" */
        if (field != 1) {
            if (skip_field(in, end, &pos, wire) != 0) return DEMOD_INVALID_PACKET;
            continue;
        }
        size_t n;
        if (wire == 2) {
            uint32_t v;
            if (get_varint32(in, end, &pos, &v) != 0) return DEMOD_INVALID_PACKET;
            if (v > end - pos) return DEMOD_INVALID_PACKET;
            n = v;
            if (n > DEMOD_MAX_FRAME_PAYLOAD) return DEMOD_FRAME_TOO_LARGE;
        } else if (wire == 0) {
            n = 0;
            do {
                if (pos + n >= end || ++n > 10) return DEMOD_INVALID_PACKET;
            } while (in[pos + n - 1] & 0x80);
        } else if (wire == 1 || wire == 5) {
            n = wire == 1 ? 8 : 4;
            if (end - pos < n) return DEMOD_INVALID_PACKET;
        } else {
            return DEMOD_INVALID_PACKET;
        }
        *payload = in + pos;
        *payload_len = n;
        have = 1;
        pos += n;
    }
    return have ? DEMOD_OK : DEMOD_INVALID_PACKET;
}

int demod_frame_decode(const uint8_t *in, size_t len, const uint8_t **payload, size_t *payload_len,
                       size_t *consumed)
{
    if (!in || !payload || !payload_len || !consumed) return DEMOD_BAD_ARG;
    size_t pos = 0;
    uint32_t msg;
    int r = get_varint32(in, len, &pos, &msg);
    if (r == 1) return DEMOD_BUFFER_TOO_SMALL;
    if (r < 0) return DEMOD_INVALID_PACKET;
    if (msg > len - pos) return DEMOD_BUFFER_TOO_SMALL;
    const size_t end = pos + msg;
    int have_audio = 0;
    const uint8_t *pl = NULL;
    size_t pl_len = 0;
    while (pos < end) {
        uint32_t tag;
        if (get_varint32(in, end, &pos, &tag) != 0) return DEMOD_INVALID_PACKET;
        unsigned field = tag >> 3, wire = tag & 7;
        if (field == 0) return DEMOD_INVALID_PACKET;
        if (field != 1) {
            if (skip_field(in, end, &pos, wire) != 0) return DEMOD_INVALID_PACKET;
            continue;
        }
        uint32_t n;
        if (wire != 2) return DEMOD_INVALID_PACKET; /* submessage: "wrong wire type" */
        if (get_varint32(in, end, &pos, &n) != 0) return DEMOD_INVALID_PACKET;
        if (n > end - pos) return DEMOD_INVALID_PACKET;
        /* a repeated audio_data merges into the same oneof member: a later
         * occurrence's bytes replace the earlier ones */
        int rc = parse_audio_data(in, pos, pos + n, &pl, &pl_len);
        if (rc != DEMOD_OK) return rc;
        have_audio = 1;
        pos += n;
    }
    /* which_message != audio_data: network.cpp:418-421 closes the stream */
    if (!have_audio) return DEMOD_INVALID_PACKET;
    *payload = pl;
    *payload_len = pl_len;
    *consumed = end;
    return DEMOD_OK;
}

int demod_bits_per_symbol(uint32_t k)
{
    int b = 1;
    while ((1u << b) < k) ++b;
    return b;
}

int demod_pack_symbols(const uint8_t *symbols, size_t n, int bits, uint8_t *out, size_t cap)
{
    if ((!symbols && n) || !out || bits < 1 || bits > 8) return DEMOD_BAD_ARG;
    size_t nbytes = (n * (size_t)bits + 7) / 8;
    if (nbytes > cap) return DEMOD_BUFFER_TOO_SMALL;
    if (nbytes > 0x7FFFFFFF) return DEMOD_BAD_ARG;
    memset(out, 0, nbytes);
    size_t bitpos = 0;
    const unsigned mask = (1u << bits) - 1u;
    for (size_t i = 0; i < n; ++i) {
        unsigned v = symbols[i] & mask;
        for (int b = bits - 1; b >= 0; --b, ++bitpos)
            if ((v >> b) & 1u) out[bitpos >> 3] |= (uint8_t)(0x80u >> (bitpos & 7));
    }
    return (int)nbytes;
}

int demod_unpack_symbols(const uint8_t *in, size_t n, int bits, uint8_t *symbols, size_t cap)
{
    if ((!in && n) || (!symbols && n) || bits < 1 || bits > 8) return DEMOD_BAD_ARG;
    if (n > cap) return DEMOD_BUFFER_TOO_SMALL;
    if (n > 0x7FFFFFFF) return DEMOD_BAD_ARG;
    size_t bitpos = 0;
    for (size_t i = 0; i < n; ++i) {
        unsigned v = 0;
        for (int b = 0; b < bits; ++b, ++bitpos)
            v = (v << 1) | ((in[bitpos >> 3] >> (7 - (bitpos & 7))) & 1u);
        symbols[i] = (uint8_t)v;
    }
    return (int)n;
}

long long demod_frame_symbols(const uint8_t *symbols, size_t n, int bits, size_t max_payload,
                              uint8_t *out, size_t cap)
{
    if ((!symbols && n) || !out || bits < 1 || bits > 8) return DEMOD_BAD_ARG;
    if (max_payload < 1 || max_payload > DEMOD_MAX_FRAME_PAYLOAD) return DEMOD_BAD_ARG;
    /* symbols per frame: whole symbols that fit max_payload bytes */
    size_t per = (max_payload * 8) / (size_t)bits;
    uint8_t buf[DEMOD_MAX_FRAME_PAYLOAD];
    size_t written = 0;
    for (size_t i = 0; i < n; i += per) {
        size_t cnt = n - i < per ? n - i : per;
        int pl = demod_pack_symbols(symbols + i, cnt, bits, buf, sizeof(buf));
        if (pl < 0) return pl;
        int fr = demod_frame_encode(buf, (size_t)pl, out + written, cap - written);
        if (fr < 0) return fr;
        written += (size_t)fr;
    }
    return (long long)written;
}
