/*
 * demod_session.c — the ip.proto session messages around the audio stream
 * (SURVEY.md §8f row 4): the TCP 58764 hello a receiver sends when a
 * transmitter connects, the ReceiverError it may send back, and the UDP 58765
 * discovery exchange.
 *
 *   BroadcastMessage { required uint32 magic_word = 1;
 *                      oneof { bool discovery_request = 2;
 *                              DiscoveryResponse discovery_response = 3; } }
 *   DiscoveryResponse { required uint32 protocol_version = 1;
 *                       required uint64 mac_address = 2;
 *                       required string device_name = 3;      (char[128])
 *                       required bool currently_streaming = 4;
 *                       required string opus_version = 5; }   (char[128])
 *   ToTransmitter { oneof { ReceiverInformation receiver_information = 1;
 *                           ReceiverError error = 2; } }
 *   ReceiverInformation { required DiscoveryResponse discovery_data = 1;
 *                         required uint32 max_encoded_frame_size = 2;
 *                         required uint32 max_decoded_frame_size = 3; }
 *   ReceiverError { required bool audio_underflow = 1;
 *                   required bool audio_decode_error = 2; }
 * (protocol/ip.proto:8-61; nanopb layout hardware/src/protogen/ip.pb.h:17-62).
 *
 * Encoders write what the reference's nanopb pb_encode writes for the same
 * struct: every required field in tag order, strings as strlen bytes of a
 * char[128] (pb_encode.c:863-890), bools as varint 0/1. The hello is length
 * delimited (pb_encode_delimited, network.cpp:388-403); broadcast datagrams
 * are not (pb_encode / pb_decode on the datagram, network.cpp:473-492;
 * BroadcastMessage.toByteArray / parseFrom, discovery.kt:44-48,84).
 *
 * Decoders give nanopb 0.4.5's verdict and values (pb_decode.c):
 * unknown fields skipped, zero tag rejected, wire type checked per field
 * (decode_basic_field :393-460), uint32 overflow rejected (pb_dec_varint
 * :1406-1430), strings longer than 127 bytes rejected (pb_dec_string
 * :1518-1560), every required field present in each (sub)message occurrence
 * (pb_decode_inner :1100-1137), a repeated member of the same oneof merged
 * into it, a switch of oneof member resetting it (decode_static_field
 * :519-545). Parity with the reference codec is tested against
 * oracle/_ref (tests/test_session.py).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "../../include/demod.h"
#include "pbwire.h"

/* ---- encode ----------------------------------------------------------- */

/* strlen of a nanopb char[DEMOD_INFO_STRING_CAP]; -1 when unterminated
 * (pb_enc_string "unterminated string"). */
static long info_strlen(const char *s)
{
    const void *nul = memchr(s, 0, DEMOD_INFO_STRING_CAP);
    return nul ? (long)((const char *)nul - s) : -1;
}

static size_t discovery_body_size(const demod_discovery_t *d, size_t name_len, size_t ver_len)
{
    return 1 + varint_len(d->protocol_version) + 1 + varint_len(d->mac_address) + 1 +
           varint_len(name_len) + name_len + 2 + 1 + varint_len(ver_len) + ver_len;
}

static size_t put_discovery_body(uint8_t *o, const demod_discovery_t *d, size_t name_len,
                                 size_t ver_len)
{
    size_t p = 0;
    o[p++] = 0x08;
    p += put_varint(o + p, d->protocol_version);
    o[p++] = 0x10;
    p += put_varint(o + p, d->mac_address);
    o[p++] = 0x1A;
    p += put_varint(o + p, name_len);
    memcpy(o + p, d->device_name, name_len);
    p += name_len;
    o[p++] = 0x20;
    o[p++] = d->currently_streaming ? 1 : 0;
    o[p++] = 0x2A;
    p += put_varint(o + p, ver_len);
    memcpy(o + p, d->opus_version, ver_len);
    return p + ver_len;
}

int demod_broadcast_request_encode(uint8_t *out, size_t cap)
{
    if (!out) return DEMOD_BAD_ARG;
    const size_t need = 1 + varint_len(DEMOD_BROADCAST_MAGIC) + 2;
    if (cap < need) return DEMOD_BUFFER_TOO_SMALL;
    size_t p = 0;
    out[p++] = 0x08;
    p += put_varint(out + p, DEMOD_BROADCAST_MAGIC);
    out[p++] = 0x10; /* discovery_request = true */
    out[p++] = 0x01;
    return (int)p;
}

int demod_broadcast_response_encode(const demod_discovery_t *d, uint8_t *out, size_t cap)
{
    if (!d || !out) return DEMOD_BAD_ARG;
    long nl = info_strlen(d->device_name), vl = info_strlen(d->opus_version);
    if (nl < 0 || vl < 0) return DEMOD_BAD_ARG;
    size_t body = discovery_body_size(d, (size_t)nl, (size_t)vl);
    size_t need = 1 + varint_len(DEMOD_BROADCAST_MAGIC) + 1 + varint_len(body) + body;
    if (cap < need) return DEMOD_BUFFER_TOO_SMALL;
    size_t p = 0;
    out[p++] = 0x08;
    p += put_varint(out + p, DEMOD_BROADCAST_MAGIC);
    out[p++] = 0x1A;
    p += put_varint(out + p, body);
    p += put_discovery_body(out + p, d, (size_t)nl, (size_t)vl);
    return (int)p;
}

int demod_hello_encode(const demod_receiver_info_t *info, uint8_t *out, size_t cap)
{
    if (!info || !out) return DEMOD_BAD_ARG;
    const demod_discovery_t *d = &info->discovery_data;
    long nl = info_strlen(d->device_name), vl = info_strlen(d->opus_version);
    if (nl < 0 || vl < 0) return DEMOD_BAD_ARG;
    size_t body = discovery_body_size(d, (size_t)nl, (size_t)vl);
    size_t ri = 1 + varint_len(body) + body + 1 + varint_len(info->max_encoded_frame_size) + 1 +
                varint_len(info->max_decoded_frame_size);
    size_t msg = 1 + varint_len(ri) + ri;
    size_t need = varint_len(msg) + msg;
    if (cap < need) return DEMOD_BUFFER_TOO_SMALL;
    size_t p = put_varint(out, msg);
    out[p++] = 0x0A; /* ToTransmitter.receiver_information */
    p += put_varint(out + p, ri);
    out[p++] = 0x0A; /* ReceiverInformation.discovery_data */
    p += put_varint(out + p, body);
    p += put_discovery_body(out + p, d, (size_t)nl, (size_t)vl);
    out[p++] = 0x10;
    p += put_varint(out + p, info->max_encoded_frame_size);
    out[p++] = 0x18;
    p += put_varint(out + p, info->max_decoded_frame_size);
    return (int)p;
}

int demod_receiver_error_encode(const demod_receiver_error_t *e, uint8_t *out, size_t cap)
{
    if (!e || !out) return DEMOD_BAD_ARG;
    if (cap < 7) return DEMOD_BUFFER_TOO_SMALL;
    const uint8_t msg[7] = {6, 0x12, 4, 0x08, e->audio_underflow ? 1 : 0, 0x10,
                            e->audio_decode_error ? 1 : 0};
    memcpy(out, msg, sizeof msg);
    return (int)sizeof msg;
}

/* ---- decode ----------------------------------------------------------- */

/* Length-delimited field body: [*pos, *pos + n) inside [.., end). */
static int get_len(const uint8_t *in, size_t end, size_t *pos, size_t *n)
{
    uint32_t v;
    if (get_varint32(in, end, pos, &v) != 0) return -1;
    if (v > end - *pos) return -1; /* "end-of-stream" / "parent stream too short" */
    *n = v;
    return 0;
}

static int get_u32(const uint8_t *in, size_t end, size_t *pos, unsigned wire, uint32_t *out)
{
    uint64_t v;
    if (wire != 0 || get_varint64(in, end, pos, &v) != 0) return -1;
    if (v > 0xFFFFFFFFu) return -1; /* "integer too large" */
    *out = (uint32_t)v;
    return 0;
}

static int get_bool(const uint8_t *in, size_t end, size_t *pos, unsigned wire, int *out)
{
    uint32_t v;
    if (wire != 0 || get_varint32(in, end, pos, &v) != 0) return -1;
    *out = v != 0;
    return 0;
}

static int get_string(const uint8_t *in, size_t end, size_t *pos, unsigned wire, char *dst)
{
    uint32_t v;
    if (wire != 2 || get_varint32(in, end, pos, &v) != 0) return -1;
    if (v == 0xFFFFFFFFu || (size_t)v + 1 > DEMOD_INFO_STRING_CAP) return -1; /* overflow */
    if (v > end - *pos) return -1;
    memcpy(dst, in + *pos, v);
    dst[v] = 0;
    *pos += v;
    return 0;
}

/* Field loop shared by every message: reads a tag, rejects tag 0, skips
 * fields numbered above max_field; returns the field number, 0 at the end of
 * [*pos, end), -1 on malformed bytes. */
static int next_field(const uint8_t *in, size_t end, size_t *pos, unsigned max_field,
                      unsigned *wire)
{
    for (;;) {
        if (*pos >= end) return 0;
        uint32_t tag;
        if (get_varint32(in, end, pos, &tag) != 0) return -1;
        unsigned field = tag >> 3;
        *wire = tag & 7;
        if (field == 0) return -1; /* "zero tag" */
        if (field <= max_field) return (int)field;
        if (skip_field(in, end, pos, *wire) != 0) return -1;
    }
}

/* One DiscoveryResponse occurrence in [pos, end), merged into *d. */
static int parse_discovery(const uint8_t *in, size_t pos, size_t end, demod_discovery_t *d)
{
    unsigned seen = 0, wire;
    int f;
    while ((f = next_field(in, end, &pos, 5, &wire)) > 0) {
        int rc;
        switch (f) {
        case 1: rc = get_u32(in, end, &pos, wire, &d->protocol_version); break;
        case 2: rc = (wire != 0 || get_varint64(in, end, &pos, &d->mac_address) != 0) ? -1 : 0; break;
        case 3: rc = get_string(in, end, &pos, wire, d->device_name); break;
        case 4: rc = get_bool(in, end, &pos, wire, &d->currently_streaming); break;
        default: rc = get_string(in, end, &pos, wire, d->opus_version); break;
        }
        if (rc) return -1;
        seen |= 1u << f;
    }
    return (f < 0 || seen != 0x3Eu) ? -1 : 0; /* "missing required field" */
}

int demod_broadcast_decode(const uint8_t *in, size_t len, uint32_t *magic, demod_discovery_t *resp)
{
    if ((!in && len) || !magic) return DEMOD_BAD_ARG;
    demod_discovery_t tmp;
    demod_discovery_t *d = resp ? resp : &tmp;
    size_t pos = 0;
    int which = 0, have_magic = 0, f;
    unsigned wire;
    while ((f = next_field(in, len, &pos, 3, &wire)) > 0) {
        if (f == 1) {
            if (get_u32(in, len, &pos, wire, magic)) return DEMOD_INVALID_PACKET;
            have_magic = 1;
        } else if (f == 2) {
            int v;
            which = DEMOD_MSG_DISCOVERY_REQUEST;
            if (get_bool(in, len, &pos, wire, &v)) return DEMOD_INVALID_PACKET;
        } else {
            size_t n;
            if (wire != 2 || get_len(in, len, &pos, &n)) return DEMOD_INVALID_PACKET;
            if (which != DEMOD_MSG_DISCOVERY_RESPONSE) memset(d, 0, sizeof *d);
            which = DEMOD_MSG_DISCOVERY_RESPONSE;
            if (parse_discovery(in, pos, pos + n, d)) return DEMOD_INVALID_PACKET;
            pos += n;
        }
    }
    if (f < 0 || !have_magic) return DEMOD_INVALID_PACKET;
    return which;
}

static int parse_receiver_info(const uint8_t *in, size_t pos, size_t end,
                               demod_receiver_info_t *ri)
{
    unsigned seen = 0, wire;
    int f;
    while ((f = next_field(in, end, &pos, 3, &wire)) > 0) {
        if (f == 1) {
            size_t n;
            if (wire != 2 || get_len(in, end, &pos, &n)) return -1;
            if (parse_discovery(in, pos, pos + n, &ri->discovery_data)) return -1;
            pos += n;
        } else if (get_u32(in, end, &pos, wire,
                           f == 2 ? &ri->max_encoded_frame_size : &ri->max_decoded_frame_size)) {
            return -1;
        }
        seen |= 1u << f;
    }
    return (f < 0 || seen != 0xEu) ? -1 : 0;
}

static int parse_receiver_error(const uint8_t *in, size_t pos, size_t end,
                                demod_receiver_error_t *e)
{
    unsigned seen = 0, wire;
    int f;
    while ((f = next_field(in, end, &pos, 2, &wire)) > 0) {
        if (get_bool(in, end, &pos, wire, f == 1 ? &e->audio_underflow : &e->audio_decode_error))
            return -1;
        seen |= 1u << f;
    }
    return (f < 0 || seen != 0x6u) ? -1 : 0;
}

int demod_to_transmitter_decode(const uint8_t *in, size_t len, demod_receiver_info_t *info,
                                demod_receiver_error_t *err, size_t *consumed)
{
    if ((!in && len) || !consumed) return DEMOD_BAD_ARG;
    demod_receiver_info_t ti;
    demod_receiver_error_t te;
    if (!info) info = &ti;
    if (!err) err = &te;
    size_t pos = 0;
    uint32_t msg;
    int r = get_varint32(in, len, &pos, &msg);
    if (r == 1) return DEMOD_BUFFER_TOO_SMALL;
    if (r < 0) return DEMOD_INVALID_PACKET;
    if (msg > len - pos) return DEMOD_BUFFER_TOO_SMALL;
    const size_t end = pos + msg;
    int which = 0, f;
    unsigned wire;
    while ((f = next_field(in, end, &pos, 2, &wire)) > 0) {
        size_t n;
        if (wire != 2 || get_len(in, end, &pos, &n)) return DEMOD_INVALID_PACKET;
        int rc;
        if (f == DEMOD_MSG_RECEIVER_INFORMATION) {
            if (which != f) memset(info, 0, sizeof *info);
            rc = parse_receiver_info(in, pos, pos + n, info);
        } else {
            if (which != f) memset(err, 0, sizeof *err);
            rc = parse_receiver_error(in, pos, pos + n, err);
        }
        which = f;
        if (rc) return DEMOD_INVALID_PACKET;
        pos += n;
    }
    if (f < 0) return DEMOD_INVALID_PACKET;
    *consumed = end;
    return which;
}
