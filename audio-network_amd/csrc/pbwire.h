/*
 * pbwire.h — protobuf wire-format helpers shared by the ip.proto codecs
 * (demod_frame.c: ToReceiver; demod_session.c: BroadcastMessage,
 * ToTransmitter). Decode-side semantics follow the reference's nanopb 0.4.5
 * (hardware/lib/nanopb/src/pb_decode.c), cited per helper.
 */
#ifndef FSKDEMOD_PBWIRE_H
#define FSKDEMOD_PBWIRE_H
#include <stddef.h>
#include <stdint.h>

static inline size_t varint_len(uint64_t v)
{
    size_t n = 1;
    while (v >= 0x80) { v >>= 7; ++n; }
    return n;
}

static inline size_t put_varint(uint8_t *o, uint64_t v)
{
    size_t n = 0;
    while (v >= 0x80) { o[n++] = (uint8_t)(v | 0x80); v >>= 7; }
    o[n++] = (uint8_t)v;
    return n;
}

/* nanopb pb_decode_varint32 semantics (pb_decode.c:170-232): up to 10
 * bytes; bytes past bit 32 must carry no value bits (0x80/0x00) or be a sign
 * extension of a negative value; a varint ending in its 5th byte may use only
 * that byte's low 4 bits. Returns 0 ok, 1 need more bytes, -1 malformed. */
static inline int get_varint32(const uint8_t *in, size_t len, size_t *pos, uint32_t *out)
{
    if (*pos >= len) return 1;
    uint8_t b = in[(*pos)++];
    if (!(b & 0x80)) { *out = b; return 0; }
    uint32_t r = b & 0x7F;
    unsigned bitpos = 7;
    do {
        if (*pos >= len) return 1;
        b = in[(*pos)++];
        if (bitpos >= 32) {
            uint8_t sign_ext = bitpos < 63 ? 0xFF : 0x01;
            int valid = (b & 0x7F) == 0 || ((r >> 31) != 0 && b == sign_ext);
            if (bitpos >= 64 || !valid) return -1;
        } else {
            r |= (uint32_t)(b & 0x7F) << bitpos;
        }
        bitpos += 7;
    } while (b & 0x80);
    if (bitpos == 35 && (b & 0x70) != 0) return -1;
    *out = r;
    return 0;
}

/* Skip one unknown field (nanopb pb_skip_field, pb_decode.c:305-315). */
static inline int skip_field(const uint8_t *in, size_t end, size_t *pos, unsigned wire)
{
    uint32_t v;
    switch (wire) {
    case 0: /* pb_skip_varint: continuation bytes without a length limit */
        do {
            if (*pos >= end) return -1;
        } while (in[(*pos)++] & 0x80);
        return 0;
    case 1: if (end - *pos < 8) return -1; *pos += 8; return 0;
    case 5: if (end - *pos < 4) return -1; *pos += 4; return 0;
    case 2:
        if (get_varint32(in, end, pos, &v) != 0) return -1;
        if (v > end - *pos) return -1;
        *pos += v;
        return 0;
    default: return -1; /* "invalid wire_type": groups (3,4) and 6,7 */
    }
}

/* nanopb pb_decode_varint (pb_decode.c:240-259): up to 10 bytes, value bits
 * past bit 63 silently dropped, an 11th byte is "varint overflow".
 * Returns 0 ok, 1 need more bytes, -1 malformed. */
static inline int get_varint64(const uint8_t *in, size_t len, size_t *pos, uint64_t *out)
{
    uint64_t r = 0;
    unsigned bitpos = 0;
    uint8_t b;
    do {
        if (bitpos >= 64) return -1;
        if (*pos >= len) return 1;
        b = in[(*pos)++];
        r |= (uint64_t)(b & 0x7F) << bitpos;
        bitpos += 7;
    } while (b & 0x80);
    *out = r;
    return 0;
}

#endif /* FSKDEMOD_PBWIRE_H */
