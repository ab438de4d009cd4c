/*
 * nanopb_ref_harness.c — TEST INFRASTRUCTURE ONLY.
 *
 * Links the reference's own nanopb 0.4.5 runtime and its generated ip.pb.c
 * (compiled in place from /root/reference by oracle/ref.mk, output only into
 * oracle/_ref/) so tests can mint and check ToReceiver frame bytes, and the
 * session messages (BroadcastMessage, ToTransmitter), with the reference's
 * codec.
 *
 * ip.pb.h:161-162 binds AudioData's field callback to the application symbol
 * network_pb_callback_audio_data, which the firmware defines in
 * hardware/src/network.cpp:220-249 (decode only). network.cpp itself cannot
 * be compiled here (Arduino/ESP-IDF/lwIP headers are absent), so this harness
 * supplies that application callback: on decode it behaves like
 * network.cpp:220-249 (reject > 4096 B, copy the bytes out); on encode it
 * writes the tag and the bytes, which the firmware never does
 * (network.cpp:221 asserts ostream == nullptr).
 */
#include <pb.h>
#include <pb_decode.h>
#include <pb_encode.h>
#include <stdlib.h>
#include <string.h>
#include "ip.pb.h"

#define REF_MAX_ENCODED_FRAME_SIZE 4096 /* network.cpp:24 */

typedef struct {
    const uint8_t *src; /* encode: payload */
    size_t src_len;
    uint8_t *dst;       /* decode: destination */
    size_t dst_cap;
    size_t got;
    int too_large;
} ref_bytes_ctx;

/* nanopb re-initialises the oneof submessage (and its callback arg) before
 * decoding into it, which is why the firmware allocates a fresh context in the
 * callback (network.cpp:228-245); the decode side here uses this pointer. */
static ref_bytes_ctx *g_decode_ctx;

bool network_pb_callback_audio_data(pb_istream_t *istream,
                                    pb_ostream_t *ostream,
                                    const pb_field_t *field)
{
    if (field->tag != AudioData_opus_encoded_frame_tag)
        return pb_default_field_callback(istream, ostream, field);
    if (ostream != NULL) {
        ref_bytes_ctx *ctx = (ref_bytes_ctx *)((pb_callback_t *)field->pData)->arg;
        if (!pb_encode_tag_for_field(ostream, field)) return false;
        return pb_encode_string(ostream, ctx->src, ctx->src_len);
    }
    ref_bytes_ctx *ctx = g_decode_ctx;
    if (istream->bytes_left > REF_MAX_ENCODED_FRAME_SIZE) {
        ctx->too_large = 1;
        istream->errmsg = "Encoded frame exceeds max size";
        return false;
    }
    if (istream->bytes_left > ctx->dst_cap) return false;
    ctx->got = istream->bytes_left;
    return pb_read(istream, ctx->dst, istream->bytes_left);
}

/* returns bytes written, or -1 */
int ref_encode_to_receiver(const uint8_t *payload, size_t len, uint8_t *out,
                           size_t cap)
{
    ref_bytes_ctx ctx = {payload, len, NULL, 0, 0, 0};
    ToReceiver msg = ToReceiver_init_zero;
    msg.which_message = ToReceiver_audio_data_tag;
    msg.message.audio_data.opus_encoded_frame.arg = &ctx;
    pb_ostream_t os = pb_ostream_from_buffer(out, cap);
    if (!pb_encode_delimited(&os, ToReceiver_fields, &msg)) return -1;
    return (int)os.bytes_written;
}

/* returns 0 ok, -1 decode error, -10 payload too large.
 * *consumed = frame bytes read. */
int ref_decode_to_receiver(const uint8_t *in, size_t len, uint8_t *payload,
                           size_t cap, size_t *payload_len, size_t *consumed)
{
    ref_bytes_ctx ctx = {NULL, 0, payload, cap, 0, 0};
    ToReceiver msg = ToReceiver_init_zero;
    g_decode_ctx = &ctx;
    pb_istream_t is = pb_istream_from_buffer(in, len);
    bool ok = pb_decode_delimited(&is, ToReceiver_fields, &msg);
    g_decode_ctx = NULL;
    *consumed = len - is.bytes_left;
    *payload_len = ctx.got;
    if (!ok) return ctx.too_large ? -10 : -1;
    if (msg.which_message != ToReceiver_audio_data_tag) return -1;
    return 0;
}

/* ---- session messages (BroadcastMessage, ToTransmitter), reference codec --
 * Flat view of DiscoveryResponse (ip.pb.h:17-24) for ctypes. */
typedef struct {
    uint32_t protocol_version;
    uint64_t mac_address;
    char device_name[128];
    int32_t currently_streaming;
    char opus_version[128];
} ref_disc;

static void disc_to_pb(const ref_disc *d, DiscoveryResponse *p)
{
    p->protocol_version = d->protocol_version;
    p->mac_address = d->mac_address;
    memcpy(p->device_name, d->device_name, sizeof p->device_name);
    p->currently_streaming = d->currently_streaming != 0;
    memcpy(p->opus_version, d->opus_version, sizeof p->opus_version);
}

static void disc_from_pb(const DiscoveryResponse *p, ref_disc *d)
{
    d->protocol_version = p->protocol_version;
    d->mac_address = p->mac_address;
    memcpy(d->device_name, p->device_name, sizeof d->device_name);
    d->currently_streaming = p->currently_streaming;
    memcpy(d->opus_version, p->opus_version, sizeof d->opus_version);
}

/* which: 0 none, 2 discovery_request (= req), 3 discovery_response (= *d).
 * pb_encode as network.cpp:486-492. Returns bytes or -1. */
int ref_encode_broadcast(int which, uint32_t magic, int req, const ref_disc *d, uint8_t *out,
                         size_t cap)
{
    BroadcastMessage m = BroadcastMessage_init_zero;
    m.magic_word = magic;
    m.which_message = (pb_size_t)which;
    if (which == BroadcastMessage_discovery_request_tag) m.message.discovery_request = req != 0;
    if (which == BroadcastMessage_discovery_response_tag) disc_to_pb(d, &m.message.discovery_response);
    pb_ostream_t os = pb_ostream_from_buffer(out, cap);
    if (!pb_encode(&os, BroadcastMessage_fields, &m)) return -1;
    return (int)os.bytes_written;
}

/* pb_decode of one datagram (network.cpp:473-478). Returns 0 / -1. */
int ref_decode_broadcast(const uint8_t *in, size_t len, uint32_t *magic, int32_t *which,
                         ref_disc *d)
{
    BroadcastMessage m = BroadcastMessage_init_zero;
    pb_istream_t is = pb_istream_from_buffer(in, len);
    if (!pb_decode(&is, BroadcastMessage_fields, &m)) return -1;
    *magic = m.magic_word;
    *which = m.which_message;
    if (m.which_message == BroadcastMessage_discovery_response_tag)
        disc_from_pb(&m.message.discovery_response, d);
    return 0;
}

/* which: 0 none, 1 receiver_information, 2 error; pb_encode_delimited as
 * network.cpp:388-403. Returns bytes or -1. */
int ref_encode_to_transmitter(int which, const ref_disc *d, uint32_t max_enc, uint32_t max_dec,
                              int underflow, int decode_error, uint8_t *out, size_t cap)
{
    ToTransmitter m = ToTransmitter_init_zero;
    m.which_message = (pb_size_t)which;
    if (which == ToTransmitter_receiver_information_tag) {
        disc_to_pb(d, &m.message.receiver_information.discovery_data);
        m.message.receiver_information.max_encoded_frame_size = max_enc;
        m.message.receiver_information.max_decoded_frame_size = max_dec;
    } else if (which == ToTransmitter_error_tag) {
        m.message.error.audio_underflow = underflow != 0;
        m.message.error.audio_decode_error = decode_error != 0;
    }
    pb_ostream_t os = pb_ostream_from_buffer(out, cap);
    if (!pb_encode_delimited(&os, ToTransmitter_fields, &m)) return -1;
    return (int)os.bytes_written;
}

/* pb_decode_delimited of one ToTransmitter. Returns 0 / -1. */
int ref_decode_to_transmitter(const uint8_t *in, size_t len, int32_t *which, ref_disc *d,
                              uint32_t *max_enc, uint32_t *max_dec, int32_t *underflow,
                              int32_t *decode_error, size_t *consumed)
{
    ToTransmitter m = ToTransmitter_init_zero;
    pb_istream_t is = pb_istream_from_buffer(in, len);
    bool ok = pb_decode_delimited(&is, ToTransmitter_fields, &m);
    *consumed = len - is.bytes_left;
    if (!ok) return -1;
    *which = m.which_message;
    if (m.which_message == ToTransmitter_receiver_information_tag) {
        disc_from_pb(&m.message.receiver_information.discovery_data, d);
        *max_enc = m.message.receiver_information.max_encoded_frame_size;
        *max_dec = m.message.receiver_information.max_decoded_frame_size;
    } else if (m.which_message == ToTransmitter_error_tag) {
        *underflow = m.message.error.audio_underflow;
        *decode_error = m.message.error.audio_decode_error;
    }
    return 0;
}
