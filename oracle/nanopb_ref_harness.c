/*
 * nanopb_ref_harness.c — TEST INFRASTRUCTURE ONLY.
 *
 * Links the reference's own nanopb 0.4.5 runtime and its generated ip.pb.c
 * (compiled in place from /root/reference by oracle/ref.mk, output only into
 * oracle/_ref/) so tests can mint and check ToReceiver frame bytes with the
 * reference's codec.
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
