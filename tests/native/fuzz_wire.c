/*
 * fuzz_wire.c — the ABI's byte codecs under AddressSanitizer + UBSan (host
 * code only; no GPU). These parse what arrives from the network (fskrx -l/-u:
 * ToReceiver frames on TCP 58764, BroadcastMessage datagrams on UDP 58765),
 * so every decoder runs here on exact-size heap buffers, where any read past
 * the input is a sanitizer abort:
 *   - ToReceiver frames: encode/decode round trips at every payload size
 *     0..4200, truncations of every valid frame, random byte and varint
 *     mutations, pure random bytes; a decoded payload must lie inside the
 *     frame it came from;
 *   - symbol packing: pack/unpack round trips for bits 1..8, framed symbol
 *     streams decoded frame by frame;
 *   - session messages: discovery response and hello round trips with random
 *     strings, mutated and random datagrams through both decoders.
 * Built by tests/native/Makefile (target fuzz_wire) from the product sources
 * csrc/demod_frame.c and csrc/demod_session.c; run by tests/test_native.py.
 * Exit code 0 = pass.  Usage: fuzz_wire [iterations] [seed]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/demod.h"

static uint64_t rng_state;

static uint64_t next(void)
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static size_t below(size_t n) { return n ? (size_t)(next() % n) : 0; }

#define CHECK(c, ...)                                                 \
    do {                                                              \
        if (!(c)) {                                                   \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);     \
            fprintf(stderr, __VA_ARGS__);                             \
            fprintf(stderr, "\n");                                    \
            exit(1);                                                  \
        }                                                             \
    } while (0)

/* exact-size heap copy, so the sanitizer sees any read past len */
static uint8_t *dup_exact(const uint8_t *p, size_t len)
{
    uint8_t *q = malloc(len ? len : 1);
    CHECK(q != NULL, "malloc");
    if (len) memcpy(q, p, len);
    return q;
}

static long decoded_ok, rejected;

/* decode in[0..len) (an exact-size copy); a successful decode must point
 * inside the frame */
static int decode_checked(const uint8_t *src, size_t len)
{
    uint8_t *in = dup_exact(src, len);
    const uint8_t *pl = NULL;
    size_t pl_len = 0, used = 0;
    int rc = demod_frame_decode(in, len, &pl, &pl_len, &used);
    if (rc == DEMOD_OK) {
        CHECK(used >= 1 && used <= len, "consumed %zu of %zu", used, len);
        CHECK(pl_len <= DEMOD_MAX_FRAME_PAYLOAD, "payload %zu", pl_len);
        CHECK(pl_len == 0 || (pl >= in && pl + pl_len <= in + used), "payload outside the frame");
        volatile uint8_t s = 0;
        for (size_t i = 0; i < pl_len; ++i) s ^= pl[i];  /* touch every byte */
        (void)s;
        ++decoded_ok;
    } else {
        CHECK(rc == DEMOD_BUFFER_TOO_SMALL || rc == DEMOD_INVALID_PACKET ||
                  rc == DEMOD_FRAME_TOO_LARGE,
              "unexpected code %d", rc);
        ++rejected;
    }
    free(in);
    return rc;
}

static void fuzz_frames(long iters)
{
    uint8_t payload[4300], frame[4400];
    for (size_t len = 0; len <= 4200; ++len) {  /* every size, round trip */
        for (size_t i = 0; i < len; ++i) payload[i] = (uint8_t)next();
        const size_t need = demod_frame_size(len);
        uint8_t *out = malloc(need);
        CHECK(out != NULL, "malloc");
        int n = demod_frame_encode(payload, len, out, need);
        if (len > DEMOD_MAX_FRAME_PAYLOAD) {
            CHECK(n == DEMOD_FRAME_TOO_LARGE, "len %zu -> %d", len, n);
            free(out);
            continue;
        }
        CHECK(n == (int)need, "encode %zu -> %d (need %zu)", len, n, need);
        CHECK(demod_frame_encode(payload, len, out, need - 1) == DEMOD_BUFFER_TOO_SMALL,
              "short cap");
        const uint8_t *pl;
        size_t pl_len, used;
        CHECK(demod_frame_decode(out, need, &pl, &pl_len, &used) == DEMOD_OK, "decode %zu", len);
        CHECK(pl_len == len && used == need && memcmp(pl, payload, len) == 0, "round trip %zu", len);
        /* every truncation of the frame asks for more bytes */
        for (size_t cut = 0; cut < need; cut += 1 + (need > 64 ? below(need / 16) : 0))
            CHECK(decode_checked(out, cut) == DEMOD_BUFFER_TOO_SMALL, "truncated %zu/%zu", cut, need);
        free(out);
    }
    for (long it = 0; it < iters; ++it) {
        const size_t len = below(64) < 60 ? below(40) : below(4097);
        for (size_t i = 0; i < len; ++i) payload[i] = (uint8_t)next();
        int n = demod_frame_encode(payload, len, frame, sizeof frame);
        CHECK(n > 0, "encode");
        /* mutate: flip bytes, overwrite with varint-ish values, splice */
        const int muts = 1 + (int)below(4);
        for (int m = 0; m < muts; ++m) {
            const size_t at = below((size_t)n);
            switch (below(4)) {
            case 0: frame[at] ^= (uint8_t)(1u << below(8)); break;
            case 1: frame[at] = (uint8_t)next(); break;
            case 2: frame[at] = 0x80 | (uint8_t)next(); break;  /* continuation bit */
            default: frame[at] = (uint8_t)(below(8) << 3 | below(8)); break;  /* a tag */
            }
        }
        size_t fed = (size_t)n;
        if (below(4) == 0) fed = below((size_t)n + 1);
        if (below(8) == 0 && fed + 8 <= sizeof frame) {  /* trailing garbage */
            for (int i = 0; i < 8; ++i) frame[fed + i] = (uint8_t)next();
            fed += 8;
        }
        decode_checked(frame, fed);
        /* pure random bytes */
        const size_t rl = below(48);
        for (size_t i = 0; i < rl; ++i) frame[i] = (uint8_t)next();
        decode_checked(frame, rl);
    }
}

static void fuzz_symbols(long iters)
{
    static uint8_t sym[20000], back[20000], packed[20000];
    for (long it = 0; it < iters; ++it) {
        const int bits = 1 + (int)below(8);
        const size_t n = below(it % 16 == 0 ? 20000 : 300);
        for (size_t i = 0; i < n; ++i) sym[i] = (uint8_t)(next() & ((1u << bits) - 1));
        const size_t need = (n * (size_t)bits + 7) / 8;
        uint8_t *p = malloc(need ? need : 1);
        CHECK(p != NULL, "malloc");
        CHECK(demod_pack_symbols(sym, n, bits, p, need) == (int)need, "pack");
        if (need) CHECK(demod_pack_symbols(sym, n, bits, p, need - 1) < 0, "pack short cap");
        CHECK(demod_unpack_symbols(p, n, bits, back, n) == (int)n, "unpack");
        CHECK(memcmp(sym, back, n) == 0, "pack round trip bits %d n %zu", bits, n);
        if (n) CHECK(demod_unpack_symbols(p, n, bits, back, n - 1) < 0, "unpack short cap");
        free(p);
        /* framed stream: decode frame by frame, unpack, compare */
        const size_t maxp = 1 + below(it % 4 == 0 ? DEMOD_MAX_FRAME_PAYLOAD : 64);
        const size_t per = maxp * 8 / (size_t)bits;
        if (per == 0) continue;
        const size_t cap = (n / per + 1) * demod_frame_size(maxp);
        uint8_t *fr = malloc(cap);
        CHECK(fr != NULL, "malloc");
        long long w = demod_frame_symbols(sym, n, bits, maxp, fr, cap);
        CHECK(w >= 0 && (size_t)w <= cap, "frame_symbols %lld", w);
        uint8_t *exact = dup_exact(fr, (size_t)w);
        size_t pos = 0, got = 0;
        while (pos < (size_t)w) {
            const uint8_t *pl;
            size_t pl_len, used;
            CHECK(demod_frame_decode(exact + pos, (size_t)w - pos, &pl, &pl_len, &used) == DEMOD_OK,
                  "framed decode");
            const size_t cnt = n - got < per ? n - got : per;
            CHECK(pl_len == (cnt * (size_t)bits + 7) / 8, "payload size");
            memcpy(packed, pl, pl_len);
            CHECK(demod_unpack_symbols(packed, cnt, bits, back + got, cnt) == (int)cnt, "unpack");
            got += cnt;
            pos += used;
        }
        CHECK(got == n && memcmp(sym, back, n) == 0, "framed round trip");
        free(exact);
        free(fr);
    }
}

static void rand_string(char *s, size_t cap)
{
    const size_t len = below(cap);  /* <= cap - 1, NUL-terminated */
    for (size_t i = 0; i < len; ++i) s[i] = (char)(1 + below(255));
    s[len] = 0;
}

static void fuzz_session(long iters)
{
    uint8_t buf[1024];
    for (long it = 0; it < iters; ++it) {
        demod_discovery_t d, d2;
        memset(&d, 0, sizeof d);
        d.protocol_version = (uint32_t)next();
        d.mac_address = next() & 0xFFFFFFFFFFFFull;
        d.currently_streaming = (int)below(2);
        rand_string(d.device_name, sizeof d.device_name);
        rand_string(d.opus_version, sizeof d.opus_version);
        int n = demod_broadcast_response_encode(&d, buf, sizeof buf);
        CHECK(n > 0, "broadcast response encode %d", n);
        uint8_t *in = dup_exact(buf, (size_t)n);
        uint32_t magic = 0;
        memset(&d2, 0xA5, sizeof d2);
        CHECK(demod_broadcast_decode(in, (size_t)n, &magic, &d2) == DEMOD_MSG_DISCOVERY_RESPONSE,
              "broadcast decode");
        CHECK(magic == DEMOD_BROADCAST_MAGIC && d2.protocol_version == d.protocol_version &&
                  d2.mac_address == d.mac_address && !strcmp(d2.device_name, d.device_name) &&
                  !strcmp(d2.opus_version, d.opus_version) &&
                  !!d2.currently_streaming == !!d.currently_streaming,
              "broadcast round trip");
        free(in);
        demod_receiver_info_t info, info2;
        memset(&info, 0, sizeof info);
        info.discovery_data = d;
        info.max_encoded_frame_size = (uint32_t)next();
        info.max_decoded_frame_size = (uint32_t)next();
        n = demod_hello_encode(&info, buf, sizeof buf);
        CHECK(n > 0, "hello encode");
        in = dup_exact(buf, (size_t)n);
        size_t used = 0;
        CHECK(demod_to_transmitter_decode(in, (size_t)n, &info2, NULL, &used) ==
                  DEMOD_MSG_RECEIVER_INFORMATION && used == (size_t)n,
              "hello decode");
        CHECK(info2.max_encoded_frame_size == info.max_encoded_frame_size &&
                  info2.max_decoded_frame_size == info.max_decoded_frame_size &&
                  !strcmp(info2.discovery_data.device_name, d.device_name),
              "hello round trip");
        free(in);
        /* mutated and truncated copies, and random datagrams, through both */
        for (int m = 0, muts = 1 + (int)below(4); m < muts; ++m)
            buf[below((size_t)n)] ^= (uint8_t)(1u << below(8));
        const size_t fed = below(3) ? (size_t)n : below((size_t)n + 1);
        for (int pass = 0; pass < 2; ++pass) {
            size_t len = fed;
            if (pass) {
                len = below(96);
                for (size_t i = 0; i < len; ++i) buf[i] = (uint8_t)next();
            }
            in = dup_exact(buf, len);
            int r1 = demod_broadcast_decode(in, len, &magic, &d2);
            CHECK(r1 == DEMOD_MSG_NONE || r1 == DEMOD_MSG_DISCOVERY_REQUEST ||
                      r1 == DEMOD_MSG_DISCOVERY_RESPONSE || r1 == DEMOD_INVALID_PACKET,
                  "broadcast verdict %d", r1);
            if (r1 == DEMOD_MSG_DISCOVERY_RESPONSE)
                CHECK(memchr(d2.device_name, 0, sizeof d2.device_name) &&
                          memchr(d2.opus_version, 0, sizeof d2.opus_version),
                      "unterminated string");
            demod_receiver_error_t e;
            int r2 = demod_to_transmitter_decode(in, len, &info2, &e, &used);
            CHECK(r2 == DEMOD_MSG_NONE || r2 == DEMOD_MSG_RECEIVER_INFORMATION ||
                      r2 == DEMOD_MSG_RECEIVER_ERROR || r2 == DEMOD_INVALID_PACKET ||
                      r2 == DEMOD_BUFFER_TOO_SMALL,
                  "to_transmitter verdict %d", r2);
            if (r2 >= 0) CHECK(used <= len, "consumed %zu of %zu", used, len);
            free(in);
        }
    }
}

int main(int argc, char **argv)
{
    const long iters = argc > 1 ? atol(argv[1]) : 100000;
    rng_state = argc > 2 ? strtoull(argv[2], NULL, 0) : 1;
    fuzz_frames(iters);
    fuzz_symbols(iters / 20);
    fuzz_session(iters / 4);
    printf("fuzz_wire OK: %ld iterations, %ld frames decoded, %ld rejected\n", iters, decoded_ok,
           rejected);
    return 0;
}
