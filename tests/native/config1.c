/*
 * config1.c — BASELINE.json configs[0]: 2-FSK Goertzel on ONE 1024-sample
 * 48 kHz int16 buffer, native host build, no GPU required (plumbing test; the
 * role hardware/test/network.cpp plays for the reference firmware: a small C
 * program with an exit code).
 *
 * Links the C ABI (libfskdemod.so) and the test oracle (liboracle.so):
 *   1. the oracle generator makes one window with a known symbol;
 *   2. the oracle Goertzel must decide that symbol;
 *   3. demod_create: on a host without a gfx950 device it must fail loudly
 *      with DEMOD_NO_DEVICE (no CPU fallback); with a GPU, demodulate() must
 *      return the same symbol, fed in 60 ms stereo packets;
 *   4. the symbol stream is framed as ip.proto ToReceiver messages and read
 *      back with demod_frame_decode.
 * Exit code 0 = pass.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/demod.h"
#include "../../oracle/fsk_oracle.h"

#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);              \
            fprintf(stderr, "\n");                     \
            return 1;                                  \
        }                                              \
    } while (0)

int main(void)
{
    const double freqs[2] = {1500.0, 3000.0};
    int16_t pcm[1024];
    uint8_t truth, sym;
    double P[2];
    for (uint64_t seed = 1; seed <= 8; ++seed) {
        oracle_synth_fsk(48000.0, 1024, 2, freqs, seed, 0, 1, 8000, 400, pcm, &truth);
        oracle_goertzel(pcm, 1, 1024, 1024, 2, freqs, 48000.0, &sym, P);
        CHECK(sym == truth, "oracle symbol %d != transmitted %d (seed %llu)", sym, truth,
              (unsigned long long)seed);
        CHECK(P[truth] > 100.0 * P[1 - truth], "weak decision margin");
    }

    demod_cfg_t cfg;
    demod_cfg_default(&cfg);
    CHECK(cfg.n == 1024 && cfg.k == 2 && cfg.freqs[1] == 3000.0, "defaults");
    cfg.channels = 2;  /* as decoded by opus_decoder_create(48000, 2) */
    int err = 0;
    demod_t *st = demod_create(&cfg, &err);
    if (!st) {
        CHECK(err == DEMOD_NO_DEVICE, "create failed with %d (%s)", err, demod_strerror(err));
        printf("no gfx950 device: demod_create -> %s (expected on a CPU host)\n",
               demod_strerror(err));
    } else {
        /* stereo interleaved, the window on both channels, 60 ms packets */
        static int16_t stereo[2 * 2880];
        memset(stereo, 0, sizeof stereo);
        for (int i = 0; i < 1024; ++i) stereo[2 * i] = stereo[2 * i + 1] = pcm[i];
        uint8_t out[4];
        int n = demodulate(st, stereo, 2880, out, sizeof out);
        CHECK(n == 2, "demodulate returned %d", n);
        CHECK(out[0] == truth, "gpu symbol %d != %d", out[0], truth);
        CHECK(demod_pending(st) == 2880 - 2048, "carry %d", demod_pending(st));
        demod_destroy(st);
        printf("gpu demodulate: symbol %d OK\n", out[0]);

        /* the same packet on three streams at once (one batch), the middle
         * stream silent this round */
        demod_streams_t *ms = demod_streams_create(&cfg, 3, &err);
        CHECK(ms != NULL, "demod_streams_create: %s", demod_strerror(err));
        const int16_t *pk[3] = {stereo, NULL, stereo};
        const size_t nf[3] = {2880, 0, 2880};
        uint8_t all[8];
        uint32_t counts[3];
        CHECK(demod_streams_max_symbols(ms, nf) == 4, "streams bound");
        n = demod_streams_push(ms, pk, nf, all, NULL, sizeof all, counts);
        CHECK(n == 4 && counts[0] == 2 && counts[1] == 0 && counts[2] == 2, "streams push %d", n);
        CHECK(all[0] == truth && all[2] == truth, "streams symbols %d %d", all[0], all[2]);
        CHECK(demod_streams_pending(ms, 0) == 2880 - 2048 && demod_streams_pending(ms, 1) == 0,
              "streams carry");
        demod_streams_destroy(ms);
        printf("gpu demod_streams_push: 3 streams OK\n");
    }

    /* framing: 100 symbols -> ToReceiver frames -> back */
    uint8_t syms[100], back[100], frames[256];
    for (int i = 0; i < 100; ++i) syms[i] = (uint8_t)((i * 7) & 1);
    long long nb = demod_frame_symbols(syms, 100, 1, 4096, frames, sizeof frames);
    CHECK(nb > 0, "frame_symbols %lld", nb);
    const uint8_t *pl;
    size_t pl_len, used;
    CHECK(demod_frame_decode(frames, (size_t)nb, &pl, &pl_len, &used) == DEMOD_OK, "decode");
    CHECK(used == (size_t)nb && pl_len == 13, "frame sizes %zu %zu", used, pl_len);
    CHECK(demod_unpack_symbols(pl, 100, 1, back, 100) == 100, "unpack");
    CHECK(memcmp(syms, back, 100) == 0, "symbol round trip");
    printf("config1 OK (symbol %d, frame %lld bytes)\n", truth, nb);
    return 0;
}
