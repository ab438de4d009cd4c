/*
 * fskrx.c — C host receiver over the C ABI (include/demod.h): raw int16
 * little-endian PCM on stdin (as opus_decode would hand it to the playback
 * task, hardware/src/playback.cpp:115-131) -> decoded symbols -> delimited
 * ip.proto ToReceiver{AudioData} frames on stdout (the framing the reference
 * receiver reads, network.cpp:409-430, and the transmitter writes,
 * protobuf_async.kt:110-114).
 *
 *   fskrx [-c 1|2] [-m left|right|downmix] [-f f1,f2,...] [-n N] [-H hop]
 *         [-M auto|goertzel|folded|fft] [-p frames_per_read] [-b] < pcm > frames
 *
 * Default: 48 kHz mono, N = hop = 1024, 2-FSK at 1500/3000 Hz, reads of 2880
 * frames (one 60 ms packet) each passed to demodulate(). -b reads all input
 * first and makes one demodulate() call (the chunked host-buffer path).
 * Symbols are framed MSB-first, ceil(log2 K) bits each, 4096-byte payloads;
 * the final partial payload is flushed at EOF. Statistics go to stderr.
 * Exit status: 0 ok, 2 usage, 3 demod_create failed (e.g. no gfx950 device:
 * there is no CPU fallback), 4 demodulation / framing error, 5 I/O error.
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../include/demod.h"

static int usage(void)
{
    fprintf(stderr, "usage: fskrx [-c 1|2] [-m left|right|downmix] [-f f1,f2,...] [-n N] "
                    "[-H hop] [-M auto|goertzel|folded|residue|fft] [-p frames] [-b] < pcm > frames\n");
    return 2;
}

/* symbol accumulator: frames whole payloads as soon as they fill */
struct sink {
    uint8_t *sym;
    size_t n, cap, per;
    int bits;
    uint8_t *frame;
    size_t frame_cap;
    unsigned long long frames, bytes, symbols;
};

static int sink_emit(struct sink *s, size_t cnt)
{
    long long w = demod_frame_symbols(s->sym, cnt, s->bits, DEMOD_MAX_FRAME_PAYLOAD, s->frame,
                                      s->frame_cap);
    if (w < 0) {
        fprintf(stderr, "fskrx: framing: %s\n", demod_strerror((int)w));
        return 4;
    }
    if (fwrite(s->frame, 1, (size_t)w, stdout) != (size_t)w) return 5;
    s->frames += (cnt + s->per - 1) / s->per;
    s->bytes += (unsigned long long)w;
    memmove(s->sym, s->sym + cnt, s->n - cnt);
    s->n -= cnt;
    return 0;
}

static int sink_push(struct sink *s, const uint8_t *sym, size_t n)
{
    if (s->n + n > s->cap) {
        size_t cap = (s->n + n) * 2;
        uint8_t *p = realloc(s->sym, cap);
        if (!p) return 4;
        s->sym = p;
        s->cap = cap;
    }
    memcpy(s->sym + s->n, sym, n);
    s->n += n;
    s->symbols += n;
    if (s->n >= s->per) return sink_emit(s, s->n - s->n % s->per);
    return 0;
}

int main(int argc, char **argv)
{
    demod_cfg_t cfg;
    demod_cfg_default(&cfg);
    size_t per_read = 2880; /* one 60 ms packet at 48 kHz (playback.cpp:10) */
    int batch = 0;
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
        if (!strcmp(a, "-b")) { batch = 1; continue; }
        if (!v) return usage();
        ++i;
        if (!strcmp(a, "-c")) cfg.channels = (uint32_t)atoi(v);
        else if (!strcmp(a, "-n")) cfg.n = (uint32_t)atoi(v);
        else if (!strcmp(a, "-H")) cfg.hop = (uint32_t)atoi(v);
        else if (!strcmp(a, "-p")) per_read = (size_t)strtoull(v, NULL, 10);
        else if (!strcmp(a, "-m")) {
            if (!strcmp(v, "left")) cfg.channel_mode = DEMOD_CH_LEFT;
            else if (!strcmp(v, "right")) cfg.channel_mode = DEMOD_CH_RIGHT;
            else if (!strcmp(v, "downmix")) cfg.channel_mode = DEMOD_CH_DOWNMIX;
            else return usage();
        } else if (!strcmp(a, "-M")) {
            if (!strcmp(v, "auto")) cfg.method = DEMOD_METHOD_AUTO;
            else if (!strcmp(v, "goertzel")) cfg.method = DEMOD_METHOD_GOERTZEL;
            else if (!strcmp(v, "folded")) cfg.method = DEMOD_METHOD_FOLDED;
            else if (!strcmp(v, "residue")) cfg.method = DEMOD_METHOD_RESIDUE;
            else if (!strcmp(v, "fft")) cfg.method = DEMOD_METHOD_FFT;
            else return usage();
        } else if (!strcmp(a, "-f")) {
            uint32_t k = 0;
            char *end = (char *)v;
            while (*end && k < DEMOD_MAX_TONES) {
                cfg.freqs[k++] = strtod(end, &end);
                if (*end == ',') ++end;
                else if (*end) return usage();
            }
            if (*end || k == 0) return usage();
            cfg.k = k;
        } else {
            return usage();
        }
    }
    if (per_read == 0) return usage();

    int err = 0;
    demod_t *st = demod_create(&cfg, &err);
    if (!st) {
        fprintf(stderr, "fskrx: demod_create: %s\n", demod_strerror(err));
        return 3;
    }
    struct sink s;
    memset(&s, 0, sizeof s);
    s.bits = demod_bits_per_symbol(cfg.k);
    s.per = (size_t)DEMOD_MAX_FRAME_PAYLOAD * 8 / (size_t)s.bits;
    s.frame_cap = demod_frame_size(DEMOD_MAX_FRAME_PAYLOAD) * 2 + 64;
    s.frame = malloc(s.frame_cap);
    int rc = s.frame ? 0 : 4;

    const size_t ch = cfg.channels;
    size_t cap = batch ? ((size_t)1 << 20) : per_read;
    int16_t *pcm = malloc(cap * ch * sizeof(int16_t));
    uint8_t *sym = NULL;
    size_t sym_cap = 0;
    size_t have = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    unsigned long long frames_in = 0;
    while (!rc && pcm) {
        size_t got = fread(pcm + have * ch, sizeof(int16_t) * ch, cap - have, stdin);
        have += got;
        int eof = got == 0 || feof(stdin);
        if (ferror(stdin)) { rc = 5; break; }
        if (batch && !eof) {
            if (have == cap) {
                int16_t *p = realloc(pcm, cap * 2 * ch * sizeof(int16_t));
                if (!p) { rc = 4; break; }
                pcm = p;
                cap *= 2;
            }
            continue;
        }
        if (have) {
            int need = demod_max_symbols(st, have);
            if (need < 0) { rc = 4; break; }
            if ((size_t)need > sym_cap) {
                uint8_t *p = realloc(sym, (size_t)need + 16);
                if (!p) { rc = 4; break; }
                sym = p;
                sym_cap = (size_t)need + 16;
            }
            int ns = demodulate(st, pcm, have, sym, sym_cap);
            if (ns < 0) {
                fprintf(stderr, "fskrx: demodulate: %s\n", demod_strerror(ns));
                rc = 4;
                break;
            }
            frames_in += have;
            have = 0;
            if ((rc = sink_push(&s, sym, (size_t)ns)) != 0) break;
        }
        if (eof) break;
    }
    if (!rc && s.n) rc = sink_emit(&s, s.n);
    if (!rc && fflush(stdout) != 0) rc = 5;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double el = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    fprintf(stderr,
            "fskrx: %llu frames in (%.3f s of audio), %llu symbols, %llu ToReceiver frames "
            "(%llu bytes), %d samples pending, %.3f s wall (%.1f Msamples/s)\n",
            frames_in, (double)frames_in / cfg.fs, s.symbols, s.frames, s.bytes,
            demod_pending(st), el, el > 0 ? (double)frames_in / el / 1e6 : 0.0);
    free(sym);
    free(pcm);
    free(s.sym);
    free(s.frame);
    demod_destroy(st);
    return rc;
}
