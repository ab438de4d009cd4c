/*
 * fskrx.c — C host receiver over the C ABI (include/demod.h): raw int16
 * little-endian PCM on stdin (as opus_decode would hand it to the playback
 * task, hardware/src/playback.cpp:115-131) -> decoded symbols -> delimited
 * ip.proto ToReceiver{AudioData} frames on stdout (the framing the reference
 * receiver reads, network.cpp:409-430, and the transmitter writes,
 * protobuf_async.kt:110-114).
 *
 *   fskrx [-c 1|2] [-m left|right|downmix] [-f f1,f2,...] [-n N] [-H hop]
 *         [-M auto|goertzel|folded|fft] [-L lead_in] [-p frames_per_read] [-b] < pcm > frames
 *   fskrx [same options] -l tcp_port -r [-u udp_port] [-a addr] [-N name] [-1] > frames
 *   fskrx [same options] -g gpus [-S streams] -o prefix < interleaved pcm
 *
 * Default: 48 kHz mono, N = hop = 1024, 2-FSK at 1500/3000 Hz, reads of 2880
 * frames (one 60 ms packet) each passed to demodulate(). -b reads all input
 * first and makes one demodulate() call (the chunked host-buffer path).
 * -L drops the stream's first lead_in frames (demod_cfg_t.lead_in, e.g. 312
 * for PCM that came out of an Opus decoder, DEMOD_OPUS_LOOKAHEAD).
 * Symbols are framed MSB-first, ceil(log2 K) bits each, 4096-byte payloads
 * (one demod_frame_symbols call per payload); the final partial payload is
 * flushed at EOF. Statistics go to stderr.
 * Exit status: 0 ok, 2 usage, 3 demod_create failed (e.g. no gfx950 device:
 * there is no CPU fallback), 4 demodulation / framing error, 5 I/O error.
 *
 * Group mode (-g, configs[4] from the C host): S streams
 * (-S, default the number of GPUs) demodulated over the first `gpus` GPUs of
 * this process as one RCCL group (demod_group_create_local: the streams
 * sharded over the GPUs, each GPU's symbols all-gathered over RCCL,
 * demod_group_push). stdin carries the streams packet-interleaved: per
 * round, one packet of -p frames of stream 0, then stream 1, ...; a short
 * final round is dealt to the streams in order. Stream s's ToReceiver frames
 * go to <prefix><s>.bin, byte-identical to fskrx run on that stream alone.
 *
 * Network mode (-l) takes the receiver's place on the
 * wire instead of stdin: it listens on TCP (58764 in the reference,
 * network.cpp:496-516; 0 = any free port), writes the ToTransmitter hello to
 * each transmitter that connects (network.cpp:380-403), resets the stream
 * (playback_start_new_stream, network.cpp:406-407) and reads delimited
 * ToReceiver frames until the transmitter closes or sends a frame nanopb
 * would reject (network.cpp:409-430). One transmitter at a time, like the
 * firmware. With -u it also answers UDP discovery requests
 * (network.cpp:449-494). In the reference the AudioData bytes are an Opus
 * packet (MulticastAudioOutput.kt:124-130); Opus decoding is outside this
 * build (the reference libopus needs an ESP32 header this image lacks,
 * DESIGN.md §8), so a transmitter can only feed raw int16 LE PCM of the
 * configured channel layout through the same frame layout, and only when -r
 * says so. Without -r the first AudioData frame is refused — ToTransmitter
 * {error{audio_decode_error}} (ip.proto:56-61), then the connection is
 * closed — instead of demodulating Opus bytes as noise. With -r a payload
 * that is not a whole number of PCM frames (an Opus packet, or a torn
 * sample) is refused the same way (reported as DEMOD_BAD_ARG). A refused
 * stream makes the exit status 4. -1 exits after the first transmitter
 * disconnects. The bound ports are printed on stderr as
 * "fskrx: listening tcp <port> udp <port>".
 */
#define _POSIX_C_SOURCE 200112L
#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <poll.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <time.h>
#include <unistd.h>

#include "../../include/demod.h"

static int usage(void)
{
    fprintf(stderr, "usage: fskrx [-c 1|2] [-m left|right|downmix] [-f f1,f2,...] [-n N] "
                    "[-H hop] [-M auto|goertzel|folded|residue|fft] [-L lead_in] [-p frames] [-b] "
                    "< pcm > frames\n"
                    "       fskrx [options] -l tcp_port -r [-u udp_port] [-a addr] [-N name] [-1] "
                    "> frames\n"
                    "       fskrx [options] -g gpus [-S streams] -o prefix < interleaved pcm\n"
                    "  -r: AudioData payloads are raw int16 PCM (this receiver does not decode "
                    "Opus; without -r audio is refused)\n");
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
    FILE *out; /* NULL: stdout */
};

/* Frame the first cnt buffered symbols, one payload (<= per symbols) per
 * demod_frame_symbols call, so s->frame only ever holds one frame. */
static int sink_emit(struct sink *s, size_t cnt)
{
    for (size_t at = 0; at < cnt; at += s->per) {
        const size_t c = cnt - at < s->per ? cnt - at : s->per;
        long long w = demod_frame_symbols(s->sym + at, c, s->bits, DEMOD_MAX_FRAME_PAYLOAD,
                                          s->frame, s->frame_cap);
        if (w < 0) {
            fprintf(stderr, "fskrx: framing: %s\n", demod_strerror((int)w));
            return 4;
        }
        if (fwrite(s->frame, 1, (size_t)w, s->out ? s->out : stdout) != (size_t)w) return 5;
        s->frames += 1;
        s->bytes += (unsigned long long)w;
    }
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

/* ---- network mode ------------------------------------------------------ */

struct net {
    const char *addr;
    int tcp_port, udp_port; /* udp_port < 0: no discovery responder */
    const char *name;
    int once;
    int raw_pcm; /* -r: AudioData payloads are raw PCM (else audio is refused) */
};

static int bind_socket(int type, const char *addr, int port, int *bound)
{
    int fd = socket(AF_INET, type, 0);
    if (fd < 0) return -1;
    int one = 1;
    setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
    struct sockaddr_in sa;
    memset(&sa, 0, sizeof sa);
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, addr, &sa.sin_addr) != 1 ||
        bind(fd, (struct sockaddr *)&sa, sizeof sa) != 0 ||
        (type == SOCK_STREAM && listen(fd, 1) != 0)) {
        close(fd);
        return -1;
    }
    socklen_t len = sizeof sa;
    getsockname(fd, (struct sockaddr *)&sa, &len);
    *bound = ntohs(sa.sin_port);
    return fd;
}

static int send_all(int fd, const uint8_t *p, size_t n)
{
    while (n) {
        ssize_t w = send(fd, p, n, MSG_NOSIGNAL);
        if (w < 0 && errno == EINTR) continue;
        if (w <= 0) return -1;
        p += w;
        n -= (size_t)w;
    }
    return 0;
}

/* Demodulate the whole frames of pcm bytes held in buf[0..*len); keeps the
 * bytes of a frame split across payloads for the next call. */
static int feed_pcm(demod_t *st, struct sink *s, uint8_t *buf, size_t *len, size_t frame_bytes,
                    uint8_t **sym, size_t *sym_cap, unsigned long long *frames_in)
{
    size_t nf = *len / frame_bytes;
    if (!nf) return 0;
    int need = demod_max_symbols(st, nf);
    if (need < 0) return 4;
    if ((size_t)need > *sym_cap) {
        uint8_t *p = realloc(*sym, (size_t)need + 16);
        if (!p) return 4;
        *sym = p;
        *sym_cap = (size_t)need + 16;
    }
    int ns = demodulate(st, (const int16_t *)(const void *)buf, nf, *sym, *sym_cap);
    if (ns < 0) {
        fprintf(stderr, "fskrx: demodulate: %s\n", demod_strerror(ns));
        return 4;
    }
    *frames_in += nf;
    memmove(buf, buf + nf * frame_bytes, *len - nf * frame_bytes);
    *len -= nf * frame_bytes;
    return sink_push(s, *sym, (size_t)ns);
}

static int serve(demod_t *st, const demod_cfg_t *cfg, struct sink *s, const struct net *nt,
                 unsigned long long *frames_in)
{
    int tport = 0, uport = -1;
    int lfd = bind_socket(SOCK_STREAM, nt->addr, nt->tcp_port, &tport);
    int ufd = nt->udp_port >= 0 ? bind_socket(SOCK_DGRAM, nt->addr, nt->udp_port, &uport) : -1;
    if (lfd < 0 || (nt->udp_port >= 0 && ufd < 0)) {
        fprintf(stderr, "fskrx: cannot bind %s: %s\n", nt->addr, strerror(errno));
        if (lfd >= 0) close(lfd);
        return 5;
    }
    fprintf(stderr, "fskrx: listening tcp %d udp %d\n", tport, uport);
    fflush(stderr);

    demod_discovery_t disc;
    memset(&disc, 0, sizeof disc);
    disc.protocol_version = 1; /* network.cpp:374 */
    snprintf(disc.device_name, sizeof disc.device_name, "%s", nt->name);
    snprintf(disc.opus_version, sizeof disc.opus_version, "%s", demod_version_string());

    const size_t frame_bytes = sizeof(int16_t) * cfg->channels;
    size_t in_cap = 2 * demod_frame_size(DEMOD_MAX_FRAME_PAYLOAD), in_len = 0;
    size_t pcm_cap = 4 * DEMOD_MAX_FRAME_PAYLOAD, pcm_len = 0;
    uint8_t *in = malloc(in_cap), *pcm = malloc(pcm_cap), *sym = NULL;
    size_t sym_cap = 0;
    int cfd = -1, rc = (in && pcm) ? 0 : 4, done = 0;
    unsigned long long clients = 0, answered = 0, refused = 0;
    while (!rc && !done) {
        struct pollfd pf[2];
        int np = 0;
        pf[np].fd = cfd >= 0 ? cfd : lfd; /* one transmitter at a time */
        pf[np++].events = POLLIN;
        if (ufd >= 0) {
            pf[np].fd = ufd;
            pf[np++].events = POLLIN;
        }
        if (poll(pf, (nfds_t)np, -1) < 0) {
            if (errno == EINTR) continue;
            rc = 5;
            break;
        }
        if (ufd >= 0 && (pf[1].revents & POLLIN)) {
            uint8_t dg[768]; /* protobuf_buffer_len, network.cpp:450 */
            struct sockaddr_storage from;
            socklen_t flen = sizeof from;
            ssize_t n = recvfrom(ufd, dg, sizeof dg, 0, (struct sockaddr *)&from, &flen);
            uint32_t magic = 0;
            if (n >= 0 &&
                demod_broadcast_decode(dg, (size_t)n, &magic, NULL) == DEMOD_MSG_DISCOVERY_REQUEST &&
                magic == DEMOD_BROADCAST_MAGIC) {
                disc.currently_streaming = cfd >= 0;
                int w = demod_broadcast_response_encode(&disc, dg, sizeof dg);
                if (w > 0 && sendto(ufd, dg, (size_t)w, 0, (struct sockaddr *)&from, flen) == w)
                    ++answered;
            }
        }
        if (!(pf[0].revents & (POLLIN | POLLHUP | POLLERR))) continue;
        if (cfd < 0) {
            cfd = accept(lfd, NULL, NULL);
            if (cfd < 0) continue;
            ++clients;
            demod_receiver_info_t info;
            memset(&info, 0, sizeof info);
            info.discovery_data = disc;
            info.discovery_data.currently_streaming = 0;
            info.max_encoded_frame_size = DEMOD_MAX_FRAME_PAYLOAD;  /* network.cpp:392 */
            info.max_decoded_frame_size = DEMOD_MAX_DECODED_FRAME;  /* network.cpp:393 */
            uint8_t hello[512];
            int w = demod_hello_encode(&info, hello, sizeof hello);
            if (w < 0 || send_all(cfd, hello, (size_t)w) != 0) {
                fprintf(stderr, "fskrx: failed to write hello, closing connection\n");
                close(cfd);
                cfd = -1;
                continue;
            }
            demod_reset(st);
            in_len = pcm_len = 0;
            continue;
        }
        ssize_t got = recv(cfd, in + in_len, in_cap - in_len, 0);
        if (got < 0 && errno == EINTR) continue;
        int end_stream = got <= 0;
        if (got > 0) in_len += (size_t)got;
        size_t off = 0;
        while (!rc && !end_stream) {
            const uint8_t *pl;
            size_t pl_len, used;
            int d = demod_frame_decode(in + off, in_len - off, &pl, &pl_len, &used);
            if (d == DEMOD_BUFFER_TOO_SMALL) break;
            if (d != DEMOD_OK) {
                fprintf(stderr, "fskrx: bad frame (%s), closing connection\n", demod_strerror(d));
                end_stream = 1;
                break;
            }
            if (!nt->raw_pcm || pl_len % frame_bytes) {
                /* Opus bytes (or a torn PCM frame): refuse rather than
                 * demodulate noise; tell the transmitter (ip.proto:56-61) */
                if (!nt->raw_pcm)
                    fprintf(stderr, "fskrx: AudioData carries Opus in the reference and this "
                                    "receiver does not decode Opus (-r: raw PCM payloads); "
                                    "refusing the stream\n");
                else
                    fprintf(stderr, "fskrx: AudioData payload of %zu bytes is not whole %zu-byte "
                                    "PCM frames (%s); refusing the stream\n",
                            pl_len, frame_bytes, demod_strerror(DEMOD_BAD_ARG));
                demod_receiver_error_t re = {0, 1};
                uint8_t eb[16];
                int w = demod_receiver_error_encode(&re, eb, sizeof eb);
                if (w > 0) (void)send_all(cfd, eb, (size_t)w);
                ++refused;
                end_stream = 1;
                break;
            }
            if (pcm_len + pl_len > pcm_cap) {
                uint8_t *p = realloc(pcm, pcm_cap * 2 + pl_len);
                if (!p) { rc = 4; break; }
                pcm = p;
                pcm_cap = pcm_cap * 2 + pl_len;
            }
            memcpy(pcm + pcm_len, pl, pl_len);
            pcm_len += pl_len;
            off += used;
        }
        memmove(in, in + off, in_len - off);
        in_len -= off;
        if (!end_stream && in_len == in_cap) { /* a frame larger than any valid one */
            fprintf(stderr, "fskrx: oversized frame, closing connection\n");
            end_stream = 1;
        }
        if (!rc) rc = feed_pcm(st, s, pcm, &pcm_len, frame_bytes, &sym, &sym_cap, frames_in);
        if (end_stream) {
            close(cfd);
            cfd = -1;
            if (!rc && s->n) rc = sink_emit(s, s->n); /* end of this stream's symbols */
            if (!rc && fflush(stdout) != 0) rc = 5;
            done = nt->once;
        }
    }
    fprintf(stderr,
            "fskrx: %llu transmitter(s) served, %llu refused, %llu discovery request(s) answered\n",
            clients, refused, answered);
    if (!rc && refused) rc = 4;
    if (cfd >= 0) close(cfd);
    close(lfd);
    if (ufd >= 0) close(ufd);
    free(in);
    free(pcm);
    free(sym);
    return rc;
}

/* ---- group mode ---------------------------------------------------------- */

static int run_group(const demod_cfg_t *cfg, int gpus, int n_streams, size_t per_read, const char *prefix)
{
    int devs[64];
    for (int i = 0; i < gpus; ++i) devs[i] = i;
    int err = 0;
    demod_group_t *g = demod_group_create_local(cfg, (size_t)n_streams, gpus, devs, &err);
    if (!g) {
        fprintf(stderr, "fskrx: demod_group_create_local: %s\n", demod_strerror(err));
        return 3;
    }
    const size_t S = (size_t)n_streams, ch = cfg->channels;
    struct sink *sk = calloc(S, sizeof *sk);
    int16_t *pcm = malloc(S * per_read * ch * sizeof(int16_t));
    const int16_t **ptr = calloc(S, sizeof *ptr);
    size_t *nf = calloc(S, sizeof *nf);
    uint32_t *counts = calloc(S, sizeof *counts);
    const size_t cap = S * ((per_read + cfg->n) / cfg->hop + 2);
    uint8_t *sym = malloc(cap);
    int rc = (sk && pcm && ptr && nf && counts && sym) ? 0 : 4;
    for (size_t i = 0; !rc && i < S; ++i) {
        char path[4096];
        snprintf(path, sizeof path, "%s%zu.bin", prefix, i);
        sk[i].bits = demod_bits_per_symbol(cfg->k);
        sk[i].per = (size_t)DEMOD_MAX_FRAME_PAYLOAD * 8 / (size_t)sk[i].bits;
        sk[i].frame_cap = demod_frame_size(DEMOD_MAX_FRAME_PAYLOAD);
        sk[i].frame = malloc(sk[i].frame_cap);
        sk[i].out = fopen(path, "wb");
        if (!sk[i].frame || !sk[i].out) rc = 5;
    }
    unsigned long long frames_in = 0, syms = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    while (!rc) {
        const size_t got = fread(pcm, sizeof(int16_t) * ch, S * per_read, stdin);
        if (ferror(stdin)) { rc = 5; break; }
        if (!got) break;
        size_t left = got;
        for (size_t i = 0; i < S; ++i) {   /* a short final round is dealt in stream order */
            nf[i] = left < per_read ? left : per_read;
            left -= nf[i];
            ptr[i] = pcm + i * per_read * ch;
        }
        const int ns = demod_group_push(g, ptr, nf, sym, cap, counts);
        if (ns < 0) {
            fprintf(stderr, "fskrx: demod_group_push: %s\n", demod_strerror(ns));
            rc = 4;
            break;
        }
        frames_in += got;
        syms += (unsigned long long)ns;
        size_t off = 0;
        for (size_t i = 0; i < S && !rc; ++i) {
            rc = sink_push(&sk[i], sym + off, counts[i]);
            off += counts[i];
        }
        if (got < S * per_read) break;
    }
    for (size_t i = 0; i < S && sk; ++i) {
        if (!rc && sk[i].n) rc = sink_emit(&sk[i], sk[i].n);
        if (sk[i].out && fclose(sk[i].out) != 0 && !rc) rc = 5;
        free(sk[i].sym);
        free(sk[i].frame);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    const double el = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    fprintf(stderr, "fskrx: group of %d GPU(s), %d streams: %llu frames in, %llu symbols, %.3f s wall\n",
            demod_group_world(g), n_streams, frames_in, syms, el);
    free(sk);
    free(pcm);
    free(ptr);
    free(nf);
    free(counts);
    free(sym);
    demod_group_destroy(g);
    return rc;
}

int main(int argc, char **argv)
{
    demod_cfg_t cfg;
    demod_cfg_default(&cfg);
    size_t per_read = 2880; /* one 60 ms packet at 48 kHz (playback.cpp:10) */
    int batch = 0;
    struct net nt = {"0.0.0.0", -1, -1, "", 0, 0};
    int gpus = 0, n_streams = 0;
    const char *prefix = NULL;
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
        if (!strcmp(a, "-b")) { batch = 1; continue; }
        if (!strcmp(a, "-1")) { nt.once = 1; continue; }
        if (!strcmp(a, "-r")) { nt.raw_pcm = 1; continue; }
        if (!v) return usage();
        ++i;
        if (!strcmp(a, "-c")) cfg.channels = (uint32_t)atoi(v);
        else if (!strcmp(a, "-l")) nt.tcp_port = atoi(v);
        else if (!strcmp(a, "-u")) nt.udp_port = atoi(v);
        else if (!strcmp(a, "-a")) nt.addr = v;
        else if (!strcmp(a, "-N")) nt.name = v;
        else if (!strcmp(a, "-n")) cfg.n = (uint32_t)atoi(v);
        else if (!strcmp(a, "-H")) cfg.hop = (uint32_t)atoi(v);
        else if (!strcmp(a, "-p")) per_read = (size_t)strtoull(v, NULL, 10);
        else if (!strcmp(a, "-L")) cfg.lead_in = (uint32_t)strtoul(v, NULL, 10);
        else if (!strcmp(a, "-g")) gpus = atoi(v);
        else if (!strcmp(a, "-S")) n_streams = atoi(v);
        else if (!strcmp(a, "-o")) prefix = v;
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
    if (per_read == 0 || (nt.tcp_port < 0 && (nt.udp_port >= 0 || nt.once || nt.raw_pcm)) ||
        strlen(nt.name) >= DEMOD_INFO_STRING_CAP)
        return usage();

    if (gpus || n_streams || prefix) {
        if (gpus < 1 || gpus > 64 || !prefix || n_streams < 0 || batch || nt.tcp_port >= 0) return usage();
        return run_group(&cfg, gpus, n_streams ? n_streams : gpus, per_read, prefix);
    }
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
    s.frame_cap = demod_frame_size(DEMOD_MAX_FRAME_PAYLOAD); /* one frame per call */
    s.frame = malloc(s.frame_cap);
    int rc = s.frame ? 0 : 4;

    const size_t ch = cfg.channels;
    size_t cap = batch ? ((size_t)1 << 20) : per_read;
    int16_t *pcm = nt.tcp_port >= 0 ? NULL : malloc(cap * ch * sizeof(int16_t));
    uint8_t *sym = NULL;
    size_t sym_cap = 0;
    size_t have = 0;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    unsigned long long frames_in = 0;
    if (!rc && nt.tcp_port >= 0) rc = serve(st, &cfg, &s, &nt, &frames_in);
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
