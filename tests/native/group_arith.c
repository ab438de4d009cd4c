/* The multi-GPU group's shard and padding arithmetic through the C ABI
 * (include/demod.h demod_group_shard / demod_group_block_bytes; VERDICT r4
 * item 3), plus, when a gfx950 device is visible, a world-1 RCCL group whose
 * pushes must equal demod_streams_push byte for byte. Exit 0 = OK. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/demod.h"

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "group_arith: %s:%d: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                    \
        }                                                                \
    } while (0)

static int shards(void)
{
    static const size_t totals[] = {0, 1, 7, 8, 9, 127, 128, 1024, 1025, 4097};
    for (size_t t = 0; t < sizeof(totals) / sizeof(totals[0]); ++t)
        for (int world = 1; world <= 9; ++world) {
            size_t next = 0, lo = (size_t)-1, hi = 0;
            for (int r = 0; r < world; ++r) {
                size_t f = 99, c = 99;
                CHECK(demod_group_shard(totals[t], r, world, &f, &c) == DEMOD_OK);
                CHECK(f == next);                        /* contiguous, in rank order */
                next += c;
                lo = c < lo ? c : lo;
                hi = c > hi ? c : hi;
                if (r > 0) {                             /* the larger shards come first */
                    size_t f0, c0;
                    demod_group_shard(totals[t], r - 1, world, &f0, &c0);
                    CHECK(c0 >= c);
                }
            }
            CHECK(next == totals[t]);                    /* every stream exactly once */
            CHECK(hi - lo <= 1);                         /* balanced */
            CHECK(hi == (totals[t] + (size_t)world - 1) / (size_t)world);
        }
    size_t f, c;
    CHECK(demod_group_shard(8, 0, 0, &f, &c) == DEMOD_BAD_ARG);
    CHECK(demod_group_shard(8, 3, 3, &f, &c) == DEMOD_BAD_ARG);
    CHECK(demod_group_shard(8, -1, 3, &f, &c) == DEMOD_BAD_ARG);
    CHECK(demod_group_shard(8, 0, 3, NULL, &c) == DEMOD_BAD_ARG);
    return 0;
}

static int blocks(void)
{
    /* the bucket gathers steps x ceil(n / world) frame strides per rank: the
     * largest shard's frames, the others padded to it */
    const int bits[] = {1, 3, 4};
    const size_t wps[] = {1, 7, 2048, 40000};
    for (int b = 0; b < 3; ++b)
        for (int w = 0; w < 4; ++w) {
            const long long stride = demod_frame_symbols_size(wps[w], bits[b], DEMOD_MAX_FRAME_PAYLOAD);
            CHECK(stride > 0);
            for (int world = 1; world <= 8; ++world)
                for (size_t steps = 1; steps <= 16; steps *= 2) {
                    const long long blk = demod_group_block_bytes(1024, world, steps, wps[w], bits[b]);
                    CHECK(blk == (long long)steps * ((1024 + world - 1) / world) * stride);
                    size_t f, c;
                    for (int r = 0; r < world; ++r) {
                        demod_group_shard(1024, r, world, &f, &c);
                        CHECK((long long)(steps * c) * stride <= blk);   /* every rank's frames fit */
                    }
                }
        }
    /* the configs[4] step: 1024 streams, 2048 windows, 2-FSK, 16 steps, 8 GPUs */
    CHECK(demod_group_block_bytes(1024, 8, 16, 2048, 1) == 16LL * 128 * 264);
    CHECK(demod_group_block_bytes(1024, 0, 16, 2048, 1) == DEMOD_BAD_ARG);
    CHECK(demod_group_block_bytes(1024, 2, 0, 2048, 1) == DEMOD_BAD_ARG);
    return 0;
}

/* world 1 over RCCL: the group's pushes equal demod_streams_push */
static int gpu_world1(void)
{
    demod_cfg_t cfg;
    demod_cfg_default(&cfg);
    cfg.lead_in = 312;
    int err = 0;
    enum { S = 5, PK = 2880 };
    demod_streams_t *ms = demod_streams_create(&cfg, S, &err);
    if (!ms) {
        printf("group_arith: no device (%s): arithmetic only\n", demod_strerror(err));
        return 0;
    }
    uint8_t id[DEMOD_GROUP_ID_BYTES];
    CHECK(demod_group_unique_id(id) == DEMOD_OK);
    demod_group_t *g = demod_group_create(&cfg, S, 0, 1, id, &err);
    CHECK(g && err == DEMOD_OK);
    CHECK(demod_group_world(g) == 1 && demod_group_local_ranks(g) == 1);
    int16_t *pcm = malloc(sizeof(int16_t) * S * PK);
    uint8_t sym_a[S * 8], sym_b[S * 8];
    uint32_t cnt_a[S], cnt_b[S];
    unsigned long long st = 12345;
    for (int round = 0; round < 6; ++round) {
        for (int i = 0; i < S * PK; ++i) {
            st = st * 6364136223846793005ULL + 1442695040888963407ULL;
            pcm[i] = (int16_t)(st >> 48);
        }
        const int16_t *p[S];
        size_t nf[S];
        for (int s = 0; s < S; ++s) {
            p[s] = pcm + (size_t)s * PK;
            nf[s] = PK - 97 * (size_t)s;    /* ragged packets */
        }
        const int a = demod_streams_push(ms, p, nf, sym_a, NULL, sizeof(sym_a), cnt_a);
        const int b = demod_group_push(g, p, nf, sym_b, sizeof(sym_b), cnt_b);
        CHECK(a >= 0 && a == b);
        CHECK(memcmp(cnt_a, cnt_b, sizeof(cnt_a)) == 0 && memcmp(sym_a, sym_b, (size_t)a) == 0);
        CHECK(demod_group_push(g, p, nf, sym_b, 0, cnt_b) == (a ? DEMOD_BUFFER_TOO_SMALL : 0));
        const int a2 = demod_streams_push(ms, p, nf, sym_a, NULL, sizeof(sym_a), cnt_a);  /* keep in step */
        const int b2 = demod_group_push(g, p, nf, sym_b, sizeof(sym_b), cnt_b);
        CHECK(a2 == b2 && memcmp(sym_a, sym_b, (size_t)(a2 > 0 ? a2 : 0)) == 0);
    }
    free(pcm);
    demod_group_destroy(g);
    demod_streams_destroy(ms);
    printf("gpu demod_group_push: world 1 equals demod_streams_push\n");
    return 0;
}

int main(void)
{
    if (shards() || blocks()) return 1;
    printf("group arithmetic OK\n");
    return gpu_world1();
}
