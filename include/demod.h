/*
 * demod.h — C ABI of the MI355X acoustic-FSK demodulator (libfskdemod.so).
 *
 * This is the drop-in boundary for the north-star path.
 * The reference (tmarsteel/audio-network) has no demodulator; every entry
 * point below mirrors the shape of the C API that sits at the insertion
 * point in the reference receiver, right after `opus_decode`
 * (hardware/src/playback.cpp:118):
 *
 *   - an opaque handle created/destroyed like an Opus decoder
 *       opus_decoder_create / opus_decoder_destroy
 *       (hardware/lib/libopus/src/opus.h:423,512; playback.cpp:67-74);
 *   - caller-owned buffers, `int` return = count on success or a negative
 *     error code (opus_decode, opus.h:462; codes opus_defines.h:46-60);
 *   - errors are returned, never abort()ed (the reference call site aborts
 *     via OPUS_ERROR_CHECK, playback.cpp:16-22 — deliberately not copied);
 *   - frame bytes follow protocol/ip.proto:32-36,63-65 (ToReceiver{AudioData})
 *     with the varint32 length prefix of nanopb pb_encode_delimited /
 *     protobuf-java writeDelimitedTo (network.cpp:389-403,411;
 *     transmitter protobuf_async.kt:69-80,110-114).
 *
 * Threading: re-entrant across handles, not within one handle (one handle
 * serves one consumer, like the single playback task, playback.cpp:157-165).
 *
 * Decisions: every symbol is the argmax of the tone powers as the double-
 * precision definition computes them (ties to the lowest tone). The kernels
 * decide in fp32; a window whose fp32 top-2 margin lies within the powers'
 * error bound (derived from the kernel's operation sequence and constants,
 * demod_error_model) is flagged, and the decision rescue
 * decides it again in double and rewrites its symbol and powers: first by
 * 64-sample segments, or by the window folded to 128 samples where every
 * tone sits on a multiple of 8 bins, or by the residue fold (per tone the
 * 8-point DFT of the N/8-spaced samples at its residue b mod 8) for the
 * residue detector's integer-bin plans (n = 1024; each form with its own
 * derived bound against the definition's, so the rewritten powers are within
 * that bound of the definition's, not its bits; FSKD_PASS0_FOLD=0 keeps
 * segments), and where
 * that pass cannot decide, with the
 * definition's own arithmetic (powers bit-identical to it; every rescued
 * window with FSKD_RESCUE_SEG=0). The flag test runs in two stages: the int16 worst-case
 * energy first (no per-sample work), then, only for windows that test
 * flags, the window's own energy, so quiet input is not flagged wholesale.
 * The rescue runs inside the detector's own launch for every detector at
 * n = 1024 whose windows are evaluated one by one (plain bank, fold and FFT);
 * segment-shared windows (hop = 64 H < n, demod_slide_windows() > 0), the
 * residue detector's plans (their first pass lives there) and other window
 * lengths take a second launch on the same stream
 * (demod_batch_launches counts it). A batch is complete when its stream has
 * passed its launches; there is no state shared between batches, so batches
 * of one handle may run on different streams.
 *
 * Every compute entry point runs on the GPU (HIP, gfx950). There is no CPU
 * fallback: without a visible MI355X, demod_create() fails with
 * DEMOD_NO_DEVICE. The framing / packing helpers are pure host byte work.
 */
#ifndef FSKDEMOD_DEMOD_H
#define FSKDEMOD_DEMOD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- error codes (same numbering as opus_defines.h:46-60 where they overlap) */
#define DEMOD_OK                 0
#define DEMOD_BAD_ARG           -1  /* OPUS_BAD_ARG */
#define DEMOD_BUFFER_TOO_SMALL  -2  /* OPUS_BUFFER_TOO_SMALL */
#define DEMOD_INTERNAL_ERROR    -3  /* OPUS_INTERNAL_ERROR */
#define DEMOD_INVALID_PACKET    -4  /* OPUS_INVALID_PACKET: malformed frame bytes */
#define DEMOD_UNIMPLEMENTED     -5  /* OPUS_UNIMPLEMENTED */
#define DEMOD_INVALID_STATE     -6  /* OPUS_INVALID_STATE */
#define DEMOD_ALLOC_FAIL        -7  /* OPUS_ALLOC_FAIL */
#define DEMOD_DEVICE_ERROR      -8  /* a HIP runtime call failed */
#define DEMOD_NO_DEVICE         -9  /* no gfx950 device visible */
#define DEMOD_FRAME_TOO_LARGE  -10  /* payload > max encoded frame (network.cpp:24,223) */

#define DEMOD_MAX_TONES         16
/* Opus decoder delay of the transmitter's encoder settings at 48 kHz
 * (OPUS_GET_LOOKAHEAD; computed but never used by the reference,
 * transmitter OpusEncoder.kt:46-47,65-67; measured in SURVEY.md §8 a7). */
#define DEMOD_OPUS_LOOKAHEAD    312
#define DEMOD_MAX_FRAME_PAYLOAD 4096 /* MAX_ENCODED_FRAME_SIZE, network.cpp:24 */

/* channel handling for interleaved input (channels == 2) */
#define DEMOD_CH_LEFT     0   /* use channel 0 */
#define DEMOD_CH_RIGHT    1   /* use channel 1 */
#define DEMOD_CH_DOWNMIX  2   /* x = (L + R) >> 1 (arithmetic shift) */

/* detector selection */
#define DEMOD_METHOD_AUTO      0 /* FOLDED when eligible and k >= 3; else RESIDUE
                                    when eligible and k >= 5 (except overlapping
                                    windows at n = 1024, hop = 64 H <= 384, which
                                    take GOERTZEL); else GOERTZEL */
#define DEMOD_METHOD_GOERTZEL  1 /* per-window Goertzel tone bank over all n samples
                                    (n = 1024, hop = 64 H < n: 64-sample segments
                                    shared by the windows that contain them, same
                                    results as evaluating each window alone) */
#define DEMOD_METHOD_FFT       2 /* full-spectrum n-point real FFT (n = 1024), argmax
                                    over the tone bins round(f*n/fs); tones-only
                                    batches run the real split's post-pass only in
                                    the pair blocks holding a tone bin (same tone
                                    powers; demod_plan_info_t.fft_pmask;
                                    FSKD_FFT_PMASK=0 at demod_create: every block,
                                    a measurement switch) */
#define DEMOD_METHOD_FOLDED    3 /* Goertzel over the window folded to n/8 samples:
                                    exact when every tone is on a multiple of 8
                                    bins (f*n/fs integer, divisible by 8); at
                                    n = 1024, hop = 64 H < n the folded sums are
                                    carried from window to window (same results
                                    as evaluating each window alone).
                                    Magnitudes: its derived error bound implies
                                    |P_k - P_ref,k| <= 8.8e-6 P_max on an aligned
                                    window (north_star's 1e-5); the plain bank's
                                    (GOERTZEL, AUTO's choice at k <= 2) implies
                                    only 7e-5, so under AUTO configs[1]'s 1e-5
                                    magnitude bar is measured (every timed window,
                                    bench parity_all), not derived. FOLDED proves
                                    it at ~2 % of configs[1]'s step */
#define DEMOD_METHOD_RESIDUE   4 /* Goertzel over the window folded to n/8 samples per
                                    residue class of the bin mod 8: exact when every
                                    tone is on an integer bin (f*n/fs integer) */

typedef struct demod_cfg {
    double   fs;                     /* sample rate, Hz (48000) */
    uint32_t n;                      /* window length N in samples (1024) */
    uint32_t hop;                    /* window advance; == n for non-overlapping */
    uint32_t k;                      /* number of tones, 1..DEMOD_MAX_TONES */
    uint32_t channels;               /* 1 = mono, 2 = interleaved stereo */
    int32_t  channel_mode;           /* DEMOD_CH_* (ignored for mono) */
    int32_t  device;                 /* HIP device ordinal */
    int32_t  method;                 /* DEMOD_METHOD_* */
    uint32_t lead_in;                /* mono frames demodulate() drops at the start of a
                                        stream (after demod_create / demod_reset), e.g.
                                        DEMOD_OPUS_LOOKAHEAD to absorb the Opus decoder
                                        delay; 0 = none. < 2^31. Batch calls ignore it. */
    double   freqs[DEMOD_MAX_TONES]; /* tone frequencies, Hz; symbol i <-> freqs[i] */
} demod_cfg_t;

typedef struct demod demod_t;

/* Fill cfg with the 2-FSK defaults of SURVEY.md §8: fs 48 kHz, N = hop = 1024,
 * tones {1500, 3000} Hz, mono. */
void demod_cfg_default(demod_cfg_t *cfg);

/* Replaces opus_decoder_create (opus.h:423). NULL on failure, *error set. */
demod_t *demod_create(const demod_cfg_t *cfg, int *error);

/* Replaces opus_decoder_destroy (opus.h:512). NULL is accepted. */
void demod_destroy(demod_t *st);

/* Drop carried samples and re-arm cfg.lead_in; the next demodulate() starts a
 * new stream. Mirrors playback_start_new_stream (playback.cpp:67-74), which
 * recreates the Opus decoder (and with it its delay) per stream. */
int demod_reset(demod_t *st);

/* Detector the handle runs (DEMOD_METHOD_GOERTZEL / _FOLDED / _RESIDUE / _FFT). */
int demod_method(const demod_t *st);

/* Overlapping windows (n = 1024, hop = 64 H < n): the windows per tile the
 * detector's segment-shared kernel evaluates together (plain bank or fold,
 * DESIGN.md §4.8); 0 when every window is evaluated alone. The results are
 * the same either way. (FSKD_NO_SLIDE=1 in the environment at demod_create
 * turns the shared kernels off, for measurements.) */
int demod_slide_windows(const demod_t *st);

/* Number of mono samples currently carried between demodulate() calls. */
int demod_pending(const demod_t *st);

/* Upper bound on symbols the next demodulate(st, ., n_frames, ...) emits. */
int demod_max_symbols(const demod_t *st, size_t n_frames);

/* Kernel launches one device-pointer demod_batch / demod_batch_async of
 * n_windows makes (with_mags: magnitudes requested): the detector's, plus one
 * for the decision rescue where it is not inside the detector (K >= 2 on
 * segment-shared windows, residue plans or n != 1024; every other detector,
 * the FFT included, rescues inside its own launch). A Goertzel-family batch is one
 * detector launch; from 4 MiB of symbol + magnitude output it writes each
 * XCD's L2 back in a few bursts inside that launch instead of interleaving the
 * write-back with the input stream. With the environment
 * variable FSKD_WB_BURSTS=0 at demod_create (a measurement switch), batches
 * over ~10 MiB of output run as equal detector slices instead, and profilers
 * see that many dispatches. A host-pointer demod_batch over 4 MiB of samples
 * runs in chunks of 65 536 windows, each chunk counted as a batch of its own. */
int demod_batch_launches(const demod_t *st, size_t n_windows, int with_mags);

/* The decision rescue's threshold factor tau of this handle (0 when the
 * rescue is off, K = 1 or FSKD_NO_RESCUE=1): a window is re-decided in double
 * when its fp32 top-2 margin is below tau sqrt(NE P_max), NE the energy scale
 * of the window the detector transforms (n sum x^2; fold detector: (n/8)
 * sum xf^2 of the N/8-folded window, plus the oracle's share, see
 * demod_error_model_t.amb_d). tau = 4 (rho_det + rho_ref) / sqrt(n_eff) with
 * the bounds derived for the handle's tone plan and kernel (demod_error_model,
 * DESIGN.md §2a); no measured constant. For tests and diagnostics. */
double demod_rescue_tau(const demod_t *st);

/* The rescue's first pass (n = 1024: the Goertzel-family detectors, in the
 * kernel or, for segment-shared windows, in the rescue launch; and the FFT
 * detector's TONES-ONLY batches at its tone bins; a spectrum batch's flagged
 * windows always take the double FFT): a flagged window's powers in double by
 * 64-sample segments (fold plans and FFT plans whose tone bins are multiples
 * of 8: by the window folded to 128 samples) decide it when their top-2
 * margin clears tau64 sqrt(n sum x^2 P_max); windows inside that band take the
 * exact double chain (or double FFT). Returns tau64 = 4 rho_first / sqrt(n)
 * (0: every flagged window takes the exact path — n != 1024,
 * FSKD_RESCUE_SEG=0). For tests and diagnostics. */
double demod_rescue_tau64(const demod_t *st);

/* The error bounds behind the decision rescue, derived for a
 * configuration's tone plan from the kernel's operation sequence and fp32
 * constants by a forward rounding-error analysis; no device needed. For every
 * window x and tone k, with X_k the exact DFT of x at the tone (the fold /
 * residue / FFT detectors: at its bin):
 *   |sqrt(P_gpu,k) - |X_k||      <= rho_det sqrt(E_det)
 *   |sigma(P_oracle,k) - |X_k||  <= rho_ref sqrt(sum x^2)   sigma(P) = sign(P) sqrt|P|
 *   |sqrt(P_first,k) - sigma(P_oracle,k)| <= rho_first sqrt(sum x^2)  (pass 0)
 * E_det = sum x^2 of the window (plain bank, residue, FFT) or sum xf^2 of the
 * window folded to n/8 samples (energy = DEMOD_ENERGY_FOLDED). The kernels
 * flag a window when (P_1 - P_2)^2 < t2e E_eff P_1 (E_eff: the kernel's energy
 * E, Parseval's 2 sum_b P_b for the FFT (n sum x^2 from the samples on
 * tones-only batches that skip post-pass blocks), (sqrt E + amb_d)^2 for the fold
 * detector), which leaves unflagged only windows whose sqrt-power margin
 * exceeds twice the two bounds: their symbol is the oracle's. */
#define DEMOD_ENERGY_RAW      0
#define DEMOD_ENERGY_FOLDED   1
#define DEMOD_ENERGY_PARSEVAL 2
typedef struct demod_error_model {
    int32_t method;      /* the detector the configuration runs (DEMOD_METHOD_*) */
    int32_t energy;      /* DEMOD_ENERGY_*: the energy the kernel's flag test sums */
    double  rho_det;
    double  rho_ref;
    double  rho_first;   /* 0 when the configuration has no pass 0 (n != 1024, K = 1) */
    double  tau;         /* as demod_rescue_tau (0 for K = 1) */
    double  tau64;       /* as demod_rescue_tau64, before the handle's switches */
    double  t2e;         /* the stage-2 threshold factor the kernels read */
    double  t2e64;       /* pass 0's, with E its sum x^2 */
    double  amb_d;       /* fold detector: the oracle's share in units of sqrt(sum xf^2) */
} demod_error_model_t;
int demod_error_model(const demod_cfg_t *cfg, demod_error_model_t *model);

/* The tone plan a configuration runs and the fp32 constants its kernels read
 * (the arrays demod_create uploads), for operation-for-operation emulation in
 * tests; no device needed. rot receives rot_len float4 entries ([slot][g],
 * residue [slot][g][2]) when rot_cap (floats) allows, rot64 the first pass's
 * double tables ([k][16][4] then c[k]) when rot64_cap allows. */
typedef struct demod_plan_info {
    int32_t  method;        /* DEMOD_METHOD_* the configuration runs */
    int32_t  log2g;         /* lanes per window = 2^log2g = n / 64 */
    int32_t  reinsch;       /* plain bank: Reinsch-modified recurrence */
    int32_t  f16;           /* fold detector: fold by 16 (K = 8) */
    int32_t  dcls;          /* residue detector: compile-time class pattern */
    int32_t  slide;         /* segment-shared kernels (n = 1024, hop = 64 H < n) */
    uint64_t perm;          /* nibble s = the tone of kernel slot s (DCLS / F16) */
    int32_t  slot_tone[DEMOD_MAX_TONES];
    int32_t  zcls[DEMOD_MAX_TONES];
    int32_t  fft_bins[DEMOD_MAX_TONES];
    float    coef[DEMOD_MAX_TONES];
    float    sgn[DEMOD_MAX_TONES];
    double   rcoef[DEMOD_MAX_TONES];
    uint32_t rot_len;       /* float4 entries of rot */
    uint32_t rot64_len;     /* doubles of rot64 */
    int32_t  fold64;        /* pass 0's form: 1 = by the fold (rot64 rows are lane
                             * j's folded positions 8j .. 8j + 7 at the exact
                             * bins; fold detector plans), 2 = by the residue
                             * fold (residue detector plans, in the rescue
                             * launch), 0 = lane j's raw samples 64j .. */
    uint32_t fft_pmask;     /* FFT detector, tones only: bit jb = the real-split
                             * post-pass pair block jb (pairs 2jb, 2jb + 1 of
                             * every lane) holds a tone bin; only those blocks
                             * run (0xFF: all, the full spectrum's post-pass) */
} demod_plan_info_t;
int demod_plan_info(const demod_cfg_t *cfg, demod_plan_info_t *info, float *rot, size_t rot_cap,
                    double *rot64, size_t rot64_cap);

/*
 * Streaming entry point: demodulate(pcm, n) -> symbols.
 * pcm: host pointer to n_frames frames of `channels` interleaved int16
 * samples (48 kHz int16 LE, the format opus_decode writes at
 * playback.cpp:118). The stream's first cfg.lead_in frames are dropped; the
 * rest are appended to the handle's carry buffer;
 * one symbol is emitted per complete window (advance `hop`).
 * Returns the number of symbols written to symbols[0..], or a negative code.
 * If max_symbols is too small nothing is consumed and
 * DEMOD_BUFFER_TOO_SMALL is returned.
 * mags (nullable, host): receives k floats |X_k|^2 per emitted symbol.
 * Packet-sized calls (<= 16 Ki samples of carry + packet) run the kernel on
 * mapped, coherent pinned memory: one launch and one synchronize, no copies
 * (FSKD_NO_ZERO_COPY=1 in the environment at the handle's first such call
 * selects the copy path; a measurement switch, results are the same).
 */
int demodulate(demod_t *st, const int16_t *pcm, size_t n_frames,
               uint8_t *symbols, size_t max_symbols);
int demodulate_mags(demod_t *st, const int16_t *pcm, size_t n_frames,
                    uint8_t *symbols, float *mags, size_t max_symbols);

/*
 * Batch entry point (the GPU hot path): W windows of mono int16.
 * Window w starts at pcm + w * hop and is n samples long.
 * Pointers may be host or device memory (detected per call); the call is
 * synchronous. Returns W on success.
 */
int demod_batch(demod_t *st, const int16_t *pcm, size_t n_windows,
                uint8_t *symbols, float *mags);

/*
 * Asynchronous batch on a caller stream (hipStream_t passed as void*; NULL =
 * the HIP default stream, as in the HIP runtime API). All pointers must be
 * device pointers. Nothing is synchronised; returns W once enqueued.
 */
int demod_batch_async(demod_t *st, const int16_t *d_pcm, size_t n_windows,
                      uint8_t *d_symbols, float *d_mags, void *stream);

/*
 * Full-spectrum variant of demod_batch_async for DEMOD_METHOD_FFT handles:
 * additionally writes |X[b]|^2, b = 0..n/2, to d_spectrum[W][n/2 + 1]
 * (nullable). Other handles return DEMOD_UNIMPLEMENTED. Any float alignment
 * is accepted; a 16-byte-aligned d_spectrum takes the faster store path
 * (whole 16-byte stores of each 4-window group's rows).
 */
int demod_batch_spectrum_async(demod_t *st, const int16_t *d_pcm, size_t n_windows,
                               uint8_t *d_symbols, float *d_mags, float *d_spectrum,
                               void *stream);

/* ---- many streams, one launch (config 5 as a service) ----------------- */
/*
 * n_streams independent streams that share one configuration, each behaving
 * exactly like its own demod_t from that cfg (its own carry buffer and
 * lead-in). The reference runs one decoder per device (playback.cpp:157-165);
 * a receiver of many streams would otherwise make one demodulate() call --
 * one H2D copy, one kernel launch, one D2H copy -- per stream per packet.
 * demod_streams_push takes one packet per stream and demodulates every
 * complete window of every stream in ONE batch: one copy in, one detector
 * launch, one copy out (the streams' runs laid end to end on hop
 * boundaries; windows that would straddle two runs are computed and
 * dropped).
 */
typedef struct demod_streams demod_streams_t;

/* NULL on failure, *error set. n_streams >= 1. */
demod_streams_t *demod_streams_create(const demod_cfg_t *cfg, size_t n_streams, int *error);
void demod_streams_destroy(demod_streams_t *ms);

/* demod_reset for one stream (drop its carry, re-arm cfg.lead_in). */
int demod_streams_reset(demod_streams_t *ms, size_t stream);

/* Mono samples stream `stream` carries between pushes. */
int demod_streams_pending(const demod_streams_t *ms, size_t stream);

/* Upper bound on the symbols the next push with these packet sizes emits. */
long long demod_streams_max_symbols(const demod_streams_t *ms, const size_t *n_frames);

/*
 * pcm[i]: host pointer to n_frames[i] frames of stream i (`channels`
 * interleaved int16, as for demodulate; NULL allowed when n_frames[i] == 0).
 * Symbols of stream 0, then stream 1, ... are written to symbols[0..];
 * counts[i] receives the number stream i emitted; mags (nullable, host)
 * receives k floats |X_k|^2 per symbol in the same order. Returns the total,
 * or a negative code; if cap is too small nothing is consumed and
 * DEMOD_BUFFER_TOO_SMALL is returned. Symbols and magnitudes equal what
 * per-stream demodulate() calls would return.
 */
int demod_streams_push(demod_streams_t *ms, const int16_t *const *pcm, const size_t *n_frames,
                       uint8_t *symbols, float *mags, size_t cap, uint32_t *counts);

/*
 * The packet front-end of many streams (SURVEY §8 f2's decoder-agnostic half):
 * one encoded packet per stream, each decoded by `decode` with its stream's
 * decoder state, then demodulated as by demod_streams_push (per-stream carry,
 * lead-in, one batch). demod_decode_fn has opus_decode's signature
 * (libopus/src/opus.h:462; opus_decode itself, cast, is one), as the
 * reference calls it per packet (playback.cpp:115-122): it writes at most
 * frame_size frames of `channels` interleaved int16 to pcm and returns the
 * frames decoded or a negative code. decoders[i] is stream i's state (used by
 * one thread at a time: streams decode concurrently on the handle's staging
 * threads). lens[i] == 0: no packet for stream i this push (playback.cpp:105).
 * A decoder's negative code (the lowest stream's) is returned with nothing
 * pushed. Otherwise as demod_streams_push.
 */
typedef int (*demod_decode_fn)(void *decoder, const unsigned char *data, int32_t len, int16_t *pcm,
                               int frame_size, int decode_fec);
int demod_streams_push_packets(demod_streams_t *ms, demod_decode_fn decode, void *const *decoders,
                               const uint8_t *const *packets, const int32_t *lens, int frame_size,
                               uint8_t *symbols, float *mags, size_t cap, uint32_t *counts);

/* ---- many streams over many GPUs (config 5), RCCL ---------------------- */
/*
 * A group of `world` ranks, one per GPU, demodulating n_streams streams of one
 * configuration: rank r owns the contiguous stream shard
 * demod_group_shard(n_streams, r, world) and demodulates it on its own device;
 * RCCL (over xGMI) carries only the decoded result: an all-gather of every
 * rank's symbols (push) or ToReceiver frames (bucket). SURVEY.md §7 step 5 /
 * §8e: one process per GPU (demod_group_create: hipSetDevice to cfg->device +
 * ncclCommInitRank with rank 0's demod_group_unique_id, shared out of band),
 * or one process driving several GPUs (demod_group_create_local:
 * ncclCommInitAll). The reference fans one stream out to N receivers
 * (MulticastAudioOutput.kt:88-96); this gathers N GPUs' share of many streams.
 * Every call that gathers is a collective: every rank makes it.
 */
#define DEMOD_GROUP_ID_BYTES 128   /* sizeof(ncclUniqueId) */
typedef struct demod_group demod_group_t;

/* A fresh group id (ncclGetUniqueId) into id[DEMOD_GROUP_ID_BYTES]. */
int demod_group_unique_id(uint8_t *id);
/* Rank `rank`'s contiguous, balanced stream shard (pure arithmetic). */
int demod_group_shard(size_t n_streams, int rank, int world, size_t *first, size_t *count);
/* Bytes per rank of a bucket's gathered frames: steps x ceil(n_streams /
 * world) x demod_frame_symbols_size(symbols_per_stream, bits, 4096). */
long long demod_group_block_bytes(size_t n_streams, int world, size_t steps,
                                  size_t symbols_per_stream, int bits);
/* One rank of a multi-process group (cfg->device is its GPU). NULL on
 * failure, *error set. */
demod_group_t *demod_group_create(const demod_cfg_t *cfg, size_t n_streams, int rank, int world,
                                  const uint8_t *id, int *error);
/* Every rank in this process, rank i on devices[i]. */
demod_group_t *demod_group_create_local(const demod_cfg_t *cfg, size_t n_streams, int n_devices,
                                        const int *devices, int *error);
void demod_group_destroy(demod_group_t *g);
int demod_group_world(const demod_group_t *g);
int demod_group_local_ranks(const demod_group_t *g);   /* ranks this process drives */
int demod_group_rank_shard(const demod_group_t *g, int local, int *rank, size_t *first,
                           size_t *count);
/* The GPU ordinal of the local-th rank this process drives. */
int demod_group_rank_device(const demod_group_t *g, int local);
/* DEMOD_OK while the group is alive, else the code that killed it (see below). */
int demod_group_status(const demod_group_t *g);

/*
 * Errors (no abort(), negative codes; no hang). Every call
 * below is collective, and a rank never leaves one alone: each refusal is
 * decided from all-gathered words, so every rank returns the same code.
 * demod_group_push all-gathers [status, symbols == NULL, cap, per-stream
 * counts] before anything is consumed: an argument refusal on any rank
 * (demod_streams_push's own checks), a too-small cap or a total above INT_MAX
 * on any rank returns that code (the lowest failing rank's) on every rank with
 * nothing consumed. A push that fails on a rank after that point (device or
 * allocation failure) returns its code on every rank and leaves the group
 * dead: its communicator is aborted (ncclCommAbort), later calls return
 * DEMOD_INVALID_STATE and the caller destroys it. A collective that fails, or
 * does not finish within FSKD_GROUP_TIMEOUT_MS (default 120000: a peer process
 * died), aborts the communicator the same way and returns DEMOD_DEVICE_ERROR.
 */

/*
 * One packet per stream this process owns (a local group: all n_streams; one
 * rank of a multi-process group: its shard, pcm[i] = stream first + i), each
 * demodulated as demod_streams_push does (per-stream carry and lead-in).
 * Every stream's count is gathered first, then every rank's symbols; on
 * return, on every rank, symbols[] holds all n_streams streams' symbols
 * (stream 0 first) and counts[0 .. n_streams-1] their counts. Returns the
 * total; if cap is too small, every rank returns DEMOD_BUFFER_TOO_SMALL
 * before anything is consumed. A local group runs its ranks concurrently
 * (one host thread per GPU).
 */
int demod_group_push(demod_group_t *g, const int16_t *const *pcm, const size_t *n_frames,
                     uint8_t *symbols, size_t cap, uint32_t *counts);

/*
 * Config 5's step, device-resident, for each rank l this process drives
 * (arrays indexed by l): d_pcm[l] holds `ring` steps' batches of the rank's
 * streams, [ring][count][wps windows][n] (cfg.hop == n), the same batch in
 * each slot or a fresh one. `steps` (a multiple of ring) steps run as
 * steps / ring detector launches, ONE device framing launch over the steps'
 * symbol rows (one ToReceiver run per stream per step) and ONE RCCL
 * all-gather into d_all[l] ([world][block] bytes, rank q's block = its frames,
 * [step][stream][stride]), all enqueued on streams[l] (hipStream_t; NULL
 * array = default streams), so a caller may capture it in a HIP graph (make
 * one call of the shape outside capture first: it sizes the rank's buffers).
 * Every rank's status word is all-gathered beside the frames: a rank that
 * fails locally (a NULL d_pcm / d_all entry, a failed launch) still posts both
 * gathers, carrying its code, and returns that code; its peers learn it from
 * demod_group_wait. Returns block bytes (demod_group_block_bytes) or a
 * negative code (the shape, identical on every rank, is refused alike).
 */
long long demod_group_bucket_async(demod_group_t *g, const int16_t *const *d_pcm, size_t ring,
                                   size_t wps, size_t steps, uint8_t *const *d_all,
                                   void *const *streams);

/*
 * After buckets (or graph replays of one) on streams[l] (NULL array: default
 * streams): waits for them under the group's deadline, then returns the
 * lowest failing rank's status of the last bucket (the same on every rank),
 * DEMOD_OK, or DEMOD_DEVICE_ERROR when a collective failed or overran (the
 * group is then dead, as above).
 */
int demod_group_wait(demod_group_t *g, void *const *streams);

/* ---- ip.proto framing (ToReceiver{AudioData{bytes}}, delimited) ------- */

/* Bytes demod_frame_encode needs for a payload of len bytes. */
size_t demod_frame_size(size_t payload_len);

/* Encode varint32(len(msg)) || ToReceiver{audio_data{opus_encoded_frame =
 * payload}}. Returns bytes written, DEMOD_BUFFER_TOO_SMALL, or
 * DEMOD_FRAME_TOO_LARGE when len > DEMOD_MAX_FRAME_PAYLOAD. */
int demod_frame_encode(const uint8_t *payload, size_t len,
                       uint8_t *out, size_t cap);

/* Decode one delimited ToReceiver frame from in[0..len). On success
 * *payload points into `in`, *payload_len is its length, *consumed the
 * bytes of the whole frame; returns DEMOD_OK. Returns DEMOD_BUFFER_TOO_SMALL
 * when `in` holds only part of a frame (read more and retry),
 * DEMOD_INVALID_PACKET on malformed bytes, DEMOD_FRAME_TOO_LARGE when the
 * payload exceeds DEMOD_MAX_FRAME_PAYLOAD (network.cpp:223-227). */
int demod_frame_decode(const uint8_t *in, size_t len, const uint8_t **payload,
                       size_t *payload_len, size_t *consumed);

/* Bits per symbol used for packing: ceil(log2(k)), at least 1. */
int demod_bits_per_symbol(uint32_t k);

/* Pack n symbols MSB-first into ceil(n*bits/8) bytes. Returns bytes. */
int demod_pack_symbols(const uint8_t *symbols, size_t n, int bits,
                       uint8_t *out, size_t cap);
int demod_unpack_symbols(const uint8_t *in, size_t n, int bits,
                         uint8_t *symbols, size_t cap);

/* Frame a symbol stream into consecutive delimited ToReceiver frames,
 * each payload <= max_payload (<= DEMOD_MAX_FRAME_PAYLOAD) bytes of packed
 * symbols. Returns total bytes written. */
long long demod_frame_symbols(const uint8_t *symbols, size_t n, int bits,
                              size_t max_payload, uint8_t *out, size_t cap);

/* Bytes demod_frame_symbols writes for n symbols (0 for n = 0), or a
 * negative code for bad arguments. */
long long demod_frame_symbols_size(size_t n, int bits, size_t max_payload);

/* Device framing for many streams (config 5: each rank frames its own
 * streams before the RCCL gather). d_symbols holds n_streams x n symbols,
 * stream-major; stream s is framed exactly as demod_frame_symbols(symbols
 * of s, n, bits, max_payload, ...) would, into d_out + s * stride with
 * stride = demod_frame_symbols_size(n, bits, max_payload). Device pointers,
 * enqueued on `stream` (hipStream_t; NULL = default stream). Returns the
 * stride or a negative code. Stands in for nanopb pb_encode_delimited of
 * ToReceiver (network.cpp:389-403), one message per payload. */
long long demod_frame_streams_async(const uint8_t *d_symbols, size_t n_streams, size_t n,
                                    int bits, size_t max_payload, uint8_t *d_out,
                                    void *stream);

/* ---- ip.proto session messages ------------------ */
/* What a receiver exchanges around the audio stream: the delimited
 * ToTransmitter hello it writes when a transmitter connects on TCP 58764
 * (network.cpp:388-403; read by RemoteAudioReceiver.connect,
 * RemoteAudioReceiver.kt:60-68), and the BroadcastMessage datagrams of UDP
 * 58765 discovery (network.cpp:449-494; discovery.kt:23-97). Encoders emit
 * nanopb's bytes for the same struct; decoders return nanopb's verdict
 * (demod_session.c). Pure host byte work. */
#define DEMOD_PORT_AUDIO_RX    58764        /* ip.proto:28-31 (TCP) */
#define DEMOD_PORT_DISCOVERY   58765        /* ip.proto:5-7 (UDP) */
#define DEMOD_BROADCAST_MAGIC  0x2C5DA044u  /* ip.proto:10, network.cpp:448 */
#define DEMOD_INFO_STRING_CAP  128          /* char[128] strings, ip.pb.h:20,23 */
#define DEMOD_MAX_DECODED_FRAME 11520       /* AUDIO_BUFFER_SIZE, playback.cpp:10,193 */

/* oneof member tags returned by the decoders */
#define DEMOD_MSG_NONE                 0
#define DEMOD_MSG_DISCOVERY_REQUEST    2  /* BroadcastMessage.discovery_request */
#define DEMOD_MSG_DISCOVERY_RESPONSE   3  /* BroadcastMessage.discovery_response */
#define DEMOD_MSG_RECEIVER_INFORMATION 1  /* ToTransmitter.receiver_information */
#define DEMOD_MSG_RECEIVER_ERROR       2  /* ToTransmitter.error */

typedef struct {                  /* DiscoveryResponse, ip.pb.h:17-24 */
    uint32_t protocol_version;    /* 1 in the firmware (network.cpp:374) */
    uint64_t mac_address;         /* 6 MAC bytes, byte i at bits 8i (network.cpp:360-363) */
    char device_name[DEMOD_INFO_STRING_CAP];   /* NUL-terminated, <= 127 bytes */
    int currently_streaming;
    char opus_version[DEMOD_INFO_STRING_CAP];  /* NUL-terminated, <= 127 bytes */
} demod_discovery_t;

typedef struct {                  /* ReceiverInformation, ip.pb.h:55-59 */
    demod_discovery_t discovery_data;
    uint32_t max_encoded_frame_size;   /* 4096 in the firmware (network.cpp:392) */
    uint32_t max_decoded_frame_size;   /* 11520 in the firmware (network.cpp:393) */
} demod_receiver_info_t;

typedef struct {                  /* ReceiverError, ip.pb.h:61-64 */
    int audio_underflow;
    int audio_decode_error;
} demod_receiver_error_t;

/* BroadcastMessage{magic_word = DEMOD_BROADCAST_MAGIC, discovery_request =
 * true}, the datagram a transmitter broadcasts (discovery.kt:44-48).
 * Returns bytes written or DEMOD_BUFFER_TOO_SMALL. */
int demod_broadcast_request_encode(uint8_t *out, size_t cap);

/* BroadcastMessage{magic_word, discovery_response = *d}, the receiver's
 * unicast answer (network.cpp:356-378,486-492). Returns bytes written,
 * DEMOD_BUFFER_TOO_SMALL, or DEMOD_BAD_ARG for an unterminated string. */
int demod_broadcast_response_encode(const demod_discovery_t *d, uint8_t *out, size_t cap);

/* Decode one datagram as BroadcastMessage. Returns the oneof member
 * (DEMOD_MSG_NONE / _DISCOVERY_REQUEST / _DISCOVERY_RESPONSE) with *magic
 * set (and *resp filled for a response; resp may be NULL), or
 * DEMOD_INVALID_PACKET where nanopb's pb_decode fails. A receiver answers
 * exactly when this returns DEMOD_MSG_DISCOVERY_REQUEST and *magic ==
 * DEMOD_BROADCAST_MAGIC (network.cpp:473-485). */
int demod_broadcast_decode(const uint8_t *in, size_t len, uint32_t *magic,
                           demod_discovery_t *resp);

/* Length-delimited ToTransmitter{receiver_information = *info}: the hello
 * (network.cpp:388-403). Returns bytes written, DEMOD_BUFFER_TOO_SMALL or
 * DEMOD_BAD_ARG. */
int demod_hello_encode(const demod_receiver_info_t *info, uint8_t *out, size_t cap);

/* Length-delimited ToTransmitter{error = *e} (ip.proto:41-44,61-66). */
int demod_receiver_error_encode(const demod_receiver_error_t *e, uint8_t *out, size_t cap);

/* Decode one length-delimited ToTransmitter from in[0..len) (the
 * transmitter side, RemoteAudioReceiver.kt:60). Returns the oneof member
 * (DEMOD_MSG_NONE / _RECEIVER_INFORMATION / _RECEIVER_ERROR), filling *info
 * or *err (either may be NULL) and *consumed; DEMOD_BUFFER_TOO_SMALL when
 * only part of the message is in `in`; DEMOD_INVALID_PACKET where nanopb's
 * pb_decode_delimited fails. */
int demod_to_transmitter_decode(const uint8_t *in, size_t len, demod_receiver_info_t *info,
                                demod_receiver_error_t *err, size_t *consumed);

/* ---- synthetic PCM (benchmarks / tests) -------------------------------- */

/* Device generator of the seeded FSK test signal (DESIGN.md §Synthetic
 * input): windows w0 .. w0+W-1 of the stream, cfg->n mono samples each,
 * contiguous, symbols uniform
 * over cfg->k, amplitude `amplitude`, Irwin–Hall noise of std `sigma`.
 * d_pcm / d_symbols are device pointers on device cfg->device (checked:
 * DEMOD_BAD_ARG for memory of another device); enqueued on `stream`. The
 * sine table is uploaded to each device once per process: a
 * hipDeviceReset() while the library is loaded is not supported. */
int demod_synth_fsk(const demod_cfg_t *cfg, uint64_t seed, uint64_t w0,
                    size_t n_windows, int amplitude, int sigma, int16_t *d_pcm,
                    uint8_t *d_symbols, void *stream);

/* Read-only reference stream (probes): reads n_bytes (a multiple of 8192,
 * 16-byte aligned) of device memory with the detector kernels' access
 * pattern (8 KiB per wave, coalesced 16 B/lane non-temporal loads) and
 * discards it, enqueued on `stream`. A reference point for probes, not a
 * ceiling: the detector kernels measure slightly above it. */
int demod_read_ceiling_async(const void *d_buf, size_t n_bytes, void *stream);

/* ---- misc -------------------------------------------------------------- */
const char *demod_strerror(int error);   /* mirrors opus_strerror */
const char *demod_version_string(void);  /* mirrors opus_get_version_string */

#ifdef __cplusplus
}
#endif
#endif /* FSKDEMOD_DEMOD_H */
