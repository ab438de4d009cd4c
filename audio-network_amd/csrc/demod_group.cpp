// demod_group.cpp — configs[4] as a service over RCCL, from the C ABI
// (include/demod.h demod_group_*; VERDICT r4
// item 3). One process per GPU (ncclCommInitRank with rank 0's unique id,
// the `hipSetDevice + ncclCommInitRank` of SURVEY §7), or one process driving
// several GPUs (ncclCommInitAll). Rank r of `world` owns the contiguous
// stream shard demod_group_shard(n_streams, r, world) and demodulates it on
// its own device; the only collectives are the gathers of the decoded
// result (north_star: RCCL only for the final symbol gather):
//   * demod_group_push: one packet per stream (as demod_streams_push, whose
//     per-rank handle it wraps); every stream's symbol count is known before
//     the kernels run, so the ranks all-gather the counts first (one
//     uint32 per stream: a too-small caller buffer is refused on every rank
//     before anything is consumed), then the symbols (one padded block per
//     rank);
//   * demod_group_bucket_async: the bench's configs[4] step as an ABI call,
//     device-resident: S steps' detector launches (over an input ring of R
//     steps' batches each), ONE device framing launch over the S steps'
//     symbol rows (demod_frame_streams_async), ONE ncclAllGather of the
//     frames (a block of S x ceil(n_streams / world) x frame stride per
//     rank) on the caller's stream, so a caller can capture it in a HIP graph.
// The reference fans one audio stream out to N receivers (MulticastAudioOutput
// .kt:88-96); here N GPUs each demodulate their share of many streams and
// gather the frames.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/demod.h"
#include "demod_internal.h"
#include "plan.h"

namespace {

struct GroupRank {
    int device = 0, rank = 0;
    size_t first = 0, count = 0;        // the stream shard
    demod_streams_t *ms = nullptr;      // push path (per-stream carries)
    demod_t *st = nullptr;              // bucket path (device batches)
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;       // push path: copies + collectives
    uint8_t *d_send = nullptr, *d_recv = nullptr;
    size_t send_cap = 0, recv_cap = 0;
    uint8_t *d_sym = nullptr, *d_frames = nullptr;   // bucket: [S][count * wps], [S * max_count * stride]
    size_t sym_cap = 0, frames_cap = 0;
    std::vector<uint8_t> h_sym;
    std::vector<uint32_t> h_counts;
};

}  // namespace

struct demod_group {
    demod_cfg_t cfg;
    size_t n_streams = 0;
    int world = 1;
    std::vector<GroupRank> ranks;       // the ranks this process drives
    std::vector<uint8_t> h_recv;
    std::vector<uint32_t> h_counts_all;
};

#define NCCL_TRY(x)                                                               \
    do {                                                                          \
        ncclResult_t _r = (x);                                                    \
        if (_r != ncclSuccess) {                                                  \
            std::fprintf(stderr, "fskdemod: %s failed: %s\n", #x, ncclGetErrorString(_r)); \
            return DEMOD_DEVICE_ERROR;                                            \
        }                                                                         \
    } while (0)
#define HIP_TRY_G(x)                                                              \
    do {                                                                          \
        hipError_t _e = (x);                                                      \
        if (_e != hipSuccess) {                                                   \
            std::fprintf(stderr, "fskdemod: %s failed: %s\n", #x, hipGetErrorString(_e)); \
            return DEMOD_DEVICE_ERROR;                                            \
        }                                                                         \
    } while (0)

namespace {

// the caller's current device, restored on scope exit
struct DevRestore {
    int prev = -1;
    DevRestore()
    {
        if (hipGetDevice(&prev) != hipSuccess) {
            (void)hipGetLastError();
            prev = -1;
        }
    }
    ~DevRestore()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

void free_rank(GroupRank &r)
{
    if (r.stream) {
        (void)hipSetDevice(r.device);
        (void)hipStreamSynchronize(r.stream);
    }
    if (r.comm) (void)ncclCommDestroy(r.comm);
    if (r.d_send) (void)hipFree(r.d_send);
    if (r.d_recv) (void)hipFree(r.d_recv);
    if (r.d_sym) (void)hipFree(r.d_sym);
    if (r.d_frames) (void)hipFree(r.d_frames);
    if (r.stream) (void)hipStreamDestroy(r.stream);
    if (r.ms) demod_streams_destroy(r.ms);
    if (r.st) demod_destroy(r.st);
    r = GroupRank();
}

int grow(uint8_t *&p, size_t &cap, size_t need)
{
    if (need <= cap) return DEMOD_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    const size_t n = need + need / 4 + 256;
    HIP_TRY_G(hipMalloc(&p, n));
    HIP_TRY_G(hipMemset(p, 0, n));   // gathered padding is defined
    cap = n;
    return DEMOD_OK;
}

// the per-rank handles of rank r on device dev (communicator made by the caller)
int init_rank(demod_group_t *g, GroupRank &r, int rank, int device)
{
    r.rank = rank;
    r.device = device;
    demod_group_shard(g->n_streams, rank, g->world, &r.first, &r.count);
    demod_cfg_t c = g->cfg;
    c.device = device;
    int rc = DEMOD_OK;
    if (r.count) {
        r.ms = demod_streams_create(&c, r.count, &rc);
        if (!r.ms) return rc;
    }
    demod_cfg_t m = c;
    m.channels = 1;
    m.channel_mode = DEMOD_CH_LEFT;
    m.lead_in = 0;
    r.st = demod_create(&m, &rc);
    if (!r.st) return rc;
    HIP_TRY_G(hipSetDevice(device));
    HIP_TRY_G(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
    return DEMOD_OK;
}

size_t max_shard(size_t n_streams, int world) { return (n_streams + (size_t)world - 1) / (size_t)world; }

}  // namespace

extern "C" {

int demod_group_unique_id(uint8_t *id)
{
    if (!id) return DEMOD_BAD_ARG;
    static_assert(sizeof(ncclUniqueId) == DEMOD_GROUP_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    NCCL_TRY(ncclGetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return DEMOD_OK;
}

int demod_group_shard(size_t n_streams, int rank, int world, size_t *first, size_t *count)
{
    if (world < 1 || rank < 0 || rank >= world || !first || !count) return DEMOD_BAD_ARG;
    const size_t base = n_streams / (size_t)world, extra = n_streams % (size_t)world;
    *first = (size_t)rank * base + std::min((size_t)rank, extra);
    *count = base + ((size_t)rank < extra ? 1 : 0);
    return DEMOD_OK;
}

long long demod_group_block_bytes(size_t n_streams, int world, size_t steps, size_t symbols_per_stream,
                                  int bits)
{
    if (world < 1 || steps < 1) return DEMOD_BAD_ARG;
    const long long stride = demod_frame_symbols_size(symbols_per_stream, bits, DEMOD_MAX_FRAME_PAYLOAD);
    if (stride < 0) return stride;
    const unsigned long long b = (unsigned long long)steps * max_shard(n_streams, world) * (unsigned long long)stride;
    return b > (1ull << 62) ? DEMOD_BAD_ARG : (long long)b;
}

demod_group_t *demod_group_create(const demod_cfg_t *cfg, size_t n_streams, int rank, int world,
                                  const uint8_t *id, int *error)
{
    int rc = fskd::validate_cfg(cfg);
    if (rc == DEMOD_OK && (n_streams < 1 || n_streams > ((size_t)1 << 24) || world < 1 || rank < 0 ||
                           rank >= world || !id))
        rc = DEMOD_BAD_ARG;
    if (rc != DEMOD_OK) {
        if (error) *error = rc;
        return nullptr;
    }
    DevRestore keep;
    demod_group_t *g = new (std::nothrow) demod_group();
    if (!g) {
        if (error) *error = DEMOD_ALLOC_FAIL;
        return nullptr;
    }
    g->cfg = *cfg;
    g->n_streams = n_streams;
    g->world = world;
    g->ranks.resize(1);
    rc = init_rank(g, g->ranks[0], rank, cfg->device);
    if (rc == DEMOD_OK) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        (void)hipSetDevice(cfg->device);
        const ncclResult_t nr = ncclCommInitRank(&g->ranks[0].comm, world, u, rank);
        if (nr != ncclSuccess) {
            std::fprintf(stderr, "fskdemod: ncclCommInitRank failed: %s\n", ncclGetErrorString(nr));
            g->ranks[0].comm = nullptr;
            rc = DEMOD_DEVICE_ERROR;
        }
    }
    if (rc != DEMOD_OK) {
        demod_group_destroy(g);
        if (error) *error = rc;
        return nullptr;
    }
    if (error) *error = DEMOD_OK;
    return g;
}

demod_group_t *demod_group_create_local(const demod_cfg_t *cfg, size_t n_streams, int n_devices,
                                        const int *devices, int *error)
{
    int rc = fskd::validate_cfg(cfg);
    if (rc == DEMOD_OK && (n_streams < 1 || n_streams > ((size_t)1 << 24) || n_devices < 1 ||
                           n_devices > 64 || !devices))
        rc = DEMOD_BAD_ARG;
    if (rc != DEMOD_OK) {
        if (error) *error = rc;
        return nullptr;
    }
    DevRestore keep;
    demod_group_t *g = new (std::nothrow) demod_group();
    if (!g) {
        if (error) *error = DEMOD_ALLOC_FAIL;
        return nullptr;
    }
    g->cfg = *cfg;
    g->n_streams = n_streams;
    g->world = n_devices;
    g->ranks.resize(n_devices);
    for (int i = 0; i < n_devices && rc == DEMOD_OK; ++i) rc = init_rank(g, g->ranks[i], i, devices[i]);
    if (rc == DEMOD_OK) {
        std::vector<ncclComm_t> comms(n_devices);
        const ncclResult_t nr = ncclCommInitAll(comms.data(), n_devices, devices);
        if (nr != ncclSuccess) {
            std::fprintf(stderr, "fskdemod: ncclCommInitAll failed: %s\n", ncclGetErrorString(nr));
            rc = DEMOD_DEVICE_ERROR;
        } else {
            for (int i = 0; i < n_devices; ++i) g->ranks[i].comm = comms[i];
        }
    }
    if (rc != DEMOD_OK) {
        demod_group_destroy(g);
        if (error) *error = rc;
        return nullptr;
    }
    if (error) *error = DEMOD_OK;
    return g;
}

void demod_group_destroy(demod_group_t *g)
{
    if (!g) return;
    DevRestore keep;
    for (auto &r : g->ranks) free_rank(r);
    delete g;
}

int demod_group_world(const demod_group_t *g) { return g ? g->world : DEMOD_BAD_ARG; }

int demod_group_local_ranks(const demod_group_t *g) { return g ? (int)g->ranks.size() : DEMOD_BAD_ARG; }

int demod_group_rank_shard(const demod_group_t *g, int local, int *rank, size_t *first, size_t *count)
{
    if (!g || local < 0 || local >= (int)g->ranks.size()) return DEMOD_BAD_ARG;
    if (rank) *rank = g->ranks[local].rank;
    if (first) *first = g->ranks[local].first;
    if (count) *count = g->ranks[local].count;
    return DEMOD_OK;
}

int demod_group_push(demod_group_t *g, const int16_t *const *pcm, const size_t *n_frames, uint8_t *symbols,
                     size_t cap, uint32_t *counts)
{
    if (!g || !n_frames || !counts) return DEMOD_BAD_ARG;
    DevRestore keep;
    const int W = g->world, L = (int)g->ranks.size();
    const size_t ms = max_shard(g->n_streams, W);
    // this process's packets: every stream (local group) or the rank's shard
    const size_t base = L == 1 && W > 1 ? g->ranks[0].first : 0;
    // 1. every stream's symbol count (known before the kernels run), gathered
    for (auto &r : g->ranks) {
        r.h_counts.assign(ms, 0u);
        if (r.count && fskd::streams_counts(r.ms, n_frames + (r.first - base), r.h_counts.data()) < 0)
            return DEMOD_BAD_ARG;
        int rc = grow(r.d_send, r.send_cap, ms * 4);
        if (rc == DEMOD_OK) rc = grow(r.d_recv, r.recv_cap, ms * 4 * (size_t)W);
        if (rc != DEMOD_OK) return rc;
        HIP_TRY_G(hipSetDevice(r.device));
        HIP_TRY_G(hipMemcpyAsync(r.d_send, r.h_counts.data(), ms * 4, hipMemcpyHostToDevice, r.stream));
    }
    NCCL_TRY(ncclGroupStart());
    for (auto &r : g->ranks) {
        (void)hipSetDevice(r.device);
        NCCL_TRY(ncclAllGather(r.d_send, r.d_recv, ms, ncclUint32, r.comm, r.stream));
    }
    NCCL_TRY(ncclGroupEnd());
    GroupRank &r0 = g->ranks[0];
    g->h_counts_all.assign(ms * (size_t)W, 0u);
    HIP_TRY_G(hipSetDevice(r0.device));
    HIP_TRY_G(hipMemcpyAsync(g->h_counts_all.data(), r0.d_recv, ms * 4 * (size_t)W, hipMemcpyDeviceToHost,
                             r0.stream));
    for (auto &r : g->ranks) {
        HIP_TRY_G(hipSetDevice(r.device));
        HIP_TRY_G(hipStreamSynchronize(r.stream));
    }
    size_t total = 0, block = 0;
    for (int q = 0; q < W; ++q) {
        size_t f, cnt, t = 0;
        demod_group_shard(g->n_streams, q, W, &f, &cnt);
        for (size_t i = 0; i < cnt; ++i) t += g->h_counts_all[(size_t)q * ms + i];
        total += t;
        block = std::max(block, t);
    }
    if (total > cap) return DEMOD_BUFFER_TOO_SMALL;   // on every rank alike: nothing consumed
    if (total && !symbols) return DEMOD_BAD_ARG;
    // 2. each rank's push (its streams' carries and kernels), then its
    // symbols gathered as one padded block per rank
    for (auto &r : g->ranks) {
        r.h_sym.assign(std::max<size_t>(block, 1), 0);
        if (r.count) {
            std::vector<uint32_t> cnt(r.count);
            const int got = demod_streams_push(r.ms, pcm ? pcm + (r.first - base) : nullptr,
                                               n_frames + (r.first - base), r.h_sym.data(), nullptr,
                                               r.h_sym.size(), cnt.data());
            if (got < 0) return got;
        }
        int rc = grow(r.d_send, r.send_cap, std::max<size_t>(block, 1));
        if (rc == DEMOD_OK) rc = grow(r.d_recv, r.recv_cap, std::max<size_t>(block, 1) * (size_t)W);
        if (rc != DEMOD_OK) return rc;
        HIP_TRY_G(hipSetDevice(r.device));
        HIP_TRY_G(hipMemcpyAsync(r.d_send, r.h_sym.data(), std::max<size_t>(block, 1), hipMemcpyHostToDevice,
                                 r.stream));
    }
    if (block) {
        NCCL_TRY(ncclGroupStart());
        for (auto &r : g->ranks) {
            (void)hipSetDevice(r.device);
            NCCL_TRY(ncclAllGather(r.d_send, r.d_recv, block, ncclUint8, r.comm, r.stream));
        }
        NCCL_TRY(ncclGroupEnd());
        g->h_recv.resize(block * (size_t)W);
        HIP_TRY_G(hipSetDevice(r0.device));
        HIP_TRY_G(hipMemcpyAsync(g->h_recv.data(), r0.d_recv, block * (size_t)W, hipMemcpyDeviceToHost,
                                 r0.stream));
    }
    for (auto &r : g->ranks) {
        HIP_TRY_G(hipSetDevice(r.device));
        HIP_TRY_G(hipStreamSynchronize(r.stream));
    }
    // 3. stream-major: rank q's block holds its streams' symbols in order
    size_t o = 0;
    for (int q = 0; q < W; ++q) {
        size_t f, cnt, off = 0;
        demod_group_shard(g->n_streams, q, W, &f, &cnt);
        for (size_t i = 0; i < cnt; ++i) {
            const uint32_t c = g->h_counts_all[(size_t)q * ms + i];
            counts[f + i] = c;
            if (c) std::memcpy(symbols + o, g->h_recv.data() + (size_t)q * block + off, c);
            o += c;
            off += c;
        }
    }
    return (int)total;
}

long long demod_group_bucket_async(demod_group_t *g, const int16_t *const *d_pcm, size_t ring, size_t wps,
                                   size_t steps, uint8_t *const *d_all, void *const *streams)
{
    if (!g || !d_pcm || !d_all || ring < 1 || steps < 1 || steps % ring || wps < 1) return DEMOD_BAD_ARG;
    if (g->cfg.hop != g->cfg.n) return DEMOD_UNIMPLEMENTED;   // windows of a stream end to end
    DevRestore keep;
    const int W = g->world;
    const int bits = demod_bits_per_symbol(g->cfg.k);
    const long long stride = demod_frame_symbols_size(wps, bits, DEMOD_MAX_FRAME_PAYLOAD);
    const long long block = demod_group_block_bytes(g->n_streams, W, steps, wps, bits);
    if (stride < 0 || block < 0) return DEMOD_BAD_ARG;
    for (size_t l = 0; l < g->ranks.size(); ++l) {
        GroupRank &r = g->ranks[l];
        if (!d_all[l] || (r.count && !d_pcm[l])) return DEMOD_BAD_ARG;
        const size_t per = r.count * wps;   // windows per step
        int rc = grow(r.d_sym, r.sym_cap, std::max<size_t>(steps * per, 1));
        if (rc == DEMOD_OK) rc = grow(r.d_frames, r.frames_cap, (size_t)block);
        if (rc != DEMOD_OK) return rc;
        HIP_TRY_G(hipSetDevice(r.device));
        hipStream_t s = streams ? (hipStream_t)streams[l] : nullptr;
        for (size_t c = 0; per && c < steps / ring; ++c) {
            rc = demod_batch_async(r.st, d_pcm[l], ring * per, r.d_sym + c * ring * per, nullptr, s);
            if (rc < 0) return rc;
        }
        if (per) {
            const long long st = demod_frame_streams_async(r.d_sym, steps * r.count, wps, bits,
                                                           DEMOD_MAX_FRAME_PAYLOAD, r.d_frames, s);
            if (st < 0) return st;
        }
    }
    NCCL_TRY(ncclGroupStart());
    for (size_t l = 0; l < g->ranks.size(); ++l) {
        GroupRank &r = g->ranks[l];
        (void)hipSetDevice(r.device);
        NCCL_TRY(ncclAllGather(r.d_frames, d_all[l], (size_t)block, ncclUint8, r.comm,
                               streams ? (hipStream_t)streams[l] : nullptr));
    }
    NCCL_TRY(ncclGroupEnd());
    return block;
}

}  // extern "C"
