// demod_group.cpp — configs[4] as a service over RCCL, from the C ABI
// (include/demod.h demod_group_*). One process
// per GPU (ncclCommInitRank with rank 0's unique id, the `hipSetDevice +
// ncclCommInitRank` of SURVEY §7), or one process driving several GPUs
// (ncclCommInitAll; each rank then runs on a host thread of its own, so the
// GPUs work concurrently). Rank r of `world` owns the contiguous stream shard
// demod_group_shard(n_streams, r, world) and demodulates it on its own device;
// the only collectives carry the decoded result and the ranks' agreement
// (north_star: RCCL only for the final symbol gather):
//   * demod_group_push: one packet per stream (as demod_streams_push, whose
//     per-rank handle it wraps), run as group_flow.h's protocol: the ranks
//     all-gather [status | caps | per-stream counts] before anything is
//     consumed, agree on one verdict, push, all-gather the push status, then
//     the symbols (one padded block per rank). A refusal is returned by every
//     rank alike; a collective that fails or overruns the deadline aborts the
//     communicator (ncclCommAbort) and leaves the group dead, never hung;
//   * demod_group_bucket_async: the bench's configs[4] step as an ABI call,
//     device-resident: S steps' detector launches (over an input ring of R
//     steps' batches each), ONE device framing launch over the S steps'
//     symbol rows (demod_frame_streams_async), then one RCCL group of two
//     all-gathers on the caller's stream (so a caller can capture it in a HIP
//     graph): every rank's status word and the frames (a block of S x
//     ceil(n_streams / world) x frame stride per rank). A rank that fails
//     locally still posts both, carrying its code; demod_group_wait returns
//     the lowest failing rank's code on every rank.
// The reference fans one audio stream out to N receivers (MulticastAudioOutput
// .kt:88-96); here N GPUs each demodulate their share of many streams and
// gather the frames.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "../../include/demod.h"
#include "demod_internal.h"
#include "group_flow.h"
#include "plan.h"

namespace {

struct GroupRank {
    int device = 0, rank = 0;
    size_t first = 0, count = 0;        // the stream shard
    demod_streams_t *ms = nullptr;      // push path (per-stream carries)
    demod_t *st = nullptr;              // bucket path (device batches)
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;       // push path: copies + collectives
    // the agreement's words (allocated at create: the gathers that decide a
    // refusal never need an allocation): push [4 + ms] -> [world][4 + ms];
    // bucket status: [1] -> [world]
    uint32_t *d_words = nullptr, *d_words_all = nullptr;
    int32_t *d_bstat = nullptr, *d_bstat_all = nullptr;
    uint8_t *d_send = nullptr, *d_recv = nullptr;
    size_t send_cap = 0, recv_cap = 0;
    uint8_t *d_sym = nullptr, *d_frames = nullptr;   // bucket: [S][count * wps], [S * max_count * stride]
    size_t sym_cap = 0, frames_cap = 0;
    uint8_t *d_sink = nullptr;          // bucket: the frames of a call that passed no d_all
    size_t sink_cap = 0;
    std::vector<uint8_t> h_sym, h_recv;
    std::vector<uint32_t> h_words, h_all, h_cnt;
};

enum FailPhase { kFailNone = 0, kFailCheck, kFailPush, kFailBucket };

}  // namespace

struct demod_group {
    demod_cfg_t cfg;
    size_t n_streams = 0;
    int world = 1;
    std::vector<GroupRank> ranks;       // the ranks this process drives
    std::atomic<int> dead{0};           // the code that killed the group (0: alive)
    long long timeout_ms = 120000;      // FSKD_GROUP_TIMEOUT_MS: a collective's deadline
    int fail_phase = kFailNone, fail_rank = -1;   // FSKD_GROUP_FAIL=<check|push|bucket>:<rank> (tests)
};

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

size_t max_shard(size_t n_streams, int world) { return (n_streams + (size_t)world - 1) / (size_t)world; }

bool injected(const demod_group_t *g, int phase, int rank) { return g->fail_phase == phase && g->fail_rank == rank; }

void read_env(demod_group_t *g)
{
    if (const char *t = std::getenv("FSKD_GROUP_TIMEOUT_MS")) {
        const long long v = std::atoll(t);
        if (v > 0) g->timeout_ms = v;
    }
    if (const char *f = std::getenv("FSKD_GROUP_FAIL")) {
        static const struct { const char *name; int phase; } ph[] = {
            {"check:", kFailCheck}, {"push:", kFailPush}, {"bucket:", kFailBucket}};
        for (const auto &p : ph)
            if (std::strncmp(f, p.name, std::strlen(p.name)) == 0) {
                g->fail_phase = p.phase;
                g->fail_rank = std::atoi(f + std::strlen(p.name));
            }
    }
}

void free_rank(GroupRank &r)
{
    if (r.stream || r.comm) (void)hipSetDevice(r.device);
    if (r.stream) (void)hipStreamSynchronize(r.stream);
    if (r.comm) (void)ncclCommDestroy(r.comm);
    for (void *p : {(void *)r.d_send, (void *)r.d_recv, (void *)r.d_sym, (void *)r.d_frames, (void *)r.d_sink,
                    (void *)r.d_words, (void *)r.d_words_all, (void *)r.d_bstat, (void *)r.d_bstat_all})
        if (p) (void)hipFree(p);
    if (r.stream) (void)hipStreamDestroy(r.stream);
    if (r.ms) demod_streams_destroy(r.ms);
    if (r.st) demod_destroy(r.st);
    r = GroupRank();
}

// The group is dead: abort this rank's communicator (its pending collectives
// end instead of waiting for peers that will not come). Every later call
// returns DEMOD_INVALID_STATE; demod_group_destroy frees it.
void kill_rank(demod_group_t *g, GroupRank &r, int code)
{
    int expect = 0;
    (void)g->dead.compare_exchange_strong(expect, code < 0 ? code : DEMOD_DEVICE_ERROR);
    if (r.comm) {
        (void)hipSetDevice(r.device);
        (void)ncclCommAbort(r.comm);
        r.comm = nullptr;
    }
}

// Wait for `s` (a collective's stream) under the group's deadline, watching
// the communicator's asynchronous error: DEMOD_OK, or DEMOD_DEVICE_ERROR for
// a failed or overdue collective (the caller kills the group).
int wait_stream(const demod_group_t *g, const GroupRank &r, hipStream_t s)
{
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0;; ++spin) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return DEMOD_OK;
        if (e != hipErrorNotReady) {
            std::fprintf(stderr, "fskdemod: group rank %d: stream: %s\n", r.rank, hipGetErrorString(e));
            (void)hipGetLastError();
            return DEMOD_DEVICE_ERROR;
        }
        ncclResult_t ae = ncclSuccess;
        if (r.comm && ncclCommGetAsyncError(r.comm, &ae) == ncclSuccess && ae != ncclSuccess &&
            ae != ncclInProgress) {
            std::fprintf(stderr, "fskdemod: group rank %d: collective failed: %s\n", r.rank,
                         ncclGetErrorString(ae));
            return DEMOD_DEVICE_ERROR;
        }
        const auto ms =
            std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
        if (ms > g->timeout_ms) {
            std::fprintf(stderr, "fskdemod: group rank %d: collective not done after %lld ms (a peer failed?)\n",
                         r.rank, (long long)ms);
            return DEMOD_DEVICE_ERROR;
        }
        if (spin < 256) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
}

// A device buffer of >= need bytes on the rank's device, zero-filled in the
// order of `s`, the stream that uses it (gathered padding is defined).
int grow(const GroupRank &r, hipStream_t s, uint8_t *&p, size_t &cap, size_t need)
{
    if (need <= cap) return DEMOD_OK;
    HIP_TRY_G(hipSetDevice(r.device));
    // no allocation while `s` is being captured into a graph (it would
    // invalidate the capture): the caller sizes the buffers with one call of
    // the shape outside capture first
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) {
        (void)hipGetLastError();
        return DEMOD_DEVICE_ERROR;
    }
    if (cs != hipStreamCaptureStatusNone) return DEMOD_INVALID_STATE;
    if (p) {
        (void)hipStreamSynchronize(s);   // the old buffer may still be read
        (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
    const size_t n = need + need / 4 + 256;
    HIP_TRY_G(hipMalloc(&p, n));
    HIP_TRY_G(hipMemsetAsync(p, 0, n, s));
    cap = n;
    return DEMOD_OK;
}

// the per-rank handles and agreement buffers of rank r on device dev
// (communicator made by the caller)
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
    const size_t per = fskd::kGroupHeaderWords + max_shard(g->n_streams, g->world), W = (size_t)g->world;
    HIP_TRY_G(hipMalloc(&r.d_words, per * 4));
    HIP_TRY_G(hipMalloc(&r.d_words_all, per * 4 * W));
    HIP_TRY_G(hipMalloc(&r.d_bstat, 4));
    HIP_TRY_G(hipMalloc(&r.d_bstat_all, 4 * W));
    HIP_TRY_G(hipMemsetAsync(r.d_bstat_all, 0, 4 * W, r.stream));
    HIP_TRY_G(hipStreamSynchronize(r.stream));
    return DEMOD_OK;
}

// group_flow.h's operations for one rank of demod_group_push over RCCL
struct PushOps {
    demod_group_t *g;
    GroupRank &r;
    const int16_t *const *pcm;   // this rank's streams' packets
    const size_t *nf;

    int check(uint32_t *counts)
    {
        if (injected(g, kFailCheck, r.rank)) return DEMOD_INTERNAL_ERROR;
        if (!r.count) return DEMOD_OK;
        const long long w = fskd::streams_check(r.ms, pcm, nf, counts);
        return w < 0 ? (int)w : DEMOD_OK;
    }
    int gather_words(const uint32_t *send, size_t n, uint32_t *recv)
    {
        HIP_TRY_G(hipSetDevice(r.device));
        HIP_TRY_G(hipMemcpyAsync(r.d_words, send, n * 4, hipMemcpyHostToDevice, r.stream));
        const ncclResult_t nr = ncclAllGather(r.d_words, r.d_words_all, n, ncclUint32, r.comm, r.stream);
        if (nr != ncclSuccess) {
            std::fprintf(stderr, "fskdemod: ncclAllGather: %s\n", ncclGetErrorString(nr));
            return DEMOD_DEVICE_ERROR;
        }
        // the collective first, under the deadline (a copy to pageable host
        // memory would block on a collective a dead peer never finishes)
        const int w = wait_stream(g, r, r.stream);
        if (w != DEMOD_OK) return w;
        HIP_TRY_G(hipMemcpyAsync(recv, r.d_words_all, n * 4 * (size_t)g->world, hipMemcpyDeviceToHost, r.stream));
        HIP_TRY_G(hipStreamSynchronize(r.stream));
        return DEMOD_OK;
    }
    int push(size_t block)
    {
        if (injected(g, kFailPush, r.rank)) return DEMOD_DEVICE_ERROR;
        const size_t b = std::max<size_t>(block, 1);
        try {
            r.h_sym.assign(b, 0);
            r.h_cnt.resize(std::max<size_t>(r.count, 1));
        } catch (...) {
            return DEMOD_ALLOC_FAIL;
        }
        if (r.count) {
            const int got = demod_streams_push(r.ms, pcm, nf, r.h_sym.data(), nullptr, r.h_sym.size(), r.h_cnt.data());
            if (got < 0) return got;
        }
        int rc = grow(r, r.stream, r.d_send, r.send_cap, b);
        if (rc == DEMOD_OK) rc = grow(r, r.stream, r.d_recv, r.recv_cap, b * (size_t)g->world);
        if (rc != DEMOD_OK) return rc;
        HIP_TRY_G(hipSetDevice(r.device));
        HIP_TRY_G(hipMemcpyAsync(r.d_send, r.h_sym.data(), b, hipMemcpyHostToDevice, r.stream));
        return DEMOD_OK;
    }
    int gather_block(size_t block)
    {
        try {
            r.h_recv.resize(block * (size_t)g->world);
        } catch (...) {
            return DEMOD_ALLOC_FAIL;
        }
        HIP_TRY_G(hipSetDevice(r.device));
        const ncclResult_t nr = ncclAllGather(r.d_send, r.d_recv, block, ncclUint8, r.comm, r.stream);
        if (nr != ncclSuccess) {
            std::fprintf(stderr, "fskdemod: ncclAllGather: %s\n", ncclGetErrorString(nr));
            return DEMOD_DEVICE_ERROR;
        }
        const int w = wait_stream(g, r, r.stream);
        if (w != DEMOD_OK) return w;
        HIP_TRY_G(hipMemcpyAsync(r.h_recv.data(), r.d_recv, block * (size_t)g->world, hipMemcpyDeviceToHost,
                                 r.stream));
        HIP_TRY_G(hipStreamSynchronize(r.stream));
        return DEMOD_OK;
    }
    void kill(int code) { kill_rank(g, r, code); }
};

// fn(local rank) for every rank this process drives, concurrently (one host
// thread per rank beyond the first; the caller's thread runs rank 0). Returns
// the ranks' common result (they agree by construction; a disagreement is
// reported as DEMOD_INTERNAL_ERROR).
template <class F>
long long each_rank(demod_group_t *g, F fn_)
{
    // no exception leaves a rank's thread or the C ABI: a host allocation
    // that fails inside the flow ends that rank with DEMOD_ALLOC_FAIL (its
    // peers then meet the missing rank at their deadline and abort)
    auto fn = [&](size_t l) -> long long {
        try {
            return fn_(l);
        } catch (...) {
            kill_rank(g, g->ranks[l], DEMOD_ALLOC_FAIL);
            return DEMOD_ALLOC_FAIL;
        }
    };
    const size_t L = g->ranks.size();
    std::vector<long long> rc(L, DEMOD_OK);
    std::vector<std::thread> th;
    try {
        for (size_t l = 1; l < L; ++l) th.emplace_back([&, l] { rc[l] = fn(l); });
    } catch (...) {
        for (auto &t : th) t.join();
        return DEMOD_ALLOC_FAIL;   // no rank has gathered yet: the threads that started wait in the
                                   // first gather until their deadline, then kill the group
    }
    rc[0] = fn(0);
    for (auto &t : th) t.join();
    for (size_t l = 1; l < L; ++l)
        if (rc[l] != rc[0]) return DEMOD_INTERNAL_ERROR;
    return rc[0];
}

}  // namespace

extern "C" {

int demod_group_unique_id(uint8_t *id)
{
    if (!id) return DEMOD_BAD_ARG;
    static_assert(sizeof(ncclUniqueId) == DEMOD_GROUP_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    const ncclResult_t nr = ncclGetUniqueId(&u);
    if (nr != ncclSuccess) {
        std::fprintf(stderr, "fskdemod: ncclGetUniqueId: %s\n", ncclGetErrorString(nr));
        return DEMOD_DEVICE_ERROR;
    }
    std::memcpy(id, &u, sizeof(u));
    return DEMOD_OK;
}

int demod_group_shard(size_t n_streams, int rank, int world, size_t *first, size_t *count)
{
    if (world < 1 || rank < 0 || rank >= world || !first || !count) return DEMOD_BAD_ARG;
    fskd::group_shard_of(n_streams, rank, world, first, count);
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
    read_env(g);
    g->ranks.resize(1);
    rc = init_rank(g, g->ranks[0], rank, cfg->device);
    // ncclCommInitRank is itself collective: a rank whose handles failed
    // still joins it (other ranks would wait in it), then destroys the
    // communicator; its peers' first gather meets the missing rank at its
    // deadline
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    (void)hipSetDevice(cfg->device);
    const ncclResult_t nr = ncclCommInitRank(&g->ranks[0].comm, world, u, rank);
    if (nr != ncclSuccess) {
        std::fprintf(stderr, "fskdemod: ncclCommInitRank failed: %s\n", ncclGetErrorString(nr));
        g->ranks[0].comm = nullptr;
        if (rc == DEMOD_OK) rc = DEMOD_DEVICE_ERROR;
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
    read_env(g);
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

int demod_group_rank_device(const demod_group_t *g, int local)
{
    if (!g || local < 0 || local >= (int)g->ranks.size()) return DEMOD_BAD_ARG;
    return g->ranks[local].device;
}

int demod_group_status(const demod_group_t *g)
{
    if (!g) return DEMOD_BAD_ARG;
    return g->dead.load();
}

int demod_group_push(demod_group_t *g, const int16_t *const *pcm, const size_t *n_frames, uint8_t *symbols,
                     size_t cap, uint32_t *counts)
{
    if (!g || !n_frames || !counts) return DEMOD_BAD_ARG;   // the same on every rank: a caller bug
    if (g->dead.load()) return DEMOD_INVALID_STATE;
    DevRestore keep;
    const int W = g->world, L = (int)g->ranks.size();
    const size_t ms = max_shard(g->n_streams, W);
    // this process's packets: every stream (local group) or the rank's shard
    const size_t base = L == 1 && W > 1 ? g->ranks[0].first : 0;
    std::vector<size_t> blocks((size_t)L, 0);
    const long long rc = each_rank(g, [&](size_t l) -> long long {
        GroupRank &r = g->ranks[l];
        PushOps o{g, r, pcm ? pcm + (r.first - base) : nullptr, n_frames + (r.first - base)};
        return fskd::group_push_flow(o, W, g->n_streams, ms, symbols, cap, r.h_words, r.h_all, &blocks[l]);
    });
    if (rc < 0) return (int)rc;
    // stream-major: rank q's block holds its streams' symbols in order
    const GroupRank &r0 = g->ranks[0];
    const size_t per = fskd::kGroupHeaderWords + ms, block = blocks[0];
    size_t o = 0;
    for (int q = 0; q < W; ++q) {
        size_t f, cnt, off = 0;
        fskd::group_shard_of(g->n_streams, q, W, &f, &cnt);
        for (size_t i = 0; i < cnt; ++i) {
            const uint32_t c = r0.h_all[(size_t)q * per + fskd::kGroupHeaderWords + i];
            counts[f + i] = c;
            if (c) std::memcpy(symbols + o, r0.h_recv.data() + (size_t)q * block + off, c);
            o += c;
            off += c;
        }
    }
    return (int)rc;
}

long long demod_group_bucket_async(demod_group_t *g, const int16_t *const *d_pcm, size_t ring, size_t wps,
                                   size_t steps, uint8_t *const *d_all, void *const *streams)
{
    // the call's shape is the same on every rank (the contract of a
    // collective): a refusal of the shape is every rank's alike
    if (!g || !d_pcm || !d_all || ring < 1 || steps < 1 || steps % ring || wps < 1) return DEMOD_BAD_ARG;
    if (g->dead.load()) return DEMOD_INVALID_STATE;
    if (g->cfg.hop != g->cfg.n) return DEMOD_UNIMPLEMENTED;   // windows of a stream end to end
    DevRestore keep;
    const int W = g->world, L = (int)g->ranks.size();
    const int bits = demod_bits_per_symbol(g->cfg.k);
    const long long stride = demod_frame_symbols_size(wps, bits, DEMOD_MAX_FRAME_PAYLOAD);
    const long long block = demod_group_block_bytes(g->n_streams, W, steps, wps, bits);
    if (stride < 0 || block < 0) return DEMOD_BAD_ARG;
    // 1. sizing: every rank's buffers hold the call's shape before anything is
    // enqueued. Under capture nothing may allocate: a call of a new shape is
    // refused there, before anything is enqueued, with DEMOD_INVALID_STATE
    // (every rank shares the call history of the contract, so every rank
    // refuses alike). Outside capture, a rank that cannot hold its frames
    // cannot join the gather: the group is killed below.
    int sized = DEMOD_OK;
    for (int l = 0; l < L && sized == DEMOD_OK; ++l) {
        GroupRank &r = g->ranks[l];
        hipStream_t s = streams ? (hipStream_t)streams[l] : nullptr;
        sized = grow(r, s, r.d_sym, r.sym_cap, std::max<size_t>(steps * r.count * wps, 1));
        if (sized == DEMOD_OK) sized = grow(r, s, r.d_frames, r.frames_cap, (size_t)block);
        if (sized == DEMOD_OK && !d_all[l]) sized = grow(r, s, r.d_sink, r.sink_cap, (size_t)block * (size_t)W);
    }
    if (sized == DEMOD_INVALID_STATE) return sized;
    if (sized != DEMOD_OK) {
        for (auto &r : g->ranks) kill_rank(g, r, sized);
        return sized;
    }
    // 2. each rank's own work; a rank that fails still posts both gathers
    // below, with its code as the status word
    std::vector<int> st((size_t)L, DEMOD_OK);
    std::vector<uint8_t *> dst((size_t)L, nullptr);
    for (int l = 0; l < L; ++l) {
        GroupRank &r = g->ranks[l];
        hipStream_t s = streams ? (hipStream_t)streams[l] : nullptr;
        int rc = injected(g, kFailBucket, r.rank) ? DEMOD_INTERNAL_ERROR : DEMOD_OK;
        if (rc == DEMOD_OK && r.count && !d_pcm[l]) rc = DEMOD_BAD_ARG;
        if (rc == DEMOD_OK && !d_all[l]) rc = DEMOD_BAD_ARG;
        dst[l] = d_all[l] ? d_all[l] : r.d_sink;
        const size_t per = r.count * wps;   // windows per step
        if (hipSetDevice(r.device) != hipSuccess && rc == DEMOD_OK) rc = DEMOD_DEVICE_ERROR;
        for (size_t c = 0; rc == DEMOD_OK && per && c < steps / ring; ++c) {
            const int b = demod_batch_async(r.st, d_pcm[l], ring * per, r.d_sym + c * ring * per, nullptr, s);
            if (b < 0) rc = b;
        }
        if (rc == DEMOD_OK && per) {
            const long long f = demod_frame_streams_async(r.d_sym, steps * r.count, wps, bits,
                                                          DEMOD_MAX_FRAME_PAYLOAD, r.d_frames, s);
            if (f < 0) rc = (int)f;
        }
        (void)hipSetDevice(r.device);
        if (hipMemsetD32Async(r.d_bstat, (int)rc, 1, s) != hipSuccess && rc == DEMOD_OK) rc = DEMOD_DEVICE_ERROR;
        st[l] = rc;
    }
    // both gathers of every local rank, in one RCCL group (always closed)
    bool posted = true;
    ncclResult_t nr = ncclGroupStart();
    if (nr == ncclSuccess) {
        for (int l = 0; l < L; ++l) {
            GroupRank &r = g->ranks[l];
            hipStream_t s = streams ? (hipStream_t)streams[l] : nullptr;
            if (!r.comm) {
                posted = false;
                continue;
            }
            (void)hipSetDevice(r.device);
            ncclResult_t a = ncclAllGather(r.d_bstat, r.d_bstat_all, 1, ncclInt32, r.comm, s);
            if (a == ncclSuccess) a = ncclAllGather(r.d_frames, dst[l], (size_t)block, ncclUint8, r.comm, s);
            if (a != ncclSuccess) {
                std::fprintf(stderr, "fskdemod: ncclAllGather: %s\n", ncclGetErrorString(a));
                posted = false;
            }
        }
        nr = ncclGroupEnd();
    }
    if (nr != ncclSuccess || !posted) {
        // a rank could not join the collectives: its peers would wait for it
        // forever, so the communicators are aborted and the group is dead
        if (nr != ncclSuccess) std::fprintf(stderr, "fskdemod: ncclGroup: %s\n", ncclGetErrorString(nr));
        for (auto &r : g->ranks) kill_rank(g, r, DEMOD_DEVICE_ERROR);
        return DEMOD_DEVICE_ERROR;
    }
    for (int l = 0; l < L; ++l)
        if (st[l] != DEMOD_OK) return st[l];
    return block;
}

int demod_group_wait(demod_group_t *g, void *const *streams)
{
    if (!g) return DEMOD_BAD_ARG;
    if (g->dead.load()) return DEMOD_INVALID_STATE;
    DevRestore keep;
    const int W = g->world;
    for (size_t l = 0; l < g->ranks.size(); ++l) {
        GroupRank &r = g->ranks[l];
        hipStream_t s = streams ? (hipStream_t)streams[l] : nullptr;
        (void)hipSetDevice(r.device);
        if (wait_stream(g, r, s) != DEMOD_OK) {
            for (auto &q : g->ranks) kill_rank(g, q, DEMOD_DEVICE_ERROR);
            return DEMOD_DEVICE_ERROR;
        }
    }
    // every rank's status word of the last bucket (identical on every rank)
    GroupRank &r0 = g->ranks[0];
    std::vector<int32_t> sts((size_t)W, 0);
    HIP_TRY_G(hipSetDevice(r0.device));
    HIP_TRY_G(hipMemcpyAsync(sts.data(), r0.d_bstat_all, 4 * (size_t)W, hipMemcpyDeviceToHost, r0.stream));
    HIP_TRY_G(hipStreamSynchronize(r0.stream));
    return fskd::group_first_failure(sts.data(), W);
}

}  // extern "C"
