// The group's agreement protocol (audio-network_amd/csrc/group_flow.h, the
// template demod_group_push runs over RCCL) run here over threads: each rank
// is a thread, the all-gathers are an in-process exchange with a deadline,
// and failures are injected per rank and per phase. For every scenario every
// rank must return the same code, the push must not run on any rank when a
// refusal is decided before it, and no rank may wait past the deadline (a
// dead peer turns into DEMOD_DEVICE_ERROR + kill, not a hang). No device.
// Exit 0 = OK.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../../audio-network_amd/csrc/group_flow.h"

namespace {

// an all-gather of n words per rank among `world` threads; a rank that is not
// there by the deadline makes the others' gathers fail (DEMOD_DEVICE_ERROR)
struct Exchange {
    std::mutex mu;
    std::condition_variable cv;
    int world;
    int arrived = 0;
    unsigned gen = 0;
    size_t n = 0;
    std::vector<uint32_t> buf, done;
    explicit Exchange(int w) : world(w) {}

    int gather(int rank, const uint32_t *send, size_t nw, uint32_t *recv, int timeout_ms)
    {
        std::unique_lock<std::mutex> lk(mu);
        if (arrived == 0) {
            n = nw;
            buf.assign(nw * (size_t)world, 0xDEADBEEFu);
        }
        if (nw != n) return DEMOD_INTERNAL_ERROR;   // ranks disagree on a collective's size
        std::memcpy(buf.data() + (size_t)rank * nw, send, nw * 4);
        const unsigned my = gen;
        if (++arrived == world) {
            done = buf;
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else if (!cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return gen != my; })) {
            return DEMOD_DEVICE_ERROR;   // a peer never came: the deadline
        }
        std::memcpy(recv, done.data(), nw * 4 * (size_t)world);
        return DEMOD_OK;
    }
};

struct RankPlan {
    int check_rc = DEMOD_OK;
    int push_rc = DEMOD_OK;
    bool absent = false;          // the rank's process died before the call
    bool null_symbols = false;
    size_t cap = 1u << 30;
    std::vector<uint32_t> counts; // its shard's streams
};

struct FakeOps {
    Exchange &ex;
    int rank;
    const RankPlan &p;
    int timeout_ms;
    std::atomic<int> &pushes;
    bool killed = false;
    int kill_code = 0;

    int check(uint32_t *counts)
    {
        for (size_t i = 0; i < p.counts.size(); ++i) counts[i] = p.counts[i];
        return p.check_rc;
    }
    int gather_words(const uint32_t *send, size_t n, uint32_t *recv) { return ex.gather(rank, send, n, recv, timeout_ms); }
    int push(size_t)
    {
        pushes.fetch_add(1);
        return p.push_rc;
    }
    int gather_block(size_t block)
    {
        const size_t w = (block + 3) / 4;
        std::vector<uint32_t> s(w, (uint32_t)rank), r(w * (size_t)ex.world);
        const int rc = ex.gather(rank, s.data(), w, r.data(), timeout_ms);
        if (rc != DEMOD_OK) return rc;
        for (int q = 0; q < ex.world; ++q)
            if (r[(size_t)q * w] != (uint32_t)q) return DEMOD_INTERNAL_ERROR;
        return DEMOD_OK;
    }
    void kill(int code)
    {
        killed = true;
        kill_code = code;
    }
};

struct Outcome {
    std::vector<int> rc;
    std::vector<char> killed;   // not vector<bool>: ranks write their own entries concurrently
    int pushes = 0;
    double seconds = 0;
};

Outcome run(int world, size_t n_streams, const std::vector<RankPlan> &plans, int timeout_ms)
{
    Exchange ex(world);
    std::atomic<int> pushes{0};
    Outcome o;
    o.rc.assign((size_t)world, 1);
    o.killed.assign((size_t)world, 0);
    const size_t ms = (n_streams + (size_t)world - 1) / (size_t)world;
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int q = 0; q < world; ++q)
        th.emplace_back([&, q] {
            const RankPlan &p = plans[(size_t)q];
            if (p.absent) return;
            FakeOps ops{ex, q, p, timeout_ms, pushes};
            std::vector<uint32_t> words, all;
            size_t block = 0;
            static uint8_t sink[1];
            o.rc[(size_t)q] = fskd::group_push_flow(ops, world, n_streams, ms, p.null_symbols ? nullptr : sink,
                                                     p.cap, words, all, &block);
            o.killed[(size_t)q] = ops.killed;
        });
    for (auto &t : th) t.join();
    o.pushes = pushes.load();
    o.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return o;
}

std::vector<RankPlan> plans_for(int world, size_t n_streams, std::mt19937 &rng, uint32_t max_count)
{
    std::vector<RankPlan> ps((size_t)world);
    for (int q = 0; q < world; ++q) {
        size_t f, c;
        fskd::group_shard_of(n_streams, q, world, &f, &c);
        ps[(size_t)q].counts.resize(c);
        for (auto &x : ps[(size_t)q].counts) x = (uint32_t)(rng() % (max_count + 1));
    }
    return ps;
}

int failures = 0;

#define EXPECT(c, ...)                                                        \
    do {                                                                      \
        if (!(c)) {                                                           \
            std::fprintf(stderr, "group_flow_test:%d: %s: ", __LINE__, #c);   \
            std::fprintf(stderr, __VA_ARGS__);                                \
            std::fprintf(stderr, "\n");                                       \
            ++failures;                                                       \
        }                                                                     \
    } while (0)

// every present rank returned `code`
bool all_equal(const Outcome &o, const std::vector<RankPlan> &p, int code)
{
    for (size_t q = 0; q < o.rc.size(); ++q)
        if (!p[q].absent && o.rc[q] != code) return false;
    return true;
}

unsigned long long total_of(const std::vector<RankPlan> &p)
{
    unsigned long long t = 0;
    for (const auto &r : p)
        for (uint32_t c : r.counts) t += c;
    return t;
}

}  // namespace

int main()
{
    std::mt19937 rng(20261018);
    const int T = 20000;  // ms: the deadline of the healthy scenarios (never reached; generous for loaded CI hosts)
    for (int world : {1, 2, 3, 8}) {
        const size_t n_streams = 37;
        // all healthy: the total on every rank, one push each
        {
            auto p = plans_for(world, n_streams, rng, 9);
            const Outcome o = run(world, n_streams, p, T);
            EXPECT(all_equal(o, p, (int)total_of(p)) && o.pushes == world, "world %d healthy", world);
        }
        // one rank refuses its arguments: every rank returns its code, nothing pushed
        for (int bad = 0; bad < world; ++bad) {
            auto p = plans_for(world, n_streams, rng, 9);
            p[(size_t)bad].check_rc = DEMOD_BAD_ARG;
            const Outcome o = run(world, n_streams, p, T);
            EXPECT(all_equal(o, p, DEMOD_BAD_ARG) && o.pushes == 0, "world %d check fail on %d", world, bad);
            EXPECT(std::none_of(o.killed.begin(), o.killed.end(), [](char k) { return k != 0; }), "refusal killed");
        }
        // two ranks refuse with different codes: the lowest rank's code everywhere
        if (world >= 3) {
            auto p = plans_for(world, n_streams, rng, 9);
            p[2].check_rc = DEMOD_BAD_ARG;
            p[1].check_rc = DEMOD_INTERNAL_ERROR;
            const Outcome o = run(world, n_streams, p, T);
            EXPECT(all_equal(o, p, DEMOD_INTERNAL_ERROR) && o.pushes == 0, "world %d lowest rank", world);
        }
        // one rank's cap too small (its own buffer): every rank refuses
        {
            auto p = plans_for(world, n_streams, rng, 9);
            const unsigned long long t = total_of(p);
            if (t > 0) {
                p[(size_t)(world - 1)].cap = (size_t)t - 1;
                const Outcome o = run(world, n_streams, p, T);
                EXPECT(all_equal(o, p, DEMOD_BUFFER_TOO_SMALL) && o.pushes == 0, "world %d cap", world);
            }
        }
        // a NULL symbols buffer on one rank (the total is non-zero)
        {
            auto p = plans_for(world, n_streams, rng, 9);
            p[0].counts[0] = 3;
            p[0].null_symbols = true;
            const Outcome o = run(world, n_streams, p, T);
            EXPECT(all_equal(o, p, DEMOD_BAD_ARG) && o.pushes == 0, "world %d null symbols", world);
        }
        // a total above INT_MAX (each rank's own count fits): refused everywhere
        {
            auto p = plans_for(world, n_streams, rng, 9);
            for (auto &r : p)
                for (auto &c : r.counts) c = 0x7FFFFFFFu / (uint32_t)n_streams + 1000000u;
            const Outcome o = run(world, n_streams, p, T);
            EXPECT(all_equal(o, p, DEMOD_BAD_ARG) && o.pushes == 0, "world %d > INT_MAX", world);
        }
        // a push fails on one rank after the agreement: every rank returns its
        // code and every rank killed the group (some carries advanced)
        for (int bad = 0; bad < world; ++bad) {
            auto p = plans_for(world, n_streams, rng, 9);
            p[(size_t)bad].push_rc = DEMOD_DEVICE_ERROR;
            const Outcome o = run(world, n_streams, p, T);
            EXPECT(all_equal(o, p, DEMOD_DEVICE_ERROR) && o.pushes == world, "world %d push fail", world);
            EXPECT(std::all_of(o.killed.begin(), o.killed.end(), [](char k) { return k != 0; }), "push fail not killed");
        }
        // a dead peer (its process is gone): the others end at the deadline,
        // DEMOD_DEVICE_ERROR, killed, well before a hang
        if (world >= 2) {
            auto p = plans_for(world, n_streams, rng, 9);
            p[(size_t)(world / 2)].absent = true;
            const Outcome o = run(world, n_streams, p, 200);
            EXPECT(all_equal(o, p, DEMOD_DEVICE_ERROR) && o.pushes == 0 && o.seconds < 5.0,
                   "world %d dead peer (%.2f s)", world, o.seconds);
            for (int q = 0; q < world; ++q)
                EXPECT(p[(size_t)q].absent || o.killed[(size_t)q], "dead peer: rank %d not killed", q);
        }
    }
    // random fault plans: the same code on every rank, the one predicted
    const int codes[] = {DEMOD_BAD_ARG, DEMOD_INTERNAL_ERROR, DEMOD_ALLOC_FAIL, DEMOD_DEVICE_ERROR};
    for (int it = 0; it < 300; ++it) {
        const int world = 1 + (int)(rng() % 8);
        const size_t n_streams = 1 + rng() % 50;
        auto p = plans_for(world, n_streams, rng, 5);
        int expect_check = DEMOD_OK, expect_push = DEMOD_OK;
        for (int q = 0; q < world; ++q) {
            if (rng() % 6 == 0) p[(size_t)q].check_rc = codes[rng() % 4];
            if (rng() % 6 == 0) p[(size_t)q].push_rc = codes[rng() % 4];
            if (expect_check == DEMOD_OK) expect_check = p[(size_t)q].check_rc;
            if (expect_push == DEMOD_OK) expect_push = p[(size_t)q].push_rc;
        }
        const int expect = expect_check != DEMOD_OK ? expect_check
                           : expect_push != DEMOD_OK ? expect_push
                                                     : (int)total_of(p);
        const Outcome o = run(world, n_streams, p, T);
        EXPECT(all_equal(o, p, expect), "random %d: world %d expect %d got %d", it, world, expect, o.rc[0]);
        EXPECT(o.pushes == (expect_check != DEMOD_OK ? 0 : world), "random %d pushes %d", it, o.pushes);
    }
    if (failures) {
        std::fprintf(stderr, "group_flow_test: %d failure(s)\n", failures);
        return 1;
    }
    std::printf("group flow OK\n");
    return 0;
}
