// group_flow.h — how the ranks of a demod_group agree (host only: no HIP, no
// RCCL; VERDICT r5 item 1, SURVEY.md §8b "errors map to negative codes").
//
// A rank that leaves a collective protocol alone hangs its peers in the next
// collective, so demod_group_push is written as one flow every rank runs to
// the same end: every refusal is decided from all-gathered data, which is
// identical on every rank, and a rank that fails locally still joins each
// collective, carrying its error instead of its data.
//
//   1. local checks, no side effects (Ops::check: demod_streams_push's own
//      argument refusals and the per-stream counts);
//   2. all-gather #1 of [status, symbols == NULL, cap] + the counts (fixed
//      size, buffers allocated at create: nothing can fail to allocate here);
//   3. group_verdict over the gathered words: the lowest failing rank's code,
//      else the totals' checks (> INT_MAX, > the smallest cap, a NULL symbols
//      buffer). A refusal here returns on every rank alike with nothing consumed;
//   4. the push (carries advance) and all-gather #2 of its status;
//   5. if any rank's push failed, every rank returns that code and the group
//      is dead (some carries advanced, so it cannot be resumed: the caller
//      destroys it); else all-gather #3 of the symbols, padded per rank.
// A collective that itself fails or does not finish within the group's
// deadline (a peer process died) ends in Ops::kill (ncclCommAbort): the group
// is dead and the call returns DEMOD_DEVICE_ERROR instead of hanging.
//
// demod_group.cpp runs it over RCCL and the rank's demod_streams handle;
// tests/native/group_flow_test.cpp runs the same template over threads with
// injected failures (every rank returns the same code, no rank waits).
#pragma once
#include <climits>
#include <cstddef>
#include <cstdint>
#include <vector>

#include "../../include/demod.h"

namespace fskd {

// all-gather #1's words per rank: the header, then ceil(n_streams / world) counts
constexpr size_t kGroupHeaderWords = 4;   // status, symbols == NULL, cap low, cap high

inline void group_shard_of(size_t n_streams, int rank, int world, size_t *first, size_t *count)
{
    const size_t base = n_streams / (size_t)world, extra = n_streams % (size_t)world;
    *first = (size_t)rank * base + ((size_t)rank < extra ? (size_t)rank : extra);
    *count = base + ((size_t)rank < extra ? 1 : 0);
}

// The lowest rank's negative status, else DEMOD_OK (identical on every rank
// that holds the same gathered words).
inline int group_first_failure(const int32_t *status, int world, size_t stride_words = 1)
{
    for (int q = 0; q < world; ++q) {
        const int32_t s = status[(size_t)q * stride_words];
        if (s < 0) return s;
        if (s > 0) return DEMOD_INTERNAL_ERROR;   // not a code any rank sends
    }
    return DEMOD_OK;
}

// Step 3: the verdict from all-gather #1's words ([world][4 + ms]). On
// DEMOD_OK, *total = every stream's symbols, *block = the largest rank's.
inline int group_verdict(const uint32_t *all, int world, size_t n_streams, size_t ms, size_t *total,
                         size_t *block)
{
    const size_t per = kGroupHeaderWords + ms;
    const int bad = group_first_failure(reinterpret_cast<const int32_t *>(all), world, per);
    if (bad != DEMOD_OK) return bad;
    unsigned long long tot = 0, blk = 0, cap = ~0ull;
    bool null_sym = false;
    for (int q = 0; q < world; ++q) {
        const uint32_t *h = all + (size_t)q * per;
        size_t f, cnt;
        group_shard_of(n_streams, q, world, &f, &cnt);
        unsigned long long t = 0;
        for (size_t i = 0; i < cnt && i < ms; ++i) t += h[kGroupHeaderWords + i];
        tot += t;
        blk = t > blk ? t : blk;
        const unsigned long long c = (unsigned long long)h[2] | ((unsigned long long)h[3] << 32);
        cap = c < cap ? c : cap;
        null_sym = null_sym || h[1] != 0;
    }
    if (tot > (unsigned long long)INT_MAX) return DEMOD_BAD_ARG;   // the return value must stay a count
    if (tot > cap) return DEMOD_BUFFER_TOO_SMALL;
    if (tot && null_sym) return DEMOD_BAD_ARG;
    *total = (size_t)tot;
    *block = (size_t)blk;
    return DEMOD_OK;
}

// One rank's header of all-gather #1.
inline void group_header(int32_t status, const void *symbols, size_t cap, uint32_t *h)
{
    h[0] = (uint32_t)status;
    h[1] = symbols ? 0u : 1u;
    const unsigned long long c = (unsigned long long)cap;
    h[2] = (uint32_t)(c & 0xFFFFFFFFu);
    h[3] = (uint32_t)(c >> 32);
}

// The flow of one rank (steps 1-5). Ops (one rank's view):
//   int  check(uint32_t *counts)                  local refusal or DEMOD_OK, no side effects;
//                                                 counts[0 .. ms) (zero past the shard)
//   int  gather_words(const uint32_t *send, size_t n, uint32_t *recv)
//                                                 all-gather of n words per rank; DEMOD_OK or
//                                                 the transport's failure (after its deadline)
//   int  push(size_t block)                       the rank's push, its symbols padded to block
//                                                 bytes staged for gather_block
//   int  gather_block(size_t block)               all-gather of the padded blocks
//   void kill(int code)                           the group is dead (abort the transport)
// words / all: scratch of 4 + ms and world x (4 + ms) words. Returns the
// total (>= 0) or the code every rank returns; *block_out the padded block.
template <class Ops>
int group_push_flow(Ops &o, int world, size_t n_streams, size_t ms, const void *symbols, size_t cap,
                    std::vector<uint32_t> &words, std::vector<uint32_t> &all, size_t *block_out)
{
    const size_t per = kGroupHeaderWords + ms;
    words.assign(per, 0u);
    all.assign(per * (size_t)world, 0u);
    // 1-2: local checks, then the header + counts gathered
    const int local = o.check(words.data() + kGroupHeaderWords);
    if (local != DEMOD_OK)
        for (size_t i = 0; i < ms; ++i) words[kGroupHeaderWords + i] = 0;
    group_header(local, symbols, cap, words.data());
    int rc = o.gather_words(words.data(), per, all.data());
    if (rc != DEMOD_OK) {
        o.kill(rc);
        return rc;
    }
    // 3: the same verdict on every rank
    size_t total = 0, block = 0;
    rc = group_verdict(all.data(), world, n_streams, ms, &total, &block);
    if (rc != DEMOD_OK) return rc;
    // 4: the push, and its status gathered (a rank that failed still joins)
    uint32_t st = (uint32_t)o.push(block);
    std::vector<uint32_t> sts((size_t)world, 0u);
    rc = o.gather_words(&st, 1, sts.data());
    if (rc != DEMOD_OK) {
        o.kill(rc);
        return rc;
    }
    rc = group_first_failure(reinterpret_cast<const int32_t *>(sts.data()), world);
    if (rc != DEMOD_OK) {
        o.kill(rc);   // some ranks' carries advanced: the group cannot go on
        return rc;
    }
    // 5: the symbols
    if (block) {
        rc = o.gather_block(block);
        if (rc != DEMOD_OK) {
            o.kill(rc);
            return rc;
        }
    }
    *block_out = block;
    return (int)total;
}

}  // namespace fskd
