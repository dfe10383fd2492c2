// Host test of the rank path's scene hand-over protocol (audiorenderingv2_amd/csrc/arx_scene_share.hpp,
// used by arx_group_set_scene with one GPU per process): W ranks as threads over an in-memory
// transport whose collectives block until every rank has entered them -- so a rank that skips a
// collective makes the others wait, and the watchdog below turns that hang into a failure.
//
//   scene_share_test <case>   case: ok | root_fails | stage_fails | consume_fails | rank0_skips
// (rank0_skips: rank 0 returns without entering the collectives, as the round-3 code did when its
// input check failed -- the watchdog must report the hang)
// Prints one line per rank, "rank r: <result> <bytes>", exits 0 when every rank returned the expected
// result in time, 1 on a wrong result, 2 on a hang.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <algorithm>
#include <vector>

#include "arx_scene_share.hpp"

namespace {

constexpr int kRanks = 3;

// A barrier-based group: each collective is one generation; rank 0's value (bcast) or the max over
// ranks (max) is published when the last rank arrives.
struct Group {
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    uint64_t pending = 0;  // this generation's contributions ...
    std::vector<uint8_t> pending_bytes;
    uint64_t result = 0;   // ... published when the last rank arrives
    std::vector<uint8_t> bytes;

    // enter(pending, pending_bytes) under the lock; returns the published (result, bytes) of this
    // generation, read under the lock before any rank can start the next one
    template <class Enter>
    std::pair<uint64_t, std::vector<uint8_t>> collective(Enter enter) {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t my = gen;
        if (arrived == 0) {
            pending = 0;
            pending_bytes.clear();
        }
        enter(pending, pending_bytes);
        if (++arrived == kRanks) {
            result = pending;
            bytes = pending_bytes;
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != my; });
        }
        return {result, bytes};
    }
};

struct ThreadChannel {
    Group* g;
    int rank;
    bool fail_stage = false;
    std::vector<uint8_t> staged;

    bool bcast_u64(uint64_t* v) {
        const uint64_t mine = *v;
        *v = g->collective([&](uint64_t& p, std::vector<uint8_t>&) { if (rank == 0) p = mine; }).first;
        return true;
    }
    bool max_u64(uint64_t* v) {
        const uint64_t mine = *v;
        *v = g->collective([&](uint64_t& p, std::vector<uint8_t>&) { p = std::max(p, mine); }).first;
        return true;
    }
    bool stage(uint64_t bytes) {
        if (fail_stage) return false;
        staged.resize(bytes);
        return true;
    }
    bool bcast_bytes(uint8_t* host, uint64_t n) {
        const auto out = g->collective([&](uint64_t&, std::vector<uint8_t>& pb) {
            if (rank == 0) pb.assign(host, host + n);
        }).second;
        if (out.size() != n) return false;
        std::memcpy(host, out.data(), n);
        return true;
    }
};

const char* name(arx::ShareResult r) {
    switch (r) {
        case arx::ShareResult::ok: return "ok";
        case arx::ShareResult::root_failed: return "root_failed";
        case arx::ShareResult::staging_failed: return "staging_failed";
        case arx::ShareResult::consume_failed: return "consume_failed";
        case arx::ShareResult::transport_failed: return "transport_failed";
    }
    return "?";
}

}  // namespace

int main(int argc, char** argv) {
    const std::string mode = argc > 1 ? argv[1] : "ok";
    const arx::ShareResult want = mode == "ok"             ? arx::ShareResult::ok
                                  : mode == "root_fails"    ? arx::ShareResult::root_failed
                                  : mode == "stage_fails"   ? arx::ShareResult::staging_failed
                                  : mode == "consume_fails" ? arx::ShareResult::consume_failed
                                                            : arx::ShareResult::transport_failed;
    const std::vector<uint8_t> image = {'A', 'R', 'X', 'S', 'C', 'E', '1', 0, 1, 2, 3, 4, 5};
    Group g;
    std::vector<arx::ShareResult> res(kRanks, arx::ShareResult::transport_failed);
    std::vector<std::vector<uint8_t>> got(kRanks);
    std::atomic<int> done{0};
    std::vector<std::thread> th;
    for (int r = 0; r < kRanks; ++r)
        th.emplace_back([&, r] {
            ThreadChannel ch{&g, r};
            ch.fail_stage = mode == "stage_fails" && r == 2;
            if (mode == "rank0_skips" && r == 0) {  // the old protocol's early return: the others must hang
                done.fetch_add(1);
                return;
            }
            res[r] = arx::share_from_rank0(
                ch, r,
                [&](std::vector<uint8_t>& bytes) {  // rank 0: "invalid absorption" -> no image
                    if (mode == "root_fails") return false;
                    bytes = image;
                    return true;
                },
                [&](const std::vector<uint8_t>& bytes) {
                    got[r] = bytes;
                    return !(mode == "consume_fails" && r == 1);
                });
            done.fetch_add(1);
        });
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(10);
    while (done.load() < kRanks && std::chrono::steady_clock::now() < deadline)
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
    if (done.load() < kRanks) {
        std::printf("HANG: %d of %d ranks returned\n", done.load(), kRanks);
        std::fflush(stdout);
        std::_Exit(2);
    }
    for (auto& t : th) t.join();
    bool ok = true;
    for (int r = 0; r < kRanks; ++r) {
        std::printf("rank %d: %s %zu\n", r, name(res[r]), got[r].size());
        ok = ok && res[r] == want;
        if (want == arx::ShareResult::ok && r > 0) ok = ok && got[r] == image;
    }
    return ok ? 0 : 1;
}
