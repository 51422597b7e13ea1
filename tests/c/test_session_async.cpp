// Host-mode sessions of np ranks as threads of one process: every rank starts
// the same named async all-reduces (kf_session_all_reduce_async) in its OWN
// random order, two steps back to back, then one blocking all-reduce; every
// result is checked exactly (int32 sums). The reference runs each
// GoKungfuAllReduce on its own goroutine and pairs peers' messages by name
// (srcs/go/libkungfu-comm/collective.go:34-45, rchannel/handler/
// collective.go:48-64), so any start order per rank must work.
//
// Built by tests/test_c_consumer.py against libkungfu_amd.so, and by
// tools/sanitize_session.sh against ThreadSanitizer / AddressSanitizer builds
// of the same sources (host code only; host mode makes no HIP call).
//
// "dead" as a fourth argument: the last rank destroys its session once every
// rank's session is up (its connections close: EOF at every peer) and the
// others' async all-reduces must FAIL within 30 s, not hang (kf_session.hip's
// poll loop fails every call still waiting for a message from a closed peer).
//
//   test_session_async <np> <steps> <sock_dir> [dead]
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "kungfu_amd.h"

namespace
{
int fold_i32(const void *own, const void *peer, void *dst, int64_t n, int dt, int op)
{
    if (dt != KungFu_INT32 || op != KungFu_SUM) return 1;
    const int32_t *a = static_cast<const int32_t *>(own);
    const int32_t *b = static_cast<const int32_t *>(peer);
    int32_t *z       = static_cast<int32_t *>(dst);
    for (int64_t i = 0; i < n; ++i) z[i] = static_cast<int32_t>(uint32_t(a[i]) + uint32_t(b[i]));
    return 0;
}

const size_t kCounts[] = {5, 262144, 327683, 4099, 77, 196608, 1};
constexpr int kNames   = sizeof(kCounts) / sizeof(kCounts[0]);

int32_t value(int rank, int step, int name, size_t i)
{
    return static_cast<int32_t>((rank + 1) * 1000003u + step * 7919u + name * 131u + i);
}

std::atomic<int> g_failures{0};

struct Done {
    std::atomic<int> calls{0};
    std::atomic<int> bad{0};
};

void on_done(int status, void *arg)
{
    auto *d = static_cast<Done *>(arg);
    if (status != KF_OK) d->bad.fetch_add(1);
    d->calls.fetch_add(1);
}

void rank_main(int rank, int np, int steps, const char *dir)
{
    kf_session_t *s = kf_session_create(rank, np, dir, 0, 0);
    if (!s) {
        std::fprintf(stderr, "rank %d: kf_session_create: %s\n", rank, kf_session_last_error());
        g_failures.fetch_add(1);
        return;
    }
    kf_session_set_host_reduce(s, fold_i32);
    std::vector<std::vector<int32_t>> send(steps * kNames), recv(steps * kNames);
    std::mt19937 rng(1234 + rank);
    Done done;
    for (int step = 0; step < steps; ++step) {
        std::vector<int> order(kNames);
        for (int j = 0; j < kNames; ++j) order[j] = j;
        std::shuffle(order.begin(), order.end(), rng);
        for (int j : order) {
            auto &x = send[step * kNames + j];
            auto &y = recv[step * kNames + j];
            x.resize(kCounts[j]);
            y.assign(kCounts[j], -1);
            for (size_t i = 0; i < kCounts[j]; ++i) x[i] = value(rank, step, j, i);
            const bool inplace = j % 3 == 0;
            if (inplace) y = x;
            const std::string name = "w" + std::to_string(j);
            const int rc = kf_session_all_reduce_async(s, inplace ? y.data() : x.data(), y.data(),
                                                       kCounts[j], KungFu_INT32, KungFu_SUM,
                                                       name.c_str(), nullptr, on_done, &done);
            if (rc != KF_OK) {
                std::fprintf(stderr, "rank %d: submit %s: %d\n", rank, name.c_str(), rc);
                g_failures.fetch_add(1);
            }
            if (rng() % 4 == 0) std::this_thread::sleep_for(std::chrono::milliseconds(2));
        }
    }
    if (kf_session_wait_all(s) != KF_OK) {
        std::fprintf(stderr, "rank %d: wait_all: %s\n", rank, kf_session_last_error());
        g_failures.fetch_add(1);
    }
    if (done.calls.load() != steps * kNames || done.bad.load() != 0) {
        std::fprintf(stderr, "rank %d: %d callbacks, %d failed\n", rank, done.calls.load(),
                     done.bad.load());
        g_failures.fetch_add(1);
    }
    for (int step = 0; step < steps; ++step) {
        for (int j = 0; j < kNames; ++j) {
            const auto &y = recv[step * kNames + j];
            for (size_t i = 0; i < kCounts[j]; ++i) {
                uint32_t want = 0;
                for (int r = 0; r < np; ++r) want += uint32_t(value(r, step, j, i));
                if (uint32_t(y[i]) != want) {
                    std::fprintf(stderr, "rank %d step %d name w%d [%zu]: %d != %u\n", rank, step,
                                 j, i, y[i], want);
                    g_failures.fetch_add(1);
                    break;
                }
            }
        }
    }
    // a blocking all-reduce after the async ones
    std::vector<int32_t> z(1000, rank + 1), zr(1000, 0);
    if (kf_session_all_reduce(s, z.data(), zr.data(), z.size(), KungFu_INT32, KungFu_SUM, "after",
                              nullptr) != KF_OK ||
        zr[999] != np * (np + 1) / 2) {
        std::fprintf(stderr, "rank %d: blocking all-reduce after the async ones failed\n", rank);
        g_failures.fetch_add(1);
    }
    kf_session_destroy(s);
}
std::atomic<int> g_created{0};

void dead_main(int rank, int np, const char *dir)
{
    kf_session_t *s = kf_session_create(rank, np, dir, 0, 0);
    if (!s) {
        std::fprintf(stderr, "rank %d: kf_session_create: %s\n", rank, kf_session_last_error());
        g_failures.fetch_add(1);
        g_created.fetch_add(1);
        return;
    }
    kf_session_set_host_reduce(s, fold_i32);
    g_created.fetch_add(1);
    while (g_created.load() < np) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    if (rank == np - 1) {  // gone before its first chunk
        kf_session_destroy(s);
        return;
    }
    std::vector<std::vector<int32_t>> bufs(kNames);
    Done done;
    const auto t0 = std::chrono::steady_clock::now();
    for (int j = 0; j < kNames; ++j) {
        bufs[j].assign(kCounts[j], rank + 1);
        const std::string name = "d" + std::to_string(j);
        if (kf_session_all_reduce_async(s, bufs[j].data(), bufs[j].data(), kCounts[j], KungFu_INT32,
                                        KungFu_SUM, name.c_str(), nullptr, on_done,
                                        &done) != KF_OK) {
            g_failures.fetch_add(1);
        }
    }
    const int rc  = kf_session_wait_all(s);
    const double dt =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (rc == KF_OK || done.bad.load() == 0) {
        std::fprintf(stderr, "rank %d: all-reduces succeeded with rank %d gone\n", rank, np - 1);
        g_failures.fetch_add(1);
    } else if (dt > 30) {
        std::fprintf(stderr, "rank %d: the failure took %.1f s\n", rank, dt);
        g_failures.fetch_add(1);
    }
    kf_session_destroy(s);  // a peer still waiting on this one sees it close
}
}  // namespace

int main(int argc, char **argv)
{
    const int np    = argc > 1 ? std::atoi(argv[1]) : 3;
    const int steps = argc > 2 ? std::atoi(argv[2]) : 2;
    const char *dir = argc > 3 ? argv[3] : "/tmp";
    const bool dead = argc > 4 && std::string(argv[4]) == "dead";
    std::vector<std::thread> ts;
    for (int r = 0; r < np; ++r) {
        if (dead) ts.emplace_back(dead_main, r, np, dir);
        else ts.emplace_back(rank_main, r, np, steps, dir);
    }
    for (auto &t : ts) t.join();
    if (g_failures.load() != 0) {
        std::printf("FAIL %d\n", g_failures.load());
        return 1;
    }
    if (kf_shutdown() != KF_OK) {
        std::printf("kf_shutdown: %s\n", kf_last_error());
        return 1;
    }
    std::printf("OK np=%d steps=%d%s\n", np, steps, dead ? " dead" : "");
    return 0;
}
