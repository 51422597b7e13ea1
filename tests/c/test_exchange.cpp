// A C++ host of the multi-GPU exchange through the C ABI only (the shape a
// kungfu::Peer / NCCL-controller binding takes): id from
// kf_exchange_unique_id, communicator, a batch of buckets all-reduced with the
// S-SGD epilogue, the ordered scheduler with done callbacks, the SMA batch.
// One rank (world 1): every all-reduce is the identity, the order is checked;
// then three ranks as threads over the test library's loopback transport
// (tests/c/kf_testing.h, plugged in through kf_exchange_create_transport):
// batches, and name-keyed all-reduces started in a different order per rank.
// Exit 0 = pass, 77 = no device (build checked only).
//   g++ -std=c++17 -D__HIP_PLATFORM_AMD__ -I include -I tests/c -I /opt/rocm/include
//       tests/c/test_exchange.cpp -L kungfu_amd -lkungfu_amd -L tests/c -lkf_testing
//       -L /opt/rocm/lib -lamdhip64 -o /tmp/test_exchange
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "kf_testing.h"
#include "kungfu_amd.h"

#define CHECK(c)                                                                \
    do {                                                                        \
        if (!(c)) {                                                             \
            std::fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #c, \
                         kf_exchange_last_error());                             \
            return 1;                                                           \
        }                                                                       \
    } while (0)

namespace
{
std::mutex g_mu;
std::vector<int> g_done;  // callback order: bucket index

void on_done(int status, void *arg)
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_done.push_back(status == KF_OK ? static_cast<int>(reinterpret_cast<intptr_t>(arg)) : -1);
}
}  // namespace

// `world` ranks as threads over the loopback transport, each with its own
// exchange, stream and buckets: S-SGD average of two buckets (one with a tail
// of count % world) must be the rank-order fold / world on every rank, for
// both algos, unpipelined and pipelined.
int multi_rank_loopback(int world)
{
    kf_loopback_t *g = kf_loopback_create(world);
    CHECK(g != nullptr);
    const std::vector<size_t> counts = {3 * 1024 + 1, 100003};
    std::vector<int> rc(world, 0);
    std::vector<std::thread> ts;
    for (int r = 0; r < world; ++r) {
        ts.emplace_back([&, r] {
            rc[r] = [&]() -> int {
                CHECK(hipSetDevice(0) == hipSuccess);
                kf_exchange_t *ex = kf_exchange_create_loopback(g, r, 0);
                CHECK(ex != nullptr);
                hipStream_t s;
                CHECK(hipStreamCreate(&s) == hipSuccess);
                std::vector<void *> bufs(2);
                for (int b = 0; b < 2; ++b) {
                    std::vector<float> h(counts[b]);
                    for (size_t i = 0; i < counts[b]; ++i) h[i] = 0.5f * (r + 1) + (i % 97);
                    CHECK(hipMalloc(&bufs[b], counts[b] * 4) == hipSuccess);
                    CHECK(hipMemcpy(bufs[b], h.data(), counts[b] * 4, hipMemcpyHostToDevice) ==
                          hipSuccess);
                }
                // groups 2: the pipelined schedule (kf_exchange_set_pipeline), each
                // bucket its own group, folds on the exchange's second stream
                for (int run = 0; run < 4; ++run) {
                    const int algo = run % 2 ? KF_ALGO_ALL_TO_ALL : KF_ALGO_REDUCE_SCATTER;
                    CHECK(kf_exchange_set_pipeline(ex, run < 2 ? 1 : 2) == KF_OK);
                    if (run > 0) {  // reset to the inputs
                        for (int b = 0; b < 2; ++b) {
                            std::vector<float> h(counts[b]);
                            for (size_t i = 0; i < counts[b]; ++i) h[i] = 0.5f * (r + 1) + (i % 97);
                            CHECK(hipMemcpy(bufs[b], h.data(), counts[b] * 4,
                                            hipMemcpyHostToDevice) == hipSuccess);
                        }
                    }
                    CHECK(kf_exchange_all_reduce_batch(
                              ex, const_cast<const void *const *>(bufs.data()), bufs.data(),
                              counts.data(), 2, KungFu_FLOAT, KungFu_SUM, 1, algo, s) == KF_OK);
                    CHECK(hipStreamSynchronize(s) == hipSuccess);
                    for (int b = 0; b < 2; ++b) {
                        std::vector<float> got(counts[b]);
                        CHECK(hipMemcpy(got.data(), bufs[b], counts[b] * 4,
                                        hipMemcpyDeviceToHost) == hipSuccess);
                        for (size_t i = 0; i < counts[b]; ++i) {
                            float acc = 0.5f * 1 + (i % 97);
                            for (int q = 1; q < world; ++q) acc += 0.5f * (q + 1) + (i % 97);
                            CHECK(got[i] == acc / world);
                        }
                    }
                }
                for (void *p : bufs) CHECK(hipFree(p) == hipSuccess);
                CHECK(hipStreamDestroy(s) == hipSuccess);
                kf_exchange_destroy(ex);
                return 0;
            }();
        });
    }
    for (auto &t : ts) t.join();
    kf_loopback_destroy(g);
    for (int r = 0; r < world; ++r) CHECK(rc[r] == 0);
    return 0;
}

// name-keyed: rank r starts the names rotated by r (and reversed on odd
// ranks); every bucket must still be the sum over ranks of ITS name
int multi_rank_named(int world)
{
    kf_loopback_t *g = kf_loopback_create(world);
    CHECK(g != nullptr);
    const int nn = 9;
    std::vector<int> rc(world, 0);
    std::vector<std::thread> ts;
    for (int r = 0; r < world; ++r) {
        ts.emplace_back([&, r] {
            rc[r] = [&]() -> int {
                CHECK(hipSetDevice(0) == hipSuccess);
                kf_exchange_t *ex = kf_exchange_create_loopback(g, r, 0);
                CHECK(ex != nullptr);
                hipStream_t s;
                CHECK(hipStreamCreate(&s) == hipSuccess);
                std::vector<void *> bufs(nn);
                std::vector<size_t> counts(nn);
                for (int b = 0; b < nn; ++b) {
                    counts[b] = 1 + 1000 * b + b % 3;
                    std::vector<int32_t> h(counts[b]);
                    for (size_t i = 0; i < counts[b]; ++i) h[i] = (r + 1) * (b + 1) + int(i % 11);
                    CHECK(hipMalloc(&bufs[b], counts[b] * 4) == hipSuccess);
                    CHECK(hipMemcpy(bufs[b], h.data(), counts[b] * 4, hipMemcpyHostToDevice) ==
                          hipSuccess);
                }
                for (int k = 0; k < nn; ++k) {
                    int b = (k + 2 * r) % nn;
                    if (r % 2) b = nn - 1 - b;
                    const std::string name = "grad/" + std::to_string(b);
                    CHECK(kf_exchange_all_reduce_named(ex, name.c_str(), bufs[b], bufs[b],
                                                       counts[b], KungFu_INT32, KungFu_SUM, 0,
                                                       KF_ALGO_AUTO, s, nullptr,
                                                       nullptr) == KF_OK);
                }
                CHECK(kf_exchange_wait_named(ex) == KF_OK);
                for (int b = 0; b < nn; ++b) {
                    std::vector<int32_t> got(counts[b]);
                    CHECK(hipMemcpy(got.data(), bufs[b], counts[b] * 4, hipMemcpyDeviceToHost) ==
                          hipSuccess);
                    for (size_t i = 0; i < counts[b]; ++i) {
                        int32_t want = 0;
                        for (int q = 0; q < world; ++q) want += (q + 1) * (b + 1) + int(i % 11);
                        CHECK(got[i] == want);
                    }
                    CHECK(hipFree(bufs[b]) == hipSuccess);
                }
                CHECK(hipStreamDestroy(s) == hipSuccess);
                kf_exchange_destroy(ex);
                return 0;
            }();
        });
    }
    for (auto &t : ts) t.join();
    kf_loopback_destroy(g);
    for (int r = 0; r < world; ++r) CHECK(rc[r] == 0);
    return 0;
}

int main()
{
    std::setvbuf(stdout, nullptr, _IOLBF, 0);  // lines survive an abort at exit
    if (kf_device_count() < 1) {
        std::printf("no device: build checked only\n");
        return 77;
    }
    unsigned char id[KF_UNIQUE_ID_BYTES];
    CHECK(kf_exchange_unique_id(id) == KF_OK);
    kf_exchange_t *ex = kf_exchange_create(id, 0, 1, 0);
    CHECK(ex != nullptr);
    int rank = -1, world = -1, dev = -1;
    CHECK(kf_exchange_info(ex, &rank, &world, &dev) == KF_OK);
    CHECK(rank == 0 && world == 1 && dev == 0);

    const int nb = 5;
    std::vector<size_t> counts = {1, 1000, 4097, 1 << 20, 3};
    std::vector<void *> bufs(nb);
    std::vector<std::vector<float>> host(nb);
    for (int b = 0; b < nb; ++b) {
        host[b].resize(counts[b]);
        for (size_t i = 0; i < counts[b]; ++i) host[b][i] = 0.25f * (b + 1) + i;
        CHECK(hipMalloc(&bufs[b], counts[b] * 4) == hipSuccess);
        CHECK(hipMemcpy(bufs[b], host[b].data(), counts[b] * 4, hipMemcpyHostToDevice) ==
              hipSuccess);
    }
    hipStream_t s;
    CHECK(hipStreamCreate(&s) == hipSuccess);
    for (int algo : {KF_ALGO_AUTO, KF_ALGO_REDUCE_SCATTER, KF_ALGO_ALL_TO_ALL}) {
        CHECK(kf_exchange_all_reduce_batch(ex, const_cast<const void *const *>(bufs.data()),
                                           bufs.data(), counts.data(), nb, KungFu_FLOAT,
                                           KungFu_SUM, 1, algo, s) == KF_OK);
    }
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    CHECK(kf_exchange_check(ex) == KF_OK);
    for (int b = 0; b < nb; ++b) {
        std::vector<float> got(counts[b]);
        CHECK(hipMemcpy(got.data(), bufs[b], counts[b] * 4, hipMemcpyDeviceToHost) == hipSuccess);
        CHECK(std::memcmp(got.data(), host[b].data(), counts[b] * 4) == 0);
    }
    // NCCLScheduler: names started in reverse, issued (and done) in order
    std::vector<std::string> names = {"grad/a", "grad/b", "grad/c", "grad/d", "grad/e"};
    std::vector<const char *> cn;
    for (auto &n : names) cn.push_back(n.c_str());
    CHECK(kf_exchange_begin_step(ex, cn.data(), nb, 0) == KF_OK);
    for (int b = nb - 1; b >= 0; --b) {
        CHECK(kf_exchange_start(ex, cn[b], bufs[b], bufs[b], counts[b], KungFu_FLOAT, KungFu_SUM,
                                1, KF_ALGO_AUTO, s, on_done,
                                reinterpret_cast<void *>(static_cast<intptr_t>(b))) == KF_OK);
    }
    int32_t order[nb];
    CHECK(kf_exchange_wait_all(ex, order) == KF_OK);
    for (int b = 0; b < nb; ++b) CHECK(order[b] == b);
    CHECK(g_done.size() == static_cast<size_t>(nb));
    for (int b = 0; b < nb; ++b) CHECK(g_done[b] == b);
    // an unknown name and a second start are refused
    CHECK(kf_exchange_begin_step(ex, cn.data(), 1, 0) == KF_OK);
    CHECK(kf_exchange_start(ex, "nope", bufs[0], bufs[0], 1, KungFu_FLOAT, KungFu_SUM, 0,
                            KF_ALGO_AUTO, s, nullptr, nullptr) == KF_ERR_ARG);
    CHECK(kf_exchange_start(ex, cn[0], bufs[0], bufs[0], 1, KungFu_FLOAT, KungFu_SUM, 0,
                            KF_ALGO_AUTO, s, nullptr, nullptr) == KF_OK);
    CHECK(kf_exchange_start(ex, cn[0], bufs[0], bufs[0], 1, KungFu_FLOAT, KungFu_SUM, 0,
                            KF_ALGO_AUTO, s, nullptr, nullptr) == KF_ERR_ARG);
    CHECK(kf_exchange_wait_all(ex, nullptr) == KF_OK);
    // SMA of one rank, alpha = 0.5: v' = 0.5 v + 0.5 (v / 1) = v for these values
    std::vector<void *> sums(nb);
    for (int b = 0; b < nb; ++b) CHECK(hipMalloc(&sums[b], counts[b] * 4) == hipSuccess);
    CHECK(kf_exchange_sma_batch(ex, bufs.data(), sums.data(), counts.data(), nb, KungFu_FLOAT, 0.5,
                                KF_ALGO_AUTO, s) == KF_OK);
    CHECK(hipStreamSynchronize(s) == hipSuccess);
    for (int b = 0; b < nb; ++b) {
        std::vector<float> got(counts[b]);
        CHECK(hipMemcpy(got.data(), bufs[b], counts[b] * 4, hipMemcpyDeviceToHost) == hipSuccess);
        CHECK(std::memcmp(got.data(), host[b].data(), counts[b] * 4) == 0);
        CHECK(hipFree(bufs[b]) == hipSuccess && hipFree(sums[b]) == hipSuccess);
    }
    kf_exchange_destroy(ex);
    CHECK(hipStreamDestroy(s) == hipSuccess);
    CHECK(multi_rank_loopback(3) == 0);
    CHECK(multi_rank_named(3) == 0);
    CHECK(kf_shutdown() == KF_OK);  // HIP resources back while the runtime is up
    std::printf("exchange ok\n");
    return 0;
}
