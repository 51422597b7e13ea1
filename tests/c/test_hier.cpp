// The hierarchical all-reduce from C++ through the C ABI alone
// (kf_hier_all_reduce; the reference's ScheduledHierarchicalNcclAllReduce,
// srcs/cpp/src/tensorflow/ops/gpu/collective.cpp:108-162, with
// CrossAllReduceGpu, srcs/cpp/src/nccl/controller.cpp:7-39), ranks as threads
// of one process on one GPU:
//   * hosts are emulated by loopback addresses (127.0.0.1, 127.0.0.2): the
//     cross-host step runs over real device-mode KungFu sessions
//     (kf_session_create_peers: unix sockets inside a host, TCP across);
//   * inside a host the exchange runs over the test library's loopback
//     transport (tests/c/kf_testing.h; RCCL refuses two ranks on one GPU).
// Cases: 2 hosts x 2 ranks (the sharded path, both algos, tails, average and
// MAX), 2 + 1 ranks (hosts of different sizes: the reference's masters path),
// and 2 hosts x 1 rank with the host exchange from kf_exchange_create_local
// (its RCCL ids shared over the session). Every result must equal, bit for
// bit, the per-host rank-order fold combined across the two hosts (a single
// addition, so any order gives it), / np.
//   test_hier <base_port> <sock_dir>    exit 0 = pass, 77 = no device
#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "kf_testing.h"
#include "kungfu_amd.h"

#define CHECK(c)                                                                      \
    do {                                                                              \
        if (!(c)) {                                                                   \
            std::fprintf(stderr, "FAIL %s:%d: %s (%s | %s)\n", __FILE__, __LINE__, #c, \
                         kf_exchange_last_error(), kf_session_last_error());          \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

namespace
{
float value(int rank, size_t i, int seed)
{
    uint32_t x = static_cast<uint32_t>(i * 2654435761u) ^ static_cast<uint32_t>(rank * 40503 + seed);
    x ^= x >> 13;
    x *= 0x5bd1e995u;
    x ^= x >> 15;
    return (static_cast<int32_t>(x) / 2147483648.0f) * (1.0f + rank);  // ~U(-1,1) x (r + 1)
}

// the bits the sharded or masters path must give: each host's rank-order
// fold, the hosts' sums added (two operands: one addition), / np
std::vector<float> expected(const std::vector<std::vector<int>> &hosts, size_t n, int seed,
                            bool maxop, bool average, int np)
{
    std::vector<float> out(n);
    for (size_t i = 0; i < n; ++i) {
        std::vector<float> hs;
        for (auto &h : hosts) {
            float a = value(h[0], i, seed);
            for (size_t j = 1; j < h.size(); ++j) {
                const float b = value(h[j], i, seed);
                a             = maxop ? (a < b ? b : a) : a + b;
            }
            hs.push_back(a);
        }
        float t = hs[0];
        for (size_t k = 1; k < hs.size(); ++k) t = maxop ? (t < hs[k] ? hs[k] : t) : t + hs[k];
        out[i] = average ? t / static_cast<float>(np) : t;
    }
    return out;
}

int run_rank(int rank, const std::string &peers, const std::string &self, const char *dir,
             kf_exchange_t *local, const std::vector<std::vector<int>> &hosts, int np)
{
    CHECK(hipSetDevice(0) == hipSuccess);
    kf_session_t *s = kf_session_create_peers(peers.c_str(), self.c_str(), dir, 77, 1);
    CHECK(s != nullptr);
    int r = -1, size = -1, lr = -1, ls = -1, hc = -1;
    CHECK(kf_session_info(s, &r, &size, &lr, &ls, &hc) == KF_OK);
    CHECK(r == rank && size == np && hc == static_cast<int>(hosts.size()));
    bool own_local = false;
    if (!local) {  // gpu_collective::new_local over this session
        local     = kf_exchange_create_local(s, 0);
        own_local = true;
        CHECK(local != nullptr);
    }
    int er = -1, ew = -1;
    CHECK(kf_exchange_info(local, &er, &ew, nullptr) == KF_OK);
    CHECK(er == lr && ew == ls);
    hipStream_t st;
    CHECK(hipStreamCreate(&st) == hipSuccess);
    int seed = 0;
    for (size_t n : {size_t(1), size_t(1000), size_t(4099), size_t(262147)}) {
        for (int algo : {KF_ALGO_REDUCE_SCATTER, KF_ALGO_ALL_TO_ALL}) {
            for (int mode = 0; mode < 2; ++mode) {  // 0: S-SGD average, 1: MAX
                ++seed;
                std::vector<float> h(n);
                for (size_t i = 0; i < n; ++i) h[i] = value(rank, i, seed);
                void *d = nullptr;
                CHECK(hipMalloc(&d, n * 4) == hipSuccess);
                CHECK(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice) == hipSuccess);
                const std::string name = "grad/" + std::to_string(seed);
                CHECK(kf_hier_all_reduce(local, s, d, d, n, KungFu_FLOAT,
                                         mode ? KungFu_MAX : KungFu_SUM, mode ? 0 : 1, algo,
                                         name.c_str(), st) == KF_OK);
                CHECK(hipStreamSynchronize(st) == hipSuccess);
                std::vector<float> got(n);
                CHECK(hipMemcpy(got.data(), d, n * 4, hipMemcpyDeviceToHost) == hipSuccess);
                const auto want = expected(hosts, n, seed, mode == 1, mode == 0, np);
                CHECK(std::memcmp(got.data(), want.data(), n * 4) == 0);
                CHECK(hipFree(d) == hipSuccess);
            }
        }
    }
    CHECK(hipStreamDestroy(st) == hipSuccess);
    if (own_local) kf_exchange_destroy(local);
    kf_session_destroy(s);
    return 0;
}

// hosts[h] = the global ranks of host h; loopback groups for the host
// exchanges (use_local: kf_exchange_create_local instead)
int run_layout(const std::vector<std::vector<int>> &hosts, int base_port, const char *dir,
               bool use_local)
{
    int np = 0;
    for (auto &h : hosts) np += static_cast<int>(h.size());
    std::vector<std::string> spec(np);
    std::string peers;
    for (size_t h = 0; h < hosts.size(); ++h) {
        for (int g : hosts[h]) {
            spec[g] = "127.0.0." + std::to_string(h + 1) + ":" + std::to_string(base_port + g);
        }
    }
    for (int g = 0; g < np; ++g) peers += (g ? "," : "") + spec[g];
    std::vector<kf_loopback_t *> groups;
    std::vector<kf_exchange_t *> locals(np, nullptr);
    if (!use_local) {
        for (auto &h : hosts) {
            groups.push_back(kf_loopback_create(static_cast<int>(h.size())));
            for (size_t j = 0; j < h.size(); ++j) {
                locals[h[j]] = kf_exchange_create_loopback(groups.back(), static_cast<int>(j), 0);
                CHECK(locals[h[j]] != nullptr);
            }
        }
    }
    std::vector<int> rc(np, -1);
    std::vector<std::thread> ts;
    for (int g = 0; g < np; ++g) {
        ts.emplace_back([&, g] { rc[g] = run_rank(g, peers, spec[g], dir, locals[g], hosts, np); });
    }
    for (auto &t : ts) t.join();
    for (auto *ex : locals) kf_exchange_destroy(ex);
    for (auto *gp : groups) kf_loopback_destroy(gp);
    for (int g = 0; g < np; ++g) CHECK(rc[g] == 0);
    return 0;
}
}  // namespace

int main(int argc, char **argv)
{
    std::setvbuf(stdout, nullptr, _IOLBF, 0);  // lines survive an abort at exit
    if (argc < 3) {
        std::fprintf(stderr, "usage: test_hier <base_port> <sock_dir>\n");
        return 2;
    }
    if (kf_device_count() < 1) {
        std::printf("no device: build checked only\n");
        return 77;
    }
    const int port = std::atoi(argv[1]);
    CHECK(run_layout({{0, 1}, {2, 3}}, port, argv[2], false) == 0);
    std::printf("2 hosts x 2 ranks ok\n");
    CHECK(run_layout({{0, 1}, {2}}, port + 10, argv[2], false) == 0);
    std::printf("2 + 1 ranks ok\n");
    CHECK(run_layout({{0}, {1}}, port + 20, argv[2], true) == 0);
    std::printf("2 hosts x 1 rank (kf_exchange_create_local) ok\n");
    CHECK(kf_shutdown() == KF_OK);  // HIP resources back while the runtime is up
    std::printf("hier ok\n");
    return 0;
}
