// The reference's own C++ collective tests, restated against kungfu_amd.hpp
// (the Peer facade over the C ABI):
//   tests/cpp/unit/test_operations.cpp:3-26   test_allreduce<int32_t>(kf, 10 / 100)
//                                              with one peer: y[i] == i + 1
//   tests/cpp/integration/fake_agent.cpp:15-44 test_AllReduce(world, np):
//                                              iota(4 np) summed over np peers
//                                              == i * np, exit(1) otherwise
// usage: test_peer                      one peer (needs no GPU)
//        test_peer RANK SIZE DIR [dev]  one of SIZE peers on this host over unix
//                                       sockets in DIR; "dev": HBM buffers
#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "kungfu_amd.hpp"

using kungfu_amd::Peer;
using kungfu_amd::Waiter;

template <typename T> int test_allreduce(Peer &kf, const int count)
{
    const auto dtype = kungfu_amd::type_encoder<T>::value();
    std::vector<T> x(count);
    std::vector<T> y(count);
    std::iota(x.begin(), x.end(), 1);
    std::fill(y.begin(), y.end(), 0);
    Waiter waiter;
    if (kf.AllReduce(x.data(), y.data(), count, dtype, KungFu_SUM, "test",
                     [&waiter] { waiter.done(); }) != 0)
        return 1;
    waiter.wait();
    for (int i = 0; i < count; ++i) {
        if (y[i] != static_cast<T>(i + 1)) {
            std::printf("y[%d] = %d, want %d\n", i, int(y[i]), i + 1);
            return 1;
        }
    }
    return 0;
}

int test_AllReduce(Peer &world, int np, bool device)
{
    using T     = int32_t;
    const int n = np * 4;
    std::vector<T> x(n);
    std::vector<T> y(n);
    const auto dtype = kungfu_amd::type_encoder<T>::value();
    std::iota(x.begin(), x.end(), 0);
    void *px = x.data(), *py = y.data();
    if (device) {
        if (hipMalloc(&px, n * sizeof(T)) != hipSuccess ||
            hipMalloc(&py, n * sizeof(T)) != hipSuccess ||
            hipMemcpy(px, x.data(), n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
            return 1;
    }
    Waiter waiter;
    if (world.AllReduce(px, py, n, dtype, KungFu_SUM, "test-tensor",
                        [&waiter] { waiter.done(); }) != 0)
        return 1;
    waiter.wait();
    if (device) {
        if (hipDeviceSynchronize() != hipSuccess ||
            hipMemcpy(y.data(), py, n * sizeof(T), hipMemcpyDeviceToHost) != hipSuccess)
            return 1;
        (void)hipFree(px);
        (void)hipFree(py);
    }
    int failed = 0;
    for (int i = 0; i < n; ++i) {
        const int expected = i * np;
        if (y[i] != expected) {
            std::printf("expected y[%d]=%d, but got %d\n", i, expected, y[i]);
            ++failed;
        }
    }
    if (failed) {
        std::printf("reduce %d elements among %d agents, %d elements failed\n", n, np, failed);
        return 1;
    }
    return world.Barrier();
}

int main(int argc, char **argv)
{
    std::setvbuf(stdout, nullptr, _IOLBF, 0);  // lines survive an abort at exit
    if (argc < 4) {
        Peer kf;
        if (kf.Rank() != 0 || kf.Size() != 1) return 1;
        if (test_allreduce<int32_t>(kf, 10) || test_allreduce<int32_t>(kf, 100)) return 1;
        std::printf("peer ok (1 peer)\n");
        return 0;
    }
    const int rank = std::atoi(argv[1]), size = std::atoi(argv[2]);
    const bool device = argc > 4 && std::strcmp(argv[4], "dev") == 0;
    {
        Peer world(rank, size, device ? Peer::Device : Peer::Host, argv[3]);
        if (test_AllReduce(world, size, device)) return 1;
    }
    // the session is gone; the drop-in's HIP resources go back while the
    // runtime is up (no library destructor touches HIP at exit)
    if (kf_shutdown() != KF_OK) {
        std::printf("kf_shutdown: %s\n", kf_last_error());
        return 1;
    }
    std::printf("peer ok (%d of %d, %s)\n", rank, size, device ? "device" : "host");
    return 0;
}
