// pcie_explore.hip — what the host link gives the copy-inclusive path:
// pinned H2D alone, D2H alone, and both directions at once on two streams.
//   hipcc --offload-arch=gfx950 -O3 -o pcie_explore pcie_explore.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

int main()
{
    const size_t B = size_t(256) << 20;
    void *h_in, *h_out, *d_in, *d_out;
    CHECK(hipHostMalloc(&h_in, 2 * B, hipHostMallocDefault));
    CHECK(hipHostMalloc(&h_out, B, hipHostMallocDefault));
    CHECK(hipMalloc(&d_in, 2 * B));
    CHECK(hipMalloc(&d_out, B));
    hipStream_t s0, s1;
    CHECK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    for (int rep = 0; rep < 2; ++rep) {
        double t0 = now();
        CHECK(hipMemcpyAsync(d_in, h_in, 2 * B, hipMemcpyHostToDevice, s0));
        CHECK(hipStreamSynchronize(s0));
        double t1 = now();
        CHECK(hipMemcpyAsync(h_out, d_out, B, hipMemcpyDeviceToHost, s1));
        CHECK(hipStreamSynchronize(s1));
        double t2 = now();
        CHECK(hipMemcpyAsync(d_in, h_in, 2 * B, hipMemcpyHostToDevice, s0));
        CHECK(hipMemcpyAsync(h_out, d_out, B, hipMemcpyDeviceToHost, s1));
        CHECK(hipStreamSynchronize(s0));
        CHECK(hipStreamSynchronize(s1));
        double t3 = now();
        // chunked: 16 MiB pieces, H2D on s0, D2H on s1 interleaved
        const size_t C = size_t(16) << 20;
        for (size_t off = 0; off < B; off += C) {
            CHECK(hipMemcpyAsync((char *)d_in + 2 * off, (char *)h_in + 2 * off, 2 * C,
                                 hipMemcpyHostToDevice, s0));
            CHECK(hipMemcpyAsync((char *)h_out + off, (char *)d_out + off, C,
                                 hipMemcpyDeviceToHost, s1));
        }
        CHECK(hipStreamSynchronize(s0));
        CHECK(hipStreamSynchronize(s1));
        double t4 = now();
        if (rep == 1) {
            printf("{\"h2d_512MiB_ms\": %.3f, \"h2d_GBps\": %.1f, \"d2h_256MiB_ms\": %.3f, "
                   "\"d2h_GBps\": %.1f, \"both_concurrent_ms\": %.3f, \"both_chunked_ms\": %.3f, "
                   "\"serial_sum_ms\": %.3f}\n",
                   (t1 - t0) * 1e3, 2 * B / (t1 - t0) / 1e9, (t2 - t1) * 1e3,
                   B / (t2 - t1) / 1e9, (t3 - t2) * 1e3, (t4 - t3) * 1e3,
                   (t2 - t0) * 1e3);
        }
    }
    return 0;
}
