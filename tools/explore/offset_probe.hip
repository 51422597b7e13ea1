// offset_probe.hip — does the distance between a kernel's streams matter?
// The C5 blend batch ran 0.771 of 8 TB/s with v flat and each sum in its own
// allocation, 0.803 with every bucket and sum in its own allocation, 0.819
// as one flat range (profiles/r06/sma_layout_probe_r06v.jsonl): same bytes,
// same kernel, only the addresses differ. Here ONE kf_sma_blend over C5's
// 218,976,256 B per stream, v at the base of one allocation and s at
// v + bytes + delta, for a sweep of deltas; and C2's z = x + y (fp32,
// 256 MiB per stream) with y and z placed the same way. 3 rotating sets
// (each its own allocation), median of 7 x 24 launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include \
//       -o tools/explore/offset_probe tools/explore/offset_probe.hip \
//       -L kungfu_amd -lkungfu_amd -Wl,-rpath,'$ORIGIN/../../kungfu_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "kungfu_amd.h"

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(2);                                                            \
        }                                                                       \
    } while (0)
#define KF(x)                                                                   \
    do {                                                                        \
        int rc_ = (x);                                                          \
        if (rc_ != 0) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, kf_last_error());                  \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

__global__ void fill(uint32_t *p, size_t n, uint32_t seed)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = static_cast<uint32_t>(i) * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        const uint32_t lo = (x & 0x807fu) | ((124u + (x >> 8) % 6u) << 7);
        const uint32_t hi = ((x >> 16) & 0x807fu) | ((124u + (x >> 24) % 6u) << 7);
        p[i] = lo | (hi << 16);
    }
}

int main()
{
    const size_t deltas[] = {0, 4096, 16384, 65536, 262144, 1u << 20, 2u << 20, 4u << 20,
                             (1u << 20) + 4096, (3u << 20) + 20480, 12345 * 16};
    const int NS = 3;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int which = 0; which < 2; ++which) {
        const bool sma = which == 0;
        const size_t bytes = sma ? 218976256 : (256u << 20);
        const int nstreams = sma ? 2 : 3;
        for (size_t delta : deltas) {
            std::vector<char *> base(NS);
            const size_t span = nstreams * (bytes + delta) + (4u << 20);
            for (int k = 0; k < NS; ++k) {
                CHECK(hipMalloc(&base[k], span));
                fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(base[k]), span / 4, 17u + k);
            }
            CHECK(hipDeviceSynchronize());
            auto run = [&](int k) {
                char *a = base[k], *b = a + bytes + delta, *c = b + bytes + delta;
                if (sma) {
                    KF(kf_sma_blend(a, b, bytes / 2, KungFu_BFLOAT16, 8, 0.1, nullptr));
                } else {
                    const void *in[2] = {a, b};
                    KF(kf_bucket_reduce(in, 2, c, bytes / 4, KungFu_FLOAT, KungFu_SUM, nullptr));
                }
            };
            std::vector<float> ts;
            for (int round = 0; round < 7; ++round) {
                for (int k = 0; k < NS; ++k) run(k);
                CHECK(hipEventRecord(e0));
                for (int i = 0; i < 24; ++i) run(i % NS);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                ts.push_back(ms * 1e3f / 24);
            }
            std::sort(ts.begin(), ts.end());
            const double us = ts[ts.size() / 2];
            printf("{\"kernel\": \"%s\", \"delta\": %zu, \"us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n",
                   sma ? "sma_bf16_c5" : "c2_f32", delta, us, ts[0], 3.0 * bytes / us / 8e6);
            fflush(stdout);
            for (int k = 0; k < NS; ++k) CHECK(hipFree(base[k]));
        }
    }
    return 0;
}
