// same_box_probe.hip — the shipped C-ABI kernels at C2's and C5's sizes on
// ONE box, interleaved. Across boxes the in-place bf16 traffic ran at 0.81
// (r06a, 256 MiB) and 0.78 (r06m, C5's 219 MB), and the tail probe
// (tail_probe.hip, r06n) found no cost in a half-filled last round of blocks;
// this separates size from box.
//
//   c2_f32            kf_bucket_reduce f32 SUM, x + y -> z (the headline)
//   c2_f32_inplace    the same into x
//   add_bf16          kf_bucket_reduce bf16 SUM, out of place
//   sma_bf16          kf_sma_blend bf16 in place, np 8, alpha 0.1
//   sma_batch_c5      kf_sma_blend_batch over C5's 13 contiguous buckets
//   xor_inplace       v ^= s, whole tiles unguarded (the shipped body's shape)
//
// each at 256 MiB per stream and at C5's 218,976,256 B per stream (sma_batch
// at C5's only); 3 rotating sets, median of 7 x 24 launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I kungfu_amd/csrc \
//       -o tools/explore/same_box_probe tools/explore/same_box_probe.hip \
//       -L kungfu_amd -lkungfu_amd -Wl,-rpath,$PWD/kungfu_amd
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "kf_reduce_kernels.hpp"
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

using kf::u32x4;
constexpr int BLOCK = 256, U = 4;

__global__ void __launch_bounds__(BLOCK) xor_inplace(u32x4 *v, const u32x4 *s, size_t n)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK < n) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(v + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(s + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u] ^ b[u], v + v0 + u * BLOCK);
    } else {
        for (int u = 0; u < U; ++u) {
            const size_t vi = v0 + u * BLOCK;
            if (vi >= n) break;
            v[vi] = v[vi] ^ s[vi];
        }
    }
}

__global__ void fill(uint32_t *p, size_t n, uint32_t seed)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = static_cast<uint32_t>(i) * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        // finite bf16 / f32 halves of moderate magnitude
        const uint32_t lo = (x & 0x807fu) | ((124u + (x >> 8) % 6u) << 7);
        const uint32_t hi = ((x >> 16) & 0x807fu) | ((124u + (x >> 24) % 6u) << 7);
        p[i] = lo | (hi << 16);
    }
}

int main()
{
    const size_t C5N = 109488128;  // bf16 elements of C5's 13 buckets
    const size_t cnt[13] = {23441408, 8075264, 8269824, 7680000, 7088128, 7088128, 7088128,
                            7088128,  7088128, 7088128, 7088128, 7088128, 5316608};
    const size_t big = 256u << 20;
    const int NS = 3;
    std::vector<char *> X(NS), Y(NS), Z(NS);
    for (int k = 0; k < NS; ++k) {
        CHECK(hipMalloc(&X[k], big));
        CHECK(hipMalloc(&Y[k], big));
        CHECK(hipMalloc(&Z[k], big));
        fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(X[k]), big / 4, 17u + k);
        fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(Y[k]), big / 4, 71u + k);
    }
    CHECK(hipDeviceSynchronize());
    std::vector<std::vector<void *>> vs(NS), ss(NS);
    for (int k = 0; k < NS; ++k) {
        size_t off = 0;
        for (size_t c : cnt) {
            vs[k].push_back(X[k] + off * 2);
            ss[k].push_back(Y[k] + off * 2);
            off += c;
        }
    }
    struct Var {
        std::string name;
        double bytes;
        std::function<void(int)> run;
    };
    std::vector<Var> vars;
    for (size_t bytes : {big, C5N * 2}) {
        const std::string tag = bytes == big ? "_256M" : "_c5";
        vars.push_back({"c2_f32" + tag, 3.0 * bytes, [=](int k) {
                            const void *in[2] = {X[k], Y[k]};
                            KF(kf_bucket_reduce(in, 2, Z[k], bytes / 4, KungFu_FLOAT, KungFu_SUM, nullptr));
                        }});
        vars.push_back({"c2_f32_inplace" + tag, 3.0 * bytes, [=](int k) {
                            const void *in[2] = {Z[k], Y[k]};
                            KF(kf_bucket_reduce(in, 2, Z[k], bytes / 4, KungFu_FLOAT, KungFu_SUM, nullptr));
                        }});
        vars.push_back({"add_bf16" + tag, 3.0 * bytes, [=](int k) {
                            const void *in[2] = {X[k], Y[k]};
                            KF(kf_bucket_reduce(in, 2, Z[k], bytes / 2, KungFu_BFLOAT16, KungFu_SUM, nullptr));
                        }});
        vars.push_back({"sma_bf16" + tag, 3.0 * bytes, [=](int k) {
                            KF(kf_sma_blend(X[k], Y[k], bytes / 2, KungFu_BFLOAT16, 8, 0.1, nullptr));
                        }});
        vars.push_back({"xor_inplace" + tag, 3.0 * bytes, [=](int k) {
                            const size_t n = bytes / 16;
                            xor_inplace<<<static_cast<unsigned>((n + BLOCK * U - 1) / (BLOCK * U)), BLOCK>>>(
                                reinterpret_cast<u32x4 *>(X[k]), reinterpret_cast<const u32x4 *>(Y[k]), n);
                        }});
    }
    vars.push_back({"sma_batch_c5", 6.0 * C5N, [&](int k) {
                        KF(kf_sma_blend_batch(vs[k].data(), const_cast<const void *const *>(ss[k].data()), cnt,
                                              13, KungFu_BFLOAT16, 8, 0.1, nullptr));
                    }});
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ts(vars.size());
    for (int round = 0; round < 7; ++round) {
        // the in-place blends and xors drift the data: refill every round
        for (int k = 0; k < NS; ++k) {
            fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(X[k]), big / 4, 17u + k + round);
            fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(Z[k]), big / 4, 29u + k + round);
        }
        for (size_t v = 0; v < vars.size(); ++v) {
            for (int k = 0; k < NS; ++k) vars[v].run(k);
            CHECK(hipEventRecord(e0));
            for (int i = 0; i < 24; ++i) vars[v].run(i % NS);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ts[v].push_back(ms * 1e3f / 24);
        }
    }
    CHECK(hipGetLastError());
    for (size_t v = 0; v < vars.size(); ++v) {
        std::sort(ts[v].begin(), ts[v].end());
        const double us = ts[v][ts[v].size() / 2];
        printf("{\"variant\": \"%s\", \"us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n", vars[v].name.c_str(), us,
               ts[v][0], vars[v].bytes / us / 8e6);
    }
    return 0;
}
