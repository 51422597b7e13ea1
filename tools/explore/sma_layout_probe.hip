// sma_layout_probe.hip — the C5 blend batch runs ~2 % behind one kf_sma_blend
// over the same bytes (profiles/r06/ab_sma_sched_r06p.jsonl: 0.794 against
// 0.816 at 256 MiB; sma_sched_probe_r06p.jsonl: no size effect). Segments or
// allocations? One process, interleaved, C5's 13 bf16 bucket sizes:
//
//   single        kf_sma_blend over one flat range of all 13 buckets' bytes
//   batch_flat    kf_sma_blend_batch, buckets AND sums carved back to back
//                 from one allocation each (the launch merges them: = single)
//   batch_seg     buckets back to back in one allocation, sums each in its
//                 own allocation (no merge: 13 segments over flat v)
//   batch_alloc   every bucket and every sum its own hipMalloc (the line's
//                 16 MiB-bucket layout, GradBuckets(bucket_bytes=16 MiB))
//
// 3 rotating sets, median of 7 x 24 launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I kungfu_amd/csrc \
//       -o tools/explore/sma_layout_probe tools/explore/sma_layout_probe.hip \
//       -L kungfu_amd -lkungfu_amd -Wl,-rpath,'$ORIGIN/../../kungfu_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
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

constexpr int NB = 13;

int main()
{
    const size_t cnt[NB] = {23441408, 8075264, 8269824, 7680000, 7088128, 7088128, 7088128,
                            7088128,  7088128, 7088128, 7088128, 7088128, 5316608};
    size_t total = 0;
    for (size_t c : cnt) total += c;
    const int NS = 3;
    struct Set {
        char *vflat, *sflat;
        std::vector<void *> vf, sf, ssep, va, sa;  // carved / own allocations
    };
    std::vector<Set> sets(NS);
    auto fill_bytes = [](void *p, size_t bytes, uint32_t seed) {
        fill<<<2048, 256>>>(reinterpret_cast<uint32_t *>(p), bytes / 4, seed);
    };
    for (int k = 0; k < NS; ++k) {
        Set &st = sets[k];
        CHECK(hipMalloc(&st.vflat, total * 2));
        CHECK(hipMalloc(&st.sflat, total * 2));
        fill_bytes(st.vflat, total * 2, 17u + k);
        fill_bytes(st.sflat, total * 2, 71u + k);
        size_t off = 0;
        for (int b = 0; b < NB; ++b) {
            st.vf.push_back(st.vflat + off * 2);
            st.sf.push_back(st.sflat + off * 2);
            void *p;
            CHECK(hipMalloc(&p, cnt[b] * 2));
            fill_bytes(p, cnt[b] * 2, 31u + b + 100 * k);
            st.ssep.push_back(p);
            CHECK(hipMalloc(&p, cnt[b] * 2));
            fill_bytes(p, cnt[b] * 2, 37u + b + 100 * k);
            st.va.push_back(p);
            CHECK(hipMalloc(&p, cnt[b] * 2));
            fill_bytes(p, cnt[b] * 2, 41u + b + 100 * k);
            st.sa.push_back(p);
            off += cnt[b];
        }
    }
    CHECK(hipDeviceSynchronize());
    auto batch = [&](std::vector<void *> &v, std::vector<void *> &s) {
        KF(kf_sma_blend_batch(v.data(), const_cast<const void *const *>(s.data()), cnt, NB, KungFu_BFLOAT16, 8,
                              0.1, nullptr));
    };
    struct Var {
        std::string name;
        std::function<void(int)> run;
    };
    std::vector<Var> vars = {
        {"single", [&](int k) { KF(kf_sma_blend(sets[k].vflat, sets[k].sflat, total, KungFu_BFLOAT16, 8, 0.1, nullptr)); }},
        {"batch_flat", [&](int k) { batch(sets[k].vf, sets[k].sf); }},
        {"batch_seg", [&](int k) { batch(sets[k].vf, sets[k].ssep); }},
        {"batch_alloc", [&](int k) { batch(sets[k].va, sets[k].sa); }},
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ts(vars.size());
    for (int round = 0; round < 7; ++round) {
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
               ts[v][0], 6.0 * total / us / 8e6);
    }
    return 0;
}
