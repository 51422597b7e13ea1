// kfold_prod_vs_probe.hip — the product's k-input fold (kf_bucket_reduce
// through libkungfu_amd.so) against the probe kernel of kfold_occ.hip on the
// SAME hipMalloc'd buffers, capped (48 KiB) and uncapped, rounds interleaved:
// does the product kernel itself differ from the probe, or only the buffers
// the two were measured on?
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o kfold_prod_vs_probe \
//         tools/explore/kfold_prod_vs_probe.hip -L kungfu_amd -lkungfu_amd
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "kungfu_amd.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

struct Ptrs {
    const f32x4 *p[16];
};

__global__ void __launch_bounds__(256) fold(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * 1024 + threadIdx.x;
    if (v0 + 768 >= nvec) return;
    f32x4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = __builtin_nontemporal_load(in.p[0] + v0 + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = __builtin_nontemporal_load(in.p[1] + v0 + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += b[u];
    for (int j = 2; j < k; ++j) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {  // one vector in flight (the product's schedule)
            const f32x4 *q = in.p[j] + v0 + u * 256;
            f32x4 v;
            asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(q));
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(v));
            a[u] += v;
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(a[u], out + v0 + u * 256);
}

int main()
{
    const size_t n = 64ull << 20, bytes = n * 4, nvec = n / 4;
    const int kmax = 8, sets = 3, launches = 10, rounds = 5;
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    std::vector<std::vector<float *>> in(sets, std::vector<float *>(kmax));
    std::vector<float *> out(sets);
    for (int st = 0; st < sets; ++st) {
        for (int j = 0; j < kmax; ++j) {
            CHECK(hipMalloc(&in[st][j], bytes));
            CHECK(hipMemset(in[st][j], 0x3c, bytes));
        }
        CHECK(hipMalloc(&out[st], bytes));
    }
    struct V {
        std::string name;
        int k;
        std::function<void(int)> run;
    };
    std::vector<V> vs;
    for (int k : {4, 8}) {
        for (int lds : {0, 32 << 10, 40 << 10, 48 << 10}) {
            vs.push_back({"product_lds" + std::to_string(lds >> 10) + "K", k, [&, k, lds](int st) {
                              kf_set_occupancy(0, lds);
                              const void *p[16];
                              for (int j = 0; j < k; ++j) p[j] = in[st][j];
                              if (kf_bucket_reduce(p, k, out[st], n, KungFu_FLOAT, KungFu_SUM, s) != 0)
                                  exit(4);
                          }});
            vs.push_back({"probe_lds" + std::to_string(lds >> 10) + "K", k, [&, k, lds](int st) {
                              Ptrs p;
                              for (int j = 0; j < 16; ++j)
                                  p.p[j] = reinterpret_cast<const f32x4 *>(in[st][j % kmax]);
                              fold<<<nvec / 1024, 256, lds, s>>>(p, k, reinterpret_cast<f32x4 *>(out[st]),
                                                                 nvec);
                          }});
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<double>> t(vs.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            vs[i].run(0);
            CHECK(hipEventRecord(e0, s));
            for (int l = 0; l < launches; ++l) vs[i].run(l % sets);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1e3 / launches);
        }
    }
    kf_set_occupancy(0, 32 << 10);
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(t[i].begin(), t[i].end());
        const double med = t[i][rounds / 2], algo = (vs[i].k + 1.0) * bytes;
        printf("{\"variant\": \"%s\", \"k\": %d, \"median_us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n",
               vs[i].name.c_str(), vs[i].k, med, t[i][0], algo / med / 8e6);
    }
    return 0;
}
