// write_explore.hip — the store stream alone (C2's output stream; DESIGN.md
// §10 item 3): 256 MiB written per launch by store shapes and cache-policy
// bits, against hipMemsetD32Async. 2 rotating buffers, median of 7 x 10.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o write_explore write_explore.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

// POL: 0 plain, 1 nt (builtin), 2 asm "sc0 sc1", 3 asm "nt sc0 sc1", 4 asm "sc1"
template <int POL>
__device__ __forceinline__ void st(f32x4 *p, f32x4 v)
{
    if constexpr (POL == 0) *p = v;
    else if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
    else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

template <int BLOCK, int U, int POL>
__global__ void __launch_bounds__(BLOCK) wr(f32x4 *out, size_t nvec, float c)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
    const f32x4 v{c, c, c, c};
#pragma unroll
    for (int u = 0; u < U; ++u) st<POL>(out + v0 + u * BLOCK, v);
}

// grid-stride persistent
template <int BLOCK, int U, int POL>
__global__ void __launch_bounds__(BLOCK) wr_gs(f32x4 *out, size_t nvec, float c)
{
    const f32x4 v{c, c, c, c};
    for (size_t t = blockIdx.x; (t + 1) * (BLOCK * U) <= nvec; t += gridDim.x) {
        const size_t v0 = t * (BLOCK * U) + threadIdx.x;
#pragma unroll
        for (int u = 0; u < U; ++u) st<POL>(out + v0 + u * BLOCK, v);
    }
}

int main()
{
    const size_t n = 64ull << 20, bytes = n * 4, nvec = n / 4;
    const int sets = 2, launches = 10, rounds = 7;
    std::vector<f32x4 *> out(sets);
    for (auto &o : out) CHECK(hipMalloc(&o, bytes));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    struct V {
        std::string name;
        std::function<void(f32x4 *)> run;
    };
    auto g = [&](int block, int u) { return static_cast<unsigned>(nvec / (block * u)); };
    std::vector<V> vs = {
        {"nt_256x4", [&](f32x4 *o) { wr<256, 4, 1><<<g(256, 4), 256, 0, s>>>(o, nvec, 0.5f); }},
        {"plain_256x4", [&](f32x4 *o) { wr<256, 4, 0><<<g(256, 4), 256, 0, s>>>(o, nvec, 0.5f); }},
        {"sc0sc1_256x4", [&](f32x4 *o) { wr<256, 4, 2><<<g(256, 4), 256, 0, s>>>(o, nvec, 0.5f); }},
        {"ntsc0sc1_256x4", [&](f32x4 *o) { wr<256, 4, 3><<<g(256, 4), 256, 0, s>>>(o, nvec, 0.5f); }},
        {"sc1_256x4", [&](f32x4 *o) { wr<256, 4, 4><<<g(256, 4), 256, 0, s>>>(o, nvec, 0.5f); }},
        {"nt_256x1", [&](f32x4 *o) { wr<256, 1, 1><<<g(256, 1), 256, 0, s>>>(o, nvec, 0.5f); }},
        {"nt_256x8", [&](f32x4 *o) { wr<256, 8, 1><<<g(256, 8), 256, 0, s>>>(o, nvec, 0.5f); }},
        {"nt_512x4", [&](f32x4 *o) { wr<512, 4, 1><<<g(512, 4), 512, 0, s>>>(o, nvec, 0.5f); }},
        {"nt_1024x4", [&](f32x4 *o) { wr<1024, 4, 1><<<g(1024, 4), 1024, 0, s>>>(o, nvec, 0.5f); }},
        {"nt_gs1024", [&](f32x4 *o) { wr_gs<256, 4, 1><<<1024, 256, 0, s>>>(o, nvec, 0.5f); }},
        {"nt_gs2048", [&](f32x4 *o) { wr_gs<256, 4, 1><<<2048, 256, 0, s>>>(o, nvec, 0.5f); }},
        {"nt_gs4096", [&](f32x4 *o) { wr_gs<256, 4, 1><<<4096, 256, 0, s>>>(o, nvec, 0.5f); }},
        {"plain_gs2048", [&](f32x4 *o) { wr_gs<256, 4, 0><<<2048, 256, 0, s>>>(o, nvec, 0.5f); }},
        {"hipMemsetD32", [&](f32x4 *o) { CHECK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(o), 0x3f000000, n, s)); }},
    };
    {  // every variant writes every element
        std::vector<float> h(n);
        for (auto &v : vs) {
            CHECK(hipMemset(out[0], 0, bytes));
            v.run(out[0]);
            CHECK(hipMemcpy(h.data(), out[0], bytes, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; ++i) {
                if (h[i] != 0.5f) {
                    fprintf(stderr, "%s missed element %zu\n", v.name.c_str(), i);
                    return 3;
                }
            }
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<double>> t(vs.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            vs[i].run(out[1]);
            CHECK(hipEventRecord(e0, s));
            for (int l = 0; l < launches; ++l) vs[i].run(out[l % sets]);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1e3 / launches);
        }
    }
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(t[i].begin(), t[i].end());
        const double med = t[i][rounds / 2];
        printf("{\"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"GBps\": %.1f, \"frac\": %.4f}\n",
               vs[i].name.c_str(), med, t[i][0], bytes / med / 1e3, bytes / med / 8e6);
    }
    return 0;
}
