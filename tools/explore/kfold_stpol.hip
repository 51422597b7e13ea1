// kfold_stpol.hip — the k-input fold (k = 4, 8) with the output stream's
// cache-policy bits varied: nt (shipped), plain, sc1, sc0 sc1, nt sc0 sc1.
// Written alone, sc1 stores of this shape ran 6 % faster than nt
// (write_explore.jsonl); does that carry into the fold? Same three
// allocations, round-robin (follow-up to kfold_defer.hip).
// Two timings per variant: every launch on the same allocation ("same": the
// 256 MiB output can stay in the 256 MiB Infinity Cache between launches) and
// launches cycling over the three allocations ("rotate", bench.py's setting).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kfold_stpol kfold_stpol.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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

constexpr int BLOCK = 256, U = 4;

struct Ptrs {
    const f32x4 *p[16];
};

__global__ void __launch_bounds__(BLOCK) fold_k(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(in.p[0] + v0 + u * BLOCK);
    for (int j = 1; j < k; ++j) {
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[j] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] += b[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u], out + v0 + u * BLOCK);
}

// POL: 0 plain, 1 nt, 2 sc0 sc1, 3 nt sc0 sc1, 4 sc1
template <int POL>
__device__ __forceinline__ void stp(f32x4 *p, f32x4 v)
{
    if constexpr (POL == 0) *p = v;
    else if constexpr (POL == 1) __builtin_nontemporal_store(v, p);
    else if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off nt sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

template <int POL>
__global__ void __launch_bounds__(BLOCK) fold_pol(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(in.p[0] + v0 + u * BLOCK);
    for (int j = 1; j < k; ++j) {
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[j] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] += b[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) stp<POL>(out + v0 + u * BLOCK, a[u]);
}

int main()
{
    const size_t n = 64ull << 20, bytes = n * 4, nvec = n / 4;
    const size_t ntile = nvec / (BLOCK * U);
    const int allocs = 3, launches = 12, rounds = 7, kmax = 8;
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<char *> base(allocs);
    for (auto &b : base) {
        CHECK(hipMalloc(&b, (kmax + 1) * bytes));
        CHECK(hipMemset(b, 0x3c, (kmax + 1) * bytes));
    }
    const char *names[] = {"plain", "nt", "sc0sc1", "ntsc0sc1", "sc1"};
    const int nv = 5;
    auto run = [&](int v, int k, const Ptrs &p, f32x4 *o) {
        switch (v) {
        case 0: fold_pol<0><<<ntile, BLOCK, 0, s>>>(p, k, o, nvec); break;
        case 1: fold_pol<1><<<ntile, BLOCK, 0, s>>>(p, k, o, nvec); break;
        case 2: fold_pol<2><<<ntile, BLOCK, 0, s>>>(p, k, o, nvec); break;
        case 3: fold_pol<3><<<ntile, BLOCK, 0, s>>>(p, k, o, nvec); break;
        case 4: fold_pol<4><<<ntile, BLOCK, 0, s>>>(p, k, o, nvec); break;
        }
    };
    for (int k : {2, 4, 8}) {
        // t[mode][v]: mode 0 = same allocation (alloc 0), 1 = rotate over 3
        std::vector<std::vector<std::vector<double>>> t(2, std::vector<std::vector<double>>(nv));
        auto ptrs = [&](int a) {
            Ptrs p;
            for (int j = 0; j < 16; ++j) p.p[j] = reinterpret_cast<const f32x4 *>(base[a] + (j % k) * bytes);
            return p;
        };
        auto outp = [&](int a) { return reinterpret_cast<f32x4 *>(base[a] + kmax * bytes); };
        for (int r = 0; r < rounds; ++r) {
            for (int mode = 0; mode < 2; ++mode) {
                for (int v = 0; v < nv; ++v) {
                    run(v, k, ptrs(0), outp(0));
                    CHECK(hipEventRecord(e0, s));
                    for (int i = 0; i < launches; ++i) {
                        const int a = mode ? i % allocs : 0;
                        run(v, k, ptrs(a), outp(a));
                    }
                    CHECK(hipEventRecord(e1, s));
                    CHECK(hipEventSynchronize(e1));
                    float ms;
                    CHECK(hipEventElapsedTime(&ms, e0, e1));
                    t[mode][v].push_back(ms * 1e3 / launches);
                }
            }
        }
        for (int mode = 0; mode < 2; ++mode) {
            for (int v = 0; v < nv; ++v) {
                auto &x = t[mode][v];
                std::sort(x.begin(), x.end());
                const double med = x[rounds / 2], algo = (k + 1.0) * bytes;
                printf("{\"k\": %d, \"buffers\": \"%s\", \"store\": \"%s\", \"median_us\": %.2f, "
                       "\"min_us\": %.2f, \"frac\": %.4f}\n", k, mode ? "rotate3" : "same", names[v],
                       med, x[0], algo / med / 8e6);
            }
        }
    }
    return 0;
}
