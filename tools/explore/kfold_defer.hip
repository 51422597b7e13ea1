// kfold_defer.hip — the k = 8 fold's writes made burstier: each block folds
// D adjacent tiles and writes them only after the last one's inputs are in
// (D = 1 is the shipped shape), and a grid-stride variant that stores tile
// t-1 after issuing tile t's loads. Each variant runs on the same three
// allocations, round-robin, so placement and clocks are shared
// (follow-up to kfold_placement.hip).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kfold_defer kfold_defer.hip
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

template <int D>
__global__ void __launch_bounds__(BLOCK) fold_defer(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t t0 = static_cast<size_t>(blockIdx.x) * D;
    f32x4 a[D][U];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const size_t v0 = (t0 + d) * (BLOCK * U) + threadIdx.x;
        f32x4 b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[d][u] = __builtin_nontemporal_load(in.p[0] + v0 + u * BLOCK);
        for (int j = 1; j < k; ++j) {
#pragma unroll
            for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[j] + v0 + u * BLOCK);
#pragma unroll
            for (int u = 0; u < U; ++u) a[d][u] += b[u];
        }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const size_t v0 = (t0 + d) * (BLOCK * U) + threadIdx.x;
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[d][u], out + v0 + u * BLOCK);
    }
}

// grid-stride: tile t's result is stored after tile t+stride's first loads
__global__ void __launch_bounds__(BLOCK) fold_lag(Ptrs in, int k, f32x4 *out, size_t ntile)
{
    f32x4 prev[U];
    size_t pt = ~size_t(0);
    for (size_t t = blockIdx.x; t < ntile; t += gridDim.x) {
        const size_t v0 = t * (BLOCK * U) + threadIdx.x;
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(in.p[0] + v0 + u * BLOCK);
        if (pt != ~size_t(0)) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                __builtin_nontemporal_store(prev[u], out + pt * (BLOCK * U) + threadIdx.x + u * BLOCK);
        }
        for (int j = 1; j < k; ++j) {
#pragma unroll
            for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[j] + v0 + u * BLOCK);
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] += b[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) prev[u] = a[u];
        pt = t;
    }
    if (pt != ~size_t(0)) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_nontemporal_store(prev[u], out + pt * (BLOCK * U) + threadIdx.x + u * BLOCK);
    }
}

int main()
{
    const size_t n = 64ull << 20, bytes = n * 4, nvec = n / 4;
    const size_t ntile = nvec / (BLOCK * U);
    const int allocs = 3, launches = 10, rounds = 7, k = 8;
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<char *> base(allocs);
    for (auto &b : base) {
        CHECK(hipMalloc(&b, (k + 1) * bytes));
        CHECK(hipMemset(b, 0x3c, (k + 1) * bytes));
    }
    const char *names[] = {"shipped", "defer2", "defer4", "lag_g2048", "lag_g4096"};
    const int nv = 5;
    auto run = [&](int v, const Ptrs &p, f32x4 *o) {
        switch (v) {
        case 0: fold_k<<<ntile, BLOCK, 0, s>>>(p, k, o, nvec); break;
        case 1: fold_defer<2><<<ntile / 2, BLOCK, 0, s>>>(p, k, o, nvec); break;
        case 2: fold_defer<4><<<ntile / 4, BLOCK, 0, s>>>(p, k, o, nvec); break;
        case 3: fold_lag<<<2048, BLOCK, 0, s>>>(p, k, o, ntile); break;
        case 4: fold_lag<<<4096, BLOCK, 0, s>>>(p, k, o, ntile); break;
        }
    };
    {  // every variant writes the shipped bits
        std::vector<float> want(n), got(n);
        Ptrs p;
        for (int j = 0; j < 16; ++j) p.p[j] = reinterpret_cast<const f32x4 *>(base[0] + (j % k) * bytes);
        f32x4 *o = reinterpret_cast<f32x4 *>(base[0] + k * bytes);
        run(0, p, o);
        CHECK(hipMemcpy(want.data(), o, bytes, hipMemcpyDeviceToHost));
        for (int v = 1; v < nv; ++v) {
            CHECK(hipMemset(o, 0, bytes));
            run(v, p, o);
            CHECK(hipMemcpy(got.data(), o, bytes, hipMemcpyDeviceToHost));
            if (got != want) {
                fprintf(stderr, "%s differs\n", names[v]);
                return 3;
            }
        }
    }
    std::vector<std::vector<std::vector<double>>> t(allocs, std::vector<std::vector<double>>(nv));
    for (int r = 0; r < rounds; ++r) {
        for (int a = 0; a < allocs; ++a) {
            Ptrs p;
            for (int j = 0; j < 16; ++j) p.p[j] = reinterpret_cast<const f32x4 *>(base[a] + (j % k) * bytes);
            f32x4 *o = reinterpret_cast<f32x4 *>(base[a] + k * bytes);
            for (int v = 0; v < nv; ++v) {
                run(v, p, o);
                CHECK(hipEventRecord(e0, s));
                for (int i = 0; i < launches; ++i) run(v, p, o);
                CHECK(hipEventRecord(e1, s));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                t[a][v].push_back(ms * 1e3 / launches);
            }
        }
    }
    for (int a = 0; a < allocs; ++a) {
        for (int v = 0; v < nv; ++v) {
            auto &x = t[a][v];
            std::sort(x.begin(), x.end());
            const double med = x[rounds / 2], algo = (k + 1.0) * bytes;
            printf("{\"k\": %d, \"alloc\": %d, \"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, "
                   "\"frac\": %.4f}\n", k, a, names[v], med, x[0], algo / med / 8e6);
        }
    }
    return 0;
}
