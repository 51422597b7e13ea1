// c2_explore4.hip — C2 (z = x + y, 256 MiB fp32) with the shipped 256 x 4
// load schedule (8 loads in flight per lane) but an address map in which each
// of a lane's 4 vectors lies in a different quarter of the bucket: vector u of
// block b, lane t is ((u * nb + b) * 256 + t). Every store instruction across
// consecutive blocks then forms the 4 KiB-per-block pattern that wrote
// fastest in write_explore.hip (256 x 1, 6.63 TB/s) while each lane keeps 4
// vectors of each input in flight. Against the shipped map, same process,
// 3 rotating bucket sets, median of 7 x 20.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o c2_explore4 c2_explore4.hip
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

__device__ __forceinline__ f32x4 ld(const f32x4 *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(f32x4 *p, f32x4 v) { __builtin_nontemporal_store(v, p); }

// shipped: block b covers vectors [b*B*U, (b+1)*B*U), lane t vector u at b*B*U + u*B + t
template <int B, int U>
__global__ void __launch_bounds__(B) c2_block(const f32x4 *x, const f32x4 *y, f32x4 *z)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (B * U) + threadIdx.x;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld(x + v0 + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = ld(y + v0 + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u) st(z + v0 + u * B, a[u] + b[u]);
}

// spread: lane t of block b, vector u at (u*nb + b)*B + t
template <int B, int U>
__global__ void __launch_bounds__(B) c2_spread(const f32x4 *x, const f32x4 *y, f32x4 *z)
{
    const size_t nb = gridDim.x;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld(x + (u * nb + blockIdx.x) * B + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = ld(y + (u * nb + blockIdx.x) * B + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u) st(z + (u * nb + blockIdx.x) * B + threadIdx.x, a[u] + b[u]);
}

// spread, stores issued as soon as each sum is ready (interleaved)
template <int B, int U>
__global__ void __launch_bounds__(B) c2_spread_pairs(const f32x4 *x, const f32x4 *y, f32x4 *z)
{
    const size_t nb = gridDim.x;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        a[u] = ld(x + (u * nb + blockIdx.x) * B + threadIdx.x);
        b[u] = ld(y + (u * nb + blockIdx.x) * B + threadIdx.x);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) st(z + (u * nb + blockIdx.x) * B + threadIdx.x, a[u] + b[u]);
}

int main()
{
    const size_t n = 64ull << 20, bytes = n * 4, nvec = n / 4;
    const int sets = 3, launches = 20, rounds = 7;
    std::vector<f32x4 *> X(sets), Y(sets), Z(sets);
    std::vector<float> h(n);
    for (int s = 0; s < sets; ++s) {
        CHECK(hipMalloc(&X[s], bytes));
        CHECK(hipMalloc(&Y[s], bytes));
        CHECK(hipMalloc(&Z[s], bytes));
        for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u + s) % 1000) * 1e-3f;
        CHECK(hipMemcpy(X[s], h.data(), bytes, hipMemcpyHostToDevice));
        for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 40503u + 7 * s) % 999) * 1e-3f;
        CHECK(hipMemcpy(Y[s], h.data(), bytes, hipMemcpyHostToDevice));
    }
    hipStream_t st_;
    CHECK(hipStreamCreate(&st_));
    struct V {
        std::string name;
        std::function<void(int)> run;
    };
    std::vector<V> vs = {
        {"block_256x4", [&](int s) { c2_block<256, 4><<<nvec / 1024, 256, 0, st_>>>(X[s], Y[s], Z[s]); }},
        {"block_256x1", [&](int s) { c2_block<256, 1><<<nvec / 256, 256, 0, st_>>>(X[s], Y[s], Z[s]); }},
        {"spread_256x4", [&](int s) { c2_spread<256, 4><<<nvec / 1024, 256, 0, st_>>>(X[s], Y[s], Z[s]); }},
        {"spread_256x2", [&](int s) { c2_spread<256, 2><<<nvec / 512, 256, 0, st_>>>(X[s], Y[s], Z[s]); }},
        {"spread_256x8", [&](int s) { c2_spread<256, 8><<<nvec / 2048, 256, 0, st_>>>(X[s], Y[s], Z[s]); }},
        {"spread_pairs_256x4", [&](int s) { c2_spread_pairs<256, 4><<<nvec / 1024, 256, 0, st_>>>(X[s], Y[s], Z[s]); }},
        {"spread_128x4", [&](int s) { c2_spread<128, 4><<<nvec / 512, 128, 0, st_>>>(X[s], Y[s], Z[s]); }},
        {"spread_512x4", [&](int s) { c2_spread<512, 4><<<nvec / 2048, 512, 0, st_>>>(X[s], Y[s], Z[s]); }},
    };
    {  // every variant: z == x + y exactly
        std::vector<float> hx(n), hy(n), hz(n);
        CHECK(hipMemcpy(hx.data(), X[0], bytes, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hy.data(), Y[0], bytes, hipMemcpyDeviceToHost));
        for (auto &v : vs) {
            CHECK(hipMemset(Z[0], 0, bytes));
            v.run(0);
            CHECK(hipMemcpy(hz.data(), Z[0], bytes, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; ++i) {
                if (hz[i] != hx[i] + hy[i]) {
                    fprintf(stderr, "%s wrong at %zu\n", v.name.c_str(), i);
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
            vs[i].run(0);
            CHECK(hipEventRecord(e0, st_));
            for (int l = 0; l < launches; ++l) vs[i].run(l % sets);
            CHECK(hipEventRecord(e1, st_));
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
               vs[i].name.c_str(), med, t[i][0], 3.0 * bytes / med / 1e3, 3.0 * bytes / med / 8e6);
    }
    return 0;
}
