// c2_explore3.hip — third standalone C2 experiment (z = x + y, fp32, 256 MiB
// per input, launches cycling over 3 independent sets): staging the inputs
// through LDS with gfx950's LDS-DMA (global_load_lds_dwordx4) instead of
// loading them straight into VGPRs. Not part of the product; it measures what
// the north_star's "LDS-staged" wording would cost on this element-wise path.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o c2_explore3 c2_explore3.hip
//
//   base       the shipped shape: 256 threads, 4 x 16 B per thread per input
//              straight to VGPRs (non-temporal), add, non-temporal store
//   glds_xy_uU both inputs land in LDS by LDS-DMA (each wave its own U x 1 KiB
//              slice per input, so no block barrier: the wave waits vmcnt(0)
//              and reads back its own bytes with ds_read_b128), add, store
//   glds_x_uU  x by LDS-DMA, y straight to VGPRs
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const void *gptr_t;
typedef __attribute__((address_space(3))) void *lptr_t;

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

__device__ __forceinline__ f32x4 ld(const f32x4 *p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(f32x4 v, f32x4 *p) { __builtin_nontemporal_store(v, p); }

template <int U>
__global__ void __launch_bounds__(256) add_base(const f32x4 *x, const f32x4 *y, f32x4 *z)
{
    const size_t base = static_cast<size_t>(blockIdx.x) * 256 * U + threadIdx.x;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld(x + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = ld(y + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) st(a[u] + b[u], z + base + u * 256);
}

// Each wave stages its own slices, laid out lane-linear (the LDS-DMA writes
// wave-uniform base + lane x 16 B), so thread t's vector u of the tile sits
// at lds[wave][u][lane] — the same element the register version loads.
template <int U, bool BOTH>
__global__ void __launch_bounds__(256) add_glds(const f32x4 *x, const f32x4 *y, f32x4 *z)
{
    __shared__ f32x4 lds[(BOTH ? 2 : 1) * 4 * U * 64];
    const int w = threadIdx.x / 64, l = threadIdx.x % 64;
    const size_t base = static_cast<size_t>(blockIdx.x) * 256 * U + threadIdx.x;
    f32x4 *lx = lds + w * U * 64;
    f32x4 *ly = lds + (4 + w) * U * 64;
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_amdgcn_global_load_lds((gptr_t)(x + base + u * 256), (lptr_t)(lx + u * 64), 16,
                                         0, 0);
    f32x4 b[U];
    if constexpr (BOTH) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_global_load_lds((gptr_t)(y + base + u * 256), (lptr_t)(ly + u * 64),
                                             16, 0, 0);
    } else {
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld(y + base + u * 256);
    }
    __builtin_amdgcn_s_waitcnt(0);  // every load (and LDS-DMA write) of this wave retired
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const f32x4 a = lx[u * 64 + l];
        const f32x4 c = BOTH ? ly[u * 64 + l] : b[u];
        st(a + c, z + base + u * 256);
    }
}

struct Variant {
    std::string name;
    std::function<void(const f32x4 *, const f32x4 *, f32x4 *, size_t, hipStream_t)> run;
};

template <int U>
Variant make_base()
{
    return {"base_u" + std::to_string(U),
            [](const f32x4 *x, const f32x4 *y, f32x4 *z, size_t nvec, hipStream_t s) {
                add_base<U><<<nvec / (256 * U), 256, 0, s>>>(x, y, z);
            }};
}

template <int U, bool BOTH>
Variant make_glds()
{
    return {std::string(BOTH ? "glds_xy_u" : "glds_x_u") + std::to_string(U),
            [](const f32x4 *x, const f32x4 *y, f32x4 *z, size_t nvec, hipStream_t s) {
                add_glds<U, BOTH><<<nvec / (256 * U), 256, 0, s>>>(x, y, z);
            }};
}

int main()
{
    const size_t n = 64ull << 20, bytes = n * 4, nvec = n / 4;
    const int sets = 3, launches = 40, rounds = 5;
    std::vector<Variant> vs = {make_base<4>(),         make_base<2>(),        make_glds<4, true>(),
                               make_glds<2, true>(),   make_glds<1, true>(),  make_glds<4, false>(),
                               make_glds<2, false>()};
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    std::vector<f32x4 *> X(sets), Y(sets), Z(sets);
    std::vector<float> h(n), g(n);
    for (size_t i = 0; i < n; ++i) {
        h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
        g[i] = (float)((i * 40503u) % 777) * 1e-2f;
    }
    for (int r = 0; r < sets; ++r) {
        CHECK(hipMalloc(&X[r], bytes));
        CHECK(hipMalloc(&Y[r], bytes));
        CHECK(hipMalloc(&Z[r], bytes));
        CHECK(hipMemcpy(X[r], h.data(), bytes, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(Y[r], g.data(), bytes, hipMemcpyHostToDevice));
    }
    {
        std::vector<float> hz(n);
        for (auto &v : vs) {
            CHECK(hipMemset(Z[0], 0, bytes));
            v.run(X[0], Y[0], Z[0], nvec, s);
            CHECK(hipStreamSynchronize(s));
            CHECK(hipMemcpy(hz.data(), Z[0], bytes, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; ++i)
                if (hz[i] != h[i] + g[i]) {
                    fprintf(stderr, "variant %s wrong at %zu\n", v.name.c_str(), i);
                    return 3;
                }
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto time_variant = [&](const Variant &v) {
        for (int i = 0; i < 3; ++i) v.run(X[i % sets], Y[i % sets], Z[i % sets], nvec, s);
        CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < launches; ++i) v.run(X[i % sets], Y[i % sets], Z[i % sets], nvec, s);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1e3 / launches;
    };
    std::vector<std::vector<double>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) t[i].push_back(time_variant(vs[i]));
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(t[i].begin(), t[i].end());
        const double med = t[i][rounds / 2];
        printf("{\"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"GBps\": %.1f, "
               "\"frac\": %.4f}\n",
               vs[i].name.c_str(), med, t[i][0], 3.0 * bytes / med / 1e3,
               3.0 * bytes / med / 8e6);
    }
    return 0;
}
