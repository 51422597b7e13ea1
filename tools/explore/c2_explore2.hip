// c2_explore2.hip — second standalone C2 experiment (z = x + y, fp32, 256 MiB
// per input, launches cycling over 3 independent sets): block -> tile
// mappings the first sweep (c2_explore.hip) did not cover. Not part of the
// product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o c2_explore2 c2_explore2.hip
//
//   base      the shipped shape: 256 threads, 4 x 16 B per thread per input,
//             thread t loads vectors t, t+256, t+512, t+768 of the block's tile
//   wavecont  each wave owns 4 consecutive KiB of the tile (4 back-to-back
//             1-KiB wave-instructions) instead of a 1-KiB slice every 4 KiB
//   xcd       tile = XCD-major remap of blockIdx (consecutive tiles on one
//             XCD: dispatch is round-robin over the 8 XCDs)
//   persist   grid = CUs x occupancy, grid-stride over tiles, the next tile's
//             loads issued before the current tile's stores (software pipeline)
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
__device__ __forceinline__ void st(f32x4 v, f32x4 *p) { __builtin_nontemporal_store(v, p); }

template <int U>
__device__ __forceinline__ void tile_add(const f32x4 *x, const f32x4 *y, f32x4 *z, size_t base,
                                         int stride)
{
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld(x + base + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = ld(y + base + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) st(a[u] + b[u], z + base + u * stride);
}

// MODE 0 base, 1 wavecont, 2 xcd
template <int BLOCK, int U, int MODE>
__global__ void __launch_bounds__(BLOCK) add(const f32x4 *x, const f32x4 *y, f32x4 *z, size_t nvec)
{
    size_t t = blockIdx.x;
    if constexpr (MODE == 2) {
        const size_t per = gridDim.x / 8;  // grid is a multiple of 8 here
        t = (blockIdx.x % 8) * per + blockIdx.x / 8;
    }
    const size_t tile = static_cast<size_t>(BLOCK) * U;
    if constexpr (MODE == 1) {
        const int w = threadIdx.x / 64, l = threadIdx.x % 64;
        tile_add<U>(x, y, z, t * tile + static_cast<size_t>(w) * 64 * U + l, 64);
    } else {
        tile_add<U>(x, y, z, t * tile + threadIdx.x, BLOCK);
    }
}

template <int BLOCK, int U>
__global__ void __launch_bounds__(BLOCK) add_persist(const f32x4 *x, const f32x4 *y, f32x4 *z,
                                                     size_t nvec)
{
    const size_t tile   = static_cast<size_t>(BLOCK) * U;
    const size_t ntiles = nvec / tile;
    size_t t            = blockIdx.x;
    if (t >= ntiles) return;
    f32x4 a[U], b[U];
    size_t base = t * tile + threadIdx.x;
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld(x + base + u * BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = ld(y + base + u * BLOCK);
    for (;;) {
        const size_t tn = t + gridDim.x;
        f32x4 c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = a[u] + b[u];
        if (tn < ntiles) {
            const size_t nb = tn * tile + threadIdx.x;
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] = ld(x + nb + u * BLOCK);
#pragma unroll
            for (int u = 0; u < U; ++u) b[u] = ld(y + nb + u * BLOCK);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st(c[u], z + base + u * BLOCK);
        if (tn >= ntiles) break;
        t    = tn;
        base = t * tile + threadIdx.x;
    }
}

struct Variant {
    std::string name;
    std::function<void(const f32x4 *, const f32x4 *, f32x4 *, size_t, hipStream_t)> run;
};

template <int BLOCK, int U, int MODE>
Variant make(const char *tag)
{
    Variant v;
    v.name = std::string(tag) + "_b" + std::to_string(BLOCK) + "_u" + std::to_string(U);
    v.run  = [](const f32x4 *x, const f32x4 *y, f32x4 *z, size_t nvec, hipStream_t s) {
        add<BLOCK, U, MODE><<<nvec / (BLOCK * U), BLOCK, 0, s>>>(x, y, z, nvec);
    };
    return v;
}

template <int BLOCK, int U>
Variant make_persist(int per_cu)
{
    Variant v;
    v.name = "persist_b" + std::to_string(BLOCK) + "_u" + std::to_string(U) + "_x" +
             std::to_string(per_cu);
    v.run = [per_cu](const f32x4 *x, const f32x4 *y, f32x4 *z, size_t nvec, hipStream_t s) {
        add_persist<BLOCK, U><<<256 * per_cu, BLOCK, 0, s>>>(x, y, z, nvec);
    };
    return v;
}

int main()
{
    const size_t n = 64ull << 20, bytes = n * 4, nvec = n / 4;
    const int sets = 3, launches = 40, rounds = 5;
    std::vector<Variant> vs = {
        make<256, 4, 0>("base"),       make<1024, 1, 0>("base"),     make<256, 4, 1>("wavecont"),
        make<256, 8, 1>("wavecont"),   make<256, 4, 2>("xcd"),       make<1024, 1, 2>("xcd"),
        make_persist<256, 4>(8),       make_persist<256, 4>(4),      make_persist<256, 2>(8),
        make_persist<256, 2>(16),      make_persist<512, 2>(4),      make_persist<1024, 1>(2),
    };
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    std::vector<f32x4 *> X(sets), Y(sets), Z(sets);
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
    for (int r = 0; r < sets; ++r) {
        CHECK(hipMalloc(&X[r], bytes));
        CHECK(hipMalloc(&Y[r], bytes));
        CHECK(hipMalloc(&Z[r], bytes));
        CHECK(hipMemcpy(X[r], h.data(), bytes, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(Y[r], h.data(), bytes, hipMemcpyHostToDevice));
    }
    {
        std::vector<float> hz(n);
        for (auto &v : vs) {
            CHECK(hipMemset(Z[0], 0, bytes));
            v.run(X[0], Y[0], Z[0], nvec, s);
            CHECK(hipStreamSynchronize(s));
            CHECK(hipMemcpy(hz.data(), Z[0], bytes, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; i += 997)
                if (hz[i] != h[i] + h[i]) {
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
