// kfold_occ.hip — does limiting occupancy (fewer resident blocks per CU, so
// a narrower window of every stream is open at once) help the k-input fold?
// The span probe (kfold_explore2) found WIDER windows slower. Occupancy is
// capped with dynamic LDS the kernel never touches: 160 KiB per CU / L bytes
// per block = blocks per CU. Same register shape as the product (256 x U, nt
// loads and stores, inputs 0 and 1 up front then one at a time), same
// buffers for every variant, 2 rotating sets, rounds interleaved.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kfold_occ kfold_occ.hip
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

struct Ptrs {
    const f32x4 *p[16];
};

template <int U>
__global__ void __launch_bounds__(256) fold(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (256 * U) + threadIdx.x;
    if (v0 + (U - 1) * 256 >= nvec) return;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(in.p[0] + v0 + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[1] + v0 + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] += b[u];
    for (int j = 2; j < k; ++j) {
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[j] + v0 + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] += b[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u], out + v0 + u * 256);
}

// grid-stride: `grid` blocks, block b folds tiles b, b + grid, ... (the number
// of resident blocks, and so the open window of every stream, is set by the
// grid instead of by LDS)
template <int U>
__global__ void __launch_bounds__(256) fold_gs(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t ntile = nvec / (256 * U);
    for (size_t t = blockIdx.x; t < ntile; t += gridDim.x) {
        const size_t v0 = t * (256 * U) + threadIdx.x;
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(in.p[0] + v0 + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[1] + v0 + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] += b[u];
        for (int j = 2; j < k; ++j) {
#pragma unroll
            for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[j] + v0 + u * 256);
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] += b[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u], out + v0 + u * 256);
    }
}

struct Variant {
    std::string name;
    int k;
    std::function<void(const Ptrs &, f32x4 *, size_t, hipStream_t)> run;
};

template <int U>
Variant make(int k, int lds)
{
    return {"256x" + std::to_string(U) + "_lds" + std::to_string(lds >> 10) + "K", k,
            [k, lds](const Ptrs &p, f32x4 *o, size_t nvec, hipStream_t s) {
                const unsigned g = static_cast<unsigned>(nvec / (256 * U));
                fold<U><<<g, 256, lds, s>>>(p, k, o, nvec);
            }};
}

Variant make_gs(int k, int grid)
{
    return {"gs256x4_grid" + std::to_string(grid), k,
            [k, grid](const Ptrs &p, f32x4 *o, size_t nvec, hipStream_t s) {
                fold_gs<4><<<grid, 256, 0, s>>>(p, k, o, nvec);
            }};
}

int main(int argc, char **argv)
{
    const size_t n     = 64ull << 20;  // fp32 per input
    const size_t bytes = n * 4;
    const size_t nvec  = n / 4;
    const int kmax = 8, sets = 2, launches = 10, rounds = 5;
    std::vector<Variant> vs;
    const int sweep = argc > 1 ? std::atoi(argv[1]) : 0;
    if (sweep == 0) {
        for (int k : {2, 4, 8}) {
            for (int lds : {0, 32 << 10, 40 << 10, 54 << 10, 80 << 10}) vs.push_back(make<4>(k, lds));
            for (int lds : {40 << 10, 80 << 10}) vs.push_back(make<8>(k, lds));
            vs.push_back(make<2>(k, 0));
        }
    } else if (sweep == 2) {  // LDS cap vs a grid-stride grid of the same residency
        for (int k : {2, 4, 8}) {
            vs.push_back(make<4>(k, 0));
            vs.push_back(make<4>(k, 48 << 10));
            for (int g : {512, 768, 1024, 1536}) vs.push_back(make_gs(k, g));
        }
    } else {  // finer: blocks per CU 8 (0), 6 (24K), 5 (32K), 4 (40K), 3 (48K), 2 (80K)
        for (int k : {3, 4, 6, 8}) {
            for (int lds : {0, 24 << 10, 32 << 10, 40 << 10, 48 << 10, 80 << 10})
                vs.push_back(make<4>(k, lds));
            for (int lds : {48 << 10, 80 << 10}) vs.push_back(make<8>(k, lds));
        }
    }
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    std::vector<std::vector<f32x4 *>> in(sets, std::vector<f32x4 *>(kmax));
    std::vector<f32x4 *> out(sets);
    std::vector<float> h(n);
    for (int st = 0; st < sets; ++st) {
        for (int j = 0; j < kmax; ++j) {
            CHECK(hipMalloc(&in[st][j], bytes));
            for (size_t i = 0; i < n; ++i) h[i] = (float)(((i + 7 * j + st) * 2654435761u) % 1000) * 1e-3f;
            CHECK(hipMemcpy(in[st][j], h.data(), bytes, hipMemcpyHostToDevice));
        }
        CHECK(hipMalloc(&out[st], bytes));
    }
    auto ptrs = [&](int st) {
        Ptrs p;
        for (int j = 0; j < 16; ++j) p.p[j] = in[st][j % kmax];
        return p;
    };
    {  // correctness of every variant against the in-order fold on the host
        std::vector<std::vector<float>> hin(kmax, std::vector<float>(n));
        for (int j = 0; j < kmax; ++j)
            CHECK(hipMemcpy(hin[j].data(), in[0][j], bytes, hipMemcpyDeviceToHost));
        std::vector<float> hz(n);
        for (auto &v : vs) {
            CHECK(hipMemset(out[0], 0, bytes));
            v.run(ptrs(0), out[0], nvec, s);
            CHECK(hipStreamSynchronize(s));
            CHECK(hipMemcpy(hz.data(), out[0], bytes, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; ++i) {
                float a = hin[0][i];
                for (int j = 1; j < v.k; ++j) a += hin[j][i];
                if (hz[i] != a) {
                    fprintf(stderr, "variant %s k=%d wrong at %zu\n", v.name.c_str(), v.k, i);
                    return 3;
                }
            }
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto time_variant = [&](const Variant &v) {
        for (int i = 0; i < 2; ++i) v.run(ptrs(i % sets), out[i % sets], nvec, s);
        CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < launches; ++i) v.run(ptrs(i % sets), out[i % sets], nvec, s);
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1e3 / launches;
    };
    std::vector<std::vector<double>> t(vs.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) t[i].push_back(time_variant(vs[i]));
        fprintf(stderr, "round %d done\n", r);
    }
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(t[i].begin(), t[i].end());
        const double med  = t[i][rounds / 2];
        const double algo = (vs[i].k + 1.0) * bytes;
        printf("{\"variant\": \"%s\", \"k\": %d, \"median_us\": %.2f, \"min_us\": %.2f, "
               "\"GBps\": %.1f, \"frac\": %.4f}\n",
               vs[i].name.c_str(), vs[i].k, med, t[i][0], algo / med / 1e3, algo / med / 8e6);
    }
    return 0;
}
