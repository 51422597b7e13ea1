// kfold_explore.hip — standalone experiment for the k-input fold (star roots,
// the P2P shard fold, bench checks): z = ((x0 + x1) + x2) + ... (fp32, 256 MiB
// per input, k = 3, 4, 8). Not part of the product; results feed the k > 2
// path in kf_capi.hip / kf_reduce_kernels.hpp.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kfold_explore kfold_explore.hip
//   ./kfold_explore > results.jsonl
//
// Load schedules compared (the adds are always in input order, so every
// variant is bit-identical):
//   serial   inputs 0 and 1 up front, then one input at a time (the shipped
//            runtime-k loop): a thread waits a full DRAM latency per input;
//   pipe     input j+1's loads are issued before input j is added, so two
//            inputs' loads are always in flight per thread;
//   all      every input's loads before the first add (compile-time k);
//   pipe2    like pipe, two inputs ahead.
// Timing: HIP events around 20 launches cycling over 2 independent input
// sets (cold Infinity Cache), 5 interleaved rounds, median.
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

__device__ __forceinline__ f32x4 ld(const f32x4 *p) { return __builtin_nontemporal_load(p); }

// MODE 0 serial, 1 pipe, 3 pipe2 (runtime k); MODE 2 all (compile-time K)
template <int BLOCK, int U, int MODE, int K>
__global__ void __launch_bounds__(BLOCK) fold(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;  // exact multiple in this harness
    f32x4 acc[U];
    if constexpr (MODE == 2) {
        f32x4 v[K][U];
#pragma unroll
        for (int j = 0; j < K; ++j)
#pragma unroll
            for (int u = 0; u < U; ++u) v[j][u] = ld(in.p[j] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc[u] = v[0][u];
#pragma unroll
            for (int j = 1; j < K; ++j) acc[u] += v[j][u];
        }
    } else if constexpr (MODE == 0) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld(in.p[0] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld(in.p[1] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = a[u] + b[u];
        for (int j = 2; j < k; ++j) {
#pragma unroll
            for (int u = 0; u < U; ++u) b[u] = ld(in.p[j] + v0 + u * BLOCK);
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] += b[u];
        }
    } else if constexpr (MODE == 1) {
        f32x4 a[U], b[U], c[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld(in.p[0] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld(in.p[1] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = ld(in.p[2] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = a[u] + b[u];
        for (int j = 3; j < k; ++j) {
#pragma unroll
            for (int u = 0; u < U; ++u) b[u] = ld(in.p[j] + v0 + u * BLOCK);
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] += c[u];
#pragma unroll
            for (int u = 0; u < U; ++u) c[u] = b[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += c[u];
    } else {  // MODE 3: two inputs ahead
        f32x4 a[U], b[U], c[U], d[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld(in.p[0] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld(in.p[1] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = ld(in.p[2] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) d[u] = ld(in.p[3 < k ? 3 : 2] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] = a[u] + b[u];
        for (int j = 4; j < k; ++j) {
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] = ld(in.p[j] + v0 + u * BLOCK);
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] += c[u];
#pragma unroll
            for (int u = 0; u < U; ++u) { c[u] = d[u]; d[u] = a[u]; }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += c[u];
        if (k > 3) {
#pragma unroll
            for (int u = 0; u < U; ++u) acc[u] += d[u];
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(acc[u], out + v0 + u * BLOCK);
}

struct Variant {
    std::string name;
    int k;
    std::function<void(const Ptrs &, f32x4 *, size_t, hipStream_t)> run;
};

template <int BLOCK, int U, int MODE, int K>
Variant make(int k)
{
    static const char *modes[] = {"serial", "pipe", "all", "pipe2"};
    Variant v;
    v.k    = k;
    v.name = std::string(modes[MODE]) + "_b" + std::to_string(BLOCK) + "_u" + std::to_string(U) +
             "_k" + std::to_string(k);
    v.run = [k](const Ptrs &p, f32x4 *out, size_t nvec, hipStream_t s) {
        fold<BLOCK, U, MODE, K><<<nvec / (BLOCK * U), BLOCK, 0, s>>>(p, k, out, nvec);
    };
    return v;
}

template <int K>
void add_k(std::vector<Variant> &vs)
{
    vs.push_back(make<256, 4, 0, 0>(K));
    vs.push_back(make<256, 2, 0, 0>(K));
    vs.push_back(make<256, 1, 0, 0>(K));
    vs.push_back(make<1024, 1, 0, 0>(K));
    vs.push_back(make<256, 4, 1, 0>(K));
    vs.push_back(make<256, 2, 1, 0>(K));
    vs.push_back(make<256, 1, 1, 0>(K));
    vs.push_back(make<512, 2, 1, 0>(K));
    vs.push_back(make<1024, 1, 1, 0>(K));
    vs.push_back(make<256, 2, 3, 0>(K));
    vs.push_back(make<256, 1, 3, 0>(K));
    vs.push_back(make<256, 1, 2, K>(K));
    vs.push_back(make<256, 2, 2, K>(K));
    vs.push_back(make<1024, 1, 2, K>(K));
}

int main()
{
    const size_t n     = 64ull << 20;  // fp32 per input
    const size_t bytes = n * 4;
    const size_t nvec  = n / 4;
    const int kmax = 8, sets = 2, launches = 20, rounds = 5;
    std::vector<Variant> vs;
    add_k<3>(vs);
    add_k<4>(vs);
    add_k<8>(vs);
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    std::vector<std::vector<f32x4 *>> in(sets, std::vector<f32x4 *>(kmax));
    std::vector<f32x4 *> out(sets);
    std::vector<float> h(n);
    for (int st = 0; st < sets; ++st) {
        for (int j = 0; j < kmax; ++j) {
            CHECK(hipMalloc(&in[st][j], bytes));
            for (size_t i = 0; i < n; ++i) h[i] = (float)(((i + 7 * j) * 2654435761u) % 1000) * 1e-3f;
            CHECK(hipMemcpy(in[st][j], h.data(), bytes, hipMemcpyHostToDevice));
        }
        CHECK(hipMalloc(&out[st], bytes));
    }
    auto ptrs = [&](int st) {
        Ptrs p;
        for (int j = 0; j < 16; ++j) p.p[j] = in[st][j % kmax];
        return p;
    };
    // correctness: every variant equals the in-order fold (host), sampled
    {
        std::vector<std::vector<float>> hin(kmax, std::vector<float>(n));
        for (int j = 0; j < kmax; ++j)
            CHECK(hipMemcpy(hin[j].data(), in[0][j], bytes, hipMemcpyDeviceToHost));
        std::vector<float> hz(n);
        for (auto &v : vs) {
            CHECK(hipMemset(out[0], 0, bytes));
            v.run(ptrs(0), out[0], nvec, s);
            CHECK(hipStreamSynchronize(s));
            CHECK(hipMemcpy(hz.data(), out[0], bytes, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; i += 4099) {
                float a = hin[0][i];
                for (int j = 1; j < v.k; ++j) a += hin[j][i];
                if (hz[i] != a) {
                    fprintf(stderr, "variant %s wrong at %zu: %g vs %g\n", v.name.c_str(), i,
                            hz[i], a);
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
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) t[i].push_back(time_variant(vs[i]));
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(t[i].begin(), t[i].end());
        const double med = t[i][rounds / 2];
        const double algo = (vs[i].k + 1.0) * bytes;
        printf("{\"variant\": \"%s\", \"k\": %d, \"median_us\": %.2f, \"min_us\": %.2f, "
               "\"GBps\": %.1f, \"frac\": %.4f}\n",
               vs[i].name.c_str(), vs[i].k, med, t[i][0], algo / med / 1e3, algo / med / 8e6);
    }
    return 0;
}
