// kfold_ceiling.hip — what bounds the k-input fold at k = 4..8 (DESIGN.md §10
// item 2): the device's stream ceilings measured with the same register shape
// (256 threads x 4 16-B vectors per input, nt loads and stores, one tile per
// block) as the shipped fold, and the two-level fold VERDICT r01 asked for.
//
//   read_k    k input streams, no output stream (each lane folds its vectors
//             and stores only if the fold hits an impossible pattern): the
//             read ceiling for k concurrent streams
//   write     one output stream, no input
//   fold_k    the shipped shape (inputs 0 and 1 up front, then one at a time)
//   twolevel  k = 8 as fold(x0..x3) -> t, then fold(t, x4..x7) -> out: same
//             left-fold bits, 11 stream-units of traffic for 9 algorithmic
//
// Rates are algorithmic bytes / time (read_k: k units, write: 1, fold_k: k+1,
// twolevel: 9). 256 MiB per stream, 2 rotating sets, median of 5 x 20 launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kfold_ceiling kfold_ceiling.hip
//   ./kfold_ceiling > profiles/r02/kfold_ceiling.jsonl
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

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

__global__ void __launch_bounds__(BLOCK) read_k(Ptrs in, int k, u32x4 *sink, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
    u32x4 a[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = u32x4{0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
        f32x4 b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[j] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] ^= __builtin_bit_cast(u32x4, b[u]);
    }
    u32x4 r = a[0] ^ a[1] ^ a[2] ^ a[3];
    // never true for the data below (every input word is a float in [0, 1))
    if (r.x == 0xffffffffu && r.y == 0xffffffffu) sink[threadIdx.x] = r;
}

__global__ void __launch_bounds__(BLOCK) write_1(f32x4 *out, size_t nvec, float c)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_nontemporal_store(f32x4{c, c, c, c}, out + v0 + u * BLOCK);
}

// the shipped register fold (kf_reduce_kernels.hpp reduce_kernel, KC = 0, f32 SUM)
__global__ void __launch_bounds__(BLOCK) fold_k(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(in.p[0] + v0 + u * BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[1] + v0 + u * BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] += b[u];
    for (int j = 2; j < k; ++j) {
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[j] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] += b[u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u], out + v0 + u * BLOCK);
}

struct Variant {
    std::string name;
    int k;
    double units;  // algorithmic bytes / stream bytes
    std::function<void(int set, hipStream_t)> run;
};

int main()
{
    const size_t n     = 64ull << 20;  // fp32 per stream
    const size_t bytes = n * 4;
    const size_t nvec  = n / 4;
    const unsigned g   = static_cast<unsigned>(nvec / (BLOCK * U));
    const int kmax = 8, sets = 2, launches = 20, rounds = 5;
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    std::vector<std::vector<f32x4 *>> in(sets, std::vector<f32x4 *>(kmax));
    std::vector<f32x4 *> out(sets), tmp(sets);
    u32x4 *sink;
    CHECK(hipMalloc(&sink, BLOCK * sizeof(u32x4)));
    std::vector<float> h(n);
    for (int st = 0; st < sets; ++st) {
        for (int j = 0; j < kmax; ++j) {
            CHECK(hipMalloc(&in[st][j], bytes));
            for (size_t i = 0; i < n; ++i) h[i] = (float)(((i + 7 * j + st) * 2654435761u) % 1000) * 1e-3f;
            CHECK(hipMemcpy(in[st][j], h.data(), bytes, hipMemcpyHostToDevice));
        }
        CHECK(hipMalloc(&out[st], bytes));
        CHECK(hipMalloc(&tmp[st], bytes));
    }
    auto ptrs = [&](int st, int from) {
        Ptrs p;
        for (int j = 0; j < 16; ++j) p.p[j] = in[st][(from + j) % kmax];
        return p;
    };
    std::vector<Variant> vs;
    for (int k : {1, 2, 4, 8}) {
        vs.push_back({"read_" + std::to_string(k), k, double(k), [&, k](int st, hipStream_t q) {
                          read_k<<<g, BLOCK, 0, q>>>(ptrs(st, 0), k, sink, nvec);
                      }});
    }
    vs.push_back({"write", 0, 1.0, [&](int st, hipStream_t q) {
                      write_1<<<g, BLOCK, 0, q>>>(out[st], nvec, 0.5f);
                  }});
    for (int k : {2, 4, 8}) {
        vs.push_back({"fold_" + std::to_string(k), k, k + 1.0, [&, k](int st, hipStream_t q) {
                          fold_k<<<g, BLOCK, 0, q>>>(ptrs(st, 0), k, out[st], nvec);
                      }});
    }
    vs.push_back({"twolevel_8", 8, 9.0, [&](int st, hipStream_t q) {
                      fold_k<<<g, BLOCK, 0, q>>>(ptrs(st, 0), 4, tmp[st], nvec);
                      Ptrs p = ptrs(st, 3);  // p[0] = in[3] is replaced by t
                      p.p[0] = tmp[st];
                      fold_k<<<g, BLOCK, 0, q>>>(p, 5, out[st], nvec);
                  }});
    {  // the two-level fold gives the one-level bits
        std::vector<float> a(n), b(n);
        vs[vs.size() - 2].run(0, s);
        CHECK(hipStreamSynchronize(s));
        CHECK(hipMemcpy(a.data(), out[0], bytes, hipMemcpyDeviceToHost));
        CHECK(hipMemset(out[0], 0, bytes));
        vs.back().run(0, s);
        CHECK(hipStreamSynchronize(s));
        CHECK(hipMemcpy(b.data(), out[0], bytes, hipMemcpyDeviceToHost));
        if (std::memcmp(a.data(), b.data(), bytes) != 0) {
            fprintf(stderr, "two-level fold differs from the one-level fold\n");
            return 3;
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto time_variant = [&](const Variant &v) {
        for (int i = 0; i < 2; ++i) v.run(i % sets, s);
        CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < launches; ++i) v.run(i % sets, s);
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
        const double med  = t[i][rounds / 2];
        const double algo = vs[i].units * bytes;
        printf("{\"variant\": \"%s\", \"k\": %d, \"median_us\": %.2f, \"min_us\": %.2f, "
               "\"GBps\": %.1f, \"frac\": %.4f}\n",
               vs[i].name.c_str(), vs[i].k, med, t[i][0], algo / med / 1e3, algo / med / 8e6);
    }
    return 0;
}
