// kfold_ceiling4.hip — (follow-up to kfold_ceiling{,2,3}.hip: the layout rule, over several allocations) what bounds the k-input fold at k = 4..8 (DESIGN.md §10
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


// the fold without its output stream: stores only on an impossible value
__global__ void __launch_bounds__(BLOCK) fold_nostore(Ptrs in, int k, f32x4 *out, size_t nvec)
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
    f32x4 r = a[0] + a[1] + a[2] + a[3];
    if (r.x == -1.0f && r.y == -2.0f) out[threadIdx.x] = r;
}


struct Variant {
    int k;
    size_t in_gap, out_off;  // input j at j*(bytes+in_gap), output at k*bytes+out_off
};

int main()
{
    const size_t n     = 64ull << 20;
    const size_t bytes = n * 4;
    const size_t nvec  = n / 4;
    const unsigned g   = static_cast<unsigned>(nvec / (BLOCK * U));
    const int sets = 2, allocs = 3, launches = 20, rounds = 5;
    const size_t G1 = 4096, G2 = 65536 + 256;
    const std::vector<Variant> vs = {
        {8, G1, 8 * G1}, {8, G1, 0}, {8, 0, 8 * G1}, {8, 0, 0}, {8, G1 + 64, 8 * (G1 + 64)},
        {8, 2 * G1, 16 * G1}, {8, 512, 8 * 512}, {8, 16384, 8 * 16384},
        {4, G1, 4 * G1}, {4, 0, 0}, {2, G1, 2 * G1}, {2, 0, 0},
    };
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    const size_t span = 8 * (bytes + G2) + bytes + 8 * G2 + 65536;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<char *> keep;
    for (int al = 0; al < allocs; ++al) {
    std::vector<char *> base(sets);
    for (int st = 0; st < sets; ++st) {
        CHECK(hipMalloc(&base[st], span));
        CHECK(hipMemset(base[st], 0x3c, span));
    }
    for (const Variant &v : vs) {
        auto run = [&](int st) {
            Ptrs p;
            for (int j = 0; j < 16; ++j)
                p.p[j] = reinterpret_cast<const f32x4 *>(base[st] + (j % v.k) * (bytes + v.in_gap));
            f32x4 *o = reinterpret_cast<f32x4 *>(base[st] + v.k * bytes + v.out_off);
            fold_k<<<g, BLOCK, 0, s>>>(p, v.k, o, nvec);
        };
        std::vector<double> t;
        for (int r = 0; r < rounds; ++r) {
            for (int i = 0; i < 2; ++i) run(i % sets);
            CHECK(hipEventRecord(e0, s));
            for (int i = 0; i < launches; ++i) run(i % sets);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1e3 / launches);
        }
        std::sort(t.begin(), t.end());
        const double med  = t[rounds / 2];
        const double algo = (v.k + 1.0) * bytes;
        printf("{\"alloc\": %d, \"k\": %d, \"in_gap\": %zu, \"out_off\": %zu, \"median_us\": %.2f, \"min_us\": %.2f, "
               "\"GBps\": %.1f, \"frac\": %.4f}\n",
               al, v.k, v.in_gap, v.out_off, med, t[0], algo / med / 1e3, algo / med / 8e6);
    }
        for (char *p : base) keep.push_back(p);  // the next allocation lands elsewhere
    }
    return 0;
}
