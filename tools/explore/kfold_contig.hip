// kfold_contig.hip — kfold_placement.hip with half of the allocations made
// with hipExtMallocWithFlags(hipDeviceMallocContiguous): does physically
// contiguous memory take the placement lottery out of the k = 8 fold and C2?
// Allocations alternate default / contiguous, timed round-robin.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kfold_contig kfold_contig.hip
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

int main()
{
    const size_t n = 64ull << 20, bytes = n * 4, nvec = n / 4;
    const unsigned g = static_cast<unsigned>(nvec / (BLOCK * U));
    const int allocs = 12, launches = 10, rounds = 7;
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int k : {8, 2}) {
        std::vector<char *> base(allocs);
        for (int a = 0; a < allocs; ++a) {
            auto &b = base[a];
            if (a % 2) CHECK(hipExtMallocWithFlags(reinterpret_cast<void **>(&b), (k + 1) * bytes,
                                                   hipDeviceMallocContiguous));
            else CHECK(hipMalloc(&b, (k + 1) * bytes));
            CHECK(hipMemset(b, 0x3c, (k + 1) * bytes));
        }
        std::vector<std::vector<double>> t(allocs);
        for (int r = 0; r < rounds; ++r) {
            for (int a = 0; a < allocs; ++a) {
                Ptrs p;
                for (int j = 0; j < 16; ++j) p.p[j] = reinterpret_cast<const f32x4 *>(base[a] + (j % k) * bytes);
                f32x4 *o = reinterpret_cast<f32x4 *>(base[a] + k * bytes);
                fold_k<<<g, BLOCK, 0, s>>>(p, k, o, nvec);
                CHECK(hipEventRecord(e0, s));
                for (int i = 0; i < launches; ++i) fold_k<<<g, BLOCK, 0, s>>>(p, k, o, nvec);
                CHECK(hipEventRecord(e1, s));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                t[a].push_back(ms * 1e3 / launches);
            }
        }
        for (int a = 0; a < allocs; ++a) {
            std::sort(t[a].begin(), t[a].end());
            const double med = t[a][rounds / 2], algo = (k + 1.0) * bytes;
            printf("{\"k\": %d, \"alloc\": %d, \"contiguous\": %d, \"va\": \"%p\", \"median_us\": %.2f, \"min_us\": %.2f, "
                   "\"max_us\": %.2f, \"frac\": %.4f}\n",
                   k, a, a % 2, (void *)base[a], med, t[a][0], t[a].back(), algo / med / 8e6);
        }
        for (auto b : base) CHECK(hipFree(b));
    }
    return 0;
}
