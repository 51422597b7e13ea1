// c2_rot.hip — C2 (z = x + y, 256 MiB fp32, 3 rotating sets) with the order
// of a lane's 4 vectors rotated per block (block b starts at vector b mod 4),
// for the stores only, the loads only, or both, against the shipped order —
// so the blocks resident together do not all hit the same 4 KiB quarter of
// their 16 KiB tiles with the same instruction. Not part of the product.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o c2_rot tools/explore/c2_rot.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

template <int ROTL, int ROTS>
__global__ void __launch_bounds__(256) c2(const f4 *x, const f4 *y, f4 *z)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * 1024 + threadIdx.x;
    const int r     = blockIdx.x & 3;
    f4 a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int u = ROTL ? (i + r) & 3 : i;
        a[i] = __builtin_nontemporal_load(x + v0 + u * 256);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int u = ROTL ? (i + r) & 3 : i;
        b[i] = __builtin_nontemporal_load(y + v0 + u * 256);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        // element i holds vector (ROTL ? (i + r) & 3 : i)
        const int j = ROTS ? (i + r) & 3 : i;           // store order
        const int src = ROTL ? (j - r) & 3 : j;         // which register holds vector j
        f4 s = a[0] + b[0];
        if (src == 1) s = a[1] + b[1];
        if (src == 2) s = a[2] + b[2];
        if (src == 3) s = a[3] + b[3];
        __builtin_nontemporal_store(s, z + v0 + j * 256);
    }
}

int main()
{
    const size_t n = 64ull << 20, bytes = n * 4, nv = n / 4;
    const int sets = 3, launches = 20, rounds = 7;
    std::vector<f4 *> X(sets), Y(sets), Z(sets);
    std::vector<float> h(n);
    for (int s = 0; s < sets; ++s) {
        CHECK(hipMalloc(&X[s], bytes));
        CHECK(hipMalloc(&Y[s], bytes));
        CHECK(hipMalloc(&Z[s], bytes));
        for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u + s) % 1000) * 1e-3f;
        CHECK(hipMemcpy(X[s], h.data(), bytes, hipMemcpyHostToDevice));
        for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 40503u + 7 * s) % 997) * 1e-3f;
        CHECK(hipMemcpy(Y[s], h.data(), bytes, hipMemcpyHostToDevice));
    }
    hipStream_t st;
    CHECK(hipStreamCreate(&st));
    struct V {
        std::string name;
        void (*k)(const f4 *, const f4 *, f4 *);
    };
    std::vector<V> vs = {{"shipped", c2<0, 0>}, {"rot_stores", c2<0, 1>}, {"rot_loads", c2<1, 0>},
                         {"rot_both", c2<1, 1>}};
    const unsigned g = static_cast<unsigned>(nv / 1024);
    {  // correctness
        std::vector<float> hx(n), hy(n), hz(n);
        CHECK(hipMemcpy(hx.data(), X[0], bytes, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hy.data(), Y[0], bytes, hipMemcpyDeviceToHost));
        for (auto &v : vs) {
            CHECK(hipMemset(Z[0], 0, bytes));
            v.k<<<g, 256, 0, st>>>(X[0], Y[0], Z[0]);
            CHECK(hipStreamSynchronize(st));
            CHECK(hipMemcpy(hz.data(), Z[0], bytes, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; ++i)
                if (hz[i] != hx[i] + hy[i]) {
                    fprintf(stderr, "%s wrong at %zu\n", v.name.c_str(), i);
                    return 3;
                }
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<double>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) {
            vs[i].k<<<g, 256, 0, st>>>(X[0], Y[0], Z[0]);
            CHECK(hipEventRecord(e0, st));
            for (int l = 0; l < launches; ++l)
                vs[i].k<<<g, 256, 0, st>>>(X[l % sets], Y[l % sets], Z[l % sets]);
            CHECK(hipEventRecord(e1, st));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1e3 / launches);
        }
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(t[i].begin(), t[i].end());
        const double med = t[i][rounds / 2];
        printf("{\"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n",
               vs[i].name.c_str(), med, t[i][0], 3.0 * bytes / med / 8e6);
    }
    return 0;
}
