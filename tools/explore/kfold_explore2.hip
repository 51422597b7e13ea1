// kfold_explore2.hip — register-path variants of the k-input fold (block size,
// unroll, cache policy, per-block spans, pairwise loads); DESIGN.md §10 item 2
//
// The shipped runtime-k fold sits at 5.9-6.1 TB/s for k = 4..8 (0.74-0.76 of
// 8 TB/s), which is the guide's in-order register read sweep (6.0-6.1 TB/s);
// the guide's LDS-DMA weight stream reads at 6.5-6.8 TB/s with nt. Here each
// one-wave workgroup streams its tiles through a wave-private LDS ring of S
// stages: global_load_lds_dwordx4 (16 B per lane, nt) of the k inputs of tile
// i+S-1, a counted `s_waitcnt vmcnt` that retires tile i (this wave's own
// DMAs, so no barrier), ds_read_b128 of the k vectors, the left fold in input
// order (bit-identical to the product), a non-temporal 16-B store.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kfold_explore2 kfold_explore2.hip
//   ./kfold_explore2 > results.jsonl
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

struct Ptrs {
    const f32x4 *p[16];
};

__device__ __forceinline__ f32x4 ld(const f32x4 *p) { return __builtin_nontemporal_load(p); }

// The shipped shape: BLOCK x U, inputs 0 and 1 up front, then one at a time.
// LNT / SNT: non-temporal loads / stores. SPAN: each block walks SPAN
// consecutive tiles (DRAM row locality per block) instead of one tile.
template <int BLOCK, int U, int LNT, int SNT, int SPAN>
__global__ void __launch_bounds__(BLOCK) fold_reg(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    auto L = [](const f32x4 *p) { return LNT ? __builtin_nontemporal_load(p) : *p; };
    for (int sp = 0; sp < SPAN; ++sp) {
        const size_t tile = static_cast<size_t>(blockIdx.x) * SPAN + sp;
        const size_t v0   = tile * (BLOCK * U) + threadIdx.x;
        if (v0 + (U - 1) * BLOCK >= nvec) return;
        f32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = L(in.p[0] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = L(in.p[1] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] += b[u];
        for (int j = 2; j < k; ++j) {
#pragma unroll
            for (int u = 0; u < U; ++u) b[u] = L(in.p[j] + v0 + u * BLOCK);
#pragma unroll
            for (int u = 0; u < U; ++u) a[u] += b[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (SNT) __builtin_nontemporal_store(a[u], out + v0 + u * BLOCK);
            else out[v0 + u * BLOCK] = a[u];
        }
    }
}

// two-level: inputs folded in pairs with both loads of a pair in flight
// ((x0+x1)+x2)+x3... order kept: acc += x_j one at a time, but the loads of
// x_j and x_{j+1} are issued together
template <int BLOCK, int U>
__global__ void __launch_bounds__(BLOCK) fold_pairs(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
    f32x4 a[U], b[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(in.p[0] + v0 + u * BLOCK);
    int j = 1;
    for (; j + 1 < k; j += 2) {
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(in.p[j] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) c[u] = __builtin_nontemporal_load(in.p[j + 1] + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = (a[u] + b[u]) + c[u];
    }
    for (; j < k; ++j) {
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
    std::function<void(const Ptrs &, f32x4 *, size_t, hipStream_t)> run;
};

template <int BLOCK, int U, int LNT, int SNT, int SPAN>
Variant make_reg(int k)
{
    return {"reg_" + std::to_string(BLOCK) + "x" + std::to_string(U) + "_l" + std::to_string(LNT) +
                "s" + std::to_string(SNT) + "_span" + std::to_string(SPAN),
            k, [k](const Ptrs &p, f32x4 *o, size_t nvec, hipStream_t s) {
                const unsigned g = static_cast<unsigned>(nvec / (BLOCK * U) / SPAN);
                fold_reg<BLOCK, U, LNT, SNT, SPAN><<<g, BLOCK, 0, s>>>(p, k, o, nvec);
            }};
}

template <int BLOCK, int U>
Variant make_pairs(int k)
{
    return {"pairs_" + std::to_string(BLOCK) + "x" + std::to_string(U), k,
            [k](const Ptrs &p, f32x4 *o, size_t nvec, hipStream_t s) {
                const unsigned g = static_cast<unsigned>(nvec / (BLOCK * U));
                fold_pairs<BLOCK, U><<<g, BLOCK, 0, s>>>(p, k, o, nvec);
            }};
}

template <int K>
void add_k(std::vector<Variant> &vs)
{
    vs.push_back(make_reg<256, 4, 1, 1, 1>(K));  // shipped
    vs.push_back(make_reg<256, 2, 1, 1, 1>(K));
    vs.push_back(make_reg<512, 4, 1, 1, 1>(K));
    vs.push_back(make_reg<256, 8, 1, 1, 1>(K));
    vs.push_back(make_reg<256, 4, 0, 1, 1>(K));
    vs.push_back(make_reg<256, 4, 1, 0, 1>(K));
    vs.push_back(make_reg<256, 4, 1, 1, 4>(K));
    vs.push_back(make_reg<256, 4, 1, 1, 16>(K));
    vs.push_back(make_pairs<256, 4>(K));
    vs.push_back(make_pairs<256, 2>(K));
}

int main()
{
    const size_t n     = 64ull << 20;  // fp32 per input
    const size_t bytes = n * 4;
    const size_t nvec  = n / 4;
    const int kmax = 8, sets = 2, launches = 20, rounds = 5;
    std::vector<Variant> vs;
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
    {  // correctness: every element against the in-order fold on the host
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
                    fprintf(stderr, "variant %s k=%d wrong at %zu: %g vs %g\n", v.name.c_str(),
                            v.k, i, hz[i], a);
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
        const double med  = t[i][rounds / 2];
        const double algo = (vs[i].k + 1.0) * bytes;
        printf("{\"variant\": \"%s\", \"k\": %d, \"median_us\": %.2f, \"min_us\": %.2f, "
               "\"GBps\": %.1f, \"frac\": %.4f}\n",
               vs[i].name.c_str(), vs[i].k, med, t[i][0], algo / med / 1e3, algo / med / 8e6);
    }
    return 0;
}
