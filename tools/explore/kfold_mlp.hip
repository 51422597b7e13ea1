// kfold_mlp.hip — loads in flight per wave x resident blocks per CU for the
// k-input fold. The probe kernel of kfold_occ.hip compiled to "1 load, wait,
// 3 loads, wait" per input while the product issues all 4 loads of an input
// before its adds, and the probe gained more from the occupancy cap
// (kfold_prod_vs_probe). Here the schedule is pinned with sched_barrier:
//   L4  x_j's 4 loads, then 4 adds (the product's order)
//   L13 1 load, add, 3 loads, adds (the probe's compiled order)
//   L22 2 loads, wait, 2 loads
//   L1  load, add, load, add ... (one load in flight past x0/x1)
// (the waits are inline `s_waitcnt vmcnt(0)` with a memory clobber, which keeps
// the later loads behind them)
// each at 0 / 32 / 48 / 64 KiB of dynamic LDS (8 / 5 / 3 / 2 blocks per CU),
// k = 4 and 8, same buffers, rounds interleaved.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o kfold_mlp kfold_mlp.hip
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

// a 16-B non-temporal load the compiler can neither move nor wait for: the
// schedule below is exactly the program order of these statements and of the
// explicit waits (which also redefine the loaded registers, so no use can be
// scheduled before its wait)
__device__ __forceinline__ f32x4 ld_asm(const f32x4 *p)
{
    f32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p));
    return v;
}
#define WAIT2(x, y) asm volatile("s_waitcnt vmcnt(0)" : "+v"(x), "+v"(y))
#define WAIT1(x) asm volatile("s_waitcnt vmcnt(0)" : "+v"(x))

// asm-pinned schedules past x0/x1: 4: pairs (2 in flight), 5: 1 then 3,
// 6: one at a time, 7: all 4
template <int MODE>
__global__ void __launch_bounds__(256) fold_asm(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * 1024 + threadIdx.x;
    if (v0 + 768 >= nvec) return;
    f32x4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = ld(in.p[0] + v0 + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = ld(in.p[1] + v0 + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += b[u];
    for (int j = 2; j < k; ++j) {
        const f32x4 *pj = in.p[j] + v0;
        if (MODE == 4) {
            b[0] = ld_asm(pj);
            b[1] = ld_asm(pj + 256);
            WAIT2(b[0], b[1]);
            a[0] += b[0];
            a[1] += b[1];
            b[2] = ld_asm(pj + 512);
            b[3] = ld_asm(pj + 768);
            WAIT2(b[2], b[3]);
            a[2] += b[2];
            a[3] += b[3];
        } else if (MODE == 5) {
            b[0] = ld_asm(pj);
            WAIT1(b[0]);
            a[0] += b[0];
            b[1] = ld_asm(pj + 256);
            b[2] = ld_asm(pj + 512);
            b[3] = ld_asm(pj + 768);
            WAIT2(b[1], b[2]);
            WAIT1(b[3]);
            a[1] += b[1];
            a[2] += b[2];
            a[3] += b[3];
        } else if (MODE == 6) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                b[u] = ld_asm(pj + u * 256);
                WAIT1(b[u]);
                a[u] += b[u];
            }
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) b[u] = ld_asm(pj + u * 256);
            WAIT2(b[0], b[1]);
            WAIT2(b[2], b[3]);
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] += b[u];
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(a[u], out + v0 + u * 256);
}

// k = 2 (the C2 sum) with pinned schedules: 8 = all 8 vectors of x and y in
// flight (the product), 4 = (x,y) of two tiles then wait, twice, 2 = one
// (x,y) pair at a time
template <int INFL>
__global__ void __launch_bounds__(256) sum2_asm(Ptrs in, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * 1024 + threadIdx.x;
    if (v0 + 768 >= nvec) return;
    const f32x4 *x = in.p[0] + v0, *y = in.p[1] + v0;
    f32x4 a[4], b[4];
    if (INFL == 8) {
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] = ld(x + u * 256);
#pragma unroll
        for (int u = 0; u < 4; ++u) b[u] = ld(y + u * 256);
    } else if (INFL == 4) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            a[2 * h] = ld_asm(x + 2 * h * 256);
            b[2 * h] = ld_asm(y + 2 * h * 256);
            a[2 * h + 1] = ld_asm(x + (2 * h + 1) * 256);
            b[2 * h + 1] = ld_asm(y + (2 * h + 1) * 256);
            WAIT2(a[2 * h], b[2 * h]);
            WAIT2(a[2 * h + 1], b[2 * h + 1]);
        }
    } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a[u] = ld_asm(x + u * 256);
            b[u] = ld_asm(y + u * 256);
            WAIT2(a[u], b[u]);
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(a[u] + b[u], out + v0 + u * 256);
}

template <int MODE>  // 0: L4, 1: L13, 2: L22, 3: L1
__global__ void __launch_bounds__(256) fold(Ptrs in, int k, f32x4 *out, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * 1024 + threadIdx.x;
    if (v0 + 768 >= nvec) return;
    f32x4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] = ld(in.p[0] + v0 + u * 256);
#pragma unroll
    for (int u = 0; u < 4; ++u) b[u] = ld(in.p[1] + v0 + u * 256);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += b[u];
    for (int j = 2; j < k; ++j) {
        const f32x4 *pj = in.p[j] + v0;
        if (MODE == 0) {
#pragma unroll
            for (int u = 0; u < 4; ++u) b[u] = ld(pj + u * 256);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] += b[u];
        } else if (MODE == 1) {  // 1 load, wait, 3 loads
            b[0] = ld(pj);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            a[0] += b[0];
#pragma unroll
            for (int u = 1; u < 4; ++u) b[u] = ld(pj + u * 256);
#pragma unroll
            for (int u = 1; u < 4; ++u) a[u] += b[u];
        } else if (MODE == 2) {  // 2 loads, wait, 2 loads
            b[0] = ld(pj);
            b[1] = ld(pj + 256);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            a[0] += b[0];
            a[1] += b[1];
            b[2] = ld(pj + 512);
            b[3] = ld(pj + 768);
            a[2] += b[2];
            a[3] += b[3];
        } else {  // one load in flight
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                b[u] = ld(pj + u * 256);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                a[u] += b[u];
            }
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(a[u], out + v0 + u * 256);
}


struct Variant {
    std::string name;
    int k;
    std::function<void(const Ptrs &, f32x4 *, size_t, hipStream_t)> run;
};

template <int MODE>
Variant make(int k, int lds)
{
    static const char *nm[] = {"L4", "L13", "L22", "L1"};
    return {std::string(nm[MODE]) + "_lds" + std::to_string(lds >> 10) + "K", k,
            [k, lds](const Ptrs &p, f32x4 *o, size_t nvec, hipStream_t s) {
                fold<MODE><<<static_cast<unsigned>(nvec / 1024), 256, lds, s>>>(p, k, o, nvec);
            }};
}

template <int MODE>
Variant make_asm(int k, int lds)
{
    static const char *nm[] = {"A22", "A13", "A1", "A4"};
    return {std::string(nm[MODE - 4]) + "_lds" + std::to_string(lds >> 10) + "K", k,
            [k, lds](const Ptrs &p, f32x4 *o, size_t nvec, hipStream_t s) {
                fold_asm<MODE><<<static_cast<unsigned>(nvec / 1024), 256, lds, s>>>(p, k, o, nvec);
            }};
}

template <int INFL>
Variant make_sum2(int lds)
{
    return {"S" + std::to_string(INFL) + "_lds" + std::to_string(lds >> 10) + "K", 2,
            [lds](const Ptrs &p, f32x4 *o, size_t nvec, hipStream_t s) {
                sum2_asm<INFL><<<static_cast<unsigned>(nvec / 1024), 256, lds, s>>>(p, o, nvec);
            }};
}

int main(int argc, char **argv)
{
    // argv[2]: elements per input (default 64 Mi = 256 MiB)
    const size_t n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : (64ull << 20);
    const size_t bytes = n * 4, nvec = n / 4;
    const int kmax = 8, sets = 3, launches = 50, rounds = 5;
    std::vector<Variant> vs;
    if (argc > 1 && argv[1][0] == 's') {  // small sizes: A4 vs A1, uncapped
        for (int k : {3, 4, 8}) {
            vs.push_back(make_asm<7>(k, 0));
            vs.push_back(make_asm<6>(k, 0));
            vs.push_back(make_asm<4>(k, 0));
        }
    } else if (argc > 1 && argv[1][0] == 'm') {  // mid sizes: A4 uncapped vs A1 capped
        for (int k : {3, 4, 8}) {
            vs.push_back(make_asm<7>(k, 0));
            vs.push_back(make_asm<6>(k, 0));
            vs.push_back(make_asm<6>(k, 32 << 10));
        }
    } else if (argc > 1 && argv[1][0] == '2') {  // k = 2 schedules
        for (int lds : {0, 20 << 10, 24 << 10, 32 << 10, 40 << 10}) {
            vs.push_back(make_sum2<8>(lds));
            vs.push_back(make_sum2<4>(lds));
            vs.push_back(make_sum2<2>(lds));
        }
    } else if (argc > 1) {  // the asm-pinned schedules
        for (int k : {3, 4, 6, 8})
            for (int lds : {0, 24 << 10, 32 << 10, 40 << 10, 48 << 10}) {
                vs.push_back(make_asm<4>(k, lds));
                vs.push_back(make_asm<5>(k, lds));
                vs.push_back(make_asm<6>(k, lds));
                vs.push_back(make_asm<7>(k, lds));
            }
    } else {
        for (int k : {4, 8})
            for (int lds : {0, 32 << 10, 48 << 10, 64 << 10}) {
                vs.push_back(make<0>(k, lds));
                vs.push_back(make<1>(k, lds));
                vs.push_back(make<2>(k, lds));
                vs.push_back(make<3>(k, lds));
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
    std::vector<std::vector<double>> t(vs.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            vs[i].run(ptrs(0), out[0], nvec, s);
            CHECK(hipEventRecord(e0, s));
            for (int l = 0; l < launches; ++l) vs[i].run(ptrs(l % sets), out[l % sets], nvec, s);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms * 1e3 / launches);
        }
        fprintf(stderr, "round %d\n", r);
    }
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(t[i].begin(), t[i].end());
        const double med = t[i][rounds / 2], algo = (vs[i].k + 1.0) * bytes;
        printf("{\"variant\": \"%s\", \"k\": %d, \"median_us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n",
               vs[i].name.c_str(), vs[i].k, med, t[i][0], algo / med / 8e6);
    }
    return 0;
}
