// fold_probe.hip — C5's rank-order fold at N = 8 (bench.py kernels
// `c5_a2a_fold_n8_bf16`: 13 BERT-base buckets, each a workspace of the 8
// received bf16 shards back to back, folded in rank order with fp32
// accumulation, /8 fused, one RNE narrow) runs at 0.72-0.73 of 8 TB/s with
// 1.0005x algorithmic PMC traffic (profiles/r06/pmc_c5_r06a.jsonl). What is
// the rest?
//
//   shipped     kf_bucket_reduce_batch (runtime-k batch kernel, 4 vectors per
//               lane, all of an input's vectors in flight at this size)
//   k8_u{1,2,4} a compile-time k = 8 fold, every input's U vectors issued before
//               the first add, scalar fp32 adds (the shipped arithmetic)
//   k8pk_u{2,4} the same with the adds on pairs of lanes in packed fp32
//               (v_pk_add_f32 / v_pk_mul_f32: per lane the same IEEE ops)
//   copy9       the same 9 streams with no arithmetic (8 reads xor-ed, one
//               write): the traffic ceiling of this launch shape
//
// Bits of every fold variant are checked against the shipped kernel.
// Launches cycle over enough sets (>= 0.75 GiB) for a cold Infinity Cache;
// median of 7 x 20.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//       -I kungfu_amd/csrc -o tools/explore/fold_probe tools/explore/fold_probe.hip \
//       -L kungfu_amd -lkungfu_amd -Wl,-rpath,$PWD/kungfu_amd
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "kf_reduce_kernels.hpp"
#include "kungfu_amd.h"

#pragma clang fp contract(off)

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

using namespace kf;
constexpr int BLOCK = 256, K = 8, NB = 13;

struct Args {
    const char *ws[NB];  // 8 shards of q[b] elements back to back
    char *out[NB];
    size_t q[NB];
    unsigned blk0[NB + 1];
};

__device__ __forceinline__ int seg(const Args &a, unsigned b)
{
    int s = 0;
    while (s + 1 < NB && b >= a.blk0[s + 1]) ++s;
    return s;
}

template <int U, bool PK, bool COPY>
__global__ void __launch_bounds__(BLOCK) fold8(Args a)
{
    const int s       = seg(a, blockIdx.x);
    const size_t nvec = a.q[s] / 8;  // 8 bf16 per 16-B vector (q % 8 == 0 here)
    const size_t v0   = static_cast<size_t>(blockIdx.x - a.blk0[s]) * (BLOCK * U) + threadIdx.x;
    const size_t sb   = a.q[s] * 2;  // shard bytes
    u32x4 v[K][U];
#pragma unroll
    for (int j = 0; j < K; ++j) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t vi = v0 + u * BLOCK;
            v[j][u] = vi < nvec ? __builtin_nontemporal_load(
                                      reinterpret_cast<const u32x4 *>(a.ws[s] + j * sb) + vi)
                                : u32x4{0, 0, 0, 0};
        }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        if (vi >= nvec) break;
        u32x4 r;
        if constexpr (COPY) {
            r = v[0][u];
#pragma unroll
            for (int j = 1; j < K; ++j) r ^= v[j][u];
        } else {
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                if constexpr (PK) {
                    f32x2 acc = {__uint_as_float(v[0][u][w] << 16), __uint_as_float(v[0][u][w] & 0xffff0000u)};
#pragma unroll
                    for (int j = 1; j < K; ++j) {
                        acc = acc + f32x2{__uint_as_float(v[j][u][w] << 16),
                                          __uint_as_float(v[j][u][w] & 0xffff0000u)};
                    }
                    acc = acc * f32x2{0.125f, 0.125f};
                    r[w] = static_cast<uint32_t>(f32_to_bf16(acc.x)) |
                           (static_cast<uint32_t>(f32_to_bf16(acc.y)) << 16);
                } else {
                    float lo = __uint_as_float(v[0][u][w] << 16), hi = __uint_as_float(v[0][u][w] & 0xffff0000u);
#pragma unroll
                    for (int j = 1; j < K; ++j) {
                        lo = __fadd_rn(lo, __uint_as_float(v[j][u][w] << 16));
                        hi = __fadd_rn(hi, __uint_as_float(v[j][u][w] & 0xffff0000u));
                    }
                    r[w] = static_cast<uint32_t>(f32_to_bf16(__fmul_rn(lo, 0.125f))) |
                           (static_cast<uint32_t>(f32_to_bf16(__fmul_rn(hi, 0.125f))) << 16);
                }
            }
        }
        __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(a.out[s]) + vi);
    }
}

__global__ void fill(uint32_t *p, size_t n, uint32_t seed)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = static_cast<uint32_t>(i) * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        const uint32_t lo = (x & 0x807fu) | ((124u + (x >> 8) % 6u) << 7);
        const uint32_t hi = ((x >> 16) & 0x807fu) | ((124u + (x >> 24) % 6u) << 7);
        p[i] = lo | (hi << 16);
    }
}

int main()
{
    const size_t q[NB] = {2930176, 1009408, 1033728, 960000, 886016, 886016, 886016,
                          886016,  886016,  886016,  886016, 886016, 664576};
    size_t per_set = 0;
    for (size_t x : q) per_set += (K + 1) * x * 2;
    const int NS = static_cast<int>(std::max<size_t>(2, ((768ull << 20) + per_set - 1) / per_set));
    struct Set {
        std::vector<void *> ws, out;
    };
    std::vector<Set> sets(NS);
    for (auto &st : sets) {
        for (int b = 0; b < NB; ++b) {
            void *w, *o;
            CHECK(hipMalloc(&w, K * q[b] * 2));
            CHECK(hipMalloc(&o, q[b] * 2));
            fill<<<2048, 256>>>(static_cast<uint32_t *>(w), K * q[b] / 2, 7u * b + 1000u * (&st - sets.data()));
            st.ws.push_back(w);
            st.out.push_back(o);
        }
    }
    CHECK(hipDeviceSynchronize());
    hipStream_t s = nullptr;
    auto args = [&](int i, int U) {
        Args a{};
        unsigned blocks = 0;
        for (int b = 0; b < NB; ++b) {
            a.ws[b]   = static_cast<const char *>(sets[i].ws[b]);
            a.out[b]  = static_cast<char *>(sets[i].out[b]);
            a.q[b]    = q[b];
            a.blk0[b] = blocks;
            blocks += static_cast<unsigned>((q[b] / 8 + BLOCK * U - 1) / (BLOCK * U));
        }
        a.blk0[NB] = blocks;
        return a;
    };
    // the shipped launch's pointer tables
    std::vector<std::vector<const void *>> ins(NS);
    std::vector<std::vector<void *>> outs(NS);
    for (int i = 0; i < NS; ++i) {
        for (int b = 0; b < NB; ++b) {
            for (int j = 0; j < K; ++j) ins[i].push_back(static_cast<const char *>(sets[i].ws[b]) + j * q[b] * 2);
            outs[i].push_back(sets[i].out[b]);
        }
    }
    auto shipped = [&](int i) {
        int rc = kf_bucket_reduce_batch(ins[i].data(), K, outs[i].data(), q, NB, KungFu_BFLOAT16, KungFu_SUM, K, s);
        if (rc) {
            fprintf(stderr, "kf_bucket_reduce_batch: %s\n", kf_last_error());
            exit(2);
        }
    };
    struct Var {
        std::string name;
        std::function<void(int)> run;
        bool fold;
    };
    std::vector<Var> vars = {
        {"shipped", shipped, true},
        {"k8_u1", [&](int i) { Args a = args(i, 1); fold8<1, false, false><<<a.blk0[NB], BLOCK>>>(a); }, true},
        {"k8_u2", [&](int i) { Args a = args(i, 2); fold8<2, false, false><<<a.blk0[NB], BLOCK>>>(a); }, true},
        {"k8_u4", [&](int i) { Args a = args(i, 4); fold8<4, false, false><<<a.blk0[NB], BLOCK>>>(a); }, true},
        {"k8pk_u2", [&](int i) { Args a = args(i, 2); fold8<2, true, false><<<a.blk0[NB], BLOCK>>>(a); }, true},
        {"k8pk_u4", [&](int i) { Args a = args(i, 4); fold8<4, true, false><<<a.blk0[NB], BLOCK>>>(a); }, true},
        {"copy9_u2", [&](int i) { Args a = args(i, 2); fold8<2, false, true><<<a.blk0[NB], BLOCK>>>(a); }, false},
        {"copy9_u4", [&](int i) { Args a = args(i, 4); fold8<4, false, true><<<a.blk0[NB], BLOCK>>>(a); }, false},
    };
    // bits: every fold variant against the shipped kernel on set 0
    std::vector<std::vector<uint16_t>> want(NB);
    shipped(0);
    CHECK(hipDeviceSynchronize());
    for (int b = 0; b < NB; ++b) {
        want[b].resize(q[b]);
        CHECK(hipMemcpy(want[b].data(), sets[0].out[b], q[b] * 2, hipMemcpyDeviceToHost));
    }
    for (auto &v : vars) {
        if (!v.fold || v.name == "shipped") continue;
        for (int b = 0; b < NB; ++b) CHECK(hipMemset(sets[0].out[b], 0xff, q[b] * 2));
        v.run(0);
        CHECK(hipDeviceSynchronize());
        size_t bad = 0;
        for (int b = 0; b < NB; ++b) {
            std::vector<uint16_t> got(q[b]);
            CHECK(hipMemcpy(got.data(), sets[0].out[b], q[b] * 2, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < q[b]; ++i) bad += got[i] != want[b][i];
        }
        printf("{\"check\": \"%s\", \"mismatches\": %zu}\n", v.name.c_str(), bad);
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ts(vars.size());
    for (int round = 0; round < 7; ++round) {
        for (size_t v = 0; v < vars.size(); ++v) {
            for (int i = 0; i < NS; ++i) vars[v].run(i);
            CHECK(hipEventRecord(e0, s));
            for (int i = 0; i < 20; ++i) vars[v].run(i % NS);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ts[v].push_back(ms * 1e3f / 20);
        }
    }
    CHECK(hipGetLastError());
    for (size_t v = 0; v < vars.size(); ++v) {
        std::sort(ts[v].begin(), ts[v].end());
        const double us = ts[v][ts[v].size() / 2];
        printf("{\"variant\": \"%s\", \"us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f, \"sets\": %d}\n",
               vars[v].name.c_str(), us, ts[v][0], per_set / us / 8e6, NS);
    }
    return 0;
}
