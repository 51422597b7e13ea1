// sma_batch_probe.hip — C5's SMA blend step (bench.py kernels
// `sma_batch_c5_bf16`: kf_sma_blend_batch over BERT-base's 13 bf16 buckets
// of 16 MiB-bucket layout, in place, 656,928,768 algorithmic bytes) runs at
// 0.77-0.78 of 8 TB/s with 1.0001x PMC traffic; the packed-fp32 blend changed
// nothing (profiles/r06/ab_sma_pk_r06c.jsonl). What bounds it? (VERDICT r05
// item 2.) Same buckets, same block table, interleaved rounds:
//
//   shipped      kf_sma_blend_batch (the C ABI)
//   xor_u4       the same launch shape with no arithmetic: v ^= s in place
//                (4 vectors per lane, all loads first, store per vector):
//                the traffic ceiling of this launch
//   xor_u4_late  the same, every store after the last xor (stores grouped)
//   sma_u4_late  the shipped blend with its stores grouped after all math
//   oop_u4       the shipped blend written to a third buffer (out of place)
//   xor_flat_u4  the xor over the same bytes as ONE flat range: since round
//                6 the shipped launch merges buckets that are contiguous in v
//                and in the sums (as here), so this is its ceiling
//
// Each blend variant's bits are checked against the shipped kernel's.
// 3 rotating sets, median of 7 x 24 launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//       -I kungfu_amd/csrc -o tools/explore/sma_batch_probe tools/explore/sma_batch_probe.hip \
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
constexpr int BLOCK = 256, U = 4, NB = 13;

struct Args {
    uint16_t *v[NB];
    const uint16_t *s[NB];
    uint16_t *o[NB];
    size_t nvec[NB];
    unsigned blk0[NB + 1];
};

__device__ __forceinline__ int seg(const Args &a, unsigned b)
{
    int i = 0;
    while (i + 1 < NB && b >= a.blk0[i + 1]) ++i;
    return i;
}

// MODE 0: xor, store per vector; 1: xor, stores grouped; 2: blend, stores
// grouped; 3: blend out of place
template <int MODE>
__global__ void __launch_bounds__(BLOCK) probe(Args a, float c1, float c2, Div np)
{
    const int i     = seg(a, blockIdx.x);
    const size_t v0 = static_cast<size_t>(blockIdx.x - a.blk0[i]) * (BLOCK * U) + threadIdx.x;
    const size_t n  = a.nvec[i];
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        x[u] = vi < n ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a.v[i]) + vi)
                      : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        y[u] = vi < n ? __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(a.s[i]) + vi)
                      : u32x4{0, 0, 0, 0};
    }
    u32x4 *dst = reinterpret_cast<u32x4 *>(MODE == 3 ? a.o[i] : a.v[i]);
    if constexpr (MODE == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t vi = v0 + u * BLOCK;
            if (vi < n) __builtin_nontemporal_store(x[u] ^ y[u], dst + vi);
        }
    } else {
        u32x4 r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (MODE == 1) {
                r[u] = x[u] ^ y[u];
            } else {
                Vec<uint16_t> va, vb;
                __builtin_memcpy(&va, &x[u], 16);
                __builtin_memcpy(&vb, &y[u], 16);
                const Vec<uint16_t> vr = SmaMath<bf16_t>::blend_vec<true>(va, vb, c1, c2, np);
                __builtin_memcpy(&r[u], &vr, 16);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t vi = v0 + u * BLOCK;
            if (vi < n) __builtin_nontemporal_store(r[u], dst + vi);
        }
    }
}

// the same bytes as ONE flat range (what the shipped launch does since
// round 6 when the buckets and the sums are both contiguous): the ceiling of
// the merged launch
__global__ void __launch_bounds__(BLOCK) xor_flat(u32x4 *v, const u32x4 *s, size_t nvec)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        x[u] = vi < nvec ? __builtin_nontemporal_load(v + vi) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        y[u] = vi < nvec ? __builtin_nontemporal_load(s + vi) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        if (vi < nvec) __builtin_nontemporal_store(x[u] ^ y[u], v + vi);
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
    // C5's buckets (GradBuckets(bert[:201], bf16, world 8, bucket_bytes 16 MiB))
    const size_t cnt[NB] = {23441408, 8075264, 8269824, 7680000, 7088128, 7088128, 7088128,
                            7088128,  7088128, 7088128, 7088128, 7088128, 5316608};
    size_t total = 0;
    for (size_t c : cnt) total += c;
    const int NS = 3;
    // one flat allocation per set for v (as GradBuckets), sums separate
    std::vector<uint16_t *> V(NS), S(NS), O(NS);
    for (int k = 0; k < NS; ++k) {
        CHECK(hipMalloc(&V[k], total * 2));
        CHECK(hipMalloc(&S[k], total * 2));
        CHECK(hipMalloc(&O[k], total * 2));
    }
    auto refill = [&]() {
        for (int k = 0; k < NS; ++k) {
            fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(V[k]), total / 2, 17u + k);
            fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(S[k]), total / 2, 71u + k);
        }
        CHECK(hipDeviceSynchronize());
    };
    refill();
    const Div np{8.f, 0.125f, 8.0, 0.125, 1};
    const float c1 = 0.9f, c2 = 0.1f;
    std::vector<Args> args(NS);
    std::vector<std::vector<void *>> vs(NS), ss(NS);
    for (int k = 0; k < NS; ++k) {
        size_t off = 0;
        unsigned blocks = 0;
        for (int b = 0; b < NB; ++b) {
            args[k].v[b]    = V[k] + off;
            args[k].s[b]    = S[k] + off;
            args[k].o[b]    = O[k] + off;
            args[k].nvec[b] = cnt[b] / 8;
            args[k].blk0[b] = blocks;
            blocks += static_cast<unsigned>((cnt[b] / 8 + BLOCK * U - 1) / (BLOCK * U));
            vs[k].push_back(V[k] + off);
            ss[k].push_back(S[k] + off);
            off += cnt[b];
        }
        args[k].blk0[NB] = blocks;
    }
    const unsigned grid = args[0].blk0[NB];
    auto shipped = [&](int k) {
        int rc = kf_sma_blend_batch(vs[k].data(), const_cast<const void *const *>(ss[k].data()), cnt, NB,
                                    KungFu_BFLOAT16, 8, 0.1, nullptr);
        if (rc) {
            fprintf(stderr, "kf_sma_blend_batch: %s\n", kf_last_error());
            exit(2);
        }
    };
    struct Var {
        std::string name;
        std::function<void(int)> run;
    };
    std::vector<Var> vars = {
        {"shipped", shipped},
        {"xor_u4", [&](int k) { probe<0><<<grid, BLOCK>>>(args[k], c1, c2, np); }},
        {"xor_u4_late", [&](int k) { probe<1><<<grid, BLOCK>>>(args[k], c1, c2, np); }},
        {"sma_u4_late", [&](int k) { probe<2><<<grid, BLOCK>>>(args[k], c1, c2, np); }},
        {"oop_u4", [&](int k) { probe<3><<<grid, BLOCK>>>(args[k], c1, c2, np); }},
        {"xor_flat_u4", [&](int k) {
             const size_t nv = total / 8;
             xor_flat<<<static_cast<unsigned>((nv + BLOCK * U - 1) / (BLOCK * U)), BLOCK>>>(
                 reinterpret_cast<u32x4 *>(V[k]), reinterpret_cast<const u32x4 *>(S[k]), nv);
         }},
    };
    // bits (set 0): the blend variants against the shipped kernel
    {
        std::vector<uint16_t> v0(total), want(total), got(total);
        CHECK(hipMemcpy(v0.data(), V[0], total * 2, hipMemcpyDeviceToHost));
        shipped(0);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(want.data(), V[0], total * 2, hipMemcpyDeviceToHost));
        for (int m : {2, 3}) {
            CHECK(hipMemcpy(V[0], v0.data(), total * 2, hipMemcpyHostToDevice));
            if (m == 2) probe<2><<<grid, BLOCK>>>(args[0], c1, c2, np);
            else probe<3><<<grid, BLOCK>>>(args[0], c1, c2, np);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(got.data(), m == 2 ? V[0] : O[0], total * 2, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < total; ++i) bad += got[i] != want[i];
            printf("{\"check\": \"%s\", \"mismatches\": %zu}\n", m == 2 ? "sma_u4_late" : "oop_u4", bad);
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ts(vars.size());
    for (int round = 0; round < 7; ++round) {
        refill();  // the in-place runs drift the data
        for (size_t v = 0; v < vars.size(); ++v) {
            for (int k = 0; k < NS; ++k) vars[v].run(k);
            CHECK(hipEventRecord(e0));
            for (int i = 0; i < 24; ++i) vars[v].run(i % NS);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ts[v].push_back(ms * 1e3f / 24);
        }
    }
    CHECK(hipGetLastError());
    const double algo = 3.0 * 2 * total;
    for (size_t v = 0; v < vars.size(); ++v) {
        std::sort(ts[v].begin(), ts[v].end());
        const double us = ts[v][ts[v].size() / 2];
        printf("{\"variant\": \"%s\", \"us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f, \"grid\": %u}\n",
               vars[v].name.c_str(), us, ts[v][0], algo / us / 8e6, grid);
    }
    return 0;
}
