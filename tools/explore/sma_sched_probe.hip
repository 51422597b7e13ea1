// sma_sched_probe.hip — the shipped bf16 SMA blend issues its full tile's
// eight 16-B loads as 3, wait, 5: held to 64 VGPRs (8 waves per SIMD), the
// compiler's scheduler starts blending the first vector before it has issued
// the rest, so a wave keeps fewer loads in flight than the xor/add kernels
// (which issue all eight first). On one box (profiles/r06/same_box_probe_r06o)
// the blend ran at 0.792 of 8 TB/s against 0.814 for an in-place xor of the
// same bytes. Variants (same body as kf::sma_body's full tile; the ragged
// tile as shipped):
//
//   shipped     kf_sma_blend (C ABI)
//   local       the full-tile path restated here, waves_per_eu(8, 8)
//   sb          the same with a scheduling barrier between the loads and the
//               blend: all eight loads issued before the first wait
//   sb_free     sb without the waves_per_eu attribute
//   xor         v ^= s, all loads first (the traffic ceiling)
//
// Bits of local/sb/sb_free against the shipped kernel; 256 MiB and C5's
// 218,976,256 B per stream; 3 rotating sets; median of 7 x 24 launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//       -I kungfu_amd/csrc -o tools/explore/sma_sched_probe tools/explore/sma_sched_probe.hip \
//       -L kungfu_amd -lkungfu_amd -Wl,-rpath,'$ORIGIN/../../kungfu_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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
#define KF(x)                                                                   \
    do {                                                                        \
        int rc_ = (x);                                                          \
        if (rc_ != 0) {                                                         \
            fprintf(stderr, "%s: %s\n", #x, kf_last_error());                  \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

using namespace kf;
constexpr int BLOCK = 256, U = 4;

template <bool SB>
__device__ __forceinline__ void body(uint16_t *v, const uint16_t *s, size_t nvec, float c1, float c2,
                                     const Div &np)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK < nvec) {
        Vec<uint16_t> a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = ld_vec<uint16_t, 1>(v, v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = ld_vec<uint16_t, 1>(s, v0 + u * BLOCK);
        if constexpr (SB) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            st_vec<uint16_t>(v, v0 + u * BLOCK, SmaMath<bf16_t>::blend_vec<true>(a[u], b[u], c1, c2, np));
    } else {
        for (int u = 0; u < U; ++u) {
            const size_t vi = v0 + u * BLOCK;
            if (vi >= nvec) break;
            const Vec<uint16_t> a = ld_vec<uint16_t, 1>(v, vi), b = ld_vec<uint16_t, 1>(s, vi);
            st_vec<uint16_t>(v, vi, SmaMath<bf16_t>::blend_vec<true>(a, b, c1, c2, np));
        }
    }
}

template <bool SB>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8)))
    sma_capped(uint16_t *v, const uint16_t *s, size_t nvec, float c1, float c2, Div np)
{
    body<SB>(v, s, nvec, c1, c2, np);
}

__global__ void __launch_bounds__(BLOCK) sma_free(uint16_t *v, const uint16_t *s, size_t nvec, float c1, float c2,
                                                  Div np)
{
    body<true>(v, s, nvec, c1, c2, np);
}

__global__ void __launch_bounds__(BLOCK) xor_inplace(u32x4 *v, const u32x4 *s, size_t n)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK < n) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(v + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(s + v0 + u * BLOCK);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(a[u] ^ b[u], v + v0 + u * BLOCK);
    } else {
        for (int u = 0; u < U; ++u) {
            const size_t vi = v0 + u * BLOCK;
            if (vi >= n) break;
            v[vi] = v[vi] ^ s[vi];
        }
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
    const size_t big = 256u << 20, c5 = 218976256;
    const int NS = 3;
    std::vector<uint16_t *> V(NS), S(NS);
    for (int k = 0; k < NS; ++k) {
        CHECK(hipMalloc(&V[k], big));
        CHECK(hipMalloc(&S[k], big));
        fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(S[k]), big / 4, 71u + k);
    }
    auto refill = [&](uint32_t r) {
        for (int k = 0; k < NS; ++k) fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(V[k]), big / 4, 17u + k + r);
        CHECK(hipDeviceSynchronize());
    };
    refill(0);
    const float c1 = static_cast<float>(1.0 - 0.1), c2 = static_cast<float>(0.1);
    const Div np{8.f, 0.125f, 8.0, 0.125, 1};
    struct Var {
        std::string name;
        std::function<void(int, size_t)> run;  // (set, bytes per stream)
    };
    std::vector<Var> vars = {
        {"shipped", [&](int k, size_t b) { KF(kf_sma_blend(V[k], S[k], b / 2, KungFu_BFLOAT16, 8, 0.1, nullptr)); }},
        {"local", [&](int k, size_t b) {
             const size_t n = b / 16;
             sma_capped<false><<<static_cast<unsigned>((n + BLOCK * U - 1) / (BLOCK * U)), BLOCK>>>(V[k], S[k], n, c1,
                                                                                                     c2, np);
         }},
        {"sb", [&](int k, size_t b) {
             const size_t n = b / 16;
             sma_capped<true><<<static_cast<unsigned>((n + BLOCK * U - 1) / (BLOCK * U)), BLOCK>>>(V[k], S[k], n, c1,
                                                                                                    c2, np);
         }},
        {"sb_free", [&](int k, size_t b) {
             const size_t n = b / 16;
             sma_free<<<static_cast<unsigned>((n + BLOCK * U - 1) / (BLOCK * U)), BLOCK>>>(V[k], S[k], n, c1, c2, np);
         }},
        {"xor", [&](int k, size_t b) {
             const size_t n = b / 16;
             xor_inplace<<<static_cast<unsigned>((n + BLOCK * U - 1) / (BLOCK * U)), BLOCK>>>(
                 reinterpret_cast<u32x4 *>(V[k]), reinterpret_cast<const u32x4 *>(S[k]), n);
         }},
    };
    // bits: every blend variant against the shipped kernel, at C5's size
    {
        const size_t n = c5 / 2;
        std::vector<uint16_t> v0(n), want(n), got(n);
        CHECK(hipMemcpy(v0.data(), V[0], n * 2, hipMemcpyDeviceToHost));
        vars[0].run(0, c5);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(want.data(), V[0], n * 2, hipMemcpyDeviceToHost));
        for (int m = 1; m <= 3; ++m) {
            CHECK(hipMemcpy(V[0], v0.data(), n * 2, hipMemcpyHostToDevice));
            vars[m].run(0, c5);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(got.data(), V[0], n * 2, hipMemcpyDeviceToHost));
            size_t bad = 0;
            for (size_t i = 0; i < n; ++i) bad += got[i] != want[i];
            printf("{\"check\": \"%s\", \"mismatches\": %zu}\n", vars[m].name.c_str(), bad);
        }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (size_t bytes : {big, c5}) {
        std::vector<std::vector<float>> ts(vars.size());
        for (int round = 0; round < 7; ++round) {
            refill(round + 1);
            for (size_t v = 0; v < vars.size(); ++v) {
                for (int k = 0; k < NS; ++k) vars[v].run(k, bytes);
                CHECK(hipEventRecord(e0));
                for (int i = 0; i < 24; ++i) vars[v].run(i % NS, bytes);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                ts[v].push_back(ms * 1e3f / 24);
            }
        }
        CHECK(hipGetLastError());
        for (size_t v = 0; v < vars.size(); ++v) {
            std::sort(ts[v].begin(), ts[v].end());
            const double us = ts[v][ts[v].size() / 2];
            printf("{\"bytes_per_stream\": %zu, \"variant\": \"%s\", \"us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n",
                   bytes, vars[v].name.c_str(), us, ts[v][0], 3.0 * bytes / us / 8e6);
        }
    }
    return 0;
}
