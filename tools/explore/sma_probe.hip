// sma_probe.hip — why does C5's SMA blend (v = (1-a) v + a (s / np), bf16, in
// place) run at 0.76-0.78 of 8 TB/s when C2's z = x + y (fp32, out of place)
// runs at 0.83? (VERDICT r05 "next" item 2.) Same three streams per element in
// both; the candidates are the in-place write, the bf16 conversion VALU and the
// tile shape. Every variant streams 256 MiB per stream over 3 rotating sets,
// timed with HIP events (median of 7 x 20 launches), interleaved by round.
//
//   c2_f32            the shipped reduce_kernel<float, SUM, NONE, 2> (C2)
//   c2_f32_inplace    the same kernel with z = x (written over an input)
//   add_bf16          shipped reduce_kernel<bf16, SUM, NONE, 2>, out of place
//   add_bf16_inplace  the same, z = x
//   sma_f32           shipped sma_kernel<float> (in place)
//   sma_bf16_u{2,4,8} shipped sma_kernel<bf16> at UNROLL 2 / 4 (shipped) / 8
//   sma_bf16_oop      the shipped blend arithmetic, written to a third buffer
//   xor_bf16_inplace  v ^= s: the in-place traffic with no arithmetic
//   sma_bf16_pk       the blend in packed-fp32 arithmetic (v_pk_mul_f32 /
//                     v_pk_add_f32 on pairs), same IEEE ops, same bits
//
// Each variant's output is checked against the shipped kernel's bits.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//       -I kungfu_amd/csrc -o tools/explore/sma_probe tools/explore/sma_probe.hip
//   tools/explore/sma_probe > profiles/r06/sma_probe.jsonl
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <numeric>
#include <string>
#include <vector>

#include "kf_reduce_kernels.hpp"

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
constexpr int BLOCK = 256;

// the shipped blend arithmetic, out of place
template <int U>
__global__ void __launch_bounds__(BLOCK) sma_oop(const void *v, const void *s, void *out, size_t nvec,
                                                 float c1, float c2, Div np)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
    Vec<uint16_t> a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = ld_vec<uint16_t, 1>(v, v0 + u * BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = ld_vec<uint16_t, 1>(s, v0 + u * BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        Vec<uint16_t> r;
#pragma unroll
        for (int e = 0; e < 8; ++e) r.e[e] = SmaMath<bf16_t>::blend<true>(a[u].e[e], b[u].e[e], c1, c2, np);
        st_vec<uint16_t>(out, v0 + u * BLOCK, r);
    }
}

__global__ void __launch_bounds__(BLOCK) xor_inplace(void *v, const void *s, size_t nvec)
{
    constexpr int U = 4;
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
    u32x4 a[U], b[U];
    const u32x4 *pv = reinterpret_cast<const u32x4 *>(v);
    const u32x4 *ps = reinterpret_cast<const u32x4 *>(s);
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(pv + v0 + u * BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(ps + v0 + u * BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u)
        __builtin_nontemporal_store(a[u] ^ b[u], reinterpret_cast<u32x4 *>(v) + v0 + u * BLOCK);
}

// the blend on pairs of lanes in packed fp32 (gfx950 v_pk_mul_f32 /
// v_pk_add_f32: two IEEE fp32 ops per instruction, each correctly rounded, no
// contraction), then one v_cvt_pk_bf16_f32 per pair
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t blend_pair(uint32_t vv, uint32_t ss, f32x2 c1, f32x2 c2, f32x2 inv)
{
    const f32x2 v = {__uint_as_float(vv << 16), __uint_as_float(vv & 0xffff0000u)};
    const f32x2 s = {__uint_as_float(ss << 16), __uint_as_float(ss & 0xffff0000u)};
    const f32x2 avg = s * inv;
    const f32x2 r   = c1 * v + c2 * avg;  // contract(off): mul, mul, add
    const uint16_t lo = f32_to_bf16(r.x), hi = f32_to_bf16(r.y);
    return static_cast<uint32_t>(lo) | (static_cast<uint32_t>(hi) << 16);
}

__global__ void __launch_bounds__(BLOCK) sma_pk(void *v, const void *s, size_t nvec, float c1,
                                                float c2, Div np)
{
    constexpr int U = 4;
    const size_t v0 = static_cast<size_t>(blockIdx.x) * (BLOCK * U) + threadIdx.x;
    if (v0 + (U - 1) * BLOCK >= nvec) return;
    u32x4 a[U], b[U];
    const u32x4 *pv = reinterpret_cast<const u32x4 *>(v);
    const u32x4 *ps = reinterpret_cast<const u32x4 *>(s);
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = __builtin_nontemporal_load(pv + v0 + u * BLOCK);
#pragma unroll
    for (int u = 0; u < U; ++u) b[u] = __builtin_nontemporal_load(ps + v0 + u * BLOCK);
    const f32x2 C1 = {c1, c1}, C2 = {c2, c2}, I = {np.fi, np.fi};
#pragma unroll
    for (int u = 0; u < U; ++u) {
        u32x4 r;
        r.x = blend_pair(a[u].x, b[u].x, C1, C2, I);
        r.y = blend_pair(a[u].y, b[u].y, C1, C2, I);
        r.z = blend_pair(a[u].z, b[u].z, C1, C2, I);
        r.w = blend_pair(a[u].w, b[u].w, C1, C2, I);
        __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(v) + v0 + u * BLOCK);
    }
}

__global__ void fill(uint32_t *p, size_t n, uint32_t seed, int bf)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = static_cast<uint32_t>(i) * 2654435761u ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        if (bf) {  // two bf16 in [-2, 2): sign, exponent 126..128, random mantissa
            const uint32_t lo = (x & 0x807fu) | ((126u + (x >> 8) % 3u) << 7);
            const uint32_t hi = ((x >> 16) & 0x807fu) | ((126u + (x >> 24) % 3u) << 7);
            p[i] = lo | (hi << 16);
        } else {
            p[i] = (x & 0x807fffffu) | ((126u + (x >> 23) % 3u) << 23);
        }
    }
}

int main()
{
    const size_t bytes = 256ull << 20, nvec = bytes / 16, nw = bytes / 4;
    const int NS = 3;
    std::vector<void *> X(NS), Y(NS), Z(NS);
    for (int i = 0; i < NS; ++i) {
        CHECK(hipMalloc(&X[i], bytes));
        CHECK(hipMalloc(&Y[i], bytes));
        CHECK(hipMalloc(&Z[i], bytes));
    }
    auto refill = [&](int bf) {
        for (int i = 0; i < NS; ++i) {
            fill<<<4096, 256>>>(static_cast<uint32_t *>(X[i]), nw, 11u + i, bf);
            fill<<<4096, 256>>>(static_cast<uint32_t *>(Y[i]), nw, 101u + i, bf);
        }
        CHECK(hipDeviceSynchronize());
    };
    const Div np = {8.0f, 0.125f, 8.0, 0.125, 1};
    const float c1 = 0.9f, c2 = 0.1f;
    const unsigned g4 = static_cast<unsigned>(nvec / (BLOCK * 4));
    const size_t nbf = bytes / 2, nf = bytes / 4;

    struct Var {
        std::string name;
        int bf;  // data kind
        std::function<void(int)> run;
    };
    auto in2 = [&](int i) {
        InPtrs p{};
        p.p[0] = X[i];
        p.p[1] = Y[i];
        return p;
    };
    std::vector<Var> vars = {
        {"c2_f32", 0, [&](int i) {
             reduce_kernel<float, OP_SUM, EPI_NONE, 2, BLOCK, 4, 1, 0><<<g4, BLOCK>>>(in2(i), 2, Z[i], nf, 0, nvec, np, 0);
         }},
        {"c2_f32_inplace", 0, [&](int i) {
             reduce_kernel<float, OP_SUM, EPI_NONE, 2, BLOCK, 4, 1, 0><<<g4, BLOCK>>>(in2(i), 2, X[i], nf, 0, nvec, np, 0);
         }},
        {"sma_f32", 0, [&](int i) {
             sma_kernel<float, float, BLOCK, 4><<<g4, BLOCK>>>(X[i], Y[i], nf, 0, nvec, c1, c2, np, 1);
         }},
        {"add_bf16", 1, [&](int i) {
             reduce_kernel<bf16_t, OP_SUM, EPI_NONE, 2, BLOCK, 4, 1, 0><<<g4, BLOCK>>>(in2(i), 2, Z[i], nbf, 0, nvec, np, 0);
         }},
        {"add_bf16_inplace", 1, [&](int i) {
             reduce_kernel<bf16_t, OP_SUM, EPI_NONE, 2, BLOCK, 4, 1, 0><<<g4, BLOCK>>>(in2(i), 2, X[i], nbf, 0, nvec, np, 0);
         }},
        {"sma_bf16_u4", 1, [&](int i) {
             sma_kernel<bf16_t, float, BLOCK, 4><<<g4, BLOCK>>>(X[i], Y[i], nbf, 0, nvec, c1, c2, np, 1);
         }},
        {"sma_bf16_u2", 1, [&](int i) {
             sma_kernel<bf16_t, float, BLOCK, 2><<<g4 * 2, BLOCK>>>(X[i], Y[i], nbf, 0, nvec, c1, c2, np, 1);
         }},
        {"sma_bf16_u8", 1, [&](int i) {
             sma_kernel<bf16_t, float, BLOCK, 8><<<g4 / 2, BLOCK>>>(X[i], Y[i], nbf, 0, nvec, c1, c2, np, 1);
         }},
        {"sma_bf16_oop", 1, [&](int i) {
             sma_oop<4><<<g4, BLOCK>>>(X[i], Y[i], Z[i], nvec, c1, c2, np);
         }},
        {"xor_bf16_inplace", 1, [&](int i) { xor_inplace<<<g4, BLOCK>>>(X[i], Y[i], nvec); }},
        {"sma_bf16_pk", 1, [&](int i) { sma_pk<<<g4, BLOCK>>>(X[i], Y[i], nvec, c1, c2, np); }},
    };

    // bit checks on set 0: every bf16 blend variant against the shipped u4 kernel
    {
        refill(1);
        std::vector<uint16_t> want(nbf), got(nbf);
        CHECK(hipMemcpy(Z[1], X[0], bytes, hipMemcpyDeviceToDevice));  // keep v
        sma_kernel<bf16_t, float, BLOCK, 4><<<g4, BLOCK>>>(X[0], Y[0], nbf, 0, nvec, c1, c2, np, 1);
        CHECK(hipMemcpy(want.data(), X[0], bytes, hipMemcpyDeviceToHost));
        const char *names[] = {"sma_bf16_u2", "sma_bf16_u8", "sma_bf16_oop", "sma_bf16_pk"};
        for (const char *nm : names) {
            CHECK(hipMemcpy(X[0], Z[1], bytes, hipMemcpyDeviceToDevice));
            void *out = X[0];
            if (!strcmp(nm, "sma_bf16_u2"))
                sma_kernel<bf16_t, float, BLOCK, 2><<<g4 * 2, BLOCK>>>(X[0], Y[0], nbf, 0, nvec, c1, c2, np, 1);
            else if (!strcmp(nm, "sma_bf16_u8"))
                sma_kernel<bf16_t, float, BLOCK, 8><<<g4 / 2, BLOCK>>>(X[0], Y[0], nbf, 0, nvec, c1, c2, np, 1);
            else if (!strcmp(nm, "sma_bf16_oop")) {
                out = Z[2];
                sma_oop<4><<<g4, BLOCK>>>(X[0], Y[0], Z[2], nvec, c1, c2, np);
            } else
                sma_pk<<<g4, BLOCK>>>(X[0], Y[0], nvec, c1, c2, np);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(got.data(), out, bytes, hipMemcpyDeviceToHost));
            const size_t bad = std::inner_product(want.begin(), want.end(), got.begin(), size_t(0),
                                                  std::plus<size_t>(), std::not_equal_to<uint16_t>());
            printf("{\"check\": \"%s\", \"mismatches\": %zu}\n", nm, bad);
        }
    }

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<std::vector<float>> ts(vars.size());
    int cur = -1;
    for (int round = 0; round < 7; ++round) {
        for (size_t v = 0; v < vars.size(); ++v) {
            if (vars[v].bf != cur) {
                refill(vars[v].bf);
                cur = vars[v].bf;
            }
            for (int i = 0; i < NS; ++i) vars[v].run(i);
            CHECK(hipEventRecord(e0));
            for (int i = 0; i < 20; ++i) vars[v].run(i % NS);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            ts[v].push_back(ms * 1e3f / 20);
        }
        // the in-place runs drift the data; refill both kinds every round
        cur = -1;
    }
    CHECK(hipGetLastError());
    for (size_t v = 0; v < vars.size(); ++v) {
        std::sort(ts[v].begin(), ts[v].end());
        const double us = ts[v][ts[v].size() / 2];
        printf("{\"variant\": \"%s\", \"us\": %.2f, \"min_us\": %.2f, \"frac\": %.4f}\n",
               vars[v].name.c_str(), us, ts[v][0], 3.0 * bytes / us / 8e6);
    }
    return 0;
}
