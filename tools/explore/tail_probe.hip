// tail_probe.hip — does the last, partly filled round of blocks cost C5?
//
// The streaming kernels give every block one tile of 256 lanes x 4 vectors
// (16 KiB per stream). At C2's 256 MiB that is 16384 tiles: exactly 8 rounds
// of the 2048 blocks the chip holds at once (256 CUs x 8 blocks of 4 waves).
// C5's blend covers 218,976,256 B per stream: 13,365 tiles, 6.53 rounds, so
// the last round runs the chip half full. The same in-place xor (read v,
// read s, write v: the blend's traffic with no arithmetic) ran at 0.81 of
// 8 TB/s at 256 MiB and 0.78 on C5's bytes (profiles/r06/sma_probe_r06a.jsonl,
// sma_batch_probe_r06m.jsonl).
//
//   oneshot    one tile per block (the shipped shape)
//   bal<G>     G blocks (a multiple of the resident count), each a
//              contiguous, equal share of the range, in tiles of 1024
//              vectors with a ragged last tile
//   stride<G>  G blocks striding over the 1024-vector tiles
//   even       one tile per block, the tile shrunk so the tile count is a
//              whole number of rounds (lanes x u vectors, u <= 4 at run time)
//
// Sizes: C5's flat bytes, 256 MiB and 200 MiB per stream. Median of 7 x 24.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I kungfu_amd/csrc \
//       -o tools/explore/tail_probe tools/explore/tail_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "kf_reduce_kernels.hpp"

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

using kf::u32x4;
constexpr int BLOCK = 256, U = 4, TILE = BLOCK * U;

__device__ __forceinline__ void tile_xor(u32x4 *v, const u32x4 *s, size_t t0, size_t end)
{
    const size_t v0 = t0 + threadIdx.x;
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        x[u] = vi < end ? __builtin_nontemporal_load(v + vi) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        y[u] = vi < end ? __builtin_nontemporal_load(s + vi) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        if (vi < end) __builtin_nontemporal_store(x[u] ^ y[u], v + vi);
    }
}

__global__ void __launch_bounds__(BLOCK) oneshot(u32x4 *v, const u32x4 *s, size_t n)
{
    tile_xor(v, s, static_cast<size_t>(blockIdx.x) * TILE, n);
}

__global__ void __launch_bounds__(BLOCK) bal(u32x4 *v, const u32x4 *s, size_t n)
{
    // equal shares, rounded to whole lanes-worth (256 vectors)
    const size_t units = (n + BLOCK - 1) / BLOCK;
    const size_t b0 = units * blockIdx.x / gridDim.x * BLOCK;
    const size_t b1 = std::min(n, units * (blockIdx.x + 1) / gridDim.x * BLOCK);
    for (size_t t = b0; t < b1; t += TILE) tile_xor(v, s, t, b1);
}

__global__ void __launch_bounds__(BLOCK) stride(u32x4 *v, const u32x4 *s, size_t n)
{
    for (size_t t = static_cast<size_t>(blockIdx.x) * TILE; t < n; t += static_cast<size_t>(gridDim.x) * TILE)
        tile_xor(v, s, t, n);
}

// one tile of BLOCK x uu vectors per block (uu <= U, chosen on the host)
__global__ void __launch_bounds__(BLOCK) even(u32x4 *v, const u32x4 *s, size_t n, int uu)
{
    const size_t v0 = static_cast<size_t>(blockIdx.x) * BLOCK * uu + threadIdx.x;
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        x[u] = (u < uu && vi < n) ? __builtin_nontemporal_load(v + vi) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        y[u] = (u < uu && vi < n) ? __builtin_nontemporal_load(s + vi) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const size_t vi = v0 + u * BLOCK;
        if (u < uu && vi < n) __builtin_nontemporal_store(x[u] ^ y[u], v + vi);
    }
}

__global__ void fill(uint32_t *p, size_t n, uint32_t seed)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = static_cast<uint32_t>(i) * 2654435761u ^ seed;
}

int main()
{
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    int occ = 0;
    CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, oneshot, BLOCK, 0));
    const unsigned resident = static_cast<unsigned>(prop.multiProcessorCount * occ);
    printf("{\"cus\": %d, \"blocks_per_cu\": %d, \"resident\": %u}\n", prop.multiProcessorCount, occ, resident);
    const size_t sizes[] = {218976256, 256u << 20, 200u << 20};  // bytes per stream
    const int NS = 3;
    const size_t maxb = 256u << 20;
    std::vector<u32x4 *> V(NS), S(NS);
    for (int k = 0; k < NS; ++k) {
        CHECK(hipMalloc(&V[k], maxb));
        CHECK(hipMalloc(&S[k], maxb));
        fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(V[k]), maxb / 4, 17u + k);
        fill<<<4096, 256>>>(reinterpret_cast<uint32_t *>(S[k]), maxb / 4, 71u + k);
    }
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (size_t bytes : sizes) {
        const size_t n = bytes / 16;
        const unsigned tiles = static_cast<unsigned>((n + TILE - 1) / TILE);
        struct Var {
            std::string name;
            std::function<void(int)> run;
        };
        std::vector<Var> vars;
        vars.push_back({"oneshot", [=](int k) { oneshot<<<tiles, BLOCK>>>(V[k], S[k], n); }});
        for (unsigned m : {1u, 2u, 4u, 6u, 7u, 8u}) {
            const unsigned g = resident * m;
            vars.push_back({"bal" + std::to_string(m), [=](int k) { bal<<<g, BLOCK>>>(V[k], S[k], n); }});
            vars.push_back({"stride" + std::to_string(m), [=](int k) { stride<<<g, BLOCK>>>(V[k], S[k], n); }});
        }
        {
            // rounds = ceil(tiles / resident); vectors per lane so that
            // resident x rounds blocks cover n
            const unsigned rounds = (tiles + resident - 1) / resident;
            const size_t per_block = (n + static_cast<size_t>(resident) * rounds - 1) / (static_cast<size_t>(resident) * rounds);
            const int uu = static_cast<int>((per_block + BLOCK - 1) / BLOCK);
            const unsigned g = static_cast<unsigned>((n + static_cast<size_t>(BLOCK) * uu - 1) / (static_cast<size_t>(BLOCK) * uu));
            if (uu <= U)
                vars.push_back({"even_u" + std::to_string(uu) + "_g" + std::to_string(g),
                                [=](int k) { even<<<g, BLOCK>>>(V[k], S[k], n, uu); }});
            // more, smaller rounds: lanes x 2 and lanes x 3 tiles, whole rounds
            for (int u2 : {2, 3}) {
                const size_t cap = static_cast<size_t>(resident) * BLOCK * u2;
                const size_t r2 = (n + cap - 1) / cap;
                const size_t pb = (n + resident * r2 - 1) / (resident * r2);
                const int uq = static_cast<int>((pb + BLOCK - 1) / BLOCK);
                const unsigned g2 = static_cast<unsigned>((n + static_cast<size_t>(BLOCK) * uq - 1) / (static_cast<size_t>(BLOCK) * uq));
                vars.push_back({"even_u" + std::to_string(uq) + "_g" + std::to_string(g2),
                                [=](int k) { even<<<g2, BLOCK>>>(V[k], S[k], n, uq); }});
            }
        }
        std::vector<std::vector<float>> ts(vars.size());
        for (int round = 0; round < 7; ++round)
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
        CHECK(hipGetLastError());
        for (size_t v = 0; v < vars.size(); ++v) {
            std::sort(ts[v].begin(), ts[v].end());
            const double us = ts[v][ts[v].size() / 2];
            printf("{\"bytes_per_stream\": %zu, \"tiles\": %u, \"variant\": \"%s\", \"us\": %.2f, \"min_us\": %.2f, "
                   "\"frac\": %.4f}\n",
                   bytes, tiles, vars[v].name.c_str(), us, ts[v][0], 3.0 * bytes / us / 8e6);
        }
    }
    return 0;
}
