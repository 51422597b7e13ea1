// shard_xcd_probe.hip — why does the shard /np of C3 at N = 8 (64 shards of
// 0.5 MiB) take ~15.3 us in bench.py but ~12.9 us in shard_probe.hip? The
// bench's shards are slices of 4 MiB buckets (one shard every 4 MiB of
// address space, as in the exchange), the probe's are separate 0.5 MiB
// allocations. If address translation is the cost, an XCD-aware map of
// blocks to shards (the 8 XCDs each sweep 1/8 of the shards, so each XCD's
// translation cache holds 8 shards' pages, not 64) should recover it.
//
// Layouts: "packed" (shards back to back), "strided" (shard b at b * 4 MiB
// + 3 * 0.5 MiB inside one allocation, the exchange's layout).
// Maps: "rows" (the product's 2-D grid: block x of row b; consecutive
// blocks of a shard go to consecutive XCDs) and "xcd" (linear block L runs
// on XCD L % 8; that XCD's j-th block takes shard (L % 8) + 8 * (j / per)).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o shard_xcd_probe shard_xcd_probe.hip
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

constexpr int kSeg = 64, B = 256;

struct Segs {
    f32x4 *p[kSeg];
    unsigned nvec;  // every shard the same
    unsigned per;   // blocks per shard
    int nseg;
};

template <int U>
__device__ __forceinline__ void tile(f32x4 *p, unsigned nv, unsigned t)
{
    const size_t v0 = static_cast<size_t>(t) * (B * U) + threadIdx.x;
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) v[u] = __builtin_nontemporal_load(p + v0 + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) __builtin_nontemporal_store(v[u] * 0.125f, p + v0 + u * B);
}

template <int U>
__global__ void __launch_bounds__(B) rows_kernel(Segs a)
{
    tile<U>(a.p[blockIdx.y], a.nvec, blockIdx.x);
}

// rows, each shard's tiles taken from a rotated start: blocks of different
// shards running at the same moment touch different offsets (shards at the
// same address modulo 4 MiB otherwise hit the same DRAM channels together)
template <int U>
__global__ void __launch_bounds__(B) rows_rot_kernel(Segs a, unsigned step)
{
    const unsigned t = (blockIdx.x + blockIdx.y * step) % a.per;
    tile<U>(a.p[blockIdx.y], a.nvec, t);
}

// 1-D grid of nseg * per blocks; requires nseg % 8 == 0
template <int U>
__global__ void __launch_bounds__(B) xcd_kernel(Segs a)
{
    const unsigned L    = blockIdx.x;
    const unsigned xcd  = L & 7;
    const unsigned j    = L >> 3;        // this XCD's j-th block
    const unsigned s    = xcd + 8 * (j / a.per);
    const unsigned t    = j % a.per;
    tile<U>(a.p[s], a.nvec, t);
}

template <typename Launch>
double time_us(Launch launch, int nsets);

// the same map on the product's 2-D grid (per x nseg): the dispatch order is
// linear (x fastest), so the linear id picks the XCD
template <int U>
__global__ void __launch_bounds__(B) xcd2d_kernel(Segs a)
{
    const unsigned L   = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned xcd = L & 7;
    const unsigned j   = L >> 3;
    const unsigned s   = xcd + 8 * (j / gridDim.x);
    const unsigned t   = j % gridDim.x;
    tile<U>(a.p[s], a.nvec, t);
}

// C4 at N = 8: 16 buckets of 1,598,976 floats back to back in one flat
// buffer, rank 3's shard of each (199,872 floats)
void c4_flat()
{
    const int nb = 16;
    const size_t c = 1598976, q = c / 8;
    const unsigned nvec = static_cast<unsigned>(q / 4);
    const double bytes  = 2.0 * nb * q * 4;
    const int nsets = 8;
    std::vector<Segs> segs(nsets);
    std::vector<void *> allocs;
    for (int i = 0; i < nsets; ++i) {
        char *base = nullptr;
        CHECK(hipMalloc(&base, nb * c * 4));
        CHECK(hipMemset(base, 0x3f, nb * c * 4));
        allocs.push_back(base);
        segs[i].nseg = nb;
        segs[i].nvec = nvec;
        segs[i].per  = (nvec + B * 2 - 1) / (B * 2);
        for (int s = 0; s < nb; ++s)
            segs[i].p[s] = reinterpret_cast<f32x4 *>(base + s * c * 4 + 3 * q * 4);
    }
    const unsigned per = segs[0].per;
    for (int map = 0; map < 2; ++map) {
        auto launch = [&](int i) {
            if (map == 0) rows_kernel<2><<<dim3(per, nb), B>>>(segs[i]);
            else xcd2d_kernel<2><<<dim3(per, nb), B>>>(segs[i]);
        };
        const double us = time_us(launch, nsets);
        printf("{\"layout\": \"c4 flat\", \"map\": \"%s\", \"unroll\": 2, \"us\": %.2f, "
               "\"frac\": %.4f}\n", map ? "xcd 2-D" : "rows", us, bytes / us / 1e3 / 8000.0);
        fflush(stdout);
    }
    for (auto p : allocs) CHECK(hipFree(p));
}

template <typename Launch>
double time_us(Launch launch, int nsets)
{
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int i = 0; i < nsets; ++i) launch(i);
    CHECK(hipDeviceSynchronize());
    std::vector<double> ts;
    for (int rep = 0; rep < 7; ++rep) {
        CHECK(hipEventRecord(e0));
        for (int i = 0; i < 4 * nsets; ++i) launch(i % nsets);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms * 1e3 / (4 * nsets));
    }
    std::sort(ts.begin(), ts.end());
    return ts[3];
}

int main()
{
    const size_t q      = (1u << 20) / 8;  // 131072 floats: C3's shard at N = 8
    const unsigned nvec = static_cast<unsigned>(q / 4);
    const double bytes  = 2.0 * kSeg * q * 4;
    const int nsets     = 12;
    for (int layout = 0; layout < 2; ++layout) {
        std::vector<Segs> segs(nsets);
        std::vector<void *> allocs;
        for (int i = 0; i < nsets; ++i) {
            Segs &a = segs[i];
            a.nseg  = kSeg;
            a.nvec  = nvec;
            if (layout == 0) {  // packed: one allocation, shards back to back
                f32x4 *base = nullptr;
                CHECK(hipMalloc(&base, kSeg * q * 4));
                CHECK(hipMemset(base, 0x3f, kSeg * q * 4));
                allocs.push_back(base);
                for (int s = 0; s < kSeg; ++s) a.p[s] = base + s * (q / 4);
            } else {  // strided: 64 buckets of 4 MiB, rank 3's shard of each
                char *base = nullptr;
                CHECK(hipMalloc(&base, static_cast<size_t>(kSeg) << 22));
                CHECK(hipMemset(base, 0x3f, static_cast<size_t>(kSeg) << 22));
                allocs.push_back(base);
                for (int s = 0; s < kSeg; ++s)
                    a.p[s] = reinterpret_cast<f32x4 *>(base + (static_cast<size_t>(s) << 22) + 3 * q * 4);
            }
        }
        for (int u = 0; u < 2; ++u) {
            const int U          = u == 0 ? 2 : 4;
            const unsigned per   = (nvec + B * U - 1) / (B * U);
            for (auto &a : segs) a.per = per;
            for (int map = 0; map < 5; ++map) {
                const unsigned step = map == 2 ? 1u : (per / 8 ? per / 8 : 1u) * 3 + 1;
                auto launch = [&](int i) {
                    if (map == 4) {
                        if (U == 2) xcd2d_kernel<2><<<dim3(per, kSeg), B>>>(segs[i]);
                        else xcd2d_kernel<4><<<dim3(per, kSeg), B>>>(segs[i]);
                    } else if (map >= 2) {
                        if (U == 2) rows_rot_kernel<2><<<dim3(per, kSeg), B>>>(segs[i], step);
                        else rows_rot_kernel<4><<<dim3(per, kSeg), B>>>(segs[i], step);
                    } else if (map == 0) {
                        if (U == 2) rows_kernel<2><<<dim3(per, kSeg), B>>>(segs[i]);
                        else rows_kernel<4><<<dim3(per, kSeg), B>>>(segs[i]);
                    } else {
                        if (U == 2) xcd_kernel<2><<<per * kSeg, B>>>(segs[i]);
                        else xcd_kernel<4><<<per * kSeg, B>>>(segs[i]);
                    }
                };
                const double us = time_us(launch, nsets);
                printf("{\"layout\": \"%s\", \"map\": \"%s\", \"unroll\": %d, \"us\": %.2f, "
                       "\"frac\": %.4f}\n",
                       layout ? "strided" : "packed",
                       map == 0 ? "rows" : map == 1 ? "xcd" : map == 2 ? "rows rot 1" : map == 3 ? "rows rot 3p/8+1" : "xcd 2-D",
                       U, us,
                       bytes / us / 1e3 / 8000.0);
                fflush(stdout);
            }
        }
        // correctness of the xcd map: every shard scaled exactly once
        {
            std::vector<float> h(q, 8.0f);
            for (int s = 0; s < kSeg; ++s)
                CHECK(hipMemcpy(segs[0].p[s], h.data(), q * 4, hipMemcpyHostToDevice));
            segs[0].per = (nvec + B * 2 - 1) / (B * 2);
            xcd_kernel<2><<<segs[0].per * kSeg, B>>>(segs[0]);
            for (int s = 0; s < kSeg; ++s) {
                CHECK(hipMemcpy(h.data(), segs[0].p[s], q * 4, hipMemcpyDeviceToHost));
                for (size_t i = 0; i < q; ++i) {
                    if (h[i] != 1.0f) {
                        fprintf(stderr, "xcd map wrong at shard %d elem %zu: %f\n", s, i, h[i]);
                        return 3;
                    }
                }
                std::fill(h.begin(), h.end(), 8.0f);
            }
        }
        for (auto p : allocs) CHECK(hipFree(p));
    }
    c4_flat();
    return 0;
}
