// shard_probe.hip — the exchange's shard /np epilogue at N = 8 (in place,
// x *= 1/8, exact for a power of two), the kernel furthest below its
// roofline in the r04 line (C4: 16 shards of ~0.76 MiB, 8.0 us = 0.40 of
// 8 TB/s; C3: 64 shards of 0.5 MiB, 0.54). Shapes of one launch varied:
// threads per block, vectors per lane, cache policy, a persistent
// grid-stride form that issues the next tile's loads before storing the
// current one, and shard-interleaved block order. Launches cycle over enough
// shard sets (>= 0.75 GiB) that none is served from the Infinity Cache, as
// bench.py's `kernels` does; "warm" repeats one set (the exchange's real
// case: the reduce-scatter has just written the shard).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -o shard_probe shard_probe.hip \
//         -L../../kungfu_amd -lkungfu_amd -Wl,-rpath,'$ORIGIN/../../kungfu_amd'
// ("library": the product's kf_bucket_reduce_batch on the same shards)
//   ./shard_probe            # one JSON line per (config, variant)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kungfu_amd.h"
#include "../../kungfu_amd/csrc/kf_reduce_kernels.hpp"

typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

constexpr int kMaxSeg = 64;

struct Segs {
    f32x4 *p[kMaxSeg];
    unsigned nvec[kMaxSeg];
    unsigned blk0[kMaxSeg + 1];  // first block of each shard (contiguous mapping)
    unsigned tile0[kMaxSeg + 1]; // first tile of each shard (flattened tile space)
    int nseg;
};

template <int POL>
__device__ __forceinline__ f32x4 ldp(const f32x4 *p)
{
    if constexpr (POL & 1) return __builtin_nontemporal_load(p);
    else return *p;
}

template <int POL>
__device__ __forceinline__ void stp(f32x4 *p, f32x4 v)
{
    if constexpr (POL & 2) __builtin_nontemporal_store(v, p);
    else *p = v;
}

__device__ __forceinline__ int seg_of(const unsigned *starts, int nseg, unsigned b)
{
    int lo = 0, hi = nseg - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (b >= starts[mid]) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// one tile (B * U vectors) per block, shards' blocks contiguous (the product's map)
template <int B, int U, int POL>
__global__ void __launch_bounds__(B) tile_kernel(Segs a)
{
    const int s       = seg_of(a.blk0, a.nseg, blockIdx.x);
    const unsigned t  = blockIdx.x - a.blk0[s];
    const size_t v0   = static_cast<size_t>(t) * (B * U) + threadIdx.x;
    f32x4 *p          = a.p[s];
    const unsigned nv = a.nvec[s];
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) v[u] = ldp<POL>(p + v0 + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) stp<POL>(p + v0 + u * B, v[u] * 0.125f);
}

// the tile kernel with its argument block padded to the product's ~2.8 KB
// (BatchArgsT<64, 1>): does the kernarg size cost launch time?
struct SegsPadded {
    Segs a;
    char pad[1536];
};
template <int B, int U, int POL>
__global__ void __launch_bounds__(B) tile_kernel_padded(SegsPadded pa)
{
    const Segs &a     = pa.a;
    const int s       = seg_of(a.blk0, a.nseg, blockIdx.x);
    const unsigned t  = blockIdx.x - a.blk0[s];
    const size_t v0   = static_cast<size_t>(t) * (B * U) + threadIdx.x;
    f32x4 *p          = a.p[s];
    const unsigned nv = a.nvec[s];
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) v[u] = ldp<POL>(p + v0 + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) stp<POL>(p + v0 + u * B, v[u] * 0.125f);
}

// the tile kernel with the shard found by one division (every shard has the
// same block count) instead of a binary search over the kernarg table
template <int B, int U, int POL>
__global__ void __launch_bounds__(B) tile_kernel_uniform(Segs a, unsigned per)
{
    const int s       = blockIdx.x / per;
    const unsigned t  = blockIdx.x - s * per;
    const size_t v0   = static_cast<size_t>(t) * (B * U) + threadIdx.x;
    f32x4 *p          = a.p[s];
    const unsigned nv = a.nvec[s];
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) v[u] = ldp<POL>(p + v0 + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) stp<POL>(p + v0 + u * B, v[u] * 0.125f);
}

// the same, block b taking tile (b / nseg) of shard (b % nseg): every shard
// is swept by every part of the grid at once
template <int B, int U, int POL>
__global__ void __launch_bounds__(B) interleaved_kernel(Segs a, unsigned tiles_max)
{
    const int s       = blockIdx.x % a.nseg;
    const unsigned t  = blockIdx.x / a.nseg;
    const unsigned nv = a.nvec[s];
    const size_t v0   = static_cast<size_t>(t) * (B * U) + threadIdx.x;
    if (v0 >= nv) return;
    f32x4 *p = a.p[s];
    f32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) v[u] = ldp<POL>(p + v0 + u * B);
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) stp<POL>(p + v0 + u * B, v[u] * 0.125f);
    (void)tiles_max;
}

// persistent: gridDim blocks stride over the flattened tile space; the next
// tile's loads are issued before the current tile is stored
template <int B, int U, int POL>
__global__ void __launch_bounds__(B) persistent_kernel(Segs a)
{
    const unsigned ntiles = a.tile0[a.nseg];
    unsigned t            = blockIdx.x;
    if (t >= ntiles) return;
    auto locate = [&](unsigned tt, f32x4 *&p, size_t &v0, unsigned &nv) {
        const int s = seg_of(a.tile0, a.nseg, tt);
        p           = a.p[s];
        nv          = a.nvec[s];
        v0          = static_cast<size_t>(tt - a.tile0[s]) * (B * U) + threadIdx.x;
    };
    f32x4 *p;
    size_t v0;
    unsigned nv;
    locate(t, p, v0, nv);
    f32x4 cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
        if (v0 + u * B < nv) cur[u] = ldp<POL>(p + v0 + u * B);
    for (;;) {
        const unsigned tn = t + gridDim.x;
        f32x4 *pn         = nullptr;
        size_t vn         = 0;
        unsigned nvn      = 0;
        f32x4 nxt[U];
        if (tn < ntiles) {
            locate(tn, pn, vn, nvn);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (vn + u * B < nvn) nxt[u] = ldp<POL>(pn + vn + u * B);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (v0 + u * B < nv) stp<POL>(p + v0 + u * B, cur[u] * 0.125f);
        if (tn >= ntiles) break;
        t = tn;
        p = pn;
        v0 = vn;
        nv = nvn;
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
}

struct Set {
    std::vector<f32x4 *> shards;
};

template <int B, int U>
Segs make_segs(const Set &s, const std::vector<unsigned> &nvec)
{
    Segs a{};
    a.nseg        = static_cast<int>(nvec.size());
    unsigned blk  = 0;
    for (int i = 0; i < a.nseg; ++i) {
        a.p[i]     = s.shards[i];
        a.nvec[i]  = nvec[i];
        a.blk0[i]  = blk;
        a.tile0[i] = blk;
        blk += (nvec[i] + B * U - 1) / (B * U);
    }
    a.blk0[a.nseg]  = blk;
    a.tile0[a.nseg] = blk;
    return a;
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
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return ts[3];
}

template <int B, int U, int POL>
void run_variant(const char *cfg, const char *name, int form, const std::vector<Set> &sets,
                 const std::vector<unsigned> &nvec, double bytes, bool warm)
{
    const int nsets = warm ? 1 : static_cast<int>(sets.size());
    std::vector<Segs> segs;
    for (auto &s : sets) segs.push_back(make_segs<B, U>(s, nvec));
    const unsigned nblk = segs[0].blk0[segs[0].nseg];
    unsigned maxt       = 0;
    for (unsigned nv : nvec) maxt = std::max(maxt, (nv + B * U - 1) / (B * U));
    int dev = 0, ncu = 0;
    CHECK(hipGetDevice(&dev));
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const unsigned pgrid = std::min<unsigned>(nblk, static_cast<unsigned>(ncu) * 4);
    auto launch = [&](int i) {
        if (form == 4) {
            tile_kernel_uniform<B, U, POL><<<nblk, B>>>(segs[i], nblk / segs[i].nseg);
        } else if (form == 3) {
            SegsPadded pa{};
            pa.a = segs[i];
            tile_kernel_padded<B, U, POL><<<nblk, B>>>(pa);
        } else if (form == 0) {
            tile_kernel<B, U, POL><<<nblk, B>>>(segs[i]);
        } else if (form == 1) {
            interleaved_kernel<B, U, POL><<<maxt * segs[i].nseg, B>>>(segs[i], maxt);
        } else {
            persistent_kernel<B, U, POL><<<pgrid, B>>>(segs[i]);
        }
    };
    const double us = time_us(launch, nsets);
    printf("{\"config\": \"%s\", \"variant\": \"%s\", \"block\": %d, \"unroll\": %d, \"pol\": %d, "
           "\"form\": %d, \"warm\": %s, \"us\": %.2f, \"frac\": %.4f}\n",
           cfg, name, B, U, POL, form, warm ? "true" : "false", us, bytes / us / 1e3 / 8000.0);
    fflush(stdout);
}

void config(const char *cfg, const std::vector<size_t> &counts)
{
    std::vector<unsigned> nvec;
    size_t per_set = 0;
    for (size_t c : counts) {
        nvec.push_back(static_cast<unsigned>(c / 4));
        per_set += c * 4;
    }
    const int nsets = std::max<int>(2, static_cast<int>(((768u << 20) + per_set - 1) / per_set));
    std::vector<Set> sets(nsets);
    for (auto &s : sets) {
        for (size_t c : counts) {
            f32x4 *p = nullptr;
            CHECK(hipMalloc(&p, c * 4));
            CHECK(hipMemset(p, 0x3f, c * 4));
            s.shards.push_back(p);
        }
    }
    // correctness of every form once: x *= 1/8 on a known value
    {
        float h = 0;
        const float one = 8.0f;
        std::vector<float> init(counts[0], one);
        CHECK(hipMemcpy(sets[0].shards[0], init.data(), counts[0] * 4, hipMemcpyHostToDevice));
        auto a = make_segs<256, 2>(sets[0], nvec);
        persistent_kernel<256, 2, 3><<<64, 256>>>(a);
        CHECK(hipMemcpy(&h, reinterpret_cast<float *>(sets[0].shards[0]) + counts[0] - 1, 4,
                        hipMemcpyDeviceToHost));
        if (h != 1.0f) {
            fprintf(stderr, "persistent form wrong: %f\n", h);
            exit(3);
        }
    }
    const double bytes = 2.0 * per_set;
    {  // the product entry point, same shards, same timing
        std::vector<std::vector<void *>> ptrs(nsets);
        std::vector<size_t> cnt(counts.begin(), counts.end());
        for (int i = 0; i < nsets; ++i)
            for (auto p : sets[i].shards) ptrs[i].push_back(p);
        auto launch = [&](int i) {
            const int rc = kf_bucket_reduce_batch(const_cast<const void *const *>(ptrs[i].data()), 1,
                                                  ptrs[i].data(), cnt.data(),
                                                  static_cast<int>(cnt.size()), KungFu_FLOAT,
                                                  KungFu_SUM, 8, nullptr);
            if (rc != KF_OK) {
                fprintf(stderr, "kf_bucket_reduce_batch: %d\n", rc);
                exit(4);
            }
        };
        for (int warm = 0; warm < 2; ++warm) {
            const double us = time_us(launch, warm ? 1 : nsets);
            printf("{\"config\": \"%s\", \"variant\": \"library kf_bucket_reduce_batch\", "
                   "\"warm\": %s, \"us\": %.2f, \"frac\": %.4f}\n",
                   cfg, warm ? "true" : "false", us, bytes / us / 1e3 / 8000.0);
        }
    }
    // the product's batch kernel itself, launched here with the arguments the
    // host builds (so the launch path is the probe's), per = common blocks or 0
    for (int variant = 0; variant < 3; ++variant) {
        constexpr int B = 256;
        const int U = variant == 2 ? 4 : 2;
        std::vector<kf::BatchArgsT<64, 1>> args(nsets);
        unsigned nblk_total = 0;
        for (int i = 0; i < nsets; ++i) {
            auto &a = args[i];
            memset(&a, 0, sizeof(a));
            a.nseg = static_cast<int>(nvec.size());
            unsigned blk = 0;
            const unsigned per = (nvec[0] + B * U - 1) / (B * U);
            for (int j = 0; j < a.nseg; ++j) {
                a.in[j][0] = sets[i].shards[j];
                a.out[j]   = sets[i].shards[j];
                a.n[j]     = counts[j];
                a.head[j]  = 0;
                a.nvec[j]  = nvec[j];
                a.blk0[j]  = blk;
                blk += per;
            }
            a.blk0[a.nseg] = blk;
            a.serial       = 0;
            nblk_total     = blk;
        }
        kf::Div np{};
        np.f = 8.0f; np.fi = 0.125f; np.d = 8.0; np.di = 0.125; np.pow2 = 1;
        for (int warm = 0; warm < 2; ++warm) {
            const unsigned nseg = static_cast<unsigned>(nvec.size());
            const dim3 grid = variant == 1 ? dim3(nblk_total) : dim3(nblk_total / nseg, nseg);
            auto launch = [&](int i) {
                if (U == 2)
                    kf::reduce_batch_kernel<float, kf::OP_SUM, kf::EPI_DIV, 1, 256, 2, 64, 1>
                        <<<grid, 256>>>(args[i], 1, np);
                else
                    kf::reduce_batch_kernel<float, kf::OP_SUM, kf::EPI_DIV, 1, 256, 4, 64, 1>
                        <<<grid, 256>>>(args[i], 1, np);
            };
            const double us = time_us(launch, warm ? 1 : nsets);
            printf("{\"config\": \"%s\", \"variant\": \"product kernel U=%d %s\", "
                   "\"warm\": %s, \"us\": %.2f, \"frac\": %.4f}\n",
                   cfg, U, variant == 1 ? "search" : "grid rows", warm ? "true" : "false", us,
                   bytes / us / 1e3 / 8000.0);
        }
    }
    for (int warm = 0; warm < 2; ++warm) {
        run_variant<256, 2, 3>(cfg, "tile 256x2 nt (product)", 0, sets, nvec, bytes, warm);
        run_variant<256, 2, 3>(cfg, "tile 256x2 nt, 2.8 KB args", 3, sets, nvec, bytes, warm);
        run_variant<256, 2, 3>(cfg, "tile 256x2 nt, shard by division", 4, sets, nvec, bytes, warm);
        run_variant<256, 4, 3>(cfg, "tile 256x4 nt, shard by division", 4, sets, nvec, bytes, warm);
        if (warm) continue;
        run_variant<256, 1, 3>(cfg, "tile 256x1 nt", 0, sets, nvec, bytes, false);
        run_variant<256, 4, 3>(cfg, "tile 256x4 nt", 0, sets, nvec, bytes, false);
        run_variant<512, 2, 3>(cfg, "tile 512x2 nt", 0, sets, nvec, bytes, false);
        run_variant<1024, 1, 3>(cfg, "tile 1024x1 nt", 0, sets, nvec, bytes, false);
        run_variant<256, 2, 0>(cfg, "tile 256x2 plain", 0, sets, nvec, bytes, false);
        run_variant<256, 2, 1>(cfg, "tile 256x2 nt-load plain-store", 0, sets, nvec, bytes, false);
        run_variant<256, 2, 2>(cfg, "tile 256x2 plain-load nt-store", 0, sets, nvec, bytes, false);
        run_variant<256, 2, 3>(cfg, "interleaved 256x2 nt", 1, sets, nvec, bytes, false);
        run_variant<256, 1, 3>(cfg, "interleaved 256x1 nt", 1, sets, nvec, bytes, false);
        run_variant<256, 2, 3>(cfg, "persistent 4/CU 256x2 nt", 2, sets, nvec, bytes, false);
        run_variant<256, 1, 3>(cfg, "persistent 4/CU 256x1 nt", 2, sets, nvec, bytes, false);
        run_variant<512, 1, 3>(cfg, "persistent 4/CU 512x1 nt", 2, sets, nvec, bytes, false);
    }
    for (auto &s : sets)
        for (auto p : s.shards) CHECK(hipFree(p));
}

int main()
{
    // C4 at N = 8: ResNet-50's 25,583,592 fp32 gradients in 16 buckets, one
    // shard of each (~1.6 M elements per bucket / 8)
    std::vector<size_t> c4(16, 199872);
    config("c4_shard_n8", c4);
    // C3 at N = 8: 64 buckets of 4 MiB, a 0.5 MiB shard of each
    std::vector<size_t> c3(64, 131072);
    config("c3_shard_n8", c3);
    return 0;
}
