// c2_explore.hip — standalone experiment for the C2 kernel (z = x + y, fp32,
// 256 MiB per input): block size x unroll x cache-policy bits x buffer offsets.
// Not part of the product; results feed the defaults in kf_capi.hip.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o c2_explore c2_explore.hip
//   ./c2_explore > results.jsonl
//
// Timing: HIP events around 40 back-to-back launches that cycle over 3
// independent bucket sets (cold Infinity Cache), 5 interleaved rounds, median.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

// cache policy aux bits (gfx950): sc0 = 1, nt = 2, sc1 = 16
template <int BLOCK, int UNROLL, int LD, int ST>
__global__ void __launch_bounds__(BLOCK)
    add_buf(const float *x, const float *y, float *z, unsigned nvec)
{
    const unsigned bytes = nvec * 16u;
    auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x), 0, bytes, 0x00020000);
    auto ry = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(y), 0, bytes, 0x00020000);
    auto rz = __builtin_amdgcn_make_buffer_rsrc(z, 0, bytes, 0x00020000);
    const unsigned v0 = blockIdx.x * (BLOCK * UNROLL) + threadIdx.x;
    u32x4 a[UNROLL], b[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
        a[u] = __builtin_amdgcn_raw_buffer_load_b128(rx, (v0 + u * BLOCK) * 16u, 0, LD);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
        b[u] = __builtin_amdgcn_raw_buffer_load_b128(ry, (v0 + u * BLOCK) * 16u, 0, LD);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
        f32x4 fa = __builtin_bit_cast(f32x4, a[u]);
        f32x4 fb = __builtin_bit_cast(f32x4, b[u]);
        f32x4 fc = fa + fb;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, fc), rz,
                                               (v0 + u * BLOCK) * 16u, 0, ST);
    }
}

struct Variant {
    std::string name;
    int block, unroll, ld, st;
    std::function<void(const float *, const float *, float *, unsigned, hipStream_t)> run;
};

template <int BLOCK, int UNROLL, int LD, int ST>
Variant make()
{
    Variant v;
    v.block  = BLOCK;
    v.unroll = UNROLL;
    v.ld     = LD;
    v.st     = ST;
    v.name   = "b" + std::to_string(BLOCK) + "_u" + std::to_string(UNROLL) +
             "_ld" + std::to_string(LD) + "_st" + std::to_string(ST);
    v.run = [](const float *x, const float *y, float *z, unsigned nvec, hipStream_t s) {
        const unsigned tile = BLOCK * UNROLL;
        add_buf<BLOCK, UNROLL, LD, ST><<<nvec / tile, BLOCK, 0, s>>>(x, y, z, nvec);
    };
    return v;
}

int main(int argc, char **argv)
{
    const size_t n     = 64ull << 20;  // fp32 elements per input
    const size_t bytes = n * 4;
    const int rotate   = 3;
    const int launches = 40, rounds = 5;
    // offsets (bytes) applied to y and z relative to x within each set
    std::vector<std::pair<size_t, size_t>> offsets = {{0, 0}, {4096, 8192}, {65536, 131072},
                                                      {1 << 20, 2 << 20}, {2048, 6144}};
    std::vector<Variant> vs = {
        // block x unroll at nt/nt
        make<256, 2, 2, 2>(), make<256, 4, 2, 2>(), make<256, 8, 2, 2>(),
        make<512, 2, 2, 2>(), make<512, 4, 2, 2>(), make<512, 8, 2, 2>(),
        make<1024, 1, 2, 2>(), make<1024, 2, 2, 2>(), make<1024, 4, 2, 2>(),
        make<128, 4, 2, 2>(), make<128, 8, 2, 2>(), make<64, 8, 2, 2>(),
        // cache policy at 256 x 4
        make<256, 4, 0, 0>(), make<256, 4, 0, 2>(), make<256, 4, 2, 0>(),
        make<256, 4, 16, 2>(), make<256, 4, 18, 2>(), make<256, 4, 1, 2>(),
        make<256, 4, 3, 2>(), make<256, 4, 19, 2>(), make<256, 4, 2, 17>(),
        make<256, 4, 2, 19>(), make<256, 4, 2, 16>(), make<256, 4, 2, 18>(),
        make<256, 4, 18, 18>(), make<256, 4, 2, 1>(), make<256, 4, 2, 3>(),
    };
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    // one big allocation per set so offsets stay inside it
    const size_t slack = 4 << 20;
    std::vector<char *> base(rotate);
    for (int r = 0; r < rotate; ++r) {
        CHECK(hipMalloc(&base[r], 3 * bytes + 3 * slack));
        std::vector<float> h(n);
        for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
        CHECK(hipMemcpy(base[r], h.data(), bytes, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(base[r] + bytes + slack, h.data(), bytes, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const unsigned nvec = n / 4;
    auto ptrs = [&](int r, size_t oy, size_t oz) {
        char *b = base[r];
        return std::make_tuple((const float *)b, (const float *)(b + bytes + slack + oy),
                               (float *)(b + 2 * (bytes + slack) + oz));
    };
    auto time_variant = [&](const Variant &v, size_t oy, size_t oz) {
        for (int i = 0; i < 3; ++i) {
            auto [x, y, z] = ptrs(i % rotate, oy, oz);
            v.run(x, y, z, nvec, s);
        }
        CHECK(hipEventRecord(e0, s));
        for (int i = 0; i < launches; ++i) {
            auto [x, y, z] = ptrs(i % rotate, oy, oz);
            v.run(x, y, z, nvec, s);
        }
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms * 1e3 / launches;
    };
    // correctness of every variant once
    {
        std::vector<float> hx(n), hz(n);
        CHECK(hipMemcpy(hx.data(), base[0], bytes, hipMemcpyDeviceToHost));
        for (auto &v : vs) {
            auto [x, y, z] = ptrs(0, 0, 0);
            CHECK(hipMemset((void *)z, 0, bytes));
            v.run(x, y, z, nvec, s);
            CHECK(hipStreamSynchronize(s));
            CHECK(hipMemcpy(hz.data(), z, bytes, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < n; i += 4099)
                if (hz[i] != hx[i] + hx[i]) {
                    fprintf(stderr, "variant %s wrong at %zu\n", v.name.c_str(), i);
                    return 3;
                }
        }
    }
    std::vector<std::vector<double>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t i = 0; i < vs.size(); ++i) t[i].push_back(time_variant(vs[i], 0, 0));
    size_t best = 0;
    for (size_t i = 0; i < vs.size(); ++i) {
        std::sort(t[i].begin(), t[i].end());
        double med = t[i][rounds / 2];
        if (med < t[best][rounds / 2]) best = i;
        printf("{\"variant\": \"%s\", \"block\": %d, \"unroll\": %d, \"ld\": %d, \"st\": %d, "
               "\"median_us\": %.2f, \"min_us\": %.2f, \"GBps\": %.1f}\n",
               vs[i].name.c_str(), vs[i].block, vs[i].unroll, vs[i].ld, vs[i].st, med,
               t[i][0], 3.0 * bytes / med / 1e3);
    }
    // offsets on the best variant
    for (auto [oy, oz] : offsets) {
        std::vector<double> tt;
        for (int r = 0; r < rounds; ++r) tt.push_back(time_variant(vs[best], oy, oz));
        std::sort(tt.begin(), tt.end());
        printf("{\"variant\": \"%s\", \"offset_y\": %zu, \"offset_z\": %zu, \"median_us\": %.2f, "
               "\"GBps\": %.1f}\n",
               vs[best].name.c_str(), oy, oz, tt[rounds / 2], 3.0 * bytes / tt[rounds / 2] / 1e3);
    }
    return 0;
}
