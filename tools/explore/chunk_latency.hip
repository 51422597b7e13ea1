// chunk_latency.hip — where the time of ONE 1 MiB fp32 drop-in call goes
// (std_transform_2 on page-locked host buffers, the reference's unit of work:
// session.go:301-326 cuts every bucket into 1 MiB chunks). Not part of the
// product; results decide the B1 host path.
//
// Rows (median of REPS calls each, us):
//   product      std_transform_2 from libkungfu_amd.so
//   attrs        6 x hipPointerGetAttributes (the product's classify())
//   empty        launch of an empty kernel + hipStreamSynchronize
//   empty_spin   launch of an empty kernel that stores a flag into host
//                memory; the host spins on the flag (no runtime sync)
//   zc_sync      zero-copy add kernel (G blocks) + hipStreamSynchronize
//   zc_spin      same kernel, last block stores the done flag, host spins
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o /tmp/chunk_latency \
//         tools/explore/chunk_latency.hip -L kungfu_amd -lkungfu_amd
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kungfu_amd.h"

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void empty_kernel() {}

__global__ void flag_kernel(unsigned long long *flag, unsigned long long seq)
{
    if (threadIdx.x == 0)
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// grid-stride float4 add over host memory; with SPIN the last block to finish
// stores `seq` into the host flag after every block's stores are released
template <bool SPIN>
__global__ void __launch_bounds__(256) zc_add(const f4 *x, const f4 *y, f4 *z, size_t nv,
                                              unsigned *count, unsigned long long *flag,
                                              unsigned long long seq)
{
    const size_t stride = static_cast<size_t>(gridDim.x) * 256 * 4;
    for (size_t b = static_cast<size_t>(blockIdx.x) * 256 * 4 + threadIdx.x; b < nv;
         b += stride) {
        f4 a[4], c[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (b + u * 256 < nv) {
                a[u] = __builtin_nontemporal_load(x + b + u * 256);
                c[u] = __builtin_nontemporal_load(y + b + u * 256);
            }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (b + u * 256 < nv) __builtin_nontemporal_store(a[u] + c[u], z + b + u * 256);
    }
    if (SPIN) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            const unsigned prev = atomicAdd(count, 1u);
            if (prev == gridDim.x - 1) {
                *count = 0;
                __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

template <typename F>
static double median_us(F f, int reps)
{
    std::vector<double> t(reps);
    for (int i = 0; i < 20; ++i) f();
    for (int i = 0; i < reps; ++i) {
        const double t0 = now();
        f();
        t[i] = (now() - t0) * 1e6;
    }
    std::sort(t.begin(), t.end());
    return t[reps / 2];
}

int main(int argc, char **argv)
{
    const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (1u << 20);
    const int reps     = 2000;
    const size_t n     = bytes / 4;
    float *x, *y, *z;
    CHECK(hipHostMalloc(&x, bytes, hipHostMallocDefault));
    CHECK(hipHostMalloc(&y, bytes, hipHostMallocDefault));
    CHECK(hipHostMalloc(&z, bytes, hipHostMallocDefault));
    for (size_t i = 0; i < n; ++i) {
        x[i] = static_cast<float>(i % 1000) * 0.5f;
        y[i] = static_cast<float>(i % 777) * 0.25f;
    }
    unsigned long long *flag;
    CHECK(hipHostMalloc(&flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
    *flag = 0;
    unsigned *count;
    CHECK(hipMalloc(&count, 64));
    CHECK(hipMemset(count, 0, 64));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    volatile unsigned long long *vflag = flag;
    unsigned long long seq             = 0;

    auto check = [&](const char *what) {
        for (size_t i = 0; i < n; ++i)
            if (z[i] != x[i] + y[i]) {
                fprintf(stderr, "%s: mismatch at %zu\n", what, i);
                exit(3);
            }
        std::fill(z, z + n, -1.0f);
    };

    const double product = median_us(
        [&] { std_transform_2(x, y, z, static_cast<int>(n), KungFu_FLOAT, KungFu_SUM); }, reps);
    check("product");
    const double attrs = median_us(
        [&] {
            hipPointerAttribute_t a;
            for (int i = 0; i < 3; ++i) {
                (void)hipPointerGetAttributes(&a, x);
                (void)hipPointerGetAttributes(&a, x + n - 1);
            }
        },
        reps);
    const double empty = median_us(
        [&] {
            empty_kernel<<<1, 64, 0, s>>>();
            (void)hipStreamSynchronize(s);
        },
        reps);
    const double empty_spin = median_us(
        [&] {
            ++seq;
            flag_kernel<<<1, 64, 0, s>>>(flag, seq);
            while (*vflag != seq) {
            }
        },
        reps);
    (void)hipStreamSynchronize(s);
    printf("{\"bytes\": %zu, \"product_us\": %.2f, \"attrs6_us\": %.2f, \"empty_sync_us\": %.2f, "
           "\"empty_spin_us\": %.2f}\n",
           bytes, product, attrs, empty, empty_spin);
    const size_t nv = n / 4;
    for (int g : {16, 32, 64, 128}) {
        const double zs = median_us(
            [&] {
                zc_add<false><<<g, 256, 0, s>>>(reinterpret_cast<const f4 *>(x),
                                                reinterpret_cast<const f4 *>(y),
                                                reinterpret_cast<f4 *>(z), nv, count, flag, 0);
                (void)hipStreamSynchronize(s);
            },
            reps);
        check("zc_sync");
        const double zp = median_us(
            [&] {
                ++seq;
                zc_add<true><<<g, 256, 0, s>>>(reinterpret_cast<const f4 *>(x),
                                               reinterpret_cast<const f4 *>(y),
                                               reinterpret_cast<f4 *>(z), nv, count, flag, seq);
                while (*vflag != seq) {
                }
            },
            reps);
        (void)hipStreamSynchronize(s);
        check("zc_spin");
        printf("{\"bytes\": %zu, \"grid\": %d, \"zc_sync_us\": %.2f, \"zc_spin_us\": %.2f}\n",
               bytes, g, zs, zp);
    }
    return 0;
}
