// chunk_latency2.hip — can ONE 1 MiB drop-in call (std_transform_2 on
// page-locked host buffers, zero copy) get under the reference's CPU reduce
// of the same chunk (~55-60 us)? Not part of the product.
//
// Variants (median of REPS calls each, us; every result checked):
//   kernel shape  gs   grid-stride, 4 x/y vectors per lane, then 4 stores (shipped)
//                 pipe software-pipelined: the next 4+4 loads are issued before
//                      the current 4 stores
//   completion    sync hipStreamSynchronize
//                 ev   hipEventRecord + hipEventSynchronize
//                 qry  hipStreamQuery in a loop
//                 spin last block stores a flag into host memory, host spins
//   grid          8 .. 64 blocks of 256
// Plus the kernel alone from HIP events around 200 back-to-back launches.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -o /tmp/chunk_latency2 \
//         tools/explore/chunk_latency2.hip -L kungfu_amd -lkungfu_amd
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

template <bool SPIN>
__device__ __forceinline__ void finish(unsigned *count, unsigned long long *flag,
                                       unsigned long long seq)
{
    if (SPIN) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            const unsigned prev = atomicAdd(count, 1u);
            if (prev == gridDim.x - 1) {
                atomicExch(count, 0u);
                __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

template <bool SPIN>
__global__ void __launch_bounds__(256) zc_gs(const f4 *x, const f4 *y, f4 *z, size_t nv,
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
    finish<SPIN>(count, flag, seq);
}

// the next tile's loads are in flight while the current tile is stored
template <bool SPIN>
__global__ void __launch_bounds__(256) zc_pipe(const f4 *x, const f4 *y, f4 *z, size_t nv,
                                               unsigned *count, unsigned long long *flag,
                                               unsigned long long seq)
{
    const size_t stride = static_cast<size_t>(gridDim.x) * 256 * 4;
    size_t b            = static_cast<size_t>(blockIdx.x) * 256 * 4 + threadIdx.x;
    f4 a[4], c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (b + u * 256 < nv) {
            a[u] = __builtin_nontemporal_load(x + b + u * 256);
            c[u] = __builtin_nontemporal_load(y + b + u * 256);
        }
    while (b < nv) {
        const size_t nb = b + stride;
        f4 a2[4], c2[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (nb + u * 256 < nv) {
                a2[u] = __builtin_nontemporal_load(x + nb + u * 256);
                c2[u] = __builtin_nontemporal_load(y + nb + u * 256);
            }
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (b + u * 256 < nv) __builtin_nontemporal_store(a[u] + c[u], z + b + u * 256);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a[u] = a2[u];
            c[u] = c2[u];
        }
        b = nb;
    }
    finish<SPIN>(count, flag, seq);
}

// completion by a second, one-wave kernel queued behind the reduce on the same
// stream: it starts after the reduce kernel has ended (its stores released),
// and stores `seq` into host memory for the host to spin on
__global__ void flag_after(unsigned long long *flag, unsigned long long seq)
{
    if (threadIdx.x == 0)
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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
    const int reps     = argc > 2 ? std::atoi(argv[2]) : 1000;
    const size_t n     = bytes / 4;
    const size_t nv    = n / 4;
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
    hipEvent_t done, e0, e1;
    CHECK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
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
    printf("{\"bytes\": %zu, \"variant\": \"product\", \"us\": %.2f}\n", bytes, product);
    fflush(stdout);

    const f4 *X = reinterpret_cast<const f4 *>(x), *Y = reinterpret_cast<const f4 *>(y);
    f4 *Z       = reinterpret_cast<f4 *>(z);
    for (int pipe = 0; pipe < 2; ++pipe) {
        for (int g : {8, 16, 32, 64}) {
            auto launch = [&](bool spin, unsigned long long sq) {
                if (pipe) {
                    if (spin) zc_pipe<true><<<g, 256, 0, s>>>(X, Y, Z, nv, count, flag, sq);
                    else zc_pipe<false><<<g, 256, 0, s>>>(X, Y, Z, nv, count, flag, sq);
                } else {
                    if (spin) zc_gs<true><<<g, 256, 0, s>>>(X, Y, Z, nv, count, flag, sq);
                    else zc_gs<false><<<g, 256, 0, s>>>(X, Y, Z, nv, count, flag, sq);
                }
            };
            const char *kname = pipe ? "pipe" : "gs";
            // kernel alone: 200 back-to-back launches between two events
            launch(false, 0);
            CHECK(hipStreamSynchronize(s));
            CHECK(hipEventRecord(e0, s));
            for (int i = 0; i < 200; ++i) launch(false, 0);
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            check("b2b");
            const double sync = median_us(
                [&] {
                    launch(false, 0);
                    (void)hipStreamSynchronize(s);
                },
                reps);
            check("sync");
            const double ev = median_us(
                [&] {
                    launch(false, 0);
                    (void)hipEventRecord(done, s);
                    (void)hipEventSynchronize(done);
                },
                reps);
            check("ev");
            const double qry = median_us(
                [&] {
                    launch(false, 0);
                    while (hipStreamQuery(s) == hipErrorNotReady) {
                    }
                },
                reps);
            check("qry");
            const double spin = median_us(
                [&] {
                    ++seq;
                    launch(true, seq);
                    while (*vflag != seq) {
                    }
                },
                reps);
            CHECK(hipStreamSynchronize(s));
            check("spin");
            // the flag kernel behind the reduce; every call checked right
            // after the flag (fresh y each call, so a stale z would show)
            int bad = 0;
            const double spin2 = median_us(
                [&] {
                    ++seq;
                    y[(seq * 7919) % n] = static_cast<float>(seq % 1000);
                    launch(false, 0);
                    flag_after<<<1, 64, 0, s>>>(flag, seq);
                    while (*vflag != seq) {
                    }
                    const size_t i = (seq * 7919) % n;
                    if (z[i] != x[i] + y[i]) ++bad;
                },
                reps);
            CHECK(hipStreamSynchronize(s));
            if (bad) {
                fprintf(stderr, "flag kernel: %d stale results\n", bad);
                exit(3);
            }
            check("spin2");
            printf("{\"bytes\": %zu, \"variant\": \"%s\", \"grid\": %d, \"kernel_b2b_us\": %.2f, "
                   "\"sync_us\": %.2f, \"ev_us\": %.2f, \"qry_us\": %.2f, \"spin_us\": %.2f, "
                   "\"flag_kernel_spin_us\": %.2f}\n",
                   bytes, kname, g, ms * 1e3 / 200, sync, ev, qry, spin, spin2);
            fflush(stdout);
        }
    }
    const double cpu = median_us(
        [&] {
            for (size_t i = 0; i < n; ++i) z[i] = x[i] + y[i];
        },
        reps);
    printf("{\"bytes\": %zu, \"variant\": \"cpu_loop_1thread\", \"us\": %.2f}\n", bytes, cpu);
    return 0;
}
