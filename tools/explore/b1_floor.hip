// b1_floor.hip — what one std_transform_2 call costs at the chunk sizes the
// reference passes (session.go:301-326: chunks of at most 1 MiB), split with a
// host timer into its parts:
//
//   attr6      six hipPointerGetAttributes (two per buffer: first and last
//              byte), the classification every call made before round 6
//   launch     host time of the zero-copy launch itself (the shipped
//              reduce_kernel<float, SUM, NONE, 2>, 32 blocks, non-blocking
//              stream), returned before the kernel runs
//   sync       hipStreamSynchronize right after it: the kernel's run over
//              PCIe plus the completion signal
//   empty      an empty kernel's launch + sync on the same stream: the
//              floor of any GPU round trip
//   call_reg   std_transform_2 end to end, buffers malloc'd and page-locked
//              with kf_host_register (the registry lookup, no attributes)
//   call_pin   std_transform_2 end to end, buffers from hipHostMalloc (not
//              registered through the library: six attribute queries)
//   cpu        z = x + y on one core, the reference's loop (op.cpp:22-35)
//
// Medians of 9 rounds of `reps` calls; z checked against x + y.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off -I include \
//       -I kungfu_amd/csrc -o tools/explore/b1_floor tools/explore/b1_floor.hip \
//       -L kungfu_amd -lkungfu_amd -Wl,-rpath,$PWD/kungfu_amd
//   tools/explore/b1_floor > profiles/r06/b1_floor.jsonl
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "kf_reduce_kernels.hpp"
#include "kungfu_amd.h"

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

__global__ void empty_kernel() {}

using clk = std::chrono::steady_clock;

static double us_since(clk::time_point t0)
{
    return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
}

__attribute__((noinline)) void cpu_add(const float *x, const float *y, float *z, size_t n)
{
    for (size_t i = 0; i < n; ++i) z[i] = x[i] + y[i];
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main()
{
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t sizes[] = {64 << 10, 256 << 10, 1 << 20, 4 << 20};
    for (size_t bytes : sizes) {
        const size_t n = bytes / 4;
        const int reps = bytes <= (256 << 10) ? 400 : 100;
        // page-locked by the runtime
        float *px, *py, *pz;
        CHECK(hipHostMalloc(&px, bytes, 0));
        CHECK(hipHostMalloc(&py, bytes, 0));
        CHECK(hipHostMalloc(&pz, bytes, 0));
        // malloc'd, registered through the library
        float *rx = static_cast<float *>(aligned_alloc(4096, bytes));
        float *ry = static_cast<float *>(aligned_alloc(4096, bytes));
        float *rz = static_cast<float *>(aligned_alloc(4096, bytes));
        for (size_t i = 0; i < n; ++i) {
            px[i] = rx[i] = 0.25f * static_cast<float>(i % 977);
            py[i] = ry[i] = 1.5f - 0.125f * static_cast<float>(i % 613);
        }
        if (kf_host_register(rx, bytes) || kf_host_register(ry, bytes) || kf_host_register(rz, bytes)) {
            fprintf(stderr, "kf_host_register: %s\n", kf_last_error());
            return 2;
        }
        void *dx, *dy, *dz;
        CHECK(hipHostGetDevicePointer(&dx, px, 0));
        CHECK(hipHostGetDevicePointer(&dy, py, 0));
        CHECK(hipHostGetDevicePointer(&dz, pz, 0));
        kf::InPtrs in{};
        in.p[0] = dx;
        in.p[1] = dy;
        const kf::Div np{1.f, 1.f, 1.0, 1.0, 1};
        const size_t nvec = n / 4;

        std::vector<double> attr, launch, sync, empty, call_reg, call_pin, cpu;
        for (int round = 0; round < 9; ++round) {
            auto t0 = clk::now();
            for (int r = 0; r < reps; ++r) {
                hipPointerAttribute_t a;
                const void *ps[3] = {px, py, pz};
                for (const void *p : ps) {
                    CHECK(hipPointerGetAttributes(&a, p));
                    CHECK(hipPointerGetAttributes(&a, static_cast<const char *>(p) + bytes - 1));
                }
            }
            attr.push_back(us_since(t0) / reps);
            double tl = 0, ts = 0;
            for (int r = 0; r < reps; ++r) {
                auto a = clk::now();
                kf::reduce_kernel<float, kf::OP_SUM, kf::EPI_NONE, 2, 256, 4, 1, 0>
                    <<<32, 256, 0, s>>>(in, 2, dz, n, 0, nvec, np, 0);
                auto b = clk::now();
                CHECK(hipStreamSynchronize(s));
                tl += std::chrono::duration<double, std::micro>(b - a).count();
                ts += us_since(b);
            }
            launch.push_back(tl / reps);
            sync.push_back(ts / reps);
            t0 = clk::now();
            for (int r = 0; r < reps; ++r) {
                empty_kernel<<<1, 64, 0, s>>>();
                CHECK(hipStreamSynchronize(s));
            }
            empty.push_back(us_since(t0) / reps);
            t0 = clk::now();
            for (int r = 0; r < reps; ++r) std_transform_2(rx, ry, rz, static_cast<int>(n), KungFu_FLOAT, KungFu_SUM);
            call_reg.push_back(us_since(t0) / reps);
            t0 = clk::now();
            for (int r = 0; r < reps; ++r) std_transform_2(px, py, pz, static_cast<int>(n), KungFu_FLOAT, KungFu_SUM);
            call_pin.push_back(us_since(t0) / reps);
            t0 = clk::now();
            for (int r = 0; r < reps; ++r) cpu_add(rx, ry, rz + 0, n);
            cpu.push_back(us_since(t0) / reps);
        }
        // correctness of the two end-to-end paths
        std_transform_2(rx, ry, rz, static_cast<int>(n), KungFu_FLOAT, KungFu_SUM);
        std_transform_2(px, py, pz, static_cast<int>(n), KungFu_FLOAT, KungFu_SUM);
        size_t bad = 0;
        for (size_t i = 0; i < n; ++i) bad += (rz[i] != rx[i] + ry[i]) + (pz[i] != px[i] + py[i]);
        printf("{\"chunk_KiB\": %zu, \"attr6_us\": %.2f, \"launch_us\": %.2f, \"sync_us\": %.2f, "
               "\"empty_roundtrip_us\": %.2f, \"call_registered_us\": %.2f, \"call_hipHostMalloc_us\": %.2f, "
               "\"cpu_1thread_us\": %.2f, \"mismatches\": %zu}\n",
               bytes >> 10, median(attr), median(launch), median(sync), median(empty), median(call_reg),
               median(call_pin), median(cpu), bad);
        fflush(stdout);
        kf_host_unregister(rx);
        kf_host_unregister(ry);
        kf_host_unregister(rz);
        free(rx);
        free(ry);
        free(rz);
        CHECK(hipHostFree(px));
        CHECK(hipHostFree(py));
        CHECK(hipHostFree(pz));
    }
    return 0;
}
