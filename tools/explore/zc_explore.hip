// zc_explore.hip — host-memory reduce z = x + y (fp32) with x, y, z in
// page-locked host memory: staged copies (H2D, kernel, D2H on two streams)
// against a zero-copy kernel that reads and writes the host buffers over PCIe
// directly, and against the ingest shape (peer chunk in host memory, own chunk
// and result in HBM). Not part of the product; results decide the host path.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o zc_explore zc_explore.hip
//   ./zc_explore > zc.jsonl
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

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

// grid-stride float4 sum; UNROLL vectors per lane in flight
template <int UNROLL>
__global__ void __launch_bounds__(256) add_kernel(const f4 *x, const f4 *y, f4 *z, size_t nv)
{
    const size_t stride = static_cast<size_t>(gridDim.x) * 256 * UNROLL;
    for (size_t b = static_cast<size_t>(blockIdx.x) * 256 * UNROLL + threadIdx.x; b < nv;
         b += stride) {
        f4 a[UNROLL], c[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t i = b + u * 256;
            if (i < nv) {
                a[u] = __builtin_nontemporal_load(x + i);
                c[u] = __builtin_nontemporal_load(y + i);
            }
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t i = b + u * 256;
            if (i < nv) __builtin_nontemporal_store(a[u] + c[u], z + i);
        }
    }
}

struct Bufs {
    float *hx, *hy, *hz;  // host
    float *dx, *dy, *dz;  // device
};

static void fill(float *p, size_t n, float s)
{
    for (size_t i = 0; i < n; ++i) p[i] = s * static_cast<float>(i % 1024);
}

static bool check(const float *z, size_t n)
{
    for (size_t i = 0; i < n; ++i)
        if (z[i] != 3.0f * static_cast<float>(i % 1024)) return false;
    return true;
}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main()
{
    const size_t maxb = size_t(256) << 20;
    hipStream_t s0, s1;
    CHECK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    hipEvent_t ev;
    CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const char *kinds[] = {"hostmalloc_coherent", "hostmalloc_noncoherent", "registered"};
    for (int kind = 0; kind < 3; ++kind) {
        Bufs b{};
        float **hs[3] = {&b.hx, &b.hy, &b.hz};
        for (auto h : hs) {
            if (kind == 0) {
                CHECK(hipHostMalloc(reinterpret_cast<void **>(h), maxb, hipHostMallocCoherent));
            } else if (kind == 1) {
                CHECK(hipHostMalloc(reinterpret_cast<void **>(h), maxb, hipHostMallocNonCoherent));
            } else {
                void *p = nullptr;
                if (posix_memalign(&p, 4096, maxb) != 0) exit(3);
                memset(p, 0, maxb);
                CHECK(hipHostRegister(p, maxb, hipHostRegisterMapped));
                *h = static_cast<float *>(p);
            }
        }
        float *ghx = b.hx, *ghy = b.hy, *ghz = b.hz;  // device views of the host buffers
        CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&ghx), b.hx, 0));
        CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&ghy), b.hy, 0));
        CHECK(hipHostGetDevicePointer(reinterpret_cast<void **>(&ghz), b.hz, 0));
        CHECK(hipMalloc(&b.dx, maxb));
        CHECK(hipMalloc(&b.dy, maxb));
        CHECK(hipMalloc(&b.dz, maxb));
        fill(b.hx, maxb / 4, 1.0f);
        fill(b.hy, maxb / 4, 2.0f);
        CHECK(hipMemcpy(b.dy, b.hy, maxb, hipMemcpyHostToDevice));
        for (size_t bytes : {size_t(1) << 20, size_t(4) << 20, size_t(16) << 20, size_t(64) << 20,
                             size_t(256) << 20}) {
            const size_t n = bytes / 4, nv = n / 4;
            const int reps = bytes <= (size_t(4) << 20) ? 200 : (bytes <= (size_t(64) << 20) ? 20 : 5);
            // (A) staged: whole-buffer copies, H2D + kernel on s0, D2H on s1
            {
                std::vector<double> t;
                for (int r = 0; r < reps + 2; ++r) {
                    memset(b.hz, 0, bytes);
                    double t0 = now();
                    CHECK(hipMemcpyAsync(b.dx, b.hx, bytes, hipMemcpyHostToDevice, s0));
                    CHECK(hipMemcpyAsync(b.dy, b.hy, bytes, hipMemcpyHostToDevice, s0));
                    unsigned grid = static_cast<unsigned>(std::min<size_t>((nv + 1023) / 1024, 16384));
                    add_kernel<4><<<grid, 256, 0, s0>>>(reinterpret_cast<f4 *>(b.dx),
                                                        reinterpret_cast<f4 *>(b.dy),
                                                        reinterpret_cast<f4 *>(b.dz), nv);
                    CHECK(hipEventRecord(ev, s0));
                    CHECK(hipStreamWaitEvent(s1, ev, 0));
                    CHECK(hipMemcpyAsync(b.hz, b.dz, bytes, hipMemcpyDeviceToHost, s1));
                    CHECK(hipStreamSynchronize(s1));
                    if (r >= 2) t.push_back(now() - t0);
                }
                const double m = median(t);
                printf("{\"kind\": \"%s\", \"path\": \"staged\", \"bytes\": %zu, \"us\": %.2f, "
                       "\"bucket_GBps\": %.2f, \"ok\": %d}\n",
                       kinds[kind], bytes, m * 1e6, bytes / m / 1e9, check(b.hz, n));
            }
            // (B) zero-copy: the kernel reads host x, y and writes host z
            for (unsigned grid : {64u, 256u, 1024u, 4096u}) {
                for (int unroll : {1, 4}) {
                    std::vector<double> t;
                    for (int r = 0; r < reps + 2; ++r) {
                        memset(b.hz, 0, bytes);
                        double t0 = now();
                        if (unroll == 1)
                            add_kernel<1><<<grid, 256, 0, s0>>>(reinterpret_cast<f4 *>(ghx),
                                                                reinterpret_cast<f4 *>(ghy),
                                                                reinterpret_cast<f4 *>(ghz), nv);
                        else
                            add_kernel<4><<<grid, 256, 0, s0>>>(reinterpret_cast<f4 *>(ghx),
                                                                reinterpret_cast<f4 *>(ghy),
                                                                reinterpret_cast<f4 *>(ghz), nv);
                        CHECK(hipStreamSynchronize(s0));
                        if (r >= 2) t.push_back(now() - t0);
                    }
                    const double m = median(t);
                    printf("{\"kind\": \"%s\", \"path\": \"zerocopy\", \"grid\": %u, \"unroll\": %d, "
                           "\"bytes\": %zu, \"us\": %.2f, \"bucket_GBps\": %.2f, \"ok\": %d}\n",
                           kinds[kind], grid, unroll, bytes, m * 1e6, bytes / m / 1e9,
                           check(b.hz, n));
                }
            }
            // (C) ingest shape: peer chunk in host memory, own + result in HBM
            for (unsigned grid : {256u, 1024u}) {
                std::vector<double> t;
                for (int r = 0; r < reps + 2; ++r) {
                    double t0 = now();
                    add_kernel<4><<<grid, 256, 0, s0>>>(reinterpret_cast<f4 *>(ghx),
                                                        reinterpret_cast<f4 *>(b.dy),
                                                        reinterpret_cast<f4 *>(b.dz), nv);
                    CHECK(hipStreamSynchronize(s0));
                    if (r >= 2) t.push_back(now() - t0);
                }
                const double m = median(t);
                printf("{\"kind\": \"%s\", \"path\": \"ingest_zerocopy\", \"grid\": %u, "
                       "\"bytes\": %zu, \"us\": %.2f, \"bucket_GBps\": %.2f}\n",
                       kinds[kind], grid, bytes, m * 1e6, bytes / m / 1e9);
            }
            {  // (C') ingest staged: H2D of the peer chunk, then the kernel
                std::vector<double> t;
                for (int r = 0; r < reps + 2; ++r) {
                    double t0 = now();
                    CHECK(hipMemcpyAsync(b.dx, b.hx, bytes, hipMemcpyHostToDevice, s0));
                    unsigned grid = static_cast<unsigned>(std::min<size_t>((nv + 1023) / 1024, 16384));
                    add_kernel<4><<<grid, 256, 0, s0>>>(reinterpret_cast<f4 *>(b.dx),
                                                        reinterpret_cast<f4 *>(b.dy),
                                                        reinterpret_cast<f4 *>(b.dz), nv);
                    CHECK(hipStreamSynchronize(s0));
                    if (r >= 2) t.push_back(now() - t0);
                }
                const double m = median(t);
                printf("{\"kind\": \"%s\", \"path\": \"ingest_staged\", \"bytes\": %zu, "
                       "\"us\": %.2f, \"bucket_GBps\": %.2f}\n",
                       kinds[kind], bytes, m * 1e6, bytes / m / 1e9);
            }
            fflush(stdout);
        }
        CHECK(hipFree(b.dx));
        CHECK(hipFree(b.dy));
        CHECK(hipFree(b.dz));
        for (auto h : hs) {
            if (kind < 2) {
                CHECK(hipHostFree(*h));
            } else {
                CHECK(hipHostUnregister(*h));
                free(*h);
            }
        }
    }
    return 0;
}
