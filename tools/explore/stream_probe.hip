// stream_probe.hip — what a kernel pays to move 1 MiB between HBM and
// page-locked host memory, by memory kind and fence scheme (kf_stream.hip's
// design question). Each variant: 256 blocks x 256 lanes x 16 B, average of
// 50 launches timed with HIP events; hipMemcpyAsync for comparison.
//
//     hipcc --offload-arch=gfx950 -O3 -o tools/explore/stream_probe tools/explore/stream_probe.hip
//     tools/explore/stream_probe          # one JSON line
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

constexpr unsigned kLen = 1u << 20, kBlock = 4096, kLanes = 256;

// fence: 0 none, 1 system fence + release add per block, 2 relaxed add only
// store: 0 plain 16 B, 1 two 8-B system-scope relaxed stores
template <int Fence, int Store>
__global__ void __launch_bounds__(kLanes) out_k(const uint4 *src, char *host, unsigned *done)
{
    const unsigned i = blockIdx.x * (kBlock / 16) + threadIdx.x;
    const uint4 v    = src[i];
    if (Store == 0) {
        reinterpret_cast<uint4 *>(host)[i] = v;
    } else {
        auto *h = reinterpret_cast<unsigned long long *>(host) + 2 * i;
        __hip_atomic_store(h, (unsigned long long)v.x | ((unsigned long long)v.y << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(h + 1, (unsigned long long)v.z | ((unsigned long long)v.w << 32),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (Fence == 1) __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0 && Fence == 1) {
        __hip_atomic_fetch_add(done + blockIdx.x / 16, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (threadIdx.x == 0 && Fence == 2) {
        __hip_atomic_fetch_add(done + blockIdx.x / 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// one flag word per block instead of a counter: flag: 0 system release
// fence + relaxed system store, 1 each wave waits for its stores, barrier,
// plain store of the flag
template <int Flag>
__global__ void __launch_bounds__(kLanes) out_flag_k(const uint4 *src, char *host, unsigned *flags)
{
    const unsigned i = blockIdx.x * (kBlock / 16) + threadIdx.x;
    reinterpret_cast<uint4 *>(host)[i] = src[i];
    if (Flag == 0) {
        __threadfence_system();
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (Flag == 0) {
            __hip_atomic_store(flags + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        } else {
            *reinterpret_cast<volatile unsigned *>(flags + blockIdx.x) = 1u;
        }
    }
}

// acq: 0 none, 1 one system acquire per block after a relaxed poll, 2 the
// poll itself an acquire load (one iteration: the flag is already set)
// load: 0 plain 16 B, 1 two 8-B system-scope relaxed loads
template <int Acq, int Load>
__global__ void __launch_bounds__(kLanes) in_k(const char *host, uint4 *dst, const unsigned *flag)
{
    __shared__ int ok;
    if (threadIdx.x == 0) {
        if (Acq == 2) {
            ok = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        } else {
            ok = __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
        }
    }
    __syncthreads();
    if (Acq == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    const unsigned i = blockIdx.x * (kBlock / 16) + threadIdx.x;
    uint4 v;
    if (Load == 0) {
        v = reinterpret_cast<const uint4 *>(host)[i];
    } else {
        auto *h = reinterpret_cast<const unsigned long long *>(host) + 2 * i;
        const unsigned long long a = __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        const unsigned long long b = __hip_atomic_load(h + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        v = make_uint4(unsigned(a), unsigned(a >> 32), unsigned(b), unsigned(b >> 32));
    }
    if (ok) dst[i] = v;
}

// the session root's whole-chunk fold: out(host) = own(HBM) + landing(host),
// 1 MiB fp32, grid-stride over 16-B vectors with `blocks` blocks
__global__ void __launch_bounds__(kLanes) fold_grid_k(const float4 *own, const float4 *landing,
                                                       float4 *out, unsigned nvec)
{
    for (unsigned i = blockIdx.x * kLanes + threadIdx.x; i < nvec; i += gridDim.x * kLanes) {
        const float4 a = own[i], b = landing[i];
        out[i]         = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
}

// 16-B buffer stores / loads with a cache policy (aux: 1 sc0, 16 sc1, 17 sc0 sc1)
template <int AUX>
__global__ void __launch_bounds__(kLanes) out_buf_k(const uint4 *src, char *host, unsigned *flags)
{
    const unsigned i = blockIdx.x * (kBlock / 16) + threadIdx.x;
    const uint4 v    = src[i];
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(host, 0, kLen, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const __attribute__((ext_vector_type(4))) unsigned *>(&v),
                                           r, i * 16, 0, AUX);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(flags + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <int AUX>
__global__ void __launch_bounds__(kLanes) in_buf_k(const char *host, uint4 *dst)
{
    const unsigned i = blockIdx.x * (kBlock / 16) + threadIdx.x;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(host), 0, kLen, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, i * 16, 0, AUX);
    dst[i]       = make_uint4(v[0], v[1], v[2], v[3]);
}

template <typename F>
float timed(hipStream_t s, F f)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int r = 0; r < 5; ++r) f();
    CK(hipEventRecord(a, s));
    for (int r = 0; r < 50; ++r) f();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1000.f / 50;
}

int main()
{
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    void *dev, *dev2, *hc, *hn, *hcd, *hnd, *ctl, *ctld;
    CK(hipMalloc(&dev, kLen));
    CK(hipMalloc(&dev2, kLen));
    CK(hipMemset(dev, 1, kLen));
    CK(hipHostMalloc(&hc, kLen, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc(&hn, kLen, hipHostMallocMapped | hipHostMallocNonCoherent));
    CK(hipHostMalloc(&ctl, 8192, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer(&hcd, hc, 0));
    CK(hipHostGetDevicePointer(&hnd, hn, 0));
    CK(hipHostGetDevicePointer(&ctld, ctl, 0));
    std::memset(ctl, 0, 8192);
    *static_cast<unsigned *>(ctl) = 1;  // flag set: the in-kernels never wait
    auto *done = static_cast<unsigned *>(ctld) + 64;  // counters, or one flag per block
    auto *flag = static_cast<const unsigned *>(ctld);
    const dim3 g(kLen / kBlock), b(kLanes);
    auto *src = static_cast<const uint4 *>(dev);
    auto *dst = static_cast<uint4 *>(dev2);
    void *hd, *hdd;
    CK(hipHostMalloc(&hd, kLen, hipHostMallocDefault));
    CK(hipHostGetDevicePointer(&hdd, hd, 0));
    struct Mem {
        const char *name;
        char *d;
        void *h;
    } mems[3] = {{"coherent", static_cast<char *>(hcd), hc},
                 {"noncoherent", static_cast<char *>(hnd), hn},
                 {"default", static_cast<char *>(hdd), hd}};
    std::printf("{");
    bool first = true;
    auto put   = [&](const char *mem, const char *what, float us) {
        std::printf("%s\"%s/%s\": %.2f", first ? "" : ", ", mem, what, us);
        first = false;
    };
    for (auto &m : mems) {
        char *h = m.d;
        put(m.name, "out_plain_nofence_us", timed(s, [&] { out_k<0, 0><<<g, b, 0, s>>>(src, h, done); }));
        put(m.name, "out_plain_sysfence_release_us",
            timed(s, [&] { out_k<1, 0><<<g, b, 0, s>>>(src, h, done); }));
        put(m.name, "out_plain_relaxed_add_us", timed(s, [&] { out_k<2, 0><<<g, b, 0, s>>>(src, h, done); }));
        put(m.name, "out_sys8_relaxed_add_us", timed(s, [&] { out_k<2, 1><<<g, b, 0, s>>>(src, h, done); }));
        put(m.name, "out_flag_sysfence_us", timed(s, [&] { out_flag_k<0><<<g, b, 0, s>>>(src, h, done); }));
        put(m.name, "out_flag_waitcnt_us", timed(s, [&] { out_flag_k<1><<<g, b, 0, s>>>(src, h, done); }));
        put(m.name, "out_buf_sc0_flag_us", timed(s, [&] { out_buf_k<1><<<g, b, 0, s>>>(src, h, done); }));
        put(m.name, "out_buf_sc1_flag_us", timed(s, [&] { out_buf_k<16><<<g, b, 0, s>>>(src, h, done); }));
        put(m.name, "out_buf_sc0sc1_flag_us", timed(s, [&] { out_buf_k<17><<<g, b, 0, s>>>(src, h, done); }));
        put(m.name, "in_buf_plain_us", timed(s, [&] { in_buf_k<0><<<g, b, 0, s>>>(h, dst); }));
        put(m.name, "in_buf_sc0sc1_us", timed(s, [&] { in_buf_k<17><<<g, b, 0, s>>>(h, dst); }));
        put(m.name, "in_plain_noacq_us", timed(s, [&] { in_k<0, 0><<<g, b, 0, s>>>(h, dst, flag); }));
        put(m.name, "in_plain_one_acq_us", timed(s, [&] { in_k<1, 0><<<g, b, 0, s>>>(h, dst, flag); }));
        put(m.name, "in_plain_acq_poll_us", timed(s, [&] { in_k<2, 0><<<g, b, 0, s>>>(h, dst, flag); }));
        put(m.name, "in_sys8_us", timed(s, [&] { in_k<0, 1><<<g, b, 0, s>>>(h, dst, flag); }));
        put(m.name, "memcpy_d2h_us",
            timed(s, [&] { CK(hipMemcpyAsync(m.h, dev, kLen, hipMemcpyDeviceToHost, s)); }));
        put(m.name, "memcpy_h2d_us",
            timed(s, [&] { CK(hipMemcpyAsync(dev2, m.h, kLen, hipMemcpyHostToDevice, s)); }));
    }
    for (auto &m : mems) {  // one copy, launch to completion, as a chunk sees it
        hipEvent_t e;
        CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        double tot = 0;
        for (int r = 0; r < 20; ++r) {
            auto t0 = std::chrono::steady_clock::now();
            CK(hipMemcpyAsync(m.h, dev, kLen, hipMemcpyDeviceToHost, s));
            CK(hipEventRecord(e, s));
            CK(hipEventSynchronize(e));
            if (r >= 5) tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        }
        put(m.name, "memcpy_d2h_one_wall_us", float(tot / 15));
        CK(hipEventDestroy(e));
    }
    for (unsigned blocks : {32u, 64u, 128u, 256u, 512u}) {  // grid of the root's fold
        char name[64];
        std::snprintf(name, sizeof(name), "fold_host_in_out_%u_blocks_us", blocks);
        auto *land = reinterpret_cast<const float4 *>(mems[2].d);
        auto *outh = reinterpret_cast<float4 *>(mems[1].d);
        put("default", name, timed(s, [&] {
                fold_grid_k<<<blocks, kLanes, 0, s>>>(reinterpret_cast<const float4 *>(dev), land, outh,
                                                      kLen / 16);
            }));
    }
    {  // the CPU's side: memcpy of 1 MiB into and out of each kind (what read()/write() do)
        static char buf[kLen];
        std::memset(buf, 3, kLen);
        for (auto &m : mems) {
            for (int dir = 0; dir < 2; ++dir) {
                double best = 1e9;
                for (int r = 0; r < 20; ++r) {
                    auto t0 = std::chrono::steady_clock::now();
                    if (dir == 0) std::memcpy(m.h, buf, kLen);
                    else std::memcpy(buf, m.h, kLen);
                    best = std::min(best, std::chrono::duration<double, std::micro>(
                                              std::chrono::steady_clock::now() - t0).count());
                }
                put(m.name, dir == 0 ? "cpu_memcpy_into_us" : "cpu_memcpy_out_of_us", float(best));
            }
        }
    }
    std::printf("}\n");
    CK(hipStreamSynchronize(s));
    return 0;
}
