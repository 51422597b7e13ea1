// xproc_probe.hip — does a kernel that waits in the GPU (kf_stream's kind:
// one watcher lane polling page-locked memory, 257 blocks polling an HBM
// word) slow another PROCESS's copies and launches on the same GPU? C1 runs
// both peers on one GPU, and its streamed runs slowed the other peer.
//
// The process forks before any HIP call. The child launches `waiter` kernels
// (each waits ~2 ms of wall clock, like a chunk's kernel waiting for its
// body) back to back for the whole measurement, or nothing (baseline). The
// parent measures, each median of 200: a 1 MiB D2H into page-locked memory,
// a 1 MiB H2D, and an empty kernel's launch-to-completion.
//
//     hipcc --offload-arch=gfx950 -O3 -o tools/explore/xproc_probe tools/explore/xproc_probe.hip
//     tools/explore/xproc_probe      # one JSON line
#include <hip/hip_runtime.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

__device__ unsigned long long g_word;

// block 0 lane 0 polls page-locked memory; the others poll an HBM word with
// s_sleep(sleep_units); everyone leaves after `ticks` of wall clock
__global__ void waiter(const unsigned *host_flag, unsigned long long ticks, int sleep_units)
{
    const unsigned long long t0 = wall_clock64();
    if (threadIdx.x != 0) return;
    for (;;) {
        if (blockIdx.x == 0) {
            if (__hip_atomic_load(host_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        } else if (__hip_atomic_load(&g_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1) {
            break;
        }
        if (wall_clock64() - t0 > ticks) break;
        if (sleep_units > 8) {
            __builtin_amdgcn_s_sleep(20);
        } else {
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

__global__ void empty_k() {}

static double median(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static void child(int mode, int begin_fd, int go_fd, int stop_fd)
{
    char c;
    if (read(begin_fd, &c, 1) != 1) std::exit(1);  // HIP only from here on
    unsigned *flag = nullptr, *flag_d = nullptr;
    hipStream_t s  = nullptr;
    if (mode > 0) {
        CK(hipHostMalloc(&flag, 4096, hipHostMallocMapped | hipHostMallocCoherent));
        *flag = 0;
        CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&flag_d), flag, 0));
        CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    if (write(go_fd, &c, 1) != 1) std::exit(1);
    for (;;) {  // ~2 ms per kernel at 100 MHz
        if (mode > 0) {
            waiter<<<258, 256, 0, s>>>(flag_d, 200000ull, mode);
            CK(hipStreamSynchronize(s));
        } else {
            usleep(2000);
        }
        fd_set fs;
        FD_ZERO(&fs);
        FD_SET(stop_fd, &fs);
        timeval tv{0, 0};
        if (select(stop_fd + 1, &fs, nullptr, nullptr, &tv) > 0) break;
    }
    std::exit(0);
}

int main()
{
    // every child is forked before this process makes its first HIP call
    const char *names[] = {"idle_neighbour", "waiting_neighbour_sleep1", "waiting_neighbour_sleep20"};
    const int modes[]   = {0, 1, 20};
    int begin[3][2], go[3][2], stop[3][2];
    pid_t pid[3];
    for (int m = 0; m < 3; ++m) {
        if (pipe(begin[m]) || pipe(go[m]) || pipe(stop[m])) return 1;
        pid[m] = fork();
        if (pid[m] == 0) child(modes[m], begin[m][0], go[m][1], stop[m][0]);
    }
    void *dev, *host;
    hipStream_t s;
    CK(hipMalloc(&dev, 1 << 20));
    CK(hipHostMalloc(&host, 1 << 20, hipHostMallocDefault));
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::printf("{");
    for (int m = 0; m < 3; ++m) {
        char c = 1;
        if (write(begin[m][1], &c, 1) != 1 || read(go[m][0], &c, 1) != 1) return 1;
        usleep(20000);
        std::vector<double> d2h, h2d, launch;
        for (int r = 0; r < 200; ++r) {
            auto t0 = std::chrono::steady_clock::now();
            CK(hipMemcpyAsync(host, dev, 1 << 20, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            auto t1 = std::chrono::steady_clock::now();
            CK(hipMemcpyAsync(dev, host, 1 << 20, hipMemcpyHostToDevice, s));
            CK(hipStreamSynchronize(s));
            auto t2 = std::chrono::steady_clock::now();
            empty_k<<<1, 64, 0, s>>>();
            CK(hipStreamSynchronize(s));
            auto t3 = std::chrono::steady_clock::now();
            d2h.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            h2d.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
            launch.push_back(std::chrono::duration<double, std::micro>(t3 - t2).count());
        }
        if (write(stop[m][1], &c, 1) != 1) return 1;
        int st = 0;
        waitpid(pid[m], &st, 0);
        std::printf("%s\"%s\": {\"d2h_1MiB_us\": %.1f, \"h2d_1MiB_us\": %.1f, \"empty_kernel_us\": %.1f, "
                    "\"child_status\": %d}",
                    m ? ", " : "", names[m], median(d2h), median(h2d), median(launch), st);
        std::fflush(stdout);
    }
    std::printf("}\n");
    return 0;
}
