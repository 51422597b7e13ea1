// kf_p2p.hip — peer-to-peer pieces for an all-reduce over xGMI without RCCL:
// HIP IPC export/import of device buffers between the processes of one node,
// and a gather kernel that pulls several peers' shards in one launch.
//
// The exchange built on them (kungfu_amd/p2p.py): every rank folds ITS shard
// of the bucket straight out of every peer's HBM with the k-input reduce
// kernel (kf_bucket_reduce_avg, ranks in order — deterministic), then gathers
// the other shards from their owners with kf_gather_segments. On MI355X every
// GPU has a direct xGMI link to each of the 7 others, so both phases spread
// their reads over all links at once.
//
// Between the phases every rank must know that its peers are done. The host
// way (sync + dist.barrier) costs a round trip through the host and RCCL per
// phase; kf_peer_barrier does it on the device instead, in stream order: one
// workgroup stores the barrier's epoch into each peer's signal array over
// xGMI and spins on its own (fine-grained, uncached) array until every peer
// has arrived, with a wall-clock bound so that no wave can spin forever.
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "kungfu_amd.h"

namespace
{
thread_local std::string t_p2p_error;

int hip_fail(hipError_t e, const char *what)
{
    t_p2p_error = std::string(what) + ": " + hipGetErrorString(e);
    return KF_ERR_HIP;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Segs {
    const char *src[KF_MAX_SEGMENTS];
    size_t off[KF_MAX_SEGMENTS];
    size_t len[KF_MAX_SEGMENTS];  // bytes, multiple of 16
};

// 1-D grid, segment = blockIdx.x % nseg: consecutive blocks (dispatched
// together) pull from different peers, so every link is busy from the start
// instead of one peer's segment after another. Each block copies 4 x 16 B per
// thread per tile, non-temporal both ways (each byte moves once).
__global__ void __launch_bounds__(256) gather_kernel(char *dst, Segs segs, int nseg)
{
    const int s       = static_cast<int>(blockIdx.x % nseg);
    const size_t nvec = segs.len[s] / 16;
    const u32x4 *src  = reinterpret_cast<const u32x4 *>(segs.src[s] + segs.off[s]);
    u32x4 *out        = reinterpret_cast<u32x4 *>(dst + segs.off[s]);
    const size_t tile = 256 * 4;
    const size_t nblk = gridDim.x / nseg;  // blocks per segment
    for (size_t t = blockIdx.x / nseg; t * tile < nvec; t += nblk) {
        const size_t v0 = t * tile + threadIdx.x;
        u32x4 r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (v0 + u * 256 < nvec) r[u] = __builtin_nontemporal_load(src + v0 + u * 256);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (v0 + u * 256 < nvec) __builtin_nontemporal_store(r[u], out + v0 + u * 256);
        }
    }
}

// Per-segment source AND destination (the push exchange writes into peers'
// HBM over their links): same block interleave and tile as gather_kernel.
struct CopySegs {
    const char *src[KF_MAX_SEGMENTS];
    char *dst[KF_MAX_SEGMENTS];
    size_t len[KF_MAX_SEGMENTS];  // bytes, multiple of 16
};

__global__ void __launch_bounds__(256) copy_kernel(CopySegs segs, int nseg)
{
    const int s       = static_cast<int>(blockIdx.x % nseg);
    const size_t nvec = segs.len[s] / 16;
    const u32x4 *src  = reinterpret_cast<const u32x4 *>(segs.src[s]);
    u32x4 *out        = reinterpret_cast<u32x4 *>(segs.dst[s]);
    const size_t tile = 256 * 4;
    const size_t nblk = gridDim.x / nseg;
    for (size_t t = blockIdx.x / nseg; t * tile < nvec; t += nblk) {
        const size_t v0 = t * tile + threadIdx.x;
        u32x4 r[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (v0 + u * 256 < nvec) r[u] = __builtin_nontemporal_load(src + v0 + u * 256);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (v0 + u * 256 < nvec) __builtin_nontemporal_store(r[u], out + v0 + u * 256);
        }
    }
}

struct PeerSigs {
    unsigned long long *p[64];  // p[r]: rank r's signal array, as mapped here
};

// One 64-lane workgroup. Lane r (r != rank, r < world) first stores `epoch`
// into word `rank` of rank r's array (a posted write over xGMI), then waits
// for word r of this rank's own array to reach `epoch`. The release store at
// system scope orders it after every store of this kernel; the work queued
// before the barrier on this stream has already been released at its kernel
// end. The acquire loads bypass the caches (uncached memory, system scope).
// s_memrealtime ticks at the device's wall-clock rate; past `limit` ticks the
// lane stops and records KF_ERR_TIMEOUT in the host-visible status word.
__global__ void __launch_bounds__(64) peer_barrier_kernel(PeerSigs sigs, int world, int rank,
                                                          unsigned long long epoch,
                                                          unsigned long long limit,
                                                          unsigned long long *status)
{
    const int r = static_cast<int>(threadIdx.x);
    if (r >= world || r == rank) return;
    __hip_atomic_store(sigs.p[r] + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned long long *mine = sigs.p[rank] + r;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
        if (wall_clock64() - t0 > limit) {
            __hip_atomic_store(status, static_cast<unsigned long long>(KF_ERR_TIMEOUT),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

}  // namespace

extern "C" {

int kf_ipc_export(const void *dev_ptr, void *handle, size_t *offset)
{
    if (!dev_ptr || !handle || !offset) return KF_ERR_ARG;
    hipDeviceptr_t base = nullptr;
    size_t size         = 0;
    hipError_t e = hipMemGetAddressRange(&base, &size, const_cast<void *>(dev_ptr));
    if (e != hipSuccess) return hip_fail(e, "hipMemGetAddressRange");
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, base);
    if (e != hipSuccess) return hip_fail(e, "hipIpcGetMemHandle");
    static_assert(sizeof(hipIpcMemHandle_t) <= KF_IPC_HANDLE_BYTES, "handle size");
    std::memset(handle, 0, KF_IPC_HANDLE_BYTES);
    std::memcpy(handle, &h, sizeof(h));
    *offset = static_cast<size_t>(static_cast<const char *>(dev_ptr) -
                                  static_cast<const char *>(base));
    return KF_OK;
}

int kf_ipc_import(const void *handle, void **base_out)
{
    if (!handle || !base_out) return KF_ERR_ARG;
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    hipError_t e = hipIpcOpenMemHandle(base_out, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return hip_fail(e, "hipIpcOpenMemHandle");
    return KF_OK;
}

int kf_ipc_close(void *base)
{
    if (!base) return KF_ERR_ARG;
    hipError_t e = hipIpcCloseMemHandle(base);
    if (e != hipSuccess) return hip_fail(e, "hipIpcCloseMemHandle");
    return KF_OK;
}

int kf_gather_segments(void *dst, const void *const *srcs, const size_t *offsets,
                       const size_t *lens, int nseg, void *stream)
{
    if (nseg < 0 || nseg > KF_MAX_SEGMENTS) return KF_ERR_ARG;
    if (nseg == 0) return KF_OK;
    if (!dst || !srcs || !offsets || !lens) return KF_ERR_ARG;
    Segs segs;
    size_t maxlen = 0;
    for (int i = 0; i < nseg; ++i) {
        if (!srcs[i] || (lens[i] % 16) || (offsets[i] % 16) ||
            (reinterpret_cast<uintptr_t>(srcs[i]) % 16) ||
            (reinterpret_cast<uintptr_t>(dst) % 16)) {
            t_p2p_error = "kf_gather_segments: segments must be 16-byte aligned";
            return KF_ERR_ARG;
        }
        segs.src[i] = static_cast<const char *>(srcs[i]);
        segs.off[i] = offsets[i];
        segs.len[i] = lens[i];
        if (lens[i] > maxlen) maxlen = lens[i];
    }
    const size_t tile   = 256 * 4 * 16;
    size_t bx           = (maxlen + tile - 1) / tile;  // blocks per segment
    if (bx > (size_t(1) << 16)) bx = size_t(1) << 16;
    if (bx < 1) bx = 1;
    gather_kernel<<<static_cast<unsigned>(bx * nseg), 256, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<char *>(dst), segs, nseg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "gather_kernel launch");
    return KF_OK;
}

int kf_copy_segments(void *const *dsts, const void *const *srcs, const size_t *lens, int nseg,
                     void *stream)
{
    if (nseg < 0 || nseg > KF_MAX_SEGMENTS) return KF_ERR_ARG;
    if (nseg == 0) return KF_OK;
    if (!dsts || !srcs || !lens) return KF_ERR_ARG;
    CopySegs segs;
    size_t maxlen = 0;
    for (int i = 0; i < nseg; ++i) {
        if (!srcs[i] || !dsts[i] || (lens[i] % 16) ||
            (reinterpret_cast<uintptr_t>(srcs[i]) % 16) ||
            (reinterpret_cast<uintptr_t>(dsts[i]) % 16)) {
            t_p2p_error = "kf_copy_segments: segments must be 16-byte aligned";
            return KF_ERR_ARG;
        }
        segs.src[i] = static_cast<const char *>(srcs[i]);
        segs.dst[i] = static_cast<char *>(dsts[i]);
        segs.len[i] = lens[i];
        if (lens[i] > maxlen) maxlen = lens[i];
    }
    if (maxlen == 0) return KF_OK;
    const size_t tile = 256 * 4 * 16;
    size_t bx         = (maxlen + tile - 1) / tile;  // blocks per segment
    if (bx > (size_t(1) << 16)) bx = size_t(1) << 16;
    copy_kernel<<<static_cast<unsigned>(bx * nseg), 256, 0, static_cast<hipStream_t>(stream)>>>(
        segs, nseg);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "copy_kernel launch");
    return KF_OK;
}

int kf_signal_alloc(size_t nwords, int host, void **ptr)
{
    if (!ptr || nwords == 0) return KF_ERR_ARG;
    *ptr            = nullptr;
    const size_t sz = nwords * sizeof(unsigned long long);
    hipError_t e;
    if (host) {
        e = hipHostMalloc(ptr, sz, hipHostMallocMapped | hipHostMallocCoherent);
        if (e != hipSuccess) return hip_fail(e, "hipHostMalloc(signal)");
        std::memset(*ptr, 0, sz);
        return KF_OK;
    }
    // uncached fine-grained device memory: peers' stores land in HBM, the
    // spinning loads never hit a stale cache line
    e = hipExtMallocWithFlags(ptr, sz, hipDeviceMallocUncached);
    if (e != hipSuccess) return hip_fail(e, "hipExtMallocWithFlags(uncached signal)");
    e = hipMemset(*ptr, 0, sz);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        (void)hipFree(*ptr);
        *ptr = nullptr;
        return hip_fail(e, "hipMemset(signal)");
    }
    return KF_OK;
}

int kf_signal_free(void *ptr, int host)
{
    if (!ptr) return KF_ERR_ARG;
    hipError_t e = host ? hipHostFree(ptr) : hipFree(ptr);
    if (e != hipSuccess) return hip_fail(e, "signal free");
    return KF_OK;
}

int kf_peer_barrier(void *const *sigs, int world, int rank, uint64_t epoch, uint32_t timeout_us,
                    void *status, void *stream)
{
    if (!sigs || !status || world < 1 || world > 64 || rank < 0 || rank >= world) {
        t_p2p_error = "kf_peer_barrier: bad arguments";
        return KF_ERR_ARG;
    }
    if (world == 1) return KF_OK;
    PeerSigs ps;
    for (int r = 0; r < world; ++r) {
        if (!sigs[r] || (reinterpret_cast<uintptr_t>(sigs[r]) % 8)) {
            t_p2p_error = "kf_peer_barrier: signal arrays must be non-null, 8-byte aligned";
            return KF_ERR_ARG;
        }
        ps.p[r] = static_cast<unsigned long long *>(sigs[r]);
    }
    static thread_local int khz = 0;  // wall-clock rate, kHz (100 MHz on MI355X)
    if (khz == 0) {
        int dev      = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev);
        if (e != hipSuccess) return hip_fail(e, "hipDeviceAttributeWallClockRate");
        if (khz <= 0) khz = 100000;
    }
    const unsigned long long limit =
        static_cast<unsigned long long>(timeout_us) * static_cast<unsigned long long>(khz) / 1000;
    peer_barrier_kernel<<<1, 64, 0, static_cast<hipStream_t>(stream)>>>(
        ps, world, rank, static_cast<unsigned long long>(epoch), limit,
        static_cast<unsigned long long *>(status));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "peer_barrier_kernel launch");
    return KF_OK;
}

const char *kf_p2p_last_error(void) { return t_p2p_error.c_str(); }

}  // extern "C"
