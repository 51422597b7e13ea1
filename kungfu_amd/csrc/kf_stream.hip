// kf_stream.hip — one kernel per chunk that folds or copies the chunk while
// the socket still delivers it (kf_stream.hpp has the why). Library-internal.
//
// Every data block owns 4 KiB of the chunk (256 lanes x 16 B). One extra
// block, the watcher (block 0, dispatched first), is the only reader of the
// host's page-locked `landed` word: relaxed system-scope loads, s_sleep
// between polls, a system acquire fence whenever the count moves, then the
// count is re-published in HBM (an agent-scope release store of epoch:bytes
// into a device word). The data blocks poll that device word (agent-scope
// loads, served by the L2s: no PCIe reads) and then fold (SUM, the dtype's
// own arithmetic: kf_reduce_kernels.hpp Elt<T>) or copy their bytes, reading
// the landing slot system-coherent (sc0 sc1 buffer loads: from memory, past
// every GPU cache) and writing a page-locked output through the L2 (sc0 sc1), so
// no block takes an L2-wide fence. A block whose output a sender reads
// (`mark`) drains its stores (every wave's vmcnt(0), the barrier) and its
// first lane stores the block's done flag: one word per block, no atomics on
// host memory. The host sender spins on those flags and writes every piece
// once all its blocks are flagged. A deadline (wall clock) and the host's
// abort word end every wait. kf_stream.hpp and DESIGN.md §4 have the
// measurements behind each of these choices. Bits: element-wise, so those of
// one whole-chunk launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <immintrin.h>

#include "kf_reduce_kernels.hpp"
#include "kf_stream.hpp"

#ifndef KF_STREAM_HOST_STORE_AUX
// sc0 sc1: system scope, the policy the memory model gives for stores another
// agent (the host) reads without a release fence. r04 shipped sc1 alone
// (agent scope), which wrote through on the boxes measured but is not what
// the model promises; the flag after vmcnt(0) relies on it.
#define KF_STREAM_HOST_STORE_AUX 17
#endif

namespace kf_stream
{
namespace
{
constexpr int kLanes = 256;
constexpr uint32_t kSeen = 4096;     // device words for the watchers' counts (per board)
constexpr uint32_t kGaveUp = 1u << 31;  // in a count: the watcher stopped waiting

__device__ __forceinline__ unsigned long long seen_word(uint32_t epoch, uint32_t v)
{
    return (static_cast<unsigned long long>(epoch) << 32) | v;
}

// block 0's first lane: the host's count, re-published in HBM as it moves
__device__ void watch(Ctl *c, uint32_t len, unsigned long long *seen, uint32_t epoch,
                      unsigned long long limit)
{
    const unsigned long long t0 = wall_clock64();
    uint32_t last = 0;
    for (;;) {
        const uint32_t l = __hip_atomic_load(&c->landed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (l != last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            last = min(l, len);
            __hip_atomic_store(seen, seen_word(epoch, last), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            if (last >= len) return;
        } else if (__hip_atomic_load(&c->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0 ||
                   wall_clock64() - t0 > limit) {
            __hip_atomic_store(&c->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(seen, seen_word(epoch, kGaveUp), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// a data block's first lane: until the watcher's count covers `need`
__device__ int wait_seen(Ctl *c, const unsigned long long *seen, uint32_t epoch, uint32_t need,
                         unsigned long long limit)
{
    const unsigned long long t0 = wall_clock64();
    for (;;) {
        const unsigned long long v = __hip_atomic_load(seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (static_cast<uint32_t>(v >> 32) == epoch) {
            const uint32_t n = static_cast<uint32_t>(v);
            if (n & kGaveUp) return 0;
            if (n >= need) return 1;
        }
        if (wall_clock64() - t0 > limit) {  // the watcher never ran, or never finished
            __hip_atomic_store(&c->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return 0;
        }
        __builtin_amdgcn_s_sleep(20);  // ~1300 cycles: 257 pollers stay off the L2
    }
}

// block 0 watches (returns false); a data block waits for its bytes (its
// first lane polls, the block meets at a barrier)
__device__ __forceinline__ bool block_wait(Ctl *c, uint32_t len, uint32_t need,
                                           unsigned long long *seen, uint32_t epoch,
                                           unsigned long long limit, bool *ok)
{
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) watch(c, len, seen, epoch, limit);
        return false;
    }
    __shared__ int got;
    if (threadIdx.x == 0) got = wait_seen(c, seen, epoch, need, limit + limit / 8);
    __syncthreads();
    *ok = got != 0;
    return true;
}

// Page-locked bytes move with an explicit cache policy instead of fences:
// the landing slot is read system-coherent (sc0 sc1: from memory, past every
// GPU cache, so no acquire fence per block), and a page-locked output is
// written through at system scope (kHostStore) so that once the block's stores have drained
// (vmcnt(0)) they are in host memory and one flag store publishes them — no
// L2 writeback per block. Per-block system fences cost a write-back and an
// invalidate of the whole XCD L2 each: 257 of them per chunk held every
// chunk's last piece 65-240 us past its last byte in C1.
using v4u = __attribute__((ext_vector_type(4))) unsigned;
constexpr int kHostLoad  = 17;  // sc0 sc1
constexpr int kHostStore = KF_STREAM_HOST_STORE_AUX;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, bytes, 0x00020000);
}

// 16 bytes (n of them at the end) of page-locked memory at base + off
__device__ __forceinline__ void load16_host(__amdgpu_buffer_rsrc_t r, const char *base, uint32_t off,
                                            uint32_t n, unsigned char *buf)
{
    if (n == 16 && ((reinterpret_cast<uintptr_t>(base) + off) & 15) == 0) {
        const v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kHostLoad);
        std::memcpy(buf, &v, 16);
    } else {
        for (uint32_t i = 0; i < n; ++i) buf[i] = __builtin_amdgcn_raw_buffer_load_b8(r, off + i, 0, kHostLoad);
    }
}

__device__ __forceinline__ void store16_host(__amdgpu_buffer_rsrc_t r, const char *base, uint32_t off,
                                             uint32_t n, const unsigned char *buf)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(base) + off;
    if (n == 16 && (a & 15) == 0) {
        v4u v;
        std::memcpy(&v, buf, 16);
        __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kHostStore);
    } else if (n % 4 == 0 && (a & 3) == 0) {
        for (uint32_t i = 0; i < n; i += 4) {
            uint32_t w;
            std::memcpy(&w, buf + i, 4);
            __builtin_amdgcn_raw_buffer_store_b32(w, r, off + i, 0, kHostStore);
        }
    } else {
        for (uint32_t i = 0; i < n; ++i) __builtin_amdgcn_raw_buffer_store_b8(buf[i], r, off + i, 0, kHostStore);
    }
}

// this block's written-through stores have drained: flag it for the sender
__device__ __forceinline__ void block_done(Ctl *c, uint32_t b)
{
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __hip_atomic_store(&c->done[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// 16 bytes of a lane from `src + off` in HBM (any alignment)
__device__ __forceinline__ void load16(const char *src, uint32_t n, unsigned char *buf)
{
    if (n == 16 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
        *reinterpret_cast<uint4 *>(buf) = *reinterpret_cast<const uint4 *>(src);
    } else {
        for (uint32_t i = 0; i < n; ++i) buf[i] = static_cast<unsigned char>(src[i]);
    }
}

__device__ __forceinline__ void store16(char *dst, uint32_t n, const unsigned char *buf)
{
    if (n == 16 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        *reinterpret_cast<uint4 *>(dst) = *reinterpret_cast<const uint4 *>(buf);
    } else if (n % 4 == 0 && (reinterpret_cast<uintptr_t>(dst) & 3) == 0) {
        for (uint32_t i = 0; i < n; i += 4) {
            *reinterpret_cast<uint32_t *>(dst + i) = *reinterpret_cast<const uint32_t *>(buf + i);
        }
    } else {
        for (uint32_t i = 0; i < n; ++i) dst[i] = static_cast<char>(buf[i]);
    }
}

// out = own + landed body, element by element, as each 4 KiB lands; `mark`:
// out is page-locked (written through, flagged), otherwise HBM
template <typename T>
__global__ void __launch_bounds__(kLanes)
    fold_kernel(const typename kf::Elt<T>::S *own, const char *landing,
                typename kf::Elt<T>::S *out, uint32_t len, int mark, Ctl *c,
                unsigned long long *seen, uint32_t epoch, unsigned long long limit)
{
    using S              = typename kf::Elt<T>::S;
    const uint32_t b     = blockIdx.x - 1;
    const uint32_t start = b * kBlockBytes;
    const uint32_t end   = min(start + kBlockBytes, len);
    bool ok              = false;
    if (!block_wait(c, len, end, seen, epoch, limit, &ok)) return;
    const uint32_t off = start + threadIdx.x * 16;
    if (ok && off < end) {
        const uint32_t nb = min(16u, end - off);
        alignas(16) unsigned char buf[16];
        load16_host(rsrc(landing, len), landing, off, nb, buf);
        S peer[16 / sizeof(S)], res[16 / sizeof(S)];
        std::memcpy(peer, buf, sizeof(peer));
        const size_t e0 = off / sizeof(S);
        for (uint32_t j = 0; j < nb / sizeof(S); ++j) {
            res[j] = kf::finish<T, kf::OP_SUM>(
                kf::Elt<T>::template combine<kf::OP_SUM>(kf::Elt<T>::load(own[e0 + j]), peer[j]));
        }
        std::memcpy(buf, res, sizeof(res));
        char *o = reinterpret_cast<char *>(out);
        if (mark) {
            store16_host(rsrc(o, len), o, off, nb, buf);
        } else {
            store16(o + off, nb, buf);
        }
    }
    if (mark && ok) block_done(c, b);  // a block that gave up is never final
}

// dst (HBM) = landed body, as each 4 KiB lands
__global__ void __launch_bounds__(kLanes)
    copy_in_kernel(const char *landing, char *dst, uint32_t len, Ctl *c, unsigned long long *seen,
                   uint32_t epoch, unsigned long long limit)
{
    const uint32_t b     = blockIdx.x - 1;
    const uint32_t start = b * kBlockBytes;
    const uint32_t end   = min(start + kBlockBytes, len);
    bool ok              = false;
    if (!block_wait(c, len, end, seen, epoch, limit, &ok)) return;
    const uint32_t off = start + threadIdx.x * 16;
    if (ok && off < end) {
        const uint32_t nb = min(16u, end - off);
        alignas(16) unsigned char buf[16];
        load16_host(rsrc(landing, len), landing, off, nb, buf);
        store16(dst + off, nb, buf);
    }
}

// host (page-locked, written through) = src (HBM), each block flagged
__global__ void __launch_bounds__(kLanes)
    copy_out_kernel(const char *src, char *host, uint32_t len, Ctl *c)
{
    const uint32_t off = blockIdx.x * kBlockBytes + threadIdx.x * 16;
    const uint32_t end = min(blockIdx.x * kBlockBytes + kBlockBytes, len);
    if (off < end) {
        const uint32_t nb = min(16u, end - off);
        alignas(16) unsigned char buf[16];
        load16(src + off, nb, buf);
        store16_host(rsrc(host, len), host, off, nb, buf);
    }
    block_done(c, blockIdx.x);
}

// dst = src, 16 B per lane, one 4 KiB block per block of the grid
__global__ void __launch_bounds__(kLanes) copy_kernel(char *dst, const char *src, size_t len)
{
    const size_t start = static_cast<size_t>(blockIdx.x) * kBlockBytes;
    const size_t off   = start + threadIdx.x * 16;
    if (off < len) {
        const uint32_t nb = static_cast<uint32_t>(min(static_cast<size_t>(16), len - off));
        alignas(16) unsigned char buf[16];
        load16(src + off, nb, buf);
        store16(dst + off, nb, buf);
    }
}

unsigned long long ticks(int ms)
{
    static const int khz = [] {
        int dev = 0, v = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) != hipSuccess || v <= 0) {
            v = 100000;  // 100 MHz on MI355X
        }
        return v;
    }();
    return static_cast<unsigned long long>(std::max(ms, 1)) * static_cast<unsigned long long>(khz);
}

unsigned blocks(uint32_t len) { return (len + kBlockBytes - 1) / kBlockBytes; }



// a device word and an epoch for one launch's watcher
struct Seen {
    unsigned long long *word;
    uint32_t epoch;
};
}  // namespace

// The watchers' words live in HBM the session allocated (hipMalloc) on the
// thread that created it, before its other threads start: no module-scope
// __device__ variable, so nothing is resolved lazily under a second thread's
// launch (r04: a first-use hipGetSymbolAddress of one aborted a rank in the
// HIP runtime, profiles/r05/failures.md).
struct Board {
    unsigned long long *words = nullptr;
    int device                = 0;
    std::atomic<unsigned long long> launches{0};
};

namespace
{
Seen next_seen(Board *b)
{
    if (!b || !b->words) return Seen{nullptr, 0};
    const unsigned long long n = b->launches.fetch_add(1, std::memory_order_relaxed);
    // a word is reused kSeen launches later; the epoch tells its owners apart
    // (epoch 0 is the zeroed word's: never a launch's)
    return Seen{b->words + n % kSeen, static_cast<uint32_t>(n % 0xffffffffu) + 1};
}

template <typename T>
int fold_as(const void *own, const void *landing, void *out, uint32_t len, int mark, Ctl *c,
            Board *board, unsigned long long limit, hipStream_t s)
{
    using S = typename kf::Elt<T>::S;
    if (len % sizeof(S)) return KF_ERR_ARG;
    const Seen w = next_seen(board);
    if (!w.word) return KF_ERR_HIP;
    (void)hipGetLastError();  // the check below is about this launch only
    fold_kernel<T><<<blocks(len) + 1, kLanes, 0, s>>>(
        static_cast<const S *>(own), static_cast<const char *>(landing), static_cast<S *>(out), len,
        mark, c, w.word, w.epoch, limit);
    return hipGetLastError() == hipSuccess ? KF_OK : KF_ERR_HIP;
}

bool fits(uint32_t len, uint32_t piece)
{
    return piece >= kBlockBytes && piece % kBlockBytes == 0 && blocks(len) <= kMaxBlocks;
}
}  // namespace

bool supported(KungFu_Datatype dt, KungFu_Op op)
{
    if (op != KungFu_SUM) return false;
    switch (dt) {
    case KungFu_UINT8: case KungFu_UINT16: case KungFu_UINT32: case KungFu_UINT64:
    case KungFu_INT8: case KungFu_INT16: case KungFu_INT32: case KungFu_INT64:
    case KungFu_FLOAT16: case KungFu_FLOAT: case KungFu_DOUBLE: case KungFu_BFLOAT16: return true;
    default: return false;
    }
}

void reset(Ctl *c, uint32_t piece)
{
    std::memset(c, 0, sizeof(*c));
    c->bpp = piece / kBlockBytes;
    std::atomic_thread_fence(std::memory_order_release);
}

void publish(Ctl *c, uint32_t bytes) { __atomic_store_n(&c->landed, bytes, __ATOMIC_RELEASE); }

void abort_wait(Ctl *c) { __atomic_store_n(&c->abort, 1u, __ATOMIC_RELEASE); }

int launch_fold(KungFu_Datatype dt, const void *own, const void *landing_dev, void *out,
                uint32_t len, uint32_t piece, Ctl *c_dev, Board *board, int deadline_ms, bool mark,
                void *stream)
{
    if (len == 0) return KF_OK;
    if (!fits(len, piece)) return KF_ERR_ARG;
    const unsigned long long lim = ticks(deadline_ms);
    hipStream_t s                = static_cast<hipStream_t>(stream);
    const int m                  = mark ? 1 : 0;
    switch (dt) {
    case KungFu_UINT8: return fold_as<uint8_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_UINT16: return fold_as<uint16_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_UINT32: return fold_as<uint32_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_UINT64: return fold_as<uint64_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_INT8: return fold_as<int8_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_INT16: return fold_as<int16_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_INT32: return fold_as<int32_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_INT64: return fold_as<int64_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_FLOAT16: return fold_as<kf::f16_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_FLOAT: return fold_as<float>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_DOUBLE: return fold_as<double>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    case KungFu_BFLOAT16: return fold_as<kf::bf16_t>(own, landing_dev, out, len, m, c_dev, board, lim, s);
    default: return KF_ERR_DTYPE;
    }
}

int launch_copy_in(const void *landing_dev, void *dst, uint32_t len, uint32_t piece, Ctl *c_dev,
                   Board *board, int deadline_ms, void *stream)
{
    if (len == 0) return KF_OK;
    if (!fits(len, piece)) return KF_ERR_ARG;
    const Seen w = next_seen(board);
    if (!w.word) return KF_ERR_HIP;
    (void)hipGetLastError();
    copy_in_kernel<<<blocks(len) + 1, kLanes, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const char *>(landing_dev), static_cast<char *>(dst), len, c_dev, w.word,
        w.epoch, ticks(deadline_ms));
    return hipGetLastError() == hipSuccess ? KF_OK : KF_ERR_HIP;
}

int launch_copy_out(const void *src, void *host_dev, uint32_t len, uint32_t piece, Ctl *c_dev,
                    void *stream)
{
    if (len == 0) return KF_OK;
    if (!fits(len, piece)) return KF_ERR_ARG;
    (void)hipGetLastError();
    copy_out_kernel<<<blocks(len), kLanes, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const char *>(src), static_cast<char *>(host_dev), len, c_dev);
    return hipGetLastError() == hipSuccess ? KF_OK : KF_ERR_HIP;
}

namespace
{
// Every kernel of this file resolved on the calling thread (its code object
// loaded for the current device), so the session's threads only launch.
template <typename T>
bool warm_fold()
{
    hipFuncAttributes a;
    return hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&fold_kernel<T>)) == hipSuccess;
}
}  // namespace

Board *board_create()
{
    auto *b = new Board;
    hipFuncAttributes a;
    const bool warm =
        warm_fold<uint8_t>() && warm_fold<uint16_t>() && warm_fold<uint32_t>() &&
        warm_fold<uint64_t>() && warm_fold<int8_t>() && warm_fold<int16_t>() &&
        warm_fold<int32_t>() && warm_fold<int64_t>() && warm_fold<kf::f16_t>() &&
        warm_fold<float>() && warm_fold<double>() && warm_fold<kf::bf16_t>() &&
        hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&copy_in_kernel)) == hipSuccess &&
        hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&copy_out_kernel)) == hipSuccess &&
        hipFuncGetAttributes(&a, reinterpret_cast<const void *>(&copy_kernel)) == hipSuccess;
    // zeroed on a stream of its own: the null stream (torch's default) may
    // hold another session's streamed kernel that waits for bytes this
    // thread has yet to send (sessions created in threads of one process)
    const size_t bytes = kSeen * sizeof(unsigned long long);
    hipStream_t st     = nullptr;
    const bool ok = warm && hipGetDevice(&b->device) == hipSuccess &&
                    hipMalloc(reinterpret_cast<void **>(&b->words), bytes) == hipSuccess &&
                    hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
                    hipMemsetAsync(b->words, 0, bytes, st) == hipSuccess &&
                    hipStreamSynchronize(st) == hipSuccess;
    if (st) (void)hipStreamDestroy(st);
    if (!ok) {
        board_destroy(b);
        return nullptr;
    }
    return b;
}

void board_destroy(Board *b)
{
    if (!b) return;
    if (b->words) (void)hipFree(b->words);
    delete b;
}

bool copy_kernels()
{
    static const bool on = [] {
        const char *e = std::getenv("KUNGFU_AMD_COPY_KERNEL");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

int launch_copy(void *dst, const void *src, size_t len, void *stream)
{
    if (len == 0) return KF_OK;
    const size_t nblk = (len + kBlockBytes - 1) / kBlockBytes;
    if (nblk > 0x7fffffffu) return KF_ERR_ARG;
    (void)hipGetLastError();
    copy_kernel<<<static_cast<unsigned>(nblk), kLanes, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<char *>(dst), static_cast<const char *>(src), len);
    return hipGetLastError() == hipSuccess ? KF_OK : KF_ERR_HIP;
}

namespace
{
// the blocks of piece k are all flagged
bool piece_done(const Ctl *c, uint32_t k, uint32_t nb)
{
    const uint32_t b0 = k * c->bpp, b1 = std::min(b0 + c->bpp, nb);
    for (uint32_t b = b0; b < b1; ++b) {
        if (!__atomic_load_n(&c->done[b], __ATOMIC_ACQUIRE)) return false;
    }
    return true;
}
}  // namespace

int wait_piece(const Ctl *c, uint32_t k, uint32_t len, int timeout_ms)
{
    const uint32_t nb = blocks(len);
    const auto t0     = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
        if (piece_done(c, k, nb)) return KF_OK;
        // a block that gave up never flags its piece: the word says so at once
        if (__atomic_load_n(&c->err, __ATOMIC_ACQUIRE)) return KF_ERR_HIP;
        if ((spin & 1023) == 1023) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) {
                return KF_ERR_TIMEOUT;
            }
        }
        _mm_pause();
    }
}

uint32_t ready_run(const Ctl *c, uint32_t k, uint32_t len)
{
    const uint32_t nb = blocks(len);
    const uint32_t np = (nb + c->bpp - 1) / c->bpp;
    uint32_t j        = k;
    while (j < np && piece_done(c, j, nb)) ++j;
    return j - k;
}
}  // namespace kf_stream

namespace kf_sync
{
namespace
{
bool blocking()
{
    static const bool b = [] {
        const char *e = std::getenv("KUNGFU_AMD_BLOCKING_SYNC");
        return e && std::atoi(e) != 0;
    }();
    return b;
}
}  // namespace

unsigned event_flags()
{
    return hipEventDisableTiming | (blocking() ? hipEventBlockingSync : 0u);
}

int stream_sync(void *stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!blocking()) return hipStreamSynchronize(s) == hipSuccess ? KF_OK : KF_ERR_HIP;
    hipEvent_t e = nullptr;  // a blocking event behind the stream's work: the thread sleeps
    const bool ok = hipEventCreateWithFlags(&e, event_flags()) == hipSuccess &&
                    hipEventRecord(e, s) == hipSuccess && hipEventSynchronize(e) == hipSuccess;
    if (e) (void)hipEventDestroy(e);
    return ok ? KF_OK : KF_ERR_HIP;
}
}  // namespace kf_sync
