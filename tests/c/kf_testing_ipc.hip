// kf_testing_ipc.hip — the cross-process "ipc" test transport
// (tests/c/kf_testing.h): `world` PROCESSES on one device, each with its own
// exchange, the exchange's collectives moved through HIP-IPC-mapped staging
// buffers and rendezvous words in a POSIX shared-memory segment. This lets
// bench.py's N > 1 branch (ranks started by torch.distributed.run, one per
// process) run the native exchange with N ranks on one GPU, where RCCL refuses
// two ranks per device. Test infrastructure: nothing in kungfu_amd/ links or
// loads it, and it makes no performance claim (host rendezvous per call).
//
// Every collective call is synchronous and runs the same steps on every rank:
//   1. the rank's staging buffer grows if this call's input does not fit (the
//      size is the same on every rank, so they all grow together: allocate,
//      export the IPC handle into the segment, rendezvous, import the peers');
//   2. the input is copied into the rank's own staging buffer, stream synced;
//   3. rendezvous A: every rank's input is staged;
//   4. the rank pulls what it receives from the peers' staging buffers into
//      its own output (copies, or the rank-order fold kernel below for the
//      reduce-scatter), stream synced;
//   5. rendezvous B: nobody reads a staging buffer any more.
// A rank that fails, or a rendezvous that times out, marks the segment broken:
// every rank's pending and later calls then fail instead of waiting.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cerrno>
#include <cstring>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "kf_testing.h"

#pragma clang fp contract(off)

namespace
{
thread_local std::string t_err;

constexpr int kMaxRanks = 16;
constexpr int kHandleBytes = 64;
static_assert(sizeof(hipIpcMemHandle_t) <= kHandleBytes, "IPC handle size");

enum {
    IPC_OK      = 0,
    IPC_HIP     = 1,
    IPC_DTYPE   = 2,
    IPC_ARG     = 3,
    IPC_TIMEOUT = 4,
    IPC_BROKEN  = 5,
    IPC_SHM     = 6,
};

struct Slot {
    char handle[kHandleBytes];  // this rank's staging buffer
    uint64_t cap;
    int32_t color, key;  // split
    // the call this rank is in (checked by every rank after rendezvous A: a
    // rank whose call differs is a caller bug, failed loudly instead of
    // moving mismatched bytes)
    uint64_t seq, bytes;
    int32_t kind, root;
    int32_t grow_ok[2];  // this rank's export / import of a growth attempt
};

struct Seg {
    std::atomic<uint64_t> arrive;
    std::atomic<uint64_t> gen;
    std::atomic<int32_t> broken;
    int32_t world;
    Slot slot[kMaxRanks];
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "process-shared atomics");

struct IpcComm {
    std::string name;
    Seg *seg       = nullptr;
    int rank       = 0;
    int world      = 1;
    int device     = 0;
    int timeout_ms = 120000;
    void *stage    = nullptr;
    size_t cap     = 0;
    std::vector<void *> peer;  // every rank's staging buffer as mapped here
    uint64_t nsplit = 0;
    uint64_t ncalls = 0;
};

Seg *map_segment(const std::string &name)
{
    const int fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
    if (fd < 0) return nullptr;
    // zero-filled on creation; every member truncates to the same size
    if (ftruncate(fd, sizeof(Seg)) != 0) {
        close(fd);
        return nullptr;
    }
    void *p = mmap(nullptr, sizeof(Seg), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    return p == MAP_FAILED ? nullptr : static_cast<Seg *>(p);
}

int fail(IpcComm *c, int code, const std::string &what)
{
    t_err = what;
    if (c && c->seg) c->seg->broken.store(1, std::memory_order_release);
    return code;
}

int hip_fail(IpcComm *c, hipError_t e, const char *what)
{
    return fail(c, IPC_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// centralised barrier: the last arrival resets the count, then advances the
// generation the others wait on
int barrier(IpcComm *c)
{
    Seg *s = c->seg;
    if (s->broken.load(std::memory_order_acquire)) return IPC_BROKEN;
    const uint64_t g = s->gen.load(std::memory_order_acquire);
    if (s->arrive.fetch_add(1, std::memory_order_acq_rel) + 1 == static_cast<uint64_t>(c->world)) {
        s->arrive.store(0, std::memory_order_relaxed);
        s->gen.fetch_add(1, std::memory_order_release);
        return IPC_OK;
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned i = 0;; ++i) {
        if (s->gen.load(std::memory_order_acquire) != g) return IPC_OK;
        if (s->broken.load(std::memory_order_acquire)) return IPC_BROKEN;
        if (i < 2000) {
            sched_yield();
            continue;
        }
        struct timespec ts = {0, 20000};
        nanosleep(&ts, nullptr);
        if ((i & 255) == 0 && std::chrono::steady_clock::now() - t0 >
                                  std::chrono::milliseconds(c->timeout_ms)) {
            return fail(c, IPC_TIMEOUT, "ipc transport: rendezvous timed out");
        }
    }
}

void drop_peers(IpcComm *c)
{
    for (int j = 0; j < c->world; ++j) {
        if (j != c->rank && c->peer[j]) (void)hipIpcCloseMemHandle(c->peer[j]);
        c->peer[j] = nullptr;
    }
}

// this rank's half of one growth attempt: a fresh staging buffer of `cap`
// bytes, exported into its slot; false with *why on failure
bool stage_export(IpcComm *c, size_t cap, std::string *why)
{
    drop_peers(c);
    if (c->stage) (void)hipFree(c->stage);
    c->stage = nullptr;
    c->cap   = 0;
    hipError_t e = hipMalloc(&c->stage, cap);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        c->stage = nullptr;
        *why     = std::string("hipMalloc of the staging buffer: ") + hipGetErrorString(e);
        return false;
    }
    void *base  = nullptr;
    size_t span = 0;
    e           = hipMemGetAddressRange(&base, &span, c->stage);
    if (e != hipSuccess || base != c->stage) {
        (void)hipGetLastError();
        *why = "the staging buffer is not the base of its allocation";
        return false;
    }
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, c->stage);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        *why = std::string("hipIpcGetMemHandle of the staging buffer: ") + hipGetErrorString(e);
        return false;
    }
    std::memcpy(c->seg->slot[c->rank].handle, &h, sizeof(h));
    c->seg->slot[c->rank].cap = cap;
    c->cap                    = cap;
    return true;
}

// the other half: map every peer's exported buffer
bool stage_import(IpcComm *c, size_t cap, std::string *why)
{
    c->peer[c->rank] = c->stage;
    for (int j = 0; j < c->world; ++j) {
        if (j == c->rank) continue;
        if (c->seg->slot[j].cap != cap) {
            *why = "ranks disagree on a size";
            return false;
        }
        hipIpcMemHandle_t ph;
        std::memcpy(&ph, c->seg->slot[j].handle, sizeof(ph));
        hipError_t e = hipIpcOpenMemHandle(&c->peer[j], ph, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            c->peer[j] = nullptr;
            *why = std::string("hipIpcOpenMemHandle of rank ") + std::to_string(j) +
                   "'s staging: " + hipGetErrorString(e);
            return false;
        }
    }
    return true;
}

bool all_ok(IpcComm *c, int which)
{
    for (int j = 0; j < c->world; ++j) {
        if (!c->seg->slot[j].grow_ok[which]) return false;
    }
    return true;
}

// Every rank calls with the same `need` (the collectives are symmetric), so
// they grow together, and every rank takes the same decision from the flags
// all of them post: an export or import refused on any rank (seen now and
// then with 4 and 8 processes on one GPU, r06d and r06zz) makes every rank
// drop the attempt and try again with fresh buffers, up to four times. At
// least 64 MiB: a smaller hipMalloc may be carved out of a shared block, and
// exporting such a piece was refused (r06d); the buffer must be the whole
// allocation its handle describes.
int ensure(IpcComm *c, size_t need)
{
    if (need <= c->cap) return IPC_OK;
    size_t cap = size_t(64) << 20;
    while (cap < need) cap <<= 1;
    std::string why;
    for (int attempt = 0;; ++attempt) {
        Slot &me      = c->seg->slot[c->rank];
        me.grow_ok[0] = stage_export(c, cap, &why) ? 1 : 0;
        int rc        = barrier(c);
        if (rc != IPC_OK) return rc;
        bool ok       = all_ok(c, 0);
        me.grow_ok[1] = ok && stage_import(c, cap, &why) ? 1 : 0;
        if ((rc = barrier(c)) != IPC_OK) return rc;
        ok = all_ok(c, 1);
        // the flags and handles are read before any rank rewrites them
        if ((rc = barrier(c)) != IPC_OK) return rc;
        if (ok) return IPC_OK;
        if (attempt == 3) {
            return fail(c, IPC_HIP, "ipc transport: staging buffers not shared after 4 attempts" +
                                        (why.empty() ? std::string() : " (this rank: " + why + ")"));
        }
        struct timespec ts = {0, 5000000};
        nanosleep(&ts, nullptr);
    }
}

enum { K_RS = 1, K_AG = 2, K_A2A = 3, K_BC = 4 };

template <typename Pull>
int collective(void *comm, int kind, int root, const void *send, size_t in_bytes, bool stage_mine,
               void *stream, Pull pull)
{
    auto *c        = static_cast<IpcComm *>(comm);
    hipStream_t st = static_cast<hipStream_t>(stream);
    t_err.clear();
    if (c->seg->broken.load(std::memory_order_acquire)) {
        t_err = "ipc transport: the group failed earlier";
        return IPC_BROKEN;
    }
    int rc = ensure(c, in_bytes);
    if (rc != IPC_OK) return rc;
    Slot &me = c->seg->slot[c->rank];
    me.seq   = c->ncalls++;
    me.bytes = in_bytes;
    me.kind  = kind;
    me.root  = root;
    if (stage_mine && in_bytes) {
        hipError_t e = hipMemcpyAsync(c->stage, send, in_bytes, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return hip_fail(c, e, "ipc transport: staging copy");
    }
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(c, e, "ipc transport: stream sync");
    if ((rc = barrier(c)) != IPC_OK) return rc;
    for (int j = 0; j < c->world; ++j) {
        const Slot &p = c->seg->slot[j];
        if (p.seq != me.seq || p.kind != kind || p.bytes != in_bytes || p.root != root) {
            return fail(c, IPC_ARG,
                        "ipc transport: rank " + std::to_string(j) + " is in call #" +
                            std::to_string(p.seq) + " (kind " + std::to_string(p.kind) + ", " +
                            std::to_string(p.bytes) + " B), rank " + std::to_string(c->rank) +
                            " in #" + std::to_string(me.seq) + " (kind " + std::to_string(kind) +
                            ", " + std::to_string(in_bytes) + " B)");
        }
    }
    if ((rc = pull(c, st)) != IPC_OK) return fail(c, rc, t_err.empty() ? "ipc transport: pull" : t_err);
    e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(c, e, "ipc transport: stream sync");
    return barrier(c);
}

size_t dsize(KungFu_Datatype dt)
{
    switch (dt) {
    case KungFu_UINT8: case KungFu_INT8: return 1;
    case KungFu_UINT16: case KungFu_INT16: case KungFu_FLOAT16: case KungFu_BFLOAT16: return 2;
    case KungFu_UINT32: case KungFu_INT32: case KungFu_FLOAT: return 4;
    default: return 8;
    }
}

// ---------------------------------------------------------------------------
// the reduce-scatter's fold: out[i] = in_0[off + i] op in_1[off + i] op ...,
// in rank order (integers wrap, MIN / MAX are std::min / std::max selects,
// AVG is ncclAvg's float form: every input premultiplied by 1 / k)
// ---------------------------------------------------------------------------
struct FoldIn {
    const void *p[kMaxRanks];
};

template <typename T> struct Wide {
    using U = T;
};
template <> struct Wide<int8_t> { using U = uint32_t; };
template <> struct Wide<uint8_t> { using U = uint32_t; };
template <> struct Wide<int32_t> { using U = uint32_t; };
template <> struct Wide<uint32_t> { using U = uint32_t; };
template <> struct Wide<int64_t> { using U = uint64_t; };
template <> struct Wide<uint64_t> { using U = uint64_t; };

template <typename T>
__device__ __forceinline__ T combine(T a, T b, int op)
{
    if constexpr (std::is_floating_point<T>::value) {
        if (op == KungFu_SUM || op == KF_TRANSPORT_OP_AVG) return a + b;
        if (op == KungFu_PROD) return a * b;
    } else {
        using U = typename Wide<T>::U;
        using M = typename std::make_unsigned<T>::type;
        if (op == KungFu_SUM) return static_cast<T>(static_cast<U>(static_cast<M>(a)) + static_cast<U>(static_cast<M>(b)));
        if (op == KungFu_PROD) return static_cast<T>(static_cast<U>(static_cast<M>(a)) * static_cast<U>(static_cast<M>(b)));
    }
    if (op == KungFu_MIN) return (b < a) ? b : a;
    return (a < b) ? b : a;
}

template <typename T>
__global__ void fold_kernel(FoldIn in, int k, size_t off, T *out, size_t n, int op)
{
    const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
    for (size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
        if constexpr (std::is_floating_point<T>::value) {
            if (op == KF_TRANSPORT_OP_AVG) {
                const T w = static_cast<T>(1) / static_cast<T>(k);
                T a       = static_cast<const T *>(in.p[0])[off + i] * w;
                for (int j = 1; j < k; ++j) a = a + static_cast<const T *>(in.p[j])[off + i] * w;
                out[i] = a;
                continue;
            }
        }
        T a = static_cast<const T *>(in.p[0])[off + i];
        for (int j = 1; j < k; ++j) a = combine<T>(a, static_cast<const T *>(in.p[j])[off + i], op);
        out[i] = a;
    }
}

template <typename T>
int launch_fold(const FoldIn &in, int k, size_t off, void *out, size_t n, int op, hipStream_t st)
{
    if (n == 0) return IPC_OK;
    size_t blocks = (n + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    fold_kernel<T><<<static_cast<unsigned>(blocks), 256, 0, st>>>(in, k, off, static_cast<T *>(out), n, op);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        t_err = std::string("ipc transport: fold launch: ") + hipGetErrorString(e);
        return IPC_HIP;
    }
    return IPC_OK;
}

int ipc_reduce_scatter(const void *send, void *recv, size_t count, KungFu_Datatype dt, KungFu_Op op,
                       void *comm, void *stream)
{
    auto *c      = static_cast<IpcComm *>(comm);
    const int o  = static_cast<int>(op);
    const bool fl = dt == KungFu_FLOAT || dt == KungFu_DOUBLE;
    if (dt == KungFu_FLOAT16 || dt == KungFu_BFLOAT16 || dt == KungFu_UINT16 || dt == KungFu_INT16 ||
        (o == KF_TRANSPORT_OP_AVG && !fl)) {
        t_err = "ipc transport: no reduce-scatter for this dtype / op";
        return IPC_DTYPE;  // refused before any rendezvous, on every rank alike
    }
    const size_t sz = dsize(dt);
    return collective(comm, K_RS, o, send, count * c->world * sz, true, stream,
                      [&](IpcComm *cc, hipStream_t st) {
        FoldIn in{};
        for (int j = 0; j < cc->world; ++j) in.p[j] = cc->peer[j];
        const size_t off = static_cast<size_t>(cc->rank) * count;
        switch (dt) {
        case KungFu_INT8: return launch_fold<int8_t>(in, cc->world, off, recv, count, o, st);
        case KungFu_UINT8: return launch_fold<uint8_t>(in, cc->world, off, recv, count, o, st);
        case KungFu_INT32: return launch_fold<int32_t>(in, cc->world, off, recv, count, o, st);
        case KungFu_UINT32: return launch_fold<uint32_t>(in, cc->world, off, recv, count, o, st);
        case KungFu_INT64: return launch_fold<int64_t>(in, cc->world, off, recv, count, o, st);
        case KungFu_UINT64: return launch_fold<uint64_t>(in, cc->world, off, recv, count, o, st);
        case KungFu_FLOAT: return launch_fold<float>(in, cc->world, off, recv, count, o, st);
        default: return launch_fold<double>(in, cc->world, off, recv, count, o, st);
        }
    });
}

int copy(void *dst, const void *src, size_t b, hipStream_t st)
{
    if (b == 0 || dst == src) return IPC_OK;
    hipError_t e = hipMemcpyAsync(dst, src, b, hipMemcpyDeviceToDevice, st);
    if (e != hipSuccess) {
        t_err = std::string("ipc transport: copy: ") + hipGetErrorString(e);
        return IPC_HIP;
    }
    return IPC_OK;
}

int ipc_all_gather(const void *send, void *recv, size_t b, void *comm, void *stream)
{
    return collective(comm, K_AG, 0, send, b, true, stream, [&](IpcComm *c, hipStream_t st) {
        for (int j = 0; j < c->world; ++j) {
            int rc = copy(static_cast<char *>(recv) + j * b, c->peer[j], b, st);
            if (rc != IPC_OK) return rc;
        }
        return int(IPC_OK);
    });
}

int ipc_all_to_all(const void *send, void *recv, size_t b, void *comm, void *stream)
{
    auto *c = static_cast<IpcComm *>(comm);
    return collective(comm, K_A2A, 0, send, b * c->world, true, stream,
                      [&](IpcComm *cc, hipStream_t st) {
        for (int j = 0; j < cc->world; ++j) {
            int rc = copy(static_cast<char *>(recv) + j * b,
                          static_cast<const char *>(cc->peer[j]) + cc->rank * b, b, st);
            if (rc != IPC_OK) return rc;
        }
        return int(IPC_OK);
    });
}

int ipc_broadcast(const void *send, void *recv, size_t b, int root, void *comm, void *stream)
{
    auto *c = static_cast<IpcComm *>(comm);
    if (root < 0 || root >= c->world) return IPC_ARG;
    return collective(comm, K_BC, root, send, b, c->rank == root, stream,
                      [&](IpcComm *cc, hipStream_t st) {
        return copy(recv, cc->peer[root], b, st);
    });
}

int open_comm(IpcComm *c);

// ncclCommSplit's contract: ranks of one color form a communicator ordered by
// (key, rank); color < 0 joins none
int ipc_split(void *comm, int color, int key, void **newcomm)
{
    auto *c  = static_cast<IpcComm *>(comm);
    *newcomm = nullptr;
    t_err.clear();
    if (c->seg->broken.load(std::memory_order_acquire)) return IPC_BROKEN;
    c->seg->slot[c->rank].color = color;
    c->seg->slot[c->rank].key   = key;
    int rc = barrier(c);
    if (rc != IPC_OK) return rc;
    const uint64_t seq = c->nsplit++;
    std::vector<std::pair<int32_t, int>> mine;
    for (int j = 0; j < c->world; ++j) {
        if (color >= 0 && c->seg->slot[j].color == color) mine.emplace_back(c->seg->slot[j].key, j);
    }
    IpcComm *n = nullptr;
    if (color >= 0) {
        std::sort(mine.begin(), mine.end());
        n         = new IpcComm;
        n->name   = c->name + ".s" + std::to_string(seq) + "c" + std::to_string(color);
        n->world  = static_cast<int>(mine.size());
        n->device = c->device;
        n->timeout_ms = c->timeout_ms;
        for (size_t i = 0; i < mine.size(); ++i) {
            if (mine[i].second == c->rank) n->rank = static_cast<int>(i);
        }
        if ((rc = open_comm(n)) != IPC_OK) {
            delete n;
            return fail(c, rc, t_err);
        }
    }
    // every member has mapped its segment: the name can go
    rc = barrier(c);
    if (rc != IPC_OK) {
        if (n) {
            shm_unlink(n->name.c_str());
            munmap(n->seg, sizeof(Seg));
            delete n;
        }
        return rc;
    }
    if (n && n->rank == 0) shm_unlink(n->name.c_str());
    *newcomm = n;
    return IPC_OK;
}

int open_comm(IpcComm *c)
{
    if (c->world < 1 || c->world > kMaxRanks || c->rank < 0 || c->rank >= c->world) {
        t_err = "ipc transport: bad rank / world";
        return IPC_ARG;
    }
    c->seg = map_segment(c->name);
    if (!c->seg) {
        t_err = "ipc transport: shm_open / mmap of " + c->name + ": " + std::strerror(errno);
        return IPC_SHM;
    }
    c->peer.assign(c->world, nullptr);
    return IPC_OK;
}

int ipc_nop(void *) { return IPC_OK; }
int ipc_async_error(void *comm)
{
    return static_cast<IpcComm *>(comm)->seg->broken.load(std::memory_order_acquire) ? IPC_BROKEN : IPC_OK;
}
void ipc_destroy(void *comm)
{
    auto *c = static_cast<IpcComm *>(comm);
    drop_peers(c);
    if (c->stage) (void)hipFree(c->stage);
    if (c->seg) munmap(c->seg, sizeof(Seg));
    delete c;
}
const char *ipc_error_string(int code)
{
    // the failing call's own message when this thread has one (the exchange
    // asks right after the failed call, on the same thread)
    thread_local std::string msg;
    if (!t_err.empty() && code != IPC_OK) {
        msg = t_err;
        return msg.c_str();
    }
    switch (code) {
    case IPC_HIP: return "ipc transport: a HIP call failed";
    case IPC_DTYPE: return "ipc transport: no reduce-scatter for this dtype";
    case IPC_ARG: return "ipc transport: bad arguments";
    case IPC_TIMEOUT: return "ipc transport: rendezvous timed out";
    case IPC_BROKEN: return "ipc transport: the group failed earlier";
    case IPC_SHM: return "ipc transport: shared memory segment unavailable";
    default: return "ipc transport error";
    }
}

const kf_transport_ops kIpcOps = {
    ipc_nop,       ipc_nop,   ipc_reduce_scatter, ipc_all_gather, ipc_all_to_all,
    ipc_broadcast, ipc_split, ipc_async_error,    ipc_destroy,    ipc_error_string,
};

}  // namespace

extern "C" {

kf_exchange_t *kf_exchange_create_ipc(const char *name, int rank, int world, int device, int timeout_ms)
{
    if (!name || name[0] != '/' || std::strchr(name + 1, '/')) {
        t_err = "kf_exchange_create_ipc: the name must be one /name component";
        return nullptr;
    }
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        t_err = std::string("hipSetDevice: ") + hipGetErrorString(e);
        return nullptr;
    }
    auto *c       = new IpcComm;
    c->name       = name;
    c->rank       = rank;
    c->world      = world;
    c->device     = device;
    c->timeout_ms = timeout_ms > 0 ? timeout_ms : 120000;
    if (open_comm(c) != IPC_OK) {
        delete c;
        return nullptr;
    }
    // every rank has mapped the segment before its name is removed
    if (barrier(c) != IPC_OK) {  // a rank never came: leave no segment behind
        shm_unlink(name);
        munmap(c->seg, sizeof(Seg));
        delete c;
        return nullptr;
    }
    if (rank == 0) shm_unlink(name);
    // staging for calls of up to 256 MiB from the start (every shape the
    // bench and the tests use), so no growth falls in the middle of a run
    if (ensure(c, size_t(256) << 20) != IPC_OK) {
        ipc_destroy(c);
        return nullptr;
    }
    kf_exchange_t *ex = kf_exchange_create_transport(&kIpcOps, c, rank, world, device);
    if (!ex) {
        t_err = kf_exchange_last_error();
        ipc_destroy(c);
    }
    return ex;
}

const char *kf_ipc_last_error(void) { return t_err.c_str(); }

}  // extern "C"
