// kf_exchange.hip — the multi-GPU bucket exchange over RCCL behind the C ABI
// (include/kungfu_amd.h, "multi-GPU exchange").
//
// Reference: srcs/cpp/src/nccl/gpu_collective.cpp. There, one communicator per
// process is built from an ncclUniqueId that rank 0 creates and KungFu
// broadcasts (new_global, :190-200), and every tensor goes through
// ncclAllReduce followed by a stream sync (:151-165); the TF ops order the
// calls across ranks with NCCLScheduler (srcs/cpp/src/nccl/scheduler.cpp).
//
// Here a bucket's all-reduce is split so that the element-wise sum is the
// build's HIP kernel where the semantics call for it (north_star: RCCL
// reduce-scatter + all-gather over xGMI):
//   reduce-scatter algo: ncclReduceScatter -> kf_bucket_div on the shard ->
//                        in-place ncclAllGather;
//   all-to-all algo:     ncclAllToAll of the shards -> HIP k-input fold of
//                        the received shards in rank order (/np fused) ->
//                        in-place ncclAllGather. Same xGMI bytes as the
//                        reduce-scatter ((w-1)/w of the bucket out and in per
//                        rank), one extra HBM pass over the received shards,
//                        and the result is the oracle's rank-order fold for
//                        every dtype (bf16: fp32 accumulation, one rounding).
// Many buckets go in ONE call: every phase is one ncclGroupStart/End (RCCL
// fuses the group into one launch) and all shard epilogues are one batched
// HIP launch (kf_bucket_reduce_batch), so 64 x 4 MiB buckets cost 3 launches.
//
// librccl is opened at run time (dlopen "librccl.so.1"): the B1 drop-in does
// not need it, and in a process where torch already loaded its RCCL (same
// soname) both use that one library.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "kungfu_amd.h"

// kf_session.hip (library-internal)
int kf_session_device_mode_internal(const kf_session_t *s);

namespace
{
thread_local std::string t_ex_error;

int fail(int rc, const std::string &msg)
{
    t_ex_error = msg;
    return rc;
}

int hip_fail(hipError_t e, const char *what)
{
    return fail(KF_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define KF_HIP(call)                                                           \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess) return hip_fail(e_, #call);                      \
    } while (0)

// ---------------------------------------------------------------------------
// librccl, resolved at run time
// ---------------------------------------------------------------------------
struct Rccl {
    bool ok = false;
    std::string why;
    decltype(&::ncclGetUniqueId) GetUniqueId             = nullptr;
    decltype(&::ncclCommInitRank) CommInitRank           = nullptr;
    decltype(&::ncclCommDestroy) CommDestroy             = nullptr;
    decltype(&::ncclCommAbort) CommAbort                 = nullptr;
    decltype(&::ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&::ncclReduceScatter) ReduceScatter         = nullptr;
    decltype(&::ncclAllGather) AllGather                 = nullptr;
    decltype(&::ncclAllToAll) AllToAll                   = nullptr;
    decltype(&::ncclBroadcast) Broadcast                 = nullptr;
    decltype(&::ncclGroupStart) GroupStart               = nullptr;
    decltype(&::ncclGroupEnd) GroupEnd                   = nullptr;
    decltype(&::ncclGetErrorString) GetErrorString       = nullptr;
};

const Rccl &rccl()
{
    static const Rccl r = [] {
        Rccl x;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char *e = dlerror();
            x.why         = std::string("dlopen librccl.so.1: ") + (e ? e : "?");
            return x;
        }
#define KF_LOAD(field, sym)                                                    \
    x.field = reinterpret_cast<decltype(x.field)>(dlsym(h, #sym));             \
    if (!x.field) {                                                            \
        x.why = "librccl.so.1 lacks " #sym;                                    \
        return x;                                                              \
    }
        KF_LOAD(GetUniqueId, ncclGetUniqueId)
        KF_LOAD(CommInitRank, ncclCommInitRank)
        KF_LOAD(CommDestroy, ncclCommDestroy)
        KF_LOAD(CommAbort, ncclCommAbort)
        KF_LOAD(CommGetAsyncError, ncclCommGetAsyncError)
        KF_LOAD(ReduceScatter, ncclReduceScatter)
        KF_LOAD(AllGather, ncclAllGather)
        KF_LOAD(AllToAll, ncclAllToAll)
        KF_LOAD(Broadcast, ncclBroadcast)
        KF_LOAD(GroupStart, ncclGroupStart)
        KF_LOAD(GroupEnd, ncclGroupEnd)
        KF_LOAD(GetErrorString, ncclGetErrorString)
#undef KF_LOAD
        x.ok = true;
        return x;
    }();
    return r;
}

int nccl_fail(ncclResult_t r, const char *what)
{
    const char *why = rccl().ok ? rccl().GetErrorString(r) : "RCCL error";
    return fail(KF_ERR_RCCL, std::string(what) + ": " + why + " (" + std::to_string(int(r)) + ")");
}

#define KF_NCCL(call)                                                          \
    do {                                                                       \
        ncclResult_t r_ = (call);                                              \
        if (r_ != ncclSuccess) return nccl_fail(r_, #call);                    \
    } while (0)

int need_rccl()
{
    if (!rccl().ok) return fail(KF_ERR_RCCL, rccl().why);
    return KF_OK;
}

// The caller's device is restored after every entry point.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~DeviceGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int tsize(KungFu_Datatype dt)
{
    switch (dt) {
    case KungFu_UINT8: case KungFu_INT8: return 1;
    case KungFu_UINT16: case KungFu_INT16: case KungFu_FLOAT16: case KungFu_BFLOAT16: return 2;
    case KungFu_UINT32: case KungFu_INT32: case KungFu_FLOAT: return 4;
    case KungFu_UINT64: case KungFu_INT64: case KungFu_DOUBLE: return 8;
    default: return 0;
    }
}

bool is_float(KungFu_Datatype dt)
{
    return dt == KungFu_FLOAT16 || dt == KungFu_BFLOAT16 || dt == KungFu_FLOAT ||
           dt == KungFu_DOUBLE;
}

// dtypes RCCL can reduce (gpu_collective.cpp:60-73 maps int32/f16/f32)
bool nccl_type(KungFu_Datatype dt, ncclDataType_t *t)
{
    switch (dt) {
    case KungFu_UINT8: *t = ncclUint8; return true;
    case KungFu_INT8: *t = ncclInt8; return true;
    case KungFu_UINT32: *t = ncclUint32; return true;
    case KungFu_INT32: *t = ncclInt32; return true;
    case KungFu_UINT64: *t = ncclUint64; return true;
    case KungFu_INT64: *t = ncclInt64; return true;
    case KungFu_FLOAT16: *t = ncclFloat16; return true;
    case KungFu_FLOAT: *t = ncclFloat32; return true;
    case KungFu_DOUBLE: *t = ncclFloat64; return true;
    case KungFu_BFLOAT16: *t = ncclBfloat16; return true;
    default: return false;  // u16 / i16: no RCCL reduction type
    }
}

ncclRedOp_t nccl_op(KungFu_Op op)
{
    switch (op) {
    case KungFu_MIN: return ncclMin;
    case KungFu_MAX: return ncclMax;
    case KungFu_PROD: return ncclProd;
    default: return ncclSum;
    }
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// Testing only: KUNGFU_AMD_EXCHANGE_W1_COLLECTIVES=1 sends a one-rank
// exchange through the RCCL calls and the batched epilogue instead of the
// identity copy, so a one-GPU box exercises librccl's own entry points with
// the exchange's exact arguments (RCCL refuses two ranks on one device).
bool w1_collectives()
{
    static const bool on = [] {
        const char *e = std::getenv("KUNGFU_AMD_EXCHANGE_W1_COLLECTIVES");
        return e && e[0] == '1';
    }();
    return on;
}

// ---------------------------------------------------------------------------
// Loopback transport (testing): the RCCL entry points the exchange uses,
// re-implemented for `world` ranks that are threads of ONE process on ONE
// device, so the sharding, tails, workspace and fold logic of every world
// size runs on a single GPU (RCCL itself refuses two ranks on one device).
// Every collective is a rendezvous: each rank synchronises its stream and
// posts its buffers; the last to arrive moves the bytes (hipMemcpy, and for
// the reduce-scatter a host fold in rank order) and releases the others.
// ---------------------------------------------------------------------------
struct LoopSlot {
    int arrived = 0, left = 0;
    bool done   = false;
    std::vector<const void *> send;
    std::vector<void *> recv;
};

struct LoopGroup {
    int world;
    std::mutex mu;
    std::condition_variable cv;
    std::map<uint64_t, LoopSlot> slots;
    explicit LoopGroup(int w) : world(w) {}
};

struct LoopComm {
    LoopGroup *g;
    int rank;
    uint64_t seq = 0;
};

size_t nccl_size(ncclDataType_t t)
{
    switch (t) {
    case ncclInt8: case ncclUint8: return 1;
    case ncclFloat16: case ncclBfloat16: return 2;
    case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
    case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
    default: return 0;
    }
}

template <typename T>
void host_fold(const std::vector<std::vector<char>> &in, size_t off, size_t n, ncclRedOp_t op,
               char *out)
{
    for (size_t i = 0; i < n; ++i) {
        T a = reinterpret_cast<const T *>(in[0].data() + off)[i];
        for (size_t j = 1; j < in.size(); ++j) {
            const T b = reinterpret_cast<const T *>(in[j].data() + off)[i];
            if (op == ncclSum) a = static_cast<T>(a + b);
            else if (op == ncclProd) a = static_cast<T>(a * b);
            else if (op == ncclMin) a = (b < a) ? b : a;
            else a = (a < b) ? b : a;
        }
        reinterpret_cast<T *>(out)[i] = a;
    }
}

// rendezvous; `move` runs once, on the last rank to arrive, with every
// rank's posted buffers
template <typename F>
ncclResult_t loop_collective(ncclComm_t comm, const void *send, void *recv, hipStream_t s, F move)
{
    auto *c = reinterpret_cast<LoopComm *>(comm);
    if (hipStreamSynchronize(s) != hipSuccess) return ncclUnhandledCudaError;
    LoopGroup *g = c->g;
    std::unique_lock<std::mutex> lk(g->mu);
    LoopSlot &sl = g->slots[c->seq];
    const uint64_t seq = c->seq++;
    if (sl.send.empty()) {
        sl.send.assign(g->world, nullptr);
        sl.recv.assign(g->world, nullptr);
    }
    sl.send[c->rank] = send;
    sl.recv[c->rank] = recv;
    ncclResult_t rc = ncclSuccess;
    if (++sl.arrived == g->world) {
        rc      = move(sl.send, sl.recv);
        sl.done = true;
        g->cv.notify_all();
    } else {
        g->cv.wait(lk, [&] { return sl.done; });
    }
    if (++sl.left == g->world) g->slots.erase(seq);
    return rc;
}

ncclResult_t loop_reduce_scatter(const void *send, void *recv, size_t count, ncclDataType_t t,
                                 ncclRedOp_t op, ncclComm_t comm, hipStream_t s)
{
    return loop_collective(comm, send, recv, s, [&](const std::vector<const void *> &sd,
                                                     const std::vector<void *> &rv) {
        const size_t sz = nccl_size(t), W = sd.size();
        if (sz == 0 || t == ncclFloat16 || t == ncclBfloat16) return ncclInvalidArgument;
        std::vector<std::vector<char>> in(W, std::vector<char>(count * W * sz));
        for (size_t j = 0; j < W; ++j) {
            if (hipMemcpy(in[j].data(), sd[j], count * W * sz, hipMemcpyDeviceToHost) != hipSuccess)
                return ncclUnhandledCudaError;
        }
        std::vector<char> out(count * sz);
        for (size_t r = 0; r < W; ++r) {
            const size_t off = r * count * sz;
            switch (t) {
            case ncclInt8: host_fold<int8_t>(in, off, count, op, out.data()); break;
            case ncclUint8: host_fold<uint8_t>(in, off, count, op, out.data()); break;
            case ncclInt32: host_fold<int32_t>(in, off, count, op, out.data()); break;
            case ncclUint32: host_fold<uint32_t>(in, off, count, op, out.data()); break;
            case ncclInt64: host_fold<int64_t>(in, off, count, op, out.data()); break;
            case ncclUint64: host_fold<uint64_t>(in, off, count, op, out.data()); break;
            case ncclFloat32: host_fold<float>(in, off, count, op, out.data()); break;
            default: host_fold<double>(in, off, count, op, out.data()); break;
            }
            if (hipMemcpy(rv[r], out.data(), count * sz, hipMemcpyHostToDevice) != hipSuccess)
                return ncclUnhandledCudaError;
        }
        return ncclSuccess;
    });
}

ncclResult_t loop_all_gather(const void *send, void *recv, size_t count, ncclDataType_t t,
                             ncclComm_t comm, hipStream_t s)
{
    return loop_collective(comm, send, recv, s, [&](const std::vector<const void *> &sd,
                                                     const std::vector<void *> &rv) {
        const size_t b = count * nccl_size(t), W = sd.size();
        for (size_t r = 0; r < W; ++r) {
            for (size_t j = 0; j < W; ++j) {
                char *dst = static_cast<char *>(rv[r]) + j * b;
                if (dst == sd[j]) continue;  // in place
                if (hipMemcpy(dst, sd[j], b, hipMemcpyDeviceToDevice) != hipSuccess)
                    return ncclUnhandledCudaError;
            }
        }
        return ncclSuccess;
    });
}

ncclResult_t loop_all_to_all(const void *send, void *recv, size_t count, ncclDataType_t t,
                             ncclComm_t comm, hipStream_t s)
{
    return loop_collective(comm, send, recv, s, [&](const std::vector<const void *> &sd,
                                                     const std::vector<void *> &rv) {
        const size_t b = count * nccl_size(t), W = sd.size();
        for (size_t r = 0; r < W; ++r) {
            for (size_t j = 0; j < W; ++j) {
                if (hipMemcpy(static_cast<char *>(rv[r]) + j * b,
                              static_cast<const char *>(sd[j]) + r * b, b,
                              hipMemcpyDeviceToDevice) != hipSuccess)
                    return ncclUnhandledCudaError;
            }
        }
        return ncclSuccess;
    });
}

ncclResult_t loop_broadcast(const void *send, void *recv, size_t count, ncclDataType_t t, int root,
                            ncclComm_t comm, hipStream_t s)
{
    return loop_collective(comm, send, recv, s, [&](const std::vector<const void *> &sd,
                                                     const std::vector<void *> &rv) {
        const size_t b = count * nccl_size(t);
        for (size_t r = 0; r < rv.size(); ++r) {
            if (rv[r] == sd[root]) continue;
            if (hipMemcpy(rv[r], sd[root], b, hipMemcpyDeviceToDevice) != hipSuccess)
                return ncclUnhandledCudaError;
        }
        return ncclSuccess;
    });
}

ncclResult_t loop_nop() { return ncclSuccess; }
ncclResult_t loop_async_error(ncclComm_t, ncclResult_t *e)
{
    *e = ncclSuccess;
    return ncclSuccess;
}
ncclResult_t loop_destroy(ncclComm_t comm)
{
    delete reinterpret_cast<LoopComm *>(comm);
    return ncclSuccess;
}
const char *loop_error_string(ncclResult_t) { return "loopback transport error"; }

const Rccl &loop_rccl()
{
    static const Rccl r = [] {
        Rccl x;
        x.CommDestroy       = loop_destroy;
        x.CommGetAsyncError = loop_async_error;
        x.ReduceScatter     = loop_reduce_scatter;
        x.AllGather         = loop_all_gather;
        x.AllToAll          = loop_all_to_all;
        x.Broadcast         = loop_broadcast;
        x.GroupStart        = loop_nop;
        x.GroupEnd          = loop_nop;
        x.GetErrorString    = loop_error_string;
        x.ok                = true;
        return x;
    }();
    return r;
}

}  // namespace

// ---------------------------------------------------------------------------
// the exchange
// ---------------------------------------------------------------------------
struct Task {
    const void *send = nullptr;
    void *recv       = nullptr;
    size_t count     = 0;
    KungFu_Datatype dt;
    KungFu_Op op;
    int average = 0, algo = 0;
    hipStream_t stream = nullptr;
    kf_done_fn done    = nullptr;
    void *arg          = nullptr;
    bool started       = false;
};

struct Done {
    hipEvent_t ev;
    kf_done_fn done;
    void *arg;
    int status;
};

struct kf_exchange {
    const Rccl *R   = nullptr;  // librccl, or the loopback transport
    ncclComm_t comm = nullptr;
    int rank = 0, world = 1, device = 0;
    std::mutex mu;  // one collective sequence at a time

    // workspace (received shards, tails), ordered between streams by ws_ev
    void *ws            = nullptr;
    size_t ws_cap       = 0;
    hipEvent_t ws_ev    = nullptr;
    hipStream_t ws_last = nullptr;
    bool ws_used        = false;
    hipStream_t own     = nullptr;  // internal (order broadcast)

    // pipelined schedule (kf_exchange_set_pipeline): the buckets of a call in
    // `groups` groups; RCCL phases on the caller's stream, the element-wise
    // work (folds, /np, SMA blends) on `comp`, so group g's HIP work runs
    // while group g+1's collectives move bytes
    int groups         = 1;
    hipStream_t comp   = nullptr;
    std::vector<hipEvent_t> pev;  // 3 per group

    // NCCLScheduler / LinearExecutor
    std::mutex smu;
    std::condition_variable scv;
    std::map<std::string, int> idx;
    std::vector<int32_t> order, arrive, first_arrive;
    std::vector<Task> tasks;
    size_t issued = 0, completed = 0, ntasks = 0;
    int steps      = 0;
    int sstatus    = KF_OK;
    std::string serr;  // the first failure's message (the worker threads' own)
    bool stop      = false;
    std::deque<Done> cq;
    std::thread issuer, completer;

    int ensure_ws(size_t bytes, hipStream_t s);
    void release_ws(hipStream_t s);
    // sma_alpha != nullptr: SMA, sends = the variables, recvs = the sum workspaces,
    // each variable blended once its sum is gathered
    int batch(const void *const *sends, void *const *recvs, const size_t *counts, int nb,
              KungFu_Datatype dt, KungFu_Op op, int average, int algo, hipStream_t s,
              const double *sma_alpha = nullptr);
    void issue_loop();
    void complete_loop();
    ~kf_exchange();
};

int kf_exchange::ensure_ws(size_t bytes, hipStream_t s)
{
    if (ws_used && ws_last != s) KF_HIP(hipStreamWaitEvent(s, ws_ev, 0));
    if (bytes > ws_cap) {
        if (ws) {
            if (ws_used) KF_HIP(hipEventSynchronize(ws_ev));
            KF_HIP(hipFree(ws));
            ws     = nullptr;
            ws_cap = 0;
        }
        const size_t cap = align_up(bytes, size_t(2) << 20);
        KF_HIP(hipMalloc(&ws, cap));
        ws_cap = cap;
    }
    return KF_OK;
}

void kf_exchange::release_ws(hipStream_t s)
{
    if (hipEventRecord(ws_ev, s) == hipSuccess) {
        ws_last = s;
        ws_used = true;
    }
}

// Resolve KF_ALGO_AUTO; KF_ERR_* for a combination that cannot run.
static int resolve_algo(int algo, KungFu_Datatype dt, KungFu_Op op, int world, int *out)
{
    ncclDataType_t t;
    const bool rs_ok = nccl_type(dt, &t);
    if (algo == KF_ALGO_REDUCE_SCATTER) {
        if (!rs_ok) return fail(KF_ERR_DTYPE, "no RCCL reduction type for this dtype");
        *out = algo;
        return KF_OK;
    }
    if (algo == KF_ALGO_ALL_TO_ALL) {
        if (world > KF_MAX_INPUTS) {
            return fail(KF_ERR_ARG, "all-to-all fold supports at most 16 ranks");
        }
        *out = algo;
        return KF_OK;
    }
    if (algo != KF_ALGO_AUTO) return fail(KF_ERR_ARG, "unknown algo");
    (void)op;  // MIN/MAX through RCCL differ from std::min/max only on NaN inputs
    const bool own_semantics = dt == KungFu_FLOAT16 || dt == KungFu_BFLOAT16;
    if (world <= KF_MAX_INPUTS && (own_semantics || !rs_ok)) {
        *out = KF_ALGO_ALL_TO_ALL;
    } else if (rs_ok) {
        *out = KF_ALGO_REDUCE_SCATTER;
    } else {
        return fail(KF_ERR_DTYPE, "dtype needs the all-to-all fold (at most 16 ranks)");
    }
    return KF_OK;
}

int kf_exchange::batch(const void *const *sends, void *const *recvs, const size_t *counts,
                       int nb, KungFu_Datatype dt, KungFu_Op op, int average, int algo,
                       hipStream_t s, const double *sma_alpha)
{
    const Rccl &R = *this->R;
    const int sz  = tsize(dt);
    const int W = world, r = rank;
    const bool sma = sma_alpha != nullptr;
    if (W == 1 && !w1_collectives()) {  // a single peer: the sum is the bucket, x / 1 == x
        for (int b = 0; b < nb; ++b) {
            if (counts[b] && sends[b] != recvs[b]) {
                KF_HIP(hipMemcpyAsync(recvs[b], sends[b], counts[b] * sz, hipMemcpyDeviceToDevice, s));
            }
        }
        if (sma) {
            std::vector<void *> vv(nb);
            for (int b = 0; b < nb; ++b) vv[b] = const_cast<void *>(sends[b]);
            const int rc = kf_sma_blend_batch(vv.data(), const_cast<const void *const *>(recvs),
                                              counts, nb, dt, W, *sma_alpha, s);
            if (rc != KF_OK) return fail(rc, "kf_sma_blend_batch");
        }
        return KF_OK;
    }
    int a  = 0;
    int rc = resolve_algo(algo, dt, op, W, &a);
    if (rc != KF_OK) return rc;
    ncclDataType_t nt = ncclUint8;
    nccl_type(dt, &nt);

    // workspace: received shards (all-to-all) and gathered tails
    std::vector<size_t> wsoff(nb, 0), toff(nb, 0);
    size_t need = 0;
    for (int b = 0; b < nb; ++b) {
        const size_t q = counts[b] / W, t = counts[b] % W;
        if (a == KF_ALGO_ALL_TO_ALL && q) {
            wsoff[b] = need;
            need += align_up(q * W * sz, 256);
        }
        if (t) {
            toff[b] = need;
            need += align_up(t * W * sz, 256);
        }
    }
    if (need) {
        rc = ensure_ws(need, s);
        if (rc != KF_OK) return rc;
    }
    char *wsp = static_cast<char *>(ws);

    auto group_end = [&](int status) -> int {
        ncclResult_t e = R.GroupEnd();
        if (status != KF_OK) return status;
        if (e != ncclSuccess) return nccl_fail(e, "ncclGroupEnd");
        return KF_OK;
    };

    // phase 1: every bucket's reduce-scatter (or all-to-all) and tail gather
    auto phase1 = [&](int b0, int b1) -> int {
        KF_NCCL(R.GroupStart());
        int rc1 = KF_OK;
        for (int b = b0; b < b1 && rc1 == KF_OK; ++b) {
            const size_t q = counts[b] / W, t = counts[b] % W;
            const char *snd = static_cast<const char *>(sends[b]);
            char *rcv       = static_cast<char *>(recvs[b]);
            ncclResult_t e  = ncclSuccess;
            if (q && a == KF_ALGO_REDUCE_SCATTER) {
                e = R.ReduceScatter(snd, rcv + r * q * sz, q, nt, nccl_op(op), comm, s);
            } else if (q) {
                e = R.AllToAll(snd, wsp + wsoff[b], q * sz, ncclUint8, comm, s);
            }
            if (e == ncclSuccess && t) {
                e = R.AllGather(snd + q * W * sz, wsp + toff[b], t * sz, ncclUint8, comm, s);
            }
            if (e != ncclSuccess) rc1 = nccl_fail(e, "phase-1 collective");
        }
        return group_end(rc1);
    };

    // phase 2: the element-wise work, batched over the buckets
    auto phase2 = [&](int b0, int b1, hipStream_t cs) -> int {
        std::vector<const void *> ins;
        std::vector<void *> outs;
        std::vector<size_t> cnts;
        if (a == KF_ALGO_REDUCE_SCATTER && average) {
            for (int b = b0; b < b1; ++b) {
                const size_t q = counts[b] / W;
                if (!q) continue;
                char *sh = static_cast<char *>(recvs[b]) + r * q * sz;
                ins.push_back(sh);
                outs.push_back(sh);
                cnts.push_back(q);
            }
            if (!outs.empty()) {
                const int e = kf_bucket_reduce_batch(ins.data(), 1, outs.data(), cnts.data(),
                                                     static_cast<int>(outs.size()), dt, KungFu_SUM,
                                                     W, cs);
                if (e != KF_OK) return fail(e, "shard /np epilogue");
            }
            ins.clear();
            outs.clear();
            cnts.clear();
        }
        for (int b = b0; b < b1; ++b) {  // rank-order folds: shards and tails
            const size_t q = counts[b] / W, t = counts[b] % W;
            char *rcv      = static_cast<char *>(recvs[b]);
            if (q && a == KF_ALGO_ALL_TO_ALL) {
                for (int j = 0; j < W; ++j) ins.push_back(wsp + wsoff[b] + j * q * sz);
                outs.push_back(rcv + r * q * sz);
                cnts.push_back(q);
            }
            if (t) {
                for (int j = 0; j < W; ++j) ins.push_back(wsp + toff[b] + j * t * sz);
                outs.push_back(rcv + q * W * sz);
                cnts.push_back(t);
            }
        }
        if (!outs.empty()) {
            const int e = kf_bucket_reduce_batch(ins.data(), W, outs.data(), cnts.data(),
                                                 static_cast<int>(outs.size()), dt, op,
                                                 average ? W : 0, cs);
            if (e != KF_OK) return fail(e, "rank-order fold of the received shards");
        }
        return KF_OK;
    };

    // phase 3: in-place all-gather of every reduced shard
    auto phase3 = [&](int b0, int b1) -> int {
        KF_NCCL(R.GroupStart());
        int rc3 = KF_OK;
        for (int b = b0; b < b1 && rc3 == KF_OK; ++b) {
            const size_t q = counts[b] / W;
            if (!q) continue;
            char *rcv      = static_cast<char *>(recvs[b]);
            ncclResult_t e = R.AllGather(rcv + r * q * sz, rcv, q * sz, ncclUint8, comm, s);
            if (e != ncclSuccess) rc3 = nccl_fail(e, "ncclAllGather");
        }
        return group_end(rc3);
    };

    // SMA: v = (1 - alpha) v + alpha (sum / world), once the sum is gathered;
    // the buckets' blends in one batched launch
    auto blend = [&](int b0, int b1, hipStream_t cs) -> int {
        if (!sma || b1 <= b0) return KF_OK;
        std::vector<void *> vv(b1 - b0);
        for (int b = b0; b < b1; ++b) vv[b - b0] = const_cast<void *>(sends[b]);
        const int e = kf_sma_blend_batch(vv.data(), const_cast<const void *const *>(recvs + b0),
                                         counts + b0, b1 - b0, dt, W, *sma_alpha, cs);
        if (e != KF_OK) return fail(e, "kf_sma_blend_batch");
        return KF_OK;
    };

    const int G = std::min(groups, nb);
    if (G <= 1) {
        rc = phase1(0, nb);
        if (rc == KF_OK) rc = phase2(0, nb, s);
        if (rc == KF_OK) rc = phase3(0, nb);
        if (rc == KF_OK) rc = blend(0, nb, s);
        if (rc != KF_OK) return rc;
        if (need) release_ws(s);
        return KF_OK;
    }

    // pipelined: groups of consecutive buckets with about equal bytes;
    //   caller stream s: p1(0) p1(1) [wait p2(0)] p3(0) p1(2) [wait p2(1)] p3(1) ...
    //   comp stream:     [wait p1(0)] p2(0) [wait p1(1)] p2(1) [wait p3(0)] blend(0) ...
    // every wait is on an event recorded earlier on the other stream, so
    // neither stream can wait on the other in a cycle; the RCCL calls keep the
    // same order on every rank
    std::vector<int> gb(1, 0);  // group g = buckets [gb[g], gb[g+1])
    {
        size_t total = 0, acc = 0;
        for (int b = 0; b < nb; ++b) total += counts[b];
        for (int b = 0; b < nb; ++b) {
            acc += counts[b];
            const int left = nb - b - 1, want = G - static_cast<int>(gb.size());
            if (want > 0 && left >= want && acc * G >= total * gb.size()) gb.push_back(b + 1);
        }
        gb.push_back(nb);
    }
    const int ng = static_cast<int>(gb.size()) - 1;
    if (!comp) KF_HIP(hipStreamCreateWithFlags(&comp, hipStreamNonBlocking));
    while (pev.size() < static_cast<size_t>(3 * ng + 1)) {
        hipEvent_t e;
        KF_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        pev.push_back(e);
    }
    auto e1 = [&](int g) { return pev[3 * g]; };
    auto e2 = [&](int g) { return pev[3 * g + 1]; };
    auto e3 = [&](int g) { return pev[3 * g + 2]; };
    hipEvent_t e_end = pev[3 * ng];
    auto finish = [&](int g) -> int {  // gather group g, then blend it
        KF_HIP(hipStreamWaitEvent(s, e2(g), 0));
        int f = phase3(gb[g], gb[g + 1]);
        if (f != KF_OK || !sma) return f;
        KF_HIP(hipEventRecord(e3(g), s));
        KF_HIP(hipStreamWaitEvent(comp, e3(g), 0));
        return blend(gb[g], gb[g + 1], comp);
    };
    for (int g = 0; g < ng && rc == KF_OK; ++g) {
        rc = phase1(gb[g], gb[g + 1]);
        if (rc != KF_OK) break;
        KF_HIP(hipEventRecord(e1(g), s));
        KF_HIP(hipStreamWaitEvent(comp, e1(g), 0));
        rc = phase2(gb[g], gb[g + 1], comp);
        if (rc != KF_OK) break;
        KF_HIP(hipEventRecord(e2(g), comp));
        if (g > 0) rc = finish(g - 1);
    }
    if (rc == KF_OK) rc = finish(ng - 1);
    if (rc == KF_OK && sma) {  // the caller's stream ends after the last blend
        KF_HIP(hipEventRecord(e_end, comp));
        KF_HIP(hipStreamWaitEvent(s, e_end, 0));
    }
    if (rc != KF_OK) return rc;
    if (need) release_ws(s);
    return KF_OK;
}

// Issue thread: the tasks of the step, strictly in `order`
// (LinearExecutor, scheduler.cpp:40-58).
void kf_exchange::issue_loop()
{
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(smu);
    for (;;) {
        scv.wait(lk, [&] {
            return stop || (issued < ntasks && tasks[order[issued]].started);
        });
        if (stop) return;
        Task t = tasks[order[issued]];
        lk.unlock();
        int rc;
        {
            std::lock_guard<std::mutex> g(mu);
            const void *sp = t.send;
            void *rp       = t.recv;
            rc = batch(&sp, &rp, &t.count, 1, t.dt, t.op, t.average, t.algo, t.stream);
        }
        const std::string why = rc == KF_OK ? std::string() : t_ex_error;
        hipEvent_t ev = nullptr;
        if (rc == KF_OK && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess) {
            if (hipEventRecord(ev, t.stream) != hipSuccess) {
                (void)hipEventDestroy(ev);
                ev = nullptr;
                rc = fail(KF_ERR_HIP, "hipEventRecord");
            }
        } else if (rc == KF_OK) {
            rc = fail(KF_ERR_HIP, "hipEventCreate");
        }
        lk.lock();
        if (rc != KF_OK && serr.empty()) serr = why.empty() ? t_ex_error : why;
        cq.push_back(Done{ev, t.done, t.arg, rc});
        ++issued;
        scv.notify_all();
    }
}

// Completion thread: done(status, arg) once each issued all-reduce finished.
void kf_exchange::complete_loop()
{
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(smu);
    for (;;) {
        scv.wait(lk, [&] { return stop || !cq.empty(); });
        if (cq.empty() && stop) return;
        Done d = cq.front();
        cq.pop_front();
        lk.unlock();
        int rc = d.status;
        if (d.ev) {
            if (hipEventSynchronize(d.ev) != hipSuccess) rc = KF_ERR_HIP;
            (void)hipEventDestroy(d.ev);
        }
        if (rc == KF_OK) {
            ncclResult_t ae = ncclSuccess;
            if (R->CommGetAsyncError(comm, &ae) != ncclSuccess || ae != ncclSuccess) {
                rc = KF_ERR_RCCL;
            }
        }
        if (d.done) d.done(rc, d.arg);
        lk.lock();
        if (rc != KF_OK && sstatus == KF_OK) {
            sstatus = rc;
            if (serr.empty()) serr = "an issued all-reduce failed on the device or in RCCL";
        }
        ++completed;
        scv.notify_all();
    }
}

kf_exchange::~kf_exchange()
{
    {
        std::lock_guard<std::mutex> lk(smu);
        stop = true;
    }
    scv.notify_all();
    if (issuer.joinable()) issuer.join();
    if (completer.joinable()) completer.join();
    DeviceGuard g(device);
    if (comm) (void)R->CommDestroy(comm);
    if (ws) (void)hipFree(ws);
    if (ws_ev) (void)hipEventDestroy(ws_ev);
    if (own) (void)hipStreamDestroy(own);
    if (comp) (void)hipStreamDestroy(comp);
    for (auto e : pev) (void)hipEventDestroy(e);
}

extern "C" {

int kf_exchange_unique_id(void *id)
{
    if (!id) return KF_ERR_ARG;
    int rc = need_rccl();
    if (rc != KF_OK) return rc;
    static_assert(sizeof(ncclUniqueId) == KF_UNIQUE_ID_BYTES, "id size");
    ncclUniqueId u;
    KF_NCCL(rccl().GetUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return KF_OK;
}

int kf_exchange_share_id(kf_session_t *s, void *id)
{
    if (!s || !id) return KF_ERR_ARG;
    const int dm = kf_session_device_mode_internal(s);
    if (dm == 0) {
        return kf_session_broadcast(s, id, id, KF_UNIQUE_ID_BYTES, KungFu_UINT8, "nccl id", nullptr);
    }
    void *d = nullptr;
    KF_HIP(hipMalloc(&d, KF_UNIQUE_ID_BYTES));
    int rc = KF_OK;
    hipError_t e = hipMemcpy(d, id, KF_UNIQUE_ID_BYTES, hipMemcpyHostToDevice);
    if (e != hipSuccess) rc = hip_fail(e, "hipMemcpy(id)");
    if (rc == KF_OK) {
        rc = kf_session_broadcast(s, d, d, KF_UNIQUE_ID_BYTES, KungFu_UINT8, "nccl id", nullptr);
    }
    if (rc == KF_OK) {
        e = hipMemcpy(id, d, KF_UNIQUE_ID_BYTES, hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = hip_fail(e, "hipMemcpy(id)");
    }
    (void)hipFree(d);
    return rc;
}

kf_exchange_t *kf_exchange_create(const void *id, int rank, int world, int device)
{
    if (!id || world < 1 || rank < 0 || rank >= world || device < 0) {
        fail(KF_ERR_ARG, "kf_exchange_create: bad arguments");
        return nullptr;
    }
    if (need_rccl() != KF_OK) return nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) {
        fail(KF_ERR_NO_DEVICE, "kf_exchange_create: no HIP device " + std::to_string(device));
        return nullptr;
    }
    DeviceGuard g(device);
    auto *ex   = new kf_exchange;
    ex->R      = &rccl();
    ex->rank   = rank;
    ex->world  = world;
    ex->device = device;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclResult_t e = rccl().CommInitRank(&ex->comm, world, u, rank);
    if (e != ncclSuccess) {
        nccl_fail(e, "ncclCommInitRank");
        ex->comm = nullptr;
        delete ex;
        return nullptr;
    }
    if (hipEventCreateWithFlags(&ex->ws_ev, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&ex->own, hipStreamNonBlocking) != hipSuccess) {
        fail(KF_ERR_HIP, "kf_exchange_create: event/stream");
        delete ex;
        return nullptr;
    }
    return ex;
}

kf_exchange_t *kf_exchange_create_session(kf_session_t *s, int rank, int world, int device)
{
    unsigned char id[KF_UNIQUE_ID_BYTES] = {0};
    if (rank == 0 && kf_exchange_unique_id(id) != KF_OK) {
        // the peers still wait for an id: send the zeros, they fail in init
        std::string why = t_ex_error;
        (void)kf_exchange_share_id(s, id);
        fail(KF_ERR_RCCL, why);
        return nullptr;
    }
    int rc = kf_exchange_share_id(s, id);
    if (rc != KF_OK) {
        fail(rc, "kf_exchange_share_id failed");
        return nullptr;
    }
    return kf_exchange_create(id, rank, world, device);
}

static int check_bucket_args(kf_exchange_t *ex, const void *const *sends, void *const *recvs,
                             const size_t *counts, int nb, KungFu_Datatype dt, KungFu_Op op,
                             int average)
{
    if (!ex || nb < 0 || (nb > 0 && (!sends || !recvs || !counts))) {
        return fail(KF_ERR_ARG, "bad arguments");
    }
    if (tsize(dt) == 0) return fail(KF_ERR_DTYPE, "unsupported dtype");
    if (static_cast<unsigned>(op) > KungFu_PROD) return fail(KF_ERR_OP, "unsupported op");
    if (dt == KungFu_FLOAT16 && op != KungFu_SUM) return fail(KF_ERR_OP, "fp16 supports SUM only");
    if (average && (op != KungFu_SUM || !is_float(dt))) {
        return fail(KF_ERR_OP, "average needs SUM on a float dtype");
    }
    for (int b = 0; b < nb; ++b) {
        if (counts[b] && (!sends[b] || !recvs[b])) return fail(KF_ERR_ARG, "null bucket");
    }
    return KF_OK;
}

int kf_exchange_all_reduce_batch(kf_exchange_t *ex, const void *const *sends, void *const *recvs,
                                 const size_t *counts, int nb, KungFu_Datatype dt, KungFu_Op op,
                                 int average, int algo, void *stream)
{
    int rc = check_bucket_args(ex, sends, recvs, counts, nb, dt, op, average);
    if (rc != KF_OK || nb == 0) return rc;
    DeviceGuard g(ex->device);
    std::lock_guard<std::mutex> lk(ex->mu);
    return ex->batch(sends, recvs, counts, nb, dt, op, average, algo,
                     static_cast<hipStream_t>(stream));
}

int kf_exchange_all_reduce(kf_exchange_t *ex, const void *send, void *recv, size_t count,
                           KungFu_Datatype dt, KungFu_Op op, int average, int algo, void *stream)
{
    return kf_exchange_all_reduce_batch(ex, &send, &recv, &count, 1, dt, op, average, algo, stream);
}

int kf_exchange_sma_batch(kf_exchange_t *ex, void *const *vs, void *const *sums,
                          const size_t *counts, int nb, KungFu_Datatype dt, double alpha,
                          int algo, void *stream)
{
    int rc = check_bucket_args(ex, vs, sums, counts, nb, dt, KungFu_SUM, 0);
    if (rc != KF_OK || nb == 0) return rc;
    if (!is_float(dt)) return fail(KF_ERR_DTYPE, "SMA needs a float dtype");
    DeviceGuard g(ex->device);
    std::lock_guard<std::mutex> lk(ex->mu);
    hipStream_t s = static_cast<hipStream_t>(stream);
    std::vector<const void *> snd(vs, vs + nb);
    return ex->batch(snd.data(), sums, counts, nb, dt, KungFu_SUM, 0, algo, s, &alpha);
}

int kf_exchange_set_pipeline(kf_exchange_t *ex, int groups)
{
    if (!ex || groups < 1) return fail(KF_ERR_ARG, "kf_exchange_set_pipeline: groups >= 1");
    std::lock_guard<std::mutex> lk(ex->mu);
    ex->groups = groups;
    return KF_OK;
}

int kf_exchange_begin_step(kf_exchange_t *ex, const char *const *names, int n, int auto_order)
{
    if (!ex || n < 0 || (n > 0 && !names)) return fail(KF_ERR_ARG, "bad arguments");
    std::unique_lock<std::mutex> lk(ex->smu);
    ex->scv.wait(lk, [&] { return ex->completed == ex->ntasks; });  // previous step done
    std::map<std::string, int> idx;
    for (int i = 0; i < n; ++i) {
        if (!names[i] || !idx.emplace(names[i], i).second) {
            return fail(KF_ERR_ARG, "names must be distinct and non-null");
        }
    }
    if (ex->steps == 1 && auto_order && ex->first_arrive.size() == static_cast<size_t>(n)) {
        // NCCLScheduler::Reset (scheduler.cpp:96-118): the second step takes
        // rank 0's arrival order of the first
        lk.unlock();
        DeviceGuard g(ex->device);
        std::vector<int32_t> ord = ex->first_arrive;
        int rc      = KF_OK;
        int32_t *d  = nullptr;
        const size_t bytes = sizeof(int32_t) * n;
        hipError_t e = hipMalloc(&d, bytes);
        if (e == hipSuccess) e = hipMemcpyAsync(d, ord.data(), bytes, hipMemcpyHostToDevice, ex->own);
        if (e != hipSuccess) rc = hip_fail(e, "order broadcast buffer");
        if (rc == KF_OK) {
            std::lock_guard<std::mutex> g2(ex->mu);
            ncclResult_t r = ex->R->Broadcast(d, d, n, ncclInt32, 0, ex->comm, ex->own);
            if (r != ncclSuccess) rc = nccl_fail(r, "ncclBroadcast(order)");
        }
        if (rc == KF_OK) {
            e = hipMemcpyAsync(ord.data(), d, bytes, hipMemcpyDeviceToHost, ex->own);
            if (e == hipSuccess) e = hipStreamSynchronize(ex->own);
            if (e != hipSuccess) rc = hip_fail(e, "order broadcast");
        }
        if (d) (void)hipFree(d);
        if (rc != KF_OK) return rc;
        lk.lock();
        ex->order = ord;
    } else if (ex->order.size() != static_cast<size_t>(n)) {
        ex->order.resize(n);
        std::iota(ex->order.begin(), ex->order.end(), 0);
    }
    ex->idx = std::move(idx);
    ex->tasks.assign(n, Task{});
    ex->arrive.clear();
    ex->issued = ex->completed = 0;
    ex->ntasks  = n;
    ex->sstatus = KF_OK;
    ex->serr.clear();
    ex->steps++;
    if (!ex->issuer.joinable()) {
        ex->issuer    = std::thread([ex] { ex->issue_loop(); });
        ex->completer = std::thread([ex] { ex->complete_loop(); });
    }
    return KF_OK;
}

int kf_exchange_start(kf_exchange_t *ex, const char *name, const void *send, void *recv,
                      size_t count, KungFu_Datatype dt, KungFu_Op op, int average, int algo,
                      void *stream, kf_done_fn done, void *arg)
{
    if (!ex || !name) return fail(KF_ERR_ARG, "bad arguments");
    size_t c  = count;
    int rc    = check_bucket_args(ex, &send, &recv, &c, 1, dt, op, average);
    if (rc != KF_OK) return rc;
    std::lock_guard<std::mutex> lk(ex->smu);
    auto it = ex->idx.find(name);
    if (it == ex->idx.end()) return fail(KF_ERR_ARG, std::string("name not in this step: ") + name);
    Task &t = ex->tasks[it->second];
    if (t.started) return fail(KF_ERR_ARG, std::string("started twice: ") + name);
    t = Task{send, recv, count, dt, op, average, algo, static_cast<hipStream_t>(stream), done, arg,
             true};
    ex->arrive.push_back(it->second);
    if (ex->steps == 1) ex->first_arrive = ex->arrive;
    ex->scv.notify_all();
    return KF_OK;
}

int kf_exchange_wait_all(kf_exchange_t *ex, int32_t *order)
{
    if (!ex) return KF_ERR_ARG;
    if (std::this_thread::get_id() == ex->completer.get_id()) {
        return fail(KF_ERR_ARG, "kf_exchange_wait_all from a done callback");
    }
    std::unique_lock<std::mutex> lk(ex->smu);
    ex->scv.wait(lk, [&] { return ex->completed == ex->ntasks; });
    if (order) std::copy(ex->order.begin(), ex->order.end(), order);
    if (ex->sstatus != KF_OK) t_ex_error = ex->serr;  // the message, on the caller's thread
    return ex->sstatus;
}

int kf_exchange_check(kf_exchange_t *ex)
{
    if (!ex) return KF_ERR_ARG;
    ncclResult_t ae = ncclSuccess;
    KF_NCCL(ex->R->CommGetAsyncError(ex->comm, &ae));
    if (ae != ncclSuccess) return nccl_fail(ae, "RCCL asynchronous error");
    return KF_OK;
}

int kf_exchange_info(kf_exchange_t *ex, int *rank, int *world, int *device)
{
    if (!ex) return KF_ERR_ARG;
    if (rank) *rank = ex->rank;
    if (world) *world = ex->world;
    if (device) *device = ex->device;
    return KF_OK;
}

void kf_exchange_destroy(kf_exchange_t *ex) { delete ex; }

kf_loopback_t *kf_loopback_create(int world)
{
    if (world < 1) return nullptr;
    return reinterpret_cast<kf_loopback_t *>(new LoopGroup(world));
}

void kf_loopback_destroy(kf_loopback_t *g) { delete reinterpret_cast<LoopGroup *>(g); }

kf_exchange_t *kf_exchange_create_loopback(kf_loopback_t *g, int rank, int device)
{
    auto *lg = reinterpret_cast<LoopGroup *>(g);
    if (!lg || rank < 0 || rank >= lg->world || device < 0) {
        fail(KF_ERR_ARG, "kf_exchange_create_loopback: bad arguments");
        return nullptr;
    }
    DeviceGuard dg(device);
    auto *ex   = new kf_exchange;
    ex->R      = &loop_rccl();
    ex->rank   = rank;
    ex->world  = lg->world;
    ex->device = device;
    ex->comm   = reinterpret_cast<ncclComm_t>(new LoopComm{lg, rank});
    if (hipEventCreateWithFlags(&ex->ws_ev, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&ex->own, hipStreamNonBlocking) != hipSuccess) {
        fail(KF_ERR_HIP, "kf_exchange_create_loopback: event/stream");
        delete ex;
        return nullptr;
    }
    return ex;
}

const char *kf_exchange_last_error(void) { return t_ex_error.c_str(); }

}  // extern "C"
