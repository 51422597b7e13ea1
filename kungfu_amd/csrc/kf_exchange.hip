// kf_exchange.hip — the multi-GPU bucket exchange behind the C ABI
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
//   reduce-scatter algo: reduce-scatter -> kf_bucket_div on the shard ->
//                        in-place all-gather;
//   all-to-all algo:     all-to-all of the shards -> HIP k-input fold of the
//                        received shards in rank order (/np fused) ->
//                        in-place all-gather. Same xGMI bytes as the
//                        reduce-scatter ((w-1)/w of the bucket out and in per
//                        rank), one extra HBM pass over the received shards,
//                        and the result is the oracle's rank-order fold for
//                        every dtype (bf16: fp32 accumulation, one rounding).
// Many buckets go in ONE call: every phase is one group (RCCL fuses the group
// into one launch) and all shard epilogues are one batched HIP launch
// (kf_bucket_reduce_batch), so 64 x 4 MiB buckets cost 3 launches.
//
// The bytes move through a transport (kf_transport_ops): the built-in one is
// librccl, opened at run time (dlopen "librccl.so.1": the B1 drop-in does not
// need it, and in a process where torch already loaded its RCCL, same soname,
// both use that one library). Hosts may bind another (kf_exchange_create_
// transport); the test library's in-process loopback is one.
//
// Three ways to issue:
//   direct        kf_exchange_all_reduce(_batch) / _sma_batch: every rank calls
//                 in the same order (RCCL's rule);
//   ordered       kf_exchange_begin_step / start: NCCLScheduler's fixed name
//                 list per step (scheduler.cpp:37-119);
//   name-keyed    kf_exchange_all_reduce_named: ranks start names in any
//                 order and tensors pair by name, as KungFu's own all-reduce
//                 pairs messages by name (rchannel/handler/collective.go:
//                 48-64). A negotiation thread agrees the issue order with
//                 the peers in cycles over a split-off control communicator.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
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
int kf_session_hosts_internal(const kf_session_t *s, int *host_of);

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
    decltype(&::ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&::ncclCommSplit) CommSplit                 = nullptr;
    decltype(&::ncclReduceScatter) ReduceScatter         = nullptr;
    decltype(&::ncclAllGather) AllGather                 = nullptr;
    decltype(&::ncclAllToAll) AllToAll                   = nullptr;
    decltype(&::ncclBroadcast) Broadcast                 = nullptr;
    decltype(&::ncclGroupStart) GroupStart               = nullptr;
    decltype(&::ncclGroupEnd) GroupEnd                   = nullptr;
    decltype(&::ncclGetErrorString) GetErrorString       = nullptr;
    // optional (reporting only): kf_exchange_transport_info
    decltype(&::ncclCommCount) CommCount                 = nullptr;
    decltype(&::ncclGetVersion) GetVersion               = nullptr;
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
        KF_LOAD(CommGetAsyncError, ncclCommGetAsyncError)
        KF_LOAD(CommSplit, ncclCommSplit)
        KF_LOAD(ReduceScatter, ncclReduceScatter)
        KF_LOAD(AllGather, ncclAllGather)
        KF_LOAD(AllToAll, ncclAllToAll)
        KF_LOAD(Broadcast, ncclBroadcast)
        KF_LOAD(GroupStart, ncclGroupStart)
        KF_LOAD(GroupEnd, ncclGroupEnd)
        KF_LOAD(GetErrorString, ncclGetErrorString)
#undef KF_LOAD
        x.CommCount  = reinterpret_cast<decltype(x.CommCount)>(dlsym(h, "ncclCommCount"));
        x.GetVersion = reinterpret_cast<decltype(x.GetVersion)>(dlsym(h, "ncclGetVersion"));
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
    switch (static_cast<int>(op)) {
    case KF_TRANSPORT_OP_AVG: return ncclAvg;
    case KungFu_MIN: return ncclMin;
    case KungFu_MAX: return ncclMax;
    case KungFu_PROD: return ncclProd;
    default: return ncclSum;
    }
}

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------
// the built-in transport: librccl
// ---------------------------------------------------------------------------
ncclComm_t C(void *comm) { return static_cast<ncclComm_t>(comm); }
hipStream_t S(void *stream) { return static_cast<hipStream_t>(stream); }

int rccl_group_start(void *) { return rccl().GroupStart(); }
int rccl_group_end(void *) { return rccl().GroupEnd(); }
int rccl_reduce_scatter(const void *send, void *recv, size_t count, KungFu_Datatype dt,
                        KungFu_Op op, void *comm, void *stream)
{
    ncclDataType_t t;
    if (!nccl_type(dt, &t)) return ncclInvalidArgument;
    return rccl().ReduceScatter(send, recv, count, t, nccl_op(op), C(comm), S(stream));
}
int rccl_all_gather(const void *send, void *recv, size_t bytes, void *comm, void *stream)
{
    return rccl().AllGather(send, recv, bytes, ncclUint8, C(comm), S(stream));
}
int rccl_all_to_all(const void *send, void *recv, size_t bytes, void *comm, void *stream)
{
    return rccl().AllToAll(send, recv, bytes, ncclUint8, C(comm), S(stream));
}
int rccl_broadcast(const void *send, void *recv, size_t bytes, int root, void *comm, void *stream)
{
    return rccl().Broadcast(send, recv, bytes, ncclUint8, root, C(comm), S(stream));
}
int rccl_split(void *comm, int color, int key, void **newcomm)
{
    ncclComm_t n = nullptr;
    const ncclResult_t r =
        rccl().CommSplit(C(comm), color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &n, nullptr);
    *newcomm = n;
    return r;
}
int rccl_async_error(void *comm)
{
    ncclResult_t ae = ncclSuccess;
    const ncclResult_t r = rccl().CommGetAsyncError(C(comm), &ae);
    return r != ncclSuccess ? r : ae;
}
void rccl_destroy(void *comm) { (void)rccl().CommDestroy(C(comm)); }
const char *rccl_error_string(int code)
{
    return rccl().ok ? rccl().GetErrorString(static_cast<ncclResult_t>(code)) : "RCCL unavailable";
}

const kf_transport_ops kRcclOps = {
    rccl_group_start, rccl_group_end, rccl_reduce_scatter, rccl_all_gather, rccl_all_to_all,
    rccl_broadcast,   rccl_split,     rccl_async_error,    rccl_destroy,    rccl_error_string,
};

// ---------------------------------------------------------------------------
// name-keyed negotiation: one control-row per rank per cycle
// ---------------------------------------------------------------------------
struct CtrlEntry {
    uint64_t h1, h2, count;
    uint32_t sig, pad;
};
static_assert(sizeof(CtrlEntry) == 32, "control entry");
constexpr size_t kCtrlRow = 4096;                        // bytes per rank per cycle
constexpr int kCtrlMax    = kCtrlRow / sizeof(CtrlEntry) - 1;  // entry 0 is the header

uint64_t fnv1a(const char *s, uint64_t basis)
{
    uint64_t h = basis;
    for (; *s; ++s) {
        h ^= static_cast<unsigned char>(*s);
        h *= 0x100000001b3ull;
    }
    return h;
}

uint32_t task_sig(KungFu_Datatype dt, KungFu_Op op, int average, int algo)
{
    return (static_cast<uint32_t>(dt) << 8) ^ (static_cast<uint32_t>(op) << 4) ^
           (static_cast<uint32_t>(average != 0) << 3) ^ static_cast<uint32_t>(algo);
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
    hipEvent_t ready = nullptr;  // named tasks: the start event, destroyed here
    std::string why;             // named tasks: the failure's message
};

struct NamedTask {
    std::string name;
    uint64_t h1 = 0, h2 = 0;
    const void *send = nullptr;
    void *recv       = nullptr;
    size_t count     = 0;
    KungFu_Datatype dt;
    KungFu_Op op;
    int average = 0, algo = 0;
    hipEvent_t ready = nullptr;
    kf_done_fn done  = nullptr;
    void *arg        = nullptr;
};

struct kf_exchange {
    const kf_transport_ops *T = nullptr;  // librccl, or a host's transport
    void *comm                = nullptr;
    bool builtin              = false;    // the RCCL transport (world-1 shortcut)
    int rank = 0, world = 1, device = 0;
    std::mutex mu;  // one collective sequence at a time

    // workspace (received shards, tails), ordered between streams by ws_ev
    void *ws            = nullptr;
    size_t ws_cap       = 0;
    hipEvent_t ws_ev    = nullptr;
    hipStream_t ws_last = nullptr;
    bool ws_used        = false;
    hipStream_t own     = nullptr;  // internal (order broadcast, split)

    // pipelined schedule (kf_exchange_set_pipeline): the buckets of a call in
    // `groups` groups; collectives on the caller's stream, the element-wise
    // work (folds, /np, SMA blends) on `comp`, so group g's HIP work runs
    // while group g+1's collectives move bytes
    int groups         = 1;
    hipStream_t comp   = nullptr;
    std::vector<hipEvent_t> pev;  // 3 per group

    // opt-in per-phase timing (kf_exchange_set_timing): five timing events on
    // the caller's stream at the phase boundaries of every un-pipelined batch
    // call; the sums are taken when asked (kf_exchange_phase_times)
    struct Marks {
        hipEvent_t e[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    };
    bool timing = false;
    std::deque<Marks> marks_used;
    std::vector<Marks> marks_free;
    double phase_us[4]   = {0, 0, 0, 0};
    int64_t timed_calls  = 0;
    int64_t untimed_calls = 0;  // pipelined calls: their phases overlap
    Marks *take_marks();
    int harvest_marks();

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

    // name-keyed all-reduce (kf_exchange_all_reduce_named)
    std::mutex nmu;
    std::condition_variable ncv;
    std::map<std::string, NamedTask> nwait;  // started here, not yet issued
    std::deque<std::string> nfresh;          // started, not yet reported to the peers
    std::map<std::pair<uint64_t, uint64_t>, std::string> nhash;  // outstanding names
    size_t nstarted = 0, nfinished = 0;
    uint64_t anon_seq = 0;  // names of the anonymous (empty-name) calls, in call order
    int nstatus      = KF_OK;
    std::string nerr;
    bool nstop = false, nbroken = false, nready = false;
    std::deque<Done> ndq;
    std::thread negotiator, nfinisher;
    kf_exchange *ctrl   = nullptr;  // the control communicator (split off)
    hipStream_t nstream = nullptr;  // the named tasks' data stream
    hipStream_t cstream = nullptr;  // the control all-gathers
    bool ntrace         = false;    // KUNGFU_AMD_TRACE_NAMED=1: every issued batch to stderr
    void *cdev = nullptr, *chost = nullptr;  // [row | W rows], device and page-locked

    int tfail(int code, const std::string &what) const
    {
        const char *why = T && T->error_string ? T->error_string(code) : nullptr;
        return fail(KF_ERR_RCCL, what + ": " + (why ? why : "transport error") + " (" +
                                     std::to_string(code) + ")");
    }
    int ensure_ws(size_t bytes, hipStream_t s);
    void release_ws(hipStream_t s);
    // sma_alpha != nullptr: SMA, sends = the variables, recvs = the sum workspaces,
    // each variable blended once its sum is gathered
    // phases: which of the three to run (kAll; the hierarchical all-reduce
    // runs 1+2, its cross-host step, then 3)
    int batch(const void *const *sends, void *const *recvs, const size_t *counts, int nb,
              KungFu_Datatype dt, KungFu_Op op, int average, int algo, hipStream_t s,
              const double *sma_alpha = nullptr, int phases = 7);
    int hier(kf_session_t *cross, const void *send, void *recv, size_t count, KungFu_Datatype dt,
             KungFu_Op op, int average, int algo, const std::string &name, hipStream_t s);
    kf_exchange *split(int color, int key, int *status);  // caller holds mu
    int start_named();                                     // caller holds mu
    void issue_loop();
    void complete_loop();
    void negotiate_loop();
    void finish_loop();
    void fail_outstanding(int rc, const std::string &why);
    ~kf_exchange();
};

namespace
{
kf_exchange *new_exchange(const kf_transport_ops *T, void *comm, bool builtin, int rank, int world,
                          int device)
{
    auto *ex    = new kf_exchange;
    ex->T       = T;
    ex->comm    = comm;
    ex->builtin = builtin;
    ex->rank    = rank;
    ex->world   = world;
    ex->device  = device;
    if (hipEventCreateWithFlags(&ex->ws_ev, hipEventDisableTiming) != hipSuccess ||
        hipStreamCreateWithFlags(&ex->own, hipStreamNonBlocking) != hipSuccess) {
        fail(KF_ERR_HIP, "exchange: event/stream");
        ex->comm = nullptr;  // the caller keeps it
        delete ex;
        return nullptr;
    }
    return ex;
}
}  // namespace

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
    if (algo == KF_ALGO_REDUCE_SCATTER || algo == KF_ALGO_REDUCE_SCATTER_AVG) {
        if (!rs_ok) return fail(KF_ERR_DTYPE, "no reduce-scatter type for this dtype");
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
                       hipStream_t s, const double *sma_alpha, int phases)
{
    const int sz = tsize(dt);
    const int W = world, r = rank;
    const bool sma = sma_alpha != nullptr;
    if (W == 1 && builtin) {  // a single peer: the sum is the bucket, x / 1 == x
        for (int b = 0; b < nb && (phases & 1); ++b) {
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
    if (a == KF_ALGO_REDUCE_SCATTER_AVG && !average) a = KF_ALGO_REDUCE_SCATTER;
    // the /np inside the collective (ncclAvg): no shard epilogue
    const KungFu_Op rs_op =
        a == KF_ALGO_REDUCE_SCATTER_AVG ? static_cast<KungFu_Op>(KF_TRANSPORT_OP_AVG) : op;

    // workspace: received shards (all-to-all) and gathered tails
    std::vector<size_t> wsoff(nb, 0), toff(nb, 0);
    size_t need = 0;
    for (int b = 0; b < nb && (phases & 3); ++b) {
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
        const int e = T->group_end(comm);
        if (status != KF_OK) return status;
        if (e != 0) return tfail(e, "group_end");
        return KF_OK;
    };

    // phase 1: every bucket's reduce-scatter (or all-to-all) and tail gather
    auto phase1 = [&](int b0, int b1) -> int {
        const int e0 = T->group_start(comm);
        if (e0 != 0) return tfail(e0, "group_start");
        int rc1 = KF_OK;
        for (int b = b0; b < b1 && rc1 == KF_OK; ++b) {
            const size_t q = counts[b] / W, t = counts[b] % W;
            const char *snd = static_cast<const char *>(sends[b]);
            char *rcv       = static_cast<char *>(recvs[b]);
            int e           = 0;
            if (q && (a == KF_ALGO_REDUCE_SCATTER || a == KF_ALGO_REDUCE_SCATTER_AVG)) {
                e = T->reduce_scatter(snd, rcv + r * q * sz, q, dt, rs_op, comm, s);
            } else if (q) {
                e = T->all_to_all(snd, wsp + wsoff[b], q * sz, comm, s);
            }
            if (e == 0 && t) {
                e = T->all_gather(snd + q * W * sz, wsp + toff[b], t * sz, comm, s);
            }
            if (e != 0) rc1 = tfail(e, "phase-1 collective");
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
        const int e0 = T->group_start(comm);
        if (e0 != 0) return tfail(e0, "group_start");
        int rc3 = KF_OK;
        for (int b = b0; b < b1 && rc3 == KF_OK; ++b) {
            const size_t q = counts[b] / W;
            if (!q) continue;
            char *rcv   = static_cast<char *>(recvs[b]);
            const int e = T->all_gather(rcv + r * q * sz, rcv, q * sz, comm, s);
            if (e != 0) rc3 = tfail(e, "all_gather");
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

    const int G = phases == 7 ? std::min(groups, nb) : 1;
    if (G <= 1) {
        Marks *mk = timing ? take_marks() : nullptr;
        auto mark = [&](int k) {
            if (mk) (void)hipEventRecord(mk->e[k], s);
        };
        mark(0);
        if (phases & 1) rc = phase1(0, nb);
        mark(1);
        if (rc == KF_OK && (phases & 2)) rc = phase2(0, nb, s);
        mark(2);
        if (rc == KF_OK && (phases & 4)) rc = phase3(0, nb);
        mark(3);
        if (rc == KF_OK && phases == 7) rc = blend(0, nb, s);
        mark(4);
        if (need) release_ws(s);  // whatever ran reads the workspace in stream order
        return rc;
    }
    if (timing) ++untimed_calls;

    // pipelined: groups of consecutive buckets with about equal bytes;
    //   caller stream s: p1(0) p1(1) [wait p2(0)] p3(0) p1(2) [wait p2(1)] p3(1) ...
    //   comp stream:     [wait p1(0)] p2(0) [wait p1(1)] p2(1) [wait p3(0)] blend(0) ...
    // every wait is on an event recorded earlier on the other stream, so
    // neither stream can wait on the other in a cycle; the collectives keep
    // the same order on every rank
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
    bool comp_used   = false;
    // every failure below leaves through the same exit (no early return), so
    // the folds already queued on comp are joined and the workspace released
    auto hip_ok = [&](hipError_t e, const char *what) -> int {
        return e == hipSuccess ? KF_OK : hip_fail(e, what);
    };
    auto finish = [&](int g) -> int {  // gather group g, then blend it
        int f = hip_ok(hipStreamWaitEvent(s, e2(g), 0), "hipStreamWaitEvent(p2)");
        if (f == KF_OK) f = phase3(gb[g], gb[g + 1]);
        if (f != KF_OK || !sma) return f;
        f = hip_ok(hipEventRecord(e3(g), s), "hipEventRecord(p3)");
        if (f == KF_OK) f = hip_ok(hipStreamWaitEvent(comp, e3(g), 0), "hipStreamWaitEvent(p3)");
        if (f == KF_OK) f = blend(gb[g], gb[g + 1], comp);
        return f;
    };
    for (int g = 0; g < ng && rc == KF_OK; ++g) {
        rc = phase1(gb[g], gb[g + 1]);
        if (rc == KF_OK) rc = hip_ok(hipEventRecord(e1(g), s), "hipEventRecord(p1)");
        if (rc == KF_OK) rc = hip_ok(hipStreamWaitEvent(comp, e1(g), 0), "hipStreamWaitEvent(p1)");
        if (rc != KF_OK) break;
        comp_used = true;
        rc = phase2(gb[g], gb[g + 1], comp);
        if (rc == KF_OK) rc = hip_ok(hipEventRecord(e2(g), comp), "hipEventRecord(p2)");
        if (rc == KF_OK && g > 0) rc = finish(g - 1);
    }
    if (rc == KF_OK) rc = finish(ng - 1);
    // the caller's stream ends after everything queued on comp (the last
    // blend; after a failure, the folds already queued), so neither the
    // workspace nor the buckets are reused under them; if even that join
    // cannot be queued, wait for comp here
    if (comp_used && (sma || rc != KF_OK)) {
        if (hipEventRecord(e_end, comp) != hipSuccess || hipStreamWaitEvent(s, e_end, 0) != hipSuccess) {
            (void)hipStreamSynchronize(comp);
        }
    }
    if (need) release_ws(s);
    return rc;
}

kf_exchange::Marks *kf_exchange::take_marks()
{
    if (marks_free.empty()) {
        Marks m;
        for (auto &e : m.e) {
            if (hipEventCreate(&e) != hipSuccess) {
                for (auto &f : m.e)
                    if (f) (void)hipEventDestroy(f);
                return nullptr;  // this call goes untimed
            }
        }
        marks_free.push_back(m);
    }
    marks_used.push_back(marks_free.back());
    marks_free.pop_back();
    return &marks_used.back();
}

// sum the finished calls' phase times (waits for the last one queued)
int kf_exchange::harvest_marks()
{
    int rc = KF_OK;
    while (!marks_used.empty()) {
        Marks m = marks_used.front();
        marks_used.pop_front();
        if (rc == KF_OK && hipEventSynchronize(m.e[4]) == hipSuccess) {
            for (int k = 0; k < 4; ++k) {
                float ms = 0;
                if (hipEventElapsedTime(&ms, m.e[k], m.e[k + 1]) == hipSuccess) phase_us[k] += 1e3 * ms;
            }
            ++timed_calls;
        } else {
            rc = fail(KF_ERR_HIP, "kf_exchange_phase_times: a timed call's events");
        }
        marks_free.push_back(m);
    }
    return rc;
}

// A sub-communicator of the ranks that pass `color` (gpu_collective.cpp:
// 202-243): the (color, key) of every rank are all-gathered first, so each
// rank knows its place and the group's size without asking the transport.
kf_exchange *kf_exchange::split(int color, int key, int *status)
{
    auto bad = [&](int rc) -> kf_exchange * {
        *status = rc;
        return nullptr;
    };
    if (!T->split) return bad(fail(KF_ERR_ARG, "the transport cannot split"));
    const int W = world;
    std::vector<int32_t> ck(2 * W, 0);
    if (W > 1) {
        int32_t *d = nullptr;
        hipError_t e = hipMalloc(&d, sizeof(int32_t) * 2 * (W + 1));
        if (e != hipSuccess) return bad(hip_fail(e, "split: hipMalloc"));
        const int32_t mine[2] = {color, key};
        int rc = KF_OK;
        e = hipMemcpyAsync(d, mine, sizeof(mine), hipMemcpyHostToDevice, own);
        if (e != hipSuccess) rc = hip_fail(e, "split: hipMemcpyAsync");
        if (rc == KF_OK) {
            const int t = T->all_gather(d, d + 2, sizeof(mine), comm, own);
            if (t != 0) rc = tfail(t, "split: all_gather");
        }
        if (rc == KF_OK) {
            e = hipMemcpyAsync(ck.data(), d + 2, sizeof(int32_t) * 2 * W, hipMemcpyDeviceToHost, own);
            if (e == hipSuccess) e = hipStreamSynchronize(own);
            if (e != hipSuccess) rc = hip_fail(e, "split: hipMemcpyAsync");
        }
        (void)hipFree(d);
        if (rc != KF_OK) return bad(rc);
    } else {
        ck = {color, key};
    }
    // ranks of my color, ordered by (key, rank): ncclCommSplit's order
    std::vector<std::pair<int32_t, int>> mem;
    for (int j = 0; j < W; ++j) {
        if (ck[2 * j] == color && color >= 0) mem.emplace_back(ck[2 * j + 1], j);
    }
    std::sort(mem.begin(), mem.end());
    void *nc   = nullptr;
    const int t = T->split(comm, color, key, &nc);
    if (t != 0) return bad(tfail(t, "split"));
    if (color < 0) {
        *status = KF_OK;
        return nullptr;
    }
    int nr = 0;
    for (size_t i = 0; i < mem.size(); ++i) {
        if (mem[i].second == rank) nr = static_cast<int>(i);
    }
    kf_exchange *ex = new_exchange(T, nc, builtin, nr, static_cast<int>(mem.size()), device);
    if (!ex) {
        T->destroy(nc);
        return bad(KF_ERR_HIP);
    }
    ex->groups = groups;
    *status    = KF_OK;
    return ex;
}

// The hierarchical all-reduce (kf_hier_all_reduce); caller holds mu.
int kf_exchange::hier(kf_session_t *cross, const void *send, void *recv, size_t count,
                      KungFu_Datatype dt, KungFu_Op op, int average, int algo,
                      const std::string &name, hipStream_t s)
{
    if (kf_session_device_mode_internal(cross) != 1) {
        return fail(KF_ERR_ARG, "kf_hier_all_reduce: the cross-host session must be device-mode");
    }
    int grank = 0, gsize = 0;
    (void)kf_session_info(cross, &grank, &gsize, nullptr, nullptr, nullptr);
    std::vector<int> host(gsize);
    (void)kf_session_hosts_internal(cross, host.data());
    const int H = *std::max_element(host.begin(), host.end()) + 1;
    std::vector<std::vector<int>> members(H);  // global ranks per host, in order
    std::vector<int> lrank(gsize);
    for (int g = 0; g < gsize; ++g) {
        lrank[g] = static_cast<int>(members[host[g]].size());
        members[host[g]].push_back(g);
    }
    if (lrank[grank] != rank || static_cast<int>(members[host[grank]].size()) != world) {
        return fail(KF_ERR_ARG, "kf_hier_all_reduce: the local exchange must hold this host's "
                                "ranks of the session, in its order");
    }
    bool equal = true;
    for (auto &m : members) equal = equal && m.size() == members[0].size();
    const int W = world;
    const int sz = tsize(dt);
    char *out    = static_cast<char *>(recv);
    std::vector<int32_t> forest(gsize);
    int rc = KF_OK;
    auto scale = [&](char *p, size_t n) -> int {
        if (!average || !n) return KF_OK;
        const int e = kf_bucket_div(p, n, dt, gsize, s);
        return e == KF_OK ? KF_OK : fail(e, "kf_hier_all_reduce: / np");
    };
    if (equal) {
        // one tree per local rank: the ranks holding the same shard, rooted
        // at host 0's (graph.go:46-62's forest array)
        for (int g = 0; g < gsize; ++g) forest[g] = members[0][lrank[g]];
        const size_t q = count / W, t = count % W;
        rc = batch(&send, &recv, &count, 1, dt, op, 0, algo, s, nullptr, 3);
        if (rc == KF_OK && q) {
            char *sh = out + rank * q * sz;
            rc = kf_session_subset_all_reduce(cross, sh, sh, q, dt, op, forest.data(),
                                              (name + "/shard").c_str(), s);
            if (rc != KF_OK) rc = fail(rc, std::string("cross-host shard all-reduce: ") +
                                               kf_session_last_error());
            if (rc == KF_OK) rc = scale(sh, q);
        }
        if (rc == KF_OK && t) {  // every local rank holds its host's tail sum
            char *tl = out + q * W * sz;
            rc = kf_session_subset_all_reduce(cross, tl, tl, t, dt, op, forest.data(),
                                              (name + "/tail").c_str(), s);
            if (rc != KF_OK) rc = fail(rc, std::string("cross-host tail all-reduce: ") +
                                               kf_session_last_error());
            if (rc == KF_OK) rc = scale(tl, t);
        }
        if (rc == KF_OK) rc = batch(&recv, &recv, &count, 1, dt, op, 0, algo, s, nullptr, 4);
        return rc;
    }
    // hosts of different sizes: the reference's structure (collective.cpp:
    // 144-160) — host all-reduce, the hosts' first ranks across, host broadcast
    for (int g = 0; g < gsize; ++g) forest[g] = lrank[g] == 0 ? members[0][0] : g;
    rc = batch(&send, &recv, &count, 1, dt, op, 0, algo, s);
    if (rc == KF_OK) {
        rc = kf_session_subset_all_reduce(cross, recv, recv, count, dt, op, forest.data(),
                                          name.c_str(), s);
        if (rc != KF_OK) rc = fail(rc, std::string("cross-host all-reduce: ") + kf_session_last_error());
    }
    if (rc == KF_OK && rank == 0) rc = scale(out, count);
    if (rc == KF_OK && W > 1 && !(builtin && W == 1) && count) {
        const int e = T->broadcast(recv, recv, count * sz, 0, comm, s);
        if (e != 0) rc = tfail(e, "host broadcast");
    }
    return rc;
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
        if (rc == KF_OK && T->async_error(comm) != 0) rc = KF_ERR_RCCL;
        if (d.done) d.done(rc, d.arg);
        lk.lock();
        if (rc != KF_OK && sstatus == KF_OK) {
            sstatus = rc;
            if (serr.empty()) serr = "an issued all-reduce failed on the device or in the transport";
        }
        ++completed;
        scv.notify_all();
    }
}

// ---------------------------------------------------------------------------
// name-keyed all-reduce
//
// Every cycle, each rank that has work (names started and not yet issued)
// all-gathers one control row over the control communicator: the names it
// started since its last row (hash pair, count, dtype/op signature). Every
// rank sees the same rows, so every rank counts the same reporters per name
// and finds the same names complete (reported by all ranks) in the same
// cycle; those are issued in rank 0's start order. A rank with nothing to do
// does not enter a cycle: its peers wait in the all-gather until it starts a
// name, which it must (same name set on every rank). Cycles that carry no
// news back off (50 us doubling to 1 ms) until a local start arrives.
// ---------------------------------------------------------------------------
int kf_exchange::start_named()
{
    if (nready) return KF_OK;
    // the built-in transport's single rank has nothing to agree; any other
    // transport negotiates even alone, so a one-GPU box runs the control
    // communicator through it (tests/c/kf_testing.cpp's one-rank librccl)
    if (world > 1 || !builtin) {
        int st = KF_OK;
        ctrl   = split(0, rank, &st);
        if (!ctrl) return st != KF_OK ? st : fail(KF_ERR_RCCL, "control communicator");
        KF_HIP(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
        KF_HIP(hipMalloc(&cdev, kCtrlRow * (world + 1)));
        KF_HIP(hipHostMalloc(&chost, kCtrlRow * (world + 1), hipHostMallocDefault));
    }
    KF_HIP(hipStreamCreateWithFlags(&nstream, hipStreamNonBlocking));
    const char *tr = std::getenv("KUNGFU_AMD_TRACE_NAMED");
    ntrace         = tr && tr[0] == '1';
    nready     = true;
    negotiator = std::thread([this] { negotiate_loop(); });
    nfinisher  = std::thread([this] { finish_loop(); });
    return KF_OK;
}

// every task still waiting fails (a broken control channel, or shutdown)
void kf_exchange::fail_outstanding(int rc, const std::string &why)
{
    std::lock_guard<std::mutex> lk(nmu);
    nbroken = true;
    for (auto &kv : nwait) {
        ndq.push_back(Done{nullptr, kv.second.done, kv.second.arg, rc, kv.second.ready, why});
    }
    nwait.clear();
    nfresh.clear();
    nhash.clear();
    ncv.notify_all();
}

void kf_exchange::negotiate_loop()
{
    (void)hipSetDevice(device);
    const int W         = world;
    const bool negotiate = ctrl != nullptr;
    struct Seen {
        int n        = 0;
        uint32_t sig = 0;
        uint64_t count = 0, key0 = 0;
        bool bad = false;
    };
    std::map<std::pair<uint64_t, uint64_t>, Seen> seen;
    uint64_t cycle = 0;
    int idle       = 0;
    char *row      = static_cast<char *>(chost);
    char *all      = row ? row + kCtrlRow : nullptr;
    for (;;) {
        std::vector<std::pair<uint64_t, uint64_t>> complete;
        int sent = 0;
        {
            std::unique_lock<std::mutex> lk(nmu);
            ncv.wait(lk, [&] { return nstop || !nfresh.empty() || !nwait.empty(); });
            if (nstop) return;
            if (idle > 0 && nfresh.empty()) {
                const auto us = std::chrono::microseconds(std::min(1000, 50 << std::min(idle - 1, 5)));
                ncv.wait_for(lk, us, [&] { return nstop || !nfresh.empty(); });
                if (nstop) return;
            }
            if (!negotiate) {  // one rank, built-in transport: issue in start order
                for (; !nfresh.empty(); nfresh.pop_front()) {
                    const NamedTask &t = nwait.at(nfresh.front());
                    complete.emplace_back(t.h1, t.h2);
                }
            } else {
                auto *ent = reinterpret_cast<CtrlEntry *>(row);
                for (; !nfresh.empty() && sent < kCtrlMax; nfresh.pop_front()) {
                    const NamedTask &t = nwait.at(nfresh.front());
                    ent[1 + sent++]    = CtrlEntry{t.h1, t.h2, t.count,
                                                task_sig(t.dt, t.op, t.average, t.algo), 0};
                }
                ent[0] = CtrlEntry{static_cast<uint64_t>(sent), 0, 0, 0, 0};
            }
        }
        bool news = !complete.empty();
        if (negotiate) {
            int rc        = KF_OK;
            char *d       = static_cast<char *>(cdev);
            hipError_t e  = hipMemcpyAsync(d, row, kCtrlRow, hipMemcpyHostToDevice, cstream);
            if (e != hipSuccess) rc = hip_fail(e, "control row H2D");
            if (rc == KF_OK) {
                const int t = T->all_gather(d, d + kCtrlRow, kCtrlRow, ctrl->comm, cstream);
                if (t != 0) rc = tfail(t, "control all_gather");
            }
            if (rc == KF_OK) {
                e = hipMemcpyAsync(all, d + kCtrlRow, kCtrlRow * W, hipMemcpyDeviceToHost, cstream);
                if (e == hipSuccess) e = hipStreamSynchronize(cstream);
                if (e != hipSuccess) rc = hip_fail(e, "control rows D2H");
            }
            if (rc != KF_OK) {
                fail_outstanding(rc, "name negotiation failed: " + t_ex_error);
                return;
            }
            for (int j = 0; j < W; ++j) {
                const auto *ent = reinterpret_cast<const CtrlEntry *>(all + j * kCtrlRow);
                const int n     = static_cast<int>(std::min<uint64_t>(ent[0].h1, kCtrlMax));
                news            = news || n > 0;
                for (int i = 0; i < n; ++i) {
                    const CtrlEntry &c = ent[1 + i];
                    Seen &s            = seen[{c.h1, c.h2}];
                    if (s.n == 0) {
                        s.sig   = c.sig;
                        s.count = c.count;
                    } else if (s.sig != c.sig || s.count != c.count) {
                        s.bad = true;
                    }
                    if (j == 0) s.key0 = cycle * (kCtrlMax + 1) + i;
                    if (++s.n == W) complete.emplace_back(c.h1, c.h2);
                }
            }
            if (ntrace) {
                std::string line = "[kf named] rank " + std::to_string(rank) + " cycle " +
                                   std::to_string(cycle) + " rows:";
                for (int j = 0; j < W; ++j) {
                    const auto *ent = reinterpret_cast<const CtrlEntry *>(all + j * kCtrlRow);
                    line += " " + std::to_string(ent[0].h1);
                    for (uint64_t i = 0; i < std::min<uint64_t>(ent[0].h1, kCtrlMax); ++i) {
                        line += ":" + std::to_string(ent[1 + i].h1 % 1000);
                    }
                }
                line += " complete " + std::to_string(complete.size()) + " seen " +
                        std::to_string(seen.size());
                std::fprintf(stderr, "%s\n", line.c_str());
            }
            // rank 0's start order (NCCLScheduler::Reset adopts rank 0's
            // arrival order the same way, scheduler.cpp:96-118)
            std::sort(complete.begin(), complete.end(), [&](const auto &x, const auto &y) {
                return seen[x].key0 < seen[y].key0;
            });
            ++cycle;
        }
        idle = news ? 0 : idle + 1;
        if (complete.empty()) continue;

        // the completed tasks, in issue order
        std::vector<NamedTask> ts;
        std::vector<bool> bad;
        {
            std::lock_guard<std::mutex> lk(nmu);
            for (const auto &h : complete) {
                auto hn = nhash.find(h);
                if (hn == nhash.end()) {  // cannot happen: this rank reported it
                    std::fprintf(stderr, "[kf named] rank %d: completed name not outstanding\n",
                                 rank);
                    continue;
                }
                auto it = nwait.find(hn->second);
                ts.push_back(it->second);
                nwait.erase(it);
                nhash.erase(hn);
                auto sn = seen.find(h);
                bad.push_back(sn != seen.end() && sn->second.bad);
                if (sn != seen.end()) seen.erase(sn);
            }
        }
        // runs of one dtype / op / average / algo go out as one batched call
        for (size_t i = 0; i < ts.size();) {
            if (bad[i]) {
                std::lock_guard<std::mutex> lk(nmu);
                ndq.push_back(Done{nullptr, ts[i].done, ts[i].arg, KF_ERR_ARG, ts[i].ready,
                                   "named all-reduce '" + ts[i].name +
                                       "': count, dtype, op or average differ across ranks"});
                ncv.notify_all();
                ++i;
                continue;
            }
            size_t j = i + 1;
            while (j < ts.size() && !bad[j] && ts[j].dt == ts[i].dt && ts[j].op == ts[i].op &&
                   ts[j].average == ts[i].average && ts[j].algo == ts[i].algo) {
                ++j;
            }
            std::vector<const void *> snd;
            std::vector<void *> rcv;
            std::vector<size_t> cnt;
            int rc = KF_OK;
            for (size_t k = i; k < j; ++k) {
                if (hipStreamWaitEvent(nstream, ts[k].ready, 0) != hipSuccess && rc == KF_OK) {
                    rc = fail(KF_ERR_HIP, "hipStreamWaitEvent(start)");
                }
                snd.push_back(ts[k].send);
                rcv.push_back(ts[k].recv);
                cnt.push_back(ts[k].count);
            }
            if (ntrace) {
                std::string line = "[kf named] rank " + std::to_string(rank) + " cycle " +
                                   std::to_string(cycle) + " batch:";
                for (size_t k = i; k < j; ++k) line += " " + ts[k].name;
                std::fprintf(stderr, "%s\n", line.c_str());
            }
            if (rc == KF_OK) {
                std::lock_guard<std::mutex> g(mu);
                rc = batch(snd.data(), rcv.data(), cnt.data(), static_cast<int>(j - i), ts[i].dt,
                           ts[i].op, ts[i].average, ts[i].algo, nstream);
            }
            const std::string why = rc == KF_OK ? std::string() : t_ex_error;
            std::lock_guard<std::mutex> lk(nmu);
            for (size_t k = i; k < j; ++k) {
                hipEvent_t ev = nullptr;
                int st        = rc;
                if (st == KF_OK &&
                    (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
                     hipEventRecord(ev, nstream) != hipSuccess)) {
                    st = KF_ERR_HIP;
                }
                ndq.push_back(Done{ev, ts[k].done, ts[k].arg, st, ts[k].ready,
                                   st == KF_OK ? std::string() : (why.empty() ? "hipEventRecord" : why)});
            }
            ncv.notify_all();
            i = j;
        }
    }
}

// done(status, arg) once each issued named all-reduce finished on the device
void kf_exchange::finish_loop()
{
    (void)hipSetDevice(device);
    std::unique_lock<std::mutex> lk(nmu);
    for (;;) {
        ncv.wait(lk, [&] { return nstop || !ndq.empty(); });
        if (ndq.empty() && nstop) return;
        Done d = ndq.front();
        ndq.pop_front();
        lk.unlock();
        int rc = d.status;
        if (d.ev) {
            if (hipEventSynchronize(d.ev) != hipSuccess) {
                rc    = KF_ERR_HIP;
                d.why = "the all-reduce failed on the device";
            }
            (void)hipEventDestroy(d.ev);
        }
        if (rc == KF_OK && T->async_error(comm) != 0) {
            rc    = KF_ERR_RCCL;
            d.why = "asynchronous transport error";
        }
        if (d.ready) (void)hipEventDestroy(d.ready);
        t_ex_error = d.why;
        if (d.done) d.done(rc, d.arg);
        lk.lock();
        if (rc != KF_OK && nstatus == KF_OK) {
            nstatus = rc;
            nerr    = d.why;
        }
        ++nfinished;
        ncv.notify_all();
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
    {
        std::lock_guard<std::mutex> lk(nmu);
        nstop = true;
    }
    ncv.notify_all();
    if (negotiator.joinable()) negotiator.join();
    if (nfinisher.joinable()) nfinisher.join();
    DeviceGuard g(device);
    delete ctrl;
    if (comm) T->destroy(comm);
    if (ws) (void)hipFree(ws);
    if (ws_ev) (void)hipEventDestroy(ws_ev);
    if (own) (void)hipStreamDestroy(own);
    if (comp) (void)hipStreamDestroy(comp);
    if (nstream) (void)hipStreamDestroy(nstream);
    if (cstream) (void)hipStreamDestroy(cstream);
    if (cdev) (void)hipFree(cdev);
    if (chost) (void)hipHostFree(chost);
    for (auto e : pev) (void)hipEventDestroy(e);
    for (auto &m : marks_used) marks_free.push_back(m);
    for (auto &m : marks_free)
        for (auto e : m.e) (void)hipEventDestroy(e);
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

static bool device_ok(int device)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev) {
        fail(KF_ERR_NO_DEVICE, "no HIP device " + std::to_string(device));
        return false;
    }
    return true;
}

kf_exchange_t *kf_exchange_create(const void *id, int rank, int world, int device)
{
    return kf_exchange_create_timeout(id, rank, world, device, -1);
}

// ncclCommInitRank blocks until every rank has joined. With a timeout it runs
// on a helper thread; if the time passes first the call fails with
// KF_ERR_TIMEOUT and the helper is abandoned: it stays in the init until the
// missing ranks come (then it releases the communicator it got) or the
// process ends. RCCL's non-blocking init would make every later call of the
// communicator non-blocking as well, so it is not used.
kf_exchange_t *kf_exchange_create_timeout(const void *id, int rank, int world, int device,
                                          int timeout_ms)
{
    if (!id || world < 1 || rank < 0 || rank >= world || device < 0) {
        fail(KF_ERR_ARG, "kf_exchange_create: bad arguments");
        return nullptr;
    }
    if (need_rccl() != KF_OK || !device_ok(device)) return nullptr;
    DeviceGuard g(device);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    ncclResult_t e  = ncclSuccess;
    if (timeout_ms < 0) {
        e = rccl().CommInitRank(&comm, world, u, rank);
    } else {
        struct Init {
            std::mutex m;
            std::condition_variable cv;
            bool done = false, abandoned = false;
            ncclComm_t comm = nullptr;
            ncclResult_t e  = ncclSuccess;
        };
        auto job = std::make_shared<Init>();
        std::thread([job, u, world, rank, device] {
            (void)hipSetDevice(device);
            ncclComm_t c     = nullptr;
            ncclResult_t r   = rccl().CommInitRank(&c, world, u, rank);
            std::lock_guard<std::mutex> l(job->m);
            if (job->abandoned) {  // nobody waits for it any more
                if (r == ncclSuccess && c) (void)rccl().CommDestroy(c);
                return;
            }
            job->comm = c;
            job->e    = r;
            job->done = true;
            job->cv.notify_all();
        }).detach();
        std::unique_lock<std::mutex> l(job->m);
        if (!job->cv.wait_for(l, std::chrono::milliseconds(timeout_ms), [&] { return job->done; })) {
            job->abandoned = true;
            fail(KF_ERR_TIMEOUT, "ncclCommInitRank: not every rank joined within " +
                                     std::to_string(timeout_ms) + " ms");
            return nullptr;
        }
        comm = job->comm;
        e    = job->e;
    }
    if (e != ncclSuccess) {
        nccl_fail(e, "ncclCommInitRank");
        return nullptr;
    }
    kf_exchange *ex = new_exchange(&kRcclOps, comm, true, rank, world, device);
    if (!ex) (void)rccl().CommDestroy(comm);
    return ex;
}

kf_exchange_t *kf_exchange_create_transport(const kf_transport_ops *ops, void *comm, int rank,
                                            int world, int device)
{
    if (!ops || !ops->group_start || !ops->group_end || !ops->reduce_scatter ||
        !ops->all_gather || !ops->all_to_all || !ops->broadcast || !ops->async_error ||
        !ops->destroy || world < 1 || rank < 0 || rank >= world || device < 0) {
        fail(KF_ERR_ARG, "kf_exchange_create_transport: bad arguments");
        return nullptr;
    }
    if (!device_ok(device)) return nullptr;
    DeviceGuard g(device);
    return new_exchange(ops, comm, false, rank, world, device);
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

kf_exchange_t *kf_exchange_split(kf_exchange_t *ex, int color, int key, int *status)
{
    int st = KF_OK;
    if (!status) status = &st;
    if (!ex) {
        *status = fail(KF_ERR_ARG, "kf_exchange_split: no exchange");
        return nullptr;
    }
    DeviceGuard g(ex->device);
    std::lock_guard<std::mutex> lk(ex->mu);
    return ex->split(color, key, status);
}

static int check_bucket_args(kf_exchange_t *ex, const void *const *sends, void *const *recvs,
                             const size_t *counts, int nb, KungFu_Datatype dt, KungFu_Op op,
                             int average);

kf_exchange_t *kf_exchange_create_local(kf_session_t *s, int device)
{
    int rank = 0, size = 0, lr = 0, ls = 0, hosts = 0;
    if (!s || kf_session_info(s, &rank, &size, &lr, &ls, &hosts) != KF_OK) {
        fail(KF_ERR_ARG, "kf_exchange_create_local: no session");
        return nullptr;
    }
    std::vector<int> host(size);
    (void)kf_session_hosts_internal(s, host.data());
    // [every host's id][one status byte per host]: the host's first rank
    // writes its host's id, or 1 in its host's status byte if it could not
    // make one, so every rank of that host fails with the reason instead of
    // calling the communicator init with an id that is all zeros
    const size_t idbytes = static_cast<size_t>(hosts) * KF_UNIQUE_ID_BYTES;
    const size_t bytes   = idbytes + static_cast<size_t>(hosts);
    std::vector<unsigned char> ids(bytes, 0);
    int rc = KF_OK;
    std::string why;
    if (lr == 0 && kf_exchange_unique_id(ids.data() + host[rank] * KF_UNIQUE_ID_BYTES) != KF_OK) {
        why = t_ex_error;
        rc  = KF_ERR_RCCL;
        ids[idbytes + host[rank]] = 1;
    }
    // every host's id in one all-reduce: one contributor per slot, so the sum is the id
    int e = KF_OK;
    if (kf_session_device_mode_internal(s) == 0) {
        e = kf_session_all_reduce(s, ids.data(), ids.data(), bytes, KungFu_UINT8, KungFu_SUM,
                                  "local nccl ids", nullptr);
    } else {
        DeviceGuard g(device);
        void *d = nullptr;
        if (hipMalloc(&d, bytes) != hipSuccess) {
            fail(KF_ERR_HIP, "kf_exchange_create_local: hipMalloc");
            return nullptr;
        }
        e = hipMemcpy(d, ids.data(), bytes, hipMemcpyHostToDevice) == hipSuccess ? KF_OK : KF_ERR_HIP;
        if (e == KF_OK) {
            e = kf_session_all_reduce(s, d, d, bytes, KungFu_UINT8, KungFu_SUM, "local nccl ids",
                                      nullptr);
        }
        if (e == KF_OK && hipMemcpy(ids.data(), d, bytes, hipMemcpyDeviceToHost) != hipSuccess) {
            e = KF_ERR_HIP;
        }
        (void)hipFree(d);
    }
    if (e != KF_OK) {
        fail(e, std::string("kf_exchange_create_local: sharing the ids: ") + kf_session_last_error());
        return nullptr;
    }
    if (rc != KF_OK) {
        fail(rc, why);
        return nullptr;
    }
    if (ids[idbytes + host[rank]] != 0) {
        fail(KF_ERR_RCCL, "kf_exchange_create_local: this host's first rank could not create "
                          "the RCCL id (its own error says why)");
        return nullptr;
    }
    return kf_exchange_create(ids.data() + host[rank] * KF_UNIQUE_ID_BYTES, lr, ls, device);
}

int kf_hier_all_reduce(kf_exchange_t *local, kf_session_t *cross, const void *send, void *recv,
                       size_t count, KungFu_Datatype dt, KungFu_Op op, int average, int algo,
                       const char *name, void *stream)
{
    if (!cross || !name) return fail(KF_ERR_ARG, "kf_hier_all_reduce: bad arguments");
    int rc = check_bucket_args(local, &send, &recv, &count, 1, dt, op, average);
    if (rc != KF_OK || count == 0) return rc;
    DeviceGuard g(local->device);
    std::lock_guard<std::mutex> lk(local->mu);
    return local->hier(cross, send, recv, count, dt, op, average, algo, name,
                       static_cast<hipStream_t>(stream));
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

int kf_exchange_set_timing(kf_exchange_t *ex, int on)
{
    if (!ex) return fail(KF_ERR_ARG, "kf_exchange_set_timing: null exchange");
    std::lock_guard<std::mutex> lk(ex->mu);
    DeviceGuard g(ex->device);
    const int rc = ex->harvest_marks();  // what was queued before counts for the old window
    ex->timing   = on != 0;
    for (double &v : ex->phase_us) v = 0;
    ex->timed_calls = ex->untimed_calls = 0;
    return rc;
}

int kf_exchange_phase_times(kf_exchange_t *ex, double *us, int64_t *calls, int64_t *untimed)
{
    if (!ex || !us) return fail(KF_ERR_ARG, "kf_exchange_phase_times: null argument");
    std::lock_guard<std::mutex> lk(ex->mu);
    DeviceGuard g(ex->device);
    const int rc = ex->harvest_marks();
    for (int k = 0; k < 4; ++k) us[k] = ex->phase_us[k];
    if (calls) *calls = ex->timed_calls;
    if (untimed) *untimed = ex->untimed_calls;
    return rc;
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
            const int t = ex->T->broadcast(d, d, bytes, 0, ex->comm, ex->own);
            if (t != 0) rc = ex->tfail(t, "broadcast(order)");
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

int kf_exchange_all_reduce_named(kf_exchange_t *ex, const char *name, const void *send, void *recv,
                                 size_t count, KungFu_Datatype dt, KungFu_Op op, int average,
                                 int algo, void *stream, kf_done_fn done, void *arg)
{
    if (!ex || !name) return fail(KF_ERR_ARG, "bad arguments");
    size_t c = count;
    int rc   = check_bucket_args(ex, &send, &recv, &c, 1, dt, op, average);
    if (rc != KF_OK) return rc;
    if (algo < KF_ALGO_AUTO || algo > KF_ALGO_REDUCE_SCATTER_AVG) return fail(KF_ERR_ARG, "unknown algo");
    DeviceGuard g(ex->device);
    {
        std::lock_guard<std::mutex> lk(ex->mu);
        rc = ex->start_named();
        if (rc != KF_OK) return rc;
    }
    NamedTask t;
    t.name = name;
    if (t.name.empty()) {  // the blocking op's anonymous call: paired by call order
        std::lock_guard<std::mutex> lk(ex->nmu);
        t.name = "::anon::" + std::to_string(ex->anon_seq++);
    }
    t.h1 = fnv1a(t.name.c_str(), 0xcbf29ce484222325ull);
    t.h2 = fnv1a(t.name.c_str(), 0x6c62272e07bb0142ull) ^ (t.name.size() * 0x9e3779b97f4a7c15ull);
    t.send    = send;
    t.recv    = recv;
    t.count   = count;
    t.dt      = dt;
    t.op      = op;
    t.average = average ? 1 : 0;
    t.algo    = algo;
    t.done    = done;
    t.arg     = arg;
    KF_HIP(hipEventCreateWithFlags(&t.ready, hipEventDisableTiming));
    hipError_t e = hipEventRecord(t.ready, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
        (void)hipEventDestroy(t.ready);
        return hip_fail(e, "hipEventRecord(start)");
    }
    std::lock_guard<std::mutex> lk(ex->nmu);
    rc = KF_OK;
    if (ex->nbroken) {
        rc = fail(KF_ERR_RCCL, "the name negotiation has failed on this exchange");
    } else if (ex->nwait.count(t.name)) {
        rc = fail(KF_ERR_ARG, "name already outstanding: " + t.name);
    } else if (ex->nhash.count({t.h1, t.h2})) {
        rc = fail(KF_ERR_ARG, "name hash collides with an outstanding name: " + t.name);
    }
    if (rc != KF_OK) {
        (void)hipEventDestroy(t.ready);
        return rc;
    }
    const std::string key   = t.name;
    ex->nhash[{t.h1, t.h2}] = key;
    ex->nfresh.push_back(key);
    ex->nwait.emplace(key, std::move(t));
    ex->nstarted++;
    ex->ncv.notify_all();
    return KF_OK;
}

int kf_exchange_wait_named(kf_exchange_t *ex)
{
    if (!ex) return KF_ERR_ARG;
    if (std::this_thread::get_id() == ex->nfinisher.get_id()) {
        return fail(KF_ERR_ARG, "kf_exchange_wait_named from a done callback");
    }
    std::unique_lock<std::mutex> lk(ex->nmu);
    ex->ncv.wait(lk, [&] { return ex->nfinished == ex->nstarted; });
    const int rc = ex->nstatus;
    if (rc != KF_OK) t_ex_error = ex->nerr;
    ex->nstatus = KF_OK;
    ex->nerr.clear();
    return rc;
}

int kf_exchange_check(kf_exchange_t *ex)
{
    if (!ex) return KF_ERR_ARG;
    const int e = ex->T->async_error(ex->comm);
    if (e != 0) return ex->tfail(e, "asynchronous transport error");
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

int kf_exchange_transport_info(kf_exchange_t *ex, int *comm_count, int *rccl_version)
{
    if (!ex) return KF_ERR_ARG;
    if (comm_count) *comm_count = -1;
    if (rccl_version) *rccl_version = 0;
    if (!ex->builtin) return KF_OK;  // a host's own transport: nothing to ask RCCL
    const Rccl &r = rccl();
    if (!r.ok) return fail(KF_ERR_RCCL, r.why);
    if (comm_count && r.CommCount) {
        int n = -1;
        const ncclResult_t e = r.CommCount(static_cast<ncclComm_t>(ex->comm), &n);
        if (e != ncclSuccess) return nccl_fail(e, "ncclCommCount");
        *comm_count = n;
    }
    if (rccl_version && r.GetVersion) {
        int v = 0;
        const ncclResult_t e = r.GetVersion(&v);
        if (e != ncclSuccess) return nccl_fail(e, "ncclGetVersion");
        *rccl_version = v;
    }
    return KF_OK;
}

void kf_exchange_destroy(kf_exchange_t *ex) { delete ex; }

const char *kf_exchange_last_error(void) { return t_ex_error.c_str(); }

}  // extern "C"
