// kf_testing.cpp — test-only transports for libkungfu_amd.so's exchange
// (tests/c/kf_testing.h). Test infrastructure: nothing in kungfu_amd/ links or
// loads this library.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "kf_testing.h"

namespace
{
thread_local std::string t_err;

// ---------------------------------------------------------------------------
// loopback: every collective is a rendezvous of the group's threads
// ---------------------------------------------------------------------------
enum { LB_OK = 0, LB_HIP = 1, LB_DTYPE = 2, LB_ARG = 3, LB_INJECTED = 4 };

struct LoopSlot {
    int arrived = 0, left = 0;
    bool done   = false;
    std::vector<const void *> send;
    std::vector<void *> recv;
};

struct LoopGroup {
    int world;
    int64_t fail_at = -1;  // kf_loopback_fail_at: this call index of every rank fails
    std::mutex mu;
    std::condition_variable cv;
    std::map<uint64_t, LoopSlot> slots;
    std::vector<std::unique_ptr<LoopGroup>> children;  // made by splits
    explicit LoopGroup(int w) : world(w) {}
};

struct LoopComm {
    LoopGroup *g;
    int rank;
    uint64_t seq   = 0;
    int64_t calls  = 0;  // collective calls made (injection counter)
};

size_t dsize(KungFu_Datatype dt)
{
    switch (dt) {
    case KungFu_UINT8: case KungFu_INT8: return 1;
    case KungFu_UINT16: case KungFu_INT16: case KungFu_FLOAT16: case KungFu_BFLOAT16: return 2;
    case KungFu_UINT32: case KungFu_INT32: case KungFu_FLOAT: return 4;
    default: return 8;
    }
}

template <typename T>
void host_fold(const std::vector<std::vector<char>> &in, size_t off, size_t n, KungFu_Op op,
               char *out)
{
    if (static_cast<int>(op) == KF_TRANSPORT_OP_AVG) {  // ncclAvg's float form: premultiply
        const T w = static_cast<T>(1) / static_cast<T>(in.size());
        for (size_t i = 0; i < n; ++i) {
            T a = reinterpret_cast<const T *>(in[0].data() + off)[i] * w;
            for (size_t j = 1; j < in.size(); ++j) {
                a = static_cast<T>(a + reinterpret_cast<const T *>(in[j].data() + off)[i] * w);
            }
            reinterpret_cast<T *>(out)[i] = a;
        }
        return;
    }
    for (size_t i = 0; i < n; ++i) {
        T a = reinterpret_cast<const T *>(in[0].data() + off)[i];
        for (size_t j = 1; j < in.size(); ++j) {
            const T b = reinterpret_cast<const T *>(in[j].data() + off)[i];
            if (op == KungFu_SUM) a = static_cast<T>(a + b);
            else if (op == KungFu_PROD) a = static_cast<T>(a * b);
            else if (op == KungFu_MIN) a = (b < a) ? b : a;
            else a = (a < b) ? b : a;
        }
        reinterpret_cast<T *>(out)[i] = a;
    }
}

// rendezvous; `move` runs once, on the last rank to arrive, with every rank's
// posted buffers. stream == nullptr: nothing to drain first.
template <typename F>
int loop_collective(void *comm, const void *send, void *recv, void *stream, F move)
{
    auto *c = static_cast<LoopComm *>(comm);
    // every rank fails the same call before its rendezvous, so none waits
    if (c->calls++ == c->g->fail_at) return LB_INJECTED;
    if (stream && hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess) return LB_HIP;
    LoopGroup *g = c->g;
    std::unique_lock<std::mutex> lk(g->mu);
    LoopSlot &sl       = g->slots[c->seq];
    const uint64_t seq = c->seq++;
    if (sl.send.empty()) {
        sl.send.assign(g->world, nullptr);
        sl.recv.assign(g->world, nullptr);
    }
    sl.send[c->rank] = send;
    sl.recv[c->rank] = recv;
    int rc           = LB_OK;
    if (++sl.arrived == g->world) {
        rc = move(sl.send, sl.recv);
        // a device-to-device hipMemcpy returns once queued on the null
        // stream, not once landed; the ranks' non-blocking streams do not
        // order behind it, so the copies must be complete before anyone reads
        if (hipStreamSynchronize(nullptr) != hipSuccess && rc == LB_OK) rc = LB_HIP;
        sl.done = true;
        g->cv.notify_all();
    } else {
        g->cv.wait(lk, [&] { return sl.done; });
    }
    if (++sl.left == g->world) g->slots.erase(seq);
    return rc;
}

int lb_reduce_scatter(const void *send, void *recv, size_t count, KungFu_Datatype dt, KungFu_Op op,
                      void *comm, void *stream)
{
    return loop_collective(comm, send, recv, stream, [&](const std::vector<const void *> &sd,
                                                         const std::vector<void *> &rv) {
        if (dt == KungFu_FLOAT16 || dt == KungFu_BFLOAT16 || dt == KungFu_UINT16 ||
            dt == KungFu_INT16) {
            return int(LB_DTYPE);
        }
        if (static_cast<int>(op) == KF_TRANSPORT_OP_AVG && dt != KungFu_FLOAT && dt != KungFu_DOUBLE) {
            return int(LB_DTYPE);  // the loopback averages floats only
        }
        const size_t sz = dsize(dt), W = sd.size();
        std::vector<std::vector<char>> in(W, std::vector<char>(count * W * sz));
        for (size_t j = 0; j < W; ++j) {
            if (hipMemcpy(in[j].data(), sd[j], count * W * sz, hipMemcpyDeviceToHost) != hipSuccess)
                return int(LB_HIP);
        }
        std::vector<char> out(count * sz);
        for (size_t r = 0; r < W; ++r) {
            const size_t off = r * count * sz;
            switch (dt) {
            case KungFu_INT8: host_fold<int8_t>(in, off, count, op, out.data()); break;
            case KungFu_UINT8: host_fold<uint8_t>(in, off, count, op, out.data()); break;
            case KungFu_INT32: host_fold<int32_t>(in, off, count, op, out.data()); break;
            case KungFu_UINT32: host_fold<uint32_t>(in, off, count, op, out.data()); break;
            case KungFu_INT64: host_fold<int64_t>(in, off, count, op, out.data()); break;
            case KungFu_UINT64: host_fold<uint64_t>(in, off, count, op, out.data()); break;
            case KungFu_FLOAT: host_fold<float>(in, off, count, op, out.data()); break;
            default: host_fold<double>(in, off, count, op, out.data()); break;
            }
            if (hipMemcpy(rv[r], out.data(), count * sz, hipMemcpyHostToDevice) != hipSuccess)
                return int(LB_HIP);
        }
        return int(LB_OK);
    });
}

int lb_all_gather(const void *send, void *recv, size_t b, void *comm, void *stream)
{
    return loop_collective(comm, send, recv, stream, [&](const std::vector<const void *> &sd,
                                                         const std::vector<void *> &rv) {
        const size_t W = sd.size();
        for (size_t r = 0; r < W; ++r) {
            for (size_t j = 0; j < W; ++j) {
                char *dst = static_cast<char *>(rv[r]) + j * b;
                if (dst == sd[j]) continue;  // in place
                if (hipMemcpy(dst, sd[j], b, hipMemcpyDeviceToDevice) != hipSuccess) return int(LB_HIP);
            }
        }
        return int(LB_OK);
    });
}

int lb_all_to_all(const void *send, void *recv, size_t b, void *comm, void *stream)
{
    return loop_collective(comm, send, recv, stream, [&](const std::vector<const void *> &sd,
                                                         const std::vector<void *> &rv) {
        const size_t W = sd.size();
        for (size_t r = 0; r < W; ++r) {
            for (size_t j = 0; j < W; ++j) {
                if (hipMemcpy(static_cast<char *>(rv[r]) + j * b,
                              static_cast<const char *>(sd[j]) + r * b, b,
                              hipMemcpyDeviceToDevice) != hipSuccess)
                    return int(LB_HIP);
            }
        }
        return int(LB_OK);
    });
}

int lb_broadcast(const void *send, void *recv, size_t b, int root, void *comm, void *stream)
{
    return loop_collective(comm, send, recv, stream, [&](const std::vector<const void *> &sd,
                                                         const std::vector<void *> &rv) {
        for (size_t r = 0; r < rv.size(); ++r) {
            if (rv[r] == sd[root]) continue;
            if (hipMemcpy(rv[r], sd[root], b, hipMemcpyDeviceToDevice) != hipSuccess) return int(LB_HIP);
        }
        return int(LB_OK);
    });
}

// ncclCommSplit's contract: ranks of one color form a group ordered by
// (key, rank); color < 0 joins none
int lb_split(void *comm, int color, int key, void **newcomm)
{
    auto *c           = static_cast<LoopComm *>(comm);
    const int32_t mine[2] = {color, key};
    *newcomm          = nullptr;
    return loop_collective(comm, mine, newcomm, nullptr, [&](const std::vector<const void *> &sd,
                                                             const std::vector<void *> &rv) {
        const int W = static_cast<int>(sd.size());
        std::map<int, std::vector<std::pair<int32_t, int>>> by;
        for (int j = 0; j < W; ++j) {
            const auto *ck = static_cast<const int32_t *>(sd[j]);
            if (ck[0] >= 0) by[ck[0]].emplace_back(ck[1], j);
        }
        for (auto &kv : by) {
            std::sort(kv.second.begin(), kv.second.end());
            c->g->children.emplace_back(new LoopGroup(static_cast<int>(kv.second.size())));
            LoopGroup *ng = c->g->children.back().get();
            for (size_t i = 0; i < kv.second.size(); ++i) {
                *static_cast<void **>(rv[kv.second[i].second]) =
                    new LoopComm{ng, static_cast<int>(i)};
            }
        }
        return int(LB_OK);
    });
}

int lb_nop(void *) { return LB_OK; }
int lb_async_error(void *) { return LB_OK; }
void lb_destroy(void *comm) { delete static_cast<LoopComm *>(comm); }
const char *lb_error_string(int code)
{
    switch (code) {
    case LB_HIP: return "loopback: a HIP copy failed";
    case LB_DTYPE: return "loopback: no reduce-scatter for this dtype";
    case LB_INJECTED: return "loopback: injected failure";
    default: return "loopback transport error";
    }
}

const kf_transport_ops kLoopOps = {
    lb_nop,       lb_nop,   lb_reduce_scatter, lb_all_gather, lb_all_to_all,
    lb_broadcast, lb_split, lb_async_error,    lb_destroy,    lb_error_string,
};

// ---------------------------------------------------------------------------
// rccl1: librccl's entry points with a one-rank communicator
// ---------------------------------------------------------------------------
struct R {
    decltype(&::ncclGetUniqueId) GetUniqueId;
    decltype(&::ncclCommInitRank) CommInitRank;
    decltype(&::ncclCommDestroy) CommDestroy;
    decltype(&::ncclCommGetAsyncError) CommGetAsyncError;
    decltype(&::ncclCommSplit) CommSplit;
    decltype(&::ncclReduceScatter) ReduceScatter;
    decltype(&::ncclAllGather) AllGather;
    decltype(&::ncclAllToAll) AllToAll;
    decltype(&::ncclBroadcast) Broadcast;
    decltype(&::ncclGroupStart) GroupStart;
    decltype(&::ncclGroupEnd) GroupEnd;
    decltype(&::ncclGetErrorString) GetErrorString;
};

const R *rcl()
{
    static const R *r = []() -> const R * {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return nullptr;
        static R x;
#define L(f, s)                                                                \
    x.f = reinterpret_cast<decltype(x.f)>(dlsym(h, #s));                       \
    if (!x.f) return nullptr;
        L(GetUniqueId, ncclGetUniqueId)
        L(CommInitRank, ncclCommInitRank)
        L(CommDestroy, ncclCommDestroy)
        L(CommGetAsyncError, ncclCommGetAsyncError)
        L(CommSplit, ncclCommSplit)
        L(ReduceScatter, ncclReduceScatter)
        L(AllGather, ncclAllGather)
        L(AllToAll, ncclAllToAll)
        L(Broadcast, ncclBroadcast)
        L(GroupStart, ncclGroupStart)
        L(GroupEnd, ncclGroupEnd)
        L(GetErrorString, ncclGetErrorString)
#undef L
        return &x;
    }();
    return r;
}

ncclComm_t C(void *c) { return static_cast<ncclComm_t>(c); }
hipStream_t S(void *s) { return static_cast<hipStream_t>(s); }

bool ntype(KungFu_Datatype dt, ncclDataType_t *t)
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
    default: return false;
    }
}

int r1_gs(void *) { return rcl()->GroupStart(); }
int r1_ge(void *) { return rcl()->GroupEnd(); }
int r1_rs(const void *s, void *r, size_t n, KungFu_Datatype dt, KungFu_Op op, void *c, void *st)
{
    ncclDataType_t t;
    if (!ntype(dt, &t)) return ncclInvalidArgument;
    const ncclRedOp_t o = static_cast<int>(op) == KF_TRANSPORT_OP_AVG ? ncclAvg
                          : op == KungFu_MIN ? ncclMin : op == KungFu_MAX ? ncclMax
                          : op == KungFu_PROD ? ncclProd : ncclSum;
    return rcl()->ReduceScatter(s, r, n, t, o, C(c), S(st));
}
int r1_ag(const void *s, void *r, size_t b, void *c, void *st)
{
    return rcl()->AllGather(s, r, b, ncclUint8, C(c), S(st));
}
int r1_a2a(const void *s, void *r, size_t b, void *c, void *st)
{
    return rcl()->AllToAll(s, r, b, ncclUint8, C(c), S(st));
}
int r1_bc(const void *s, void *r, size_t b, int root, void *c, void *st)
{
    return rcl()->Broadcast(s, r, b, ncclUint8, root, C(c), S(st));
}
int r1_split(void *c, int color, int key, void **out)
{
    ncclComm_t n = nullptr;
    const int rc = rcl()->CommSplit(C(c), color < 0 ? NCCL_SPLIT_NOCOLOR : color, key, &n, nullptr);
    *out         = n;
    return rc;
}
int r1_err(void *c)
{
    ncclResult_t ae = ncclSuccess;
    const ncclResult_t r = rcl()->CommGetAsyncError(C(c), &ae);
    return r != ncclSuccess ? r : ae;
}
void r1_destroy(void *c) { (void)rcl()->CommDestroy(C(c)); }
const char *r1_str(int code) { return rcl()->GetErrorString(static_cast<ncclResult_t>(code)); }

const kf_transport_ops kRccl1Ops = {r1_gs, r1_ge,    r1_rs,  r1_ag,      r1_a2a,
                                    r1_bc, r1_split, r1_err, r1_destroy, r1_str};

}  // namespace

struct kf_loopback {
    LoopGroup g;
    explicit kf_loopback(int w) : g(w) {}
};

extern "C" {

kf_loopback_t *kf_loopback_create(int world)
{
    if (world < 1) return nullptr;
    return new kf_loopback(world);
}

void kf_loopback_destroy(kf_loopback_t *g) { delete g; }

void kf_loopback_fail_at(kf_loopback_t *g, int64_t call)
{
    if (g) g->g.fail_at = call;
}

kf_exchange_t *kf_exchange_create_loopback(kf_loopback_t *g, int rank, int device)
{
    if (!g || rank < 0 || rank >= g->g.world) {
        t_err = "kf_exchange_create_loopback: bad arguments";
        return nullptr;
    }
    auto *c           = new LoopComm{&g->g, rank};
    kf_exchange_t *ex = kf_exchange_create_transport(&kLoopOps, c, rank, g->g.world, device);
    if (!ex) {
        t_err = kf_exchange_last_error();
        delete c;
    }
    return ex;
}

kf_exchange_t *kf_exchange_create_rccl1(int device)
{
    if (!rcl()) {
        t_err = "librccl.so.1 not loadable";
        return nullptr;
    }
    if (hipSetDevice(device) != hipSuccess) {
        t_err = "hipSetDevice";
        return nullptr;
    }
    ncclUniqueId id;
    ncclComm_t c = nullptr;
    if (rcl()->GetUniqueId(&id) != ncclSuccess || rcl()->CommInitRank(&c, 1, id, 0) != ncclSuccess) {
        t_err = "one-rank ncclCommInitRank failed";
        return nullptr;
    }
    kf_exchange_t *ex = kf_exchange_create_transport(&kRccl1Ops, c, 0, 1, device);
    if (!ex) {
        t_err = kf_exchange_last_error();
        (void)rcl()->CommDestroy(c);
    }
    return ex;
}

const char *kf_testing_last_error(void) { return t_err.c_str(); }

}  // extern "C"
