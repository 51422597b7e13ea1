// torch_ops.cpp — the reference's torch extension surface with its
// signatures (srcs/cpp/src/torch/module_cuda.cpp:28-40,
// srcs/cpp/src/torch/ops/cuda/collective.cpp:20-55), over the C ABI of
// libkungfu_amd.so instead of a host round trip.
//
// The reference copies a CUDA tensor into a host buffer, all-reduces it there
// through Peer::GetDefault()->AllReduce keyed by the tensor's name, and copies
// it back (collective.cpp:24-29, 41-53). Here the process's exchange
// (kf_exchange_*: RCCL over xGMI for the bytes, the HIP kernels for the sum)
// reduces it in HBM, and the pairing across ranks is the reference's: by
// NAME, through kf_exchange_all_reduce_named, so ranks may start their
// tensors in different orders (the torch optimizer starts them in parameter
// or hook order, sync_sgd.py:12-22):
//
//   all_reduce_cuda(input, output, type, op)             collective.cpp:20-30
//       blocking; the reference names it "" and relies on call order, so
//       here every rank's k-th synchronous call is the name "::sync::k"
//   all_reduce_cuda_async(input, output, type, op, name) collective.cpp:32-55
//       -> int handle; wait_handle(h) / wait_all_handles(hs) block until done
//          (the reference's HandleManager, handler_manager.hpp:6-84) and
//          raise the failure if there was one
//
// The data moves after the work queued on torch's current stream before the
// call (an event recorded there), on the exchange's own stream, so it
// overlaps whatever the caller queues next.
//
// `type` is the tensor's x.type() string (torch/ops/clib.py maps
// 'torch.cuda.FloatTensor'; the reference converts only Float,
// collective.cpp:10-18 — here every dtype the exchange supports), `op` one of
// sum / min / max / prod (srcs/cpp/src/torch/common.cpp:41-46).
//
// Peer::GetDefault() is init_exchange(id, rank, size, device): the id is
// rank 0's kf_exchange_unique_id() bytes, shared by the caller (torch.distributed
// in kungfu_amd/torch/ops.py), as gpu_collective.cpp:190-200 shares it.
// bind_exchange(handle) makes an exchange built elsewhere (a C++ host's
// kf_exchange_create_session, kf_exchange_split, a host transport) the one
// this thread's ops use.
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "kungfu_amd.h"

namespace
{
kf_exchange_t *g_ex = nullptr;              // init_exchange's (Peer::GetDefault)
thread_local kf_exchange_t *t_ex = nullptr; // bind_exchange's, this thread only
std::mutex g_mu;

struct Pending {
    std::mutex m;
    std::condition_variable cv;
    bool done  = false;
    int status = KF_OK;
    std::string why;
    torch::Tensor input, output;  // alive until waited for (released with the GIL held)
};
std::map<int, std::shared_ptr<Pending>> g_handles;
int g_next = 0;
std::atomic<int> g_algo{KF_ALGO_AUTO};  // set_algo: the exchange schedule of every op

void check(int rc, const char *what)
{
    if (rc != KF_OK) {
        throw std::runtime_error(std::string(what) + " failed (status " + std::to_string(rc) +
                                 "): " + kf_exchange_last_error());
    }
}

kf_exchange_t *current()
{
    kf_exchange_t *ex = t_ex ? t_ex : g_ex;
    if (!ex) throw std::runtime_error("kungfu_amd: init_exchange() first");
    return ex;
}

// x.type() strings of CUDA tensors -> KungFu dtype codes (dtype.h:21-39)
KungFu_Datatype from_type(const std::string &type)
{
    static const std::map<std::string, KungFu_Datatype> m = {
        {"torch.cuda.FloatTensor", KungFu_FLOAT},   {"torch.cuda.DoubleTensor", KungFu_DOUBLE},
        {"torch.cuda.HalfTensor", KungFu_FLOAT16},  {"torch.cuda.BFloat16Tensor", KungFu_BFLOAT16},
        {"torch.cuda.IntTensor", KungFu_INT32},     {"torch.cuda.LongTensor", KungFu_INT64},
        {"torch.cuda.ShortTensor", KungFu_INT16},   {"torch.cuda.CharTensor", KungFu_INT8},
        {"torch.cuda.ByteTensor", KungFu_UINT8},
    };
    auto it = m.find(type);
    if (it == m.end()) throw std::runtime_error("kungfu_amd: not implemented for " + type);
    return it->second;
}

KungFu_Op from_op(const std::string &op)
{
    static const std::map<std::string, KungFu_Op> m = {
        {"sum", KungFu_SUM}, {"min", KungFu_MIN}, {"max", KungFu_MAX}, {"prod", KungFu_PROD}};
    auto it = m.find(op);
    if (it == m.end()) throw std::runtime_error("kungfu_amd: unknown op " + op);
    return it->second;
}

void on_done(int status, void *arg)
{
    auto *ref = static_cast<std::shared_ptr<Pending> *>(arg);
    std::shared_ptr<Pending> p = *ref;
    delete ref;
    {
        std::lock_guard<std::mutex> lk(p->m);
        p->status = status;
        if (status != KF_OK) p->why = kf_exchange_last_error();  // set for done()
        p->done = true;
    }
    p->cv.notify_all();
}

std::shared_ptr<Pending> start(const torch::Tensor &input, torch::Tensor &output,
                               const std::string &type, const std::string &op_name,
                               const std::string &name)
{
    kf_exchange_t *ex = current();
    if (!input.is_cuda() || !output.is_cuda()) {
        throw std::runtime_error("kungfu_amd: all_reduce_cuda needs CUDA tensors");
    }
    if (!input.is_contiguous() || !output.is_contiguous() || input.numel() != output.numel() ||
        input.scalar_type() != output.scalar_type()) {
        throw std::runtime_error("kungfu_amd: input/output must be contiguous, same size and dtype");
    }
    const KungFu_Datatype dt = from_type(type);
    if (kungfu_type_size(dt) != static_cast<uint32_t>(input.element_size())) {
        throw std::runtime_error("kungfu_amd: type string does not match the tensor");
    }
    const KungFu_Op op = from_op(op_name);
    int dev = -1;
    check(kf_exchange_info(ex, nullptr, nullptr, &dev), "kf_exchange_info");
    if (input.get_device() != dev || output.get_device() != dev) {
        throw std::runtime_error("kungfu_amd: tensor not on the exchange's device");
    }
    hipStream_t s = c10::hip::getCurrentHIPStream(dev).stream();
    auto p        = std::make_shared<Pending>();
    p->input      = input;
    p->output     = output;
    auto *ref     = new std::shared_ptr<Pending>(p);
    void *in_ptr = input.data_ptr(), *out_ptr = output.data_ptr();
    const size_t n = static_cast<size_t>(input.numel());
    int rc;
    {
        // the exchange may wait for its negotiation thread (which runs the
        // collectives): never with the GIL held, so other Python threads
        // (other ranks in a test, the training loop) keep running
        py::gil_scoped_release nogil;
        rc = kf_exchange_all_reduce_named(ex, name.c_str(), in_ptr, out_ptr, n, dt, op, 0,
                                          g_algo.load(), s, on_done, ref);
    }
    if (rc != KF_OK) {
        delete ref;
        check(rc, "kf_exchange_all_reduce_named");
    }
    return p;
}

void wait(const std::shared_ptr<Pending> &p)
{
    std::string why;
    int status;
    {
        py::gil_scoped_release nogil;
        std::unique_lock<std::mutex> lk(p->m);
        p->cv.wait(lk, [&] { return p->done; });
        status = p->status;
        why    = p->why;
    }
    p->input.reset();
    p->output.reset();
    if (status != KF_OK) {
        throw std::runtime_error("kungfu_amd: all-reduce failed (status " +
                                 std::to_string(status) + "): " + why);
    }
}
}  // namespace

void init_exchange(py::bytes uid, int rank, int size, int device)
{
    std::string id = uid;
    if (id.size() != KF_UNIQUE_ID_BYTES) throw std::runtime_error("kungfu_amd: id must be 128 bytes");
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ex) {
        (void)kf_exchange_wait_named(g_ex);
        kf_exchange_destroy(g_ex);
    }
    // a rank that never joins costs KUNGFU_AMD_INIT_TIMEOUT_S (default 300 s,
    // whole seconds in [1, 86400]), then every rank learns it in
    // ops.bring_up's agreement and takes the torch.distributed path. A timed-out
    // init leaves its thread blocked in ncclCommInitRank until the process
    // exits (RCCL has no way to cancel it).
    int timeout_ms = 300 * 1000;
    if (const char *e = std::getenv("KUNGFU_AMD_INIT_TIMEOUT_S")) {
        char *end      = nullptr;
        const long sec = std::strtol(e, &end, 10);
        if (end == e || *end != '\0' || sec <= 0 || sec > 86400) {
            throw std::runtime_error(std::string("kungfu_amd: KUNGFU_AMD_INIT_TIMEOUT_S must be "
                                                 "whole seconds in [1, 86400], got '") + e + "'");
        }
        timeout_ms = static_cast<int>(static_cast<long long>(sec) * 1000LL);
    }
    {
        py::gil_scoped_release nogil;
        g_ex = kf_exchange_create_timeout(id.data(), rank, size, device, timeout_ms);
    }
    if (!g_ex) throw std::runtime_error(std::string("kf_exchange_create: ") + kf_exchange_last_error());
}

py::bytes unique_id()
{
    std::string id(KF_UNIQUE_ID_BYTES, '\0');
    check(kf_exchange_unique_id(&id[0]), "kf_exchange_unique_id");
    return py::bytes(id);
}

bool initialized() { return g_ex != nullptr; }

// this thread's ops use `handle` (a kf_exchange_t* as an integer; 0 = back to
// the process exchange); the caller keeps it alive while bound
void bind_exchange(uintptr_t handle) { t_ex = reinterpret_cast<kf_exchange_t *>(handle); }

// the schedule of every later op: "auto" (the exchange's choice, default),
// "rs" (RCCL reduce-scatter), "a2a" (all-to-all + the HIP rank-order fold)
void set_algo(const std::string &algo)
{
    static const std::map<std::string, int> m = {
        {"auto", KF_ALGO_AUTO}, {"rs", KF_ALGO_REDUCE_SCATTER}, {"a2a", KF_ALGO_ALL_TO_ALL},
        {"rs_avg", KF_ALGO_REDUCE_SCATTER_AVG}};
    auto it = m.find(algo);
    if (it == m.end()) throw std::runtime_error("kungfu_amd: algo must be auto, rs, a2a or rs_avg");
    g_algo = it->second;
}

void finalize()
{
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ex) {
        py::gil_scoped_release nogil;
        (void)kf_exchange_wait_named(g_ex);
        kf_exchange_destroy(g_ex);
    }
    g_ex = nullptr;
}

// the blocking op: an anonymous call, named by the exchange's own counter
// (kf_exchange_all_reduce_named with ""), so the calls pair by their order on
// every rank's exchange and a new exchange starts its count at zero
void all_reduce_cuda(torch::Tensor input, torch::Tensor output, const std::string &type,
                     const std::string &op_name)
{
    wait(start(input, output, type, op_name, ""));
}

int all_reduce_cuda_async(torch::Tensor input, torch::Tensor output, const std::string &type,
                          const std::string &op_name, const std::string &tensor_name)
{
    auto p = start(input, output, type, op_name, tensor_name);
    std::lock_guard<std::mutex> lk(g_mu);
    const int h  = g_next++;
    g_handles[h] = p;
    return h;
}

void wait_handle(int handle)
{
    std::shared_ptr<Pending> p;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_handles.find(handle);
        if (it == g_handles.end()) throw std::runtime_error("kungfu_amd: unknown handle");
        p = it->second;
        g_handles.erase(it);
    }
    wait(p);
}

void wait_all_handles(const std::vector<int> &handles)
{
    std::string first;
    for (int h : handles) {
        try {
            wait_handle(h);
        } catch (const std::runtime_error &e) {
            if (first.empty()) first = e.what();
        }
    }
    if (!first.empty()) throw std::runtime_error(first);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m)
{
    m.def("unique_id", &unique_id);
    m.def("init_exchange", &init_exchange);
    m.def("initialized", &initialized);
    m.def("bind_exchange", &bind_exchange);
    m.def("finalize", &finalize);
    m.def("set_algo", &set_algo);
    m.def("all_reduce_cuda", &all_reduce_cuda);
    m.def("all_reduce_cuda_async", &all_reduce_cuda_async);
    m.def("wait_handle", &wait_handle);
    m.def("wait_all_handles", &wait_all_handles);
}
