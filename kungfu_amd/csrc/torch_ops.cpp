// torch_ops.cpp — the reference's torch extension surface with its
// signatures (srcs/cpp/src/torch/module_cuda.cpp:28-40,
// srcs/cpp/src/torch/ops/cuda/collective.cpp:20-55), over the C ABI of
// libkungfu_amd.so instead of a host round trip.
//
// The reference copies a CUDA tensor into a std::vector, all-reduces it on the
// host through Peer::GetDefault()->AllReduce, and copies it back
// (collective.cpp:24-29). Here the process's exchange (kf_exchange_*, RCCL
// over xGMI for the bytes, the HIP kernels for the sum) reduces it in HBM,
// queued on torch's current HIP stream:
//
//   all_reduce_cuda(input, output, type, op)             collective.cpp:20-30
//   all_reduce_cuda_async(input, output, type, op, name) collective.cpp:32-55
//       -> int handle; wait_handle(h) / wait_all_handles(hs) block until done
//          (the reference's HandleManager, handler_manager.hpp:6-84)
//
// `type` is the tensor's x.type() string (torch/ops/clib.py maps
// 'torch.cuda.FloatTensor'; the reference converts only Float,
// collective.cpp:10-18 — here every dtype the exchange supports), `op` one of
// sum / min / max / prod (srcs/cpp/src/torch/common.cpp:41-46).
//
// Peer::GetDefault() is init_exchange(id, rank, size, device): the id is
// rank 0's kf_exchange_unique_id() bytes, shared by the caller (torch.distributed
// in kungfu_amd/torch/ops.py), as gpu_collective.cpp:190-200 shares it.
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "kungfu_amd.h"

namespace
{
kf_exchange_t *g_ex = nullptr;
std::mutex g_mu;
std::map<int, hipEvent_t> g_handles;
int g_next = 0;

void check(int rc, const char *what)
{
    if (rc != KF_OK) {
        throw std::runtime_error(std::string(what) + " failed (status " + std::to_string(rc) +
                                 "): " + kf_exchange_last_error());
    }
}

void check_hip(hipError_t e, const char *what)
{
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
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

hipStream_t issue(const torch::Tensor &input, torch::Tensor &output, const std::string &type,
                  const std::string &op_name)
{
    if (!g_ex) throw std::runtime_error("kungfu_amd: init_exchange() first");
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
    int dev = -1;
    check(kf_exchange_info(g_ex, nullptr, nullptr, &dev), "kf_exchange_info");
    if (input.get_device() != dev) {
        throw std::runtime_error("kungfu_amd: tensor not on the exchange's device");
    }
    hipStream_t s = c10::hip::getCurrentHIPStream(dev).stream();
    check(kf_exchange_all_reduce(g_ex, input.data_ptr(), output.data_ptr(),
                                 static_cast<size_t>(input.numel()), dt, from_op(op_name), 0,
                                 KF_ALGO_AUTO, s),
          "kf_exchange_all_reduce");
    return s;
}
}  // namespace

void init_exchange(py::bytes uid, int rank, int size, int device)
{
    std::string id = uid;
    if (id.size() != KF_UNIQUE_ID_BYTES) throw std::runtime_error("kungfu_amd: id must be 128 bytes");
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ex) kf_exchange_destroy(g_ex);
    g_ex = kf_exchange_create(id.data(), rank, size, device);
    if (!g_ex) throw std::runtime_error(std::string("kf_exchange_create: ") + kf_exchange_last_error());
}

py::bytes unique_id()
{
    std::string id(KF_UNIQUE_ID_BYTES, '\0');
    check(kf_exchange_unique_id(&id[0]), "kf_exchange_unique_id");
    return py::bytes(id);
}

bool initialized() { return g_ex != nullptr; }

void finalize()
{
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto &kv : g_handles) (void)hipEventDestroy(kv.second);
    g_handles.clear();
    if (g_ex) kf_exchange_destroy(g_ex);
    g_ex = nullptr;
}

void all_reduce_cuda(torch::Tensor input, torch::Tensor output, const std::string &type,
                     const std::string &op_name)
{
    issue(input, output, type, op_name);
}

int all_reduce_cuda_async(torch::Tensor input, torch::Tensor output, const std::string &type,
                          const std::string &op_name, const std::string & /*tensor_name*/)
{
    // every rank issues its all-reduces in one order (RCCL's rule; the
    // reference keys them by name instead), the name is kept for the API
    hipStream_t s = issue(input, output, type, op_name);
    hipEvent_t ev;
    check_hip(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
    check_hip(hipEventRecord(ev, s), "hipEventRecord");
    std::lock_guard<std::mutex> lk(g_mu);
    const int h  = g_next++;
    g_handles[h] = ev;
    return h;
}

void wait_handle(int handle)
{
    hipEvent_t ev;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_handles.find(handle);
        if (it == g_handles.end()) throw std::runtime_error("kungfu_amd: unknown handle");
        ev = it->second;
        g_handles.erase(it);
    }
    hipError_t e = hipEventSynchronize(ev);
    (void)hipEventDestroy(ev);
    check_hip(e, "hipEventSynchronize");
    check(kf_exchange_check(g_ex), "kf_exchange_check");
}

void wait_all_handles(const std::vector<int> &handles)
{
    for (int h : handles) wait_handle(h);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m)
{
    m.def("unique_id", &unique_id);
    m.def("init_exchange", &init_exchange);
    m.def("initialized", &initialized);
    m.def("finalize", &finalize);
    m.def("all_reduce_cuda", &all_reduce_cuda);
    m.def("all_reduce_cuda_async", &all_reduce_cuda_async);
    m.def("wait_handle", &wait_handle);
    m.def("wait_all_handles", &wait_all_handles);
}
