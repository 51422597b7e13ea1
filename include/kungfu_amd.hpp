// kungfu_amd.hpp — header-only C++ host over the C ABI (kungfu_amd.h) with the
// shape of the reference's C++ Peer facade (srcs/cpp/include/kungfu/peer.hpp),
// its dtype traits (srcs/cpp/include/kungfu/dtype.hpp) and Waiter
// (srcs/cpp/include/kungfu/utils/waiter.hpp), so C++ callers and the
// reference's own C++ tests (tests/cpp/unit/test_operations.cpp,
// tests/cpp/integration/fake_agent.cpp) read the same against this build.
//
//   kungfu_amd::Peer kf;                  // KUNGFU_INIT_PEERS / KUNGFU_SELF_SPEC, or one peer
//   kf.AllReduce(x, y, n, kungfu_amd::type_encoder<float>::value(), KungFu_SUM,
//                "grad", [&] { waiter.done(); });
//
// Peer::AllReduce is the session engine's all-reduce (kf_session_all_reduce,
// the counterpart of GoKungfuAllReduce): host buffers by default, HBM
// buffers with Peer::Device. The reduce of every received chunk runs on the
// GPU (std_transform_2's HIP kernel, or the device-mode fold); there is no CPU
// reduce behind it.
#pragma once

#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>

#include "kungfu_amd.h"

namespace kungfu_amd
{
using DoneCallback = std::function<void()>;

// dtype.hpp:18-97: C++ type -> KungFu_Datatype
template <typename T> struct type_encoder;
#define KUNGFU_AMD_TYPE(T, code)                                                \
    template <> struct type_encoder<T> {                                        \
        static KungFu_Datatype value() { return code; }                         \
    };
KUNGFU_AMD_TYPE(uint8_t, KungFu_UINT8)
KUNGFU_AMD_TYPE(uint16_t, KungFu_UINT16)
KUNGFU_AMD_TYPE(uint32_t, KungFu_UINT32)
KUNGFU_AMD_TYPE(uint64_t, KungFu_UINT64)
KUNGFU_AMD_TYPE(int8_t, KungFu_INT8)
KUNGFU_AMD_TYPE(int16_t, KungFu_INT16)
KUNGFU_AMD_TYPE(int32_t, KungFu_INT32)
KUNGFU_AMD_TYPE(int64_t, KungFu_INT64)
KUNGFU_AMD_TYPE(float, KungFu_FLOAT)
KUNGFU_AMD_TYPE(double, KungFu_DOUBLE)
#undef KUNGFU_AMD_TYPE

// utils/waiter.hpp: one-shot completion flag
class Waiter
{
    std::mutex mu_;
    std::condition_variable cv_;
    bool done_ = false;

  public:
    void done()
    {
        std::lock_guard<std::mutex> lk(mu_);
        done_ = true;
        cv_.notify_all();
    }
    void wait()
    {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return done_; });
    }
};

class Peer
{
  public:
    enum Buffers { Host = 0, Device = 1 };

    // peer.cpp:13-29: the peer kungfu-run describes in the environment
    // (KUNGFU_INIT_PEERS, KUNGFU_SELF_SPEC; env/envs.go:9-11), or a single
    // peer when there is none (env/config.go:54-56)
    explicit Peer(Buffers b = Host, const char *sock_dir = "/tmp")
    {
        const char *peers = std::getenv("KUNGFU_INIT_PEERS");
        const char *self  = std::getenv("KUNGFU_SELF_SPEC");
        if (peers && self) {
            s_ = kf_session_create_peers(peers, self, sock_dir, 0, b);
            // rank = self's index in the comma-separated list (plan/peerlist.go)
            const std::string list = std::string(peers) + ",", me(self);
            size_ = 0;
            for (size_t p = 0, q; (q = list.find(',', p)) != std::string::npos; p = q + 1) {
                if (list.compare(p, q - p, me) == 0) rank_ = size_;
                ++size_;
            }
        } else {
            s_ = kf_session_create(0, 1, sock_dir, 0, b);
        }
        check_created();
    }

    // peer.hpp:22 "Single Machine Multi-Process"
    Peer(int rank, int size, Buffers b = Host, const char *sock_dir = "/tmp")
        : rank_(rank), size_(size)
    {
        s_ = kf_session_create(rank, size, sock_dir, 0, b);
        check_created();
    }

    ~Peer()
    {
        if (s_) kf_session_destroy(s_);
    }
    Peer(const Peer &)            = delete;
    Peer &operator=(const Peer &) = delete;

    int Rank() const { return rank_; }
    int Size() const { return size_; }

    // peer.hpp:92-96; returns 0 on success, as GoKungfuAllReduce
    int AllReduce(const void *sendbuf, void *recvbuf, int count, KungFu_Datatype dtype,
                  KungFu_Op op, const char *name)
    {
        return kf_session_all_reduce(s_, sendbuf, recvbuf, static_cast<size_t>(count), dtype, op,
                                     name, stream_) == KF_OK
                   ? 0
                   : 1;
    }

    // the async overload: done runs on the session's worker thread once the
    // all-reduce has finished (main.go:184-191)
    int AllReduce(const void *sendbuf, void *recvbuf, int count, KungFu_Datatype dtype,
                  KungFu_Op op, const char *name, const DoneCallback &done)
    {
        auto *cb = new DoneCallback(done);
        const int rc = kf_session_all_reduce_async(s_, sendbuf, recvbuf, static_cast<size_t>(count),
                                                   dtype, op, name, stream_, &Peer::invoke, cb);
        if (rc != KF_OK) {
            delete cb;
            return 1;
        }
        return 0;
    }

    // Barrier (peer.hpp:78, GoKungfuBarrier)
    int Barrier() { return kf_session_barrier(s_) == KF_OK ? 0 : 1; }

    // device mode: the HIP stream the folds are queued on (hipStream_t)
    void SetStream(void *stream) { stream_ = stream; }
    kf_session_t *Session() { return s_; }

  private:
    static void invoke(int /*status*/, void *arg)
    {
        auto *cb = static_cast<DoneCallback *>(arg);
        (*cb)();  // the reference ignores the status (main.go:188)
        delete cb;
    }

    void check_created()
    {
        if (!s_) throw std::runtime_error(std::string("kungfu_amd::Peer: ") + kf_session_last_error());
    }

    kf_session_t *s_ = nullptr;
    int rank_ = 0, size_ = 1;
    void *stream_ = nullptr;
};
}  // namespace kungfu_amd
