// kf_ingest.hip — host ingestion: KungFu's rchannel wire format and the
// device-side recvOnto / sendInto steps of Session.runGraphs.
//
// Wire format (little-endian), restated from the reference:
//   connection header  {u16 type, u16 src_port, u32 src_ipv4}   connection.go:73-80,
//                                                               message.go:44-56
//   connection ack     {u32 token}                              connection.go:28-40, 81-92
//   message header     {u32 name_len, name bytes, u32 flags}    message.go:90-128
//   message body       {u32 len, payload}                       message.go:160-198
//   flags: WaitRecvBuf = 1 (receiver reads straight into its registered
//   RecvBuf, handler/collective.go:43-61)
//
// Ingest: a peer chunk is read from the socket straight into a page-locked
// slot and folded onto the device-resident accumulator by the same HIP kernel
// as kf_bucket_reduce, which reads the slot in place over PCIe (zero copy: the
// slot is mapped into the GPU's address space) — replacing "Recv into a pooled
// Go []byte, then std_transform_2 on the host" (session.go:255-264). For the
// session's 1 MiB chunks that is 33 us against 39 us for an H2D copy + fold
// (tools/explore/zc_explore.hip). recvInto (bcast) still copies the slot to
// HBM with the SDMA engine. Slots are reused round-robin; a slot is refilled
// only after the copy or fold that read it completed (per-slot event), so the
// socket read of chunk i+1 overlaps the fold of chunk i.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "kf_stream.hpp"
#include "kungfu_amd.h"

namespace
{
thread_local std::string t_ingest_error;

int io_fail(const char *what)
{
    t_ingest_error = std::string(what) + ": " + std::strerror(errno);
    return KF_ERR_IO;
}

int proto_fail(const std::string &what)
{
    t_ingest_error = what;
    return KF_ERR_PROTO;
}

int hip_fail(hipError_t e, const char *what)
{
    t_ingest_error = std::string(what) + ": " + hipGetErrorString(e);
    return KF_ERR_HIP;
}

#define ING_HIP(call)                                                          \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess) return hip_fail(e_, #call);                      \
    } while (0)

// readN (message.go:204-213): loop until exactly n bytes arrived
int read_full(int fd, void *buf, size_t n)
{
    char *p = static_cast<char *>(buf);
    while (n > 0) {
        ssize_t r = ::read(fd, p, n);
        if (r < 0) {
            if (errno == EINTR) continue;
            return io_fail("read");
        }
        if (r == 0) return proto_fail("unexpected end of stream");
        p += r;
        n -= static_cast<size_t>(r);
    }
    return KF_OK;
}

// writev without SIGPIPE: a peer that died must fail the write (EPIPE), not
// kill this process (a C or Go host does not ignore SIGPIPE as Python does)
inline ssize_t writev_nosig(int fd, struct iovec *iov, int cnt)
{
    struct msghdr m {};
    m.msg_iov    = iov;
    m.msg_iovlen = static_cast<size_t>(cnt);
    const ssize_t w = ::sendmsg(fd, &m, MSG_NOSIGNAL);
    if (w < 0 && errno == ENOTSOCK) return ::writev(fd, iov, cnt);
    return w;
}

int write_full(int fd, struct iovec *iov, int cnt)
{
    while (cnt > 0) {
        ssize_t w = writev_nosig(fd, iov, cnt);
        if (w < 0) {
            if (errno == EINTR) continue;
            return io_fail("writev");
        }
        size_t left = static_cast<size_t>(w);
        while (cnt > 0 && left >= iov->iov_len) {
            left -= iov->iov_len;
            ++iov;
            --cnt;
        }
        if (cnt > 0) {
            iov->iov_base = static_cast<char *>(iov->iov_base) + left;
            iov->iov_len -= left;
        }
    }
    return KF_OK;
}

inline void put_u32(unsigned char *p, uint32_t v)
{
    p[0] = v & 0xff;
    p[1] = (v >> 8) & 0xff;
    p[2] = (v >> 16) & 0xff;
    p[3] = (v >> 24) & 0xff;
}

inline uint32_t get_u32(const unsigned char *p)
{
    return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) |
           (uint32_t(p[3]) << 24);
}

}  // namespace

struct kf_ingest {
    size_t slot_bytes = 0;
    int nslots        = 0;
    int next          = 0;
    std::vector<void *> host;   // page-locked slots
    std::vector<void *> hmap;   // the same slots as the GPU addresses them
    std::vector<hipEvent_t> done;
    std::vector<hipEvent_t> pre;  // streamed receives: the caller stream's work before the kernel
    std::vector<bool> armed;
    std::mutex mu;  // slot bookkeeping; callers may share one ingest object

    ~kf_ingest()
    {
        for (auto e : done)
            if (e) (void)hipEventDestroy(e);
        for (auto e : pre)
            if (e) (void)hipEventDestroy(e);
        for (auto p : host)
            if (p) (void)hipHostFree(p);
    }

    // next free slot: wait until its previous H2D has finished
    int take(int *slot)
    {
        std::lock_guard<std::mutex> lock(mu);
        const int s = next;
        next        = (next + 1) % nslots;
        if (armed[s]) {
            ING_HIP(hipEventSynchronize(done[s]));
            armed[s] = false;
        }
        *slot = s;
        return KF_OK;
    }
};

extern "C" {

int kf_rch_client_handshake(int fd, uint16_t conn_type, uint16_t src_port,
                            uint32_t src_ipv4, uint32_t expect_token)
{
    unsigned char h[8];
    h[0] = conn_type & 0xff;
    h[1] = conn_type >> 8;
    h[2] = src_port & 0xff;
    h[3] = src_port >> 8;
    put_u32(h + 4, src_ipv4);
    struct iovec iov = {h, sizeof(h)};
    int rc           = write_full(fd, &iov, 1);
    if (rc != KF_OK) return rc;
    unsigned char a[4];
    rc = read_full(fd, a, 4);
    if (rc != KF_OK) return rc;
    // connection.go:93-99: a token mismatch is fatal on collective connections
    if (get_u32(a) != expect_token && conn_type == KF_RCH_CONN_COLLECTIVE) {
        return proto_fail("invalid token");
    }
    return KF_OK;
}

int kf_rch_server_handshake(int fd, uint32_t token, uint16_t *conn_type,
                            uint16_t *src_port, uint32_t *src_ipv4)
{
    unsigned char h[8];
    int rc = read_full(fd, h, 8);
    if (rc != KF_OK) return rc;
    if (conn_type) *conn_type = uint16_t(h[0] | (h[1] << 8));
    if (src_port) *src_port = uint16_t(h[2] | (h[3] << 8));
    if (src_ipv4) *src_ipv4 = get_u32(h + 4);
    unsigned char a[4];
    put_u32(a, token);
    struct iovec iov = {a, 4};
    return write_full(fd, &iov, 1);
}

int kf_rch_send(int fd, const char *name, uint32_t flags, const void *data,
                uint32_t len)
{
    if (!name || (len > 0 && !data)) return KF_ERR_ARG;
    const uint32_t nl = static_cast<uint32_t>(std::strlen(name));
    unsigned char a[4], b[4], c[4];
    put_u32(a, nl);
    put_u32(b, flags);
    put_u32(c, len);
    // tcpConnection.Send: header then message, one logical write (connection.go:149-165)
    struct iovec iov[5] = {{a, 4},
                           {const_cast<char *>(name), nl},
                           {b, 4},
                           {c, 4},
                           {const_cast<void *>(data), len}};
    return write_full(fd, iov, len > 0 ? 5 : 4);
}

int kf_rch_recv_header(int fd, char *name, uint32_t cap, uint32_t *name_len,
                       uint32_t *flags)
{
    unsigned char a[4];
    int rc = read_full(fd, a, 4);
    if (rc != KF_OK) return rc;
    const uint32_t nl = get_u32(a);
    if (nl + 1 > cap || !name) return proto_fail("message name longer than buffer");
    rc = read_full(fd, name, nl);
    if (rc != KF_OK) return rc;
    name[nl] = 0;
    rc       = read_full(fd, a, 4);
    if (rc != KF_OK) return rc;
    if (name_len) *name_len = nl;
    if (flags) *flags = get_u32(a);
    return KF_OK;
}

int kf_rch_recv_body(int fd, void *dst, uint32_t expect_len)
{
    unsigned char a[4];
    int rc = read_full(fd, a, 4);
    if (rc != KF_OK) return rc;
    // Message.ReadInto (message.go:184-198): the length must match the buffer
    if (get_u32(a) != expect_len) return proto_fail("unexpected message length");
    if (expect_len == 0) return KF_OK;
    if (!dst) return KF_ERR_ARG;
    return read_full(fd, dst, expect_len);
}

kf_ingest_t *kf_ingest_create(size_t slot_bytes, int nslots)
{
    if (slot_bytes == 0 || nslots < 1) return nullptr;
    auto *g       = new kf_ingest;
    g->slot_bytes = slot_bytes;
    g->nslots     = nslots;
    g->host.assign(nslots, nullptr);
    g->hmap.assign(nslots, nullptr);
    g->done.assign(nslots, nullptr);
    g->pre.assign(nslots, nullptr);
    g->armed.assign(nslots, false);
    for (int i = 0; i < nslots; ++i) {
        // a streamed receive's kernel reads the slot behind a system acquire
        // fence (kf_stream.hip): no fine-grained memory needed here
        if (hipHostMalloc(&g->host[i], slot_bytes, hipHostMallocDefault) !=
                hipSuccess ||
            hipHostGetDevicePointer(&g->hmap[i], g->host[i], 0) != hipSuccess ||
            hipEventCreateWithFlags(&g->done[i], kf_sync::event_flags()) != hipSuccess ||
            hipEventCreateWithFlags(&g->pre[i], hipEventDisableTiming) != hipSuccess) {
            t_ingest_error = "kf_ingest_create: HIP allocation failed";
            delete g;
            return nullptr;
        }
    }
    return g;
}

void kf_ingest_destroy(kf_ingest_t *g) { delete g; }

int kf_ingest_recv_onto(kf_ingest_t *g, int fd, uint32_t len, void *dev_acc,
                        const void *dev_own, size_t count, KungFu_Datatype dt,
                        KungFu_Op op, void *stream)
{
    if (!g || !dev_acc) return KF_ERR_ARG;
    if (len > g->slot_bytes) return proto_fail("chunk larger than ingest slot");
    const uint32_t sz = kungfu_type_size(dt);
    if (static_cast<size_t>(len) != count * sz) return proto_fail("chunk length != count * type size");
    int slot;
    int rc = g->take(&slot);
    if (rc != KF_OK) return rc;
    rc = kf_rch_recv_body(fd, g->host[slot], len);
    if (rc != KF_OK) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // Transform2(RecvBuf, effective, peer): own is SendBuf before the first
    // receive, RecvBuf afterwards (session.go:241-264); peer read in place
    const void *ins[2] = {dev_own ? dev_own : dev_acc, g->hmap[slot]};
    rc                 = kf_bucket_reduce(ins, 2, dev_acc, count, dt, op, stream);
    if (rc != KF_OK) return rc;
    // the slot is free again once the fold has run
    ING_HIP(hipEventRecord(g->done[slot], s));
    {
        std::lock_guard<std::mutex> lock(g->mu);
        g->armed[slot] = true;
    }
    return KF_OK;
}

int kf_ingest_recv_into(kf_ingest_t *g, int fd, uint32_t len, void *dev_dst,
                        void *stream)
{
    if (!g || (!dev_dst && len > 0)) return KF_ERR_ARG;
    if (len > g->slot_bytes) return proto_fail("chunk larger than ingest slot");
    int slot;
    int rc = g->take(&slot);
    if (rc != KF_OK) return rc;
    rc = kf_rch_recv_body(fd, g->host[slot], len);
    if (rc != KF_OK || len == 0) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (kf_stream::copy_kernels()) {
        if (kf_stream::launch_copy(dev_dst, g->hmap[slot], len, s) != KF_OK) {
            t_ingest_error = "copy kernel launch";
            return KF_ERR_HIP;
        }
    } else {
        ING_HIP(hipMemcpyAsync(dev_dst, g->host[slot], len, hipMemcpyHostToDevice, s));
    }
    ING_HIP(hipEventRecord(g->done[slot], s));
    {
        std::lock_guard<std::mutex> lock(g->mu);
        g->armed[slot] = true;
    }
    return KF_OK;
}

// The body in pieces: piece k's device work is queued as soon as it is read,
// so a chunk's fold / copy overlaps the rest of its socket read; the last
// piece's work ends shortly after the last byte instead of a whole chunk's
// work after it. The operation is element-wise, so the bits are those of one
// launch over the chunk.
int kf_ingest_recv_onto_pieces(kf_ingest_t *g, int fd, uint32_t len, void *dev_acc,
                               const void *dev_own, size_t count, KungFu_Datatype dt,
                               KungFu_Op op, void *stream, uint32_t piece_bytes,
                               void *const *piece_events, int n_events)
{
    if (!g || !dev_acc) return KF_ERR_ARG;
    if (len > g->slot_bytes) return proto_fail("chunk larger than ingest slot");
    const uint32_t sz = kungfu_type_size(dt);
    if (static_cast<size_t>(len) != count * sz) return proto_fail("chunk length != count * type size");
    if (piece_bytes == 0 || piece_bytes % sz) return KF_ERR_ARG;
    const uint32_t npieces = len == 0 ? 0 : (len + piece_bytes - 1) / piece_bytes;
    if (piece_events && static_cast<uint32_t>(n_events) < npieces) return KF_ERR_ARG;
    int slot;
    int rc = g->take(&slot);
    if (rc != KF_OK) return rc;
    unsigned char a[4];
    rc = read_full(fd, a, 4);
    if (rc != KF_OK) return rc;
    if (get_u32(a) != len) return proto_fail("unexpected message length");
    hipStream_t s   = static_cast<hipStream_t>(stream);
    char *host      = static_cast<char *>(g->host[slot]);
    const char *dev = static_cast<const char *>(g->hmap[slot]);
    const char *own = static_cast<const char *>(dev_own ? dev_own : dev_acc);
    char *acc       = static_cast<char *>(dev_acc);
    for (uint32_t k = 0; k < npieces; ++k) {
        const uint32_t off = k * piece_bytes;
        const uint32_t pl  = std::min(piece_bytes, len - off);
        rc = read_full(fd, host + off, pl);
        if (rc != KF_OK) return rc;
        const void *ins[2] = {own + off, dev + off};
        rc = kf_bucket_reduce(ins, 2, acc + off, pl / sz, dt, op, stream);
        if (rc != KF_OK) return rc;
        if (piece_events) ING_HIP(hipEventRecord(static_cast<hipEvent_t>(piece_events[k]), s));
    }
    ING_HIP(hipEventRecord(g->done[slot], s));
    {
        std::lock_guard<std::mutex> lock(g->mu);
        g->armed[slot] = true;
    }
    return KF_OK;
}

int kf_ingest_recv_into_pieces(kf_ingest_t *g, int fd, uint32_t len, void *dev_dst,
                               void *stream, uint32_t piece_bytes)
{
    if (!g || (!dev_dst && len > 0) || piece_bytes == 0) return KF_ERR_ARG;
    if (len > g->slot_bytes) return proto_fail("chunk larger than ingest slot");
    int slot;
    int rc = g->take(&slot);
    if (rc != KF_OK) return rc;
    unsigned char a[4];
    rc = read_full(fd, a, 4);
    if (rc != KF_OK) return rc;
    if (get_u32(a) != len) return proto_fail("unexpected message length");
    if (len == 0) return KF_OK;
    hipStream_t s = static_cast<hipStream_t>(stream);
    char *host    = static_cast<char *>(g->host[slot]);
    char *dst     = static_cast<char *>(dev_dst);
    for (uint32_t off = 0; off < len; off += piece_bytes) {
        const uint32_t pl = std::min(piece_bytes, len - off);
        rc = read_full(fd, host + off, pl);
        if (rc != KF_OK) return rc;
        ING_HIP(hipMemcpyAsync(dst + off, host + off, pl, hipMemcpyHostToDevice, s));
    }
    ING_HIP(hipEventRecord(g->done[slot], s));
    {
        std::lock_guard<std::mutex> lock(g->mu);
        g->armed[slot] = true;
    }
    return KF_OK;
}

int kf_ingest_send_from_device(kf_ingest_t *g, int fd, const char *name,
                               uint32_t flags, const void *dev_src, size_t bytes,
                               void *stream)
{
    if (!g || !dev_src || !name) return KF_ERR_ARG;
    if (bytes > g->slot_bytes) return proto_fail("chunk larger than ingest slot");
    int slot;
    int rc = g->take(&slot);
    if (rc != KF_OK) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    ING_HIP(hipMemcpyAsync(g->host[slot], dev_src, bytes, hipMemcpyDeviceToHost, s));
    if (kf_sync::stream_sync(s) != KF_OK) {
        t_ingest_error = "stream sync";
        return KF_ERR_HIP;
    }
    return kf_rch_send(fd, name, flags, g->host[slot], static_cast<uint32_t>(bytes));
}

int kf_ingest_fold_host(kf_ingest_t *g, const void *host, uint32_t len, void *dev_acc,
                        const void *dev_own, size_t count, KungFu_Datatype dt, KungFu_Op op,
                        void *stream)
{
    if (!g || !dev_acc || (!host && len > 0)) return KF_ERR_ARG;
    if (len > g->slot_bytes) return proto_fail("chunk larger than ingest slot");
    int slot;
    int rc = g->take(&slot);
    if (rc != KF_OK) return rc;
    std::memcpy(g->host[slot], host, len);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const void *ins[2] = {dev_own ? dev_own : dev_acc, g->hmap[slot]};
    rc                 = kf_bucket_reduce(ins, 2, dev_acc, count, dt, op, stream);
    if (rc != KF_OK) return rc;
    ING_HIP(hipEventRecord(g->done[slot], s));
    {
        std::lock_guard<std::mutex> lock(g->mu);
        g->armed[slot] = true;
    }
    return KF_OK;
}

int kf_ingest_copy_host(kf_ingest_t *g, const void *host, uint32_t len, void *dev_dst,
                        void *stream)
{
    if (!g || (!dev_dst && len > 0) || (!host && len > 0)) return KF_ERR_ARG;
    if (len > g->slot_bytes) return proto_fail("chunk larger than ingest slot");
    int slot;
    int rc = g->take(&slot);
    if (rc != KF_OK || len == 0) return rc;
    std::memcpy(g->host[slot], host, len);
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (kf_stream::copy_kernels()) {
        if (kf_stream::launch_copy(dev_dst, g->hmap[slot], len, s) != KF_OK) {
            t_ingest_error = "copy kernel launch";
            return KF_ERR_HIP;
        }
    } else {
        ING_HIP(hipMemcpyAsync(dev_dst, g->host[slot], len, hipMemcpyHostToDevice, s));
    }
    ING_HIP(hipEventRecord(g->done[slot], s));
    {
        std::lock_guard<std::mutex> lock(g->mu);
        g->armed[slot] = true;
    }
    return KF_OK;
}

int kf_ingest_sync(kf_ingest_t *g)
{
    if (!g) return KF_ERR_ARG;
    std::lock_guard<std::mutex> lock(g->mu);
    for (int i = 0; i < g->nslots; ++i) {
        if (g->armed[i]) {
            ING_HIP(hipEventSynchronize(g->done[i]));
            g->armed[i] = false;
        }
    }
    return KF_OK;
}

const char *kf_ingest_last_error(void) { return t_ingest_error.c_str(); }

}  // extern "C"

namespace
{
// the body of the message whose header was just read, into the landing slot,
// publishing every read as it lands; on a failure the waiting kernel is told
int read_published(int fd, char *host, uint32_t len, kf_stream::Ctl *ctl)
{
    unsigned char a[4];
    int rc = read_full(fd, a, 4);
    if (rc == KF_OK && get_u32(a) != len) rc = proto_fail("unexpected message length");
    uint32_t got = 0;
    while (rc == KF_OK && got < len) {
        ssize_t r = ::read(fd, host + got, len - got);
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) {
            rc = io_fail("read");
        } else if (r == 0) {
            rc = proto_fail("unexpected end of stream");
        } else {
            got += static_cast<uint32_t>(r);
            kf_stream::publish(ctl, got);
        }
    }
    if (rc != KF_OK) kf_stream::abort_wait(ctl);
    return rc;
}

// Does other work wait behind this stream's kernels? The legacy null stream
// (torch's default) serialises with every blocking stream of the device, in
// every thread of the process, and a blocking stream with it.
bool holds_others(hipStream_t s)
{
    if (s == nullptr) return true;  // the null stream itself
    unsigned f = 0;
    if (hipStreamGetFlags(s, &f) != hipSuccess) {
        (void)hipGetLastError();  // not left for the launch check that follows
        return true;
    }
    return !(f & hipStreamNonBlocking);
}

// The slot's kernel is queued first (it waits in the GPU), then the body is
// read; the slot is free again once that kernel has run. A kernel that waits
// for bytes from a socket must not sit where unrelated work queues behind it:
// on a stream that holds others (above) it runs on `wait_stream` (a
// non-blocking stream of the session, passed when other sessions share the
// process; kf_session.hip g_device_sessions) after the caller's earlier work, and
// the caller's stream takes it back (waits for it) only once the whole body
// is in, when it finishes at once. Sessions in threads of one process that
// share the null stream otherwise queued each other's folds behind a kernel
// waiting for a peer whose own sends were queued there too (r05,
// profiles/r05/failures.md).
template <typename Launch>
int streamed(kf_ingest_t *g, int fd, uint32_t len, void *stream, void *wait_stream,
             kf_stream::Ctl *ctl, uint32_t piece, Launch launch)
{
    if (len > g->slot_bytes) return proto_fail("chunk larger than ingest slot");
    int slot;
    int rc = g->take(&slot);
    if (rc != KF_OK) return rc;
    kf_stream::reset(ctl, piece);
    hipStream_t cs = static_cast<hipStream_t>(stream), ks = cs;
    if (wait_stream && holds_others(cs)) {
        ks = static_cast<hipStream_t>(wait_stream);
        ING_HIP(hipEventRecord(g->pre[slot], cs));
        ING_HIP(hipStreamWaitEvent(ks, g->pre[slot], 0));
    }
    rc = launch(g->hmap[slot], ks);
    if (rc != KF_OK) {
        kf_stream::abort_wait(ctl);  // in case a kernel did start: it stops waiting
        t_ingest_error = "streamed receive: kernel launch failed";
        return rc;
    }
    if (hipError_t e = hipEventRecord(g->done[slot], ks); e != hipSuccess) {
        // the kernel is queued and would wait for a body nobody reads: tell
        // it to stop and let it drain before the caller may free its words
        // (its stream is not the one the caller synchronises when ks != cs)
        kf_stream::abort_wait(ctl);
        (void)hipStreamSynchronize(ks);
        return hip_fail(e, "hipEventRecord after a streamed launch");
    }
    {
        std::lock_guard<std::mutex> lock(g->mu);
        g->armed[slot] = true;
    }
    rc = read_published(fd, static_cast<char *>(g->host[slot]), len, ctl);
    // the caller's later work (the send of this chunk, the next fold) after
    // the kernel; on a failed read the kernel has been told to stop
    if (ks != cs && hipStreamWaitEvent(cs, g->done[slot], 0) != hipSuccess && rc == KF_OK) {
        rc = hip_fail(hipErrorUnknown, "hipStreamWaitEvent after a streamed receive");
    }
    return rc;
}
}  // namespace

int kf_ingest_recv_onto_streamed(kf_ingest_t *g, int fd, uint32_t len, void *dev_acc,
                                 const void *dev_own, KungFu_Datatype dt, void *stream,
                                 uint32_t piece, kf_stream::Ctl *ctl, kf_stream::Ctl *ctl_dev,
                                 kf_stream::Board *board, int deadline_ms, bool mark,
                                 void *wait_stream)
{
    if (!g || !dev_acc || !ctl || !ctl_dev || !board) return KF_ERR_ARG;
    return streamed(g, fd, len, stream, wait_stream, ctl, piece, [&](void *landing, hipStream_t ks) {
        return kf_stream::launch_fold(dt, dev_own ? dev_own : dev_acc, landing, dev_acc, len,
                                      piece, ctl_dev, board, deadline_ms, mark, ks);
    });
}

int kf_ingest_recv_into_streamed(kf_ingest_t *g, int fd, uint32_t len, void *dev_dst,
                                 void *stream, uint32_t piece, kf_stream::Ctl *ctl,
                                 kf_stream::Ctl *ctl_dev, kf_stream::Board *board,
                                 int deadline_ms, void *wait_stream)
{
    if (!g || (!dev_dst && len > 0) || !ctl || !ctl_dev || !board) return KF_ERR_ARG;
    return streamed(g, fd, len, stream, wait_stream, ctl, piece, [&](void *landing, hipStream_t ks) {
        return kf_stream::launch_copy_in(landing, dev_dst, len, piece, ctl_dev, board, deadline_ms,
                                         ks);
    });
}
