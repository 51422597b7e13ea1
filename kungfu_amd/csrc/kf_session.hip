// kf_session.hip — single-host KungFu session engine (native), the collective
// boundary of SURVEY §8b B2: kf_session_all_reduce mirrors
// GoKungfuAllReduce(sendBuf, recvBuf, count, dtype, op, name, done=nil)
// (srcs/go/libkungfu-comm/collective.go:34-45) -> Session.AllReduce
// (srcs/go/kungfu/session/allreduce.go:10-12) -> runStrategiesWithHash /
// runGraphs (session.go:231-326), for peers that share one host.
//
// What is restated, with the reduce moved onto the GPU:
//   * chunking: ceil(bytes / 1 MiB) chunks, EvenPartition by element count,
//     named "part::<name>[b:e]" (session.go:301-326, workspace.go:18-25);
//   * per chunk, the strategy sl[hash(i, name) % len(sl)] with nameBasedHash
//     (sum of squared code points, shard.go:17-23) or simpleHash (= i);
//   * strategy lists for one host (strategy.go:121-205, topology.go:17-160):
//     STAR / TREE / BINARY_TREE_STAR / MULTI_STAR / MULTI_BINARY_TREE_STAR /
//     AUTO -> a star at rank 0; CLIQUE -> k stars, rooted at r; RING -> k
//     rings, reduce chain r+1 -> ... -> r, bcast chain r -> ... -> r-1;
//     BINARY_TREE -> i's children 2i+1, 2i+2. Reduce graph = reversed bcast
//     graph + self loops (GenDefaultReduceGraph) except for RING;
//   * runGraphs: a node folds every reduce-graph predecessor's chunk IN
//     ARRIVAL ORDER into RecvBuf (effective o peer: SendBuf before the first
//     receive, RecvBuf after — recvOnto, session.go:241-264), then sends to
//     its reduce successors (sendOnto, NoFlag); in the bcast graph it takes
//     its predecessor's chunk straight into RecvBuf (recvInto, WaitRecvBuf)
//     or forwards SendBuf if it received nothing (w.Forward), then sends to
//     its bcast successors (sendInto, WaitRecvBuf).
// Chunks progress independently (the reference runs a goroutine per chunk):
// one poll loop handles whatever message arrives next — NoFlag = reduce phase,
// WaitRecvBuf = bcast phase — and one sender thread drains a FIFO, so no peer
// ever blocks on a peer that is not reading.
//
// Device mode: send/recv are HBM pointers; a peer chunk lands in a page-locked
// slot, is copied to HBM and folded by the HIP kernel (kf_ingest_recv_onto).
// A node with several reduce predecessors (the star root: np-1 of them) stages
// each arrival in HBM and folds them all in ONE k-input launch when the last
// one is in: own o p_a1 o p_a2 o ... in arrival order, the same left fold as
// the reference's chain of recvOnto calls, so the result is bit-identical
// (reads (k+1)*S and writes S once, instead of 3*S per predecessor). bf16 keeps
// the per-hop chain: its k-input kernel rounds once, not per hop.
// Host mode: host pointers; the fold is std_transform_2's GPU path
// (kf_transform2_host) or a C callback (bench.py's CPU-baseline leg).
#include <hip/hip_runtime.h>
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/eventfd.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "kf_stream.hpp"
#include "kungfu_amd.h"

namespace
{
constexpr size_t kChunk      = size_t(1) << 20;  // session.go:301-304
constexpr int kPortBase      = 10000;            // plan/hostspec.go:121-124
constexpr uint32_t kIPv4     = 0x7F000001;
constexpr int kConnRetry     = 500;              // config.go:15-18
constexpr int kRetryPeriodUs = 200000;

thread_local std::string t_sess_error;

// device-mode sessions alive in this process. A streamed kernel waiting for a
// socket body on a stream that holds others (the null stream) is harmless
// while it is the process's only session: nothing else in the process has to
// run for that body to come. With several (ranks emulated as threads, the
// hierarchical path's sessions) another session's sends may queue behind it,
// so the kernel then waits on the session's own non-blocking stream instead
// (kf_ingest.hip streamed(); that costs two cross-stream event hops per
// chunk, C1 np = 2 0.60 -> 0.65 ms, so it is not taken when not needed).
std::atomic<int> g_device_sessions{0};

int fail(int rc, const std::string &what)
{
    t_sess_error = what;
    return rc;
}

// A peer's address (plan/addr.go NetAddr): IPv4 + port. Peers with the same
// IPv4 are colocated and talk over a unix socket named by the port (SockFile,
// addr.go:24-26, under the session's directory); others over TCP
// (connection.go:58-64).
struct PeerAddr {
    uint32_t ip;
    uint16_t port;
    bool operator==(const PeerAddr &o) const { return ip == o.ip && port == o.port; }
};

// the address is in the name too, so emulated hosts (127.0.0.x) sharing a
// directory and port numbers do not collide
std::string sock_path(const std::string &dir, const PeerAddr &p)
{
    char ip[INET_ADDRSTRLEN];
    in_addr a{};
    a.s_addr = htonl(p.ip);
    ::inet_ntop(AF_INET, &a, ip, sizeof(ip));
    return dir + "/kungfu-amd-" + ip + "-" + std::to_string(p.port) + ".sock";
}

// "a.b.c.d:port" (ParsePeerID, plan/id.go:34-50)
bool parse_peer(const std::string &s, PeerAddr *p)
{
    const size_t c = s.rfind(':');
    if (c == std::string::npos) return false;
    in_addr a{};
    if (::inet_pton(AF_INET, s.substr(0, c).c_str(), &a) != 1) return false;
    char *end       = nullptr;
    const long port = std::strtol(s.c_str() + c + 1, &end, 10);
    if (*end != 0 || port <= 0 || port > 65535) return false;
    p->ip   = ntohl(a.s_addr);
    p->port = static_cast<uint16_t>(port);
    return true;
}

// comma-separated (ParsePeerList, plan/peerlist.go:180-192)
bool parse_peer_list(const std::string &s, std::vector<PeerAddr> *out)
{
    out->clear();
    size_t b = 0;
    for (;;) {
        const size_t e = s.find(',', b);
        PeerAddr p;
        if (!parse_peer(s.substr(b, e == std::string::npos ? std::string::npos : e - b), &p)) {
            return false;
        }
        out->push_back(p);
        if (e == std::string::npos) return true;
        b = e + 1;
    }
}

std::vector<std::pair<size_t, size_t>> even_partition(size_t n, size_t k)
{
    // interval.go:12-27: the first rem parts get one more element
    std::vector<std::pair<size_t, size_t>> parts;
    const size_t quo = n / k, rem = n % k;
    size_t off = 0;
    for (size_t i = 0; i < k; ++i) {
        const size_t c = quo + (i < rem ? 1 : 0);
        parts.emplace_back(off, off + c);
        off += c;
    }
    return parts;
}

// nameBasedHash (shard.go:17-23): Go ranges over a string by rune, so decode
// UTF-8 and add each code point squared (uint64 wrap-around).
uint64_t name_hash(const std::string &s)
{
    uint64_t h = 0;
    for (size_t i = 0; i < s.size();) {
        const unsigned char c = static_cast<unsigned char>(s[i]);
        uint32_t cp;
        int len;
        if (c < 0x80) {
            cp = c, len = 1;
        } else if ((c >> 5) == 0x6 && i + 1 < s.size()) {
            cp = ((c & 0x1f) << 6) | (s[i + 1] & 0x3f), len = 2;
        } else if ((c >> 4) == 0xe && i + 2 < s.size()) {
            cp = ((c & 0x0f) << 12) | ((s[i + 1] & 0x3f) << 6) | (s[i + 2] & 0x3f), len = 3;
        } else if ((c >> 3) == 0x1e && i + 3 < s.size()) {
            cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3f) << 12) | ((s[i + 2] & 0x3f) << 6) |
                 (s[i + 3] & 0x3f),
            len = 4;
        } else {
            cp = 0xfffd, len = 1;  // invalid byte: Go yields U+FFFD
        }
        h += static_cast<uint64_t>(cp) * cp;
        i += len;
    }
    return h;
}

// One communication graph: prevs / nexts per rank (graph.go:18-108).
struct Graph {
    std::vector<std::vector<int>> prev, next;
    explicit Graph(int n) : prev(n), next(n) {}
    void edge(int i, int j)
    {
        if (i == j) return;  // self loops only mark "reduces"; implicit here
        next[i].push_back(j);
        prev[j].push_back(i);
    }
    Graph reversed() const
    {
        Graph r(static_cast<int>(prev.size()));
        for (size_t i = 0; i < next.size(); ++i)
            for (int j : next[i]) r.edge(j, static_cast<int>(i));
        return r;
    }
};

struct Strategy {
    Graph reduce, bcast;
};

Strategy simple(const Graph &bg) { return Strategy{bg.reversed(), bg}; }

Graph star(int k, int r)
{
    Graph g(k);
    for (int i = 0; i < k; ++i)
        if (i != r) g.edge(r, i);
    return g;
}

// getLocalMasters (topology.go:5-15): the first rank seen on each host
std::vector<int> local_masters(const std::vector<uint32_t> &hosts, std::vector<int> *master_of)
{
    std::vector<int> masters;
    master_of->assign(hosts.size(), -1);
    for (size_t r = 0; r < hosts.size(); ++r) {
        int m = -1;
        for (int q : masters)
            if (hosts[q] == hosts[r]) m = q;
        if (m < 0) {
            masters.push_back(static_cast<int>(r));
            m = static_cast<int>(r);
        }
        (*master_of)[r] = m;
    }
    return masters;
}

// every non-master hangs off its host's master (the star inside each host)
Graph host_stars(const std::vector<uint32_t> &hosts, std::vector<int> *masters)
{
    std::vector<int> master_of;
    *masters = local_masters(hosts, &master_of);
    Graph g(static_cast<int>(hosts.size()));
    for (size_t r = 0; r < hosts.size(); ++r)
        if (master_of[r] != static_cast<int>(r)) g.edge(master_of[r], static_cast<int>(r));
    return g;
}

Graph multi_star(const std::vector<uint32_t> &hosts, int root)  // topology.go:55-74
{
    std::vector<int> m;
    Graph g = host_stars(hosts, &m);
    const int k = static_cast<int>(m.size());
    if (k > 1)
        for (int i = 0; i < k; ++i)
            if (i != root) g.edge(m[root], m[i]);
    return g;
}

Graph binary_tree_star(const std::vector<uint32_t> &hosts, int offset)  // topology.go:76-101
{
    std::vector<int> m;
    Graph g     = host_stars(hosts, &m);
    const int k = static_cast<int>(m.size());
    if (k > 1) {
        auto idx = [&](int i) { return (i + offset) % k; };
        for (int i = 0; i < k; ++i) {
            if (2 * i + 1 < k) g.edge(m[idx(i)], m[idx(2 * i + 1)]);
            if (2 * i + 2 < k) g.edge(m[idx(i)], m[idx(2 * i + 2)]);
        }
    }
    return g;
}

// strategy.go:121-205; hosts[r] = IPv4 of rank r
std::vector<Strategy> strategy_list(int strategy, const std::vector<uint32_t> &hosts)
{
    const int k = static_cast<int>(hosts.size());
    std::vector<int> masters, master_of;
    masters = local_masters(hosts, &master_of);
    if (strategy == KungFu_AUTO)  // autoSelect (strategy.go:165-174)
        strategy = masters.size() == 1 ? KungFu_Star : KungFu_BinaryTreeStar;
    std::vector<Strategy> sl;
    switch (strategy) {
    case KungFu_Star:
        sl.push_back(simple(star(k, 0)));
        break;
    case KungFu_MultiStar:
        for (size_t i = 0; i < masters.size(); ++i)
            sl.push_back(simple(multi_star(hosts, static_cast<int>(i))));
        break;
    case KungFu_Clique:
        for (int r = 0; r < k; ++r) sl.push_back(simple(star(k, r)));
        break;
    case KungFu_Ring:  // GenCircularGraphPair (topology.go:149-160)
        for (int r = 0; r < k; ++r) {
            Graph g(k), b(k);
            for (int i = 1; i < k; ++i) {
                g.edge((r + i) % k, (r + i + 1) % k);
                b.edge((r + i - 1) % k, (r + i) % k);
            }
            sl.push_back(Strategy{g, b});
        }
        break;
    case KungFu_Tree: {  // GenTree (topology.go:17-31)
        Graph g = host_stars(hosts, &masters);
        for (size_t i = 1; i < masters.size(); ++i) g.edge(masters[0], masters[i]);
        sl.push_back(simple(g));
        break;
    }
    case KungFu_BinaryTree: {  // GenBinaryTree (topology.go:42-53)
        Graph g(k);
        for (int i = 0; i < k; ++i) {
            if (2 * i + 1 < k) g.edge(i, 2 * i + 1);
            if (2 * i + 2 < k) g.edge(i, 2 * i + 2);
        }
        sl.push_back(simple(g));
        break;
    }
    case KungFu_MultiBinaryTreeStar:
        for (size_t i = 0; i < masters.size(); ++i)
            sl.push_back(simple(binary_tree_star(hosts, static_cast<int>(i))));
        break;
    default:  // KungFu_BinaryTreeStar
        sl.push_back(simple(binary_tree_star(hosts, 0)));
        break;
    }
    return sl;
}

int parse_strategy(const char *s)
{
    static const std::pair<const char *, int> names[] = {
        {"STAR", KungFu_Star},
        {"MULTI_STAR", KungFu_MultiStar},
        {"RING", KungFu_Ring},
        {"CLIQUE", KungFu_Clique},
        {"TREE", KungFu_Tree},
        {"BINARY_TREE", KungFu_BinaryTree},
        {"BINARY_TREE_STAR", KungFu_BinaryTreeStar},
        {"MULTI_BINARY_TREE_STAR", KungFu_MultiBinaryTreeStar},
        {"AUTO", KungFu_AUTO},
    };
    for (auto &n : names)
        if (std::strcmp(s, n.first) == 0) return n.second;
    return -1;
}

struct Stashed {  // a message that arrived before its all-reduce started
    int peer;
    std::string name;
    uint32_t flags;
    std::vector<char> data;
};

int read_exact(int fd, void *buf, size_t n)
{
    char *p = static_cast<char *>(buf);
    while (n > 0) {
        ssize_t r = ::read(fd, p, n);
        if (r < 0 && errno == EINTR) continue;
        if (r < 0) return fail(KF_ERR_IO, std::string("read: ") + strerror(errno));
        if (r == 0) return fail(KF_ERR_IO, "read: unexpected end of stream");
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

int write_all(int fd, struct iovec *iov, int cnt)
{
    while (cnt > 0) {
        ssize_t w = writev_nosig(fd, iov, cnt);
        if (w < 0) {
            if (errno == EINTR) continue;
            return fail(KF_ERR_IO, std::string("writev: ") + strerror(errno));
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

inline void put_le32(unsigned char *p, uint32_t v)
{
    p[0] = v & 0xff;
    p[1] = (v >> 8) & 0xff;
    p[2] = (v >> 16) & 0xff;
    p[3] = (v >> 24) & 0xff;
}

// One rchannel message written in parts (the framing of kf_rch_send,
// message.go:90-101,160-198): the header and the body length first, then the
// body as its pieces become ready. The receiver sees one message.
int write_msg_header(int fd, const std::string &name, uint32_t flags, uint32_t len)
{
    unsigned char a[4], b[4], c[4];
    put_le32(a, static_cast<uint32_t>(name.size()));
    put_le32(b, flags);
    put_le32(c, len);
    struct iovec iov[4] = {{a, 4}, {const_cast<char *>(name.data()), name.size()}, {b, 4}, {c, 4}};
    return write_all(fd, iov, 4);
}

int write_bytes(int fd, const char *p, size_t n)
{
    struct iovec iov = {const_cast<char *>(p), n};
    return write_all(fd, &iov, 1);
}

struct SessOp;

// KUNGFU_AMD_TEST_LAUNCH_RACE=1 (a regression test's hook, off otherwise):
// the sender's first copy-out launch and the poll thread's first streamed
// launch wait here for each other (5 s at most), so both threads launch
// kf_stream kernels of a fresh session at the same moment: the r04 abort
// (profiles/r05/failures.md) came from exactly that overlap.
struct LaunchRace {
    bool on = false;
    std::mutex m;
    std::condition_variable cv;
    int arrived    = 0;
    bool used[2]   = {false, false};
    void meet(int who)
    {
        if (!on) return;
        std::unique_lock<std::mutex> l(m);
        if (used[who]) return;
        used[who] = true;
        ++arrived;
        cv.notify_all();
        cv.wait_for(l, std::chrono::seconds(5), [&] { return arrived >= 2; });
    }
};

struct SendItem {  // one chunk to every fd in `fds` (the node's successors)
    std::vector<int> fds;
    std::string name;
    uint32_t flags;
    const char *ptr;
    size_t bytes;
    void *stream;
    hipEvent_t ready;  // device mode: recorded on `stream` when the chunk is final
    bool slot_ok = false;  // device mode: its D2H into a tx slot was queued
    bool host    = false;  // device mode: `ptr` is already page-locked host memory
                           // (the root's fold wrote it there): no D2H, send once
                           // `ready` has completed
    SessOp *owner = nullptr;  // the collective whose chunk this is
    int chunk     = -1;       // its index in the collective (trace only)
    // host items folded piece by piece: one event per piece (its fold's end),
    // so the sender writes each piece once it is final
    std::vector<hipEvent_t> pieces;
    int staged_pieces = 0;    // device items: the D2H went out in this many pieces
    kf_stream::Ctl *sctl = nullptr;  // streamed: the kernel marks the pieces here
};

// KUNGFU_AMD_SESSION_TRACE=<path>: every step of every chunk, timestamped,
// written to <path>.<rank> as JSON lines when the session is destroyed
// (tools/c1_trace.py reads them). Off: one branch per step.
enum TraceTag {
    TR_OP_START, TR_OP_DONE, TR_RX_HDR, TR_RX_DONE, TR_TX_QUEUED, TR_TX_STAGED, TR_TX_READY,
    TR_TX_DONE, TR_FOLD_BEGIN, TR_FOLD_END, TR_NTAGS
};
const char *const kTraceNames[TR_NTAGS] = {"op_start", "op_done",  "rx_hdr",     "rx_done",
                                           "tx_queued", "tx_staged", "tx_ready",  "tx_done",
                                           "fold_begin", "fold_end"};
struct TraceRec {
    int64_t ns;
    int tag, chunk, arg;
    unsigned thr;  // 0 poll loop, 1 sender, 2 fold worker
};

// A buffer lent to one collective in flight: HBM staging for the k-input fold,
// or the page-locked mirror (host address p, device address dev).
struct Lease {
    char *p   = nullptr;
    char *dev = nullptr;
    size_t cap = 0;
};

// The leases of one kind: the idle ones, and how many bytes are lent out. The
// pool never holds more than `cap` bytes (idle + lent): a call that would
// need more goes without (the k-input fold falls back to the chain of
// 2-input folds, the mirror to the D2H send), so memory does not grow with the
// number of calls in flight (KUNGFU_AMD_STAGE_CAP_MB, KUNGFU_AMD_MIRROR_CAP_MB).
struct LeasePool {
    std::vector<Lease> idle;
    size_t lent = 0, idle_bytes = 0;
    size_t cap  = 0;
    bool coherent = false;  // host pools: fine-grained (a kernel waits on it live)
};

// Host mode: one received chunk body to fold into RecvBuf on a worker thread
// (the reference's recvOnto runs on the chunk's own goroutine, session.go:317-
// 323, execution.go:13-25), so the poll thread reads the next message while it
// folds. Jobs of one chunk run one after another in arrival order (the lock of
// recvOnto, session.go:258-259); `own` is chosen when the job starts.
struct FoldJob {
    SessOp *o = nullptr;
    size_t i  = 0;
    const char *own = nullptr;
    char *dst       = nullptr;
    size_t n        = 0;
    std::vector<char> *body = nullptr;
    int rc = KF_OK;
    std::string err;
};

struct SessChunk {
    std::string name;
    const Strategy *st;
    size_t pending_reduce;  // reduce-graph predecessors not yet folded
    int recv_count;
    bool bcast_done;
    bool batched;              // stage the reduce arrivals, fold them in one launch
    std::vector<int> waiting;  // reduce predecessors not yet heard from
    hipEvent_t mirror_ev;      // device mode: the last fold went to the mirror (its end)
    std::vector<hipEvent_t> piece_ev;  // ... and each of its pieces' ends (streamed send)
    bool streamed = false;             // the mirror fold marks its pieces in the op's ctl
    uint8_t sctl_used = 0;  // streamed kernels that ran on its ctl: 1 its reduce fold
                            // (ctl 0), 2 its bcast copy in (ctl 1); complete() checks err
    std::deque<FoldJob *> folds;  // host mode: received, not yet folded (front: running)
};

// One collective call (all-reduce, reduce, broadcast, subset all-reduce): the
// request, its chunk plan and its progress. Several are in flight at once on
// the async path, as the reference runs a goroutine per GoKungfuAllReduce
// call (libkungfu-comm/collective.go:34-45, main.go:184-191), their messages
// told apart by chunk name (handler/collective.go:48-64).
struct SessOp {
    const char *send = nullptr;
    char *recv       = nullptr;
    size_t count     = 0;
    KungFu_Datatype dt = KungFu_FLOAT;
    KungFu_Op op       = KungFu_SUM;
    std::string name;
    void *stream = nullptr;
    int kind     = 0;
    std::vector<Strategy> own;  // SubsetAllReduce's one strategy
    kf_done_fn done = nullptr;
    void *arg       = nullptr;
    // the plan
    const std::vector<Strategy> *L = nullptr;
    size_t isz = 0, bytes = 0;
    bool inplace = false, may_forward = true, use_mirror = false, trivial = false;
    bool mir_side = false;  // a mirror's copy to HBM went to the session's side stream
    Strategy single{Graph(0), Graph(0)};
    std::vector<std::pair<size_t, size_t>> parts;
    std::vector<SessChunk> chunks;
    size_t remaining = 0;
    Lease stage, mir;
    Lease ctl;  // streamed chunks: two kf_stream::Ctl per chunk (reduce, bcast)
    size_t sends = 0;  // its chunks queued for the sender, not yet written (kf_session::mu)
    size_t folds = 0;  // host mode: its fold jobs not yet retired by the poll thread
    int rc       = KF_OK;
    std::string err;
    // KUNGFU_AMD_OP_TIMEOUT_S: the call fails with KF_ERR_TIMEOUT when no
    // message of it has come for that long (set at its start, moved on by
    // every message it takes; 0 = no deadline)
    std::chrono::steady_clock::time_point deadline{};
};

}  // namespace

struct kf_session {
    int rank = 0, size = 1;
    std::string dir;
    uint32_t token  = 0;
    int device_mode = 1;
    int strategy    = KungFu_BinaryTreeStar;  // kungfu-run default (flags.go:90)
    int hash_name   = 1;                      // NAME (config.go:45)
    std::vector<Strategy> sl;
    std::vector<PeerAddr> peers;           // rank -> address (KUNGFU_INIT_PEERS)
    int listen_unix = -1, listen_tcp = -1;
    std::unordered_map<int, int> out_fd, in_fd;  // peer -> fd
    kf_ingest_t *ingest = nullptr;
    // device mode: page-locked outgoing chunk slots (sender thread). The
    // sender copies the next queued chunks' bytes out of HBM while it writes
    // the current one to its sockets, so a chunk's D2H is off the critical
    // path of the one before it (KUNGFU_AMD_TX_SLOTS, 1 = copy, send, copy...)
    std::vector<void *> tx;
    std::vector<hipEvent_t> tx_done;  // one per slot: its D2H has landed
    size_t tx_ahead = 2;              // D2H issued ahead of the write (KUNGFU_AMD_TX_AHEAD)
    // device mode: a chunk moves through each stage in pieces of this many
    // bytes (KUNGFU_AMD_PIECE_KB; 0 = whole chunks, the default): the D2H
    // before a send, the fold or copy after a receive, the send of a fold's
    // result, so a chunk's GPU and socket stages overlap instead of running in
    // series. Every piece costs a launch or copy plus an event on the thread
    // that reads the socket; over unix sockets that loses (C1 np = 2: 0.78 ms
    // at 256 KiB, 1.01 at 128, 0.69 at 512, 0.66 whole), so it
    // is for links slow enough to hide a launch per piece (TCP between hosts)
    uint32_t piece = 0;
    // streamed chunks (KUNGFU_AMD_STREAM; kf_stream.hpp): one kernel per
    // chunk, launched before the body arrives, folds or copies it as it lands
    // and marks pieces of stream_piece bytes done for the sender. A mask of
    // the stages streamed ("out": a leaf's copy out of HBM before its send,
    // "fold": the completing fold, into the mirror and sent piece by piece —
    // the default; "in": a bcast copy in; "1" all three, "0" none; and two
    // that stream only where a stage is on the critical path: "last", the
    // copy in of a call's last chunk, and "idle", the copy out of a chunk the
    // sender will write at once, nothing staged ahead of it)
    enum { kStreamOut = 1, kStreamFold = 2, kStreamIn = 4, kStreamInLast = 8, kStreamOutIdle = 16 };
    int stream_mode        = 0;
    uint32_t stream_piece  = 64u << 10;
    int stream_deadline_ms = 30000;
    LeasePool ctl_pool;
    std::vector<kf_stream::Ctl *> tx_ctl, tx_ctl_dev;  // per tx slot (copy-out)
    std::vector<void *> tx_dev;                         // tx slots as the GPU sees them
    std::vector<hipEvent_t> tx_piece_ev;  // [slot][piece]: that piece's D2H landed
    size_t max_pieces = 0;
    hipStream_t tx_stream  = nullptr;  // sender's D2H stream
    hipStream_t mir_stream = nullptr;  // the bcast root's mirror -> HBM copies
    hipStream_t wait_stream = nullptr;  // streamed kernels while they wait for a body
                                        // (when the caller's stream holds others and
                                        // other sessions live in the process)
    bool counted = false;               // in g_device_sessions
    void *waiting_stream() const
    {
        return g_device_sessions.load(std::memory_order_relaxed) > 1 ? wait_stream : nullptr;
    }
    std::vector<hipEvent_t> ev_pool;  // free "chunk is final" events
    std::mutex ev_mu;
    kf_host_reduce_fn host_fn = nullptr;
    std::vector<char> scratch;  // host-mode landing buffer (one chunk, inline folds)
    // host mode: fold workers (KUNGFU_AMD_HOST_FOLD_THREADS, 0 = fold inline
    // on the poll thread); finished jobs go back to the poll thread, which
    // alone touches the collectives' state, through fdone + wake()
    int fold_threads = -1;  // -1: not decided yet
    std::vector<std::thread> fold_workers;
    std::mutex fmu;
    std::condition_variable fcv;
    std::deque<FoldJob *> fq, fdone;
    bool fstop = false;
    std::vector<std::vector<char> *> fbodies;  // free chunk bodies (poll thread)
    // device mode: a multi-predecessor node stages its arrivals in HBM and
    // folds them in one k-input launch (1), or folds each as it lands, the
    // reference's 2-input recvOnto chain (0, the default since round 4: with
    // the completing fold streamed the chain wins at every np measured —
    // C1 np = 3 / 4 / 8: 1.05 / 1.33 / 3.07 ms against 1.29 / 1.44 / 3.28;
    // DESIGN.md §4)
    int batch_fold = 0;
    // per collective in flight, lent from these pools (device mode):
    //  * HBM staging for the k-input fold: [predecessor arrival][bucket bytes];
    //  * a page-locked mirror of the bucket. A node that sends its finished
    //    fold onward (a star or tree root to its bcast successors, an inner
    //    tree node up) folds straight into it — the kernel writes the result
    //    over PCIe while it reads — so the sender has no D2H to wait for; the
    //    node's own HBM copy follows as an H2D off the critical path.
    //    KUNGFU_AMD_ROOT_MIRROR=0 turns it off (A/B).
    LeasePool stage_pool, mirror_pool;
    bool mirror        = true;
    int device         = 0;        // device mode: the GPU the session was created on
    kf_stream::Board *board = nullptr;  // device mode: the streamed kernels' device words
    LaunchRace race;                    // KUNGFU_AMD_TEST_LAUNCH_RACE
    // KUNGFU_AMD_OP_TIMEOUT_S (0: none): bounds each call's wait for its
    // messages (the poll) and every socket read and write (SO_RCVTIMEO /
    // SO_SNDTIMEO), so a peer that stalls fails the call instead of hanging it
    int op_timeout_ms = 0;
    // peers whose connection to us reached EOF (the poll loop, under run_mu):
    // a call that still expects a message from one fails at once
    std::unordered_set<int> closed;
    char *barrier_dev  = nullptr;  // device mode: the barrier's zeroed u8 workspace
    // KUNGFU_AMD_SESSION_TRACE (see TraceRec)
    std::string trace_path;
    std::mutex tmu;
    std::vector<TraceRec> trec;
    void tr(int tag, int chunk, int arg, unsigned thr)
    {
        if (trace_path.empty()) return;
        // CLOCK_MONOTONIC: one clock for every peer process on the host
        const int64_t ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::steady_clock::now().time_since_epoch())
                               .count();
        std::lock_guard<std::mutex> l(tmu);
        trec.push_back({ns, tag, chunk, arg, thr});
    }
    void dump_trace()
    {
        if (trace_path.empty()) return;
        FILE *f = std::fopen((trace_path + "." + std::to_string(rank)).c_str(), "w");
        if (!f) return;
        for (const auto &r : trec) {
            std::fprintf(f, "{\"t_us\": %.3f, \"ev\": \"%s\", \"chunk\": %d, \"arg\": %d, \"thr\": %u}\n",
                         r.ns / 1e3, kTraceNames[r.tag], r.chunk, r.arg, r.thr);
        }
        std::fclose(f);
    }
    std::deque<Stashed> stash;  // per-name mailbox for early messages
    std::mutex run_mu;          // one poll loop over the sockets at a time
    // the first failure of a call in flight (a dead peer, an op deadline, a
    // torn socket) breaks the session for good: late messages of the failed
    // call could otherwise be replayed from the stash into the next call that
    // reuses its name (tensor names repeat every step), so every later call
    // fails until kf_session_destroy. Guarded by run_mu.
    int broken_rc = KF_OK;
    std::string broken_err;
    int wake_fd = -1;           // eventfd: a submission, or an op's last chunk sent

    // sender thread
    std::thread sender;
    std::mutex mu;
    std::condition_variable cv_work, cv_idle;
    std::deque<SendItem> queue;
    size_t inflight = 0;
    bool stopping   = false;
    int send_rc     = KF_OK;
    std::string send_err;

    // async all-reduces: a worker thread runs every submitted one at once in
    // one poll loop (run(nullptr)), each started as soon as it is submitted,
    // so peers may start their names in different orders (a goroutine per
    // call in the reference, main.go:184-191); done(status, arg) as each
    // completes. A name submitted again waits for its previous call.
    std::thread aworker;
    std::mutex amu;
    std::condition_variable acv, aidle;
    std::deque<SessOp *> aq;  // submitted, not yet started
    size_t apending = 0;      // queued + running
    bool astop      = false;
    int arc         = KF_OK;  // first failure since the last wait_all
    std::string aerr;

    void wake()
    {
        const uint64_t one = 1;
        if (wake_fd >= 0) (void)!::write(wake_fd, &one, sizeof(one));
    }

    int submit(SessOp *op)
    {
        {
            std::lock_guard<std::mutex> l(amu);
            if (astop) return KF_ERR_ARG;
            if (!aworker.joinable()) {
                aworker = std::thread([this] {
                    if (device_mode) (void)hipSetDevice(device);
                    (void)run(nullptr);
                });
            }
            aq.push_back(op);
            ++apending;
        }
        acv.notify_one();
        wake();
        return KF_OK;
    }

    int wait_all()
    {
        std::unique_lock<std::mutex> l(amu);
        aidle.wait(l, [&] { return apending == 0; });
        const int rc = arc;
        if (rc != KF_OK) t_sess_error = aerr;
        arc = KF_OK;
        aerr.clear();
        return rc;
    }

    ~kf_session()
    {
        if (aworker.joinable()) {  // drain the queued all-reduces first
            {
                std::lock_guard<std::mutex> l(amu);
                astop = true;
            }
            acv.notify_all();
            wake();
            aworker.join();
        }
        if (!fold_workers.empty()) {
            {
                std::lock_guard<std::mutex> l(fmu);
                fstop = true;
            }
            fcv.notify_all();
            for (auto &t : fold_workers) t.join();
        }
        for (auto *b : fbodies) delete b;
        if (sender.joinable()) {
            {
                std::lock_guard<std::mutex> l(mu);
                stopping = true;
            }
            cv_work.notify_all();
            sender.join();
        }
        dump_trace();
        for (auto &kv : out_fd) ::close(kv.second);
        for (auto &kv : in_fd) ::close(kv.second);
        if (listen_unix >= 0) {
            ::close(listen_unix);
            ::unlink(sock_path(dir, peers[rank]).c_str());
        }
        if (listen_tcp >= 0) ::close(listen_tcp);
        if (ingest) kf_ingest_destroy(ingest);
        for (auto p : tx) (void)hipHostFree(p);
        for (auto e : tx_done) (void)hipEventDestroy(e);
        for (auto e : tx_piece_ev) (void)hipEventDestroy(e);
        for (auto e : ev_pool) (void)hipEventDestroy(e);
        if (tx_stream) (void)hipStreamDestroy(tx_stream);
        if (mir_stream) (void)hipStreamDestroy(mir_stream);
        if (wait_stream) (void)hipStreamDestroy(wait_stream);
        if (counted) g_device_sessions.fetch_sub(1, std::memory_order_relaxed);
        for (auto &l : stage_pool.idle) (void)hipFree(l.p);
        for (auto &l : mirror_pool.idle) (void)hipHostFree(l.p);
        for (auto &l : ctl_pool.idle) (void)hipHostFree(l.p);
        if (!tx_ctl.empty()) (void)hipHostFree(tx_ctl[0]);
        if (barrier_dev) (void)hipFree(barrier_dev);
        kf_stream::board_destroy(board);  // every kernel on it was synced by complete()
        if (wake_fd >= 0) ::close(wake_fd);
    }

    void sender_loop()
    {
        // device mode: items whose D2H into slot (first_slot + i) % nslot
        // has been issued, oldest first
        std::deque<SendItem> staged;
        size_t first_slot = 0;
        const size_t nslot = device_mode ? tx.size() : 0;
        for (;;) {
            SendItem it;
            {
                std::unique_lock<std::mutex> l(mu);
                if (staged.empty()) cv_work.wait(l, [&] { return stopping || !queue.empty(); });
                // issue the D2H of queued chunks into free slots, at most
                // tx_ahead of them before the oldest is written: a D2H takes a
                // fraction of a socket write, and every D2H issued first delays
                // the first write by its host-side cost
                while (device_mode && staged.size() < std::min(nslot, tx_ahead) && !queue.empty()) {
                    SendItem q = queue.front();
                    queue.pop_front();
                    l.unlock();
                    const size_t slot = (first_slot + staged.size()) % nslot;
                    q.slot_ok = send_rc == KF_OK && stage_d2h(q, slot, staged.empty());
                    tr(TR_TX_STAGED, q.chunk, static_cast<int>(q.flags), 1);
                    staged.push_back(std::move(q));
                    l.lock();
                }
                if (staged.empty() && queue.empty()) return;  // stopping, nothing left
                if (!device_mode) {
                    it = queue.front();
                    queue.pop_front();
                }
            }
            int rc = KF_OK;
            std::string err;
            if (device_mode) {
                it = std::move(staged.front());
                staged.pop_front();
                const size_t slot = first_slot;
                first_slot        = (first_slot + 1) % nslot;
                if (send_rc == KF_OK) rc = send_staged(it, slot, &err);
            } else if (send_rc == KF_OK) {
                rc = send_item(it, &err);
            }
            tr(TR_TX_DONE, it.chunk, static_cast<int>(it.flags), 1);
            bool last = false;
            {
                std::lock_guard<std::mutex> l(mu);
                if (rc != KF_OK && send_rc == KF_OK) {
                    send_rc  = rc;
                    send_err = err;
                }
                if (it.owner) last = --it.owner->sends == 0;
                if (--inflight == 0 || last) cv_idle.notify_all();
            }
            if (last) wake();  // that collective may complete now
        }
    }

    // Queue the D2H of a device chunk into tx slot `slot` behind the event that
    // marks the chunk final on the caller's stream; tx_done[slot] marks it landed.
    bool stage_d2h(SendItem &it, size_t slot, bool idle)
    {
        if (it.host) return it.ready != nullptr;  // synced at send time
        bool ok = it.ready && it.bytes <= kChunk + 4096 &&
                  hipStreamWaitEvent(tx_stream, it.ready, 0) == hipSuccess;
        const size_t np = piece ? (it.bytes + piece - 1) / piece : 0;
        const bool stream_out = (stream_mode & kStreamOut) || ((stream_mode & kStreamOutIdle) && idle);
        if (ok && stream_out && it.bytes > 0) {  // one kernel, pieces marked as they land
            race.meet(0);
            kf_stream::reset(tx_ctl[slot], stream_piece);
            ok = kf_stream::launch_copy_out(it.ptr, tx_dev[slot], static_cast<uint32_t>(it.bytes),
                                            stream_piece, tx_ctl_dev[slot], tx_stream) == KF_OK;
            it.sctl = tx_ctl[slot];
        } else if (ok && np >= 2 && np <= max_pieces) {  // piece by piece, an event each
            for (size_t k = 0; k < np && ok; ++k) {
                const size_t off = k * piece, pl = std::min<size_t>(piece, it.bytes - off);
                ok = hipMemcpyAsync(static_cast<char *>(tx[slot]) + off, it.ptr + off, pl,
                                    hipMemcpyDeviceToHost, tx_stream) == hipSuccess &&
                     hipEventRecord(tx_piece_ev[slot * max_pieces + k], tx_stream) == hipSuccess;
            }
            it.staged_pieces = static_cast<int>(np);
        } else if (kf_stream::copy_kernels()) {
            ok = ok && kf_stream::launch_copy(tx_dev[slot], it.ptr, it.bytes, tx_stream) == KF_OK;
        } else {
            ok = ok &&
                 hipMemcpyAsync(tx[slot], it.ptr, it.bytes, hipMemcpyDeviceToHost, tx_stream) ==
                     hipSuccess;
        }
        ok = ok && hipEventRecord(tx_done[slot], tx_stream) == hipSuccess;
        if (it.ready) {
            std::lock_guard<std::mutex> l(ev_mu);
            ev_pool.push_back(it.ready);
            it.ready = nullptr;
        }
        return ok;
    }

    // One whole message per successor in turn: the header, then each piece
    // once `ready(k)` (for the first successor; the later ones find every
    // piece landed). A message is never interleaved with another: a peer
    // that has started reading it blocks until it ends, so a sender that
    // moved on to a second socket midway could wait on a peer that waits on
    // it (three peers, each stuck in the middle of another's message).
    int send_pieces(const SendItem &it, const char *data, size_t np,
                    const std::function<bool(size_t)> &ready, std::string *err)
    {
        size_t landed = 0;
        for (int fd : it.fds) {
            if (write_msg_header(fd, it.name, it.flags, static_cast<uint32_t>(it.bytes)) != KF_OK) {
                *err = t_sess_error;
                return KF_ERR_IO;
            }
            for (size_t k = 0; k < np; ++k) {
                if (k >= landed) {
                    if (!ready(k)) {
                        *err = "a piece of an outgoing chunk did not land";
                        return KF_ERR_HIP;
                    }
                    landed = k + 1;
                }
                const size_t off = k * piece, pl = std::min<size_t>(piece, it.bytes - off);
                if (write_bytes(fd, data + off, pl) != KF_OK) {
                    *err = t_sess_error;
                    return KF_ERR_IO;
                }
            }
        }
        return KF_OK;
    }

    // One message per successor, its body written in runs of pieces as the
    // kernel marks them final in `c` (the first successor waits for them).
    int send_streamed(const SendItem &it, const char *data, const kf_stream::Ctl *c,
                      std::string *err)
    {
        const uint32_t len = static_cast<uint32_t>(it.bytes);
        const uint32_t np  = (len + stream_piece - 1) / stream_piece;
        uint32_t landed    = 0;  // pieces known final
        for (int fd : it.fds) {
            if (write_msg_header(fd, it.name, it.flags, len) != KF_OK) {
                *err = t_sess_error;
                return KF_ERR_IO;
            }
            for (uint32_t k = 0; k < np;) {
                if (k >= landed) {
                    const int w = kf_stream::wait_piece(c, k, len, stream_deadline_ms);
                    if (w != KF_OK) {
                        *err = w == KF_ERR_TIMEOUT ? "a streamed chunk's piece did not become final"
                                                   : "a streamed chunk's kernel gave up waiting";
                        return w;
                    }
                    landed = k + kf_stream::ready_run(c, k, len);
                    if (landed == np) tr(TR_FOLD_END, it.chunk, 0, 1);  // every piece final
                }
                const size_t b = static_cast<size_t>(k) * stream_piece;
                const size_t e = std::min<size_t>(static_cast<size_t>(landed) * stream_piece, len);
                if (write_bytes(fd, data + b, e - b) != KF_OK) {
                    *err = t_sess_error;
                    return KF_ERR_IO;
                }
                k = landed;
            }
        }
        return KF_OK;
    }

    int send_staged(SendItem &it, size_t slot, std::string *err)
    {
        if (it.sctl && it.slot_ok) {  // streamed: the mirror fold's or the copy-out's pieces
            tr(TR_TX_READY, it.chunk, static_cast<int>(it.flags), 1);
            const char *data = it.host ? it.ptr : static_cast<const char *>(tx[slot]);
            const int rc     = send_streamed(it, data, it.sctl, err);
            if (!it.host && rc == KF_OK && hipEventSynchronize(tx_done[slot]) != hipSuccess) {
                *err = "D2H of an outgoing chunk failed";
                return KF_ERR_HIP;
            }
            if (it.host) {
                const bool synced = hipEventSynchronize(it.ready) == hipSuccess;
                std::lock_guard<std::mutex> l(ev_mu);
                ev_pool.push_back(it.ready);
                it.ready = nullptr;
                if (rc == KF_OK && !synced) {
                    *err = "the fold of an outgoing chunk failed";
                    return KF_ERR_HIP;
                }
            }
            return rc;
        }
        if (it.host && !it.pieces.empty()) {  // the fold writes the mirror piece by piece
            int rc = KF_ERR_HIP;
            if (it.slot_ok) {
                tr(TR_TX_READY, it.chunk, static_cast<int>(it.flags), 1);
                rc = send_pieces(it, it.ptr, it.pieces.size(), [&](size_t k) {
                    return hipEventSynchronize(it.pieces[k]) == hipSuccess;
                }, err);
            }
            const bool synced = hipEventSynchronize(it.ready) == hipSuccess;
            {
                std::lock_guard<std::mutex> l(ev_mu);
                ev_pool.push_back(it.ready);
                it.ready = nullptr;
                for (auto e : it.pieces) ev_pool.push_back(e);
                it.pieces.clear();
            }
            if (rc == KF_OK && !synced) {
                *err = "the fold of an outgoing chunk failed";
                rc   = KF_ERR_HIP;
            }
            if (!it.slot_ok) *err = "the fold of an outgoing chunk failed";
            return rc;
        }
        if (!it.host && it.slot_ok && it.staged_pieces >= 2) {  // D2H landing piece by piece
            tr(TR_TX_READY, it.chunk, static_cast<int>(it.flags), 1);
            const int rc = send_pieces(it, static_cast<const char *>(tx[slot]),
                                       static_cast<size_t>(it.staged_pieces), [&](size_t k) {
                return hipEventSynchronize(tx_piece_ev[slot * max_pieces + k]) == hipSuccess;
            }, err);
            if (rc == KF_OK && hipEventSynchronize(tx_done[slot]) != hipSuccess) {
                *err = "D2H of an outgoing chunk failed";
                return KF_ERR_HIP;
            }
            return rc;
        }
        if (it.host) {  // the fold wrote the chunk to host memory: wait for it
            const bool ok = it.slot_ok && hipEventSynchronize(it.ready) == hipSuccess;
            {
                std::lock_guard<std::mutex> l(ev_mu);
                ev_pool.push_back(it.ready);
                it.ready = nullptr;
            }
            if (!ok) {
                *err = "the fold of an outgoing chunk failed";
                return KF_ERR_HIP;
            }
        } else if (!it.slot_ok || hipEventSynchronize(tx_done[slot]) != hipSuccess) {
            *err = "D2H of an outgoing chunk failed";
            return KF_ERR_HIP;
        }
        tr(TR_TX_READY, it.chunk, static_cast<int>(it.flags), 1);
        const char *data = it.host ? it.ptr : static_cast<const char *>(tx[slot]);
        for (int fd : it.fds) {
            const int rc = kf_rch_send(fd, it.name.c_str(), it.flags, data,
                                       static_cast<uint32_t>(it.bytes));
            if (rc != KF_OK) {
                *err = kf_ingest_last_error();
                return rc;
            }
        }
        return KF_OK;
    }

    // Device mode: ONE copy of the chunk to page-locked memory, then the same
    // bytes to every successor (a star root sends its reduced chunk to np-1
    // peers). The stream sync also orders the copy after the chunk's fold.
    // An event marking "this chunk is final on the caller's stream" (its fold
    // was queued before), so the sender waits for that chunk only, not for
    // the folds of later chunks queued on the same stream meanwhile.
    hipEvent_t chunk_ready(void *stream)
    {
        hipEvent_t e = nullptr;
        {
            std::lock_guard<std::mutex> l(ev_mu);
            if (!ev_pool.empty()) {
                e = ev_pool.back();
                ev_pool.pop_back();
            }
        }
        if (!e && hipEventCreateWithFlags(&e, kf_sync::event_flags()) != hipSuccess) return nullptr;
        if (hipEventRecord(e, static_cast<hipStream_t>(stream)) != hipSuccess) {
            (void)hipEventDestroy(e);
            return nullptr;
        }
        return e;
    }

    // n events from the pool (new ones if it runs dry)
    bool take_events(size_t n, std::vector<hipEvent_t> *out)
    {
        out->clear();
        {
            std::lock_guard<std::mutex> l(ev_mu);
            while (out->size() < n && !ev_pool.empty()) {
                out->push_back(ev_pool.back());
                ev_pool.pop_back();
            }
        }
        while (out->size() < n) {
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, kf_sync::event_flags()) != hipSuccess) {
                give_events(*out);
                return false;
            }
            out->push_back(e);
        }
        return true;
    }

    void give_events(std::vector<hipEvent_t> &evs)
    {
        std::lock_guard<std::mutex> l(ev_mu);
        for (auto e : evs) ev_pool.push_back(e);
        evs.clear();
    }

    int send_item(const SendItem &it, std::string *err)  // host mode
    {
        for (int fd : it.fds) {
            const int rc = kf_rch_send(fd, it.name.c_str(), it.flags, it.ptr,
                                       static_cast<uint32_t>(it.bytes));
            if (rc != KF_OK) {
                *err = kf_ingest_last_error();
                return rc;
            }
        }
        return KF_OK;
    }

    void enqueue(SendItem it)
    {
        tr(TR_TX_QUEUED, it.chunk, static_cast<int>(it.flags), 0);
        {
            std::lock_guard<std::mutex> l(mu);
            if (it.owner) ++it.owner->sends;
            queue.push_back(std::move(it));
            ++inflight;
        }
        cv_work.notify_one();
    }

    int drain()
    {
        std::unique_lock<std::mutex> l(mu);
        cv_idle.wait(l, [&] { return inflight == 0; });
        if (send_rc != KF_OK) {
            const int rc = send_rc;
            send_rc      = KF_OK;
            return fail(rc, "send: " + send_err);
        }
        return KF_OK;
    }

    bool colocated(int p) const { return peers[p].ip == peers[rank].ip; }

    std::vector<uint32_t> hosts() const
    {
        std::vector<uint32_t> h;
        for (auto &p : peers) h.push_back(p.ip);
        return h;
    }

    int rank_of(uint32_t ip, uint16_t port) const
    {
        for (size_t r = 0; r < peers.size(); ++r)
            if (peers[r] == PeerAddr{ip, port}) return static_cast<int>(r);
        return -1;
    }

    // a connected, handshaken simplex connection to peer p (client_pool.go),
    // unix socket if colocated else TCP, retried like ConnRetryCount/Period
    int dial(int p, int *out)
    {
        const PeerAddr &to = peers[p];
        for (int attempt = 0;; ++attempt) {
            int fd = -1, ok = 0;
            if (colocated(p)) {
                fd = ::socket(AF_UNIX, SOCK_STREAM, 0);
                sockaddr_un b{};
                b.sun_family = AF_UNIX;
                std::strcpy(b.sun_path, sock_path(dir, to).c_str());
                ok = fd >= 0 && ::connect(fd, reinterpret_cast<sockaddr *>(&b), sizeof(b)) == 0;
            } else {
                fd = ::socket(AF_INET, SOCK_STREAM, 0);
                sockaddr_in b{};
                b.sin_family      = AF_INET;
                b.sin_port        = htons(to.port);
                b.sin_addr.s_addr = htonl(to.ip);
                ok = fd >= 0 && ::connect(fd, reinterpret_cast<sockaddr *>(&b), sizeof(b)) == 0;
                if (ok) {
                    int one = 1;
                    (void)::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
                }
            }
            if (ok) {
                const int rc = kf_rch_client_handshake(fd, KF_RCH_CONN_COLLECTIVE, peers[rank].port,
                                                       peers[rank].ip, token);
                if (rc != KF_OK) {
                    t_sess_error = kf_ingest_last_error();
                    ::close(fd);
                    return rc;
                }
                *out = fd;
                return KF_OK;
            }
            const int err = errno;
            if (fd >= 0) ::close(fd);
            if (attempt + 1 >= kConnRetry) {
                return fail(KF_ERR_IO, "connect to peer " + std::to_string(p) + ": " + strerror(err));
            }
            ::usleep(kRetryPeriodUs);
        }
    }

    int listen_on()
    {
        bool any_local = false, any_remote = false;
        for (int p = 0; p < size; ++p) {
            if (p == rank) continue;
            (colocated(p) ? any_local : any_remote) = true;
        }
        if (any_local) {  // unix server (server.go:48-70)
            const std::string path = sock_path(dir, peers[rank]);
            ::unlink(path.c_str());
            listen_unix = ::socket(AF_UNIX, SOCK_STREAM, 0);
            sockaddr_un a{};
            a.sun_family = AF_UNIX;
            if (path.size() >= sizeof(a.sun_path)) return fail(KF_ERR_ARG, "socket path too long");
            std::strcpy(a.sun_path, path.c_str());
            if (listen_unix < 0 ||
                ::bind(listen_unix, reinterpret_cast<sockaddr *>(&a), sizeof(a)) < 0 ||
                ::listen(listen_unix, size) < 0) {
                return fail(KF_ERR_IO, "bind/listen " + path + ": " + strerror(errno));
            }
        }
        if (any_remote) {  // tcp server (server.go:24-46), on this peer's own address
            listen_tcp = ::socket(AF_INET, SOCK_STREAM, 0);
            int one    = 1;
            if (listen_tcp >= 0)
                (void)::setsockopt(listen_tcp, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
            sockaddr_in a{};
            a.sin_family      = AF_INET;
            a.sin_port        = htons(peers[rank].port);
            a.sin_addr.s_addr = htonl(peers[rank].ip);
            if (listen_tcp < 0 ||
                ::bind(listen_tcp, reinterpret_cast<sockaddr *>(&a), sizeof(a)) < 0 ||
                ::listen(listen_tcp, size) < 0) {
                return fail(KF_ERR_IO, "bind/listen tcp port " + std::to_string(peers[rank].port) +
                                           ": " + strerror(errno));
            }
        }
        return KF_OK;
    }

    int connect_all()
    {
        int rc = listen_on();
        if (rc != KF_OK) return rc;
        // full mesh: one simplex connection per ordered pair (client_pool.go);
        // the acceptor learns who dialled from the connection header
        int accept_rc = KF_OK;
        std::string accept_err;
        std::thread acceptor([&] {
            std::vector<pollfd> ls;
            if (listen_unix >= 0) ls.push_back({listen_unix, POLLIN, 0});
            if (listen_tcp >= 0) ls.push_back({listen_tcp, POLLIN, 0});
            int got = 0;
            while (got < size - 1) {
                if (::poll(ls.data(), ls.size(), -1) < 0) {
                    if (errno == EINTR) continue;
                    accept_rc  = KF_ERR_IO;
                    accept_err = std::string("poll: ") + strerror(errno);
                    return;
                }
                for (auto &l : ls) {
                    if (!(l.revents & (POLLIN | POLLHUP | POLLERR))) continue;
                    int c = ::accept(l.fd, nullptr, nullptr);
                    if (c < 0) {
                        accept_rc  = KF_ERR_IO;
                        accept_err = std::string("accept: ") + strerror(errno);
                        return;
                    }
                    if (l.fd == listen_tcp) {
                        int one = 1;
                        (void)::setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
                    }
                    uint16_t type = 0, port = 0;
                    uint32_t ip = 0;
                    int hrc     = kf_rch_server_handshake(c, token, &type, &port, &ip);
                    const int p = hrc == KF_OK ? rank_of(ip, port) : -1;
                    if (p < 0 || p == rank || in_fd.count(p)) {
                        accept_rc  = hrc != KF_OK ? hrc : KF_ERR_PROTO;
                        accept_err = hrc != KF_OK ? std::string(kf_ingest_last_error())
                                                  : "connection from a peer not in the list";
                        ::close(c);
                        return;
                    }
                    in_fd[p] = c;
                    ++got;
                }
            }
        });
        for (int p = 0; p < size && rc == KF_OK; ++p) {
            if (p == rank) continue;
            int fd = -1;
            rc     = dial(p, &fd);
            if (rc == KF_OK) out_fd[p] = fd;
        }
        if (rc != KF_OK) {  // unblock the acceptor
            if (listen_unix >= 0) ::shutdown(listen_unix, SHUT_RDWR);
            if (listen_tcp >= 0) ::shutdown(listen_tcp, SHUT_RDWR);
        }
        acceptor.join();
        if (rc != KF_OK) return rc;
        if (accept_rc != KF_OK) return fail(accept_rc, accept_err);
        return KF_OK;
    }

    // kind: kAllReduce (both graphs of the chunk's strategy), kReduce (the
    // first strategy's reduce graph only, Session.Reduce session.go:159-162),
    // kBroadcast (its bcast graph only, Session.Broadcast session.go:164-167)
    // slist: the strategies to pick from per chunk instead of the session's
    // (SubsetAllReduce's single forest strategy)
    int all_reduce(const char *send, char *recv, size_t count, KungFu_Datatype dt,
                   KungFu_Op op, const std::string &name, void *stream, int kind = 0,
                   const std::vector<Strategy> *slist = nullptr);

    // one collective's steps (SessOp), driven by the poll loop run()
    int plan(SessOp &o);
    bool expects(const SessOp &o, size_t i, uint32_t flags, int peer) const;
    int handle(SessOp &o, size_t i, uint32_t flags, int peer, int fd, const char *mem);
    void send_chunk(SessOp &o, size_t i, std::vector<int> fds, uint32_t fl);
    int mirror_done(SessOp &o, size_t i, char *dst);
    void finish_bcast(SessOp &o, size_t i);
    void finish_reduce(SessOp &o, size_t i);
    int complete(SessOp &o);
    int run(SessOp *one);
    bool fold_pool();
    void fold_loop();
    void start_fold(SessOp &o, size_t i);
    void retire_folds();
    bool take(LeasePool &pool, size_t need, bool host, Lease *out);
    // chunk i's control block, `which` 0 = its reduce-phase fold, 1 = its bcast
    kf_stream::Ctl *ctl_at(SessOp &o, size_t i, int which, bool dev = false)
    {
        char *base = dev ? o.ctl.dev : o.ctl.p;
        return reinterpret_cast<kf_stream::Ctl *>(base) + 2 * i + which;
    }
    void give(LeasePool &pool, Lease &l);
};

enum { kAllReduce = 0, kReduce = 1, kBroadcast = 2 };

// A buffer of at least `need` bytes from the pool: the smallest idle one that
// fits; else a new one of exactly `need` bytes, after freeing idle ones
// (largest first) only as far as the pool's cap requires. false: no buffer
// within the cap, or the allocation failed — the caller goes without.
bool kf_session::take(LeasePool &pool, size_t need, bool host, Lease *out)
{
    int best = -1;
    for (size_t i = 0; i < pool.idle.size(); ++i) {
        if (pool.idle[i].cap >= need && (best < 0 || pool.idle[i].cap < pool.idle[best].cap)) {
            best = static_cast<int>(i);
        }
    }
    if (best >= 0) {
        *out = pool.idle[best];
        pool.idle.erase(pool.idle.begin() + best);
        pool.idle_bytes -= out->cap;
        pool.lent += out->cap;
        return true;
    }
    if (need > pool.cap || pool.lent + need > pool.cap) return false;
    // idle buffers are too small: free the largest until the new one fits
    std::sort(pool.idle.begin(), pool.idle.end(),
              [](const Lease &a, const Lease &b) { return a.cap < b.cap; });
    while (!pool.idle.empty() && pool.lent + pool.idle_bytes + need > pool.cap) {
        Lease &l = pool.idle.back();
        host ? (void)hipHostFree(l.p) : (void)hipFree(l.p);
        pool.idle_bytes -= l.cap;
        pool.idle.pop_back();
    }
    Lease l;
    if (host) {
        void *dv = nullptr;
        const unsigned fl = pool.coherent ? hipHostMallocMapped | hipHostMallocCoherent
                                          : hipHostMallocDefault;
        if (hipHostMalloc(reinterpret_cast<void **>(&l.p), need, fl) != hipSuccess) {
            return false;
        }
        if (hipHostGetDevicePointer(&dv, l.p, 0) != hipSuccess) {
            (void)hipHostFree(l.p);
            return false;
        }
        l.dev = static_cast<char *>(dv);
    } else {
        if (hipMalloc(reinterpret_cast<void **>(&l.p), need) != hipSuccess) return false;
        l.dev = l.p;
    }
    l.cap = need;
    pool.lent += need;
    *out = l;
    return true;
}

void kf_session::give(LeasePool &pool, Lease &l)
{
    if (l.p) {
        pool.idle.push_back(l);
        pool.idle_bytes += l.cap;
        pool.lent -= l.cap;
    }
    l = Lease{};
}

// The chunk plan of one collective (session.go:301-326): chunks, their
// strategy by name hash, leases; then the chunks this node has nothing to
// receive for go out at once. o.remaining == 0 afterwards: nothing to wait for.
int kf_session::plan(SessOp &o)
{
    const std::vector<Strategy> &L = o.L ? *o.L : sl;
    o.isz     = kungfu_type_size(o.dt);
    o.inplace = o.send == o.recv;
    o.bytes   = o.count * o.isz;
    if (o.count == 0) {  // w.IsEmpty()
        o.trivial = true;
        return KF_OK;
    }
    if (size == 1) {  // every graph isolated: w.Forward()
        o.trivial = true;
        if (o.inplace) return KF_OK;
        if (device_mode) {
            hipStream_t st = static_cast<hipStream_t>(o.stream);
            if (hipMemcpyAsync(o.recv, o.send, o.bytes, hipMemcpyDeviceToDevice, st) != hipSuccess ||
                hipStreamSynchronize(st) != hipSuccess) {
                return fail(KF_ERR_HIP, "forward copy");
            }
        } else {
            std::memmove(o.recv, o.send, o.bytes);
        }
        return KF_OK;
    }
    const size_t k = (o.bytes + kChunk - 1) / kChunk;
    o.parts        = even_partition(o.count, k);
    // Reduce / Broadcast: one graph of the first strategy for every chunk (the
    // reference sends the workspace as one message; chunking it the same way
    // as the all-reduce changes no element's result)
    o.single = Strategy{o.kind == kBroadcast ? Graph(size) : L[0].reduce,
                        o.kind == kReduce ? Graph(size) : L[0].bcast};
    // runGraphs forwards SendBuf only in a graph without self loops (the bcast
    // graph) or when the node is isolated in every graph it runs
    const Strategy &sg   = o.single;
    const bool isolated  = sg.reduce.prev[rank].empty() && sg.reduce.next[rank].empty() &&
                          sg.bcast.prev[rank].empty() && sg.bcast.next[rank].empty();
    o.may_forward = o.kind != kReduce || isolated;
    o.chunks.resize(o.parts.size());
    size_t need_stage = 0;
    for (size_t i = 0; i < o.parts.size(); ++i) {
        auto &c = o.chunks[i];
        c.name  = "part::" + o.name + "[" + std::to_string(o.parts[i].first) + ":" +
                 std::to_string(o.parts[i].second) + "]";
        const uint64_t h = hash_name ? name_hash(c.name) : static_cast<uint64_t>(i);
        c.st             = o.kind == kAllReduce ? &L[h % L.size()] : &o.single;
        c.pending_reduce = c.st->reduce.prev[rank].size();
        c.waiting        = c.st->reduce.prev[rank];
        c.recv_count     = 0;
        c.bcast_done     = false;
        c.batched        = device_mode && batch_fold && o.dt != KungFu_BFLOAT16 &&
                    c.pending_reduce >= 2 && c.pending_reduce + 1 <= KF_MAX_INPUTS;
        c.mirror_ev      = nullptr;
        if (c.batched && c.pending_reduce * o.bytes > need_stage) need_stage = c.pending_reduce * o.bytes;
    }
    if (need_stage > 0 && !take(stage_pool, need_stage, false, &o.stage)) {
        // no staging within the cap: this call folds chunk by chunk as the
        // reference does (recvOnto per predecessor), same bits
        for (auto &c : o.chunks) c.batched = false;
    }
    if (device_mode && (stream_mode & (kStreamFold | kStreamIn | kStreamInLast)) &&
        !take(ctl_pool, 2 * o.chunks.size() * sizeof(kf_stream::Ctl), true, &o.ctl)) {
        o.ctl = Lease{};  // this call moves whole chunks
    }
    // the fold that completes a chunk goes to the page-locked mirror when the
    // chunk then leaves this node (reduce successors, or bcast successors of a
    // node that receives no bcast itself)
    o.use_mirror = device_mode && mirror && o.kind == kAllReduce &&
                   take(mirror_pool, o.bytes, true, &o.mir);
    o.remaining = o.chunks.size();
    for (size_t i = 0; i < o.chunks.size(); ++i) {
        if (o.chunks[i].pending_reduce == 0) {
            finish_reduce(o, i);
            if (o.chunks[i].bcast_done) --o.remaining;
        }
    }
    return KF_OK;
}

namespace
{
inline const char *cptr(const SessOp &o, const char *base, size_t i)
{
    return base + o.parts[i].first * o.isz;
}
inline size_t clen(const SessOp &o, size_t i) { return (o.parts[i].second - o.parts[i].first) * o.isz; }
inline const char *effective(const SessOp &o, size_t i)
{
    return (o.chunks[i].recv_count > 0 || o.inplace) ? cptr(o, o.recv, i) : cptr(o, o.send, i);
}
inline bool sends_onward(const SessOp &o, size_t i, int rank)
{
    const auto &st = *o.chunks[i].st;
    return !st.reduce.next[rank].empty() ||
           (st.bcast.prev[rank].empty() && !st.bcast.next[rank].empty());
}
}  // namespace

// an outgoing chunk: from the mirror if the fold wrote it there (first
// sender takes the fold's event), else from HBM (D2H by the sender)
void kf_session::send_chunk(SessOp &o, size_t i, std::vector<int> fds, uint32_t fl)
{
    auto &c = o.chunks[i];
    if (c.mirror_ev) {
        SendItem it{fds, c.name, fl, cptr(o, o.mir.p, i), clen(o, i), o.stream, c.mirror_ev};
        it.host     = true;
        it.owner    = &o;
        it.chunk    = static_cast<int>(i);
        it.pieces   = std::move(c.piece_ev);
        c.piece_ev.clear();
        if (c.streamed) it.sctl = ctl_at(o, i, 0);
        c.mirror_ev = nullptr;
        enqueue(std::move(it));
        return;
    }
    SendItem it{fds, c.name, fl, effective(o, i), clen(o, i), o.stream,
                device_mode ? chunk_ready(o.stream) : nullptr};
    it.owner = &o;
    it.chunk = static_cast<int>(i);
    enqueue(std::move(it));
}

// after the completing fold into the mirror: its end marks the chunk final
// for the sender; then this node's own copy of it goes to HBM. At the bcast
// root nothing writes that chunk of dst again in this call, so the copy runs
// on the session's side stream: the next chunk's fold on the caller's stream
// does not queue behind it (complete() waits for both streams)
int kf_session::mirror_done(SessOp &o, size_t i, char *dst)
{
    auto &c     = o.chunks[i];
    c.mirror_ev = chunk_ready(o.stream);
    if (!c.mirror_ev) return fail(KF_ERR_HIP, "mirror event");
    const bool side = mir_stream && c.st->bcast.prev[rank].empty();
    hipStream_t hs  = side ? mir_stream : static_cast<hipStream_t>(o.stream);
    const bool waited = !side || hipStreamWaitEvent(mir_stream, c.mirror_ev, 0) == hipSuccess;
    const bool copied =
        waited &&
        (kf_stream::copy_kernels()
             ? kf_stream::launch_copy(dst, cptr(o, o.mir.dev, i), clen(o, i), hs) == KF_OK
             : hipMemcpyAsync(dst, cptr(o, o.mir.p, i), clen(o, i), hipMemcpyHostToDevice, hs) ==
                   hipSuccess);
    if (!copied) {
        return fail(KF_ERR_HIP, "mirror copy to HBM");
    }
    if (side) o.mir_side = true;
    return KF_OK;
}

void kf_session::finish_bcast(SessOp &o, size_t i)  // after recvInto or at the bcast root
{
    auto &c = o.chunks[i];
    if (o.may_forward && c.st->bcast.prev[rank].empty() && c.recv_count == 0 && !o.inplace) {
        // w.Forward(): nothing received in either graph
        if (device_mode) {  // errors surface at the final stream sync
            (void)hipMemcpyAsync(const_cast<char *>(cptr(o, o.recv, i)), cptr(o, o.send, i),
                                 clen(o, i), hipMemcpyDeviceToDevice,
                                 static_cast<hipStream_t>(o.stream));
        } else {
            std::memcpy(const_cast<char *>(cptr(o, o.recv, i)), cptr(o, o.send, i), clen(o, i));
        }
    }
    std::vector<int> fds;
    for (int p : c.st->bcast.next[rank]) fds.push_back(out_fd[p]);
    if (!fds.empty()) send_chunk(o, i, fds, KF_RCH_WAIT_RECV_BUF);
    c.bcast_done = true;
}

void kf_session::finish_reduce(SessOp &o, size_t i)  // all predecessors folded
{
    auto &c = o.chunks[i];
    std::vector<int> fds;
    for (int p : c.st->reduce.next[rank]) fds.push_back(out_fd[p]);
    if (!fds.empty()) send_chunk(o, i, fds, KF_RCH_NO_FLAG);
    if (c.st->bcast.prev[rank].empty()) finish_bcast(o, i);
}

// Is this message (from `peer`) one chunk i still waits for in THIS call?
// The same names recur every step, and a peer that has finished this step
// may already send the next one's; such a message waits in the stash, as in
// the reference's per-name mailbox (handler/collective.go:27-61).
bool kf_session::expects(const SessOp &o, size_t i, uint32_t flags, int peer) const
{
    const auto &c = o.chunks[i];
    if (flags & KF_RCH_WAIT_RECV_BUF) {
        const auto &bp = c.st->bcast.prev[rank];
        return !c.bcast_done && std::find(bp.begin(), bp.end(), peer) != bp.end();
    }
    return std::find(c.waiting.begin(), c.waiting.end(), peer) != c.waiting.end();
}

// one message for chunk i: from the socket fd (mem == nullptr) or from a
// stashed copy in host memory
int kf_session::handle(SessOp &o, size_t i, uint32_t flags, int peer, int fd, const char *mem)
{
    auto &c = o.chunks[i];
    if (!(flags & KF_RCH_WAIT_RECV_BUF)) {
        c.waiting.erase(std::find(c.waiting.begin(), c.waiting.end(), peer));
    }
    const size_t n     = o.parts[i].second - o.parts[i].first;
    char *dst          = const_cast<char *>(cptr(o, o.recv, i));
    const uint32_t len = static_cast<uint32_t>(clen(o, i));
    void *stream       = o.stream;
    int r              = KF_OK;
    const bool pieces   = device_mode && !mem && piece && len > piece;
    const bool streamed = device_mode && !mem && o.ctl.p && len > 0;
    if (flags & KF_RCH_WAIT_RECV_BUF) {  // bcast: recvInto RecvBuf
        const bool stream_in = streamed && ((stream_mode & kStreamIn) ||
                                            ((stream_mode & kStreamInLast) && o.remaining == 1));
        if (device_mode && mem) {
            r = kf_ingest_copy_host(ingest, mem, len, dst, stream);
        } else if (device_mode && stream_in) {
            race.meet(1);
            c.sctl_used |= 2;
            r = kf_ingest_recv_into_streamed(ingest, fd, len, dst, stream, stream_piece,
                                             ctl_at(o, i, 1), ctl_at(o, i, 1, true), board,
                                             stream_deadline_ms, waiting_stream());
        } else if (device_mode) {
            r = pieces ? kf_ingest_recv_into_pieces(ingest, fd, len, dst, stream, piece)
                       : kf_ingest_recv_into(ingest, fd, len, dst, stream);
        } else if (mem) {
            std::memcpy(dst, mem, len);
        } else {
            r = kf_rch_recv_body(fd, dst, len);
        }
        if (r != KF_OK) return fail(r, kf_ingest_last_error());
        ++c.recv_count;
        finish_bcast(o, i);
        --o.remaining;
        return KF_OK;
    }
    if (c.batched) {  // stage arrival #recv_count; fold once all are in
        char *slot = o.stage.p + static_cast<size_t>(c.recv_count) * o.bytes + o.parts[i].first * o.isz;
        r = mem      ? kf_ingest_copy_host(ingest, mem, len, slot, stream)
            : pieces ? kf_ingest_recv_into_pieces(ingest, fd, len, slot, stream, piece)
                     : kf_ingest_recv_into(ingest, fd, len, slot, stream);
        if (r != KF_OK) return fail(r, kf_ingest_last_error());
        ++c.recv_count;
        if (--c.pending_reduce > 0) return KF_OK;
        const void *ins[KF_MAX_INPUTS];
        ins[0] = o.inplace ? dst : cptr(o, o.send, i);  // effective before the first receive
        for (int a = 0; a < c.recv_count; ++a) {
            ins[a + 1] = o.stage.p + static_cast<size_t>(a) * o.bytes + o.parts[i].first * o.isz;
        }
        if (o.use_mirror && sends_onward(o, i, rank)) {
            r = kf_bucket_reduce(ins, c.recv_count + 1, const_cast<char *>(cptr(o, o.mir.dev, i)), n,
                                 o.dt, o.op, stream);
            if (r != KF_OK) return fail(r, kf_last_error());
            r = mirror_done(o, i, dst);
            if (r != KF_OK) return r;
        } else {
            r = kf_bucket_reduce(ins, c.recv_count + 1, dst, n, o.dt, o.op, stream);
            if (r != KF_OK) return fail(r, kf_last_error());
        }
        finish_reduce(o, i);
        if (c.bcast_done) --o.remaining;
        return KF_OK;
    }
    // reduce: recvOnto, RecvBuf = effective o peer
    const char *own = effective(o, i);
    if (device_mode) {
        // the completing fold of a chunk that leaves this node goes to the mirror
        const bool to_mirror = o.use_mirror && c.pending_reduce == 1 && sends_onward(o, i, rank);
        char *out            = to_mirror ? const_cast<char *>(cptr(o, o.mir.dev, i)) : dst;
        // streamed: only the fold that completes the chunk (one per chunk per
        // call, so its control block is never reset under a running kernel)
        if (streamed && (stream_mode & kStreamFold) && c.pending_reduce == 1 &&
            kf_stream::supported(o.dt, o.op)) {
            race.meet(1);
            c.sctl_used |= 1;
            r = kf_ingest_recv_onto_streamed(ingest, fd, len, out, own, o.dt, stream, stream_piece,
                                             ctl_at(o, i, 0), ctl_at(o, i, 0, true), board,
                                             stream_deadline_ms, to_mirror, waiting_stream());
            if (r != KF_OK) return fail(r, kf_ingest_last_error());
            c.streamed = to_mirror;
        } else if (pieces) {
            // the completing fold into the mirror marks each piece, so the
            // sender can write it while the next pieces are read and folded
            std::vector<hipEvent_t> pev;
            if (to_mirror && !take_events((len + piece - 1) / piece, &pev)) {
                return fail(KF_ERR_HIP, "piece events");
            }
            r = kf_ingest_recv_onto_pieces(
                ingest, fd, len, out, own, n, o.dt, o.op, stream, piece,
                pev.empty() ? nullptr : reinterpret_cast<void *const *>(pev.data()),
                static_cast<int>(pev.size()));
            if (r != KF_OK) {
                give_events(pev);
                return fail(r, kf_ingest_last_error());
            }
            c.piece_ev = std::move(pev);
        } else {
            r = mem ? kf_ingest_fold_host(ingest, mem, len, out, own, n, o.dt, o.op, stream)
                    : kf_ingest_recv_onto(ingest, fd, len, out, own, n, o.dt, o.op, stream);
        }
        if (r != KF_OK) return fail(r, kf_ingest_last_error());
        if (to_mirror) {
            r = mirror_done(o, i, dst);
            if (r != KF_OK) return r;
        }
    } else if (fold_pool()) {  // the fold runs on a worker; the poll thread reads on
        auto *j = new FoldJob;
        j->o    = &o;
        j->i    = i;
        j->dst  = dst;
        j->n    = n;
        if (fbodies.empty()) {
            j->body = new std::vector<char>(kChunk + 64);
        } else {
            j->body = fbodies.back();
            fbodies.pop_back();
        }
        if (j->body->size() < len) j->body->resize(len);
        if (mem) {
            std::memcpy(j->body->data(), mem, len);
        } else {
            r = kf_rch_recv_body(fd, j->body->data(), len);
            if (r != KF_OK) {
                fbodies.push_back(j->body);
                delete j;
                return fail(r, kf_ingest_last_error());
            }
        }
        c.folds.push_back(j);
        ++o.folds;
        if (c.folds.size() == 1) start_fold(o, i);
        return KF_OK;  // recv_count / pending_reduce move when it is retired
    } else {
        const char *pd = mem;
        if (!mem) {
            r = kf_rch_recv_body(fd, scratch.data(), len);
            if (r != KF_OK) return fail(r, kf_ingest_last_error());
            pd = scratch.data();
        }
        if (host_fn) {
            if (host_fn(own, pd, dst, static_cast<int64_t>(n), static_cast<int>(o.dt),
                        static_cast<int>(o.op)) != 0) {
                return fail(KF_ERR_OP, "host reduce callback failed");
            }
        } else {
            r = kf_transform2_host(own, pd, dst, n, o.dt, o.op);
            if (r != KF_OK) return fail(r, kf_last_error());
        }
    }
    ++c.recv_count;
    if (--c.pending_reduce == 0) {
        finish_reduce(o, i);
        if (c.bcast_done) --o.remaining;
    }
    return KF_OK;
}

// Host mode: whether chunk folds go to the worker pool (started on first use)
bool kf_session::fold_pool()
{
    if (fold_threads < 0) {
        const unsigned hw = std::thread::hardware_concurrency();
        int t             = static_cast<int>(std::min(8u, std::max(1u, hw)));
        if (const char *e = std::getenv("KUNGFU_AMD_HOST_FOLD_THREADS")) t = std::max(0, std::atoi(e));
        fold_threads = t;
        for (int k = 0; k < t; ++k) fold_workers.emplace_back([this] { fold_loop(); });
    }
    return fold_threads > 0;
}

void kf_session::fold_loop()
{
    for (;;) {
        FoldJob *j = nullptr;
        {
            std::unique_lock<std::mutex> l(fmu);
            fcv.wait(l, [&] { return fstop || !fq.empty(); });
            if (fq.empty()) return;
            j = fq.front();
            fq.pop_front();
        }
        const KungFu_Datatype dt = j->o->dt;  // fixed for the collective's lifetime
        const KungFu_Op op       = j->o->op;
        tr(TR_FOLD_BEGIN, static_cast<int>(j->i), 0, 2);
        if (host_fn) {
            if (host_fn(j->own, j->body->data(), j->dst, static_cast<int64_t>(j->n),
                        static_cast<int>(dt), static_cast<int>(op)) != 0) {
                j->rc  = KF_ERR_OP;
                j->err = "host reduce callback failed";
            }
        } else {
            j->rc = kf_transform2_host(j->own, j->body->data(), j->dst, j->n, dt, op);
            if (j->rc != KF_OK) j->err = kf_last_error();
        }
        tr(TR_FOLD_END, static_cast<int>(j->i), j->rc, 2);
        {
            std::lock_guard<std::mutex> l(fmu);
            fdone.push_back(j);
        }
        wake();
    }
}

// the chunk's oldest received body goes to a worker: RecvBuf = effective o body
void kf_session::start_fold(SessOp &o, size_t i)
{
    FoldJob *j = o.chunks[i].folds.front();
    j->own     = effective(o, i);
    {
        std::lock_guard<std::mutex> l(fmu);
        fq.push_back(j);
    }
    fcv.notify_one();
}

// Every chunk received and every outgoing chunk written: the device work
// lands before the buffers return to the caller; the leases go back.
int kf_session::complete(SessOp &o)
{
    int rc = o.rc;
    if (!o.trivial && device_mode) {
        const int irc = kf_ingest_sync(ingest);
        if (irc != KF_OK && rc == KF_OK) rc = fail(irc, kf_ingest_last_error());
        if (kf_sync::stream_sync(o.stream) != KF_OK && rc == KF_OK) {
            rc = fail(KF_ERR_HIP, "stream sync");
        }
        if (o.mir_side && kf_sync::stream_sync(mir_stream) != KF_OK && rc == KF_OK) {
            rc = fail(KF_ERR_HIP, "mirror stream sync");
        }
        // a streamed kernel that gave up (its deadline, or the host's abort)
        // left its chunk without the peer's bytes: the call fails, whatever
        // the socket reads returned
        for (size_t i = 0; i < o.chunks.size() && rc == KF_OK && o.ctl.p; ++i) {
            for (int w = 0; w < 2; ++w) {
                if ((o.chunks[i].sctl_used & (1 << w)) &&
                    __atomic_load_n(&ctl_at(o, i, w)->err, __ATOMIC_ACQUIRE) != 0) {
                    rc = fail(KF_ERR_TIMEOUT, "chunk " + o.chunks[i].name +
                                                  ": its streamed kernel stopped waiting for the "
                                                  "body (KUNGFU_AMD_STREAM_TIMEOUT_MS or abort)");
                    break;
                }
            }
        }
    }
    for (auto &c : o.chunks) {  // a failed collective may leave a mirror event unsent
        std::lock_guard<std::mutex> l(ev_mu);
        if (c.mirror_ev) {
            ev_pool.push_back(c.mirror_ev);
            c.mirror_ev = nullptr;
        }
        for (auto e : c.piece_ev) ev_pool.push_back(e);
        c.piece_ev.clear();
    }
    give(stage_pool, o.stage);
    give(mirror_pool, o.mir);
    give(ctl_pool, o.ctl);
    if (rc != KF_OK && o.err.empty()) o.err = t_sess_error;
    o.rc = rc;
    return rc;
}

// The poll loop: every collective in flight advances on whatever message
// arrives next (a chunk's reduce-phase NoFlag message, or its bcast-phase
// WaitRecvBuf one); messages of calls not started here yet wait in the stash.
// one != nullptr: that single (blocking) call, returning its status; nullptr:
// the async worker, which starts every submitted call at once and calls
// done(status, arg) as each completes, until the session stops.
int kf_session::run(SessOp *one)
{
    std::unique_lock<std::mutex> rl(run_mu);
    std::vector<SessOp *> active;
    std::unordered_map<std::string, std::pair<SessOp *, size_t>> index;  // chunk -> op, chunk
    std::vector<pollfd> pfds;
    std::vector<int> pfd_peer;
    for (auto &kv : in_fd) {
        pfds.push_back({kv.second, POLLIN, 0});
        pfd_peer.push_back(kv.first);
    }
    if (wake_fd >= 0) {  // submissions, sends done, host folds done
        pfds.push_back({wake_fd, POLLIN, 0});
        pfd_peer.push_back(-1);
    }
    if (!device_mode && scratch.size() < kChunk + 64) scratch.resize(kChunk + 64);

    // a failure while reading the sockets leaves no message boundary to trust:
    // every collective in flight fails with it (its chunks stop being routed)
    auto mark_broken = [&](int rc, const std::string &why) {
        if (broken_rc != KF_OK) return;
        broken_rc  = rc;
        broken_err = why;
        stash.clear();  // nothing may be replayed into a later call
    };
    auto fail_all = [&](int rc) {
        const std::string why = t_sess_error;
        mark_broken(rc, why);
        for (SessOp *o : active) {
            if (o->rc == KF_OK) {
                o->rc  = rc;
                o->err = why;
            }
            for (auto &c : o->chunks) index.erase(c.name);
            o->remaining = 0;
        }
    };
    // one call fails alone: its chunks stop being routed (later messages for
    // them wait in the stash), the others in flight go on
    auto fail_op = [&](SessOp *o, int rc, const std::string &why) {
        mark_broken(rc, why);
        if (o->rc == KF_OK) {
            o->rc  = rc;
            o->err = why;
        }
        o->remaining = 0;
        for (auto &c : o->chunks) {
            auto f = index.find(c.name);
            if (f != index.end() && f->second.first == o) index.erase(f);
        }
    };
    // the first chunk of o that still waits for a message from `peer`, or -1
    auto awaits = [&](const SessOp &o, int peer) -> int {
        for (size_t i = 0; i < o.chunks.size(); ++i) {
            const auto &c  = o.chunks[i];
            const auto &bp = c.st->bcast.prev[rank];
            if (std::find(c.waiting.begin(), c.waiting.end(), peer) != c.waiting.end() ||
                (!c.bcast_done && std::find(bp.begin(), bp.end(), peer) != bp.end())) {
                return static_cast<int>(i);
            }
        }
        return -1;
    };
    auto peer_gone = [&](SessOp *o, int peer) {
        if (o->remaining == 0 || o->rc != KF_OK) return;
        const int ci = awaits(*o, peer);
        if (ci < 0) return;
        fail_op(o, fail(KF_ERR_IO, "peer " + std::to_string(peer) +
                                       " closed its connection while " + o->chunks[ci].name +
                                       " still waited for its message"),
                t_sess_error);
    };
    auto start = [&](SessOp *o) {
        tr(TR_OP_START, -1, static_cast<int>(o->count), 0);
        t_sess_error.clear();
        if (broken_rc != KF_OK) {
            o->rc        = KF_ERR_IO;
            o->err       = "the session failed earlier (" + broken_err +
                     "); destroy it and create a new one";
            o->remaining = 0;
            active.push_back(o);
            return;
        }
        if (op_timeout_ms > 0) {
            o->deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(op_timeout_ms);
        }
        o->rc = plan(*o);
        if (o->rc != KF_OK) {
            o->err       = t_sess_error;
            o->remaining = 0;
        }
        active.push_back(o);
        if (o->rc != KF_OK) return;
        for (size_t i = 0; i < o->chunks.size(); ++i) index[o->chunks[i].name] = {o, i};
        // messages of this call that arrived before it started
        for (auto it = stash.begin(); it != stash.end();) {
            auto f = index.find(it->name);
            if (f == index.end() || f->second.first != o ||
                !expects(*o, f->second.second, it->flags, it->peer)) {
                ++it;
                continue;
            }
            const int rc = handle(*o, f->second.second, it->flags, it->peer, -1, it->data.data());
            it           = stash.erase(it);
            if (rc != KF_OK) {  // a stashed copy: the sockets are intact
                mark_broken(rc, t_sess_error);
                o->rc        = rc;
                o->err       = t_sess_error;
                o->remaining = 0;
                for (auto &c : o->chunks) index.erase(c.name);
                return;
            }
        }
        // a peer that closed before this call started sends it nothing more
        for (int p : closed) peer_gone(o, p);
    };
    if (one) start(one);

    // host mode: the folds the workers finished, in the order they finished;
    // a chunk's next body goes out once the one before it is folded
    auto retire_folds = [&] {
        std::deque<FoldJob *> done;
        {
            std::lock_guard<std::mutex> l(fmu);
            done.swap(fdone);
        }
        for (FoldJob *j : done) {
            SessOp &o    = *j->o;
            const size_t i = j->i;
            auto &c      = o.chunks[i];
            c.folds.pop_front();  // j: one fold per chunk runs at a time
            --o.folds;
            fbodies.push_back(j->body);
            if (j->rc != KF_OK && o.rc == KF_OK) {
                o.rc  = j->rc;
                o.err = j->err;
            }
            delete j;
            if (o.rc != KF_OK) {  // failed (here or on a socket): its queued bodies go
                while (!c.folds.empty()) {
                    FoldJob *q = c.folds.front();
                    c.folds.pop_front();
                    --o.folds;
                    fbodies.push_back(q->body);
                    delete q;
                }
                if (o.remaining > 0) {
                    o.remaining = 0;
                    for (auto &ch : o.chunks) {
                        auto f = index.find(ch.name);
                        if (f != index.end() && f->second.first == &o) index.erase(f);
                    }
                }
                continue;
            }
            ++c.recv_count;
            if (--c.pending_reduce == 0) {
                finish_reduce(o, i);
                if (c.bcast_done) --o.remaining;
            } else if (!c.folds.empty()) {
                start_fold(o, i);
            }
        }
    };

    // a chunk of a call in flight still waits for a message (not only for its
    // folds: a peer that sent its last chunk may close before they finish)
    auto expecting_message = [&] {
        for (SessOp *o : active) {
            if (o->remaining == 0) continue;
            for (auto &c : o->chunks) {
                if (!c.waiting.empty() || (!c.bcast_done && !c.st->bcast.prev[rank].empty())) {
                    return true;
                }
            }
        }
        return false;
    };

    char hname[512];
    uint32_t flags = 0;
    for (;;) {
        retire_folds();
        if (!one) {  // start what was submitted; a name in flight waits for its call
            std::vector<SessOp *> fresh;
            {
                std::lock_guard<std::mutex> l(amu);
                std::unordered_set<std::string> busy;
                for (SessOp *o : active) busy.insert(o->name);
                for (auto it = aq.begin(); it != aq.end();) {
                    if (busy.count((*it)->name)) {
                        ++it;
                        continue;
                    }
                    busy.insert((*it)->name);
                    fresh.push_back(*it);
                    it = aq.erase(it);
                }
            }
            for (SessOp *o : fresh) start(o);
        }
        // complete the collectives whose chunks are all in and all sent
        bool retired = false;
        for (size_t a = 0; a < active.size();) {
            SessOp *o = active[a];
            bool sent = false;
            {
                std::lock_guard<std::mutex> l(mu);
                sent = o->sends == 0;
                if (sent && o->remaining == 0 && send_rc != KF_OK && o->rc == KF_OK) {
                    o->rc  = send_rc;
                    o->err = "send: " + send_err;
                }
            }
            if (o->remaining > 0 || !sent || o->folds > 0) {
                ++a;
                continue;
            }
            active.erase(active.begin() + a);
            retired = true;
            for (auto &c : o->chunks) {
                auto f = index.find(c.name);
                if (f != index.end() && f->second.first == o) index.erase(f);
            }
            if (active.empty()) {  // a send failure is reported once everything in flight saw it
                std::lock_guard<std::mutex> l(mu);
                send_rc = KF_OK;
                send_err.clear();
            }
            t_sess_error = o->err;
            const int rc = complete(*o);
            tr(TR_OP_DONE, -1, rc, 0);
            if (o == one) {
                if (rc != KF_OK) t_sess_error = o->err;
                return rc;
            }
            {
                std::lock_guard<std::mutex> l(amu);
                if (rc != KF_OK && arc == KF_OK) {
                    arc  = rc;
                    aerr = o->name + ": " + o->err;
                }
            }
            t_sess_error = o->err;
            if (o->done) o->done(rc, o->arg);
            delete o;
            {
                std::lock_guard<std::mutex> l(amu);
                if (--apending == 0) aidle.notify_all();
            }
        }
        if (!one && retired) {  // a call waiting for the name just freed starts now,
            bool queued = false;  // not after the next message: that message may
            {                     // only come once the peer sees this call's chunks
                std::lock_guard<std::mutex> l(amu);
                queued = !aq.empty();
            }
            if (queued) continue;
        }
        if (!one && active.empty()) {  // idle: wait for a submission, or the end;
            rl.unlock();               // blocking calls run their own loop meanwhile
            {
                std::unique_lock<std::mutex> l(amu);
                acv.wait(l, [&] { return astop || !aq.empty(); });
                if (aq.empty()) return KF_OK;
            }
            rl.lock();
            continue;
        }
        bool waiting_rx = false, folding = false;  // anything still to come in?
        for (SessOp *o : active) {
            waiting_rx = waiting_rx || o->remaining > 0;
            folding    = folding || o->folds > 0;
        }
        if (!waiting_rx && !folding && one) {  // only our own sends are left: the sender wakes no one here
            std::unique_lock<std::mutex> l(mu);
            cv_idle.wait(l, [&] { return one->sends == 0; });
            continue;
        }
        // checked before polling: a peer seen closing while an earlier call
        // was in flight is no longer polled, and a call started after that
        // would otherwise wait for a message that cannot come
        size_t open_fds = 0;
        for (size_t q = 0; q < pfds.size(); ++q) open_fds += pfds[q].fd >= 0 && pfd_peer[q] >= 0;
        if (open_fds == 0 && waiting_rx && expecting_message()) {
            fail_all(fail(KF_ERR_IO, "every peer connection closed before the all-reduce finished"));
            continue;
        }
        // KUNGFU_AMD_OP_TIMEOUT_S: a call past its deadline fails; the poll
        // sleeps no longer than the nearest one
        int poll_ms = -1;
        if (op_timeout_ms > 0) {
            const auto now = std::chrono::steady_clock::now();
            bool expired   = false;
            for (SessOp *o : active) {
                if (o->remaining == 0) continue;
                if (o->deadline <= now) {
                    fail_op(o, fail(KF_ERR_TIMEOUT, o->name + ": its messages did not all come within " +
                                                        std::to_string(op_timeout_ms) +
                                                        " ms of its start (KUNGFU_AMD_OP_TIMEOUT_S)"),
                            t_sess_error);
                    expired = true;
                    continue;
                }
                const auto left = std::chrono::duration_cast<std::chrono::milliseconds>(o->deadline - now).count() + 1;
                if (poll_ms < 0 || left < poll_ms) poll_ms = static_cast<int>(left);
            }
            if (expired) continue;
        }
        if (::poll(pfds.data(), pfds.size(), poll_ms) < 0) {
            if (errno == EINTR) continue;
            fail_all(fail(KF_ERR_IO, std::string("poll: ") + strerror(errno)));
            continue;
        }
        int rc  = KF_OK;
        int bad = -1;  // the socket a failure happened on
        for (size_t q = 0; q < pfds.size() && rc == KF_OK; ++q) {
            bad = static_cast<int>(q);
            if (pfds[q].fd < 0 || !(pfds[q].revents & (POLLIN | POLLHUP | POLLERR))) continue;
            const int fd = pfds[q].fd;
            if (pfd_peer[q] < 0) {  // the wake-up counter
                uint64_t v;
                (void)!::read(fd, &v, sizeof(v));
                continue;
            }
            char probe;
            if (::recv(fd, &probe, 1, MSG_PEEK | MSG_DONTWAIT) == 0) {
                // clean EOF at a message boundary: that peer sends us nothing
                // more. A finished peer closes connections we may not need, so
                // only the calls still waiting for one of its messages fail
                // (every one of them, naming the peer; at np >= 3 the other
                // connections stay open and would keep them waiting)
                pfds[q].fd = -1;
                closed.insert(pfd_peer[q]);
                for (SessOp *o : active) peer_gone(o, pfd_peer[q]);
                continue;
            }
            rc = kf_rch_recv_header(fd, hname, sizeof(hname), nullptr, &flags);
            if (rc != KF_OK) {
                t_sess_error = kf_ingest_last_error();
                break;
            }
            const int peer = pfd_peer[q];
            auto it        = index.find(hname);
            if (it != index.end() && expects(*it->second.first, it->second.second, flags, peer)) {
                const int ci = static_cast<int>(it->second.second);
                SessOp *op   = it->second.first;
                tr(TR_RX_HDR, ci, static_cast<int>(flags), 0);
                rc = handle(*op, it->second.second, flags, peer, fd, nullptr);
                tr(TR_RX_DONE, ci, static_cast<int>(flags), 0);
                if (rc == KF_OK && op_timeout_ms > 0) {  // progress: the deadline moves
                    op->deadline = std::chrono::steady_clock::now() +
                                   std::chrono::milliseconds(op_timeout_ms);
                }
                continue;
            }
            // not ours (yet): keep it for the call it belongs to
            Stashed m{peer, hname, flags, {}};
            unsigned char lb[4];
            rc = read_exact(fd, lb, 4);
            if (rc != KF_OK) break;
            const uint32_t len = uint32_t(lb[0]) | (uint32_t(lb[1]) << 8) |
                                 (uint32_t(lb[2]) << 16) | (uint32_t(lb[3]) << 24);
            m.data.resize(len);
            rc = read_exact(fd, m.data.data(), len);
            // a broken session starts no call that could take it: read and drop
            if (rc == KF_OK && broken_rc == KF_OK) stash.push_back(std::move(m));
        }
        if (rc != KF_OK) {
            pfds[bad].fd = -1;  // no message boundary left on it
            fail_all(rc);
        }
    }
}

int kf_session::all_reduce(const char *send, char *recv, size_t count, KungFu_Datatype dt,
                           KungFu_Op op, const std::string &name, void *stream, int kind,
                           const std::vector<Strategy> *slist)
{
    SessOp o;
    o.send   = send;
    o.recv   = recv;
    o.count  = count;
    o.dt     = dt;
    o.op     = op;
    o.name   = name;
    o.stream = stream;
    o.kind   = kind;
    o.L      = slist;
    return run(&o);
}

namespace
{
kf_session_t *create_session(int rank, std::vector<PeerAddr> peers, const char *sock_dir,
                             uint32_t token, int device_mode)
{
    auto *s        = new kf_session;
    s->rank        = rank;
    s->size        = static_cast<int>(peers.size());
    s->peers       = std::move(peers);
    s->dir         = sock_dir;
    s->token       = token;
    s->device_mode = device_mode ? 1 : 0;
    // the reference reads these from the environment kungfu-run sets
    // (env/envs.go:12, env/config.go:73-76, config/config.go:45,61-62)
    if (const char *e = std::getenv("KUNGFU_ALLREDUCE_STRATEGY")) {
        const int st = parse_strategy(e);
        if (st < 0) {
            t_sess_error = std::string("unknown KUNGFU_ALLREDUCE_STRATEGY ") + e;
            delete s;
            return nullptr;
        }
        s->strategy = st;
    }
    if (const char *e = std::getenv("KUNGFU_AMD_BATCH_FOLD")) s->batch_fold = std::atoi(e) != 0;
    if (const char *e = std::getenv("KUNGFU_AMD_SESSION_TRACE")) s->trace_path = e;
    s->stage_pool.cap  = size_t(8) << 30;  // HBM staging for k-input folds
    s->mirror_pool.cap = size_t(2) << 30;  // page-locked mirrors
    if (const char *e = std::getenv("KUNGFU_AMD_STAGE_CAP_MB")) {
        s->stage_pool.cap = static_cast<size_t>(std::max(0L, std::atol(e))) << 20;
    }
    if (const char *e = std::getenv("KUNGFU_AMD_MIRROR_CAP_MB")) {
        s->mirror_pool.cap = static_cast<size_t>(std::max(0L, std::atol(e))) << 20;
    }
    if (const char *e = std::getenv("KUNGFU_CONFIG_STRATEGY_HASH_METHOD")) {
        s->hash_name = std::strcmp(e, "NAME") == 0 || std::strcmp(e, "name") == 0;
    }
    s->sl = strategy_list(s->strategy, s->hosts());
    s->wake_fd = ::eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (s->wake_fd < 0) {
        t_sess_error = std::string("eventfd: ") + strerror(errno);
        delete s;
        return nullptr;
    }
    if (const char *e = std::getenv("KUNGFU_AMD_OP_TIMEOUT_S")) {
        char *end      = nullptr;
        const long sec = std::strtol(e, &end, 10);
        if (end == e || *end != '\0' || sec < 0) {
            t_sess_error = std::string("bad KUNGFU_AMD_OP_TIMEOUT_S ") + e + " (want seconds >= 0)";
            delete s;
            return nullptr;
        }
        s->op_timeout_ms = static_cast<int>(std::min<long long>(sec, 86400LL * 24) * 1000LL);
    }
    if (const char *e = std::getenv("KUNGFU_AMD_TEST_LAUNCH_RACE")) s->race.on = std::atoi(e) != 0;
    if (s->device_mode) {
        (void)hipGetDevice(&s->device);
        // the streamed kernels' words and code, on this thread, before the
        // sender / async / fold threads exist (profiles/r05/failures.md)
        s->board  = kf_stream::board_create();
        s->ingest = kf_ingest_create(kChunk + 4096, 8);
        int nslot = 4;
        if (const char *e = std::getenv("KUNGFU_AMD_TX_SLOTS")) nslot = std::max(1, std::atoi(e));
        if (const char *e = std::getenv("KUNGFU_AMD_ROOT_MIRROR")) s->mirror = std::atoi(e) != 0;
        if (const char *e = std::getenv("KUNGFU_AMD_TX_AHEAD")) {
            s->tx_ahead = static_cast<size_t>(std::max(1, std::atoi(e)));
        }
        if (const char *e = std::getenv("KUNGFU_AMD_PIECE_KB")) {
            s->piece = static_cast<uint32_t>(std::max(0, std::atoi(e))) << 10;
        }
        s->stream_mode = kf_session::kStreamFold;  // the measured-best default
        if (const char *e = std::getenv("KUNGFU_AMD_STREAM")) {  // "0", "1" (all), or a list
            const std::string v = e;
            s->stream_mode      = v == "1" ? 7 : 0;
            if (v.find("out") != std::string::npos) s->stream_mode |= kf_session::kStreamOut;
            if (v.find("fold") != std::string::npos) s->stream_mode |= kf_session::kStreamFold;
            if (v.find("in") != std::string::npos) s->stream_mode |= kf_session::kStreamIn;
            if (v.find("last") != std::string::npos) s->stream_mode |= kf_session::kStreamInLast;
            if (v.find("idle") != std::string::npos) s->stream_mode |= kf_session::kStreamOutIdle;
        }
        if (const char *e = std::getenv("KUNGFU_AMD_STREAM_PIECE_KB")) {
            const uint32_t kb = static_cast<uint32_t>(std::max(4, std::atoi(e)));
            s->stream_piece   = (kb << 10) & ~(kf_stream::kBlockBytes - 1);
        }
        if (const char *e = std::getenv("KUNGFU_AMD_STREAM_TIMEOUT_MS")) {
            s->stream_deadline_ms = std::max(1, std::atoi(e));
        }
        s->ctl_pool.cap       = size_t(64) << 20;
        s->ctl_pool.coherent  = true;

        s->piece &= ~0xFFFu;  // whole 4 KiB: every dtype's elements, aligned pieces
        bool tx_ok = true;
        for (int i = 0; i < nslot && tx_ok; ++i) {
            void *p      = nullptr;
            hipEvent_t e = nullptr;
            tx_ok = hipHostMalloc(&p, kChunk + 4096, hipHostMallocDefault) == hipSuccess;
            void *dv = nullptr;
            tx_ok    = tx_ok && hipHostGetDevicePointer(&dv, p, 0) == hipSuccess;
            if (tx_ok) {
                s->tx.push_back(p);
                s->tx_dev.push_back(dv);
            }
            tx_ok = tx_ok && hipEventCreateWithFlags(&e, kf_sync::event_flags()) == hipSuccess;
            if (tx_ok) s->tx_done.push_back(e);
        }
        if (hipStreamCreateWithFlags(&s->tx_stream, hipStreamNonBlocking) != hipSuccess) {
            s->tx_stream = nullptr;
        }
        if (hipStreamCreateWithFlags(&s->wait_stream, hipStreamNonBlocking) != hipSuccess) {
            s->wait_stream = nullptr;
        }
        const char *ms = std::getenv("KUNGFU_AMD_MIRROR_SIDE");  // 0: A/B, caller's stream
        if ((!ms || std::atoi(ms) != 0) &&
            hipStreamCreateWithFlags(&s->mir_stream, hipStreamNonBlocking) != hipSuccess) {
            s->mir_stream = nullptr;  // the copies stay on the caller's stream
        }
        if ((s->stream_mode & (kf_session::kStreamOut | kf_session::kStreamOutIdle)) && tx_ok) {
            // a control block per tx slot
            void *cp = nullptr, *cd = nullptr;
            tx_ok = hipHostMalloc(&cp, s->tx.size() * sizeof(kf_stream::Ctl),
                                  hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
                    hipHostGetDevicePointer(&cd, cp, 0) == hipSuccess;
            for (size_t k = 0; tx_ok && k < s->tx.size(); ++k) {
                s->tx_ctl.push_back(static_cast<kf_stream::Ctl *>(cp) + k);
                s->tx_ctl_dev.push_back(static_cast<kf_stream::Ctl *>(cd) + k);
            }
        }
        if (s->piece) {
            s->max_pieces = (kChunk + 4096 + s->piece - 1) / s->piece;
            for (size_t k = 0; k < s->tx.size() * s->max_pieces && tx_ok; ++k) {
                hipEvent_t e = nullptr;
                tx_ok = hipEventCreateWithFlags(&e, kf_sync::event_flags()) == hipSuccess;
                if (tx_ok) s->tx_piece_ev.push_back(e);
            }
        }
        s->counted = true;
        g_device_sessions.fetch_add(1, std::memory_order_relaxed);
        if (!s->ingest || !tx_ok || !s->tx_stream || !s->board || !s->wait_stream) {
            t_sess_error = !s->board ? "streamed kernels' device words (hipMalloc) failed"
                                     : "kf_ingest_create failed";
            delete s;
            return nullptr;
        }
    }
    if (s->size > 1 && s->connect_all() != KF_OK) {
        delete s;
        return nullptr;
    }
    if (s->op_timeout_ms > 0) {  // a peer that stalls mid-message fails the read / write
        timeval tv{};
        tv.tv_sec  = s->op_timeout_ms / 1000;
        tv.tv_usec = (s->op_timeout_ms % 1000) * 1000;
        for (auto &kv : s->in_fd) (void)::setsockopt(kv.second, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
        for (auto &kv : s->out_fd) (void)::setsockopt(kv.second, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
    }
    s->sender = std::thread([s] {
        if (s->device_mode) (void)hipSetDevice(s->device);  // its copy-out kernels
        s->sender_loop();
    });
    return s;
}
}  // namespace

extern "C" {

kf_session_t *kf_session_create(int rank, int size, const char *sock_dir, uint32_t token,
                                int device_mode)
{
    if (size < 1 || rank < 0 || rank >= size || !sock_dir) {
        t_sess_error = "bad rank/size/dir";
        return nullptr;
    }
    // one host: 127.0.0.1, ports 10000 + rank (hostspec.go:121-124)
    std::vector<PeerAddr> peers;
    for (int r = 0; r < size; ++r) peers.push_back({kIPv4, static_cast<uint16_t>(kPortBase + r)});
    return create_session(rank, std::move(peers), sock_dir, token, device_mode);
}

kf_session_t *kf_session_create_peers(const char *peer_list, const char *self_spec,
                                      const char *sock_dir, uint32_t token, int device_mode)
{
    std::vector<PeerAddr> peers;
    PeerAddr self;
    if (!peer_list || !self_spec || !sock_dir || !parse_peer_list(peer_list, &peers) ||
        !parse_peer(self_spec, &self)) {
        t_sess_error = "bad peer list / self spec (want ipv4:port[,ipv4:port...])";
        return nullptr;
    }
    int rank = -1;
    for (size_t r = 0; r < peers.size(); ++r) {
        for (size_t q = 0; q < r; ++q) {
            if (peers[q] == peers[r]) {
                t_sess_error = "duplicate peer in the list";
                return nullptr;
            }
        }
        if (peers[r] == self) rank = static_cast<int>(r);
    }
    if (rank < 0) {  // peer.go: self must be in the initial cluster
        t_sess_error = std::string("self ") + self_spec + " not in the peer list";
        return nullptr;
    }
    return create_session(rank, std::move(peers), sock_dir, token, device_mode);
}

int kf_session_set_strategy(kf_session_t *s, int strategy, int hash_by_name)
{
    if (!s || strategy < KungFu_Tree || strategy > KungFu_AUTO) return KF_ERR_ARG;
    s->strategy  = strategy;
    s->hash_name = hash_by_name ? 1 : 0;
    s->sl        = strategy_list(strategy, s->hosts());
    return KF_OK;
}

int kf_session_set_host_reduce(kf_session_t *s, kf_host_reduce_fn fn)
{
    if (!s) return KF_ERR_ARG;
    s->host_fn = fn;
    return KF_OK;
}

int kf_session_all_reduce(kf_session_t *s, const void *send, void *recv, size_t count,
                          KungFu_Datatype dt, KungFu_Op op, const char *name, void *stream)
{
    if (!s || !name || (count > 0 && (!send || !recv))) return KF_ERR_ARG;
    if (dt == KungFu_BOOL || (dt == KungFu_FLOAT16 && op != KungFu_SUM)) return KF_ERR_OP;
    t_sess_error.clear();
    if (s->aworker.joinable() && std::this_thread::get_id() == s->aworker.get_id()) {
        // from a done callback: waiting for the queue would wait for itself
        return fail(KF_ERR_ARG, "synchronous all-reduce from a done callback");
    }
    // after every all-reduce submitted before it (one message order per peer)
    const int rc = s->wait_all();
    if (rc != KF_OK) return rc;
    return s->all_reduce(static_cast<const char *>(send), static_cast<char *>(recv), count, dt,
                         op, name, stream);
}

static int blocking_collective(kf_session_t *s, const void *send, void *recv, size_t count,
                               KungFu_Datatype dt, KungFu_Op op, const char *name, void *stream,
                               int kind)
{
    if (!s || !name || (count > 0 && (!send || !recv))) return KF_ERR_ARG;
    if (dt == KungFu_BOOL || (dt == KungFu_FLOAT16 && op != KungFu_SUM)) return KF_ERR_OP;
    t_sess_error.clear();
    if (s->aworker.joinable() && std::this_thread::get_id() == s->aworker.get_id()) {
        return fail(KF_ERR_ARG, "blocking collective from a done callback");
    }
    const int rc = s->wait_all();
    if (rc != KF_OK) return rc;
    return s->all_reduce(static_cast<const char *>(send), static_cast<char *>(recv), count, dt,
                         op, name, stream, kind);
}

int kf_session_subset_all_reduce(kf_session_t *s, const void *send, void *recv, size_t count,
                                 KungFu_Datatype dt, KungFu_Op op, const int32_t *forest,
                                 const char *name, void *stream)
{
    if (!s || !forest || !name || (count > 0 && (!send || !recv))) return KF_ERR_ARG;
    if (dt == KungFu_BOOL || (dt == KungFu_FLOAT16 && op != KungFu_SUM)) return KF_ERR_OP;
    t_sess_error.clear();
    Graph bg(s->size);  // FromForestArray (graph.go:46-62)
    for (int i = 0; i < s->size; ++i) {
        if (forest[i] < 0 || forest[i] >= s->size) return fail(KF_ERR_ARG, "forest out of range");
        if (forest[i] != i) bg.edge(forest[i], i);
    }
    for (int i = 0; i < s->size; ++i) {  // the reference leaves cycles unchecked (FIXME
        int hops = 0;                    // graph.go:60); here they are an error
        for (int j = i; forest[j] != j; j = forest[j]) {
            if (++hops > s->size) return fail(KF_ERR_ARG, "forest has a cycle");
        }
    }
    if (s->aworker.joinable() && std::this_thread::get_id() == s->aworker.get_id()) {
        return fail(KF_ERR_ARG, "blocking collective from a done callback");
    }
    const int rc = s->wait_all();
    if (rc != KF_OK) return rc;
    const std::vector<Strategy> one{simple(bg)};
    return s->all_reduce(static_cast<const char *>(send), static_cast<char *>(recv), count, dt,
                         op, name, stream, kAllReduce, &one);
}

int kf_session_reduce(kf_session_t *s, const void *send, void *recv, size_t count,
                      KungFu_Datatype dt, KungFu_Op op, const char *name, void *stream)
{
    return blocking_collective(s, send, recv, count, dt, op, name, stream, kReduce);
}

int kf_session_broadcast(kf_session_t *s, const void *send, void *recv, size_t count,
                         KungFu_Datatype dt, const char *name, void *stream)
{
    // no fold: any dtype the wire can carry (BOOL included, as the reference)
    if (!s || !name || (count > 0 && (!send || !recv))) return KF_ERR_ARG;
    t_sess_error.clear();
    if (s->aworker.joinable() && std::this_thread::get_id() == s->aworker.get_id()) {
        return fail(KF_ERR_ARG, "blocking collective from a done callback");
    }
    const int rc = s->wait_all();
    if (rc != KF_OK) return rc;
    return s->all_reduce(static_cast<const char *>(send), static_cast<char *>(recv), count, dt,
                         KungFu_SUM, name, stream, kBroadcast);
}

int kf_session_all_reduce_async(kf_session_t *s, const void *send, void *recv, size_t count,
                                KungFu_Datatype dt, KungFu_Op op, const char *name, void *stream,
                                kf_done_fn done, void *arg)
{
    if (!s || !name || (count > 0 && (!send || !recv))) return KF_ERR_ARG;
    if (dt == KungFu_BOOL || (dt == KungFu_FLOAT16 && op != KungFu_SUM)) return KF_ERR_OP;
    switch (dt) {  // checked here: kungfu_type_size exits on an unknown code
    case KungFu_UINT8: case KungFu_UINT16: case KungFu_UINT32: case KungFu_UINT64:
    case KungFu_INT8: case KungFu_INT16: case KungFu_INT32: case KungFu_INT64:
    case KungFu_FLOAT16: case KungFu_FLOAT: case KungFu_DOUBLE: case KungFu_BFLOAT16: break;
    default: return KF_ERR_DTYPE;
    }
    if (static_cast<unsigned>(op) > KungFu_PROD) return KF_ERR_OP;
    auto *o   = new SessOp;
    o->send   = static_cast<const char *>(send);
    o->recv   = static_cast<char *>(recv);
    o->count  = count;
    o->dt     = dt;
    o->op     = op;
    o->name   = name;
    o->stream = stream;
    o->done   = done;
    o->arg    = arg;
    const int rc = s->submit(o);
    if (rc != KF_OK) delete o;
    return rc;
}

int kf_session_barrier(kf_session_t *s)
{
    // session.go:104-115: an all-reduce (SUM) of size() zero bytes named
    // "kungfu::barrier" over the global strategies. A device-mode session
    // moves HBM buffers only, so it keeps a zeroed workspace there.
    if (!s) return KF_ERR_ARG;
    t_sess_error.clear();
    if (s->aworker.joinable() && std::this_thread::get_id() == s->aworker.get_id()) {
        return fail(KF_ERR_ARG, "barrier from a done callback");
    }
    const int rc = s->wait_all();
    if (rc != KF_OK) return rc;
    const size_t k = static_cast<size_t>(s->size);
    if (!s->device_mode) {
        std::vector<char> send(k, 0), recv(k, 0);
        return s->all_reduce(send.data(), recv.data(), k, KungFu_UINT8, KungFu_SUM,
                             "kungfu::barrier", nullptr);
    }
    if (!s->barrier_dev) {
        if (hipMalloc(&s->barrier_dev, 2 * k) != hipSuccess) {
            s->barrier_dev = nullptr;
            return fail(KF_ERR_HIP, "hipMalloc barrier workspace");
        }
    }
    // zeroed before every barrier: the sum lands in the second half, the first
    // half is never written, but a failed barrier may leave the second dirty
    if (hipMemset(s->barrier_dev, 0, 2 * k) != hipSuccess) {
        return fail(KF_ERR_HIP, "hipMemset barrier workspace");
    }
    return s->all_reduce(s->barrier_dev, s->barrier_dev + k, k, KungFu_UINT8, KungFu_SUM,
                         "kungfu::barrier", nullptr);
}

int kf_session_wait_all(kf_session_t *s)
{
    if (!s) return KF_ERR_ARG;
    if (s->aworker.joinable() && std::this_thread::get_id() == s->aworker.get_id()) {
        return fail(KF_ERR_ARG, "kf_session_wait_all from a done callback");
    }
    return s->wait_all();
}

int kf_session_info(kf_session_t *s, int *rank, int *size, int *local_rank, int *local_size,
                    int *host_count)
{
    if (!s) return KF_ERR_ARG;
    int lr = 0, ls = 0;
    std::vector<uint32_t> ips;
    for (int r = 0; r < s->size; ++r) {
        const uint32_t ip = s->peers[r].ip;
        if (std::find(ips.begin(), ips.end(), ip) == ips.end()) ips.push_back(ip);
        if (ip == s->peers[s->rank].ip) {
            if (r < s->rank) ++lr;
            ++ls;
        }
    }
    if (rank) *rank = s->rank;
    if (size) *size = s->size;
    if (local_rank) *local_rank = lr;
    if (local_size) *local_size = ls;
    if (host_count) *host_count = static_cast<int>(ips.size());
    return KF_OK;
}

void kf_session_destroy(kf_session_t *s) { delete s; }

const char *kf_session_last_error(void) { return t_sess_error.c_str(); }

}  // extern "C"

// library-internal (hidden): whether a session moves device or host buffers
// (kf_exchange.hip broadcasts the RCCL id through it)
int kf_session_device_mode_internal(const kf_session_t *s) { return s ? s->device_mode : -1; }

// library-internal: the host index of every rank (distinct IPv4 addresses in
// order of first appearance, the reference's host list, plan/peerlist.go)
int kf_session_hosts_internal(const kf_session_t *s, int *host_of)
{
    if (!s || !host_of) return KF_ERR_ARG;
    std::vector<uint32_t> ips;
    for (int r = 0; r < s->size; ++r) {
        const uint32_t ip = s->peers[r].ip;
        auto it           = std::find(ips.begin(), ips.end(), ip);
        host_of[r]        = static_cast<int>(it - ips.begin());
        if (it == ips.end()) ips.push_back(ip);
    }
    return KF_OK;
}
