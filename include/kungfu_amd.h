/*
 * kungfu_amd.h — C-ABI of the MI355X gradient-bucket reduce.
 *
 * Two layers live behind this header (libkungfu_amd.so, built from
 * kungfu_amd/csrc/ for gfx950):
 *
 *  B1  drop-in element kernel. Link-compatible with KungFu's base package:
 *        std_transform_2   replaces /root/reference/srcs/go/kungfu/base/op.cpp:57-93
 *                          (declared in srcs/cpp/include/kungfu/op.h:17-19)
 *        kungfu_type_size  replaces srcs/go/kungfu/base/dtype.c:7-35
 *                          (declared in srcs/cpp/include/kungfu/dtype.h:46)
 *        float16_sum       replaces srcs/go/kungfu/base/f16.c:25-50
 *                          (declared in srcs/go/kungfu/base/f16.h:7)
 *      These take HOST pointers, run the reduce on the GPU (pageable host
 *      memory -> HBM -> HIP kernel -> host) and return only when the output
 *      is written, as cgo requires (srcs/go/kungfu/base/op.go:27-35). Bad
 *      dtype/op -> exit(1), exactly like op.cpp:41,52,89 and dtype.c:31-33.
 *
 *  B2  bucket-level device API (the real fast path). Device
 *      pointers, a hipStream_t passed as void*, no allocation, no host sync,
 *      error codes instead of exit(). Safe to capture into a hipGraph.
 *
 * Enum values are bit-identical to the reference ABI:
 *      KungFu_Datatype  srcs/cpp/include/kungfu/dtype.h:21-39  ((cat<<16)|(bytes<<8)|8)
 *      KungFu_Op        srcs/cpp/include/kungfu/op.h:8-13
 * KungFu_BFLOAT16 is an extension (category 2, 2 bytes, bits-per-byte field 9
 * so it cannot collide with FLOAT16); the reference has no bf16 type and maps
 * TF bf16 onto FLOAT16 (srcs/cpp/include/kungfu/tensorflow/ops.h:21-22).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The library is built with -fvisibility=hidden: exactly what this header
 * declares is exported. */
#pragma GCC visibility push(default)

/* ---- reference-compatible enums ---------------------------------------- */

enum KungFu_Datatype {
    KungFu_UINT8   = 0x00108,
    KungFu_UINT16  = 0x00208,
    KungFu_UINT32  = 0x00408,
    KungFu_UINT64  = 0x00808,
    KungFu_INT8    = 0x10108,
    KungFu_INT16   = 0x10208,
    KungFu_INT32   = 0x10408,
    KungFu_INT64   = 0x10808,
    KungFu_FLOAT16 = 0x20208,
    KungFu_FLOAT   = 0x20408,
    KungFu_DOUBLE  = 0x20808,
    KungFu_BOOL    = 0x30108,
    /* extension, not in the reference */
    KungFu_BFLOAT16 = 0x20209,
};
typedef enum KungFu_Datatype KungFu_Datatype;

enum KungFu_Op {
    KungFu_SUM  = 0,
    KungFu_MIN  = 1,
    KungFu_MAX  = 2,
    KungFu_PROD = 3,
};
typedef enum KungFu_Op KungFu_Op;

/* srcs/cpp/include/kungfu/strategy.h:7-17 */
enum KungFu_Strategy {
    KungFu_Tree                = 0,
    KungFu_BinaryTree          = 1,
    KungFu_Ring                = 2,
    KungFu_Star                = 3,
    KungFu_MultiStar           = 4,
    KungFu_Clique              = 5,
    KungFu_BinaryTreeStar      = 6,
    KungFu_MultiBinaryTreeStar = 7,
    KungFu_AUTO                = 8,
};
typedef enum KungFu_Strategy KungFu_Strategy;

/* ---- B1: drop-in host-pointer entry points ------------------------------ */

/* out[i] = o(input1[i], input2[i]) for i < n. out may alias input1 or input2
 * exactly. Replaces srcs/go/kungfu/base/op.cpp:57-93. */
void std_transform_2(const void *input1, const void *input2, void *output,
                     const int n, const KungFu_Datatype dt, const KungFu_Op o);

/* sizeof one element; unknown dtype -> message + exit(1).
 * Replaces srcs/go/kungfu/base/dtype.c:7-35. */
uint32_t kungfu_type_size(KungFu_Datatype dt);

/* z[i] = fp16(fp32(x[i]) + fp32(y[i])), round-to-nearest-even.
 * Replaces srcs/go/kungfu/base/f16.c:25-50. */
void float16_sum(void *z, const void *x, const void *y, int len);

/* ---- B2: bucket-level device API ---------------------------------------- */

enum KF_Status {
    KF_OK              = 0,
    KF_ERR_DTYPE       = 1, /* unsupported dtype                      */
    KF_ERR_OP          = 2, /* unsupported op for this dtype          */
    KF_ERR_ARG         = 3, /* null pointer with n>0, k out of range  */
    KF_ERR_HIP         = 4, /* a HIP runtime call failed              */
    KF_ERR_NO_DEVICE   = 5, /* no usable gfx950 device                */
    KF_ERR_IO          = 6, /* socket read/write failed               */
    KF_ERR_PROTO       = 7, /* rchannel framing/length/token mismatch  */
    KF_ERR_TIMEOUT     = 8, /* a device-side peer barrier gave up      */
    KF_ERR_RCCL        = 9, /* librccl missing or an RCCL call failed  */
};

/* Largest k accepted by kf_bucket_reduce*. */
#define KF_MAX_INPUTS 16

/* out[i] = (((in[0][i] o in[1][i]) o in[2][i]) ... o in[k-1][i])
 * Left fold in the given order: pass the peers in the reference's arrival or
 * ring order to reproduce its accumulation order bit for bit
 * (session.go:255-264 applies Transform2(recv, acc, peer) per hop).
 * fp16 rounds to fp16 after every hop, as the reference chain does; bf16
 * accumulates in fp32 and rounds once (build-defined, parity unpinned).
 * k == 1 is a copy. out may alias any input exactly. */
int kf_bucket_reduce(const void *const *inputs, int k, void *out, size_t n,
                     KungFu_Datatype dt, KungFu_Op op, void *stream);

/* S-SGD epilogue fused into the reduce: out[i] = fold_SUM(in[*][i]) / np,
 * a true IEEE division (TF's g / np, sync_sgd.py:103-104), so it is bit-exact
 * against "reduce, then divide" for every np. float types only. */
int kf_bucket_reduce_avg(const void *const *inputs, int k, void *out, size_t n,
                         KungFu_Datatype dt, int np, void *stream);

/* In-place scale of an already-summed shard: x[i] = x[i] / np (the step
 * between RCCL reduce-scatter and all-gather). float types only. */
int kf_bucket_div(void *x, size_t n, KungFu_Datatype dt, int np, void *stream);

/* Many independent buckets in one launch per 16 of them: bucket b is
 *   outs[b][i] = fold(inputs[b*k + 0][i], ..., inputs[b*k + k-1][i]), i < counts[b]
 * with the same arithmetic as kf_bucket_reduce (np == 0) or
 * kf_bucket_reduce_avg (np > 0: SUM then / np, float types). A bucket whose
 * pointers do not share one 16-B residue, and MIN / MAX / PROD, get a launch
 * each; k == 1 with np == 0 is a copy per bucket. For the per-bucket steps of
 * an exchange (every shard's /np, every bucket's fold of the received shards),
 * where one launch per 4 MiB bucket costs more than the bucket's HBM time. */
int kf_bucket_reduce_batch(const void *const *inputs, int k, void *const *outs,
                           const size_t *counts, int nb, KungFu_Datatype dt, KungFu_Op op,
                           int np, void *stream);

/* SMA epilogue (sma_sgd.py:60-65):
 *   v[i] = fl(fl(c1 * v[i]) + fl(c2 * fl(sum[i] / np)))
 * with c1 = (float)(1 - alpha), c2 = (float)alpha computed in double first,
 * as TF converts the Python constants. No FMA contraction. float types only. */
int kf_sma_blend(void *v, const void *sum, size_t n, KungFu_Datatype dt,
                 int np, double alpha, void *stream);
/* kf_sma_blend over nb buckets (vs[b] blended with sums[b], counts[b]
 * elements each, the same dtype, np and alpha) in one launch per 16 buckets;
 * the same bits as nb kf_sma_blend calls. */
int kf_sma_blend_batch(void *const *vs, const void *const *sums, const size_t *counts, int nb,
                       KungFu_Datatype dt, int np, double alpha, void *stream);

/* ---- runtime / diagnostics ---------------------------------------------- */

/* HIP device count visible to the library (0 on a GPU-less host). */
int kf_device_count(void);

/* Library/ABI version string. */
const char *kf_version(void);

/* Last HIP error string recorded by the library on this thread. */
const char *kf_last_error(void);

/* Release the library's process-wide HIP resources (the streams and HBM
 * scratch std_transform_2 / kf_transform2_host lend to their calls) while the
 * HIP runtime is still up. No destructor in the library calls HIP at process
 * exit, so a host that never calls this leaves those to the OS. Call it once
 * no host-API call is running (KF_ERR_ARG otherwise: the busy ones are kept);
 * the library stays usable afterwards. The Python binding calls it at
 * interpreter exit. */
int kf_shutdown(void);

/* kf_bucket_reduce / kf_bucket_reduce_avg for inputs that sit behind
 * different links (kungfu_amd/p2p.py: shard `rank` of every peer's bucket,
 * mapped over xGMI): every thread has the loads of up to 8 inputs in flight
 * before the first add, so all links carry traffic at once; the fold order is
 * still inputs[0], inputs[1], ... (bit-identical result). np > 0: SUM then
 * / np (float dtypes); np == 0: the plain op. Same contract as B2. */
int kf_bucket_reduce_peers(const void *const *inputs, int k, void *out, size_t n,
                           KungFu_Datatype dt, KungFu_Op op, int np, void *stream);

/* Page-lock / release a host range so std_transform_2 and
 * kf_transform2_host can DMA it directly (e.g. a receive-buffer pool the
 * transport reuses, srcs/go/rchannel/connection/byte_slice_pool.go:28-60).
 * The library remembers the range (a chunk inside it needs no pointer
 * queries); release it with kf_host_unregister(p), p the registered base. */
int kf_host_register(void *p, size_t bytes);
int kf_host_unregister(void *p);

/* Tuning hook (tools/tune_reduce.py only): launch geometry of the fp32 SUM
 * 2-input path — unroll in {1,2,4,8} vectors per thread, grid cap in blocks,
 * non-temporal loads, plain stores. Not thread-safe; call before launching. */
int kf_set_geometry(int unroll, int grid_cap, int loadnt, int stplain);
/* Tuning hook (A/B tools only): occupancy cap of the HBM streaming kernels
 * (kf_bucket_reduce*, kf_bucket_div, kf_sma_blend; not the batched launch), as
 * dynamic LDS bytes per 256-thread block (0 = none, at most 64 KiB) for the
 * k <= 2 kernels (two-input sum, /np, SMA) and for the k >= 3 folds.
 * Defaults: 0 and 32 KiB (five blocks per CU); the fold's cap applies to
 * launches of at least 8192 blocks (128 MiB per fp32 input). Not thread-safe. */
int kf_set_occupancy(int lds_small, int lds_fold);

/* Host-pointer reduce with a status code instead of exit(): the path
 * std_transform_2 takes. Synchronous, a stream and device scratch lent to the
 * call from a process-wide pool (kf_shutdown frees them).
 * If x, y and out are all device-accessible (page-locked by hipHostMalloc or
 * kf_host_register, or HBM of the current device) the kernel reads and writes
 * them in place (zero copy, over PCIe for host memory); otherwise pageable
 * copies through the runtime's staging to HBM scratch and back. Used by the
 * copy-inclusive measurement (bench.py host_staged). */
int kf_transform2_host(const void *x, const void *y, void *out, size_t n,
                       KungFu_Datatype dt, KungFu_Op op);

/* ---- host ingestion: rchannel wire format + device recvOnto ----------- */

/* rchannel constants (srcs/go/rchannel/connection/message.go:10-17, 71-78) */
#define KF_RCH_CONN_COLLECTIVE 2
#define KF_RCH_NO_FLAG 0u
#define KF_RCH_WAIT_RECV_BUF 1u

/* Connection handshake: client sends {u16 type, u16 src_port, u32 src_ipv4},
 * server answers {u32 token}; a token mismatch on a collective connection is
 * an error (srcs/go/rchannel/connection/connection.go:28-101). */
int kf_rch_client_handshake(int fd, uint16_t conn_type, uint16_t src_port,
                            uint32_t src_ipv4, uint32_t expect_token);
int kf_rch_server_handshake(int fd, uint32_t token, uint16_t *conn_type,
                            uint16_t *src_port, uint32_t *src_ipv4);

/* One named message: {u32 name_len, name, u32 flags} {u32 len, payload}
 * (message.go:90-198; tcpConnection.Send, connection.go:149-165). */
int kf_rch_send(int fd, const char *name, uint32_t flags, const void *data,
                uint32_t len);
/* Reads a message header; name is NUL-terminated into name[cap]. */
int kf_rch_recv_header(int fd, char *name, uint32_t cap, uint32_t *name_len,
                       uint32_t *flags);
/* Reads a message body into dst; its length must equal expect_len
 * (Message.ReadInto, message.go:184-198). */
int kf_rch_recv_body(int fd, void *dst, uint32_t expect_len);

/* Page-locked landing slots + device slots for peer chunks. */
#pragma GCC visibility pop
typedef struct kf_ingest kf_ingest_t; /* opaque; its C++ body stays hidden */
#pragma GCC visibility push(default)
kf_ingest_t *kf_ingest_create(size_t slot_bytes, int nslots);
void kf_ingest_destroy(kf_ingest_t *g);

/* recvOnto on the device (session.go:255-264): read the body of the message
 * whose header was just read (len bytes) from fd into the next page-locked
 * slot, then on `stream`: copy it to HBM and fold dev_acc = own o peer, with
 * own = dev_own (SendBuf before the first receive) or dev_acc if NULL.
 * Returns after the socket read; the device work stays queued on `stream`. */
int kf_ingest_recv_onto(kf_ingest_t *g, int fd, uint32_t len, void *dev_acc,
                        const void *dev_own, size_t count, KungFu_Datatype dt,
                        KungFu_Op op, void *stream);
/* recvInto on the device (session.go:266-270): read the body into the next
 * page-locked slot and queue its copy into dev_dst on `stream`. */
int kf_ingest_recv_into(kf_ingest_t *g, int fd, uint32_t len, void *dev_dst,
                        void *stream);
/* The same two steps with the body read in pieces of piece_bytes (a multiple
 * of the element size): each piece's fold (or copy) is queued on `stream` as
 * soon as that piece has been read, so the device work of a chunk overlaps
 * the rest of its socket read. piece_events (hipEvent_t handles, may be NULL;
 * at least ceil(len / piece_bytes) of them) gets event k recorded after piece
 * k's fold. Element-wise, so the bits equal the whole-chunk call's. */
int kf_ingest_recv_onto_pieces(kf_ingest_t *g, int fd, uint32_t len, void *dev_acc,
                               const void *dev_own, size_t count, KungFu_Datatype dt,
                               KungFu_Op op, void *stream, uint32_t piece_bytes,
                               void *const *piece_events, int n_events);
int kf_ingest_recv_into_pieces(kf_ingest_t *g, int fd, uint32_t len, void *dev_dst,
                               void *stream, uint32_t piece_bytes);
/* sendOnto/sendInto from the device: copy bytes of dev_src (after the work
 * queued on `stream`) to a page-locked slot and send it as one message. */
int kf_ingest_send_from_device(kf_ingest_t *g, int fd, const char *name,
                               uint32_t flags, const void *dev_src, size_t bytes,
                               void *stream);
/* The same two steps for a chunk already in host memory (a message read
 * ahead of its all-reduce and kept, as the reference's per-name mailbox
 * does, handler/collective.go:27-41). */
int kf_ingest_fold_host(kf_ingest_t *g, const void *host, uint32_t len,
                        void *dev_acc, const void *dev_own, size_t count,
                        KungFu_Datatype dt, KungFu_Op op, void *stream);
int kf_ingest_copy_host(kf_ingest_t *g, const void *host, uint32_t len,
                        void *dev_dst, void *stream);
/* Wait for every queued slot copy. */
int kf_ingest_sync(kf_ingest_t *g);
const char *kf_ingest_last_error(void);

/* ---- session engine (collective boundary) ---------------- */

/* Host-mode fold callback: out = x op y over n elements; 0 = ok. */
typedef int (*kf_host_reduce_fn)(const void *x, const void *y, void *out,
                                 int64_t n, int dt, int op);

#pragma GCC visibility pop
typedef struct kf_session kf_session_t; /* opaque; its C++ body stays hidden */
#pragma GCC visibility push(default)

/* Peer `rank` of `size` on this host: listens on
 * <sock_dir>/kungfu-amd-127.0.0.1-<10000+rank>.sock and connects to every other peer
 * (rchannel handshake with `token`). The strategy and chunk hash come from
 * KUNGFU_ALLREDUCE_STRATEGY / KUNGFU_CONFIG_STRATEGY_HASH_METHOD as in the
 * reference (default BINARY_TREE_STAR, NAME). device_mode = 1: buffers passed
 * to kf_session_all_reduce are HBM pointers; 0: host pointers. NULL on
 * failure (kf_session_last_error). */
kf_session_t *kf_session_create(int rank, int size, const char *sock_dir,
                                uint32_t token, int device_mode);
/* Peer `self_spec` of the cluster `peer_list`, in the formats kungfu-run
 * exports as KUNGFU_SELF_SPEC / KUNGFU_INIT_PEERS ("ipv4:port" and a
 * comma-separated list of them, plan/id.go:34-50, plan/peerlist.go:180-192);
 * the rank is self's index in the list. Peers with the same IPv4 connect over
 * <sock_dir>/kungfu-amd-<ipv4>-<port>.sock, the others over TCP to ipv4:port
 * (rchannel/connection/connection.go:58-64); every peer listens on its own
 * address. Multi-host strategies (TREE, BINARY_TREE_STAR, MULTI_*, AUTO ->
 * BINARY_TREE_STAR) follow the hosts (plan/topology.go:5-136). */
kf_session_t *kf_session_create_peers(const char *peer_list, const char *self_spec,
                                      const char *sock_dir, uint32_t token,
                                      int device_mode);
/* Override the strategy (KungFu_Strategy) and chunk hash (1 = NAME,
 * 0 = SIMPLE); every peer must use the same. */
int kf_session_set_strategy(kf_session_t *s, int strategy, int hash_by_name);
/* Host mode only: fold with `fn` instead of std_transform_2. */
int kf_session_set_host_reduce(kf_session_t *s, kf_host_reduce_fn fn);
/* Synchronous all-reduce of one bucket: the counterpart of
 * GoKungfuAllReduce(sendBuf, recvBuf, count, dtype, op, name, done = nil)
 * (srcs/go/libkungfu-comm/collective.go:34-45). send == recv is in place.
 * Every peer must call it with the same name, count, dtype and op. */
int kf_session_all_reduce(kf_session_t *s, const void *send, void *recv,
                          size_t count, KungFu_Datatype dt, KungFu_Op op,
                          const char *name, void *stream);
/* GoKungfuSubsetAllReduce (srcs/go/libkungfu-comm/collective.go:47-60) ->
 * Session.SubsetAllReduce (srcs/go/kungfu/session/allreduce.go:14-24): every
 * tree of the forest all-reduces within itself. forest[i] = i's father, a
 * root is its own (graph.go:46-62); size entries. Chunked like the
 * all-reduce, one strategy (reduce = reversed tree with self loops, bcast =
 * the tree). A lone node forwards its send. KF_ERR_ARG for an index out of
 * range or a cycle. */
int kf_session_subset_all_reduce(kf_session_t *s, const void *send, void *recv, size_t count,
                                 KungFu_Datatype dt, KungFu_Op op, const int32_t *forest,
                                 const char *name, void *stream);
/* GoKungfuReduce (srcs/go/libkungfu-comm/collective.go:109-120) ->
 * Session.Reduce (srcs/go/kungfu/session/session.go:159-162): the reduce graph
 * of the session's first strategy only. The graph's root ends with the
 * reduction in recv; an inner node with its partial fold; a leaf's recv is
 * left as it was (runGraphs forwards only in a graph without self loops),
 * unless the peer is alone. Same fold order rules as the all-reduce. */
int kf_session_reduce(kf_session_t *s, const void *send, void *recv, size_t count,
                      KungFu_Datatype dt, KungFu_Op op, const char *name, void *stream);
/* GoKungfuBroadcast (collective.go:122-132) -> Session.Broadcast
 * (session.go:164-167): the first strategy's bcast graph; every peer's recv
 * becomes the root's send (the root forwards its own). */
int kf_session_broadcast(kf_session_t *s, const void *send, void *recv, size_t count,
                         KungFu_Datatype dt, const char *name, void *stream);
/* GoKungfuAllReduce with done != nil (srcs/go/libkungfu-comm/collective.go:
 * 34-45, main.go:184-191): start the all-reduce on the session's worker
 * thread and return KF_OK at once; done(status, arg) runs on that thread when
 * it has finished (the reference drops the error, main.go:188; here it is
 * passed on). Every started all-reduce is in flight at once in the worker's
 * poll loop and peers' chunks pair by name, as with the reference's goroutine
 * per call (rchannel/handler/collective.go:48-64), so peers may start their
 * names in different orders; done callbacks come in completion order. A name
 * started while its previous call is in flight waits for it (the next step's
 * call of the same name). Buffers stay valid and untouched until done; the
 * name is copied. A synchronous
 * kf_session_all_reduce first waits for everything queued before it; from
 * inside a done callback it (and kf_session_wait_all) returns KF_ERR_ARG
 * instead of waiting for itself. */
typedef void (*kf_done_fn)(int status, void *arg);
int kf_session_all_reduce_async(kf_session_t *s, const void *send, void *recv,
                                size_t count, KungFu_Datatype dt, KungFu_Op op,
                                const char *name, void *stream, kf_done_fn done,
                                void *arg);
/* Block until every queued all-reduce has finished; the first failure since
 * the previous wait (its message in kf_session_last_error), else KF_OK. */
/* Barrier (GoKungfuBarrier, libkungfu-comm/collective.go:17-20; session.go:
 * 104-115): an all-reduce of size() zero bytes every peer joins. Blocking;
 * device-mode sessions use a workspace of their own in HBM. */
int kf_session_barrier(kf_session_t *s);
int kf_session_wait_all(kf_session_t *s);
/* Peer::Rank / Size / LocalRank / LocalSize / HostCount (include/kungfu/
 * peer.hpp): peers with the same IPv4 share a host; local ranks follow the
 * peer list's order. Any pointer may be NULL. */
int kf_session_info(kf_session_t *s, int *rank, int *size, int *local_rank, int *local_size,
                    int *host_count);
void kf_session_destroy(kf_session_t *s);
const char *kf_session_last_error(void);

/* ---- peer-to-peer over xGMI (kungfu_amd/p2p.py) ------------------------ */

#define KF_IPC_HANDLE_BYTES 64
#define KF_MAX_SEGMENTS 16

/* Export the allocation holding dev_ptr for another process of this node:
 * handle[KF_IPC_HANDLE_BYTES] + the byte offset of dev_ptr inside it. */
int kf_ipc_export(const void *dev_ptr, void *handle, size_t *offset);
/* Map a peer's exported allocation; *base_out + offset is its dev_ptr. */
int kf_ipc_import(const void *handle, void **base_out);
int kf_ipc_close(void *base);
/* One launch copying nseg byte ranges dst[off_j, off_j + len_j) <-
 * srcs[j][off_j, off_j + len_j) (e.g. the shards other GPUs reduced, read
 * over xGMI); every offset, length and pointer 16-byte aligned. */
int kf_gather_segments(void *dst, const void *const *srcs, const size_t *offsets,
                       const size_t *lens, int nseg, void *stream);
/* One launch copying nseg byte ranges dsts[j][0, lens[j]) <- srcs[j][0,
 * lens[j]), any of them in a peer's HBM (the push exchange writes shards into
 * peers' buckets over xGMI); pointers and lengths 16-byte aligned. Blocks
 * alternate between segments so every link carries traffic at once. */
int kf_copy_segments(void *const *dsts, const void *const *srcs, const size_t *lens, int nseg,
                     void *stream);
/* Signal words for the device-side peer barrier: nwords zeroed 64-bit
 * words. host == 0: fine-grained, uncached device memory, exportable with
 * kf_ipc_export (every peer stores its arrival into it over xGMI); host == 1:
 * page-locked host memory the device can store into (the barrier's status
 * word, readable by the host without a sync). */
int kf_signal_alloc(size_t nwords, int host, void **ptr);
int kf_signal_free(void *ptr, int host);
/* Device-side barrier of `world` GPUs of one node, enqueued on `stream` (no
 * host round trip, no host sync): one 64-lane workgroup stores `epoch` into
 * word `rank` of every peer's signal array sigs[r] (system scope, over
 * xGMI), then waits until every word r != rank of its own array sigs[rank]
 * holds >= epoch. Stream order makes the work queued before it visible to the
 * peers (end-of-kernel release) and the work queued after it start after
 * every peer's arrival. Bounded: after timeout_us it stops waiting and stores
 * KF_ERR_TIMEOUT into status[0] (a host == 1 signal word), so a missing peer
 * cannot leave a wave spinning. epoch grows by one per barrier on every rank;
 * world <= 64. */
int kf_peer_barrier(void *const *sigs, int world, int rank, uint64_t epoch,
                    uint32_t timeout_us, void *status, void *stream);
const char *kf_p2p_last_error(void);

/* ---- multi-GPU exchange over RCCL (kungfu_amd/csrc/kf_exchange.hip) ------
 *
 * The reference's GPU collective, srcs/cpp/src/nccl/gpu_collective.cpp:
 * a communicator per process built from a unique id that rank 0 creates and
 * KungFu broadcasts (new_global, gpu_collective.cpp:190-200), then
 * ncclAllReduce per tensor with a stream sync after each call (:151-165).
 * Here the all-reduce of a bucket is split so the sum runs where the
 * north_star puts it:
 *   KF_ALGO_REDUCE_SCATTER  ncclReduceScatter -> HIP /np on the shard
 *                           (kf_bucket_div) -> in-place ncclAllGather;
 *   KF_ALGO_ALL_TO_ALL      ncclAllToAll of the shards -> HIP fold of the
 *                           world received shards IN RANK ORDER (/np fused)
 *                           -> in-place ncclAllGather. The sum is the HIP
 *                           k-input kernel, so the bits are the oracle's
 *                           reduce over ranks 0..world-1 for every dtype —
 *                           bf16 with fp32 accumulation and one rounding,
 *                           fp16 rounded per hop — equal to the P2P path;
 *                           same xGMI bytes as the reduce-scatter.
 *   KF_ALGO_REDUCE_SCATTER_AVG
 *                           for average calls: ncclReduceScatter with
 *                           ncclAvg (each input scaled by 1/world inside the
 *                           collective) -> in-place ncclAllGather, no HIP
 *                           epilogue launch. Opt-in: for f32/f64 the bits
 *                           equal KF_ALGO_REDUCE_SCATTER's (sum, then /np)
 *                           when world is a power of two and no x / world is
 *                           subnormal (scaling by 2^-k commutes with every
 *                           rounding of the sum); otherwise each input adds
 *                           one rounding. Calls without average: as
 *                           KF_ALGO_REDUCE_SCATTER.
 *   KF_ALGO_AUTO            reduce-scatter for integers and f32/f64
 *                           (RCCL's own order; integers exact; float MIN/MAX
 *                           differ from std::min/max only on NaN inputs),
 *                           all-to-all for f16/bf16 (the build's defined
 *                           semantics) and for u16/i16 (no RCCL type).
 * A count that does not split into world shards sends its last count % world
 * elements through an all-gather and the same rank-order fold. Everything
 * is queued on the caller's stream (no host sync, like RCCL); calls on one
 * exchange must be issued in the same order on every rank, and if they use
 * different streams the exchange orders its workspace between them.
 */
#define KF_UNIQUE_ID_BYTES 128
enum KF_ExchangeAlgo {
    KF_ALGO_AUTO           = 0,
    KF_ALGO_REDUCE_SCATTER = 1,
    KF_ALGO_ALL_TO_ALL     = 2,
    KF_ALGO_REDUCE_SCATTER_AVG = 3,
};
/* the reduce_scatter op a transport is asked for under
 * KF_ALGO_REDUCE_SCATTER_AVG: the sum of the inputs each scaled by 1/world
 * (ncclAvg); a transport without it returns a non-zero code */
#define KF_TRANSPORT_OP_AVG 4
#pragma GCC visibility pop
typedef struct kf_exchange kf_exchange_t; /* opaque */
#pragma GCC visibility push(default)

/* ncclGetUniqueId (rank 0 calls it, gpu_collective.cpp:196). */
int kf_exchange_unique_id(void *id);
/* Broadcast rank 0's id[KF_UNIQUE_ID_BYTES] to every peer of a session, in
 * place (Peer::Broadcast of the id, gpu_collective.cpp:197-198). */
int kf_exchange_share_id(kf_session_t *s, void *id);
/* ncclCommInitRank on HIP device `device` (the caller's current device is
 * restored). NULL on failure (kf_exchange_last_error). */
kf_exchange_t *kf_exchange_create(const void *id, int rank, int world, int device);
/* kf_exchange_create that gives up after timeout_ms (< 0: wait as long as it
 * takes) with KF_ERR_TIMEOUT in kf_exchange_last_error, when not every rank
 * joined the communicator's init in time. The init it abandons keeps waiting
 * on a helper thread (a late completion releases its communicator). */
kf_exchange_t *kf_exchange_create_timeout(const void *id, int rank, int world, int device,
                                          int timeout_ms);
/* gpu_collective::new_global: id from rank 0, shared over the session, then
 * kf_exchange_create(id, rank, size, device). */
kf_exchange_t *kf_exchange_create_session(kf_session_t *s, int rank, int world, int device);
/* recv = all-reduce(send) (op; average != 0: SUM then / world, float types).
 * send == recv is in place. */
int kf_exchange_all_reduce(kf_exchange_t *ex, const void *send, void *recv, size_t count,
                           KungFu_Datatype dt, KungFu_Op op, int average, int algo,
                           void *stream);
/* nb buckets in one call, each reduced as by kf_exchange_all_reduce: one
 * grouped RCCL launch per phase and one batched HIP launch
 * (kf_bucket_reduce_batch) for all shard epilogues / folds. */
int kf_exchange_all_reduce_batch(kf_exchange_t *ex, const void *const *sends, void *const *recvs,
                                 const size_t *counts, int nb, KungFu_Datatype dt, KungFu_Op op,
                                 int average, int algo, void *stream);
/* SMA (sma_sgd.py:60-65) for nb variable buckets: sums[b] = all-reduce-sum of
 * vs[b], then vs[b] = (1 - alpha) vs[b] + alpha sums[b] / world
 * (kf_sma_blend). sums[b] are caller workspaces of counts[b] elements. */
int kf_exchange_sma_batch(kf_exchange_t *ex, void *const *vs, void *const *sums,
                          const size_t *counts, int nb, KungFu_Datatype dt, double alpha,
                          int algo, void *stream);
/* Pipelined schedule for the batch calls (default 1 = off): the buckets of a
 * call are split into `groups` groups of consecutive buckets of about equal
 * bytes; the RCCL phases stay on the caller's stream in the same order on
 * every rank (group g+1's reduce-scatter / all-to-all before group g's
 * all-gather), and the element-wise work of group g (its shard epilogue or
 * rank-order fold, and for SMA its blends) runs on the exchange's own stream
 * meanwhile, ordered by events. Same results bit for bit. */
int kf_exchange_set_pipeline(kf_exchange_t *ex, int groups);
/* Opt-in per-phase timing of the batch calls (kf_exchange_all_reduce,
 * kf_exchange_all_reduce_batch, kf_exchange_sma_batch) on the un-pipelined
 * schedule: timing events on the caller's stream before phase 1 (every
 * bucket's reduce-scatter or all-to-all, and the tail gathers), phase 2 (the
 * /np epilogue or rank-order fold), phase 3 (the all-gathers), the SMA blend,
 * and after it. on != 0 starts a window with zeroed sums, 0 ends it. Costs
 * five event records per call; off by default. */
int kf_exchange_set_timing(kf_exchange_t *ex, int on);
/* The window's sums in microseconds: us[0] phase 1, us[1] phase 2, us[2]
 * phase 3, us[3] blend; *calls the timed calls, *untimed the pipelined ones
 * (their phases overlap on two streams, so they are not split). Waits for the
 * timed calls queued so far. calls / untimed may be NULL. */
int kf_exchange_phase_times(kf_exchange_t *ex, double *us, int64_t *calls, int64_t *untimed);
/* Ordered issue of concurrently produced all-reduces, the reference's
 * NCCLScheduler / LinearExecutor (srcs/cpp/src/nccl/scheduler.cpp:8-130):
 * begin_step fixes this step's names in an order every rank shares;
 * kf_exchange_start may be called for them in any order from any thread, and
 * the exchange's thread issues them strictly in that order (a name waits for
 * every name before it). With auto_order, the second step adopts rank 0's
 * arrival order of the first (broadcast over the communicator, as
 * NCCLScheduler::Reset does with Peer::Broadcast). done(status, arg) runs
 * when that all-reduce has completed on the device. */
int kf_exchange_begin_step(kf_exchange_t *ex, const char *const *names, int n, int auto_order);
int kf_exchange_start(kf_exchange_t *ex, const char *name, const void *send, void *recv,
                      size_t count, KungFu_Datatype dt, KungFu_Op op, int average, int algo,
                      void *stream, kf_done_fn done, void *arg);
/* Wait until every started all-reduce of the step has completed; the first
 * failure (its message in kf_exchange_last_error on this thread), else KF_OK.
 * *order (if not NULL, n entries) receives the issue order used. Destroy an
 * exchange only after this returned: tasks still queued are not issued and
 * their done callbacks never run. */
int kf_exchange_wait_all(kf_exchange_t *ex, int32_t *order);
/* KF_OK, or KF_ERR_RCCL after an asynchronous RCCL failure
 * (ncclCommGetAsyncError). */
int kf_exchange_check(kf_exchange_t *ex);
int kf_exchange_info(kf_exchange_t *ex, int *rank, int *world, int *device);
/* What the transport itself reports, for the bench line and logs: the RCCL
 * communicator's rank count (ncclCommCount) and RCCL's version
 * (ncclGetVersion, e.g. 22703). -1 / 0 for a host's own transport
 * (kf_exchange_create_transport) or a librccl without the symbol. A count
 * other than the exchange's world means the ranks did not form one
 * communicator. (The reference's nccl path asks neither,
 * srcs/cpp/src/nccl/gpu_collective.cpp:151-165; diagnostic only.) */
int kf_exchange_transport_info(kf_exchange_t *ex, int *comm_count, int *rccl_version);
void kf_exchange_destroy(kf_exchange_t *ex);
const char *kf_exchange_last_error(void);

/* Name-keyed all-reduce: GoKungfuAllReduce(send, recv, count, dtype, op,
 * name, done) (srcs/go/libkungfu-comm/collective.go:34-45) on the exchange.
 * Each rank may start its names in ANY order, from any thread: tensors pair
 * by name across ranks, as the reference's per-name mailbox pairs messages
 * (srcs/go/rchannel/handler/collective.go:48-64), not by call order. An
 * exchange thread agrees the issue order with the peers in negotiation
 * cycles (one all-gather of the newly started names per cycle over a second
 * communicator split off at the first call, so negotiating never waits
 * behind queued data collectives); a name is issued once every rank started
 * it, in rank 0's start order, and names that become ready in one cycle with
 * the same dtype / op / average / algo go out as ONE batched call (grouped
 * RCCL phases, one HIP launch). The data moves on the exchange's own stream
 * after the work queued on `stream` before this call; done(status, arg)
 * runs once the all-reduce finished on the device (kf_exchange_last_error
 * inside done gives a failure's message). A name may be outstanding once per
 * rank; count, dtype, op and average must agree across ranks (a mismatch
 * fails that name with KF_ERR_ARG on every rank). An empty name is the
 * anonymous call of a blocking op (the reference's all_reduce_cuda): the
 * exchange names it from its own counter, so such calls pair across ranks by
 * their order on each rank's exchange. Do not interleave these with the
 * ordered calls above on one exchange. */
int kf_exchange_all_reduce_named(kf_exchange_t *ex, const char *name, const void *send, void *recv,
                                 size_t count, KungFu_Datatype dt, KungFu_Op op, int average,
                                 int algo, void *stream, kf_done_fn done, void *arg);
/* Block until every name started so far on this rank has completed; the
 * first failure since the previous wait (message in kf_exchange_last_error),
 * else KF_OK. Destroy an exchange only after this returned. */
int kf_exchange_wait_named(kf_exchange_t *ex);

/* ---- exchange transports ---------------------------------------------------
 * The exchange issues five collectives and moves every byte through them; a
 * transport is the table of those collectives bound to one communicator.
 * kf_exchange_create binds the built-in librccl transport (RCCL over xGMI).
 * kf_exchange_create_transport binds any other one — a host's own collective
 * library, or a stand-in that lets the exchange's multi-rank logic run where
 * RCCL cannot (several ranks on one device; tests/c/kf_testing.cpp). Every
 * function queues its work on `stream` (a hipStream_t) in call order and
 * returns 0, or a transport code that error_string explains. The calls
 * between group_start and group_end belong to one phase and may be fused.
 * reduce_scatter sums count elements per rank (op, dt as the exchange's own
 * kernels define them, or KF_TRANSPORT_OP_AVG) and may refuse a dtype or op
 * with a non-zero code; the
 * AUTO algo never asks for an f16 / bf16 / u16 / i16 reduce-scatter. split
 * (ncclCommSplit's contract: collective over comm; ranks of one color form a
 * communicator ordered by key) is needed by kf_exchange_split and the named
 * all-reduce. The table must outlive every exchange bound to it; the
 * exchange owns `comm` and releases it with destroy. */
typedef struct kf_transport_ops {
    int (*group_start)(void *comm);
    int (*group_end)(void *comm);
    int (*reduce_scatter)(const void *send, void *recv, size_t count, KungFu_Datatype dt,
                          KungFu_Op op, void *comm, void *stream);
    int (*all_gather)(const void *send, void *recv, size_t bytes, void *comm, void *stream);
    int (*all_to_all)(const void *send, void *recv, size_t bytes, void *comm, void *stream);
    int (*broadcast)(const void *send, void *recv, size_t bytes, int root, void *comm,
                     void *stream);
    int (*split)(void *comm, int color, int key, void **newcomm);
    int (*async_error)(void *comm);
    void (*destroy)(void *comm);
    const char *(*error_string)(int code);
} kf_transport_ops;
/* An exchange of rank `rank` of `world` on HIP device `device` over `ops`
 * bound to `comm` (ownership passes to the exchange; on failure the caller
 * keeps it). A one-rank exchange over a transport still calls it (only the
 * built-in RCCL transport short-cuts world 1 to a copy). */
kf_exchange_t *kf_exchange_create_transport(const kf_transport_ops *ops, void *comm, int rank,
                                            int world, int device);
/* gpu_collective::new_local / new_group (srcs/cpp/src/nccl/gpu_collective.cpp:
 * 202-243): a new exchange over the ranks of `ex` that pass the same color,
 * ranked by key (ties by rank), on the same device. Collective over `ex`:
 * every rank calls it at the same point of its call sequence. color < 0:
 * this rank joins none (returns NULL with KF_OK in *status). The local scope
 * is color = host index, key = rank (kf_exchange_create_local). */
kf_exchange_t *kf_exchange_split(kf_exchange_t *ex, int color, int key, int *status);

/* ---- hierarchical all-reduce (several hosts, several GPUs each) -----------
 * gpu_collective::new_local (srcs/cpp/src/nccl/gpu_collective.cpp:202-212):
 * an exchange over this host's ranks of the session `s` (same IPv4), ranked
 * in the session's order. Each host's first rank creates the RCCL id; every
 * host's id travels in ONE session all-reduce of hosts x 128 bytes (one
 * contributor per slot, so the sum is the id). Collective over `s`. */
kf_exchange_t *kf_exchange_create_local(kf_session_t *s, int device);
/* ScheduledHierarchicalNcclAllReduce (srcs/cpp/src/tensorflow/ops/gpu/
 * collective.cpp:108-162: ncclReduce in the host -> CrossAllReduceGpu over
 * the hosts, nccl/controller.cpp:7-39 -> ncclBroadcast in the host), with the
 * bucket sharded across the host's GPUs when every host has as many:
 *   1. local reduce-scatter (algo: RCCL's, or the all-to-all + HIP rank-order
 *      fold) — local rank j holds shard j of its host's sum;
 *   2. the shard all-reduced across hosts by the device-mode session `cross`
 *      among the ranks with the same local rank (kf_session_subset_all_reduce,
 *      one tree per local rank), so every link carries 1/local_size of it;
 *   3. average: / size() on the shard (kf_bucket_div);
 *   4. local in-place all-gather.
 * Hosts of different sizes take the reference's path: local all-reduce, the
 * hosts' first ranks all-reduce across hosts, local broadcast. `local` must
 * hold exactly this host's ranks in session order (kf_exchange_create_local,
 * or any transport with that layout); every rank calls with the same name,
 * count, dtype and op, in the same order. Buffers are HBM; queued on
 * `stream`, blocking on the host while the cross-host step runs. */
int kf_hier_all_reduce(kf_exchange_t *local, kf_session_t *cross, const void *send, void *recv,
                       size_t count, KungFu_Datatype dt, KungFu_Op op, int average, int algo,
                       const char *name, void *stream);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
