// kf_stream.hpp — library-internal: chunks that cross their GPU stage while
// the socket still carries them (kf_stream.hip). Not part of the C ABI.
//
// A device-mode session moves every 1 MiB chunk through a GPU stage next to
// a socket: the leaf copies its chunk out of HBM before writing it, the star
// root folds a received chunk into its own and writes the result back, the
// leaf copies the reduced chunk into HBM. Done a whole chunk at a time, each
// stage waits for the one before it (C1 np = 2: 0.66 ms against 0.43 ms for
// the reference's CPU fold on host buffers). Done in pieces with
// a launch per piece, the launches land on the thread that reads the socket
// and cost more than they hide. Here ONE kernel per chunk is launched before
// the bytes arrive and waits in the GPU for them: the reading thread only
// publishes how many bytes have landed (a release store into page-locked
// memory), each block folds or copies its 4 KiB once they are there, and marks
// its block done in page-locked memory, where the sender picks each piece up
// as soon as all its blocks are final. The wait is bounded (a deadline in the
// kernel, an abort word from the host), so a body that never comes ends the
// kernel.
//
// What the GPU pays for it (tools/explore/stream_probe.hip, 1 MiB, 256
// blocks, on the box): plain 16-B stores to page-locked memory 20 us; with
// one system-scope atomic add per block onto a per-piece counter 254 us
// (atomics to host memory serialise); one flag word per block behind a
// system release fence 36 us; written-through (sc1) stores drained before
// the flag 21.6 us — the r04 form; r05 ships the same with system scope
// (sc0 sc1, kf_stream.hip KF_STREAM_HOST_STORE_AUX). Reads: plain 24-29 us, one acquire
// fence per block 54-61 us, system-coherent (sc0 sc1) loads 26.5 us — the
// shipped form. In a running session the per-block fences also serialise on
// each XCD's L2 (a write-back and an invalidate of the whole L2 each, 257
// per chunk): the last piece came 65-240 us after the last byte with them,
// 4-5 us without.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include "kungfu_amd.h"

namespace kf_stream
{
constexpr uint32_t kBlockBytes = 4096;  // one 256-lane block moves 16 B per lane
constexpr uint32_t kMaxBlocks  = 272;   // blocks of one chunk (1 MiB + 64 KiB)

// One chunk's control block, in page-locked coherent host memory.
struct Ctl {
    uint32_t landed;  // host: body bytes in the landing buffer (release store)
    uint32_t abort;   // host: the rest of the body will not come
    uint32_t err;     // device: a block stopped waiting (deadline or abort); the
                      // host fails the collective on it (kf_session complete())
    uint32_t bpp;     // blocks per piece (the sender's unit)
    uint32_t done[kMaxBlocks];  // device: block b's output is in host memory
};

// The device words the streamed kernels' watchers publish through (HBM, one
// board per session). board_create() runs on the thread that creates the
// session, before its sender / worker threads start: it allocates the words
// and resolves every kernel of kf_stream.hip for the current device there, so
// no HIP module state is initialised lazily under a concurrent launch.
struct Board;
Board *board_create();  // nullptr on a HIP failure
void board_destroy(Board *b);

// SUM in any dtype (the S-SGD / SMA sum); other ops take the whole-chunk path
bool supported(KungFu_Datatype dt, KungFu_Op op);
// piece: bytes per sending unit, a multiple of kBlockBytes; len must fit
// kMaxBlocks blocks. Call before the launch that uses `c`.
void reset(Ctl *c, uint32_t piece);
// the page-locked landing buffer holds `bytes` of the body now
void publish(Ctl *c, uint32_t bytes);
void abort_wait(Ctl *c);

// One kernel each, queued on `stream`; `host_dev` is the device address of
// page-locked memory. deadline_ms bounds every block's wait for the body.
// mark: the fold's output is page-locked memory a sender reads piece by piece
// (each block flags its 4 KiB done); otherwise it is HBM and nothing is flagged.
int launch_fold(KungFu_Datatype dt, const void *own, const void *landing_dev, void *out,
                uint32_t len, uint32_t piece, Ctl *c_dev, Board *board, int deadline_ms,
                bool mark, void *stream);
int launch_copy_in(const void *landing_dev, void *dst, uint32_t len, uint32_t piece, Ctl *c_dev,
                   Board *board, int deadline_ms, void *stream);
int launch_copy_out(const void *src, void *host_dev, uint32_t len, uint32_t piece, Ctl *c_dev,
                    void *stream);

// A chunk's copy between HBM and page-locked memory (either way; device
// addresses) by a kernel instead of hipMemcpyAsync: on some boxes the DMA
// engines take 150 us for 1 MiB where a kernel takes 20-27 us
// (profiles/r04/stream_probe*_r04s3.json). Used where copy_kernels() says so
// (KUNGFU_AMD_COPY_KERNEL=1).
bool copy_kernels();
int launch_copy(void *dst, const void *src, size_t len, void *stream);

// Host side of the sender, for a chunk of len bytes: wait until piece k is
// final (KF_OK), the device gave up (KF_ERR_HIP) or timeout_ms passed
// (KF_ERR_TIMEOUT); how many pieces from k on are final already. A block
// that gave up (deadline, abort) sets err and never flags itself done.
int wait_piece(const Ctl *c, uint32_t k, uint32_t len, int timeout_ms);
uint32_t ready_run(const Ctl *c, uint32_t k, uint32_t len);
}  // namespace kf_stream

// How the library's host threads wait for the GPU. HIP's default event wait
// spins a core; with many peer processes on one host (C1 at np = 8: 8
// processes, 2-3 waiting threads each, on a 16-CPU quota) spinning waits
// burn the quota. KUNGFU_AMD_BLOCKING_SYNC=1 makes every event the library
// creates a blocking-sync event (the thread sleeps until the GPU signals)
// and every stream wait an event wait.
namespace kf_sync
{
unsigned event_flags();          // for hipEventCreateWithFlags
int stream_sync(void *stream);   // KF_OK or KF_ERR_HIP
}  // namespace kf_sync

// kf_ingest.hip: the streamed receives (body read into the next landing slot
// while the kernel launched before it folds / copies each landed block)
int kf_ingest_recv_onto_streamed(kf_ingest_t *g, int fd, uint32_t len, void *dev_acc,
                                 const void *dev_own, KungFu_Datatype dt, void *stream,
                                 uint32_t piece, kf_stream::Ctl *ctl, kf_stream::Ctl *ctl_dev,
                                 kf_stream::Board *board, int deadline_ms, bool mark,
                                 void *wait_stream);
int kf_ingest_recv_into_streamed(kf_ingest_t *g, int fd, uint32_t len, void *dev_dst,
                                 void *stream, uint32_t piece, kf_stream::Ctl *ctl,
                                 kf_stream::Ctl *ctl_dev, kf_stream::Board *board,
                                 int deadline_ms, void *wait_stream);
// (wait_stream: a non-blocking stream the kernel runs on while it waits for
// the body, when `stream` is one other work serialises with; kf_ingest.hip)
