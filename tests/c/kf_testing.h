/*
 * kf_testing.h — test-only transports for the exchange (tests/c/libkf_testing.so,
 * built by tests/c/Makefile). NOT part of the product library: they plug into
 * libkungfu_amd.so through kf_exchange_create_transport (include/kungfu_amd.h).
 *
 *  loopback   `world` ranks that are threads of ONE process on ONE device
 *             (RCCL refuses two ranks on one GPU). Each rank's exchange runs
 *             the product's code — shards, tails, workspace, batched folds,
 *             the ordered scheduler, the name-keyed negotiation, splits —
 *             with every collective a rendezvous of the ranks' threads that
 *             moves the bytes with hipMemcpy (the reduce-scatter folds in rank
 *             order on the host; no f16/bf16/u16/i16 reduce-scatter). Every
 *             rank's calls must come from its own thread.
 *  rccl1      a one-rank librccl communicator bound through the transport
 *             table, so the exchange calls librccl's own entry points with
 *             its exact arguments instead of the built-in world-1 copy.
 *  ipc        `world` PROCESSES on one device (tests/c/kf_testing_ipc.hip):
 *             every collective stages the rank's input in its own HBM buffer,
 *             meets the other ranks in a POSIX shared-memory segment, and
 *             pulls from the peers' staging buffers through HIP IPC mappings
 *             (the reduce-scatter folds in rank order on the device, every
 *             integer / f32 / f64 op and ncclAvg's premultiplied float form;
 *             no f16/bf16/u16/i16 reduce-scatter). Synchronous, no
 *             performance claim: it lets bench.py's N > 1 branch run the
 *             native exchange with N ranks where RCCL refuses to share a GPU.
 */
#pragma once
#include "kungfu_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct kf_loopback kf_loopback_t;
kf_loopback_t *kf_loopback_create(int world);
/* after every exchange of the group (and of its splits) was destroyed */
void kf_loopback_destroy(kf_loopback_t *g);
kf_exchange_t *kf_exchange_create_loopback(kf_loopback_t *g, int rank, int device);
/* every rank's collective call number `call` (0-based, counted per rank's
 * communicator since its creation) fails with "injected failure" before its
 * rendezvous; -1 = none. Set before the ranks call. */
void kf_loopback_fail_at(kf_loopback_t *g, int64_t call);
/* NULL on failure (kf_testing_last_error) */
kf_exchange_t *kf_exchange_create_rccl1(int device);
const char *kf_testing_last_error(void);

/* Join the cross-process group `name` (one "/name" component, unique to the
 * run; every rank passes the same) as `rank` of `world` on HIP device
 * `device`. Collective: returns once every rank has joined, or NULL after
 * timeout_ms (<= 0: 120 s) or on failure (kf_ipc_last_error). The same
 * timeout bounds every rendezvous of the group's collectives; a timeout or a
 * failure on any rank fails every later call of every rank. */
kf_exchange_t *kf_exchange_create_ipc(const char *name, int rank, int world, int device,
                                      int timeout_ms);
const char *kf_ipc_last_error(void);

#ifdef __cplusplus
}
#endif
