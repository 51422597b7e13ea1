// kf_capi.hip — C-ABI entry points of libkungfu_amd.so (include/kungfu_amd.h).
//
// B2 (device API): dtype/op/epilogue dispatch onto the templated kernels in
// kf_reduce_kernels.hpp, launch geometry, alignment handling. Never allocates,
// never synchronises: capture-safe.
//
// B1 (drop-in, host pointers): std_transform_2 / float16_sum move the caller's
// host buffers to HBM, run the same kernels, copy the result back and return
// when it is written (cgo contract, srcs/go/kungfu/base/op.go:27-35). Each
// calling OS thread gets its own stream and device scratch (the reference
// calls this concurrently from one goroutine per chunk, session.go:317-323).
// There is no CPU fallback: without a device the call prints why and exits,
// as the reference does for any unusable argument (op.cpp:41,52,89).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <vector>

#include "kf_reduce_kernels.hpp"
#include "kungfu_amd.h"

namespace
{
using namespace kf;

constexpr int kBlock = 256;

// Launch geometry for the streaming body. Defaults tuned on MI355X with
// tools/tune_reduce.py (DESIGN.md "Kernel tuning"); kf_set_geometry() exists
// only for that tuning script.
// Measured on MI355X (profiles/r01/tune_c2_rot3.jsonl: 256 MiB fp32, launches
// cycling over 3 independent bucket sets so no output is still in the 256 MiB
// Infinity Cache; 5 rounds interleaved in one process): non-temporal loads and
// stores, 4 vectors per thread, one block per tile (no grid-stride) is
// fastest at 122.0 us = 6.60 TB/s. With the same buffers every launch
// (profiles/r01/tune_c2.jsonl) it runs 116.9 us, within 2% of the best there.
struct Geometry {
    int unroll   = 4;        // 16-B vectors per thread per input per tile
    int grid_cap = 1 << 20;  // blocks; grid-stride beyond (8 GiB fp32 buckets)
    int loadnt   = 1;        // non-temporal read streams
    int stplain  = 0;        // plain (not non-temporal) stores
    // Occupancy cap of reduce_kernel, as dynamic LDS per block the kernel
    // never touches (160 KiB per CU / bytes = resident blocks per CU). The
    // k-input fold runs best with few requests outstanding chip-wide: one
    // vector in flight per lane past inputs 0 and 1 (ld_vec_serial) and five
    // 256-thread blocks per CU instead of eight — k = 3/4/6/8 at
    // 0.803/0.806/0.805/0.801 of 8 TB/s in one process on the same buffers,
    // against 0.787/0.779/0.768/0.760 for four vectors in flight uncapped
    // (tools/explore/kfold_mlp.hip, kfold_occ.hip; profiles/r02/kfold_mlp*.jsonl,
    // kfold_occ*.jsonl). Six to four blocks per CU form a plateau and three
    // fall off it (k = 8 0.72), so the cap sits in its middle; the product
    // kernel equals the probe on the same buffers (kfold_prod_vs_probe3.jsonl:
    // k = 8 0.790, k = 4 0.796). A grid-stride grid of the same residency loses.
    // Both apply to large launches only (kSerialMinBlocks, kCapMinBlocks below):
    // a grid that fits on the chip at once is latency-bound instead.
    // k <= 2 (the C2 sum, /np, SMA) shows no gain beyond the noise and stays
    // uncapped (ab_c2_occupancy.jsonl), and so does the batched launch, which
    // in the exchange's pipelined schedule runs beside RCCL kernels whose
    // blocks LDS held idle would keep out.
    int occ_small = 0;          // k <= 2
    int occ_fold  = 32 << 10;   // k >= 3: five blocks per CU
};

Geometry &geometry()
{
    static Geometry g;
    return g;
}

thread_local std::string t_last_error;

int hip_fail(hipError_t e, const char *what)
{
    t_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return KF_ERR_HIP;
}

#define KF_HIP(call)                                                           \
    do {                                                                       \
        hipError_t e_ = (call);                                                \
        if (e_ != hipSuccess) return hip_fail(e_, #call);                      \
    } while (0)

int type_size(KungFu_Datatype dt)
{
    switch (dt) {
    case KungFu_UINT8: case KungFu_INT8: case KungFu_BOOL: return 1;
    case KungFu_UINT16: case KungFu_INT16: case KungFu_FLOAT16:
    case KungFu_BFLOAT16: return 2;
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

Div make_div(int np)
{
    Div d;
    d.f    = static_cast<float>(np);
    d.d    = static_cast<double>(np);
    d.pow2 = np > 0 && (np & (np - 1)) == 0;
    d.fi   = 1.0f / d.f;  // exact for powers of two
    d.di   = 1.0 / d.d;
    return d;
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
struct Plan {
    size_t head = 0, nvec = 0;
    bool vec_ok  = false;
    int grid_cap = 0;  // 0: geometry().grid_cap (HBM); >0: host-link launch
};

// launch-mode bits passed down the dispatch chain
enum { LM_NONE = 0, LM_SPREAD = 1 };  // LM_SPREAD: inputs behind different links

// The head peels elements until the OUTPUT is 16-B aligned; the vector body
// then stores whole aligned 16-B vectors. Inputs need only element alignment:
// one whose 16-B residue differs from the output's is read with the same
// global_load_dwordx4 at an unaligned address (gfx950 runs HSA queues in
// unaligned-access mode; the wave's 1 KiB stays contiguous, so the extra
// cache line per wave-instruction costs little): 256 MiB with one input off
// the output's residue runs at 0.80-0.82 of the roofline (f32, bf16, u8), with
// all three pointers at different residues 0.72-0.79, against 0.29-0.68 for
// the element-wise kernel this replaces (tools/unaligned_rate.py;
// profiles/r02/unaligned_rate_{vector,elementwise}.jsonl).
// KUNGFU_AMD_NO_UNALIGNED_VECTOR=1 keeps such inputs on the element-wise
// kernel (A/B only).
bool unaligned_vector_ok()
{
    static const bool ok = [] {
        const char *e = std::getenv("KUNGFU_AMD_NO_UNALIGNED_VECTOR");
        return !(e && std::atoi(e) != 0);
    }();
    return ok;
}

Plan make_plan(const void *const *in, int k, const void *out, size_t n, int sz)
{
    Plan p;
    const uintptr_t r = reinterpret_cast<uintptr_t>(out) & 15u;
    if (r % sz != 0) return p;
    const bool ua = unaligned_vector_ok();
    for (int j = 0; j < k; ++j) {
        const uintptr_t rj = reinterpret_cast<uintptr_t>(in[j]) & 15u;
        if (ua ? (rj % sz != 0) : (rj != r)) return p;
    }
    size_t head = r == 0 ? 0 : (16 - r) / sz;
    if (head > n) head = n;
    p.head   = head;
    p.nvec   = (n - head) / (16 / sz);
    p.vec_ok = true;
    return p;
}

unsigned grid_for(size_t nvec, size_t nedge, int unroll, int cap = 0)
{
    const size_t tile   = static_cast<size_t>(kBlock) * unroll;
    size_t blocks       = (nvec + tile - 1) / tile;
    const size_t eblk   = (nedge + kBlock - 1) / kBlock;
    if (cap <= 0) cap = geometry().grid_cap;
    if (blocks > static_cast<size_t>(cap)) blocks = cap;
    if (blocks < eblk) blocks = eblk;
    if (blocks < 1) blocks = 1;
    return static_cast<unsigned>(blocks);
}

// The runtime-k fold's schedule and residency follow the size of the launch
// (tools/explore/kfold_mlp.hip s|m|asm; profiles/r02/kfold_mlp_{small,mid}*,
// kfold_mlp_asm.jsonl; k = 8, time per launch, batched-4 vs one-in-flight):
// below 2048 blocks (32 MiB per input) the whole grid is resident at once and
// latency-bound, so an input's four vectors go together (4 MiB: 7.6 vs
// 14.4 us; 16 MiB: 23.6 vs 24.7 us); from 2048 blocks one vector in flight
// wins (64 MiB: 92.2 vs 96.3 us), and from 8192 blocks (128 MiB) the
// residency cap adds to it (256 MiB: 382 vs 391 us uncapped, 405 batched).
constexpr unsigned kSerialMinBlocks = 2048;
// the batched launch's own threshold (tools/ab_batch_shape.py builds variants).
// At 256, 1024 or 2048 blocks, C5's a2a fold (~1670 blocks) and the
// 16 x 4 MiB k = 2 batch time within 0.5 % of each other
// (profiles/r05/ab_batch_serial_r05an.jsonl), so it stays at the fold's 2048
#ifndef KF_BATCH_SERIAL_MIN_BLOCKS
#define KF_BATCH_SERIAL_MIN_BLOCKS 2048
#endif
constexpr unsigned kBatchSerialMinBlocks = KF_BATCH_SERIAL_MIN_BLOCKS;
constexpr unsigned kCapMinBlocks    = 8192;

// dynamic LDS of an HBM streaming launch of `blocks` blocks over k inputs
// (Geometry::occ_*); none for a launch over the host link (small grid)
unsigned occ_lds(int k, size_t blocks, bool host_link = false)
{
    if (host_link) return 0;
    if (k >= 3) return blocks >= kCapMinBlocks ? static_cast<unsigned>(geometry().occ_fold) : 0;
    return static_cast<unsigned>(geometry().occ_small);
}

template <typename T, int OP, int EPI, int KC, int UNROLL, int LOADNT, int STPLAIN = 0>
void launch_vec(const InPtrs &ptrs, int k, void *out, size_t n, const Plan &p,
                const Div &np, hipStream_t s)
{
    constexpr int V  = Vec<typename Elt<T>::S>::N;
    const size_t ned = p.head + (n - p.head - p.nvec * V);
    const unsigned g = grid_for(p.nvec, ned, UNROLL, p.grid_cap);
    const int serial = KC == 0 && g >= kSerialMinBlocks ? 1 : 0;
    reduce_kernel<T, OP, EPI, KC, kBlock, UNROLL, LOADNT, STPLAIN>
        <<<g, kBlock, occ_lds(k, g, p.grid_cap > 0), s>>>(ptrs, k, out, n, p.head, p.nvec, np,
                                                          serial);
}

// The tuned fp32 2-input SUM (the headline path) carries every geometry
// variant; every other combination uses the tuned default (unroll 4,
// non-temporal loads and stores).
template <typename T, int OP, int EPI, int KC, int LOADNT, int STPLAIN>
void launch_unroll(const InPtrs &ptrs, int k, void *out, size_t n, const Plan &p,
                   const Div &np, hipStream_t s)
{
    switch (geometry().unroll) {
    case 1: return launch_vec<T, OP, EPI, KC, 1, LOADNT, STPLAIN>(ptrs, k, out, n, p, np, s);
    case 2: return launch_vec<T, OP, EPI, KC, 2, LOADNT, STPLAIN>(ptrs, k, out, n, p, np, s);
    case 8: return launch_vec<T, OP, EPI, KC, 8, LOADNT, STPLAIN>(ptrs, k, out, n, p, np, s);
    default: return launch_vec<T, OP, EPI, KC, 4, LOADNT, STPLAIN>(ptrs, k, out, n, p, np, s);
    }
}

template <typename T, int OP, int EPI, int KC>
void launch_geom(const InPtrs &ptrs, int k, void *out, size_t n, const Plan &p,
                 const Div &np, hipStream_t s)
{
    const Geometry &g = geometry();
    if constexpr (std::is_same<T, float>::value && OP == OP_SUM && KC == 2 &&
                  EPI == EPI_NONE) {
        if (g.loadnt && g.stplain) return launch_unroll<T, OP, EPI, KC, 1, 1>(ptrs, k, out, n, p, np, s);
        if (g.loadnt) return launch_unroll<T, OP, EPI, KC, 1, 0>(ptrs, k, out, n, p, np, s);
        if (g.stplain) return launch_unroll<T, OP, EPI, KC, 0, 1>(ptrs, k, out, n, p, np, s);
        return launch_unroll<T, OP, EPI, KC, 0, 0>(ptrs, k, out, n, p, np, s);
    }
    // about 8 16-B loads in flight per thread whatever k is
    constexpr int U = KC == 0 || KC <= 2 ? 4 : KC <= 4 ? 2 : 1;
    launch_vec<T, OP, EPI, KC, U, 1>(ptrs, k, out, n, p, np, s);
}

// k = 1 (the shard epilogue) and k = 2 (the hot path) are compile-time; for
// k > 2 the runtime loop — inputs 0 and 1 up front, then one input at a time —
// measured faster than loading all k inputs at once (k = 4: 221.8 vs 226.4 us,
// k = 8: 405.9 vs 419.8 us for 256 MiB fp32, profiles/r01/kernel_rates*.jsonl):
// fewer concurrent streams keep DRAM rows open longer.
template <typename T, int OP, int EPI>
void launch_k(const InPtrs &ptrs, int k, void *out, size_t n, const Plan &p,
              const Div &np, hipStream_t s)
{
    if (k == 2) return launch_geom<T, OP, EPI, 2>(ptrs, k, out, n, p, np, s);
    if (k == 1) return launch_geom<T, OP, EPI, 1>(ptrs, k, out, n, p, np, s);
    launch_geom<T, OP, EPI, 0>(ptrs, k, out, n, p, np, s);
}

template <typename T, int OP, int EPI>
int launch_typed(const void *const *in, int k, void *out, size_t n, int npi,
                 hipStream_t s, int grid_cap, int mode = LM_NONE)
{
    const Div np = make_div(npi);
    using S = typename Elt<T>::S;
    InPtrs ptrs;
    for (int j = 0; j < kMaxInputs; ++j) ptrs.p[j] = j < k ? in[j] : nullptr;
    Plan p     = make_plan(in, k, out, n, sizeof(S));
    p.grid_cap = grid_cap;
    if (p.vec_ok && (mode & LM_SPREAD) && k > 1) {
        constexpr int V  = Vec<S>::N;
        const size_t ned = p.head + (n - p.head - p.nvec * V);
        const unsigned g = grid_for(p.nvec, ned, 1);
        reduce_spread_kernel<T, OP, EPI, kBlock><<<g, kBlock, 0, s>>>(ptrs, k, out, n, p.head,
                                                                      p.nvec, np);
    } else if (!p.vec_ok) {
        size_t blocks = (n + kBlock - 1) / kBlock;
        const size_t cap = grid_cap > 0 ? static_cast<size_t>(grid_cap) : 8192;
        if (blocks > cap) blocks = cap;
        reduce_kernel_unaligned<T, OP, EPI, kBlock>
            <<<static_cast<unsigned>(blocks), kBlock, 0, s>>>(ptrs, k, out, n, np);
    } else {
        launch_k<T, OP, EPI>(ptrs, k, out, n, p, np, s);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "reduce kernel launch");
    return KF_OK;
}

template <typename T, int EPI>
int dispatch_op(const void *const *in, int k, void *out, size_t n, KungFu_Op op,
                int np, hipStream_t s, int gc, int mode)
{
    if constexpr (std::is_same<T, f16_t>::value) {
        if (op != KungFu_SUM) return KF_ERR_OP;  // op.cpp:45-54
        return launch_typed<T, OP_SUM, EPI>(in, k, out, n, np, s, gc, mode);
    } else {
        if constexpr (EPI == EPI_DIV) {
            if (op != KungFu_SUM) return KF_ERR_OP;
            return launch_typed<T, OP_SUM, EPI>(in, k, out, n, np, s, gc, mode);
        } else {
            switch (op) {
            case KungFu_SUM: return launch_typed<T, OP_SUM, EPI>(in, k, out, n, np, s, gc, mode);
            case KungFu_MIN: return launch_typed<T, OP_MIN, EPI>(in, k, out, n, np, s, gc, mode);
            case KungFu_MAX: return launch_typed<T, OP_MAX, EPI>(in, k, out, n, np, s, gc, mode);
            case KungFu_PROD: return launch_typed<T, OP_PROD, EPI>(in, k, out, n, np, s, gc, mode);
            default: return KF_ERR_OP;
            }
        }
    }
}

int dispatch_none(const void *const *in, int k, void *out, size_t n,
                  KungFu_Datatype dt, KungFu_Op op, hipStream_t s, int gc = 0,
                  int mode = LM_NONE)
{
    switch (dt) {
    case KungFu_UINT8: return dispatch_op<uint8_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_UINT16: return dispatch_op<uint16_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_UINT32: return dispatch_op<uint32_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_UINT64: return dispatch_op<uint64_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_INT8: return dispatch_op<int8_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_INT16: return dispatch_op<int16_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_INT32: return dispatch_op<int32_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_INT64: return dispatch_op<int64_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_FLOAT16: return dispatch_op<f16_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_FLOAT: return dispatch_op<float, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_DOUBLE: return dispatch_op<double, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    case KungFu_BFLOAT16: return dispatch_op<bf16_t, EPI_NONE>(in, k, out, n, op, 1, s, gc, mode);
    default: return KF_ERR_DTYPE;  // BOOL and unknown: op.cpp:88-89
    }
}

int dispatch_div(const void *const *in, int k, void *out, size_t n,
                 KungFu_Datatype dt, int np, hipStream_t s, int mode = LM_NONE)
{
    switch (dt) {
    case KungFu_FLOAT16: return dispatch_op<f16_t, EPI_DIV>(in, k, out, n, KungFu_SUM, np, s, 0, mode);
    case KungFu_FLOAT: return dispatch_op<float, EPI_DIV>(in, k, out, n, KungFu_SUM, np, s, 0, mode);
    case KungFu_DOUBLE: return dispatch_op<double, EPI_DIV>(in, k, out, n, KungFu_SUM, np, s, 0, mode);
    case KungFu_BFLOAT16: return dispatch_op<bf16_t, EPI_DIV>(in, k, out, n, KungFu_SUM, np, s, 0, mode);
    default: return KF_ERR_DTYPE;
    }
}

int check_args(const void *const *inputs, int k, const void *out, size_t n)
{
    if (k < 1 || k > KF_MAX_INPUTS) return KF_ERR_ARG;
    if (n == 0) return KF_OK;
    if (!inputs || !out) return KF_ERR_ARG;
    for (int j = 0; j < k; ++j) {
        if (!inputs[j]) return KF_ERR_ARG;
    }
    return KF_OK;
}

// ---------------------------------------------------------------------------
// batch: nb buckets, one launch per kBatchSeg of them (kf_bucket_reduce_batch)
// ---------------------------------------------------------------------------
// tile shape of the batched launch (tools/ab_batch_shape.py builds variants;
// profiles/r03/ab_batch_shape.jsonl). k = 1 (the shard /np after a
// reduce-scatter) takes two vectors per lane: its launches are small and
// latency-bound, and twice the blocks for the same bytes finish sooner (C4's
// 16 shards at N = 8: 8.4 -> 7.0 us; C3's 64: 16.2 -> 15.8 us). Four per lane
// once the grid outgrows one resident wave looked better on shards allocated
// one by one (C3 14.3 -> 13.4 us, shard_probe.hip), but the exchange's shards
// are slices of ONE flat buffer of buckets, one shard every bucket's length;
// there four per lane is 30 % slower (C3 15.2 -> 19.8 us,
// tools/explore/shard_xcd_probe.hip, profiles/r05/shard_xcd_probe_r05ae.jsonl),
// so k = 1 stays at two. k >= 2 keeps four (k = 2 16 x 4 MiB, the k = 8 fold
// of C5: equal within 1 %, one lane per vector up to 6 % slower).
#ifndef KF_BATCH_UNROLL
#define KF_BATCH_UNROLL 4
#endif
#ifndef KF_BATCH_UNROLL_K1
#define KF_BATCH_UNROLL_K1 2
#endif
#ifndef KF_BATCH_BLOCK
#define KF_BATCH_BLOCK 256
#endif
template <typename T, int OP, int EPI, int KC, int U>
int launch_batch_kc(const void *const *in, int k, void *const *outs, const size_t *counts,
                    int nb, const Div &np, int npi, hipStream_t s)
{
    using S           = typename Elt<T>::S;
    constexpr int V   = Vec<S>::N;
    constexpr int B   = KF_BATCH_BLOCK;
    constexpr int NSEG = KC == 1 ? kBatchSeg1 : kBatchSeg;
    constexpr int NPTR = KC == 1 ? 1 : kMaxInputs;
    const size_t tile = static_cast<size_t>(B) * U;
    BatchArgsT<NSEG, NPTR> a;
    a.nseg          = 0;
    size_t blocks   = 0;
    size_t per      = 0;  // the launch's common block count per bucket, 0: they differ
    auto flush      = [&]() -> int {
        if (a.nseg == 0) return KF_OK;
        a.blk0[a.nseg] = static_cast<unsigned>(blocks);
        a.serial       = KC == 0 && blocks >= kBatchSerialMinBlocks ? 1 : 0;
        // equal block counts: one grid row per bucket (the kernel reads the
        // bucket off blockIdx.y instead of searching blk0)
        const dim3 grid = per && a.nseg > 1
                              ? dim3(static_cast<unsigned>(per), static_cast<unsigned>(a.nseg))
                              : dim3(static_cast<unsigned>(blocks));
        reduce_batch_kernel<T, OP, EPI, KC, B, U, NSEG, NPTR><<<grid, B, 0, s>>>(a, k, np);
        a.nseg = 0;
        blocks = 0;
        per    = 0;
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "reduce batch kernel launch");
        return KF_OK;
    };
    for (int b = 0; b < nb; ++b) {
        const size_t n = counts[b];
        if (n == 0) continue;
        const void *const *ptrs = in + static_cast<size_t>(b) * k;
        const Plan p            = make_plan(ptrs, k, outs[b], n, sizeof(S));
        if (!p.vec_ok) {  // residues differ: this bucket gets a launch of its own
            int rc = launch_typed<T, OP, EPI>(ptrs, k, outs[b], n, npi, s, 0);
            if (rc != KF_OK) return rc;
            continue;
        }
        const size_t nedge = p.head + (n - p.head - p.nvec * V);
        size_t nblk        = (p.nvec + tile - 1) / tile;
        const size_t eblk  = (nedge + B - 1) / B;
        if (nblk > static_cast<size_t>(geometry().grid_cap)) nblk = geometry().grid_cap;
        if (nblk < eblk) nblk = eblk;
        if (nblk < 1) nblk = 1;
        if (blocks + nblk > 0xffffffffu) {
            int rc = flush();
            if (rc != KF_OK) return rc;
        }
        const int j = a.nseg;
        for (int i = 0; i < NPTR; ++i) a.in[j][i] = i < k ? ptrs[i] : nullptr;
        a.out[j]  = outs[b];
        a.n[j]    = n;
        a.head[j] = p.head;
        a.nvec[j] = p.nvec;
        a.blk0[j] = static_cast<unsigned>(blocks);
        per       = j == 0 ? nblk : (per == nblk ? per : 0);
        blocks += nblk;
        ++a.nseg;
        if (a.nseg == NSEG) {
            int rc = flush();
            if (rc != KF_OK) return rc;
        }
    }
    return flush();
}

template <typename T, int OP, int EPI>
int launch_batch(const void *const *in, int k, void *const *outs, const size_t *counts, int nb,
                 int npi, hipStream_t s)
{
    const Div np = make_div(npi);
    if (k == 1) return launch_batch_kc<T, OP, EPI, 1, KF_BATCH_UNROLL_K1>(in, k, outs, counts, nb, np, npi, s);
    if (k == 2) return launch_batch_kc<T, OP, EPI, 2, KF_BATCH_UNROLL>(in, k, outs, counts, nb, np, npi, s);
    return launch_batch_kc<T, OP, EPI, 0, KF_BATCH_UNROLL>(in, k, outs, counts, nb, np, npi, s);
}

int dispatch_batch(const void *const *in, int k, void *const *outs, const size_t *counts, int nb,
                   KungFu_Datatype dt, int np, hipStream_t s)
{
    // SUM only (plain for every dtype, / np for the float types)
    if (np > 0) {
        switch (dt) {
        case KungFu_FLOAT16: return launch_batch<f16_t, OP_SUM, EPI_DIV>(in, k, outs, counts, nb, np, s);
        case KungFu_FLOAT: return launch_batch<float, OP_SUM, EPI_DIV>(in, k, outs, counts, nb, np, s);
        case KungFu_DOUBLE: return launch_batch<double, OP_SUM, EPI_DIV>(in, k, outs, counts, nb, np, s);
        case KungFu_BFLOAT16: return launch_batch<bf16_t, OP_SUM, EPI_DIV>(in, k, outs, counts, nb, np, s);
        default: return KF_ERR_DTYPE;
        }
    }
    switch (dt) {
    case KungFu_UINT8: return launch_batch<uint8_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_UINT16: return launch_batch<uint16_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_UINT32: return launch_batch<uint32_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_UINT64: return launch_batch<uint64_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_INT8: return launch_batch<int8_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_INT16: return launch_batch<int16_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_INT32: return launch_batch<int32_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_INT64: return launch_batch<int64_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_FLOAT16: return launch_batch<f16_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_FLOAT: return launch_batch<float, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_DOUBLE: return launch_batch<double, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    case KungFu_BFLOAT16: return launch_batch<bf16_t, OP_SUM, EPI_NONE>(in, k, outs, counts, nb, 1, s);
    default: return KF_ERR_DTYPE;
    }
}

template <typename T, typename C>
int launch_sma(void *v, const void *sum, size_t n, int np, C c1, C c2,
               hipStream_t s)
{
    using S              = typename SmaMath<T>::S;
    const void *ins[1]   = {sum};
    const Plan p         = make_plan(ins, 1, v, n, sizeof(S));
    constexpr int V      = Vec<S>::N;
    size_t blocks;
    if (p.vec_ok) {
        const size_t ned = p.head + (n - p.head - p.nvec * V);
        blocks           = grid_for(p.nvec, ned, 4);
    } else {
        blocks = (n + kBlock - 1) / kBlock;
        if (blocks > 8192) blocks = 8192;
    }
    sma_kernel<T, C, kBlock, 4><<<static_cast<unsigned>(blocks), kBlock, occ_lds(1, blocks), s>>>(
        v, sum, n, p.head, p.nvec, c1, c2, make_div(np), p.vec_ok ? 1 : 0);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "sma kernel launch");
    return KF_OK;
}

// nb variable buckets in one launch per kBatchSeg of them (kf_sma_blend_batch)
template <typename T, typename C>
int launch_sma_batch(void *const *vs, const void *const *sums, const size_t *counts, int nb,
                     int np, C c1, C c2, hipStream_t s)
{
    using S         = typename SmaMath<T>::S;
    constexpr int V = Vec<S>::N;
    const Div dv    = make_div(np);
    SmaBatchArgs<C> a;
    a.nseg        = 0;
    a.c1          = c1;
    a.c2          = c2;
    size_t blocks = 0;
    auto flush    = [&]() -> int {
        if (a.nseg == 0) return KF_OK;
        a.blk0[a.nseg] = static_cast<unsigned>(blocks);
        sma_batch_kernel<T, C, kBlock, 4><<<static_cast<unsigned>(blocks), kBlock, 0, s>>>(a, dv);
        a.nseg = 0;
        blocks = 0;
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "sma batch kernel launch");
        return KF_OK;
    };
    // Buckets that sit back to back in v AND in the sums (GradBuckets' flat
    // layout with a flat sum workspace, collective.workspace_like) blend as
    // ONE range: one tile grid with no ragged edge and no bucket search per
    // bucket. Element-wise, so the bits are the per-bucket blend's.
    struct Run {
        void *v;
        const void *s;
        size_t n;
    };
    std::vector<Run> runs;
    for (int b = 0; b < nb; ++b) {
        if (counts[b] == 0) continue;
        if (!runs.empty()) {
            Run &r = runs.back();
            if (static_cast<char *>(r.v) + r.n * sizeof(S) == vs[b] &&
                static_cast<const char *>(r.s) + r.n * sizeof(S) == sums[b]) {
                r.n += counts[b];
                continue;
            }
        }
        runs.push_back(Run{vs[b], sums[b], counts[b]});
    }
    for (const Run &run : runs) {
        const size_t n     = run.n;
        const void *ins[1] = {run.s};
        const Plan p       = make_plan(ins, 1, run.v, n, sizeof(S));
        size_t nblk;
        if (p.vec_ok) {
            const size_t ned = p.head + (n - p.head - p.nvec * V);
            nblk             = grid_for(p.nvec, ned, 4);
        } else {
            nblk = (n + kBlock - 1) / kBlock;
            if (nblk > 8192) nblk = 8192;
        }
        if (blocks + nblk > 0xffffffffu) {
            int rc = flush();
            if (rc != KF_OK) return rc;
        }
        const int j = a.nseg;
        a.v[j]      = run.v;
        a.s[j]      = run.s;
        a.n[j]      = n;
        a.head[j]   = p.head;
        a.nvec[j]   = p.nvec;
        a.vec_ok[j] = p.vec_ok ? 1 : 0;
        a.blk0[j]   = static_cast<unsigned>(blocks);
        blocks += nblk;
        if (++a.nseg == kBatchSeg) {
            int rc = flush();
            if (rc != KF_OK) return rc;
        }
    }
    return flush();
}

// ---------------------------------------------------------------------------
// B1 support: host pointers
// ---------------------------------------------------------------------------
// Page-locked host memory is mapped into the GPU's address space, so when x, y
// and out are all device-accessible (page-locked host or HBM) the reduce
// kernel reads and writes them in place over PCIe: one launch, no copies.
// Measured on MI355X (tools/explore/zc_explore.hip, profiles/r01/zc.jsonl):
// 256 MiB fp32 9.39 ms (the H2D bound for 512 MiB at 57.6 GB/s is 9.3 ms)
// against 10.49 ms for 16 MiB chunks staged through HBM on two streams, and
// 59 us against 104 us for a 1 MiB chunk (the reference's chunk size). The
// link is the bound, so a small grid is enough and leaves the rest of the
// chip free: `kHostGrid` blocks (32 or 64 measured best of 32..4096:
// 9.47-9.49 ms per 256 MiB, 61 us per 1 MiB at 32; profiles/r01/zc_grid.txt).
constexpr int kHostGrid = 32;

int host_grid()
{
    static const int g = [] {
        const char *e = std::getenv("KUNGFU_AMD_HOST_GRID");  // tuning only
        const int v   = e ? std::atoi(e) : 0;
        return v > 0 ? v : kHostGrid;
    }();
    return g;
}

// Stream + HBM scratch for pageable buffers, lent to one host-API call at a
// time (std_transform_2 is called from many threads at once, session.go:317-
// 323). No destructor releases them: a hipFree / hipStreamDestroy that runs
// after main returns (a thread_local or static destructor) can reach a HIP
// runtime that is already torn down. kf_shutdown() frees the idle ones while
// the runtime is alive; whatever is left is the OS's at exit.
struct Staging {
    hipStream_t s = nullptr;
    void *dev     = nullptr;  // 3 regions: x | y | z
    size_t cap    = 0;        // bytes per region
    void *bounce  = nullptr;  // page-locked, one region: for mixed host ranges
    size_t bcap   = 0;

    void release()
    {
        if (dev) (void)hipFree(dev);
        if (bounce) (void)hipHostFree(bounce);
        if (s) (void)hipStreamDestroy(s);
        dev    = nullptr;
        bounce = nullptr;
        s      = nullptr;
        cap    = 0;
        bcap   = 0;
    }

    int ensure_bounce(size_t bytes)
    {
        if (bytes <= bcap) return KF_OK;
        if (bounce) KF_HIP(hipHostFree(bounce));
        bounce = nullptr;
        bcap   = 0;
        KF_HIP(hipHostMalloc(&bounce, bytes, hipHostMallocDefault));
        bcap = bytes;
        return KF_OK;
    }

    int ensure_stream()
    {
        if (s) return KF_OK;
        int cnt = 0;
        if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0) {
            t_last_error = "no HIP device";
            return KF_ERR_NO_DEVICE;
        }
        KF_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        return KF_OK;
    }

    int ensure(size_t bytes)
    {
        int rc = ensure_stream();
        if (rc != KF_OK) return rc;
        if (bytes > cap) {
            if (dev) KF_HIP(hipFree(dev));
            dev            = nullptr;
            cap            = 0;
            size_t rounded = (bytes + 255) & ~static_cast<size_t>(255);
            KF_HIP(hipMalloc(&dev, 3 * rounded));
            cap = rounded;
        }
        return KF_OK;
    }
};

struct StagingPool {
    std::mutex mu;
    std::vector<Staging *> idle;
    size_t lent = 0;
};

// never destroyed (see Staging)
StagingPool &staging_pool()
{
    static StagingPool *p = new StagingPool;
    return *p;
}

// one call's Staging, back to the pool at the end of the call
class StagingLease
{
  public:
    StagingLease()
    {
        StagingPool &p = staging_pool();
        std::lock_guard<std::mutex> l(p.mu);
        if (!p.idle.empty()) {
            st_ = p.idle.back();
            p.idle.pop_back();
        } else {
            st_ = new Staging;
        }
        ++p.lent;
    }
    ~StagingLease()
    {
        StagingPool &p = staging_pool();
        std::lock_guard<std::mutex> l(p.mu);
        p.idle.push_back(st_);
        --p.lent;
    }
    StagingLease(const StagingLease &)            = delete;
    StagingLease &operator=(const StagingLease &) = delete;
    Staging &operator*() const { return *st_; }

  private:
    Staging *st_;
};

// Host ranges page-locked through kf_host_register, with the address a kernel
// uses for each: std_transform_2 finds a chunk of one of them with one lookup
// under a shared lock instead of two hipPointerGetAttributes per buffer. (The
// six queries take 0.34 us together, tools/explore/b1_floor.hip: the call's
// cost is the GPU round trip) Only ranges the library
// registered itself are remembered, and kf_host_unregister forgets them, so a
// lookup is never stale as long as the host releases them through it (not
// through hipHostUnregister). Never destroyed (see Staging).
struct Registered {
    size_t bytes;
    char *dev;
};
struct Registry {
    std::shared_mutex mu;
    std::map<uintptr_t, Registered> ranges;  // base -> range
};
Registry &registry()
{
    static Registry *r = new Registry;
    return *r;
}

// 1 with *dev set if [p, p + bytes) lies in one registered range; -1 if it
// overlaps a registered range without lying inside it (page-locked in part);
// 0 if it overlaps none
int registered(const void *p, size_t bytes, const void **dev)
{
    Registry &r = registry();
    std::shared_lock<std::shared_mutex> l(r.mu);
    if (r.ranges.empty()) return 0;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto it           = r.ranges.upper_bound(a);
    // a registered range starting inside [a, a + bytes)
    const bool later = it != r.ranges.end() && it->first < a + bytes;
    if (it == r.ranges.begin()) return later ? -1 : 0;
    --it;
    const uintptr_t end = it->first + it->second.bytes;
    if (a >= end) return later ? -1 : 0;
    if (a + bytes > end) return -1;
    *dev = it->second.dev + (a - it->first);
    return 1;
}

// Where a host-API pointer lives: 0 pageable (or unknown to HIP), 1 page-locked
// host memory (hipHostMalloc / kf_host_register), 2 device memory, 3 a host
// range that is page-locked only in part (e.g. a chunk running past the end
// of a registered pool): HIP's own copies refuse those ("invalid argument",
// profiles/r06/partial_register_r06i.txt), so they go through a page-locked
// bounce buffer. `dev` is the address a kernel uses for kinds 1 and 2.
constexpr int kMixed = 3;

int host_kind(const void *p, hipPointerAttribute_t *a)
{
    if (hipPointerGetAttributes(a, p) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return a->type == hipMemoryTypeHost ? 1 : a->type == hipMemoryTypeDevice ? 2 : 0;
}

int classify(const void *p, size_t bytes, const void **dev)
{
    const int reg = registered(p, bytes, dev);
    if (reg == 1) return 1;
    if (reg < 0) return kMixed;  // straddles the edge of a kf_host_register range
    hipPointerAttribute_t a, b;
    const int kind   = host_kind(p, &a);
    const void *last = static_cast<const char *>(p) + bytes - 1;
    const int klast  = host_kind(last, &b);
    if (kind != 2 && klast != 2 && (kind == 1) != (klast == 1)) return kMixed;
    if (kind == 0 || !a.devicePointer) return 0;
    if (b.type != a.type) return 0;
    // page-locked at both ends but through two registrations whose device
    // addresses are not one run: no single pointer covers it
    if (kind == 1 && static_cast<const char *>(b.devicePointer) !=
                         static_cast<const char *>(a.devicePointer) + (bytes - 1))
        return kMixed;
    if (kind == 2) {  // HBM of another GPU: leave it to the runtime's copies
        int cur = -1;
        if (hipGetDevice(&cur) != hipSuccess || cur != a.device) return 0;
    }
    *dev = a.devicePointer;
    return kind;
}

// Host pointers -> reduce -> host. Synchronous.
//  * all three device-accessible: the kernel works on them in place (zero
//    copy; over PCIe for page-locked host memory, at the link's rate);
//  * otherwise: whole-buffer copies through the runtime's staging to HBM
//    scratch, the kernel, and a copy back.
int transform2_host(const void *x, const void *y, void *out, size_t n,
                    KungFu_Datatype dt, KungFu_Op op)
{
    const int sz = type_size(dt);
    if (sz == 0 || dt == KungFu_BOOL) return KF_ERR_DTYPE;
    if (n == 0) return KF_OK;
    const size_t bytes = n * static_cast<size_t>(sz);
    StagingLease lease;
    Staging &st = *lease;
    const void *gx = nullptr, *gy = nullptr, *gz = nullptr;
    const int kx = classify(x, bytes, &gx);
    const int ky = classify(y, bytes, &gy);
    const int kz = classify(out, bytes, &gz);
    const auto direct = [](int k) { return k == 1 || k == 2; };
    if (direct(kx) && direct(ky) && direct(kz)) {
        int rc = st.ensure_stream();
        if (rc != KF_OK) return rc;
        const bool host_link = kx == 1 || ky == 1 || kz == 1;
        const void *ins[2]   = {gx, gy};
        rc = dispatch_none(ins, 2, const_cast<void *>(gz), n, dt, op, st.s,
                           host_link ? host_grid() : 0);
        if (rc != KF_OK) return rc;
        KF_HIP(hipStreamSynchronize(st.s));
        return KF_OK;
    }
    int rc = st.ensure(bytes);
    if (rc != KF_OK) return rc;
    char *dx = static_cast<char *>(st.dev);
    char *dy = dx + st.cap;
    char *dz = dy + st.cap;
    // a mixed range is copied through the bounce buffer one at a time (the
    // CPU copy, then the DMA, then a sync before the bounce is reused)
    auto h2d = [&](char *dst, const void *src, int kind) -> int {
        if (kind != kMixed) {
            KF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st.s));
            return KF_OK;
        }
        int r = st.ensure_bounce(bytes);
        if (r != KF_OK) return r;
        KF_HIP(hipStreamSynchronize(st.s));
        std::memcpy(st.bounce, src, bytes);
        KF_HIP(hipMemcpyAsync(dst, st.bounce, bytes, hipMemcpyHostToDevice, st.s));
        return KF_OK;
    };
    rc = h2d(dx, x, kx);
    if (rc == KF_OK) rc = h2d(dy, y, ky);
    if (rc != KF_OK) return rc;
    const void *ins[2] = {dx, dy};
    rc                 = dispatch_none(ins, 2, dz, n, dt, op, st.s);
    if (rc != KF_OK) return rc;
    if (kz == kMixed) {
        rc = st.ensure_bounce(bytes);
        if (rc != KF_OK) return rc;
        KF_HIP(hipMemcpyAsync(st.bounce, dz, bytes, hipMemcpyDeviceToHost, st.s));
        KF_HIP(hipStreamSynchronize(st.s));
        std::memcpy(out, st.bounce, bytes);
        return KF_OK;
    }
    KF_HIP(hipMemcpyAsync(out, dz, bytes, hipMemcpyDeviceToHost, st.s));
    KF_HIP(hipStreamSynchronize(st.s));
    return KF_OK;
}

[[noreturn]] void die(const char *fn, int rc)
{
    std::fprintf(stderr, "kungfu_amd: %s failed (status %d): %s\n", fn, rc,
                 t_last_error.c_str());
    std::exit(1);
}

}  // namespace

extern "C" {

uint32_t kungfu_type_size(KungFu_Datatype dt)
{
    const int sz = type_size(dt);
    if (sz == 0) {
        std::fprintf(stderr, "unknown dtype: %d\n", static_cast<int>(dt));
        std::exit(1);
    }
    return static_cast<uint32_t>(sz);
}

void std_transform_2(const void *input1, const void *input2, void *output,
                     const int n, const KungFu_Datatype dt, const KungFu_Op o)
{
    if (n <= 0) return;  // std::transform over an empty range
    const int rc = transform2_host(input1, input2, output,
                                   static_cast<size_t>(n), dt, o);
    if (rc != KF_OK) die("std_transform_2", rc);
}

void float16_sum(void *z, const void *x, const void *y, int len)
{
    if (len <= 0) return;
    const int rc = transform2_host(x, y, z, static_cast<size_t>(len),
                                   KungFu_FLOAT16, KungFu_SUM);
    if (rc != KF_OK) die("float16_sum", rc);
}

int kf_bucket_reduce(const void *const *inputs, int k, void *out, size_t n,
                     KungFu_Datatype dt, KungFu_Op op, void *stream)
{
    int rc = check_args(inputs, k, out, n);
    if (rc != KF_OK || n == 0) return rc;
    const int sz = type_size(dt);
    if (sz == 0 || dt == KungFu_BOOL) return KF_ERR_DTYPE;
    if (op < KungFu_SUM || op > KungFu_PROD) return KF_ERR_OP;
    if (dt == KungFu_FLOAT16 && op != KungFu_SUM) return KF_ERR_OP;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (k == 1) {
        if (out != inputs[0]) {
            KF_HIP(hipMemcpyAsync(out, inputs[0], n * sz, hipMemcpyDeviceToDevice, s));
        }
        return KF_OK;
    }
    return dispatch_none(inputs, k, out, n, dt, op, s);
}

int kf_bucket_reduce_avg(const void *const *inputs, int k, void *out, size_t n,
                         KungFu_Datatype dt, int np, void *stream)
{
    int rc = check_args(inputs, k, out, n);
    if (rc != KF_OK || n == 0) return rc;
    if (!is_float(dt)) return KF_ERR_DTYPE;
    if (np < 1) return KF_ERR_ARG;
    return dispatch_div(inputs, k, out, n, dt, np, static_cast<hipStream_t>(stream));
}

int kf_bucket_div(void *x, size_t n, KungFu_Datatype dt, int np, void *stream)
{
    if (n == 0) return KF_OK;
    if (!x) return KF_ERR_ARG;
    if (!is_float(dt)) return KF_ERR_DTYPE;
    if (np < 1) return KF_ERR_ARG;
    const void *ins[1] = {x};
    return dispatch_div(ins, 1, x, n, dt, np, static_cast<hipStream_t>(stream));
}

int kf_sma_blend(void *v, const void *sum, size_t n, KungFu_Datatype dt, int np,
                 double alpha, void *stream)
{
    if (n == 0) return KF_OK;
    if (!v || !sum) return KF_ERR_ARG;
    if (np < 1) return KF_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // TF converts the Python constants (1 - alpha) and alpha to the tensor
    // dtype after computing them in double (sma_sgd.py:64-65).
    const float c1f = static_cast<float>(1.0 - alpha);
    const float c2f = static_cast<float>(alpha);
    switch (dt) {
    case KungFu_FLOAT: return launch_sma<float, float>(v, sum, n, np, c1f, c2f, s);
    case KungFu_DOUBLE: return launch_sma<double, double>(v, sum, n, np, 1.0 - alpha, alpha, s);
    case KungFu_FLOAT16: return launch_sma<f16_t, float>(v, sum, n, np, c1f, c2f, s);
    case KungFu_BFLOAT16: return launch_sma<bf16_t, float>(v, sum, n, np, c1f, c2f, s);
    default: return KF_ERR_DTYPE;
    }
}

int kf_sma_blend_batch(void *const *vs, const void *const *sums, const size_t *counts, int nb,
                       KungFu_Datatype dt, int np, double alpha, void *stream)
{
    if (nb < 0 || (nb > 0 && (!vs || !sums || !counts))) return KF_ERR_ARG;
    if (np < 1) return KF_ERR_ARG;
    for (int b = 0; b < nb; ++b) {
        if (counts[b] && (!vs[b] || !sums[b])) return KF_ERR_ARG;
    }
    if (nb == 0) return KF_OK;
    hipStream_t s   = static_cast<hipStream_t>(stream);
    const float c1f = static_cast<float>(1.0 - alpha);  // as kf_sma_blend
    const float c2f = static_cast<float>(alpha);
    switch (dt) {
    case KungFu_FLOAT: return launch_sma_batch<float, float>(vs, sums, counts, nb, np, c1f, c2f, s);
    case KungFu_DOUBLE:
        return launch_sma_batch<double, double>(vs, sums, counts, nb, np, 1.0 - alpha, alpha, s);
    case KungFu_FLOAT16: return launch_sma_batch<f16_t, float>(vs, sums, counts, nb, np, c1f, c2f, s);
    case KungFu_BFLOAT16: return launch_sma_batch<bf16_t, float>(vs, sums, counts, nb, np, c1f, c2f, s);
    default: return KF_ERR_DTYPE;
    }
}

int kf_bucket_reduce_peers(const void *const *inputs, int k, void *out, size_t n,
                           KungFu_Datatype dt, KungFu_Op op, int np, void *stream)
{
    int rc = check_args(inputs, k, out, n);
    if (rc != KF_OK || n == 0) return rc;
    const int sz = type_size(dt);
    if (sz == 0 || dt == KungFu_BOOL) return KF_ERR_DTYPE;
    if (np < 0) return KF_ERR_ARG;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (np > 0) {  // average: SUM then / np
        if (!is_float(dt)) return KF_ERR_DTYPE;
        if (op != KungFu_SUM) return KF_ERR_OP;
        return dispatch_div(inputs, k, out, n, dt, np, s, LM_SPREAD);
    }
    if (op < KungFu_SUM || op > KungFu_PROD) return KF_ERR_OP;
    if (dt == KungFu_FLOAT16 && op != KungFu_SUM) return KF_ERR_OP;
    if (k == 1) {
        if (out != inputs[0]) KF_HIP(hipMemcpyAsync(out, inputs[0], n * sz, hipMemcpyDefault, s));
        return KF_OK;
    }
    return dispatch_none(inputs, k, out, n, dt, op, s, 0, LM_SPREAD);
}

int kf_bucket_reduce_batch(const void *const *inputs, int k, void *const *outs,
                           const size_t *counts, int nb, KungFu_Datatype dt, KungFu_Op op,
                           int np, void *stream)
{
    if (nb < 0 || k < 1 || k > KF_MAX_INPUTS || np < 0) return KF_ERR_ARG;
    if (nb == 0) return KF_OK;
    if (!inputs || !outs || !counts) return KF_ERR_ARG;
    const int sz = type_size(dt);
    if (sz == 0 || dt == KungFu_BOOL) return KF_ERR_DTYPE;
    if (op < KungFu_SUM || op > KungFu_PROD) return KF_ERR_OP;
    if ((dt == KungFu_FLOAT16 || np > 0) && op != KungFu_SUM) return KF_ERR_OP;
    if (np > 0 && !is_float(dt)) return KF_ERR_DTYPE;
    for (int b = 0; b < nb; ++b) {
        if (counts[b] == 0) continue;
        int rc = check_args(inputs + static_cast<size_t>(b) * k, k, outs[b], counts[b]);
        if (rc != KF_OK) return rc;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (k == 1 && np == 0) {  // a copy per bucket, as kf_bucket_reduce
        for (int b = 0; b < nb; ++b) {
            if (counts[b] && outs[b] != inputs[b]) {
                KF_HIP(hipMemcpyAsync(outs[b], inputs[b], counts[b] * sz, hipMemcpyDeviceToDevice, s));
            }
        }
        return KF_OK;
    }
    if (op != KungFu_SUM) {  // MIN / MAX / PROD: one launch per bucket
        for (int b = 0; b < nb; ++b) {
            if (counts[b] == 0) continue;
            int rc = dispatch_none(inputs + static_cast<size_t>(b) * k, k, outs[b], counts[b], dt,
                                   op, s);
            if (rc != KF_OK) return rc;
        }
        return KF_OK;
    }
    return dispatch_batch(inputs, k, outs, counts, nb, dt, np, s);
}

int kf_set_geometry(int unroll, int grid_cap, int loadnt, int stplain)
{
    if (unroll != 1 && unroll != 2 && unroll != 4 && unroll != 8) return KF_ERR_ARG;
    if (grid_cap < 1) return KF_ERR_ARG;
    Geometry &g = geometry();
    g.unroll    = unroll;
    g.grid_cap  = grid_cap;
    g.loadnt    = loadnt ? 1 : 0;
    g.stplain   = stplain ? 1 : 0;
    return KF_OK;
}

int kf_set_occupancy(int lds_small, int lds_fold)
{
    if (lds_small < 0 || lds_fold < 0 || lds_small > (64 << 10) || lds_fold > (64 << 10)) {
        return KF_ERR_ARG;
    }
    Geometry &g = geometry();
    g.occ_small = lds_small;
    g.occ_fold  = lds_fold;
    return KF_OK;
}

int kf_host_register(void *p, size_t bytes)
{
    if (!p || bytes == 0) return KF_ERR_ARG;
    KF_HIP(hipHostRegister(p, bytes, hipHostRegisterDefault));
    void *dev = nullptr;
    if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess || !dev) {
        (void)hipGetLastError();
        return KF_OK;  // still page-locked; classify() asks HIP per call
    }
    Registry &r = registry();
    std::unique_lock<std::shared_mutex> l(r.mu);
    r.ranges[reinterpret_cast<uintptr_t>(p)] = Registered{bytes, static_cast<char *>(dev)};
    return KF_OK;
}

int kf_host_unregister(void *p)
{
    if (!p) return KF_ERR_ARG;
    {
        Registry &r = registry();
        std::unique_lock<std::shared_mutex> l(r.mu);
        r.ranges.erase(reinterpret_cast<uintptr_t>(p));
    }
    KF_HIP(hipHostUnregister(p));
    return KF_OK;
}

int kf_device_count(void)
{
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess) return 0;
    return cnt;
}

const char *kf_version(void) { return "kungfu_amd 0.1.0 (gfx950)"; }

const char *kf_last_error(void) { return t_last_error.c_str(); }

int kf_shutdown(void)
{
    StagingPool &p = staging_pool();
    std::lock_guard<std::mutex> l(p.mu);
    for (Staging *st : p.idle) {
        st->release();
        delete st;
    }
    p.idle.clear();
    if (p.lent != 0) {
        t_last_error = "kf_shutdown: " + std::to_string(p.lent) + " host-API call(s) still running";
        return KF_ERR_ARG;
    }
    return KF_OK;
}

int kf_transform2_host(const void *x, const void *y, void *out, size_t n,
                       KungFu_Datatype dt, KungFu_Op op)
{
    if (n > 0 && (!x || !y || !out)) return KF_ERR_ARG;
    if (dt == KungFu_FLOAT16 && op != KungFu_SUM) return KF_ERR_OP;
    return transform2_host(x, y, out, n, dt, op);
}

}  // extern "C"
