// kf_reduce_kernels.hpp — gfx950 element-wise bucket reduce kernels.
//
// The reduce is a pure streaming element-wise op: (k reads + 1 write) per
// element and at most a handful of VALU instructions, so it is HBM-bound
// (0.083 flop/B for the fp32 2-input sum) and never touches MFMA or LDS.
// What matters on MI355X is keeping enough 16-byte loads in flight per CU:
//   * every lane moves whole 16-B vectors (global_load_dwordx4 /
//     global_store_dwordx4): 1 KiB per wave-instruction, fully coalesced;
//   * loads AND stores are non-temporal: every byte is touched exactly once, so
//     nothing is worth keeping in L2 / Infinity Cache;
//   * each thread issues UNROLL = 4 independent vector loads per input before
//     the first use, and the grid has one 256-thread block per tile of 1024
//     vectors (16,384 blocks for the 256 MiB bucket, no grid-stride), so every
//     CU holds 8 blocks x 32 KiB of loads in flight (DESIGN.md "Kernel tuning").
//
// Numerics follow the reference's host reduce (op.cpp:22-54, f16.c:16-50):
//   SUM/PROD on integers wrap (done in the unsigned type of the same width),
//   MIN/MAX are std::min/std::max as selects ((b < a) ? b : a, (a < b) ? b : a),
//   fp16 SUM = widen, fp32 add, RNE narrow — per hop, as the reference chain,
//   no FMA contraction anywhere (#pragma below and explicit _rn intrinsics).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#pragma clang fp contract(off)

namespace kf
{
enum Op { OP_SUM = 0, OP_MIN = 1, OP_MAX = 2, OP_PROD = 3 };
// EPI_DIV is what the host asks for (the /np epilogue). Inside a kernel it is
// split once, at the top, on the uniform np.pow2: EPI_MUL (x * 2^-k, the same
// correctly rounded value as x / 2^k) or EPI_DIV (a true IEEE division). With
// the choice made per element instead, the fp32 k = 2 kernel carried 66 scalar
// branches and 58 division sequences (663 instructions against 172 without
// the epilogue) and ran at 0.77 of the roofline against 0.82.
enum Epi { EPI_NONE = 0, EPI_DIV = 1, EPI_MUL = 2 };

// The 1/np epilogue divisor. For np a power of two, x * 2^-k and x / 2^k are
// the same correctly rounded value, so the multiply is used (bit-identical,
// no software division); otherwise a true IEEE division (TF's g / np).
struct Div {
    float f, fi;
    double d, di;
    int pow2;
};

// Storage tags for the two 16-bit float formats (stored as raw u16 bits).
struct f16_t {
    uint16_t bits;
};
struct bf16_t {
    uint16_t bits;
};

// IEEE binary16 via the compiler's native _Float16: the widen is exact and the
// narrow is v_cvt_f16_f32 in the default round-to-nearest-even mode.
__device__ __forceinline__ float f16_to_f32(uint16_t h)
{
    return static_cast<float>(__builtin_bit_cast(_Float16, h));
}

__device__ __forceinline__ uint16_t f32_to_f16(float f)
{
    return __builtin_bit_cast(uint16_t, static_cast<_Float16>(f));
}

__device__ __forceinline__ float bf16_to_f32(uint16_t h)
{
    return __uint_as_float(static_cast<uint32_t>(h) << 16);
}

// RNE narrow; a NaN keeps its sign and upper payload and is made quiet. This
// is gfx950's v_cvt_pk_bf16_f32 (clang's float -> __bf16), which equals the
// oracle's bit recipe ((u + 0x7fff + lsb) >> 16; NaN: (u >> 16) | 0x0040) on
// all 2^32 fp32 patterns (tools/explore/bf16_cvt_check.hip, 0 mismatches,
// profiles/r01/bf16_cvt_check.json). The recipe written out in integer ops
// compiled to a divergent branch per element (613 VALU, ~60 exec-mask
// branches in the k = 2 kernel) and ran at 0.79 of the roofline vs 0.81.
__device__ __forceinline__ uint16_t f32_to_bf16(float f)
{
    return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}

// ---------------------------------------------------------------------------
// Per-dtype arithmetic. `Acc` is what the fold carries between hops.
// ---------------------------------------------------------------------------
template <typename T> struct Elt;

template <typename T> struct IntElt {
    using S   = T;  // storage
    using Acc = T;
    using W   = typename std::conditional<(sizeof(T) <= 4), uint32_t,
                                        uint64_t>::type;
    __device__ static Acc load(S s) { return s; }
    __device__ static S store(Acc a) { return a; }
    template <int OP> __device__ static Acc combine(Acc a, S b)
    {
        if constexpr (OP == OP_SUM) {
            return static_cast<T>(static_cast<W>(a) + static_cast<W>(b));
        } else if constexpr (OP == OP_PROD) {
            using U = typename std::make_unsigned<T>::type;
            return static_cast<T>(static_cast<W>(static_cast<U>(a)) *
                                  static_cast<W>(static_cast<U>(b)));
        } else if constexpr (OP == OP_MIN) {
            return (b < a) ? b : a;
        } else {
            return (a < b) ? b : a;
        }
    }
};

template <> struct Elt<uint8_t> : IntElt<uint8_t> {};
template <> struct Elt<uint16_t> : IntElt<uint16_t> {};
template <> struct Elt<uint32_t> : IntElt<uint32_t> {};
template <> struct Elt<uint64_t> : IntElt<uint64_t> {};
template <> struct Elt<int8_t> : IntElt<int8_t> {};
template <> struct Elt<int16_t> : IntElt<int16_t> {};
template <> struct Elt<int32_t> : IntElt<int32_t> {};
template <> struct Elt<int64_t> : IntElt<int64_t> {};

template <> struct Elt<float> {
    using S   = float;
    using Acc = float;
    __device__ static Acc load(S s) { return s; }
    __device__ static S store(Acc a) { return a; }
    template <int OP> __device__ static Acc combine(Acc a, S b)
    {
        if constexpr (OP == OP_SUM) {
            return __fadd_rn(a, b);
        } else if constexpr (OP == OP_PROD) {
            return __fmul_rn(a, b);
        } else if constexpr (OP == OP_MIN) {
            return (b < a) ? b : a;
        } else {
            return (a < b) ? b : a;
        }
    }
    template <bool P2> __device__ static S div(Acc a, const Div &dv)
    {
        return P2 ? __fmul_rn(a, dv.fi) : __fdiv_rn(a, dv.f);
    }
};

template <> struct Elt<double> {
    using S   = double;
    using Acc = double;
    __device__ static Acc load(S s) { return s; }
    __device__ static S store(Acc a) { return a; }
    template <int OP> __device__ static Acc combine(Acc a, S b)
    {
        if constexpr (OP == OP_SUM) {
            return __dadd_rn(a, b);
        } else if constexpr (OP == OP_PROD) {
            return __dmul_rn(a, b);
        } else if constexpr (OP == OP_MIN) {
            return (b < a) ? b : a;
        } else {
            return (a < b) ? b : a;
        }
    }
    template <bool P2> __device__ static S div(Acc a, const Div &dv)
    {
        return P2 ? __dmul_rn(a, dv.di) : __ddiv_rn(a, dv.d);
    }
};

// fp16: the reference chain rounds to fp16 after every Transform2 hop
// (f16.c:16-23), so the accumulator is re-quantised per hop. Only SUM exists
// in the reference (op.cpp:45-54); the host wrapper rejects the other ops.
template <> struct Elt<f16_t> {
    using S   = uint16_t;
    using Acc = uint16_t;
    __device__ static Acc load(S s) { return s; }
    __device__ static S store(Acc a) { return a; }
    template <int OP> __device__ static Acc combine(Acc a, S b)
    {
        static_assert(OP == OP_SUM, "fp16 supports SUM only");
        return f32_to_f16(__fadd_rn(f16_to_f32(a), f16_to_f32(b)));
    }
    template <bool P2> __device__ static S div(Acc a, const Div &dv)
    {
        const float x = f16_to_f32(a);
        return f32_to_f16(P2 ? __fmul_rn(x, dv.fi) : __fdiv_rn(x, dv.f));
    }
};

// bf16 (build-defined, not in the reference): fp32 accumulation, one RNE
// rounding at the end. MIN/MAX select an input and keep its bits.
template <> struct Elt<bf16_t> {
    using S = uint16_t;
    struct Acc {
        float f;
        uint16_t bits;
    };
    __device__ static Acc load(S s) { return Acc{bf16_to_f32(s), s}; }
    __device__ static S store(Acc a) { return a.bits; }
    template <int OP> __device__ static Acc combine(Acc a, S b)
    {
        const float fb = bf16_to_f32(b);
        if constexpr (OP == OP_SUM) {
            return Acc{__fadd_rn(a.f, fb), 0};
        } else if constexpr (OP == OP_PROD) {
            return Acc{__fmul_rn(a.f, fb), 0};
        } else if constexpr (OP == OP_MIN) {
            return (fb < a.f) ? Acc{fb, b} : a;
        } else {
            return (a.f < fb) ? Acc{fb, b} : a;
        }
    }
    template <int OP> __device__ static S finish(Acc a)
    {
        if constexpr (OP == OP_SUM || OP == OP_PROD) {
            return f32_to_bf16(a.f);
        } else {
            return a.bits;
        }
    }
    template <bool P2> __device__ static S div(Acc a, const Div &dv)
    {
        return f32_to_bf16(P2 ? __fmul_rn(a.f, dv.fi) : __fdiv_rn(a.f, dv.f));
    }
};

template <typename T, int OP>
__device__ __forceinline__ typename Elt<T>::S finish(typename Elt<T>::Acc a)
{
    if constexpr (std::is_same<T, bf16_t>::value) {
        return Elt<T>::template finish<OP>(a);
    } else {
        return Elt<T>::store(a);
    }
}

// ---------------------------------------------------------------------------
// Vector-path lanes. A lane is one element of the 16-B vector, except for the
// 8-bit integers, whose lanes are 32-bit words of 4 packed bytes: split into
// bytes, the compiler re-types the 16-B load as <16 x i8> and drops its nt
// bit (seen in the gfx950 ISA), and the byte-wise adds cost ~3x the VALU of a
// packed word. Results are the same bytes as Elt<T> element by element.
// ---------------------------------------------------------------------------
template <typename T, typename = void> struct Lane {
    using W   = typename Elt<T>::S;
    using Acc = typename Elt<T>::Acc;
    __device__ static Acc load(W w) { return Elt<T>::load(w); }
    template <int OP> __device__ static Acc combine(Acc a, W b)
    {
        return Elt<T>::template combine<OP>(a, b);
    }
    template <int OP, int EPI> __device__ static W emit(const Acc &a, const Div &np)
    {
        if constexpr (EPI == EPI_DIV || EPI == EPI_MUL) {
            return Elt<T>::template div<EPI == EPI_MUL>(a, np);
        } else {
            return finish<T, OP>(a);
        }
    }
};

template <typename T>
struct Lane<T, typename std::enable_if<std::is_integral<T>::value && sizeof(T) == 1>::type> {
    using W   = uint32_t;
    using Acc = uint32_t;
    __device__ static Acc load(W w) { return w; }
    template <int OP> __device__ static Acc combine(Acc a, W b)
    {
        if constexpr (OP == OP_SUM) {
            // per-byte add mod 2^8: low 7 bits add without crossing a byte,
            // the top bit of each byte is the xor of the inputs' and the carry
            return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
        } else {
            uint32_t r = 0;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const T x = static_cast<T>(a >> (8 * i));
                const T y = static_cast<T>(b >> (8 * i));
                const T z = Elt<T>::template combine<OP>(x, y);
                r |= static_cast<uint32_t>(static_cast<uint8_t>(z)) << (8 * i);
            }
            return r;
        }
    }
    template <int OP, int EPI> __device__ static W emit(const Acc &a, const Div &)
    {
        static_assert(EPI == EPI_NONE, "8-bit integers have no /np epilogue");
        return a;
    }
};

// ---------------------------------------------------------------------------
// Kernel arguments.
// ---------------------------------------------------------------------------
constexpr int kMaxInputs = 16;

struct InPtrs {
    const void *p[kMaxInputs];
};

// 16-byte vector of storage elements.
template <typename S> struct Vec {
    static constexpr int N = 16 / sizeof(S);
    S e[N];
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Load policy: LOADNT=1 marks the read streams non-temporal (each byte is read
// once); chosen by measurement (tools/tune_reduce.py), see DESIGN.md.
template <int LOADNT>
__device__ __forceinline__ u32x4 ld_u4(const void *base, size_t vi)
{
    const u32x4 *p = reinterpret_cast<const u32x4 *>(base) + vi;
    if constexpr (LOADNT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <typename S, int LOADNT>
__device__ __forceinline__ Vec<S> ld_vec(const void *base, size_t vi)
{
    const u32x4 *p = reinterpret_cast<const u32x4 *>(base) + vi;
    u32x4 raw;
    if constexpr (LOADNT) {
        raw = __builtin_nontemporal_load(p);
    } else {
        raw = *p;
    }
    Vec<S> v;
    __builtin_memcpy(&v, &raw, 16);
    return v;
}

// Store policy: STPLAIN=0 (default) writes non-temporally — the output is not
// re-read by this kernel; STPLAIN=1 uses plain stores (tuning variant).
// One 16-B non-temporal load that completes before the next statement: the
// load and the wait are inline asm, and the wait redefines the loaded
// registers, so the compiler can neither hoist later loads above it nor use
// the data early. The runtime-k fold reads inputs 2..k-1 this way, one vector
// in flight per lane: with fewer requests outstanding chip-wide the DRAM
// serves the k + 1 streams better — k = 3/4/6/8 at 0.803/0.806/0.805/0.801 of
// 8 TB/s (five blocks per CU) against 0.787/0.779/0.768/0.760 with all four
// vectors of an input in flight (tools/explore/kfold_mlp.hip,
// profiles/r02/kfold_mlp_asm.jsonl). Bit-identical: the adds keep their order.
template <typename S>
__device__ __forceinline__ Vec<S> ld_vec_serial(const void *base, size_t vi)
{
    const u32x4 *p = reinterpret_cast<const u32x4 *>(base) + vi;
    u32x4 raw;
    // ONE statement: no compiler-placed read or copy of `raw` can fall
    // between the load and its wait (early-clobber: raw never shares the
    // address registers)
    asm volatile("global_load_dwordx4 %0, %1, off nt\n\ts_waitcnt vmcnt(0)"
                 : "=&v"(raw)
                 : "v"(p));
    Vec<S> v;
    __builtin_memcpy(&v, &raw, 16);
    return v;
}

template <typename S, int STPLAIN = 0>
__device__ __forceinline__ void st_vec(void *base, size_t vi, const Vec<S> &v)
{
    u32x4 raw;
    __builtin_memcpy(&raw, &v, 16);
    u32x4 *p = reinterpret_cast<u32x4 *>(base) + vi;
    if constexpr (STPLAIN) {
        *p = raw;
    } else {
        __builtin_nontemporal_store(raw, p);
    }
}

// Fold one element across the k inputs (runtime k).
template <typename T, int OP, int EPI>
__device__ __forceinline__ typename Elt<T>::S
fold_scalar(const InPtrs &in, int k, size_t i, const Div &np)
{
    using S   = typename Elt<T>::S;
    auto acc  = Elt<T>::load(reinterpret_cast<const S *>(in.p[0])[i]);
    for (int j = 1; j < k; ++j) {
        acc = Elt<T>::template combine<OP>(
            acc, reinterpret_cast<const S *>(in.p[j])[i]);
    }
    if constexpr (EPI == EPI_DIV || EPI == EPI_MUL) {
        return Elt<T>::template div<EPI == EPI_MUL>(acc, np);
    } else {
        return finish<T, OP>(acc);
    }
}

// ---------------------------------------------------------------------------
// Main kernel. Elements [0, head) and [head + nvec*V, n) are done one element
// per thread; [head, head + nvec*V) as 16-B vectors (all pointers offset by
// `head` elements are 16-B aligned; the host checks this). KC = compile-time
// input count (2 for the hot path) or 0 = runtime k (pointers are then read
// from the kernel-argument block with scalar loads, never a local array).
// ---------------------------------------------------------------------------
// The body of one block, `blk` of `nblk` working on one bucket: reduce_kernel
// runs it with (blockIdx.x, gridDim.x); the batch kernel below with the block's
// index inside its bucket's share of the grid.
// KF_REDUCE_SCHED: a scheduling barrier after the compile-time-k full tile's
// loads, as for the SMA blend (KF_SMA_SCHED below). Left to itself the
// compiler split several k = 2 instantiations' eight loads around a wait
// (7 + 1 for fp16 and integer sums, 4 + 4 for bf16 min/max, 6 + 2 for the
// bf16 average batch) and spread the waits of the rest over the adds. With
// the barrier, in one process on the same 256 MiB buffers
// (tools/ab_reduce_sched.py, profiles/r06/ab_reduce_sched_r06s.jsonl), same
// bits: C2's fp32 sum 0.824 / 0.823 (unchanged), bf16 sum 0.816 -> 0.824,
// fp16 0.813 -> 0.826, i32 0.805 -> 0.822, bf16 max 0.799 -> 0.820, fp32 min
// 0.807 -> 0.822, (x + y) / 3 fp32 0.792 -> 0.802, bf16 / 8 0.785 -> 0.791,
// the 16 x 4 MiB batch 0.770 / 0.767 (unchanged).
#ifndef KF_REDUCE_SCHED
#define KF_REDUCE_SCHED 1
#endif
// KF_REDUCE_PIN: an empty asm on each loaded word after the barrier, so the
// 8-bit min/max kernels' byte unpacking cannot be placed among the loads
// (the barrier alone left them 5 + 3): u8 max 0.799 -> 0.822, i8 min
// 0.803 -> 0.820, every other case unchanged, same bits
// (tools/ab_reduce_sched.py p0/p1, profiles/r06/ab_reduce_pin_r06z5.jsonl)
#ifndef KF_REDUCE_PIN
#define KF_REDUCE_PIN 1
#endif
// KF_FOLD_SCHED: the same barrier after the runtime-k fold's first two
// inputs' loads. No effect (k = 3 / 4 / 8 fp32, k = 4 bf16 and C5's k = 8
// batch all within 0.3 %, same bits; tools/ab_fold_sched.py,
// profiles/r06/ab_fold_sched_r06x.jsonl), so it stays off.
#ifndef KF_FOLD_SCHED
#define KF_FOLD_SCHED 0
#endif
template <typename T, int OP, int EPI, int KC, int BLOCK, int UNROLL, int LOADNT,
          int STPLAIN = 0>
__device__ __forceinline__ void reduce_body(const InPtrs &in, int k, void *out, size_t n,
                                            size_t head, size_t nvec, const Div &np,
                                            size_t blk, size_t nblk, int serial)
{
    using S         = typename Elt<T>::S;
    using L         = Lane<T>;
    using W         = typename L::W;
    using Acc       = typename L::Acc;
    constexpr int V = Vec<W>::N;                 // lanes per 16-B vector
    constexpr int E = static_cast<int>(16 / sizeof(S));  // elements per vector
    const int kk    = KC > 0 ? KC : k;

    // scalar edges: head elements, then the tail after the vector body
    const size_t tid   = blk * BLOCK + threadIdx.x;
    const size_t vend  = head + nvec * E;
    const size_t nedge = head + (n - vend);
    if (tid < nedge) {
        const size_t i = tid < head ? tid : vend + (tid - head);
        reinterpret_cast<S *>(out)[i] = fold_scalar<T, OP, EPI>(in, kk, i, np);
    }

    auto src = [&](int j) {
        return reinterpret_cast<const char *>(in.p[j]) + head * sizeof(S);
    };
    char *obase = reinterpret_cast<char *>(out) + head * sizeof(S);

    auto emit = [&](const Acc &a) -> W { return L::template emit<OP, EPI>(a, np); };

    const size_t tile   = static_cast<size_t>(BLOCK) * UNROLL;
    const size_t ntiles = (nvec + tile - 1) / tile;
    for (size_t t = blk; t < ntiles; t += nblk) {
        const size_t v0 = t * tile + threadIdx.x;
        if (v0 + (UNROLL - 1) * BLOCK < nvec) {
            Acc acc[UNROLL][V];
            if constexpr (KC > 0) {
                // compile-time k: all KC x UNROLL loads issued before any use
                Vec<W> v[KC][UNROLL];
#if KF_REDUCE_SCHED
                // raw 16-B words up to the barrier, so no unpacking of a
                // loaded word (the 8-bit lanes' byte extracts) is placed
                // among the loads with a wait of its own
                u32x4 raw[KC][UNROLL];
#pragma unroll
                for (int j = 0; j < KC; ++j) {
                    const char *sj = src(j);
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) raw[j][u] = ld_u4<LOADNT>(sj, v0 + u * BLOCK);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < KC; ++j) {
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) {
#if KF_REDUCE_PIN
                        asm volatile("" : "+v"(raw[j][u]));  // pins the unpack below here
#endif
                        __builtin_memcpy(&v[j][u], &raw[j][u], 16);
                    }
                }
#else
#pragma unroll
                for (int j = 0; j < KC; ++j) {
                    const char *sj = src(j);
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) v[j][u] = ld_vec<W, LOADNT>(sj, v0 + u * BLOCK);
                }
#endif
#pragma unroll
                for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
                    for (int e = 0; e < V; ++e) {
                        acc[u][e] = L::load(v[0][u].e[e]);
#pragma unroll
                        for (int j = 1; j < KC; ++j) {
                            acc[u][e] = L::template combine<OP>(acc[u][e], v[j][u].e[e]);
                        }
                    }
                }
            } else {
                // runtime k: inputs 0 and 1 up front, then one input at a time:
                // its UNROLL vectors together (small grids, latency-bound), or
                // one vector in flight (ld_vec_serial) when `serial` (grids
                // large enough to be bandwidth-bound; chosen by the host)
                Vec<W> a[UNROLL];
                Vec<W> b[UNROLL];
                const char *s0 = src(0);
#pragma unroll
                for (int u = 0; u < UNROLL; ++u) a[u] = ld_vec<W, LOADNT>(s0, v0 + u * BLOCK);
                if (kk > 1) {
                    const char *s1 = src(1);
#pragma unroll
                    for (int u = 0; u < UNROLL; ++u) b[u] = ld_vec<W, LOADNT>(s1, v0 + u * BLOCK);
                }
#if KF_FOLD_SCHED
                __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
                for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
                    for (int e = 0; e < V; ++e) {
                        acc[u][e] = L::load(a[u].e[e]);
                        if (kk > 1) {
                            acc[u][e] = L::template combine<OP>(acc[u][e], b[u].e[e]);
                        }
                    }
                }
                for (int j = 2; j < kk; ++j) {
                    const char *sj = src(j);
                    if (LOADNT && serial) {  // wave-uniform: a kernel argument
#pragma unroll
                        for (int u = 0; u < UNROLL; ++u) {
                            b[u] = ld_vec_serial<W>(sj, v0 + u * BLOCK);
#pragma unroll
                            for (int e = 0; e < V; ++e) {
                                acc[u][e] = L::template combine<OP>(acc[u][e], b[u].e[e]);
                            }
                        }
                    } else {
#pragma unroll
                        for (int u = 0; u < UNROLL; ++u) b[u] = ld_vec<W, LOADNT>(sj, v0 + u * BLOCK);
#pragma unroll
                        for (int u = 0; u < UNROLL; ++u) {
#pragma unroll
                            for (int e = 0; e < V; ++e) {
                                acc[u][e] = L::template combine<OP>(acc[u][e], b[u].e[e]);
                            }
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                Vec<W> r;
#pragma unroll
                for (int e = 0; e < V; ++e) r.e[e] = emit(acc[u][e]);
                st_vec<W, STPLAIN>(obase, v0 + u * BLOCK, r);
            }
        } else {
            // ragged last tile
            for (int u = 0; u < UNROLL; ++u) {
                const size_t vi = v0 + u * BLOCK;
                if (vi >= nvec) break;
                Vec<W> a = ld_vec<W, LOADNT>(src(0), vi);
                Acc acc[V];
#pragma unroll
                for (int e = 0; e < V; ++e) acc[e] = L::load(a.e[e]);
                for (int j = 1; j < kk; ++j) {
                    Vec<W> b = ld_vec<W, LOADNT>(src(j), vi);
#pragma unroll
                    for (int e = 0; e < V; ++e) {
                        acc[e] = L::template combine<OP>(acc[e], b.e[e]);
                    }
                }
                Vec<W> r;
#pragma unroll
                for (int e = 0; e < V; ++e) r.e[e] = emit(acc[e]);
                st_vec<W, STPLAIN>(obase, vi, r);
            }
        }
    }
}

template <typename T, int OP, int EPI, int KC, int BLOCK, int UNROLL, int LOADNT,
          int STPLAIN = 0>
__global__ void __launch_bounds__(BLOCK)
    reduce_kernel(InPtrs in, int k, void *out, size_t n, size_t head,
                  size_t nvec, Div np, int serial)
{
    if constexpr (EPI == EPI_DIV) {
        if (np.pow2) {
            reduce_body<T, OP, EPI_MUL, KC, BLOCK, UNROLL, LOADNT, STPLAIN>(
                in, k, out, n, head, nvec, np, blockIdx.x, gridDim.x, serial);
            return;
        }
    }
    reduce_body<T, OP, EPI, KC, BLOCK, UNROLL, LOADNT, STPLAIN>(in, k, out, n, head, nvec, np,
                                                               blockIdx.x, gridDim.x, serial);
}

// ---------------------------------------------------------------------------
// Batch: many independent buckets (same dtype, op, k and epilogue) in ONE
// launch. A 4 MiB bucket is 4.5 us of launch for 1.6 us of HBM time
// (profiles/r01/size_sweep.jsonl: 0.35 of the roofline); the per-bucket steps
// of an exchange (the /np of every shard, the fold of every bucket's received
// shards) come in dozens per step. Bucket s owns blocks [blk0[s], blk0[s+1])
// of the grid, one block per tile as in reduce_kernel, so the launch streams
// all buckets with the same per-block schedule. The arguments live in the
// kernarg segment (scalar loads; the bucket index is wave-uniform).
// ---------------------------------------------------------------------------
constexpr int kBatchSeg = 16;
// k = 1 (the shard /np after a reduce-scatter: one pointer per bucket) fits
// four times as many buckets in the kernarg segment: C3's 64 shards at N = 8
// go in ONE launch instead of four (30.0 us -> see DESIGN.md §3).
constexpr int kBatchSeg1 = 64;

template <int NSEG, int NPTR> struct BatchArgsT {
    const void *in[NSEG][NPTR];
    void *out[NSEG];
    size_t n[NSEG], head[NSEG], nvec[NSEG];
    unsigned blk0[NSEG + 1];
    int nseg;
    int serial;  // the runtime-k fold's one-in-flight schedule (reduce_body)
};
using BatchArgs  = BatchArgsT<kBatchSeg, kMaxInputs>;
using BatchArgs1 = BatchArgsT<kBatchSeg1, 1>;
static_assert(sizeof(BatchArgs1) <= 3072 && sizeof(BatchArgs) <= 3072, "kernarg budget");

// the bucket of block b: the last s with blk0[s] <= b (wave-uniform, scalar
// loads from the kernarg segment; a binary search past 16 buckets)
template <int NSEG, int NPTR>
__device__ __forceinline__ int batch_segment(const BatchArgsT<NSEG, NPTR> &a, unsigned b)
{
    if constexpr (NSEG <= 16) {
        int s = 0;
        while (s + 1 < a.nseg && b >= a.blk0[s + 1]) ++s;
        return s;
    } else {
        int lo = 0, hi = a.nseg - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (b >= a.blk0[mid]) lo = mid;
            else hi = mid - 1;
        }
        return lo;
    }
}

template <typename T, int OP, int EPI, int KC, int BLOCK, int UNROLL, int NSEG, int NPTR>
__global__ void __launch_bounds__(BLOCK) reduce_batch_kernel(BatchArgsT<NSEG, NPTR> a, int k,
                                                             Div np)
{
    // Buckets with equal block counts (the exchange's shards of equal
    // buckets) come as a 2-D grid, one row per bucket: the bucket is
    // blockIdx.y, known before any kernarg load. Otherwise the bucket of block
    // b is searched in the kernarg table, one dependent scalar load per step,
    // which cost 0.4-1.5 us of a ~6 us launch (tools/explore/shard_probe.hip,
    // profiles/r05/shard_probe_r05k.jsonl).
    // With a multiple of 8 rows, the blocks are handed out XCD by XCD:
    // workgroups go to the 8 XCDs round-robin in dispatch order, so linear
    // block L runs on XCD L % 8, and that XCD's j-th block takes bucket
    // (L % 8) + 8 * (j / per). Each XCD then sweeps an eighth of the buckets
    // instead of a slice of every one. It pays with many buckets: C3's 64
    // shards of a flat bucket buffer at N = 8, 15.3 -> 14.2 us in the probe,
    // 14.6 -> 13.8 us in bench.py; with C4's 16 it lost 0.1-0.4 us, so it
    // starts at 32 rows (tools/explore/shard_xcd_probe.hip,
    // profiles/r05/shard_xcd_probe_r05ah.jsonl, phase2_graph_xcd_r05ai.json).
    const bool rows   = gridDim.y > 1;
    const bool by_xcd = rows && gridDim.y >= 32 && (gridDim.y & 7u) == 0;
    const unsigned L  = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned b  = by_xcd ? (L >> 3) % gridDim.x : blockIdx.x;
    const int s       = by_xcd ? static_cast<int>((L & 7u) + 8u * ((L >> 3) / gridDim.x))
                        : rows ? static_cast<int>(blockIdx.y)
                               : batch_segment(a, b);
    const unsigned b0 = rows ? 0u : a.blk0[s];
    const size_t nblk = rows ? gridDim.x : a.blk0[s + 1] - a.blk0[s];
    InPtrs one;  // NPTR == 1: the bucket's single input (only p[0] is read, KC == 1)
    if constexpr (NPTR == 1) one.p[0] = a.in[s][0];
    const InPtrs &in = [&]() -> const InPtrs & {
        if constexpr (NPTR == 1) return one;
        else return *reinterpret_cast<const InPtrs *>(a.in[s]);
    }();
    if constexpr (EPI == EPI_DIV) {
        if (np.pow2) {
            reduce_body<T, OP, EPI_MUL, KC, BLOCK, UNROLL, 1, 0>(
                in, k, a.out[s], a.n[s], a.head[s], a.nvec[s], np, b - b0, nblk, a.serial);
            return;
        }
    }
    reduce_body<T, OP, EPI, KC, BLOCK, UNROLL, 1, 0>(in, k, a.out[s], a.n[s], a.head[s],
                                                    a.nvec[s], np, b - b0, nblk, a.serial);
}

// Fold for inputs that sit behind DIFFERENT links (the P2P shard fold reads
// shard `rank` of every peer's bucket over that peer's xGMI link). The runtime
// k loop above issues one input at a time, and since every resident block
// walks the inputs in the same order, at any moment nearly all requests go to
// one or two peers: the links would be used one after another. Here every
// thread issues the loads of up to 8 inputs before the first add, so all links
// carry traffic at once; the adds still run in input order (rank order), so
// the result is the same left fold bit for bit. One 16-B vector per input per
// thread per tile; k > 8 goes in groups of 8.
template <typename T, int OP, int EPI, int BLOCK>
__device__ __forceinline__ void spread_body(const InPtrs &in, int k, void *out, size_t n,
                                            size_t head, size_t nvec, const Div &np)
{
    using S         = typename Elt<T>::S;
    using L         = Lane<T>;
    using W         = typename L::W;
    using Acc       = typename L::Acc;
    constexpr int V = Vec<W>::N;
    constexpr int E = static_cast<int>(16 / sizeof(S));
    constexpr int G = 8;
    const size_t tid   = static_cast<size_t>(blockIdx.x) * BLOCK + threadIdx.x;
    const size_t vend  = head + nvec * E;
    const size_t nedge = head + (n - vend);
    if (tid < nedge) {
        const size_t i = tid < head ? tid : vend + (tid - head);
        reinterpret_cast<S *>(out)[i] = fold_scalar<T, OP, EPI>(in, k, i, np);
    }
    char *obase = reinterpret_cast<char *>(out) + head * sizeof(S);
    for (size_t vi = tid; vi < nvec; vi += static_cast<size_t>(gridDim.x) * BLOCK) {
        Acc acc[V];
        for (int j0 = 0; j0 < k; j0 += G) {
            Vec<W> v[G];
#pragma unroll
            for (int j = 0; j < G; ++j) {
                if (j0 + j < k) {
                    v[j] = ld_vec<W, 1>(reinterpret_cast<const char *>(in.p[j0 + j]) +
                                            head * sizeof(S), vi);
                }
            }
#pragma unroll
            for (int j = 0; j < G; ++j) {
                if (j0 + j < k) {
#pragma unroll
                    for (int e = 0; e < V; ++e) {
                        acc[e] = (j0 + j == 0) ? L::load(v[j].e[e])
                                               : L::template combine<OP>(acc[e], v[j].e[e]);
                    }
                }
            }
        }
        Vec<W> r;
#pragma unroll
        for (int e = 0; e < V; ++e) {
            r.e[e] = L::template emit<OP, EPI>(acc[e], np);
        }
        st_vec<W>(obase, vi, r);
    }
}

template <typename T, int OP, int EPI, int BLOCK>
__global__ void __launch_bounds__(BLOCK)
    reduce_spread_kernel(InPtrs in, int k, void *out, size_t n, size_t head,
                         size_t nvec, Div np)
{
    if constexpr (EPI == EPI_DIV) {
        if (np.pow2) {
            spread_body<T, OP, EPI_MUL, BLOCK>(in, k, out, n, head, nvec, np);
            return;
        }
    }
    spread_body<T, OP, EPI, BLOCK>(in, k, out, n, head, nvec, np);
}

// Element-at-a-time kernel for inputs whose 16-B alignment residues differ
// (e.g. host-side chunk slices at odd offsets). Still coalesced per element.
template <typename T, int OP, int EPI, int BLOCK>
__global__ void __launch_bounds__(BLOCK)
    reduce_kernel_unaligned(InPtrs in, int k, void *out, size_t n, Div np)
{
    using S = typename Elt<T>::S;
    constexpr int EP = EPI == EPI_DIV ? EPI_MUL : EPI;
    const bool p2    = EPI == EPI_DIV && np.pow2;
    for (size_t i = static_cast<size_t>(blockIdx.x) * BLOCK + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * BLOCK) {
        reinterpret_cast<S *>(out)[i] = p2 ? fold_scalar<T, OP, EP>(in, k, i, np)
                                           : fold_scalar<T, OP, EPI>(in, k, i, np);
    }
}

// SMA blend: v = fl(fl(c1*v) + fl(c2*fl(s/np))) (sma_sgd.py:60-65).
//
// blend_vec does a 16-B vector's lanes two at a time in packed fp32
// (v_pk_mul_f32 / v_pk_add_f32: each lane one IEEE fp32 operation, correctly
// rounded, the same denormal mode, no contraction under the pragma above), so
// the bits are the scalar blend's. The scalar form cost C5's bf16 blend about
// 1.5 % of the roofline in VALU issue (tools/explore/sma_probe.hip,
// profiles/r06/sma_probe_r06a.jsonl: 0.797 scalar, 0.809 packed, 0.811 for the
// same in-place traffic with no arithmetic at all).
typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 sma_pair(f32x2 v, f32x2 s, f32x2 c1, f32x2 c2, f32x2 inv,
                                          const Div &dv, bool p2)
{
    const f32x2 avg = p2 ? s * inv : f32x2{__fdiv_rn(s.x, dv.f), __fdiv_rn(s.y, dv.f)};
    return c1 * v + c2 * avg;
}

template <typename T> struct SmaMath;
template <> struct SmaMath<float> {
    using S = float;
    template <bool P2> __device__ static S blend(S v, S s, float c1, float c2, const Div &dv)
    {
        float avg = P2 ? __fmul_rn(s, dv.fi) : __fdiv_rn(s, dv.f);
        return __fadd_rn(__fmul_rn(c1, v), __fmul_rn(c2, avg));
    }
    template <bool P2>
    __device__ static Vec<S> blend_vec(const Vec<S> &a, const Vec<S> &b, float c1, float c2,
                                       const Div &dv)
    {
        const f32x2 C1 = {c1, c1}, C2 = {c2, c2}, I = {dv.fi, dv.fi};
        Vec<S> r;
#pragma unroll
        for (int e = 0; e < 4; e += 2) {
            const f32x2 o = sma_pair(f32x2{a.e[e], a.e[e + 1]}, f32x2{b.e[e], b.e[e + 1]}, C1, C2,
                                     I, dv, P2);
            r.e[e]     = o.x;
            r.e[e + 1] = o.y;
        }
        return r;
    }
};
template <> struct SmaMath<double> {
    using S = double;
    template <bool P2> __device__ static S blend(S v, S s, double c1, double c2, const Div &dv)
    {
        double avg = P2 ? __dmul_rn(s, dv.di) : __ddiv_rn(s, dv.d);
        return __dadd_rn(__dmul_rn(c1, v), __dmul_rn(c2, avg));
    }
    template <bool P2>
    __device__ static Vec<S> blend_vec(const Vec<S> &a, const Vec<S> &b, double c1, double c2,
                                       const Div &dv)
    {
        Vec<S> r;
#pragma unroll
        for (int e = 0; e < 2; ++e) r.e[e] = blend<P2>(a.e[e], b.e[e], c1, c2, dv);
        return r;
    }
};
template <> struct SmaMath<f16_t> {
    using S = uint16_t;
    template <bool P2> __device__ static S blend(S v, S s, float c1, float c2, const Div &dv)
    {
        const float x = f16_to_f32(s);
        float avg     = P2 ? __fmul_rn(x, dv.fi) : __fdiv_rn(x, dv.f);
        return f32_to_f16(__fadd_rn(__fmul_rn(c1, f16_to_f32(v)), __fmul_rn(c2, avg)));
    }
    template <bool P2>
    __device__ static Vec<S> blend_vec(const Vec<S> &a, const Vec<S> &b, float c1, float c2,
                                       const Div &dv)
    {
        const f32x2 C1 = {c1, c1}, C2 = {c2, c2}, I = {dv.fi, dv.fi};
        Vec<S> r;
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
            const f32x2 o = sma_pair(f32x2{f16_to_f32(a.e[e]), f16_to_f32(a.e[e + 1])},
                                     f32x2{f16_to_f32(b.e[e]), f16_to_f32(b.e[e + 1])}, C1, C2, I,
                                     dv, P2);
            r.e[e]     = f32_to_f16(o.x);
            r.e[e + 1] = f32_to_f16(o.y);
        }
        return r;
    }
};
template <> struct SmaMath<bf16_t> {
    using S = uint16_t;
    template <bool P2> __device__ static S blend(S v, S s, float c1, float c2, const Div &dv)
    {
        const float x = bf16_to_f32(s);
        float avg     = P2 ? __fmul_rn(x, dv.fi) : __fdiv_rn(x, dv.f);
        return f32_to_bf16(__fadd_rn(__fmul_rn(c1, bf16_to_f32(v)), __fmul_rn(c2, avg)));
    }
    // a 32-bit word holds two bf16 lanes: the low one widens by a shift, the
    // high one by a mask
    template <bool P2>
    __device__ static Vec<S> blend_vec(const Vec<S> &a, const Vec<S> &b, float c1, float c2,
                                       const Div &dv)
    {
        const f32x2 C1 = {c1, c1}, C2 = {c2, c2}, I = {dv.fi, dv.fi};
        u32x4 wa, wb, wr;
        __builtin_memcpy(&wa, &a, 16);
        __builtin_memcpy(&wb, &b, 16);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const f32x2 v = {__uint_as_float(wa[w] << 16), __uint_as_float(wa[w] & 0xffff0000u)};
            const f32x2 s = {__uint_as_float(wb[w] << 16), __uint_as_float(wb[w] & 0xffff0000u)};
            const f32x2 avg = P2 ? s * I : f32x2{__fdiv_rn(s.x, dv.f), __fdiv_rn(s.y, dv.f)};
            const f32x2 o = C1 * v + C2 * avg;
            wr[w] = static_cast<uint32_t>(f32_to_bf16(o.x)) |
                    (static_cast<uint32_t>(f32_to_bf16(o.y)) << 16);
        }
        Vec<S> r;
        __builtin_memcpy(&r, &wr, 16);
        return r;
    }
};

// The full tile's load schedule. Held to 64 VGPRs, the compiler issued the
// bf16 and fp16 blends' eight 16-B loads as three, a wait for the first two,
// then five: fewer loads in flight per wave than the add kernels of the same
// bytes. A scheduling barrier after the loads keeps all eight in flight
// (57 VGPRs, no spill; tests/test_isa.py): 256 MiB bf16 0.793 -> 0.816 of
// 8 TB/s, fp16 0.794 -> 0.822, fp32 0.807 -> 0.823, fp64 0.807 -> 0.820,
// C5's batch 0.775 -> 0.794, the same bits (tools/ab_sma_sched.py,
// profiles/r06/ab_sma_sched_r06p.jsonl). 0: the compiler's order; 1: the
// barrier (shipped); 2: the loads interleaved (v0, s0, v1, s1, ...) and the
// barrier, so each vector waits for its own two (0.79-0.81: behind 1).
#ifndef KF_SMA_SCHED
#define KF_SMA_SCHED 1
#endif

// One block `blk` of `nblk` working on one variable bucket (sma_kernel: the
// grid; sma_batch_kernel: the bucket's share of it).
template <typename T, typename C, int BLOCK, int UNROLL, bool P2>
__device__ __forceinline__ void sma_body(void *v, const void *s, size_t n, size_t head,
                                         size_t nvec, C c1, C c2, const Div &np, int vec_ok,
                                         size_t blk, size_t nblk)
{
    using S         = typename SmaMath<T>::S;
    constexpr int V = Vec<S>::N;
    S *pv           = reinterpret_cast<S *>(v);
    const S *ps     = reinterpret_cast<const S *>(s);
    const size_t tid = blk * BLOCK + threadIdx.x;
    if (!vec_ok) {
        for (size_t i = tid; i < n; i += nblk * BLOCK) {
            pv[i] = SmaMath<T>::template blend<P2>(pv[i], ps[i], c1, c2, np);
        }
        return;
    }
    const size_t vend  = head + nvec * V;
    const size_t nedge = head + (n - vend);
    if (tid < nedge) {
        const size_t i = tid < head ? tid : vend + (tid - head);
        pv[i]          = SmaMath<T>::template blend<P2>(pv[i], ps[i], c1, c2, np);
    }
    char *vb       = reinterpret_cast<char *>(v) + head * sizeof(S);
    const char *sb = reinterpret_cast<const char *>(s) + head * sizeof(S);
    const size_t tile   = static_cast<size_t>(BLOCK) * UNROLL;
    const size_t ntiles = (nvec + tile - 1) / tile;
    for (size_t t = blk; t < ntiles; t += nblk) {
        const size_t v0 = t * tile + threadIdx.x;
        if (v0 + (UNROLL - 1) * BLOCK < nvec) {
            // full tile: every load issued before the first use
            Vec<S> a[UNROLL], b[UNROLL];
#if KF_SMA_SCHED == 2
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                a[u] = ld_vec<S, 1>(vb, v0 + u * BLOCK);
                b[u] = ld_vec<S, 1>(sb, v0 + u * BLOCK);
            }
#else
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) a[u] = ld_vec<S, 1>(vb, v0 + u * BLOCK);
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) b[u] = ld_vec<S, 1>(sb, v0 + u * BLOCK);
#endif
#if KF_SMA_SCHED >= 1
            __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
            for (int u = 0; u < UNROLL; ++u) {
                st_vec<S>(vb, v0 + u * BLOCK,
                          SmaMath<T>::template blend_vec<P2>(a[u], b[u], c1, c2, np));
            }
        } else {
            for (int u = 0; u < UNROLL; ++u) {
                const size_t vi = v0 + u * BLOCK;
                if (vi >= nvec) break;
                const Vec<S> a = ld_vec<S, 1>(vb, vi), b = ld_vec<S, 1>(sb, vi);
                st_vec<S>(vb, vi, SmaMath<T>::template blend_vec<P2>(a, b, c1, c2, np));
            }
        }
    }
}

// the /np choice made once per kernel (see EPI_MUL above)
// Both SMA kernels are held to 64 VGPRs, 8 waves per SIMD (two blocks per
// SIMD): left to itself the compiler took 68 for the bf16 blend, which caps a
// CU at 7 of its 8 blocks of loads in flight (see SmaMath above).
template <typename T, typename C, int BLOCK, int UNROLL>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8)))
    sma_kernel(void *v, const void *s, size_t n, size_t head, size_t nvec,
               C c1, C c2, Div np, int vec_ok)
{
    if (np.pow2) {
        sma_body<T, C, BLOCK, UNROLL, true>(v, s, n, head, nvec, c1, c2, np, vec_ok, blockIdx.x,
                                            gridDim.x);
    } else {
        sma_body<T, C, BLOCK, UNROLL, false>(v, s, n, head, nvec, c1, c2, np, vec_ok, blockIdx.x,
                                             gridDim.x);
    }
}

// The SMA blend of many variable buckets in ONE launch (an exchange's step
// blends every bucket of the model; C5's BERT-base is 14 buckets), laid out
// as the reduce batch: bucket i owns blocks [blk0[i], blk0[i+1]).
template <typename C> struct SmaBatchArgs {
    void *v[kBatchSeg];
    const void *s[kBatchSeg];
    size_t n[kBatchSeg], head[kBatchSeg], nvec[kBatchSeg];
    int vec_ok[kBatchSeg];
    unsigned blk0[kBatchSeg + 1];
    int nseg;
    C c1, c2;
};

template <typename T, typename C, int BLOCK, int UNROLL>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8)))
    sma_batch_kernel(SmaBatchArgs<C> a, Div np)
{
    const unsigned b = blockIdx.x;
    int i            = 0;
    while (i + 1 < a.nseg && b >= a.blk0[i + 1]) ++i;
    const size_t nblk = a.blk0[i + 1] - a.blk0[i];
    if (np.pow2) {
        sma_body<T, C, BLOCK, UNROLL, true>(a.v[i], a.s[i], a.n[i], a.head[i], a.nvec[i], a.c1,
                                            a.c2, np, a.vec_ok[i], b - a.blk0[i], nblk);
    } else {
        sma_body<T, C, BLOCK, UNROLL, false>(a.v[i], a.s[i], a.n[i], a.head[i], a.nvec[i], a.c1,
                                             a.c2, np, a.vec_ok[i], b - a.blk0[i], nblk);
    }
}

}  // namespace kf
