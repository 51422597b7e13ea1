/*
 * kf_oracle.c — TEST INFRASTRUCTURE ONLY. CPU restatement of KungFu's host
 * element reduce, used as the parity checker for the HIP path and as the
 * "port" CPU baseline in bench.py. Nothing in kungfu_amd/ links or calls this.
 *
 * Follows (all paths under /root/reference):
 *   srcs/go/kungfu/base/op.cpp:22-43   call_as<T>: SUM std::plus, MIN std::min,
 *                                      MAX std::max, PROD std::multiplies
 *   srcs/go/kungfu/base/op.cpp:45-54   call_as_f16: SUM only, else exit(1)
 *   srcs/go/kungfu/base/op.cpp:57-93   dispatch over 10 dtypes, else exit(1)
 *   srcs/go/kungfu/base/f16.c:16-50    fp16 -> fp32, fp32 add, fp32 -> fp16 RNE
 *   srcs/go/kungfu/base/dtype.c:7-35   element sizes
 *   srcs/python/kungfu/tensorflow/optimizers/sync_sgd.py:103-104  g / np
 *   srcs/python/kungfu/tensorflow/optimizers/sma_sgd.py:60-65     SMA blend
 *
 * Where the reference calls exit(1) the oracle returns a non-zero code so the
 * test process survives; the product's exit(1) is tested in a subprocess.
 *
 * std::min(a, b) is `(b < a) ? b : a` and std::max(a, b) is `(a < b) ? b : a`
 * (libstdc++ stl_algobase.h); this fixes NaN and signed-zero behaviour:
 * min(NaN, 1) = NaN, min(1, NaN) = 1, min(+0, -0) = +0.
 *
 * Built with the reference's cgo flags: -O2 -mavx -mf16c (CMakeLists.txt:28-30,
 * op.go:5), so the 1-thread timing is a like-for-like CPU baseline.
 *
 * bf16 is NOT in the reference. Its semantics here are the build's own
 * definition (fp32 arithmetic, one round-to-nearest-even to bf16, NaN kept a
 * quiet NaN); parity for bf16 is "unpinned" (DESIGN.md).
 */
#include <immintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

enum {
    DT_U8 = 0x00108, DT_U16 = 0x00208, DT_U32 = 0x00408, DT_U64 = 0x00808,
    DT_I8 = 0x10108, DT_I16 = 0x10208, DT_I32 = 0x10408, DT_I64 = 0x10808,
    DT_F16 = 0x20208, DT_F32 = 0x20408, DT_F64 = 0x20808, DT_BOOL = 0x30108,
    DT_BF16 = 0x20209,
};
enum { OP_SUM = 0, OP_MIN = 1, OP_MAX = 2, OP_PROD = 3 };

uint32_t oracle_type_size(int dt)
{
    switch (dt) {
    case DT_U8: case DT_I8: case DT_BOOL: return 1;
    case DT_U16: case DT_I16: case DT_F16: case DT_BF16: return 2;
    case DT_U32: case DT_I32: case DT_F32: return 4;
    case DT_U64: case DT_I64: case DT_F64: return 8;
    default: return 0; /* reference: print + exit(1) */
    }
}

/* Integer arithmetic is done in the unsigned type of the same width, which is
 * what the reference's promote-then-truncate (u8/u16/i8/i16) and two's
 * complement wrap (gcc, i32/i64) produce. Comparisons use the real type. */
#define INT_LOOP(T, UT)                                                        \
    {                                                                          \
        const T *a = (const T *)x;                                             \
        const T *b = (const T *)y;                                             \
        T *c = (T *)z;                                                         \
        switch (op) {                                                          \
        case OP_SUM:                                                           \
            for (int64_t i = 0; i < n; ++i)                                    \
                c[i] = (T)(UT)((UT)a[i] + (UT)b[i]);                           \
            return 0;                                                          \
        case OP_MIN:                                                           \
            for (int64_t i = 0; i < n; ++i) {                                  \
                T p = a[i], q = b[i];                                          \
                c[i] = (q < p) ? q : p;                                        \
            }                                                                  \
            return 0;                                                          \
        case OP_MAX:                                                           \
            for (int64_t i = 0; i < n; ++i) {                                  \
                T p = a[i], q = b[i];                                          \
                c[i] = (p < q) ? q : p;                                        \
            }                                                                  \
            return 0;                                                          \
        case OP_PROD:                                                          \
            for (int64_t i = 0; i < n; ++i)                                    \
                c[i] = (T)(UT)((UT)a[i] * (UT)b[i]);                           \
            return 0;                                                          \
        default:                                                               \
            return 2;                                                          \
        }                                                                      \
    }

#define FLOAT_LOOP(T)                                                          \
    {                                                                          \
        const T *a = (const T *)x;                                             \
        const T *b = (const T *)y;                                             \
        T *c = (T *)z;                                                         \
        switch (op) {                                                          \
        case OP_SUM:                                                           \
            for (int64_t i = 0; i < n; ++i) c[i] = a[i] + b[i];                \
            return 0;                                                          \
        case OP_MIN:                                                           \
            for (int64_t i = 0; i < n; ++i) {                                  \
                T p = a[i], q = b[i];                                          \
                c[i] = (q < p) ? q : p;                                        \
            }                                                                  \
            return 0;                                                          \
        case OP_MAX:                                                           \
            for (int64_t i = 0; i < n; ++i) {                                  \
                T p = a[i], q = b[i];                                          \
                c[i] = (p < q) ? q : p;                                        \
            }                                                                  \
            return 0;                                                          \
        case OP_PROD:                                                          \
            for (int64_t i = 0; i < n; ++i) c[i] = a[i] * b[i];                \
            return 0;                                                          \
        default:                                                               \
            return 2;                                                          \
        }                                                                      \
    }

/* fp16 sum, element by element with the scalar F16C conversions. The
 * reference converts 8 lanes at a time (f16.c:16-23) and pads the tail through
 * an 8-wide scratch (f16.c:38-49); per element the arithmetic is identical:
 * exact widen, one fp32 add, one RNE narrow (imm 0 = round to nearest even). */
void oracle_f16_sum(void *pz, const void *px, const void *py, int64_t len)
{
    const uint16_t *x = (const uint16_t *)px;
    const uint16_t *y = (const uint16_t *)py;
    uint16_t *z = (uint16_t *)pz;
    for (int64_t i = 0; i < len; ++i) {
        float s = _cvtsh_ss(x[i]) + _cvtsh_ss(y[i]);
        z[i] = (uint16_t)_cvtss_sh(s, 0);
    }
}

/* bf16 helpers: build-defined semantics (see header). */
static inline float bf16_to_f32(uint16_t h)
{
    uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

static inline uint16_t f32_to_bf16(float f)
{
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7fffffffu) > 0x7f800000u) { /* NaN: keep sign, force quiet */
        return (uint16_t)((u >> 16) | 0x0040u);
    }
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}

static int bf16_transform(const void *x, const void *y, void *z, int64_t n,
                          int op)
{
    const uint16_t *a = (const uint16_t *)x;
    const uint16_t *b = (const uint16_t *)y;
    uint16_t *c = (uint16_t *)z;
    for (int64_t i = 0; i < n; ++i) {
        float p = bf16_to_f32(a[i]), q = bf16_to_f32(b[i]);
        /* MIN/MAX select one input unchanged (its bit pattern is kept). */
        switch (op) {
        case OP_SUM: c[i] = f32_to_bf16(p + q); break;
        case OP_MIN: c[i] = (q < p) ? b[i] : a[i]; break;
        case OP_MAX: c[i] = (p < q) ? b[i] : a[i]; break;
        case OP_PROD: c[i] = f32_to_bf16(p * q); break;
        default: return 2;
        }
    }
    return 0;
}

/* std_transform_2 restated (op.cpp:57-93). Returns 0, or 1 for a dtype the
 * reference rejects (exit(1) at op.cpp:89), 2 for an op it rejects (op.cpp:41
 * for ints/floats, op.cpp:52 for fp16 non-SUM). */
int oracle_transform2(const void *x, const void *y, void *z, int64_t n, int dt,
                      int op)
{
    switch (dt) {
    case DT_U8: INT_LOOP(uint8_t, uint8_t)
    case DT_U16: INT_LOOP(uint16_t, uint16_t)
    case DT_U32: INT_LOOP(uint32_t, uint32_t)
    case DT_U64: INT_LOOP(uint64_t, uint64_t)
    case DT_I8: INT_LOOP(int8_t, uint8_t)
    case DT_I16: INT_LOOP(int16_t, uint16_t)
    case DT_I32: INT_LOOP(int32_t, uint32_t)
    case DT_I64: INT_LOOP(int64_t, uint64_t)
    case DT_F16:
        if (op != OP_SUM) return 2;
        oracle_f16_sum(z, x, y, n);
        return 0;
    case DT_F32: FLOAT_LOOP(float)
    case DT_F64: FLOAT_LOOP(double)
    case DT_BF16: return bf16_transform(x, y, z, n, op);
    default: return 1;
    }
}

/* k-input left fold: acc = in0; acc = acc o in_j for j = 1..k-1. This is the
 * accumulation a self-loop node performs, one Transform2(RecvBuf, acc, peer)
 * per received peer chunk (session.go:255-264). fp16 therefore rounds per hop.
 * bf16 (build-defined) accumulates in fp32 and rounds once. */
int oracle_reduce_k(const void *const *in, int k, void *out, int64_t n, int dt,
                    int op)
{
    uint32_t sz = oracle_type_size(dt);
    if (sz == 0 || k < 1) return 1;
    if (dt == DT_BF16 && k > 2) {
        const uint16_t *const *h = (const uint16_t *const *)in;
        uint16_t *o = (uint16_t *)out;
        for (int64_t i = 0; i < n; ++i) {
            float acc = bf16_to_f32(h[0][i]);
            uint16_t accbits = h[0][i];
            for (int j = 1; j < k; ++j) {
                float q = bf16_to_f32(h[j][i]);
                switch (op) {
                case OP_SUM: acc = acc + q; accbits = 0xffff; break;
                case OP_PROD: acc = acc * q; accbits = 0xffff; break;
                case OP_MIN: if (q < acc) { acc = q; accbits = h[j][i]; } break;
                case OP_MAX: if (acc < q) { acc = q; accbits = h[j][i]; } break;
                default: return 2;
                }
            }
            o[i] = (op == OP_MIN || op == OP_MAX) ? accbits : f32_to_bf16(acc);
        }
        return 0;
    }
    if (k == 1) {
        memmove(out, in[0], (size_t)n * sz);
        return 0;
    }
    int rc = oracle_transform2(in[0], in[1], out, n, dt, op);
    for (int j = 2; j < k && rc == 0; ++j)
        rc = oracle_transform2(out, in[j], out, n, dt, op);
    return rc;
}

/* S-SGD: sum then g / np (sync_sgd.py:103-104), true division in the tensor's
 * type. f16/bf16 (build-defined): divide in fp32 from the fp32 accumulator,
 * round once. */
int oracle_reduce_avg(const void *const *in, int k, void *out, int64_t n,
                      int dt, int np)
{
    if (dt == DT_F32) {
        int rc = oracle_reduce_k(in, k, out, n, dt, OP_SUM);
        float d = (float)np;
        float *o = (float *)out;
        for (int64_t i = 0; i < n; ++i) o[i] = o[i] / d;
        return rc;
    }
    if (dt == DT_F64) {
        int rc = oracle_reduce_k(in, k, out, n, dt, OP_SUM);
        double d = (double)np;
        double *o = (double *)out;
        for (int64_t i = 0; i < n; ++i) o[i] = o[i] / d;
        return rc;
    }
    if (dt == DT_F16) {
        int rc = oracle_reduce_k(in, k, out, n, dt, OP_SUM);
        uint16_t *o = (uint16_t *)out;
        for (int64_t i = 0; i < n; ++i)
            o[i] = (uint16_t)_cvtss_sh(_cvtsh_ss(o[i]) / (float)np, 0);
        return rc;
    }
    if (dt == DT_BF16) {
        const uint16_t *const *h = (const uint16_t *const *)in;
        uint16_t *o = (uint16_t *)out;
        for (int64_t i = 0; i < n; ++i) {
            float acc = bf16_to_f32(h[0][i]);
            for (int j = 1; j < k; ++j) acc = acc + bf16_to_f32(h[j][i]);
            o[i] = f32_to_bf16(acc / (float)np);
        }
        return 0;
    }
    return 1;
}

/* SMA blend (sma_sgd.py:60-65): avg = sum / np; v = (1-a)*v + a*avg, every
 * operation rounded separately (separate TF kernels, no contraction). The two
 * constants are Python doubles converted to the tensor dtype. */
int oracle_sma_blend(void *v, const void *sum, int64_t n, int dt, int np,
                     double alpha)
{
    if (dt == DT_F32) {
        float c1 = (float)(1.0 - alpha), c2 = (float)alpha;
        float d = (float)np;
        float *pv = (float *)v;
        const float *ps = (const float *)sum;
        for (int64_t i = 0; i < n; ++i) {
            float avg = ps[i] / d;
            float t1 = c1 * pv[i];
            float t2 = c2 * avg;
            pv[i] = t1 + t2;
        }
        return 0;
    }
    if (dt == DT_F64) {
        double c1 = 1.0 - alpha, c2 = alpha, d = (double)np;
        double *pv = (double *)v;
        const double *ps = (const double *)sum;
        for (int64_t i = 0; i < n; ++i) {
            double avg = ps[i] / d;
            double t1 = c1 * pv[i];
            double t2 = c2 * avg;
            pv[i] = t1 + t2;
        }
        return 0;
    }
    if (dt == DT_F16 || dt == DT_BF16) {
        /* build-defined: fp32 arithmetic, single rounding at the end */
        float c1 = (float)(1.0 - alpha), c2 = (float)alpha, d = (float)np;
        uint16_t *pv = (uint16_t *)v;
        const uint16_t *ps = (const uint16_t *)sum;
        for (int64_t i = 0; i < n; ++i) {
            float s = dt == DT_F16 ? _cvtsh_ss(ps[i]) : bf16_to_f32(ps[i]);
            float w = dt == DT_F16 ? _cvtsh_ss(pv[i]) : bf16_to_f32(pv[i]);
            float avg = s / d;
            float t1 = c1 * w;
            float t2 = c2 * avg;
            float r = t1 + t2;
            pv[i] = dt == DT_F16 ? (uint16_t)_cvtss_sh(r, 0) : f32_to_bf16(r);
        }
        return 0;
    }
    return 1;
}

/* ---- CPU baseline harness (bench.py cpu_baseline leg) -------------------- */

/* std_transform_2's signature (srcs/cpp/include/kungfu/op.h:17-19): lets the
 * harness time the reference's own compiled function (oracle/_ref) too */
typedef void (*transform2_fn)(const void *, const void *, void *, int, int, int);

struct chunk_job {
    const char *x, *y;
    char *z;
    int64_t n;
    int dt, op;
    int64_t chunk_elems;
    int64_t total; /* reps x chunks: chunk c is chunk c % nchunks of rep c / nchunks */
    int64_t nchunks;
    int64_t next;  /* shared counter (atomic fetch-add) */
    transform2_fn fn; /* 0: the restatement */
};

static void run_span(const struct chunk_job *j, int64_t b, int64_t e, uint32_t sz)
{
    if (j->fn) {
        j->fn(j->x + b * sz, j->y + b * sz, j->z + b * sz, (int)(e - b), j->dt, j->op);
    } else {
        oracle_transform2(j->x + b * sz, j->y + b * sz, j->z + b * sz, e - b, j->dt, j->op);
    }
}

/* One OS thread of the pool (a Go P under GOMAXPROCS): takes the next chunk
 * of the stream of all-reduces until every rep's chunks are taken, the way
 * runStrategiesWithHash's goroutine-per-chunk fan-out (session.go:317-323)
 * keeps every thread busy. The threads live for all reps: a goroutine costs
 * no thread creation, so neither does a rep here. */
static void *chunk_worker(void *arg)
{
    struct chunk_job *j = (struct chunk_job *)arg;
    uint32_t sz = oracle_type_size(j->dt);
    for (;;) {
        int64_t c = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
        if (c >= j->total) break;
        int64_t b = (c % j->nchunks) * j->chunk_elems;
        int64_t e = b + j->chunk_elems < j->n ? b + j->chunk_elems : j->n;
        run_span(j, b, e, sz);
    }
    return 0;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

#define MAX_POOL 1024

static double bench(transform2_fn fn, const void *x, const void *y, void *z, int64_t n,
                    int dt, int op, int reps, int threads, int64_t chunk_bytes)
{
    uint32_t sz = oracle_type_size(dt);
    if (sz == 0 || threads < 1 || threads > MAX_POOL || n <= 0) return -1.0;
    if (fn && n > 2147483647) return -1.0; /* the reference's n is an int */
    struct chunk_job j;
    j.x = (const char *)x; j.y = (const char *)y; j.z = (char *)z;
    j.n = n; j.dt = dt; j.op = op; j.fn = fn;
    if (threads == 1) {
        double t0 = now_s();
        for (int r = 0; r < reps; ++r) run_span(&j, 0, n, sz);
        return now_s() - t0;
    }
    j.chunk_elems = chunk_bytes / sz > 0 ? chunk_bytes / sz : 1;
    j.nchunks = (n + j.chunk_elems - 1) / j.chunk_elems;
    j.total = j.nchunks * reps;
    j.next = 0;
    pthread_t tid[MAX_POOL];
    double t0 = now_s(); /* one pool for all reps: its start-up is amortised */
    int started = 0;
    for (; started < threads; ++started) {
        if (pthread_create(&tid[started], 0, chunk_worker, &j) != 0) break;
    }
    for (int i = 0; i < started; ++i) pthread_join(tid[i], 0);
    if (started == 0) return -1.0;
    return now_s() - t0;
}

/* Time `reps` reductions of n elements, split into chunk_bytes chunks handed
 * to `threads` workers (the goroutine-per-1MiB-chunk model of
 * session.go:313-326). Returns total seconds. */
double oracle_bench_transform2(const void *x, const void *y, void *z,
                               int64_t n, int dt, int op, int reps,
                               int threads, int64_t chunk_bytes)
{
    return bench(0, x, y, z, n, dt, op, reps, threads, chunk_bytes);
}

/* The same harness around a std_transform_2-compatible function pointer
 * (bench.py: the reference's own build, oracle/_ref/libkfbase_ref.so). */
double oracle_bench_fn(void *fn, const void *x, const void *y, void *z, int64_t n,
                       int dt, int op, int reps, int threads, int64_t chunk_bytes)
{
    if (!fn) return -1.0;
    return bench((transform2_fn)fn, x, y, z, n, dt, op, reps, threads, chunk_bytes);
}

/* The session's host fold (kf_host_reduce_fn, include/kungfu_amd.h) around a
 * std_transform_2-compatible function: bench.py's C1 CPU mode folds with the
 * reference's own compiled std_transform_2 (oracle/_ref) through this. */
static transform2_fn g_fold_fn;

void oracle_set_fold_fn(void *fn) { g_fold_fn = (transform2_fn)fn; }

int oracle_fold_via_fn(const void *x, const void *y, void *out, int64_t n, int dt, int op)
{
    if (!g_fold_fn || n > 2147483647) return 3;
    g_fold_fn(x, y, out, (int)n, dt, op);
    return 0;
}
