// div_check.hip — is x / d (IEEE, correctly rounded, __fdiv_rn) equal to the
// two-FMA form q = x * r; e = fma(-q, d, x); q' = fma(e, r, q) with
// r = RN(1/d), bit for bit, for EVERY fp32 x (all 2^32 patterns: NaNs,
// infinities, subnormals included) and each integer divisor d in [2, 1024]?
// The /np epilogue (sync_sgd.py:103-104, TF's g / np) needs the IEEE
// quotient; a divisor that passes here can take the three-instruction form
// instead of the ~10-instruction division sequence. Prints one JSON line per
// divisor: mismatch count and the first mismatching input.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o div_check div_check.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

// per divisor: [0] mismatches, [1] first mismatching bits (or ~0)
__global__ void check(float d, float r, unsigned long long *res)
{
    const unsigned stride = gridDim.x * blockDim.x;
    unsigned long long bad = 0;
    unsigned first = 0xffffffffu;
    for (unsigned long long i = blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
        const float x  = __uint_as_float(static_cast<unsigned>(i));
        const float q0 = __fdiv_rn(x, d);
        const float q  = __fmul_rn(x, r);
        const float e  = __fmaf_rn(-q, d, x);
        const float q1 = __fmaf_rn(e, r, q);
        if (__float_as_uint(q0) != __float_as_uint(q1)) {
            ++bad;
            if (static_cast<unsigned>(i) < first) first = static_cast<unsigned>(i);
        }
    }
    if (bad) {
        atomicAdd(&res[0], bad);
        atomicMin(&res[1], static_cast<unsigned long long>(first));
    }
}

int main(int argc, char **argv)
{
    const int lo = argc > 1 ? atoi(argv[1]) : 2, hi = argc > 2 ? atoi(argv[2]) : 1024;
    unsigned long long *res;
    CHECK(hipMalloc(&res, 2 * sizeof(unsigned long long)));
    for (int d = lo; d <= hi; ++d) {
        if ((d & (d - 1)) == 0) continue;  // powers of two multiply exactly
        unsigned long long h[2] = {0, ~0ull};
        CHECK(hipMemcpy(res, h, sizeof h, hipMemcpyHostToDevice));
        const float df = static_cast<float>(d);
        const float r  = 1.0f / df;  // host: RN(1/d)
        check<<<4096, 256>>>(df, r, res);
        CHECK(hipMemcpy(h, res, sizeof h, hipMemcpyDeviceToHost));
        printf("{\"d\": %d, \"mismatches\": %llu, \"first\": \"0x%08llx\"}\n", d, h[0],
               h[0] ? h[1] : 0ull);
        fflush(stdout);
    }
    return 0;
}
