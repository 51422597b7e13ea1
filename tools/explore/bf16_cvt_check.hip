// Exhaustive check: gfx950's v_cvt_pk_bf16_f32 (what clang emits for a
// float -> __bf16 conversion) against the bit recipe the kernels and the
// oracle use for the bf16 narrow (RNE; a NaN keeps sign and upper payload and
// is made quiet), over all 2^32 fp32 bit patterns. Prints one JSON line.
//   hipcc --offload-arch=gfx950 -O3 -o bf16_cvt_check bf16_cvt_check.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ __forceinline__ uint16_t recipe(uint32_t u)
{
    if ((u & 0x7fffffffu) > 0x7f800000u) return static_cast<uint16_t>((u >> 16) | 0x0040u);
    return static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__global__ void check(uint64_t base, unsigned long long *count, uint32_t *samples)
{
    const uint64_t i0 = base + (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 4;
    unsigned int bad = 0;
    for (int j = 0; j < 4; ++j) {
        const uint32_t u = static_cast<uint32_t>(i0 + j);
        const uint16_t hw = __builtin_bit_cast(uint16_t, static_cast<__bf16>(__uint_as_float(u)));
        if (hw != recipe(u)) {
            ++bad;
            const unsigned long long slot = atomicAdd(count + 1, 1ull);
            if (slot < 16) {
                samples[2 * slot] = u;
                samples[2 * slot + 1] = hw;
            }
        }
    }
    if (bad) atomicAdd(count, static_cast<unsigned long long>(bad));
}

int main()
{
    unsigned long long *count;
    uint32_t *samples;
    if (hipMalloc(&count, 16) != hipSuccess || hipMalloc(&samples, 128) != hipSuccess) return 1;
    hipMemset(count, 0, 16);
    hipMemset(samples, 0, 128);
    const uint64_t per = 1ull << 30;  // patterns per launch
    for (uint64_t b = 0; b < (1ull << 32); b += per) {
        hipLaunchKernelGGL(check, dim3(per / 4 / 256), dim3(256), 0, 0, b, count, samples);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    unsigned long long h[2];
    uint32_t s[32];
    hipMemcpy(h, count, 16, hipMemcpyDeviceToHost);
    hipMemcpy(s, samples, 128, hipMemcpyDeviceToHost);
    printf("{\"patterns\": 4294967296, \"mismatches\": %llu, \"samples\": [", h[0]);
    for (unsigned long long i = 0; i < h[0] && i < 16; ++i)
        printf("%s[\"0x%08x\", \"0x%04x\"]", i ? ", " : "", s[2 * i], s[2 * i + 1]);
    printf("]}\n");
    return 0;
}
