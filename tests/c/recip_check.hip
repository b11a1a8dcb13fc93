// recip_check.hip -- exhaustive check of the engine's fast f32 reciprocal (trace.h recip_det)
// against IEEE division, 1.0f / x, for every f32 x in [2^-14, 2^64): every mantissa of every
// exponent the culled Moller-Trumbore test's det can take on the fast path (det >= kTol = 1e-4 >
// 2^-14; larger dets take the division). Built by atray_amd/csrc/Makefile into atray_amd/_lib/,
// run by tests/test_gpu_recip.py on the GPU. Prints "recip mismatches N checked M".
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../atray_amd/csrc/trace.h"

__global__ void check(unsigned long long* bad, unsigned long long* first) {
    const uint32_t e = blockIdx.y;                                     // exponent offset
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;          // mantissa
    if (m >= (1u << 23)) return;
    const uint32_t bits = ((127u - 14u + e) << 23) | m;
    const float x = __uint_as_float(bits);
    const float want = 1.0f / x;
    const float got = atr::recip_det(x);
    if (__float_as_uint(want) != __float_as_uint(got)) {
        atomicAdd(bad, 1ull);
        atomicMin(first, (unsigned long long)bits);
    }
}

int main() {
    unsigned long long *bad, *first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 8) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8);
    (void)hipMemset(first, 0xFF, 8);
    const uint32_t nexp = 64 + 14;
    hipLaunchKernelGGL(check, dim3((1u << 23) / 256, nexp), dim3(256), 0, 0, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    unsigned long long h[2];
    (void)hipMemcpy(&h[0], bad, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&h[1], first, 8, hipMemcpyDeviceToHost);
    std::printf("recip mismatches %llu checked %llu first 0x%llx\n", h[0], (unsigned long long)nexp << 23, h[1]);
    return h[0] ? 1 : 0;
}
