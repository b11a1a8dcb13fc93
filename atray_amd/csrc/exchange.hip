// exchange.hip -- the multi-GPU frame exchange's byte kernels. The framebuffer's
// fourth byte is always 0 (BGRX, texture.h:27-38: b | g << 8 | r << 16), so a shard's packed
// framebuffer travels as 3 bytes per pixel: 25% fewer bytes into rank 0 over xGMI. pack_bgr
// squeezes a rank's packed u32 frames into bytes; scatter_bgr expands rank 0's gathered bytes
// back to BGRX and writes each pixel to its image position (the assembly index) in one pass.
#include <hip/hip_runtime.h>

#include <stdint.h>

namespace atr {

// One pixel per lane; a wave's 64 pixels are 192 consecutive bytes (coalesced byte stores).
__global__ __launch_bounds__(256) void pack_bgr_kernel(const uint32_t* __restrict__ src, int64_t n,
                                                       uint8_t* __restrict__ dst) {
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = src[i];
    dst[3 * i] = uint8_t(v);
    dst[3 * i + 1] = uint8_t(v >> 8);
    dst[3 * i + 2] = uint8_t(v >> 16);
}

__global__ __launch_bounds__(256) void scatter_bgr_kernel(const uint8_t* __restrict__ src, int64_t n,
                                                          const int64_t* __restrict__ dst_index,
                                                          uint32_t* __restrict__ image) {
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = uint32_t(src[3 * i]) | (uint32_t(src[3 * i + 1]) << 8) | (uint32_t(src[3 * i + 2]) << 16);
    image[dst_index[i]] = v;
}

}  // namespace atr

extern "C" hipError_t atr_launch_pack_bgr(const uint32_t* src, int64_t n, uint8_t* dst, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(atr::pack_bgr_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, src, n, dst);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_scatter_bgr(const uint8_t* src, int64_t n, const int64_t* dst_index,
                                             uint32_t* image, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(atr::scatter_bgr_kernel, dim3(unsigned((n + 255) / 256)), dim3(256), 0, s, src, n,
                       dst_index, image);
    return hipGetLastError();
}
