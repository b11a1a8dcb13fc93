// exchange.hip -- the multi-GPU frame exchange's byte kernels. The framebuffer's
// fourth byte is always 0 (BGRX, texture.h:27-38: b | g << 8 | r << 16), so a shard's packed
// framebuffer travels as 3 bytes per pixel: 25% fewer bytes into rank 0 over xGMI. pack_bgr
// squeezes a rank's packed u32 frames into bytes; scatter_bgr expands rank 0's gathered bytes
// back to BGRX and writes each pixel to its image position (the assembly index) in one pass.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <cstring>

#include "engine.h"

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


// ---------------------------------------------------------------- masked (background) exchange
// Lossless, for frames that are mostly one value (c3: 86% of the pixels are the sky's colour): a
// bit per pixel "not the background" plus 3 bytes for each such pixel only. Stream layout (bytes):
//   [0, 16)        magic 'ATRN', bg (BGRX u32), nchunk, payload pixels in all
//   [16, +4 n)     payload pixel offset of each 8192-pixel chunk (exclusive prefix)
//   then           256 mask words (u32) per chunk, bit i of word k = pixel 32 k + i of the chunk
//   then           128 group offsets (u32) per chunk: the payload pixel offset of each 64-pixel
//                  group (written by the encoder, so a decoder needs no scan of its own)
//   then           3 bytes (B, G, R) per non-background pixel, in pixel order
// Encoder: masks and per-chunk counts (one ballot per 64 pixels), the counts' scan (one
// workgroup), the payload and group offsets; decoders: one pass.
constexpr int kMaskChunk = 8192;  // pixels per chunk = 4 waves x 32 groups of 64
constexpr uint32_t kMaskMagic = 0x4E525441u;  // "ATRN" (round 6's first layout, "ATRM", had no group offsets)

__device__ __forceinline__ uint32_t* mask_words(uint8_t* base, int64_t nchunk) {
    return reinterpret_cast<uint32_t*>(base + 16 + 4 * nchunk);
}
__device__ __forceinline__ int64_t group_offsets_at(int64_t nchunk) { return 16 + 4 * nchunk + int64_t(kMaskChunk / 8) * nchunk; }
__device__ __forceinline__ int64_t payload_at(int64_t nchunk) {
    return group_offsets_at(nchunk) + int64_t(kMaskChunk / 64) * 4 * nchunk;
}

// Wave w of chunk c covers pixels c * 8192 + w * 2048 + [0, 2048): 32 groups of 64.
__global__ __launch_bounds__(256) void masked_count_kernel(const uint32_t* __restrict__ src, int64_t n, uint32_t bg,
                                                           uint8_t* __restrict__ out, int64_t nchunk) {
    __shared__ uint32_t part[4];
    const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int64_t c = blockIdx.x;
    uint32_t* mw = mask_words(out, nchunk) + c * (kMaskChunk / 32) + w * 64;
    const int64_t p0 = c * kMaskChunk + int64_t(w) * 2048;
    uint32_t cnt = 0;
    for (int g = 0; g < 32; ++g) {
        const int64_t i = p0 + g * 64 + ln;
        const bool nb = i < n && src[i] != bg;
        const unsigned long long m = __ballot(nb);
        if (ln == 0) {
            mw[2 * g] = uint32_t(m);
            mw[2 * g + 1] = uint32_t(m >> 32);
        }
        cnt += uint32_t(__popcll(m));
    }
    if (ln == 0) part[w] = cnt;
    __syncthreads();
    if (threadIdx.x == 0)
        reinterpret_cast<uint32_t*>(out + 16)[c] = part[0] + part[1] + part[2] + part[3];
}

// Exclusive scan of the chunk counts in place (one workgroup, 1024 chunks per pass), the header
// and the stream's byte count.
__global__ __launch_bounds__(1024) void masked_scan_kernel(uint8_t* __restrict__ out, int64_t nchunk, uint32_t bg,
                                                           int64_t* __restrict__ nbytes) {
    __shared__ uint32_t wsum[16];
    __shared__ uint32_t carry_s;
    uint32_t* off = reinterpret_cast<uint32_t*>(out + 16);
    const int ln = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (threadIdx.x == 0) carry_s = 0;
    __syncthreads();
    for (int64_t b = 0; b < nchunk; b += 1024) {
        const int64_t i = b + threadIdx.x;
        const uint32_t v = i < nchunk ? off[i] : 0u;
        uint32_t x = v;  // inclusive scan within the wave
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t y = uint32_t(__shfl_up(int(x), d));
            if (ln >= d) x += y;
        }
        if (ln == 63) wsum[w] = x;
        __syncthreads();
        uint32_t before = carry_s;
        for (int k = 0; k < w; ++k) before += wsum[k];
        if (i < nchunk) off[i] = before + x - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry_s = before + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        uint32_t* h = reinterpret_cast<uint32_t*>(out);
        h[0] = kMaskMagic;
        h[1] = bg;
        h[2] = uint32_t(nchunk);
        h[3] = carry_s;
        *nbytes = payload_at(nchunk) + 3 * int64_t(carry_s);
    }
}

// A wave's first payload pixel: its chunk's offset plus the popcounts of the earlier waves' masks.
__device__ __forceinline__ uint32_t masked_wave_base(const uint32_t* off, const uint32_t* mw_chunk, int w, int ln) {
    __shared__ uint32_t part[4];
    uint32_t cnt = uint32_t(__popc(mw_chunk[w * 64 + ln]));
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cnt += uint32_t(__shfl_xor(int(cnt), o));
    if (ln == 0) part[w] = cnt;
    __syncthreads();
    uint32_t b = off[blockIdx.x];
    for (int k = 0; k < w; ++k) b += part[k];
    return b;
}

__global__ __launch_bounds__(256) void masked_payload_kernel(const uint32_t* __restrict__ src, int64_t n,
                                                             uint8_t* __restrict__ out, int64_t nchunk) {
    const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int64_t c = blockIdx.x;
    const uint32_t* mw = mask_words(out, nchunk) + c * (kMaskChunk / 32);
    uint32_t base = masked_wave_base(reinterpret_cast<const uint32_t*>(out + 16), mw, w, ln);
    uint8_t* pay = out + payload_at(nchunk);
    uint32_t* gw = reinterpret_cast<uint32_t*>(out + group_offsets_at(nchunk)) + c * (kMaskChunk / 64) + w * 32;
    const int64_t p0 = c * kMaskChunk + int64_t(w) * 2048;
    const unsigned long long below = (ln ? ~0ull >> (64 - ln) : 0ull);
    for (int g = 0; g < 32; ++g) {
        if (ln == 0) gw[g] = base;  // the group's first payload pixel
        const unsigned long long m = uint64_t(mw[w * 64 + 2 * g]) | (uint64_t(mw[w * 64 + 2 * g + 1]) << 32);
        if ((m >> ln) & 1) {
            const uint32_t v = src[p0 + g * 64 + ln];
            uint8_t* d = pay + 3 * int64_t(base + uint32_t(__popcll(m & below)));
            d[0] = uint8_t(v);
            d[1] = uint8_t(v >> 8);
            d[2] = uint8_t(v >> 16);
        }
        base += uint32_t(__popcll(m));
    }
}

__global__ __launch_bounds__(256) void masked_scatter_kernel(const uint8_t* __restrict__ in, int64_t n,
                                                             const int64_t* __restrict__ dst_index,
                                                             uint32_t* __restrict__ image, int64_t nchunk) {
    const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
    const int64_t c = blockIdx.x;
    const uint32_t bg = reinterpret_cast<const uint32_t*>(in)[1];
    const uint32_t* mw = reinterpret_cast<const uint32_t*>(in + 16 + 4 * nchunk) + c * (kMaskChunk / 32);
    uint32_t base = masked_wave_base(reinterpret_cast<const uint32_t*>(in + 16), mw, w, ln);
    const uint8_t* pay = in + payload_at(nchunk);
    const int64_t p0 = c * kMaskChunk + int64_t(w) * 2048;
    const unsigned long long below = (ln ? ~0ull >> (64 - ln) : 0ull);
    for (int g = 0; g < 32; ++g) {
        const unsigned long long m = uint64_t(mw[w * 64 + 2 * g]) | (uint64_t(mw[w * 64 + 2 * g + 1]) << 32);
        const int64_t i = p0 + g * 64 + ln;
        if (i < n) {
            uint32_t v = bg;
            if ((m >> ln) & 1) {
                const uint8_t* s = pay + 3 * int64_t(base + uint32_t(__popcll(m & below)));
                v = uint32_t(s[0]) | (uint32_t(s[1]) << 8) | (uint32_t(s[2]) << 16);
            }
            image[dst_index[i]] = v;
        }
        base += uint32_t(__popcll(m));
    }
}


// Block-structured decode (atr_unpack_masked, atr_unpack_masked_ranks): the stream of a PACKED
// render of a tile list is in its blocks' slot order, so each 8x8 block's wave finds its pixels'
// image positions from the block record (32 B per 64 pixels) instead of an 8-B index per pixel,
// and each 64-slot group's first payload pixel in the stream's group offsets. One launch decodes
// up to kMaxUnpackSrc streams (rank 0's received shards, and its own packed frames as a raw
// source): the grid is the sources' blocks back to back, each wave finding its source in the
// kernel-argument table.
constexpr int kMaxUnpackSrc = 16;
struct UnpackSrc {
    const DBlock* blocks;
    const uint8_t* in;
    int64_t own;     // packed pixels per frame
    int64_t nchunk;  // the stream's chunks
    int64_t wave0;   // its first wave (block) in the decode grid
    int32_t nblocks;
    int32_t raw;     // 1: `in` is the render's u32 PACKED frames themselves (rank 0's own), no stream
};
struct UnpackSrcs {
    UnpackSrc s[kMaxUnpackSrc];
    int32_t n, pad;
};

// One wave per (source, block), looping over the frames kUnpackFrames at a time with their loads
// issued together (mask words and group offset, then payload bytes, then the stores): the block
// record is read once for all frames and no item index has to be divided into frame and block
// (one (frame, block) item per wave measured ~0.7 TB/s of image writes, its 64-bit division and
// three dependent loads per 64 pixels dominating).
constexpr int kUnpackFrames = 4;
__global__ __launch_bounds__(256) void unpack_masked_kernel(UnpackSrcs S, int64_t nblocks_all, int32_t width,
                                                            int32_t nframes, uint32_t* __restrict__ image,
                                                            int64_t image_stride) {
    const int64_t wv = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (wv >= nblocks_all) return;
    int k = 0;  // wave-uniform
    while (k + 1 < S.n && wv >= S.s[k + 1].wave0) ++k;
    const UnpackSrc& src = S.s[k];
    const DBlock blk = src.blocks[wv - src.wave0];
    const uint64_t mask = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
    if (!((mask >> lane) & 1)) return;
    const uint8_t* __restrict__ in = src.in;
    const int64_t nchunk = src.nchunk, own = src.own;
    const int64_t slot0 = blk.out_base + __popcll(mask & ((uint64_t(1) << lane) - 1));
    uint32_t* dst = image + int64_t(blk.y0 + (lane >> 3)) * width + blk.x0 + (lane & 7);
    if (src.raw) {  // a copy of the packed frames into the image
        const uint32_t* __restrict__ fb = reinterpret_cast<const uint32_t*>(in);
        for (int32_t f = 0; f < nframes; ++f) dst[int64_t(f) * image_stride] = fb[int64_t(f) * own + slot0];
        return;
    }
    const uint32_t bg = reinterpret_cast<const uint32_t*>(in)[1];
    const uint32_t* mw = reinterpret_cast<const uint32_t*>(in + 16 + 4 * nchunk);
    const uint8_t* pay = in + payload_at(nchunk);
    const uint32_t* __restrict__ goff = reinterpret_cast<const uint32_t*>(in + group_offsets_at(nchunk));
    for (int32_t f0 = 0; f0 < nframes; f0 += kUnpackFrames) {
        uint64_t m[kUnpackFrames];
        uint32_t go[kUnpackFrames];
        int bit[kUnpackFrames];
#pragma unroll
        for (int j = 0; j < kUnpackFrames; ++j) {
            const int32_t f = f0 + j < nframes ? f0 + j : nframes - 1;
            const int64_t slot = int64_t(f) * own + slot0, g = slot >> 6;
            bit[j] = int(slot & 63);
            m[j] = uint64_t(mw[2 * g]) | (uint64_t(mw[2 * g + 1]) << 32);
            go[j] = goff[g];
        }
        uint32_t v[kUnpackFrames];
#pragma unroll
        for (int j = 0; j < kUnpackFrames; ++j) {
            v[j] = bg;
            if ((m[j] >> bit[j]) & 1) {
                const uint8_t* p = pay + 3 * int64_t(go[j] + uint32_t(__popcll(m[j] & ((uint64_t(1) << bit[j]) - 1))));
                v[j] = uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16);
            }
        }
#pragma unroll
        for (int j = 0; j < kUnpackFrames; ++j)
            if (f0 + j < nframes) dst[int64_t(f0 + j) * image_stride] = v[j];
    }
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

extern "C" int64_t atr_masked_chunks(int64_t n) { return (n + atr::kMaskChunk - 1) / atr::kMaskChunk; }

extern "C" hipError_t atr_launch_pack_bgr_masked(const uint32_t* src, int64_t n, uint32_t bg, uint8_t* out,
                                                 int64_t* nbytes, hipStream_t s) {
    const int64_t nc = atr_masked_chunks(n);
    if (nc > 0) {
        hipLaunchKernelGGL(atr::masked_count_kernel, dim3(unsigned(nc)), dim3(256), 0, s, src, n, bg, out, nc);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(atr::masked_scan_kernel, dim3(1), dim3(1024), 0, s, out, nc, bg, nbytes);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || nc == 0) return e;
    hipLaunchKernelGGL(atr::masked_payload_kernel, dim3(unsigned(nc)), dim3(256), 0, s, src, n, out, nc);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_scatter_bgr_masked(const uint8_t* in, int64_t n, const int64_t* dst_index,
                                                    uint32_t* image, hipStream_t s) {
    const int64_t nc = atr_masked_chunks(n);
    if (nc <= 0) return hipSuccess;
    hipLaunchKernelGGL(atr::masked_scatter_kernel, dim3(unsigned(nc)), dim3(256), 0, s, in, n, dst_index, image, nc);
    return hipGetLastError();
}

// Up to kMaxUnpackSrc streams into the same frames: blocks[i] (nblocks[i] blocks of a PACKED
// render, own[i] pixels per frame), in[i] its stream (or, raw[i], its u32 PACKED frames).
extern "C" int atr_unpack_max_sources() { return atr::kMaxUnpackSrc; }
extern "C" hipError_t atr_launch_unpack_masked_multi(int32_t n, const atr::DBlock* const* blocks,
                                                     const int32_t* nblocks, const int64_t* own,
                                                     const uint8_t* const* in, const int32_t* raw, int32_t width,
                                                     int32_t nframes, uint32_t* image, int64_t image_stride,
                                                     hipStream_t s) {
    if (n <= 0 || n > atr::kMaxUnpackSrc || nframes <= 0) return n > atr::kMaxUnpackSrc ? hipErrorInvalidValue : hipSuccess;
    atr::UnpackSrcs S;
    std::memset(&S, 0, sizeof(S));
    int64_t waves = 0;
    for (int32_t i = 0; i < n; ++i) {
        atr::UnpackSrc& u = S.s[S.n];
        const bool r = raw && raw[i];
        const int64_t nc = r ? 0 : atr_masked_chunks(int64_t(nframes) * own[i]);
        if ((!r && nc <= 0) || nblocks[i] <= 0 || own[i] <= 0) continue;  // nothing to decode from this source
        u.raw = r ? 1 : 0;
        u.blocks = blocks[i];
        u.in = in[i];
        u.own = own[i];
        u.nchunk = nc;
        u.wave0 = waves;  // its first block in the decode grid (a wave per block)
        u.nblocks = nblocks[i];
        waves += nblocks[i];
        ++S.n;
    }
    if (!S.n) return hipSuccess;
    hipLaunchKernelGGL(atr::unpack_masked_kernel, dim3(unsigned((waves + 3) / 4)), dim3(256), 0, s, S, waves, width,
                       nframes, image, image_stride);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_unpack_masked(const atr::DBlock* blocks, int32_t nblocks, int32_t width,
                                               const uint8_t* in, int32_t nframes, int64_t own, uint32_t* image,
                                               int64_t image_stride, hipStream_t s) {
    return atr_launch_unpack_masked_multi(1, &blocks, &nblocks, &own, &in, nullptr, width, nframes, image, image_stride,
                                          s);
}

