// render.hip -- gfx950 cell kernels of the render path: a wavefront per 8x8 pixel cell, one pixel
// per lane, the full per-pixel loop of render_tile_from_camera (renderer.cpp:294-369) -> cast_ray
// (:213-262) -> get_intersection_data (:34-160) -> octree traversal (scan.h).
//
// Shipping schedules: HYBRID (primary-only frames, the c3 default), LANE (the
// reference's exact per-lane work) and FLAT (the cell megakernel of multi-bounce renders; the
// default multi-bounce engine is the sample-parallel one in paths.hip). Schedules measured slower
// in rounds 1-3 (WAVE, TILE4/8, the leaf-major WAVEFRONT, PERSIST, path regeneration, speculative
// leaf steps, ...) were removed in round 4; git history keeps them ("Removed").
#include <hip/hip_runtime.h>

#include "scan.h"

namespace atr {

constexpr bool sched_stash(int sc) { return sc == SCHED_FLAT || sc == SCHED_HYBRID; }

// ------------------------------------------------------------------ cast_ray (renderer.cpp:213-262)
// Path state parked while a ray is traced (FLAT / HYBRID): the colour sums, throughput, PCG state
// and counters are dead during the tree query. HYBRID keeps them in a lane-private LDS column; FLAT
// in the lane's private (scratch) memory, so the kernel's LDS is only the scan's 22.5 KB.
constexpr int kStash = 16;

template <int SCHED, bool COUNT>
__device__ __forceinline__ V3 cast_ray(const DScene* __restrict__ S, V3 o, V3 d, int32_t bounce_limit,
                                       bool active, uint64_t& st, uint64_t stream, uint32_t& casts,
                                       uint32_t& traced, bool record, uint32_t& hit_face, float& hit_t,
                                       int& err, Ctr& ct, int32_t hyb_a, int32_t hyb_b, V3& acc) {
    constexpr bool STASH = sched_stash(SCHED);
    constexpr bool PRIV = SCHED == SCHED_FLAT;  // the stash in private memory (above)
    __shared__ uint32_t s_stash[STASH && !PRIV ? 4 : 1][PRIV ? 1 : kStash][64];
    // the private stash is indexed directly (scratch loads and stores; not volatile, which leaves
    // accesses generic: the array's address escapes into empty asm statements around the query
    // instead, which keeps its values in memory through the query)
    uint32_t pstash[PRIV ? kStash : 1];
    uint32_t* const L = &s_stash[(STASH && !PRIV) ? threadIdx.x >> 6 : 0][0][threadIdx.x & 63];
#define stash_put(k, v) do { if constexpr (PRIV) pstash[k] = (v); else L[64 * (k)] = (v); } while (0)
#define stash_get(k) (PRIV ? pstash[(PRIV ? (k) : 0)] : L[64 * (k)])
    V3 ret = mk(0.f, 0.f, 0.f), w = mk(1.f, 1.f, 1.f);
    int32_t i = 0;
    bool live = active;
    // the wave-wide scans need every lane in the loop until all lanes are done
    for (i = 0; ; ++i) {
        const bool go = live && i < bounce_limit;
        if constexpr (SCHED != SCHED_LANE) {
            if (__ballot(go) == 0) break;
        } else if (!go) break;
        if constexpr (COUNT) {
            const int bk = i < 2 ? i : 2;
            ct.steps[bk] += (threadIdx.x & 63) == 0 ? 1u : 0u;
            ct.active[bk] += go ? 1u : 0u;
        }
        Isect id;
        id.type = T_NONE;
        if constexpr (STASH) {
            stash_put(0, __float_as_uint(ret.x)); stash_put(1, __float_as_uint(ret.y));
            stash_put(2, __float_as_uint(ret.z)); stash_put(3, __float_as_uint(w.x));
            stash_put(4, __float_as_uint(w.y)); stash_put(5, __float_as_uint(w.z));
            stash_put(6, __float_as_uint(acc.x)); stash_put(7, __float_as_uint(acc.y));
            stash_put(8, __float_as_uint(acc.z));
            stash_put(9, uint32_t(st)); stash_put(10, uint32_t(st >> 32));
            stash_put(11, casts); stash_put(12, traced); stash_put(13, hit_face);
            stash_put(14, __float_as_uint(hit_t));
            if constexpr (PRIV) __asm__ volatile("" ::"s"(pstash) : "memory");
            __asm__ volatile("" ::: "memory");  // the values below come back from memory
        }
        if constexpr (SCHED == SCHED_LANE) intersect_scene<SCHED, FLAV_BOUNCE, COUNT>(S, o, d, go, id, err, ct, hyb_a, hyb_b);
        else if constexpr (SCHED == SCHED_HYBRID)
            intersect_scene<SCHED, FLAV_HYB_BOUNCE, COUNT>(S, o, d, go, id, err, ct, hyb_a, hyb_b);
        else if (i == 0)  // FLAT: the camera rays (one origin, coherent) take HYBRID's primary flavour
            intersect_scene<SCHED, FLAV_CAMERA, COUNT>(S, o, d, go, id, err, ct, hyb_a, hyb_b);
        else
            intersect_scene<SCHED, FLAV_BOUNCE, COUNT>(S, o, d, go, id, err, ct, hyb_a, hyb_b);
        if constexpr (STASH) {
            if constexpr (PRIV) __asm__ volatile("" ::"s"(pstash) : "memory");
            __asm__ volatile("" ::: "memory");
#define gf(k) __uint_as_float(stash_get(k))
            ret = mk(gf(0), gf(1), gf(2));
            w = mk(gf(3), gf(4), gf(5));
            acc = mk(gf(6), gf(7), gf(8));
            st = uint64_t(stash_get(9)) | (uint64_t(stash_get(10)) << 32);
            casts = stash_get(11); traced = stash_get(12); hit_face = stash_get(13);
            hit_t = gf(14);
        }
#undef gf
#undef stash_put
#undef stash_get
        if (!go) continue;
        ++traced;
        if (record && i == 0) { hit_face = id.face; hit_t = id.t; }
        const DMaterial& mat = S->mats[id.material];
        if (id.type == T_SKY) {  // :225-229
            ret = add(ret, had(w, mk(mat.ex, mat.ey, mat.ez)));
            live = false;
            casts += uint32_t(i);
            continue;
        }
        bounce_shade(mat, id, o, d, ret, w, st, stream);  // :231-258
    }
    if (live) casts += uint32_t(bounce_limit > 0 ? bounce_limit : 0);  // :260, ran to the limit
    return ret;
}

// PRIMARY: bounce_limit == 1, spp == 1, no AA. Then cast_ray is one intersection whose colour is
// the hit material's (or the sky's) emission; the three rand_bi draws and the bounce ray it builds
// feed only a second iteration that never runs (renderer.cpp:222-259), so they are skipped --
// output bit-identical, and far fewer live registers.
template <int SCHED, bool COUNT, bool PRIMARY, int OCC = 4>
__global__ __launch_bounds__(256, OCC) void render_kernel(RenderParams P) {
    // the wave index is uniform: in an SGPR, so are the cell and frame indices derived from it
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int b = remap_xcd(blockIdx.x, gridDim.x, P.xcd_chunk) * 4 + wave;
    if (b >= P.nblocks) return;  // whole wavefront
    // several frames per launch, interleaved: block b renders block b / nf of frame b % nf, so the
    // frames advance through the block list together (each frame's slow cells start early, and
    // neighbouring workgroups trace the same cells' rays)
    const int32_t nf = P.frame_blocks > 0 ? P.nblocks / P.frame_blocks : 1;
    const int32_t fidx = b % nf;
    int32_t bi = b / nf;
    if (P.frame_rotate && nf > 1)
        bi = int32_t((int64_t(bi) + int64_t(P.frame_blocks) * fidx * P.frame_rotate / (1024 * int64_t(nf))) %
                     P.frame_blocks);
    const DBlock blk = P.blocks[bi];
    const uint64_t mask = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
    const bool active = (mask >> lane) & 1;
    const int32_t x = blk.x0 + (lane & 7), y = blk.y0 + (lane >> 3);
    if (__builtin_amdgcn_readfirstlane(blk.flags) & kBlockPrio) __builtin_amdgcn_s_setprio(2);  // cell plan
    const uint64_t clk0 = P.block_cost ? clock64() : 0;
    uint64_t clk1 = 0;
    if constexpr (COUNT) clk1 = clock64();
#ifdef ATR_DIAG
    const uint64_t rt0 = P.wave_trace ? __builtin_amdgcn_s_memrealtime() : 0;
#endif
    // per-frame cameras (atr_render_start_cameras): fidx is wave-uniform, so the camera comes from
    // the kernel argument with scalar loads
    const atr_camera& cm = P.nfcam > 0 ? P.fcam[__builtin_amdgcn_readfirstlane(fidx)] : P.cam;
    const DScene* S = uniform_global(P.scene);  // global loads for materials, spheres, planes, shading
    int err = 0;
    Ctr ct;
    uint32_t casts = 0, traced = 0, hit_face = 0xFFFFFFFFu;
    float hit_t = kMaxFloat;
    V3 col = mk(0.f, 0.f, 0.f);
    const int64_t pix = int64_t(y) * cm.width + x;
    const float film_y = -1.0f + 2.0f * (float(y) / float(cm.height));                       // :317
    const float film_x = ((-1.0f + 2.0f * (float(x) / float(cm.width))) * cm.h_fov) * cm.aspect_ratio;  // :329
    const V3 eye = from(cm.eye), fc = from(cm.frame_center), cx = from(cm.camera_x), cy = from(cm.camera_y);
    V3 dir = mk(0.f, 0.f, 1.f);
    if (!cm.anti_aliasing) dir = unit(sub(add(add(fc, scale(cx, film_x)), scale(cy, film_y)), eye));  // :350-351
    if constexpr (PRIMARY) {
        Isect id;
        id.type = T_NONE;
        intersect_scene<SCHED, FLAV_PRIMARY, COUNT>(S, eye, dir, active, id, err, ct, P.hyb_a, P.hyb_b);
        if (active) {
            const DMaterial& mat = S->mats[id.material];
            col = add(col, mk(mat.ex, mat.ey, mat.ez));  // ret = (0 + (1,1,1) x emission)
            hit_face = id.face;
            hit_t = id.t;
            casts = id.type == T_SKY ? 0u : 1u;
            traced = 1;
        }
    } else {
        for (uint32_t s = 0; s < cm.samples_per_pixel; ++s) {
            uint64_t st, stream;
            path_stream(P.seed, pix, s, st, stream);  // one PCG stream per (pixel, sample), engine.h
            if (cm.anti_aliasing) {  // :338-343
                const float xo = rand_bi(st, stream) * cm.half_pixel_width + film_x;
                const float yo = rand_bi(st, stream) * cm.half_pixel_height + film_y;
                dir = unit(sub(add(add(fc, scale(cx, xo)), scale(cy, yo)), eye));
            }
            col = add(col, cast_ray<SCHED, COUNT>(S, eye, dir, cm.bounce_limit, active, st, stream, casts, traced,
                                                 s == 0, hit_face, hit_t, err, ct, P.hyb_a, P.hyb_b, col));
        }
    }
    // the output address from the cell record read again: the pixel coordinates and mask then hold
    // no registers through the trace (the asm clobber keeps the compiler from reusing the first read)
    DBlock ob = blk;
    __asm__ volatile("" ::: "memory");
    ob = P.blocks[bi];
    int olane = int(threadIdx.x);
    __asm__ volatile("" : "+v"(olane));  // recomputed here, not kept from the start
    olane &= 63;
    const uint64_t omask = uint64_t(ob.mask_lo) | (uint64_t(ob.mask_hi) << 32);
    if ((omask >> olane) & 1) {
        col = divs(col, float(cm.samples_per_pixel));  // :358
        const float cr = pl_max(0.0f, pl_min(col.x, 1.0f));
        const float cg = pl_max(0.0f, pl_min(col.y, 1.0f));
        const float cb = pl_max(0.0f, pl_min(col.z, 1.0f));
        const uint32_t r8 = uint32_t(cr * 255.0f) & 0xFFu, g8 = uint32_t(cg * 255.0f) & 0xFFu,
                       b8 = uint32_t(cb * 255.0f) & 0xFFu;
        size_t o;
        if (P.layout == ATR_LAYOUT_PACKED) o = size_t(ob.out_base) + __popcll(omask & ((uint64_t(1) << olane) - 1));
        else o = size_t(ob.y0 + (olane >> 3)) * size_t(cm.width) + size_t(ob.x0 + (olane & 7));
        o += size_t(fidx) * size_t(P.frame_stride);
        P.framebuffer[o] = b8 | (g8 << 8) | (r8 << 16);  // Set_Pixel (texture.h:27-38)
        if (P.hit_face) P.hit_face[o] = hit_face;
        if (P.hit_t) P.hit_t[o] = hit_t;
        if (P.rgb) { P.rgb[3 * o] = col.x; P.rgb[3 * o + 1] = col.y; P.rgb[3 * o + 2] = col.z; }
        if (P.ray_casts) P.ray_casts[o] = casts;
    }
    if (P.traced_rays) add_traced(P.traced_rays, traced, b);
    if (err && P.error_flag) atomicOr(P.error_flag, 1);
    // per-cell cost (calibration, the single-frame plan): a split cell's waves add up
    if (P.block_cost && lane == 0 && omask) atomicAdd(P.block_cost + ob.base, (unsigned long long)(clock64() - clk0));
#ifdef ATR_DIAG
    if (P.wave_trace && lane == 0) {  // diagnostic: where and when this wave ran
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        P.wave_trace[3 * size_t(b)] = rt0;
        P.wave_trace[3 * size_t(b) + 1] = __builtin_amdgcn_s_memrealtime();
        P.wave_trace[3 * size_t(b) + 2] = uint64_t(hw) | (uint64_t(xcc) << 32);
    }
#endif
    if constexpr (COUNT) {
        // counters[0..9]: rays, box(ref), tri, leaf, wave_tri_iters, passes, box_all, waves,
        // cluster boxes, screened primitives
        uint32_t v[6] = {ct.box, ct.tri, ct.leaf, ct.wave_tri, ct.pass, ct.box_all};
        unsigned long long* C = P.counters;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            uint32_t t = v[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
            if (lane == 0 && t) atomicAdd(C + 1 + k, (unsigned long long)t);
        }
        uint32_t t = traced;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
        if (lane == 0) { atomicAdd(C + 0, (unsigned long long)t); atomicAdd(C + 7, 1ull); }
        uint32_t w[2] = {ct.cbox, ct.screen};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            uint32_t x2 = w[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) x2 += __shfl_xor(x2, off);
            if (lane == 0 && x2) atomicAdd(C + 8 + k, (unsigned long long)x2);
        }
        // counters[16..21]: bounce-loop wave steps and tracing lanes, bounce 0 / 1 / >= 2
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            uint32_t a = ct.steps[k], q = ct.active[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) { a += __shfl_xor(a, off); q += __shfl_xor(q, off); }
            if (lane == 0 && a) atomicAdd(C + 16 + k, (unsigned long long)a);
            if (lane == 0 && q) atomicAdd(C + 19 + k, (unsigned long long)q);
        }
        // counters[22..26]: SIMD efficiency (candidate-loop wave iterations, DFS wave / lane
        // iterations, dealt rounds, dealt items)
        {
            uint32_t e[5] = {ct.cand_wave, ct.node_wave, ct.node_lane, ct.round_wave, ct.round_items};
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                uint32_t x2 = e[k];
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) x2 += __shfl_xor(x2, off);
                if (lane == 0 && x2) atomicAdd(C + 22 + k, (unsigned long long)x2);
            }
        }
        // counters[10..15]: wave clocks in DFS passes, lane-private scans, dealt rounds, whole
        // wave, per-step preparation, whole FLAT/HYBRID scan (phases: diagnostic build only)
        if (lane == 0) {
            atomicAdd(C + 10, (unsigned long long)ct.t_pass);
            atomicAdd(C + 11, (unsigned long long)ct.t_lp);
            atomicAdd(C + 12, (unsigned long long)ct.t_deal);
            atomicAdd(C + 13, (unsigned long long)(clock64() - clk1));
            atomicAdd(C + 14, (unsigned long long)ct.t_prep);
            atomicAdd(C + 15, (unsigned long long)ct.t_scan);
        }
    }
}

// The shipping instantiations (12): LANE {count} x {primary} + the 5-wave primary; HYBRID primaries
// at 6 (one frame) / 7 (frames in flight) waves/SIMD, its bounce-loop build and the COUNT builds;
// FLAT at 6 / 7 waves/SIMD and its COUNT build.
template __global__ void render_kernel<SCHED_LANE, false, false>(RenderParams);
template __global__ void render_kernel<SCHED_LANE, true, false>(RenderParams);
template __global__ void render_kernel<SCHED_LANE, true, true>(RenderParams);
template __global__ void render_kernel<SCHED_LANE, false, true, 5>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, false, true, 6>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, false, true, 7>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, false, true, 8>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, false, false>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, true, true>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, true, false>(RenderParams);
template __global__ void render_kernel<SCHED_FLAT, false, false, 6>(RenderParams);
template __global__ void render_kernel<SCHED_FLAT, false, false, 7>(RenderParams);
template __global__ void render_kernel<SCHED_FLAT, true, false>(RenderParams);

// Sum the 64 traced-ray counters of a launch into the caller's accumulator and clear them.
__global__ __launch_bounds__(64) void traced_finish_kernel(unsigned long long* __restrict__ slots,
                                                          unsigned long long* __restrict__ out) {
    const int lane = threadIdx.x;
    unsigned long long v = slots[16 * lane];
    slots[16 * lane] = 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0 && v) atomicAdd(out, v);
}

__global__ __launch_bounds__(256) void unpack_kernel(const DBlock* __restrict__ blocks, int32_t nblocks,
                                                     int32_t width, const uint32_t* __restrict__ packed,
                                                     uint32_t* __restrict__ image) {
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (b >= nblocks) return;
    const DBlock blk = blocks[b];
    const uint64_t mask = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
    if (!((mask >> lane) & 1)) return;
    const int32_t x = blk.x0 + (lane & 7), y = blk.y0 + (lane >> 3);
    image[size_t(y) * width + x] = packed[size_t(blk.out_base) + __popcll(mask & ((uint64_t(1) << lane) - 1))];
}

__global__ __launch_bounds__(256) void tile_casts_kernel(const atr_tile* __restrict__ tiles, int32_t width,
                                                         const uint32_t* __restrict__ casts,
                                                         int64_t* __restrict__ out) {
    const atr_tile t = tiles[blockIdx.x];
    const int32_t tw = t.max_x - t.min_x + 1, th = t.max_y - t.min_y + 1;
    int64_t acc = 0;
    for (int32_t i = threadIdx.x; i < tw * th; i += blockDim.x) {
        const int32_t x = t.min_x + i % tw, y = t.min_y + i / tw;
        acc += casts[size_t(y) * width + x];
    }
    __shared__ int64_t red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if (int(threadIdx.x) < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = red[0];
}

// Per-tile sums of a PACKED ray_casts buffer, frame blockIdx.y: slot i adds to the tile that owns
// its pixel (slot_tile, host-built per tile list). A shard tile's slots are one contiguous run, so
// a wave's 64 slots almost always share the tile: one wave reduction + one atomic per wave.
__global__ __launch_bounds__(256) void packed_tile_casts_kernel(const int32_t* __restrict__ slot_tile,
                                                                int64_t nslots,
                                                                const uint32_t* __restrict__ casts,
                                                                int64_t frame_stride, int32_t ntiles,
                                                                unsigned long long* __restrict__ out) {
    const int64_t i = int64_t(blockIdx.x) * 256 + threadIdx.x;
    const int64_t f = blockIdx.y;
    int32_t t = -1;
    unsigned long long v = 0;
    if (i < nslots) {
        t = slot_tile[i];
        v = casts[f * frame_stride + i];
    }
    const int32_t t0 = __builtin_amdgcn_readfirstlane(t);
    if (__ballot(t != t0) == 0) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if ((threadIdx.x & 63) == 0 && t0 >= 0 && v) atomicAdd(&out[f * ntiles + t0], v);
    } else if (t >= 0 && v) {
        atomicAdd(&out[f * ntiles + t], v);
    }
}

}  // namespace atr

// ------------------------------------------------------------------ launchers used by capi.cpp
template <int SC, bool C, bool PR, int OCC = 4>
static void launch_one(const atr::RenderParams& P, hipStream_t s) {
    const int grid = (P.nblocks + 3) / 4;
    hipLaunchKernelGGL((atr::render_kernel<SC, C, PR, OCC>), dim3(grid), dim3(256), 0, s, P);
}

// sched: 0 LANE, 6 FLAT, 7 HYBRID (capi.cpp sched_of). Occupancy per schedule and launch shape by
// measurement: HYBRID primaries one frame at 8 waves/SIMD, frames in flight at 7;
// primary_occ 6 / 7 / 8 overrides the choice.
extern "C" hipError_t atr_launch_render(const atr::RenderParams& P, int sched, int primary_occ, hipStream_t s) {
    using namespace atr;
    if (P.nblocks <= 0) return hipSuccess;
    if (P.traced_rays && P.counters) return hipErrorInvalidValue;  // traced_rays is a ring slot (engine.h)
    const bool count = P.counters != nullptr;
    const bool prim = P.cam.bounce_limit == 1 && !P.cam.anti_aliasing && P.cam.samples_per_pixel == 1;
    const bool multi = P.frame_blocks > 0;
    // default: frames in flight at 7 waves/SIMD, one frame at 8 (one frame alone 0.333 vs 0.345 ms
    // at 6 waves; frames in flight equal at 7 and 8)
    const int occ = primary_occ ? primary_occ : (multi ? 7 : 8);
    const bool prim7 = occ == 7;
    const bool prim8 = occ == 8;
    switch (sched) {
        case SCHED_HYBRID:
            if (count) { if (prim) launch_one<SCHED_HYBRID, true, true>(P, s); else launch_one<SCHED_HYBRID, true, false>(P, s); }
            else if (!prim) launch_one<SCHED_HYBRID, false, false>(P, s);  // LDS: 4 workgroups per CU
            else if (prim8) launch_one<SCHED_HYBRID, false, true, 8>(P, s);
            else if (prim7) launch_one<SCHED_HYBRID, false, true, 7>(P, s);
            else launch_one<SCHED_HYBRID, false, true, 6>(P, s);
            break;
        case SCHED_FLAT:
            if (prim && !count) launch_one<SCHED_HYBRID, false, true, 6>(P, s);  // primaries: HYBRID's kernel
            else if (count) { if (prim) launch_one<SCHED_HYBRID, true, true>(P, s); else launch_one<SCHED_FLAT, true, false>(P, s); }
            else if (multi) launch_one<SCHED_FLAT, false, false, 7>(P, s);
            else launch_one<SCHED_FLAT, false, false, 6>(P, s);
            break;
        case SCHED_LANE:
            if (count) { if (prim) launch_one<SCHED_LANE, true, true>(P, s); else launch_one<SCHED_LANE, true, false>(P, s); }
            else if (prim) launch_one<SCHED_LANE, false, true, 5>(P, s);
            else launch_one<SCHED_LANE, false, false>(P, s);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_traced_finish(unsigned long long* slots, unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(atr::traced_finish_kernel, dim3(1), dim3(64), 0, s, slots, out);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_unpack(const atr::DBlock* blocks, int32_t nblocks, int32_t width,
                                        const uint32_t* packed, uint32_t* image, hipStream_t s) {
    const int grid = (nblocks + 3) / 4;
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL(atr::unpack_kernel, dim3(grid), dim3(256), 0, s, blocks, nblocks, width, packed, image);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_packed_tile_casts(const int32_t* slot_tile, int64_t nslots, const uint32_t* casts,
                                                   int64_t frame_stride, int32_t nframes, int32_t ntiles,
                                                   unsigned long long* out, hipStream_t s) {
    const int64_t grid = (nslots + 255) / 256;
    if (grid <= 0 || nframes <= 0) return hipSuccess;
    hipLaunchKernelGGL(atr::packed_tile_casts_kernel, dim3(unsigned(grid), unsigned(nframes)), dim3(256), 0, s,
                       slot_tile, nslots, casts, frame_stride, ntiles, out);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_tile_casts(const atr_tile* tiles, int32_t ntiles, int32_t width,
                                            const uint32_t* casts, int64_t* out, hipStream_t s) {
    if (ntiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(atr::tile_casts_kernel, dim3(ntiles), dim3(256), 0, s, tiles, width, casts, out);
    return hipGetLastError();
}
