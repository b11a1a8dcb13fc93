// paths.hip -- the sample-parallel path engine for multi-bounce renders.
//
// render_tile_from_camera (renderer.cpp:336-358) runs a pixel's spp samples one after another,
// each a cast_ray bounce loop (:213-262). With one PCG stream per (pixel, sample) (engine.h
// path_stream) the samples are independent paths, so here every lane owns one PATH and a pixel's
// samples run side by side:
//   path_camera_kernel  one wavefront = 64 consecutive paths of one 8x8 cell (a pixel's samples
//                       together): the camera rays (one origin per wave: HYBRID's coherent flavour,
//                       scan.h), then the first shading step; a path that goes on is appended to a
//                       queue (a ballot, one atomic per wave);
//   path_bounce_kernel  bounce k of every queued path: persistent waves claim 64 queue entries at a
//                       time, trace them (FLAT's dealt rounds for incoherent rays), shade, and
//                       append the survivors to the other queue -- one launch per bounce level, so
//                       the trace holds no path state (loaded after the query) and each kernel has
//                       its own register budget;
//   path_resolve_kernel per pixel, the sample colours summed in sample order with the reference's
//                       f32 adds (col += cast_ray(...), :353-356), then average, clamp, BGRX byte
//                       conversion (:358-365) -- every output bit-identical to the cell kernels'.
// A batch is a range of the launch's cell list (PathParams, engine.h); the host runs camera,
// bounces and resolve per batch on one stream (capi.cpp launch_paths).
#include <hip/hip_runtime.h>

#include "scan.h"

#ifndef ATR_SORT_ILEAVE  // fine direction bits per side below the origin cell (0: direction, then origin)
#define ATR_SORT_ILEAVE 2
#endif


namespace atr {

// (The helpers take plain values: a reference to the kernel argument passed to a function made the
// compiler copy the whole 1.8-KB argument into scratch.)
// cell c of the launch's list -> its frame and block (frames interleaved, RenderParams)
__device__ __forceinline__ void cell_of(int32_t frame_blocks, int32_t nblocks, int32_t c, int32_t& fidx, int32_t& bi) {
    const int32_t nf = frame_blocks > 0 ? nblocks / frame_blocks : 1;
    fidx = c % nf;
    bi = c / nf;
}

__device__ __forceinline__ size_t out_index(int32_t layout, int32_t width, int64_t frame_stride, const DBlock& blk,
                                            uint64_t mask, int pl, int32_t fidx) {
    size_t o;
    if (layout == ATR_LAYOUT_PACKED) o = size_t(blk.out_base) + __popcll(mask & ((uint64_t(1) << pl) - 1));
    else o = size_t(blk.y0 + (pl >> 3)) * size_t(width) + size_t(blk.x0 + (pl & 7));
    return o + size_t(fidx) * size_t(frame_stride);
}

// A finished path: its colour (cast_ray's ret) and the reference's ray_casts (renderer.cpp:260),
// at its result slot o (cell x 64 spp + sample x 64 + pixel lane: the resolve's lanes read a
// sample's 64 results as one coalesced 1-KB row).
__device__ __forceinline__ void path_finish(float4_t* out, uint32_t o, V3 ret, uint32_t casts) {
    out[o] = float4_t{ret.x, ret.y, ret.z, __uint_as_float(casts)};
}

// Without AA every sample of a pixel casts the same camera ray (renderer.cpp:348-357), so when it
// meets the sky every sample's path ends there with the same colour and no ray_casts. Then only
// sample 0 writes its result slot, with this marker in place of the count (a real count is at most
// the bounce limit), and the resolve takes that colour for every sample: c4 skips ~86% of the
// camera kernel's result writes and of the resolve's reads; the sum is the same f32 adds.
constexpr uint32_t kAllSky = 0xFFFFFFFFu;
#ifndef ATR_SKY_ELIDE  // experiment builds: 0 = every sample writes its result slot (round 5)
#define ATR_SKY_ELIDE 1
#endif

// Sort key of a queued ray (PathSort, engine.h): the octahedral cell of its direction (kSortDirs x
// kSortDirs over the unfolded octahedron) and the Morton code of its origin's cell, b bits per axis
// over the scene box, interleaved as below.
__device__ __forceinline__ uint32_t spread3(uint32_t x) {  // bits 0..9 -> every third bit
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    return (x | (x << 2)) & 0x09249249u;
}
__device__ __forceinline__ uint32_t path_sort_key(V3 o, V3 d, PathSort so) {
    const float qmax = float((1 << so.bits) - 1);
    // fmaxf first: a NaN coordinate lands in cell 0
    const uint32_t qx = uint32_t(fminf(fmaxf((o.x - so.lo[0]) * so.sc[0], 0.0f), qmax));
    const uint32_t qy = uint32_t(fminf(fmaxf((o.y - so.lo[1]) * so.sc[1], 0.0f), qmax));
    const uint32_t qz = uint32_t(fminf(fmaxf((o.z - so.lo[2]) * so.sc[2], 0.0f), qmax));
    const uint32_t morton = (spread3(qx) << 2) | (spread3(qy) << 1) | spread3(qz);
    // octahedral direction: (x, y) / (|x| + |y| + |z|), the lower hemisphere folded out
    const float sum = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    float u = d.x / sum, v = d.y / sum;
    if (d.z < 0.0f) {
        const float uu = (1.0f - fabsf(v)) * (u >= 0.0f ? 1.0f : -1.0f);
        v = (1.0f - fabsf(u)) * (v >= 0.0f ? 1.0f : -1.0f);
        u = uu;
    }
    constexpr float D = float(kSortDirs);
    const uint32_t iu = uint32_t(fminf(fmaxf((u * 0.5f + 0.5f) * D, 0.0f), D - 1.0f));
    const uint32_t iv = uint32_t(fminf(fmaxf((v * 0.5f + 0.5f) * D, 0.0f), D - 1.0f));
    // coarse direction cell (the low F bits of iu, iv dropped), origin cell, then the fine bits:
    // a run of the order is one coarse direction and one region, fine directions side by side
    // (F = 2 of the 16 x 16 map: c4 +1.2%, c5 +1.5% over direction cell, then origin)
    constexpr int F = ATR_SORT_ILEAVE;
    const uint32_t coarse = (iv >> F) * uint32_t(kSortDirs >> F) + (iu >> F);
    const uint32_t fine = ((iv & ((1u << F) - 1u)) << F) | (iu & ((1u << F) - 1u));
    return (((coarse << (3 * so.bits)) | morton) << (2 * F)) | fine;
}

// Append this lane's path (if `go`) to queue q (planes `cap` entries apart): one atomic per wave for
// the wave's survivors, each at base + its rank among them. With the queue sort on, the entry also
// records its key and its rank in the key's bin (PathSort).
template <bool SORT>
__device__ __forceinline__ void path_enqueue(float4_t* q, int64_t cap, PathCtl* ctl, bool go, V3 o, V3 d,
                                             uint32_t pix, uint32_t g, V3 ret, V3 w, uint64_t st, PathSort so) {
    const uint64_t m = __ballot(go);
    if (m == 0) return;
    const int lane = threadIdx.x & 63;
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&ctl->tail, uint32_t(__popcll(m)));
    base = uint32_t(__builtin_amdgcn_readfirstlane(int(__shfl(int(base), 0))));
    if (!go) return;
    const int64_t e = int64_t(base) + __popcll(m & ((uint64_t(1) << lane) - 1));
    // sorted queues hold each entry's four records together (64 B, entry-major: q[4 e + i]) so the
    // sort moves whole 64-B blocks; unsorted queues keep the four planes (q[i cap + e])
    const int64_t e0 = SORT ? 4 * e : e, es = SORT ? 1 : cap;
    if constexpr (SORT) {
        const uint32_t key = path_sort_key(o, d, so);
        so.kr[e] = uint2_t{key, atomicAdd(so.hist + key, 1u)};
    }
    q[e0] = float4_t{o.x, o.y, o.z, d.x};
    q[es + e0] = float4_t{d.y, d.z, __uint_as_float(pix), __uint_as_float(g)};
    q[2 * es + e0] = float4_t{ret.x, ret.y, ret.z, w.x};
    q[3 * es + e0] = float4_t{w.y, w.z, __uint_as_float(uint32_t(st)), __uint_as_float(uint32_t(st >> 32))};
}

template <bool COUNT>
__device__ __forceinline__ void path_counters(unsigned long long* C, const Ctr& ct, uint32_t traced) {
    const int lane = threadIdx.x & 63;
    uint32_t v[10] = {traced, ct.box, ct.tri, ct.leaf, ct.wave_tri, ct.pass, ct.box_all, 0u, ct.cbox, ct.screen};
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        uint32_t t = v[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
        if (lane == 0 && t) atomicAdd(C + k, (unsigned long long)t);
    }
    if (lane == 0) atomicAdd(C + 7, 1ull);
    // [10..15] wave clocks of the scan phases (DIAG build only; zero otherwise), [22..26] SIMD use
    if (lane == 0) {
        atomicAdd(C + 10, (unsigned long long)ct.t_pass);
        atomicAdd(C + 11, (unsigned long long)ct.t_lp);
        atomicAdd(C + 12, (unsigned long long)ct.t_deal);
        atomicAdd(C + 14, (unsigned long long)ct.t_prep);
        atomicAdd(C + 15, (unsigned long long)ct.t_scan);
    }
    uint32_t e[5] = {ct.cand_wave, ct.node_wave, ct.node_lane, ct.round_wave, ct.round_items};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        uint32_t x = e[k];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        if (lane == 0 && x) atomicAdd(C + 22 + k, (unsigned long long)x);
    }
}

// ------------------------------------------------------------------ camera rays + first shading
template <bool COUNT, int OCC, bool SORT>
__global__ __launch_bounds__(256, OCC) void path_camera_kernel(PathParams P) {
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const uint32_t spp = uint32_t(__builtin_amdgcn_readfirstlane(int(P.cam.samples_per_pixel)));
    const int64_t wv = int64_t(remap_xcd(blockIdx.x, gridDim.x, P.xcd_chunk)) * 4 + wave;  // wave of the batch
    if (wv >= int64_t(P.ncells) * spp) return;  // whole wavefront
    // a cell's 64 x spp paths are spp consecutive waves: the cell is wave-uniform
    const int32_t cellrel = int32_t(wv / spp);
    const uint32_t r = uint32_t(wv - int64_t(cellrel) * spp) * 64u + uint32_t(lane);  // path within the cell
    const int pl = int(r / spp);  // the pixel's lane in the 8x8 cell
    const uint32_t s = r - uint32_t(pl) * spp;  // its sample
    const uint32_t g = uint32_t(cellrel) * 64u * spp + s * 64u + uint32_t(pl);  // result slot
    int32_t fidx, bi;
    cell_of(P.frame_blocks, P.nblocks, P.cell0 + cellrel, fidx, bi);
    const DBlock blk = P.blocks[bi];
    const uint64_t mask = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
    const atr_camera& cm = P.nfcam > 0 ? P.fcam[__builtin_amdgcn_readfirstlane(fidx)] : P.cam;
    const int32_t bl = cm.bounce_limit;
    const bool active = ((mask >> pl) & 1) && bl > 0;
    const uint64_t clk0 = P.block_cost ? clock64() : 0;
    const DScene* S = uniform_global(P.scene);
    const int32_t x = blk.x0 + (pl & 7), y = blk.y0 + (pl >> 3);
    const int64_t pix = int64_t(y) * cm.width + x;
    uint64_t st, stream;
    path_stream(P.seed, pix, s, st, stream);
    const float film_y = -1.0f + 2.0f * (float(y) / float(cm.height));                                  // :317
    const float film_x = ((-1.0f + 2.0f * (float(x) / float(cm.width))) * cm.h_fov) * cm.aspect_ratio;  // :329
    const V3 eye = from(cm.eye), fc = from(cm.frame_center), cx = from(cm.camera_x), cy = from(cm.camera_y);
    V3 d;
    if (cm.anti_aliasing) {  // :338-347, the sample's two jitter draws
        const float xo = rand_bi(st, stream) * cm.half_pixel_width + film_x;
        const float yo = rand_bi(st, stream) * cm.half_pixel_height + film_y;
        d = unit(sub(add(add(fc, scale(cx, xo)), scale(cy, yo)), eye));
    } else {
        d = unit(sub(add(add(fc, scale(cx, film_x)), scale(cy, film_y)), eye));  // :350-351
    }
    int err = 0;
    Ctr ct;
    Isect id;
    id.type = T_NONE;
    intersect_scene<SCHED_HYBRID, FLAV_CAMERA, COUNT>(S, eye, d, active, id, err, ct, P.hyb_a, P.hyb_b);
    bool go = false;
    V3 o = eye, ret = mk(0.f, 0.f, 0.f), w = mk(1.f, 1.f, 1.f);
    if (active) {
        if (s == 0) {  // sample 0's camera ray: the primary hit outputs
            const size_t oi = out_index(P.layout, cm.width, P.frame_stride, blk, mask, pl, fidx);
            if (P.hit_face) P.hit_face[oi] = id.face;
            if (P.hit_t) P.hit_t[oi] = id.t;
        }
        const DMaterial& mat = S->mats[id.material];
        if (id.type == T_SKY) {  // :225-229 at i = 0
            ret = add(ret, had(w, mk(mat.ex, mat.ey, mat.ez)));
            if (cm.anti_aliasing || !ATR_SKY_ELIDE) path_finish(P.out, g, ret, 0u);
            else if (s == 0) path_finish(P.out, g, ret, kAllSky);  // the pixel's every sample (kAllSky)
        } else {
            bounce_shade(mat, id, o, d, ret, w, st, stream);  // :231-258
            if (bl <= 1) path_finish(P.out, g, ret, uint32_t(bl));  // ran to the limit (:260)
            else go = true;
        }
    }
    path_enqueue<SORT>(P.q[0], P.cap, &P.ctl[0], go, o, d, uint32_t(pix), g, ret, w, st, P.sort);
    const uint32_t traced = active ? 1u : 0u;
    if (P.traced_rays) add_traced(P.traced_rays, traced, int(wv));
    if (err && P.error_flag) atomicOr(P.error_flag, 1);
    if (P.block_cost && lane == 0) atomicAdd(P.block_cost + blk.base, (unsigned long long)(clock64() - clk0));
    if constexpr (COUNT) path_counters<COUNT>(P.counters, ct, traced);
}

// ------------------------------------------------------------------ bounce k of the queued paths
// Leaf buffer entries of the bounce rays' queries (the scan is templated on it). 6 entries cut the
// LDS to 18 KB per workgroup, enough for 8 waves/SIMD, but cost re-walks: c4 71.0 ms per frame at 7
// waves and 72.1 at 8 (64 VGPRs, scratch in the hot loop) vs 69.5 with 8 entries.
#ifndef ATR_BOUNCE_LEAFBUF
#define ATR_BOUNCE_LEAFBUF kLeafBuf
#endif
constexpr int kBounceLeafBuf = ATR_BOUNCE_LEAFBUF;  // experiment builds: -DATR_BOUNCE_LEAFBUF=6
template <bool COUNT, int OCC, bool SORT>
__global__ __launch_bounds__(256, OCC) void path_bounce_kernel(PathParams P) {
    const int lane = threadIdx.x & 63;
    const int32_t k = P.bounce;  // 1 .. bounce_limit - 1
    const int32_t bl = P.cam.bounce_limit;
    const float4_t* __restrict__ qin = P.q[(k - 1) & 1];
    const uint32_t n = uint32_t(__builtin_amdgcn_readfirstlane(int(P.ctl[k - 1].tail)));
    const DScene* S = uniform_global(P.scene);
    const uint32_t spp = P.cam.samples_per_pixel;
    int err = 0;
    Ctr ct;
    uint32_t traced = 0;
    for (;;) {  // every wave leaves once the queue is claimed: the exit every wave reaches
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&P.ctl[k].head, 64u);
        base = uint32_t(__builtin_amdgcn_readfirstlane(int(__shfl(int(base), 0))));
        if (base >= n) break;
        const uint64_t clk0 = P.block_cost ? clock64() : 0;
        const uint32_t i = base + uint32_t(lane);
        const bool valid = i < n;
        // sorted queues: claimed position i of the level's key order -> its entry (PathSort)
        uint32_t e = i;
        if (SORT && valid) e = P.sort.perm[i];
        V3 o = mk(0.f, 0.f, 0.f), d = mk(0.f, 0.f, 1.f);
        if (valid) {
            const float4_t a = qin[SORT ? 4 * int64_t(e) : e], b = qin[SORT ? 4 * int64_t(e) + 1 : P.cap + e];
            o = mk(a.x, a.y, a.z);
            d = mk(a.w, b.x, b.y);
        }
        const SceneHit sh = intersect_models<SCHED_FLAT, FLAV_BOUNCE, COUNT, kBounceLeafBuf>(S, o, d, valid, err, ct, P.hyb_a, P.hyb_b);
        // the path -- its ray too -- is read again after the query instead of being held through
        // it: the memory clobber keeps the loads here, the opaque copy of the entry index keeps
        // their addresses from being formed before the query
        uint32_t ea = e;
        __asm__ volatile("" : "+v"(ea) :: "memory");
        bool go = false;
        uint32_t pix = 0, g = 0;
        V3 ret = mk(0.f, 0.f, 0.f), w = mk(1.f, 1.f, 1.f);
        uint64_t st = 0;
        if (valid) {
            traced += 1;
            const int64_t e0 = SORT ? 4 * int64_t(ea) : ea, es = SORT ? 1 : P.cap;
            const float4_t a = qin[e0], b = qin[es + e0], c = qin[2 * es + e0], q3 = qin[3 * es + e0];
            o = mk(a.x, a.y, a.z);
            d = mk(a.w, b.x, b.y);
            Isect id;
            scene_finish(S, o, d, sh.best, sh.face, sh.fu, sh.fv, sh.nm, id);  // renderer.cpp:86-160
            pix = __float_as_uint(b.z);
            g = __float_as_uint(b.w);
            ret = mk(c.x, c.y, c.z);
            w = mk(c.w, q3.x, q3.y);
            st = uint64_t(__float_as_uint(q3.z)) | (uint64_t(__float_as_uint(q3.w)) << 32);
            const uint64_t stream = (uint64_t(pix) << 1) | 1ULL;
            const DMaterial& mat = S->mats[id.material];
            if (id.type == T_SKY) {  // :225-229 at i = k
                ret = add(ret, had(w, mk(mat.ex, mat.ey, mat.ez)));
                path_finish(P.out, g, ret, uint32_t(k));
            } else {
                bounce_shade(mat, id, o, d, ret, w, st, stream);  // :231-258
                if (k + 1 >= bl) path_finish(P.out, g, ret, uint32_t(bl));  // ran to the limit (:260)
                else go = true;
            }
            if (P.block_cost) {  // calibration: the chunk's clocks split over its paths' cells
                const int32_t c = P.cell0 + int32_t(g / (64u * spp));
                int32_t fidx, bi;
                cell_of(P.frame_blocks, P.nblocks, c, fidx, bi);
                const uint32_t nv = n - base < 64u ? n - base : 64u;
                atomicAdd(P.block_cost + P.blocks[bi].base, (unsigned long long)((clock64() - clk0) / nv));
            }
        }
        path_enqueue<SORT>(P.q[k & 1], P.cap, &P.ctl[k], go, o, d, pix, g, ret, w, st, P.sort);
    }
    if (P.traced_rays) add_traced(P.traced_rays, traced, int(blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (err && P.error_flag) atomicOr(P.error_flag, 1);
    if constexpr (COUNT) path_counters<COUNT>(P.counters, ct, traced);
}

// ------------------------------------------------------------------ per-pixel resolve
__global__ __launch_bounds__(256) void path_resolve_kernel(PathParams P) {
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int32_t cellrel = int32_t(blockIdx.x) * 4 + wave;
    if (cellrel >= P.ncells) return;
    int32_t fidx, bi;
    cell_of(P.frame_blocks, P.nblocks, P.cell0 + cellrel, fidx, bi);
    const DBlock blk = P.blocks[bi];
    const uint64_t mask = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
    if (!((mask >> lane) & 1)) return;
    const atr_camera& cm = P.nfcam > 0 ? P.fcam[__builtin_amdgcn_readfirstlane(fidx)] : P.cam;
    const uint32_t spp = cm.samples_per_pixel;
    const bool traced = cm.bounce_limit > 0;
    const float4_t* src = P.out + int64_t(cellrel) * 64 * int64_t(spp) + lane;
    V3 col = mk(0.f, 0.f, 0.f);
    uint32_t casts = 0;
    // sample 0 first: kAllSky = every sample of the pixel met the sky with this colour
    const float4_t v0 = traced && spp > 0 ? src[0] : float4_t{0.f, 0.f, 0.f, 0.f};
    const bool all_sky = traced && spp > 0 && !cm.anti_aliasing && __float_as_uint(v0.w) == kAllSky;
    for (uint32_t s = 0; s < spp; ++s) {  // col += cast_ray(...) in sample order (:353-356)
        V3 c = mk(0.f, 0.f, 0.f);
        if (all_sky) {
            c = mk(v0.x, v0.y, v0.z);
        } else if (traced) {
            const float4_t v = s == 0 ? v0 : src[64 * int64_t(s)];
            c = mk(v.x, v.y, v.z);
            casts += __float_as_uint(v.w);
        }
        col = add(col, c);
    }
    col = divs(col, float(spp));  // :358
    const float cr = pl_max(0.0f, pl_min(col.x, 1.0f));
    const float cg = pl_max(0.0f, pl_min(col.y, 1.0f));
    const float cb = pl_max(0.0f, pl_min(col.z, 1.0f));
    const uint32_t r8 = uint32_t(cr * 255.0f) & 0xFFu, g8 = uint32_t(cg * 255.0f) & 0xFFu,
                   b8 = uint32_t(cb * 255.0f) & 0xFFu;
    const size_t o = out_index(P.layout, cm.width, P.frame_stride, blk, mask, lane, fidx);
    P.framebuffer[o] = b8 | (g8 << 8) | (r8 << 16);  // Set_Pixel (texture.h:27-38)
    if (!traced || spp == 0) {  // no camera ray ran: the miss record
        if (P.hit_face) P.hit_face[o] = 0xFFFFFFFFu;
        if (P.hit_t) P.hit_t[o] = kMaxFloat;
    }
    if (P.rgb) { P.rgb[3 * o] = col.x; P.rgb[3 * o + 1] = col.y; P.rgb[3 * o + 2] = col.z; }
    if (P.ray_casts) P.ray_casts[o] = casts;
}

// ------------------------------------------------------------------ queue sort (PathSort)
// Level k's bins: block b sums hist[b x kSortChunk ..) into part[b].
__global__ __launch_bounds__(256) void path_sort_sums(PathSort so) {
    const uint4_t* h = reinterpret_cast<const uint4_t*>(so.hist + int64_t(blockIdx.x) * kSortChunk);
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < kSortChunk / 1024; ++i) {
        const uint4_t v = h[i * 256 + threadIdx.x];
        t += v.x + v.y + v.z + v.w;
    }
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    __shared__ uint32_t ws[4];
    if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = t;
    __syncthreads();
    if (threadIdx.x == 0) so.part[blockIdx.x] = ws[0] + ws[1] + ws[2] + ws[3];
}

// The block sums' exclusive scan, in place (one workgroup; nbins / kSortChunk <= 2^15 sums).
__global__ __launch_bounds__(1024) void path_sort_part_scan(PathSort so) {
    __shared__ uint32_t ws[16];
    const int n = so.nbins / kSortChunk, per = (n + 1023) / 1024;
    const int i0 = int(threadIdx.x) * per, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t t = 0;
    for (int i = i0; i < i0 + per && i < n; ++i) t += so.part[i];
    uint32_t inc = t;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t run = inc - t;
    for (int w = 0; w < wave; ++w) run += ws[w];
    for (int i = i0; i < i0 + per && i < n; ++i) {
        const uint32_t v = so.part[i];
        so.part[i] = run;
        run += v;
    }
}

// Block b: its bins' exclusive starts (its block's start, then a scan of its own kSortChunk bins,
// 16 per thread), and the bins zeroed for the next level.
__global__ __launch_bounds__(256) void path_sort_scan(PathSort so) {
    __shared__ uint32_t ws[4];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t pre = so.part[blockIdx.x];
    uint4_t* h = reinterpret_cast<uint4_t*>(so.hist + int64_t(blockIdx.x) * kSortChunk) + 4 * threadIdx.x;
    uint4_t* st = reinterpret_cast<uint4_t*>(so.start + int64_t(blockIdx.x) * kSortChunk) + 4 * threadIdx.x;
    uint4_t v[4];
    uint32_t t = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[i] = h[i];
        t += v[i].x + v[i].y + v[i].z + v[i].w;
    }
    uint32_t inc = t;  // inclusive scan over the wave, then over the four waves
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(inc, off);
        if (lane >= off) inc += y;
    }
    if (lane == 63) ws[wave] = inc;
    __syncthreads();
    uint32_t run = pre + inc - t;
    for (int w = 0; w < wave; ++w) run += ws[w];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        uint4_t o;
        o.x = run; run += v[i].x;
        o.y = run; run += v[i].y;
        o.z = run; run += v[i].z;
        o.w = run; run += v[i].w;
        st[i] = o;
        h[i] = uint4_t{0u, 0u, 0u, 0u};
    }
}

// Level k's key order: perm[start[key] + rank] = entry, for every entry of the level (grid-stride
// over its tail). A slot outside the tail, impossible for consistent keys and ranks, is flagged.
__global__ __launch_bounds__(256) void path_sort_rank(PathParams P) {
    const int32_t k = P.bounce;
    const uint32_t n = uint32_t(__builtin_amdgcn_readfirstlane(int(P.ctl[k].tail)));
    const PathSort so = P.sort;
    // four entries per lane per step: their loads in flight together (c4 +0.2% over one)
    constexpr int U = 4;
    const uint32_t stride = gridDim.x * 256u;
    for (uint32_t e0 = blockIdx.x * 256u + threadIdx.x; e0 < n; e0 += U * stride) {
        uint2_t kr[U];
        uint32_t st[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t e = e0 + uint32_t(j) * stride;
            kr[j] = e < n ? so.kr[e] : uint2_t{0u, 0u};
        }
#pragma unroll
        for (int j = 0; j < U; ++j) st[j] = so.start[kr[j].x];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const uint32_t e = e0 + uint32_t(j) * stride;
            const uint32_t dst = st[j] + kr[j].y;
            if (e >= n) continue;
            if (dst < n) so.perm[dst] = e;
            else if (P.error_flag) atomicOr(P.error_flag, 2);
        }
    }
}

// Occupancy (waves/SIMD) of the two trace kernels, 5..7 (the LDS limit is 7: 22.5 KB per
// workgroup); tuning path_camera_occ / path_bounce_occ pick another (0 = these defaults). The
// camera kernel at 7 spills 21 dwords whose write-backs reach HBM (14.9 GB per c4 frame against
// 4.6 GB at 6) and is no faster.
constexpr int kCameraOcc = 6;
#ifndef ATR_BOUNCE_OCC
#define ATR_BOUNCE_OCC 7
#endif
constexpr int kBounceOcc = ATR_BOUNCE_OCC;
#if ATR_BOUNCE_OCC == 8  // experiment: the bounce kernel at 8 waves/SIMD (needs a 6-leaf buffer's LDS)
#define ATR_PATH_BOUNCE8(SORT) template __global__ void path_bounce_kernel<false, 8, SORT>(PathParams);
#else
#define ATR_PATH_BOUNCE8(SORT)
#endif
#define ATR_PATH_KERNELS(SORT)                                                  \
    template __global__ void path_camera_kernel<false, 5, SORT>(PathParams);    \
    template __global__ void path_camera_kernel<false, 6, SORT>(PathParams);    \
    template __global__ void path_camera_kernel<false, 7, SORT>(PathParams);    \
    template __global__ void path_camera_kernel<true, 4, SORT>(PathParams);     \
    template __global__ void path_bounce_kernel<false, 5, SORT>(PathParams);    \
    template __global__ void path_bounce_kernel<false, 6, SORT>(PathParams);    \
    template __global__ void path_bounce_kernel<false, 7, SORT>(PathParams);    \
    ATR_PATH_BOUNCE8(SORT)                                                      \
    template __global__ void path_bounce_kernel<true, 4, SORT>(PathParams);
ATR_PATH_KERNELS(false)
ATR_PATH_KERNELS(true)
#undef ATR_PATH_KERNELS

}  // namespace atr

// ------------------------------------------------------------------ launchers used by capi.cpp
namespace {
template <bool SORT>
void launch_camera(const atr::PathParams& P, int occ, dim3 g, hipStream_t s) {
    const dim3 b(256);
    if (P.counters) hipLaunchKernelGGL((atr::path_camera_kernel<true, 4, SORT>), g, b, 0, s, P);
    else if (occ == 5) hipLaunchKernelGGL((atr::path_camera_kernel<false, 5, SORT>), g, b, 0, s, P);
    else if (occ == 6) hipLaunchKernelGGL((atr::path_camera_kernel<false, 6, SORT>), g, b, 0, s, P);
    else hipLaunchKernelGGL((atr::path_camera_kernel<false, 7, SORT>), g, b, 0, s, P);
}
template <bool SORT>
void launch_bounce(const atr::PathParams& P, int occ, dim3 g, hipStream_t s) {
    const dim3 b(256);
    if (P.counters) hipLaunchKernelGGL((atr::path_bounce_kernel<true, 4, SORT>), g, b, 0, s, P);
    else if (occ == 5) hipLaunchKernelGGL((atr::path_bounce_kernel<false, 5, SORT>), g, b, 0, s, P);
    else if (occ == 6) hipLaunchKernelGGL((atr::path_bounce_kernel<false, 6, SORT>), g, b, 0, s, P);
#if ATR_BOUNCE_OCC == 8
    else if (occ == 8) hipLaunchKernelGGL((atr::path_bounce_kernel<false, 8, SORT>), g, b, 0, s, P);
#endif
    else hipLaunchKernelGGL((atr::path_bounce_kernel<false, 7, SORT>), g, b, 0, s, P);
}
}  // namespace

// With P.sort.bits > 0 the launch reads and writes entry-major queues and its survivors record
// their sort keys and ranks (the queue sort, PathSort).
extern "C" hipError_t atr_launch_path_camera(const atr::PathParams& P, int occ, hipStream_t s) {
    const int64_t waves = int64_t(P.ncells) * P.cam.samples_per_pixel;
    if (waves <= 0) return hipSuccess;
    const dim3 g(unsigned((waves + 3) / 4));
    if (!occ) occ = atr::kCameraOcc;
    if (P.sort.bits) launch_camera<true>(P, occ, g, s);
    else launch_camera<false>(P, occ, g, s);
    return hipGetLastError();
}

// Persistent: `ncu` x occupancy workgroups (4 waves each, one per SIMD) claim the queue 64 entries
// at a time.
extern "C" hipError_t atr_launch_path_bounce(const atr::PathParams& P, int ncu, int occ, hipStream_t s) {
    if (!occ) occ = atr::kBounceOcc;
    const dim3 g(unsigned(ncu) * unsigned(P.counters ? 4 : occ));
    if (P.sort.bits) launch_bounce<true>(P, occ, g, s);
    else launch_bounce<false>(P, occ, g, s);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_path_sort(const atr::PathParams& P, int ncu, hipStream_t s) {
    const unsigned blocks = unsigned(P.sort.nbins / atr::kSortChunk);
    hipLaunchKernelGGL(atr::path_sort_sums, dim3(blocks), dim3(256), 0, s, P.sort);
    hipLaunchKernelGGL(atr::path_sort_part_scan, dim3(1), dim3(1024), 0, s, P.sort);
    hipLaunchKernelGGL(atr::path_sort_scan, dim3(blocks), dim3(256), 0, s, P.sort);
    hipLaunchKernelGGL(atr::path_sort_rank, dim3(unsigned(ncu) * 16u), dim3(256), 0, s, P);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_path_resolve(const atr::PathParams& P, hipStream_t s) {
    if (P.ncells <= 0) return hipSuccess;
    hipLaunchKernelGGL(atr::path_resolve_kernel, dim3(unsigned((P.ncells + 3) / 4)), dim3(256), 0, s, P);
    return hipGetLastError();
}
