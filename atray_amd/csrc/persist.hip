// persist.hip -- the PERSIST schedule (the default): persistent waves whose lanes refill.
//
// The 8x8-cell schedules (render.hip) retire a wavefront only when its slowest ray is done. On
// Dragon 1920x1080 the median active wave lives 0.17 ms and the slowest 1.05 ms, so after the
// first third of a launch most SIMDs idle while those waves finish (tools/wave_trace.py,
// DESIGN.md §4c). Here a fixed grid of waves stays resident and every lane runs its pixel as a
// small state machine
//
//   FETCH -> QUERY (model: root box) -> TRAV (one octree pass: K sorted leaves)
//         -> SCAN (one leaf per step; then the next leaf, a re-walk or query done)
//         -> next model ... -> SHADE (spheres, planes, normal; next bounce, sample or pixel out)
//
// and takes the next pixel from a work queue when its pixel is done, so the wave's 64 lanes stay
// busy until the render runs out of pixels. Queues are per XCD: the render's 8x8 cells are dealt
// to them in chunks (neighbouring cells share an XCD and its L2); a wave whose queue is dry
// steals from the others. Per-ray arithmetic is the CLUSTER schedule's device code in the same
// order, so every output is bit-identical to it (and to the reference).
#include <hip/hip_runtime.h>

#include "cluster.h"
#include "shade.h"

namespace atr {

enum : int32_t { PH_FETCH = 0, PH_QUERY = 1, PH_TRAV = 2, PH_SCAN = 3, PH_SHADE = 4, PH_DONE = 5 };
#ifndef ATR_PERSIST_REFILL
#define ATR_PERSIST_REFILL 16
#endif
#ifndef ATR_PERSIST_TRAV
#define ATR_PERSIST_TRAV 16
#endif
#ifndef ATR_PERSIST_K
#define ATR_PERSIST_K 8
#endif
constexpr int kRefill = ATR_PERSIST_REFILL;  // refill once this many lanes are idle (or none has work)
constexpr int kQueueStride = 32;  // u32 words between queue heads (one 128-B line each)
constexpr int kPersistOcc = 4;    // waves per SIMD
constexpr int kTravBatch = ATR_PERSIST_TRAV;  // lanes waiting for an octree pass before the wave runs one
constexpr int kPersistK = ATR_PERSIST_K;      // sorted leaves buffered per pass

// Queue x serves the cells of chunks x, x + 8, x + 16, ... (cb cells per chunk), 64 items (lanes)
// per cell, in cell order.
__device__ __forceinline__ int32_t queue_items(int32_t x, int32_t ncells, int32_t cb) {
    const int32_t nc = (ncells + cb - 1) / cb;
    if (x >= nc) return 0;
    int32_t cells = ((nc - 1 - x) / 8 + 1) * cb;
    if ((nc - 1 - x) % 8 == 0) cells -= nc * cb - ncells;  // x holds the last, partial chunk
    return cells * 64;
}
__device__ __forceinline__ int32_t queue_cell(int32_t x, int32_t j, int32_t cb) {
    return (x + 8 * (j / (cb * 64))) * cb + (j / 64) % cb;
}

template <int K>
struct Lane {
    int32_t ph;
    int32_t px, out;      // pixel index y * width + x, output slot
    uint32_t s, bounce;   // current sample and bounce
    uint64_t rng;
    V3 col, ret, w;       // sum over samples; the sample's colour and weight (cast_ray)
    uint32_t casts, traced, hface, total;
    float ht;
    Ray r;
    int32_t mi, nm;       // model being queried; nearest model so far
    float best, fu, fv;   // closest over the models (renderer.cpp:47-84)
    uint32_t face;
    LeafBuf<K> lb;        // tree query of model mi
    int32_t nb;
    bool more;
    float bd;
    int32_t bi;
    LeafHit h;
    uint32_t c, cend;     // clusters of the leaf being scanned
};

__device__ __forceinline__ uint64_t stream_of(int32_t px) { return (uint64_t(uint32_t(px)) << 1) | 1ULL; }

template <int K>
__device__ __forceinline__ void begin_ray(Lane<K>& L, V3 o, V3 d) {
    L.r = make_ray(o, d);  // renderer.cpp:41-44
    L.mi = 0;
    L.nm = -1;
    L.best = kMaxFloat;
    L.face = 0;
    L.fu = L.fv = 0.f;
    L.ph = PH_QUERY;
}

// The sample's primary ray (renderer.cpp:336-356); cast_ray starts with weight 1.
template <int K>
__device__ __forceinline__ void begin_sample(Lane<K>& L, const atr_camera& cm) {
    const int32_t x = L.px % cm.width, y = L.px / cm.width;
    const float film_y = -1.0f + 2.0f * (float(y) / float(cm.height));                       // :317
    const float film_x = ((-1.0f + 2.0f * (float(x) / float(cm.width))) * cm.h_fov) * cm.aspect_ratio;  // :329
    const V3 eye = from(cm.eye), fc = from(cm.frame_center), cx = from(cm.camera_x), cy = from(cm.camera_y);
    V3 dir;
    if (cm.anti_aliasing) {  // :338-343
        const uint64_t st = stream_of(L.px);
        const float xo = rand_bi(L.rng, st) * cm.half_pixel_width + film_x;
        const float yo = rand_bi(L.rng, st) * cm.half_pixel_height + film_y;
        dir = unit(sub(add(add(fc, scale(cx, xo)), scale(cy, yo)), eye));
    } else {
        dir = unit(sub(add(add(fc, scale(cx, film_x)), scale(cy, film_y)), eye));  // :350-351
    }
    L.ret = mk(0.f, 0.f, 0.f);
    L.w = mk(1.f, 1.f, 1.f);
    L.bounce = 0;
    begin_ray(L, eye, dir);
}

// Average, clamp, quantize and store the pixel (renderer.cpp:358-365, texture.h:27-38).
template <int K>
__device__ __forceinline__ void pixel_out(Lane<K>& L, const RenderParams& P) {
    const V3 col = divs(L.col, float(P.cam.samples_per_pixel));
    const float cr = pl_max(0.0f, pl_min(col.x, 1.0f));
    const float cg = pl_max(0.0f, pl_min(col.y, 1.0f));
    const float cb = pl_max(0.0f, pl_min(col.z, 1.0f));
    const uint32_t r8 = uint32_t(cr * 255.0f) & 0xFFu, g8 = uint32_t(cg * 255.0f) & 0xFFu,
                   b8 = uint32_t(cb * 255.0f) & 0xFFu;
    const size_t o = size_t(L.out);
    P.framebuffer[o] = b8 | (g8 << 8) | (r8 << 16);
    if (P.hit_face) P.hit_face[o] = L.hface;
    if (P.hit_t) P.hit_t[o] = L.ht;
    if (P.rgb) { P.rgb[3 * o] = col.x; P.rgb[3 * o + 1] = col.y; P.rgb[3 * o + 2] = col.z; }
    if (P.ray_casts) P.ray_casts[o] = L.casts;
    L.total += L.traced;
    L.ph = PH_FETCH;
}

// Start the pending sample, or output the pixel when all are done. bounce_limit <= 0: cast_ray
// returns black without tracing (renderer.cpp:222).
template <int K, bool PRIMARY>
__device__ __forceinline__ void next_sample(Lane<K>& L, const RenderParams& P) {
    const atr_camera& cm = P.cam;
    if constexpr (PRIMARY) {  // one intersection serves every sample (renderer.cpp:353-356)
        begin_sample(L, cm);
        return;
    }
    for (;;) {
        if (L.s >= cm.samples_per_pixel) { pixel_out(L, P); return; }
        begin_sample(L, cm);
        if (cm.bounce_limit > 0) return;
        L.col = add(L.col, L.ret);
        ++L.s;
    }
}

template <int K, bool PRIMARY>
__device__ __forceinline__ void take_pixel(Lane<K>& L, const RenderParams& P, int32_t cell, int32_t l) {
    const DBlock blk = P.blocks[cell];
    const uint64_t mask = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
    if (!((mask >> l) & 1)) return;  // not a pixel of this render: stay idle
    const int32_t x = blk.x0 + (l & 7), y = blk.y0 + (l >> 3);
    L.px = y * P.cam.width + x;
    L.out = P.layout == ATR_LAYOUT_PACKED ? blk.out_base + __popcll(mask & ((uint64_t(1) << l) - 1)) : L.px;
    uint64_t stream;
    pixel_stream(P.seed, int64_t(L.px), L.rng, stream);
    L.col = mk(0.f, 0.f, 0.f);
    L.casts = 0;
    L.traced = 0;
    L.hface = 0xFFFFFFFFu;
    L.ht = kMaxFloat;
    L.s = 0;
    next_sample<K, PRIMARY>(L, P);
}

template <int K>
__device__ __forceinline__ void next_model(Lane<K>& L, int32_t M, int32_t nmodels) {
    L.mi = M + 1;
    L.ph = M + 1 < nmodels ? PH_QUERY : PH_SHADE;
}

// The model's tree query is done: merge it (renderer.cpp:51-57).
template <int K>
__device__ __forceinline__ void query_done(Lane<K>& L, const DModel& m, int32_t M, int32_t nmodels) {
    if (L.h.t > kTol && L.h.t < L.best) {
        L.best = L.h.t;
        L.face = m.cface[L.h.slot];
        L.fu = L.h.u;
        L.fv = L.h.v;
        L.nm = M;
    }
    next_model(L, M, nmodels);
}

// Head of the sorted leaf buffer becomes the leaf being scanned (kd_tree.cpp:437-441).
template <int K, bool COUNT>
__device__ __forceinline__ void begin_leaf(Lane<K>& L, const DModel& m, Ctr& ct) {
    const int32_t leaf = L.lb.leaf[0];
    L.bd = L.lb.d[0];
    L.bi = L.lb.leaf[0];
    const uint2_t cr = load_range(m.cl_range, leaf);
    L.c = cr.x;
    const uint32_t n = cr.y;
    L.cend = L.c + n;
    L.h.improved = false;
    L.h.rank = -1;
    if constexpr (COUNT) { ct.leaf += 1; ct.cbox += n; }
    L.ph = PH_SCAN;
}

template <int K, bool COUNT>
__device__ __forceinline__ void query_start(Lane<K>& L, const DModel& m, int32_t M, int32_t nmodels, Ctr& ct) {
    if (m.has_tree) {
        L.h.t = kMaxFloat;
        L.h.slot = 0xFFFFFFFFu;
        L.h.u = L.h.v = 0.f;
        L.h.rank = -1;
        L.h.improved = false;
        const NodeBox root = load_node(m.nodes, 0);
        if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
        if (!box_check(L.r, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) {  // kd_tree.cpp:339
            query_done(L, m, M, nmodels);
        } else if (m.root_leaf) {  // :344-361
            L.nb = 0;
            L.more = false;
            L.c = m.cl_range[0];
            L.cend = L.c + m.cl_range[1];
            if constexpr (COUNT) { ct.leaf += 1; ct.cbox += m.cl_range[1]; }
            L.ph = PH_SCAN;
        } else {
            L.bd = -__builtin_inff();
            L.bi = -1;
            L.ph = PH_TRAV;
        }
        return;
    }
    // brute force (renderer.cpp:58-82): face-ordered triangles
    if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
    if (box_entry(L.r, m.aabb[0], m.aabb[1], m.aabb[2], m.aabb[3], m.aabb[4], m.aabb[5]) != 0) {
        if constexpr (COUNT) { ct.tri += m.nfaces; }
        for (uint32_t j = 0; j < m.nfaces; ++j) {
            const DTri* t = m.tris + j;
            float u = 0.f, v = 0.f;
            const float tt = tri_hit(L.r, mk(t->ax, t->ay, t->az), mk(t->abx, t->aby, t->abz),
                                     mk(t->acx, t->acy, t->acz), u, v);
            if (tt > kTol && tt < L.best) { L.best = tt; L.fu = u; L.fv = v; L.face = j; L.nm = M; }
        }
    }
    next_model(L, M, nmodels);
}

template <bool COUNT, bool PRIMARY, int K>
__global__ __launch_bounds__(256, kPersistOcc) void persist_kernel(RenderParams P) {
    const int lane = threadIdx.x & 63;
    const uint64_t below = (uint64_t(1) << lane) - 1;
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    int32_t q = int32_t(xcc & 7u);  // this XCD's queue first
    uint32_t dry = 0;               // queues found empty (wave-uniform)
    const atr_camera& cm = P.cam;
    const DScene* __restrict__ S = P.scene;
    const int32_t nmodels = S->nmodels;
    Lane<K> L;
    L.ph = PH_FETCH;
    L.total = 0;
    Ctr ct;
    int err = 0;
    for (;;) {
        // -------------------------------------------------------- refill idle lanes
        uint64_t idle = __ballot(L.ph == PH_FETCH);
        if (idle && (__popcll(idle) >= kRefill || idle == __ballot(L.ph != PH_DONE))) {
            while (idle && dry != 0xFFu) {
                const int32_t n = __popcll(idle);
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(P.queue + q * kQueueStride, uint32_t(n));
                base = __builtin_amdgcn_readfirstlane(base);
                const int32_t size = queue_items(q, P.nblocks, P.qchunk);
                if (L.ph == PH_FETCH) {
                    const int64_t j = int64_t(base) + __popcll(idle & below);
                    if (j < size) take_pixel<K, PRIMARY>(L, P, queue_cell(q, int32_t(j), P.qchunk), int32_t(j) & 63);
                }
                const bool served = int64_t(base) + n <= int64_t(size);
                if (!served) {  // this queue ran dry: move on to the next one that is not
                    dry |= 1u << q;
                    for (int k = 1; k < 8; ++k) {
                        const int32_t x = (q + k) & 7;
                        if (!((dry >> x) & 1u)) { q = x; break; }
                    }
                }
                idle = __ballot(L.ph == PH_FETCH);
                if (served) break;
            }
            if (dry == 0xFFu && L.ph == PH_FETCH) L.ph = PH_DONE;
        }
        if (__ballot(L.ph != PH_DONE) == 0) break;

        // -------------------------------------------------------- model queries
        for (int32_t M = 0; M < nmodels; ++M)
            if (L.mi == M && L.ph == PH_QUERY) query_start<K, COUNT>(L, S->models[M], M, nmodels, ct);
        // an octree pass costs a dozen node visits: run it only for a batch of lanes, or when no
        // lane has a leaf to scan (the others wait; Aila & Laine's speculative while-while idea)
        const uint64_t trav = __ballot(L.ph == PH_TRAV);
        const bool do_trav = trav && (__popcll(trav) >= kTravBatch || __ballot(L.ph == PH_SCAN) == 0);
        for (int32_t M = 0; M < nmodels; ++M) {
            const DModel& m = S->models[M];
            if (do_trav && L.mi == M && L.ph == PH_TRAV) {  // one DFS pass (kd_tree.cpp:363-435)
                const int32_t n = traverse_pass<K, COUNT>(L.r, m.inner, L.lb, L.bd, L.bi, ct);
                if (n < 0) {
                    err = 1;
                    query_done(L, m, M, nmodels);
                } else {
                    L.nb = n < K ? n : K;
                    L.more = n > K;
                    if (L.nb == 0) query_done(L, m, M, nmodels);
                    else begin_leaf<K, COUNT>(L, m, ct);
                }
            }
        }
        for (int32_t M = 0; M < nmodels; ++M) {
            const DModel& m = S->models[M];
            if (L.mi == M && L.ph == PH_SCAN) {  // the whole leaf (kd_tree.cpp:440-456)
                cluster_range<COUNT>(L.r, m, L.c, L.cend, L.h, ct);
                L.c = L.cend;
                // stop at the first leaf that improved the hit (:457-460)
                if (L.h.improved) {
                    query_done(L, m, M, nmodels);
                } else {
                    lb_pop<K>(L.lb);
                    --L.nb;
                    if (L.nb > 0) begin_leaf<K, COUNT>(L, m, ct);
                    else if (L.more) L.ph = PH_TRAV;  // re-walk after the last scanned leaf
                    else query_done(L, m, M, nmodels);
                }
            }
        }

        // -------------------------------------------------------- hit record + cast_ray step
        if (L.ph == PH_SHADE) {
            Isect id;
            scene_finish(S, L.r.o, L.r.d, L.best, L.face, L.fu, L.fv, L.nm, id);
            const DMaterial& mat = S->mats[id.material];
            const V3 emission = mk(mat.ex, mat.ey, mat.ez);
            if constexpr (PRIMARY) {  // bounce_limit 1, no AA: the colour is the emission
                L.hface = id.face;
                L.ht = id.t;
                const uint32_t hit = id.type == T_SKY ? 0u : 1u;
                for (uint32_t s = 0; s < cm.samples_per_pixel; ++s) {
                    L.col = add(L.col, emission);
                    L.casts += hit;
                    ++L.traced;
                }
                pixel_out(L, P);
            } else {  // renderer.cpp:225-258
                ++L.traced;
                if (L.s == 0 && L.bounce == 0) { L.hface = id.face; L.ht = id.t; }
                bool sample_done = false;
                if (id.type == T_SKY) {
                    L.ret = add(L.ret, had(L.w, emission));
                    L.casts += L.bounce;  // ray_casts += i (:260)
                    sample_done = true;
                } else {
                    const V3 d = L.r.d;
                    float att = dot(neg(d), id.normal);
                    V3 n = id.normal;
                    if (att < 0) { n = neg(n); att = 0; }
                    V3 pure = sub(d, scale(n, (2 * dot(d, n))));
                    pure = unit(pure);
                    const uint64_t st = stream_of(L.px);
                    const float r0 = rand_bi(L.rng, st);
                    const float r1 = rand_bi(L.rng, st);
                    const float r2 = rand_bi(L.rng, st);
                    V3 rnd = add(mk(r0, r1, r2), n);
                    rnd = unit(rnd);
                    const V3 o2 = add(L.r.o, scale(d, id.t));
                    const V3 d2 = unit(lerp3(rnd, pure, mat.scatter));
                    L.ret = add(L.ret, had(L.w, emission));
                    L.w = had(L.w, scale(mk(mat.rx, mat.ry, mat.rz), att));
                    ++L.bounce;
                    if (int32_t(L.bounce) < cm.bounce_limit) {
                        begin_ray(L, o2, d2);
                    } else {
                        L.casts += uint32_t(cm.bounce_limit);
                        sample_done = true;
                    }
                }
                if (sample_done) {
                    L.col = add(L.col, L.ret);  // :345 / :355
                    ++L.s;
                    next_sample<K, PRIMARY>(L, P);
                }
            }
        }
    }

    // every lane is done: traced rays, errors, counters
    if (P.traced_rays) {
        uint32_t t = L.total;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
        if (lane == 0 && t) atomicAdd(P.traced_rays, (unsigned long long)t);
    }
    if (err && P.error_flag) atomicOr(P.error_flag, 1);
    if constexpr (COUNT) {
        uint32_t v[8] = {L.total, ct.box, ct.tri, ct.leaf, 0u, ct.pass, ct.box_all, 0u};
        unsigned long long* C = P.counters;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            uint32_t t = v[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
            if (lane == 0 && t) atomicAdd(C + k, (unsigned long long)t);
        }
        if (lane == 0) atomicAdd(C + 7, 1ull);
        uint32_t w[2] = {ct.cbox, ct.screen};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            uint32_t x = w[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
            if (lane == 0 && x) atomicAdd(C + 8 + k, (unsigned long long)x);
        }
    }
}

}  // namespace atr

template <bool C, bool PR>
static void launch_persist_one(const atr::RenderParams& P, int grid, hipStream_t s) {
    hipLaunchKernelGGL((atr::persist_kernel<C, PR, atr::kPersistK>), dim3(grid), dim3(256), 0, s, P);
}

// ncu: compute units of the device; the grid is kPersistOcc workgroups (one wave per SIMD each)
// per CU, fewer for small renders. P.queue: 8 zeroed queue heads, kQueueStride words apart.
extern "C" hipError_t atr_launch_persist(const atr::RenderParams& P, int ncu, hipStream_t s) {
    if (P.nblocks <= 0) return hipSuccess;
    const bool count = P.counters != nullptr;
    const bool prim = P.cam.bounce_limit == 1 && !P.cam.anti_aliasing;
    int grid = ncu * atr::kPersistOcc;
    const int need = (P.nblocks + 3) / 4;
    if (need < grid) grid = need;
    if (count) { if (prim) launch_persist_one<true, true>(P, grid, s); else launch_persist_one<true, false>(P, grid, s); }
    else { if (prim) launch_persist_one<false, true>(P, grid, s); else launch_persist_one<false, false>(P, grid, s); }
    return hipGetLastError();
}
