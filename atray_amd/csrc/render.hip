// render.hip -- gfx950 kernels of the render path: one primary ray per lane, a wavefront per
// 8x8 pixel cell, the full per-pixel loop of render_tile_from_camera (renderer.cpp:294-369)
// -> cast_ray (:213-262) -> get_intersection_data (:34-160) -> octree traversal.
//
// Two bit-identical traversal schedules of the leaf scan (the hot loop, kd_tree.cpp:437-462):
//   LANE: every lane walks its own sorted leaves with per-lane (vector) triangle loads;
//   WAVE: the wavefront repeatedly elects one leaf (the next leaf of its first lane that still
//         scans) and every lane whose next leaf it is scans it together: the leaf's triangles
//         are read with wave-uniform scalar loads (s_load, no VMEM per lane, no lane-divergent
//         addresses) and the triangle loop runs converged. Each lane still consumes its leaves
//         in its own order, so results are identical.
#include <hip/hip_runtime.h>

#include "trace.h"

namespace atr {

enum { T_NONE = 0, T_TRI = 1, T_SPHERE = 2, T_PLANE = 3, T_SKY = 4 };

struct Isect {
    int type;
    float t;
    V3 normal;
    int32_t material;
    uint32_t face;
};

constexpr int kLeafBuf = 8;

// ------------------------------------------------------------------ LANE schedule
__device__ __forceinline__ void tree_closest_lane(const Ray& r, const DModel& m, Hit& h, int& err) {
    h.t = kMaxFloat;
    h.face = 0;
    h.u = h.v = 0.f;
    const NodeBox root = load_node(m.nodes, 0);
    if (!box_check(r, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) return;  // :339
    if (root.children == 0) {  // :344-361
        scan_leaf(r, m.tris, m.leaf_range[0], m.leaf_range[1], h);
        return;
    }
    float bd = -__builtin_inff();
    int32_t bi = -1;
    for (;;) {
        LeafBuf<kLeafBuf> lb;
        const int32_t n = traverse_pass<kLeafBuf>(r, m.nodes, lb, bd, bi);
        if (n < 0) { err = 1; return; }
        const int32_t nb = n < kLeafBuf ? n : kLeafBuf;
        for (int32_t j = 0; j < nb; ++j) {
            const int32_t leaf = lb_node<kLeafBuf>(lb, j);
            if (scan_leaf(r, m.tris, m.leaf_range[2 * leaf], m.leaf_range[2 * leaf + 1], h)) return;
        }
        if (n <= kLeafBuf) return;
        bd = lb.d[kLeafBuf - 1];
        bi = lb.idx[kLeafBuf - 1];
    }
}

// ------------------------------------------------------------------ WAVE schedule
// Lane state of one tree query while the wavefront cooperates on leaf scans.
struct TreeQuery {
    LeafBuf<kLeafBuf> lb;
    float bd;
    int32_t bi;
    int32_t ncand;   // candidates of the current pass (after bound)
    int32_t pos;     // next buffer entry to scan
    int32_t state;   // 0 = needs a pass, 1 = has leaves in buffer, 2 = done
};

__device__ __forceinline__ int32_t tq_next_leaf(TreeQuery& q, const Ray& r, const DModel& m, int& err) {
    for (;;) {
        if (q.state == 2) return -1;
        if (q.state == 0) {
            q.ncand = traverse_pass<kLeafBuf>(r, m.nodes, q.lb, q.bd, q.bi);
            if (q.ncand < 0) { err = 1; q.state = 2; return -1; }
            q.pos = 0;
            q.state = 1;
        }
        const int32_t nb = q.ncand < kLeafBuf ? q.ncand : kLeafBuf;
        if (q.pos < nb) return lb_node<kLeafBuf>(q.lb, q.pos);
        if (q.ncand <= kLeafBuf) { q.state = 2; return -1; }
        q.bd = q.lb.d[kLeafBuf - 1];
        q.bi = q.lb.idx[kLeafBuf - 1];
        q.state = 0;
    }
}

// Scan a wave-uniform leaf: every operand address is uniform, so the triangle records are
// fetched by the scalar unit once per wavefront instead of once per lane.
__device__ __forceinline__ bool scan_leaf_uniform(const Ray& r, const DTri* __restrict__ tris,
                                                  uint32_t first, uint32_t count, Hit& h) {
    bool improved = false;
    for (uint32_t k = 0; k < count; ++k) {
        const DTri* t = tris + first + k;  // uniform address -> s_load_dwordx8 + s_load_dwordx2
        const V3 a = mk(t->ax, t->ay, t->az);
        const V3 ab = mk(t->abx, t->aby, t->abz);
        const V3 ac = mk(t->acx, t->acy, t->acz);
        float u = 0.f, v = 0.f;
        const float dist = tri_hit(r, a, ab, ac, u, v);
        if (dist < h.t && dist > kTol) {
            h.t = dist;
            h.face = t->face;
            h.u = u;
            h.v = v;
            improved = true;
        }
    }
    return improved;
}

__device__ __forceinline__ void tree_closest_wave(const Ray& r, const DModel& m, bool active, Hit& h,
                                                  int& err) {
    h.t = kMaxFloat;
    h.face = 0;
    h.u = h.v = 0.f;
    TreeQuery q;
    q.state = 2;
    int32_t root_leaf_scan = 0;
    if (active) {
        const NodeBox root = load_node(m.nodes, 0);
        if (box_check(r, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) {
            if (root.children == 0) root_leaf_scan = 1;
            else { q.bd = -__builtin_inff(); q.bi = -1; q.state = 0; }
        }
    }
    int32_t leaf = -1;
    if (q.state != 2) leaf = tq_next_leaf(q, r, m, err);
    if (root_leaf_scan) leaf = 0;
    for (;;) {
        const uint64_t want = __ballot(leaf >= 0);
        if (want == 0) break;
        const int src = __builtin_ctzll(want);
        const int32_t L = __builtin_amdgcn_readlane(leaf, src);  // uniform
        if (leaf == L) {
            const uint32_t first = m.leaf_range[2 * L], count = m.leaf_range[2 * L + 1];
            const bool hit = scan_leaf_uniform(r, m.tris, __builtin_amdgcn_readfirstlane(first),
                                               __builtin_amdgcn_readfirstlane(count), h);
            if (root_leaf_scan || hit) { q.state = 2; leaf = -1; }
            else { ++q.pos; leaf = tq_next_leaf(q, r, m, err); }
        }
    }
}

// ------------------------------------------------------------------ get_intersection_data
template <bool WAVE>
__device__ __forceinline__ void intersect_scene(const DScene* __restrict__ S, V3 o, V3 d, bool active,
                                                Isect& id, int& err) {
    const Ray r = make_ray(o, d);  // renderer.cpp:41-44
    float best = kMaxFloat;
    int32_t nm = -1, ns = -1, np = -1;
    uint32_t face = 0;
    float fu = 0.f, fv = 0.f;
    const int32_t nmodels = S->nmodels;
    for (int32_t i = 0; i < nmodels; ++i) {
        const DModel& m = S->models[i];
        if (m.has_tree) {  // USE_KD_TREE (:49-57)
            Hit h;
            if (WAVE) tree_closest_wave(r, m, active, h, err);
            else if (active) tree_closest_lane(r, m, h, err);
            else h.t = kMaxFloat;
            if (h.t > kTol && h.t < best) { best = h.t; face = h.face; fu = h.u; fv = h.v; nm = i; }
        } else if (active) {  // brute force (:58-82), face-ordered triangles, uniform loads
            if (box_entry(r, m.aabb[0], m.aabb[1], m.aabb[2], m.aabb[3], m.aabb[4], m.aabb[5]) != 0) {
                for (uint32_t j = 0; j < m.nfaces; ++j) {
                    const DTri* t = m.tris + j;
                    float u = 0.f, v = 0.f;
                    const float tt = tri_hit(r, mk(t->ax, t->ay, t->az), mk(t->abx, t->aby, t->abz),
                                             mk(t->acx, t->acy, t->acz), u, v);
                    if (tt > kTol && tt < best) { best = tt; fu = u; fv = v; face = j; nm = i; }
                }
            }
        }
    }
    if (!active) return;
    for (int32_t i = 0; i < S->nspheres; ++i) {  // sphere.h:12-39
        const DSphere& sp = S->spheres[i];
        const V3 pc = sub(o, mk(sp.cx, sp.cy, sp.cz));
        const float pcs = len2(pc);
        const float b = 2 * (dot(d, pc));
        const float bs = b * b;
        const float c = pcs - sp.r * sp.r;
        const float dmt = bs - (4 * c);
        float t = 0;
        if (!(dmt < 0)) {
            const float ta = (-b + sqrtf(dmt)) * 0.5f;
            const float tb = (-b - sqrtf(dmt)) * 0.5f;
            if (ta <= 0 && tb <= 0) t = 0;
            else if (tb > 0) t = tb;
            else t = ta;
        }
        if (t > kTol && t < best) { best = t; ns = i; }
    }
    for (int32_t i = 0; i < S->nplanes; ++i) {  // plane.h:12-22
        const DPlane& pl = S->planes[i];
        const V3 n = mk(pl.nx, pl.ny, pl.nz);
        const float denom = dot(n, d);
        float t = 0;
        if (!(denom > -kTol && denom < kTol)) t = (pl.d - dot(o, n)) / denom;
        if (t > kTol && t < best) { np = i; best = t; }
    }
    id.t = best;
    id.face = 0xFFFFFFFFu;
    if (np >= 0) {
        const DPlane& pl = S->planes[np];
        id.type = T_PLANE;
        id.normal = mk(pl.nx, pl.ny, pl.nz);
        id.material = pl.material;
    } else if (ns >= 0) {
        const DSphere& sp = S->spheres[ns];
        id.type = T_SPHERE;
        id.normal = sub(add(o, scale(d, best)), mk(sp.cx, sp.cy, sp.cz));  // Ray::at (ray.h:10-13)
        id.material = sp.material;
    } else if (nm >= 0) {
        const DModel& m = S->models[nm];
        id.type = T_TRI;
        id.face = face;
        const float* sh = m.shade + 9 * size_t(face);
        if (m.smooth) {  // interpolated vertex normals (:129-138)
            const V3 na = mk(sh[0], sh[1], sh[2]), nb = mk(sh[3], sh[4], sh[5]), nc = mk(sh[6], sh[7], sh[8]);
            id.normal = add(add(scale(na, (1 - fu - fv)), scale(nb, fu)), scale(nc, fv));
        } else {  // flat (:140-146)
            const V3 v0 = mk(sh[0], sh[1], sh[2]), v1 = mk(sh[3], sh[4], sh[5]), v2 = mk(sh[6], sh[7], sh[8]);
            id.normal = cross(sub(v0, v1), sub(v0, v2));
        }
        id.material = m.material;
    } else {
        id.type = T_SKY;
        id.material = 0;
    }
    if (id.type != T_SKY) id.normal = unit(id.normal);  // :157
}

// ------------------------------------------------------------------ cast_ray + pixel loop
template <bool WAVE>
__device__ __forceinline__ V3 cast_ray(const DScene* __restrict__ S, V3 o, V3 d, int32_t bounce_limit,
                                       bool active, uint64_t& st, uint64_t stream, uint32_t& casts,
                                       uint32_t& traced, bool record, uint32_t& hit_face, float& hit_t,
                                       int& err) {
    V3 ret = mk(0.f, 0.f, 0.f), w = mk(1.f, 1.f, 1.f);
    int32_t i = 0;
    bool live = active;
    // WAVE: every lane stays in the loop until all lanes are done, so the wavefront can
    // cooperate on leaf scans inside intersect_scene.
    for (i = 0; ; ++i) {
        const bool go = live && i < bounce_limit;
        if (WAVE) { if (__ballot(go) == 0) break; }
        else if (!go) break;
        Isect id;
        id.type = T_NONE;
        intersect_scene<WAVE>(S, o, d, go, id, err);
        if (!go) continue;
        ++traced;
        if (record && i == 0) { hit_face = id.face; hit_t = id.t; }
        const DMaterial& mat = S->mats[id.material];
        const V3 emission = mk(mat.ex, mat.ey, mat.ez);
        if (id.type == T_SKY) {
            ret = add(ret, had(w, emission));
            live = false;
            casts += uint32_t(i);
            continue;
        }
        float att = dot(neg(d), id.normal);
        V3 n = id.normal;
        if (att < 0) { n = neg(n); att = 0; }
        V3 pure = sub(d, scale(n, (2 * dot(d, n))));
        pure = unit(pure);
        const float r0 = rand_bi(st, stream);
        const float r1 = rand_bi(st, stream);
        const float r2 = rand_bi(st, stream);
        V3 rnd = add(mk(r0, r1, r2), n);
        rnd = unit(rnd);
        o = add(o, scale(d, id.t));
        d = unit(lerp3(rnd, pure, mat.scatter));
        ret = add(ret, had(w, emission));
        w = had(w, scale(mk(mat.rx, mat.ry, mat.rz), att));
    }
    if (live) casts += uint32_t(bounce_limit > 0 ? bounce_limit : 0);
    return ret;
}

__device__ __forceinline__ int remap_xcd(int wg, int nwg) {
    // consecutive work blocks -> same XCD (its L2 holds their shared leaves); bijective form
    const int q = nwg / 8, rm = nwg % 8, x = wg % 8;
    return (x < rm ? x * (q + 1) : rm * (q + 1) + (x - rm) * q) + wg / 8;
}

template <bool WAVE>
__global__ __launch_bounds__(256) void render_kernel(RenderParams P) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int b = remap_xcd(blockIdx.x, gridDim.x) * 4 + wave;
    if (b >= P.nblocks) return;  // whole wavefront
    const DBlock blk = P.blocks[b];
    const uint64_t mask = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
    const bool active = (mask >> lane) & 1;
    const int32_t x = blk.x0 + (lane & 7), y = blk.y0 + (lane >> 3);
    const atr_camera& cm = P.cam;
    const DScene* S = P.scene;
    int err = 0;
    uint32_t casts = 0, traced = 0, hit_face = 0xFFFFFFFFu;
    float hit_t = kMaxFloat;
    V3 col = mk(0.f, 0.f, 0.f);
    uint64_t st = 0, stream = 1;
    pixel_stream(P.seed, int64_t(y) * cm.width + x, st, stream);
    const float film_y = -1.0f + 2.0f * (float(y) / float(cm.height));                       // :317
    const float film_x = ((-1.0f + 2.0f * (float(x) / float(cm.width))) * cm.h_fov) * cm.aspect_ratio;  // :329
    const V3 eye = from(cm.eye), fc = from(cm.frame_center), cx = from(cm.camera_x), cy = from(cm.camera_y);
    V3 dir = mk(0.f, 0.f, 1.f);
    if (!cm.anti_aliasing) dir = unit(sub(add(add(fc, scale(cx, film_x)), scale(cy, film_y)), eye));  // :350-351
    for (uint32_t s = 0; s < cm.samples_per_pixel; ++s) {
        if (cm.anti_aliasing) {  // :338-343
            const float xo = rand_bi(st, stream) * cm.half_pixel_width + film_x;
            const float yo = rand_bi(st, stream) * cm.half_pixel_height + film_y;
            dir = unit(sub(add(add(fc, scale(cx, xo)), scale(cy, yo)), eye));
        }
        col = add(col, cast_ray<WAVE>(S, eye, dir, cm.bounce_limit, active, st, stream, casts, traced,
                                      s == 0, hit_face, hit_t, err));
    }
    if (active) {
        col = divs(col, float(cm.samples_per_pixel));  // :358
        const float cr = pl_max(0.0f, pl_min(col.x, 1.0f));
        const float cg = pl_max(0.0f, pl_min(col.y, 1.0f));
        const float cb = pl_max(0.0f, pl_min(col.z, 1.0f));
        const uint32_t r8 = uint32_t(cr * 255.0f) & 0xFFu, g8 = uint32_t(cg * 255.0f) & 0xFFu,
                       b8 = uint32_t(cb * 255.0f) & 0xFFu;
        size_t o;
        if (P.layout == ATR_LAYOUT_PACKED) o = size_t(blk.out_base) + __popcll(mask & ((uint64_t(1) << lane) - 1));
        else o = size_t(y) * size_t(cm.width) + size_t(x);
        P.framebuffer[o] = b8 | (g8 << 8) | (r8 << 16);  // Set_Pixel (texture.h:27-38)
        if (P.hit_face) P.hit_face[o] = hit_face;
        if (P.hit_t) P.hit_t[o] = hit_t;
        if (P.rgb) { P.rgb[3 * o] = col.x; P.rgb[3 * o + 1] = col.y; P.rgb[3 * o + 2] = col.z; }
        if (P.ray_casts) P.ray_casts[o] = casts;
    }
    if (P.traced_rays) {
        uint32_t t = traced;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
        if (lane == 0 && t) atomicAdd(P.traced_rays, (unsigned long long)t);
    }
    if (err && P.error_flag) atomicOr(P.error_flag, 1);
}

template __global__ void render_kernel<false>(RenderParams);
template __global__ void render_kernel<true>(RenderParams);

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

}  // namespace atr

// launchers used by capi.cpp
extern "C" hipError_t atr_launch_render(const atr::RenderParams& P, int wave, hipStream_t s) {
    const int grid = (P.nblocks + 3) / 4;
    if (grid <= 0) return hipSuccess;
    if (wave) hipLaunchKernelGGL(atr::render_kernel<true>, dim3(grid), dim3(256), 0, s, P);
    else hipLaunchKernelGGL(atr::render_kernel<false>, dim3(grid), dim3(256), 0, s, P);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_unpack(const atr::DBlock* blocks, int32_t nblocks, int32_t width,
                                        const uint32_t* packed, uint32_t* image, hipStream_t s) {
    const int grid = (nblocks + 3) / 4;
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL(atr::unpack_kernel, dim3(grid), dim3(256), 0, s, blocks, nblocks, width, packed, image);
    return hipGetLastError();
}

extern "C" hipError_t atr_launch_tile_casts(const atr_tile* tiles, int32_t ntiles, int32_t width,
                                            const uint32_t* casts, int64_t* out, hipStream_t s) {
    if (ntiles <= 0) return hipSuccess;
    hipLaunchKernelGGL(atr::tile_casts_kernel, dim3(ntiles), dim3(256), 0, s, tiles, width, casts, out);
    return hipGetLastError();
}
