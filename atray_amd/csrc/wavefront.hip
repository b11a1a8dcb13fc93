// wavefront.hip -- the leaf-major (ray-sorted) schedule of the render path.
//
// LANE scans leaves per lane: 60% lane efficiency and every triangle test waits on a per-lane
// global load (latency-bound). Here the rays of a whole render are
// regrouped by the leaf each one scans next, so a leaf's triangles are staged ONCE into LDS
// per 64 rays and every lane tests them by LDS broadcast:
//
//   per sample:  wf_begin (primary rays)
//   per bounce:  per model  wf_traverse (root test + first DFS pass -> 8 sorted leaves/ray,
//                           bins each ray's first leaf)
//                           repeat: wf_scan (leaf histogram -> bucket offsets + work items)
//                                   wf_scatter (ray ids into per-leaf buckets)
//                                   wf_process (one wavefront per (leaf, <=64 rays) item: stage
//                                               the leaf in LDS, test, then each ray either
//                                               finishes the model or bins its next leaf)
//                                   wf_rewalk (rays that used all 8 buffered leaves walk the
//                                              tree again after their bound)
//                until no ray has a pending leaf
//                wf_shade (spheres/planes, normal, material, bounce ray, color)
//   end:         wf_finish (average, clamp, BGRX, outputs)
//
// Every ray scans exactly the leaves the reference scans, in its own sorted order, and stops
// after the first leaf that improves its hit (kd_tree.cpp:437-462); per-ray arithmetic is the
// same device code as LANE, so outputs are bit-identical. Step-synchronous sorting needs no
// atomics on results: each (ray, model, leaf) is processed by exactly one lane.
#include <hip/hip_runtime.h>

#include "trace.h"
#include "wavefront.h"

namespace atr {

constexpr int kWfChunk = 128;  // triangles staged per wavefront LDS chunk (4.6 KB)
constexpr int kWfBlock = 256;
constexpr float kInf = __builtin_inff();

// scene pointers are loaded from the DScene record, so the compiler cannot infer their address
// space and would emit flat loads (which also count on lgkmcnt); they are global memory
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4_t ldg4(const float4_t* p) {
    const v4f v = *(const __attribute__((address_space(1))) v4f*)(p);
    return float4_t{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ float ldg1(const float* p) { return *(const __attribute__((address_space(1))) float*)(p); }

__device__ __forceinline__ int gtid() { return blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ int gsize() { return gridDim.x * blockDim.x; }

// wave-aggregated append of `pred` lanes to a list; returns the slot for the calling lane
__device__ __forceinline__ int32_t wave_append(int32_t* count, bool pred) {
    const uint64_t m = __ballot(pred);
    if (!m) return -1;
    const int lane = threadIdx.x & 63;
    const int leader = __builtin_ctzll(m);
    int32_t base = 0;
    if (lane == leader) base = atomicAdd(count, __popcll(m));
    base = __shfl(base, leader);
    return base + __popcll(m & ((uint64_t(1) << lane) - 1));
}

// Wave-aggregated histogram binning: lanes with `pred` add one to cnt[leaf] and get their slot
// in that leaf's bucket. Rays of a wavefront mostly share their next leaf, so this is about one
// atomic per distinct leaf per wave instead of one per ray (same-address atomics serialise at
// ~12 ns each: MI355X_MICROARCH.md 'fanin'). All lanes of the wave must call it.
__device__ __forceinline__ int32_t wave_bin(uint32_t* cnt, int32_t leaf, bool pred) {
    const int lane = threadIdx.x & 63;
    uint64_t todo = __ballot(pred);
    int32_t slot = -1;
    while (todo) {
        const int leader = __builtin_ctzll(todo);
        const int32_t L = __builtin_amdgcn_readlane(leaf, leader);
        const uint64_t grp = __ballot(pred && leaf == L) & todo;
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(cnt + L, uint32_t(__popcll(grp)));
        base = __shfl(base, leader);
        if ((grp >> lane) & 1) slot = int32_t(base) + __popcll(grp & ((uint64_t(1) << lane) - 1));
        todo &= ~grp;
    }
    return slot;
}

__device__ __forceinline__ V3 ld3(const float* a, int32_t n, int32_t r) { return mk(a[r], a[n + r], a[2 * n + r]); }
__device__ __forceinline__ void st3(float* a, int32_t n, int32_t r, V3 v) { a[r] = v.x; a[n + r] = v.y; a[2 * n + r] = v.z; }

// ------------------------------------------------------------------ sample start
__global__ __launch_bounds__(kWfBlock) void wf_begin(WFParams W, int32_t sample) {
    const atr_camera& cm = W.cam;
    const int32_t n = W.n;
    for (int32_t r = gtid(); r < n; r += gsize()) {
        const int32_t p = W.pix[r];
        const int32_t x = p % cm.width, y = p / cm.width;
        uint64_t st, stream;
        if (sample == 0) {
            pixel_stream(W.seed, p, st, stream);
            W.col[r] = 0.f; W.col[n + r] = 0.f; W.col[2 * n + r] = 0.f;
            W.casts[r] = 0;
            W.traced[r] = 0;
            W.hface[r] = 0xFFFFFFFFu;
            W.ht[r] = kMaxFloat;
        } else {
            st = W.rng[r];
            stream = (uint64_t(p) << 1) | 1ULL;
        }
        const float film_y = -1.0f + 2.0f * (float(y) / float(cm.height));
        const float film_x = ((-1.0f + 2.0f * (float(x) / float(cm.width))) * cm.h_fov) * cm.aspect_ratio;
        const V3 eye = from(cm.eye), fc = from(cm.frame_center), cx = from(cm.camera_x), cy = from(cm.camera_y);
        V3 dir;
        if (cm.anti_aliasing) {  // renderer.cpp:338-343
            const float xo = rand_bi(st, stream) * cm.half_pixel_width + film_x;
            const float yo = rand_bi(st, stream) * cm.half_pixel_height + film_y;
            dir = unit(sub(add(add(fc, scale(cx, xo)), scale(cy, yo)), eye));
        } else {
            dir = unit(sub(add(add(fc, scale(cx, film_x)), scale(cy, film_y)), eye));  // :350-351
        }
        W.rng[r] = st;
        st3(W.ro, n, r, eye);
        st3(W.rd, n, r, dir);
        st3(W.ret, n, r, mk(0.f, 0.f, 0.f));
        st3(W.wt, n, r, mk(1.f, 1.f, 1.f));
        W.bt[r] = kMaxFloat;
        W.bmodel[r] = -1;
        W.act[0][r] = r;
    }
    if (gtid() == 0) { W.ctl->nact[0] = cm.bounce_limit > 0 ? n : 0; W.ctl->nact[1] = 0; }
}

// ------------------------------------------------------------------ per-model tree query
__device__ __forceinline__ Ray wf_ray(const WFParams& W, int32_t r) {
    return make_ray(ld3(W.ro, W.n, r), ld3(W.rd, W.n, r));
}

// store a fresh K-buffer; returns the ray's first leaf (or -1)
__device__ __forceinline__ int32_t wf_store_pass(const WFParams& W, int32_t r, const LeafBuf<kLeafBuf>& lb,
                                                 int32_t ncand) {
    const int32_t n = W.n;
    const int32_t nb = ncand < kLeafBuf ? ncand : kLeafBuf;
#pragma unroll
    for (int k = 0; k < kLeafBuf; ++k) W.ql[k * n + r] = lb.leaf[k];
    W.qd7[r] = lb.d[kLeafBuf - 1];
    W.qi7[r] = lb.leaf[kLeafBuf - 1];
    W.qpos[r] = 0;
    W.qnb[r] = nb;
    W.qnc[r] = ncand;
    return nb > 0 ? lb.leaf[0] : -1;
}

// bin + append: every lane of the wave calls it; lanes with leaf >= 0 join step `lst`
__device__ __forceinline__ void wf_enqueue(const WFParams& W, int32_t r, int32_t leaf, int32_t lst) {
    const bool pend = leaf >= 0;
    const int32_t slot = wave_bin(W.cnt[lst], leaf, pend);
    const int32_t s = wave_append(&W.ctl->npend[lst], pend);
    if (pend) {
        W.pleaf[r] = leaf;
        W.pslot[r] = slot;
        W.pend[lst][s] = r;
    }
}

__global__ __launch_bounds__(kWfBlock) void wf_traverse(WFParams W, int32_t model, int32_t cur, int32_t abuf) {
    const DModel& m = W.scene->models[model];
    const int32_t nact = W.ctl->nact[abuf];
    const int32_t* act = W.act[abuf];
    const int32_t iters = (nact + gsize() - 1) / gsize();
    for (int32_t it = 0; it < iters; ++it) {  // uniform trip count: wave_append needs whole waves
        const int32_t i = it * gsize() + gtid();
        int32_t leaf = -1;
        int32_t r = -1;
        if (i < nact) {
            r = act[i];
            const Ray ray = wf_ray(W, r);
            const NodeBox root = load_node(m.nodes, 0);
            if (box_check(ray, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) {  // :339
                if (root.children == 0) {  // root is a leaf: scan it alone (:344-361)
                    LeafBuf<kLeafBuf> lb;
                    lb_clear<kLeafBuf>(lb);
                    lb.leaf[0] = 0;
                    leaf = wf_store_pass(W, r, lb, 1);
                } else {
                    LeafBuf<kLeafBuf> lb;
                    Ctr ct;
                    const int32_t nc = traverse_pass<kLeafBuf, false>(ray, m.inner, lb, -kInf, -1, ct);
                    if (nc < 0) { atomicOr(W.error_flag, 1); }
                    else leaf = wf_store_pass(W, r, lb, nc);
                }
            }
        }
        wf_enqueue(W, r, leaf, cur);
    }
}

// Inclusive scan of one value per thread over the 1024-thread workgroup (wave shuffles + LDS).
__device__ __forceinline__ int32_t block_scan_incl(int32_t v, int32_t* s_w) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int32_t t = __shfl_up(v, off);
        if (lane >= off) v += t;
    }
    if (lane == 63) s_w[w] = v;
    __syncthreads();
    int32_t add = 0;
    for (int k = 0; k < w; ++k) add += s_w[k];
    return v + add;
}

// One workgroup: bucket offsets (exclusive prefix of the per-leaf counts) and one record per
// non-empty leaf {leaf, first bucket slot, rays, first work item}; a work item is <= 64 rays of
// one leaf and processing waves find theirs by binary search over the records. Resets the
// counters the next step fills. Each thread owns a contiguous run of nodes: two barriers.
__global__ __launch_bounds__(1024) void wf_scan(WFParams W, int32_t nnodes, int32_t cur) {
    __shared__ int32_t s_wa[16], s_wb[16], s_wc[16];
    const int tid = threadIdx.x;
    if (tid == 0) {
        W.ctl->npend[cur ^ 1] = 0;
        W.ctl->nrw = 0;
    }
    const int32_t per = (nnodes + 1023) / 1024;
    const int32_t lo = tid * per, hi = lo + per < nnodes ? lo + per : nnodes;
    int32_t sc = 0, si = 0, sr = 0;
    for (int32_t L = lo; L < hi; ++L) {
        const int32_t c = int32_t(W.cnt[cur][L]);
        sc += c;
        si += (c + 63) / 64;
        sr += c ? 1 : 0;
    }
    const int32_t ic = block_scan_incl(sc, s_wa);
    const int32_t ii = block_scan_incl(si, s_wb);
    const int32_t ir = block_scan_incl(sr, s_wc);
    int32_t off = ic - sc, item = ii - si, rec = ir - sr;
    int4* R = reinterpret_cast<int4*>(W.items);
    for (int32_t L = lo; L < hi; ++L) {
        const int32_t c = int32_t(W.cnt[cur][L]);
        W.offs[L] = off;
        if (c) {
            R[rec++] = make_int4(L, off, c, item);
            W.cnt[cur][L] = 0;
        }
        off += c;
        item += (c + 63) / 64;
    }
    if (tid == 1023) { W.ctl->nitems = ii; W.ctl->pad[0] = ir; }
}

__global__ __launch_bounds__(kWfBlock) void wf_scatter(WFParams W, int32_t cur) {
    const int32_t np = W.ctl->npend[cur];
    const int32_t* pend = W.pend[cur];
    for (int32_t i = gtid(); i < np; i += gsize()) {
        const int32_t r = pend[i];
        W.bucket[W.offs[W.pleaf[r]] + W.pslot[r]] = r;
    }
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes have landed
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One wavefront per work item: up to 64 rays that all scan leaf L next.
__global__ __launch_bounds__(kWfBlock) void wf_process(WFParams W, int32_t model, int32_t cur) {
    __shared__ float4_t s_t0[kWfBlock / 64][kWfChunk], s_t1[kWfBlock / 64][kWfChunk];
    __shared__ float s_t2[kWfBlock / 64][kWfChunk];
    const DModel& m = W.scene->models[model];
    const int32_t n = W.n;
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int32_t nitems = W.ctl->nitems;
    const int32_t nrec = W.ctl->pad[0];
    const int32_t nwaves = gsize() / 64;
    const int32_t nxt = cur ^ 1;
    const int32_t iters = (nitems + nwaves - 1) / nwaves;
    for (int32_t it = 0; it < iters; ++it) {
        const int32_t item = it * nwaves + gtid() / 64;
        int32_t next_leaf = -1;
        int32_t r = -1;
        if (item < nitems) {  // wave-uniform
            // record with the largest first-item <= item (records are sorted by first item)
            const int4* R = reinterpret_cast<const int4*>(W.items);
            int32_t lo = 0, hi = nrec - 1;
            while (lo < hi) {
                const int32_t mid = (lo + hi + 1) >> 1;
                if (R[mid].w <= item) lo = mid; else hi = mid - 1;
            }
            const int4 Rec = R[lo];
            const int32_t L = Rec.x;
            const int32_t k = item - Rec.w;
            const int32_t cnt_rays = Rec.z - 64 * k < 64 ? Rec.z - 64 * k : 64;
            const bool has = lane < cnt_rays;
            r = has ? W.bucket[Rec.y + 64 * k + lane] : -1;
            Ray ray;
            if (has) ray = wf_ray(W, r);
            const uint32_t first = m.leaf_range[2 * L], count = m.leaf_range[2 * L + 1];
            float bt = kMaxFloat, bu = 0.f, bv = 0.f;
            uint32_t bs = 0xFFFFFFFFu;
            for (uint32_t c0 = 0; c0 < count; c0 += kWfChunk) {
                const uint32_t cc = count - c0 < uint32_t(kWfChunk) ? count - c0 : uint32_t(kWfChunk);
                for (uint32_t k = lane; k < cc; k += 64) {
                    const float4_t a = ldg4(m.t0 + first + c0 + k), b = ldg4(m.t1 + first + c0 + k);
                    const float c = ldg1(m.t2 + first + c0 + k);
                    s_t0[wv][k] = a;
                    s_t1[wv][k] = b;
                    s_t2[wv][k] = c;
                }
                wave_lds_sync();
                if (has) {
                    // two triangles per iteration from alternating register sets, so the LDS
                    // reads of the second are in flight while the first is tested
                    for (uint32_t q = 0; q < cc; q += 2) {
                        const float4_t a0 = s_t0[wv][q], b0 = s_t1[wv][q];
                        const float c0v = s_t2[wv][q];
                        const uint32_t q1 = q + 1 < cc ? q + 1 : q;
                        const float4_t a1 = s_t0[wv][q1], b1 = s_t1[wv][q1];
                        const float c1v = s_t2[wv][q1];
                        float u = 0.f, v = 0.f;
                        float dist = tri_hit(ray, mk(a0.x, a0.y, a0.z), mk(a0.w, b0.x, b0.y), mk(b0.z, b0.w, c0v), u, v);
                        if (dist < bt && dist > kTol) { bt = dist; bs = first + c0 + q; bu = u; bv = v; }
                        if (q + 1 < cc) {
                            u = 0.f; v = 0.f;
                            dist = tri_hit(ray, mk(a1.x, a1.y, a1.z), mk(a1.w, b1.x, b1.y), mk(b1.z, b1.w, c1v), u, v);
                            if (dist < bt && dist > kTol) { bt = dist; bs = first + c0 + q + 1; bu = u; bv = v; }
                        }
                    }
                }
                wave_lds_sync();
            }
            if (has) {
                if (bs != 0xFFFFFFFFu) {  // leaf improved: the model's closest hit; merge in model order
                    if (bt > kTol && bt < W.bt[r]) {
                        W.bt[r] = bt; W.bu[r] = bu; W.bv[r] = bv;
                        W.bface[r] = m.tface[bs];
                        W.bmodel[r] = model;
                    }
                } else {
                    const int32_t pos = W.qpos[r] + 1;
                    if (pos < W.qnb[r]) {
                        next_leaf = W.ql[pos * n + r];
                        W.qpos[r] = pos;
                    } else if (W.qnc[r] > kLeafBuf) {
                        const int32_t s = atomicAdd(&W.ctl->nrw, 1);
                        W.rw[s] = r;
                    }
                }
            }
        }
        wf_enqueue(W, r, next_leaf, nxt);
    }
}

__global__ __launch_bounds__(kWfBlock) void wf_rewalk(WFParams W, int32_t model, int32_t cur) {
    const DModel& m = W.scene->models[model];
    const int32_t nrw = W.ctl->nrw;
    const int32_t nxt = cur ^ 1;
    const int32_t iters = (nrw + gsize() - 1) / gsize();
    for (int32_t it = 0; it < iters; ++it) {
        const int32_t i = it * gsize() + gtid();
        int32_t leaf = -1;
        int32_t r = -1;
        if (i < nrw) {
            r = W.rw[i];
            const Ray ray = wf_ray(W, r);
            LeafBuf<kLeafBuf> lb;
            Ctr ct;
            const int32_t nc = traverse_pass<kLeafBuf, false>(ray, m.inner, lb, W.qd7[r], W.qi7[r], ct);
            if (nc < 0) atomicOr(W.error_flag, 1);
            else leaf = wf_store_pass(W, r, lb, nc);
        }
        wf_enqueue(W, r, leaf, nxt);
    }
}

// Brute-force model (renderer.cpp:58-82): triangles streamed through LDS in tiles of 256,
// all lanes of the workgroup test every tile (face order; lowest face wins ties).
__global__ __launch_bounds__(kWfBlock) void wf_brute(WFParams W, int32_t model, int32_t abuf) {
    __shared__ float4_t s_t0[kWfBlock], s_t1[kWfBlock];
    __shared__ float s_t2[kWfBlock];
    const DModel& m = W.scene->models[model];
    const int32_t nact = W.ctl->nact[abuf];
    const int32_t* act = W.act[abuf];
    const int32_t ngroups = (nact + kWfBlock - 1) / kWfBlock;
    for (int32_t g = blockIdx.x; g < ngroups; g += gridDim.x) {  // workgroup-uniform
        const int32_t i = g * kWfBlock + threadIdx.x;
        bool live = false;
        int32_t r = -1;
        Ray ray;
        if (i < nact) {
            r = act[i];
            ray = wf_ray(W, r);
            live = box_entry(ray, m.aabb[0], m.aabb[1], m.aabb[2], m.aabb[3], m.aabb[4], m.aabb[5]) != 0;
        }
        float bt = live ? W.bt[r] : kMaxFloat, bu = 0.f, bv = 0.f;
        int32_t bf = -1;
        const int32_t any = __syncthreads_or(live);
        if (any) {
            for (uint32_t t0 = 0; t0 < m.nfaces; t0 += kWfBlock) {
                const uint32_t cc = m.nfaces - t0 < uint32_t(kWfBlock) ? m.nfaces - t0 : uint32_t(kWfBlock);
                if (threadIdx.x < cc) {
                    const DTri& t = m.tris[t0 + threadIdx.x];
                    s_t0[threadIdx.x] = float4_t{t.ax, t.ay, t.az, t.abx};
                    s_t1[threadIdx.x] = float4_t{t.aby, t.abz, t.acx, t.acy};
                    s_t2[threadIdx.x] = t.acz;
                }
                __syncthreads();
                if (live) {
                    for (uint32_t k = 0; k < cc; ++k) {
                        const float4_t a = s_t0[k], b = s_t1[k];
                        const float c = s_t2[k];
                        float u = 0.f, v = 0.f;
                        const float tt = tri_hit(ray, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, c), u, v);
                        if (tt > kTol && tt < bt) { bt = tt; bu = u; bv = v; bf = int32_t(t0 + k); }
                    }
                }
                __syncthreads();
            }
        }
        if (live && bf >= 0) {
            W.bt[r] = bt; W.bu[r] = bu; W.bv[r] = bv;
            W.bface[r] = uint32_t(bf);
            W.bmodel[r] = model;
        }
    }
}

// ------------------------------------------------------------------ shading (cast_ray body)
__global__ __launch_bounds__(kWfBlock) void wf_shade(WFParams W, int32_t bounce, int32_t sample, int32_t abuf) {
    const DScene* __restrict__ S = W.scene;
    const int32_t n = W.n;
    const int32_t nact = W.ctl->nact[abuf];
    const int32_t* act = W.act[abuf];
    const int32_t nb = abuf ^ 1;
    const int32_t iters = (nact + gsize() - 1) / gsize();
    const int32_t limit = W.cam.bounce_limit;
    for (int32_t it = 0; it < iters; ++it) {
        const int32_t i = it * gsize() + gtid();
        bool again = false;
        int32_t r = -1;
        if (i < nact) {
            r = act[i];
            const V3 o = ld3(W.ro, n, r), d = ld3(W.rd, n, r);
            float best = W.bt[r];
            const int32_t nm = W.bmodel[r];
            int32_t ns = -1, np = -1;
            for (int32_t k = 0; k < S->nspheres; ++k) {  // sphere.h:12-39
                const DSphere& sp = S->spheres[k];
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
                if (t > kTol && t < best) { best = t; ns = k; }
            }
            for (int32_t k = 0; k < S->nplanes; ++k) {  // plane.h:12-22
                const DPlane& pl = S->planes[k];
                const V3 nn = mk(pl.nx, pl.ny, pl.nz);
                const float denom = dot(nn, d);
                float t = 0;
                if (!(denom > -kTol && denom < kTol)) t = (pl.d - dot(o, nn)) / denom;
                if (t > kTol && t < best) { np = k; best = t; }
            }
            int type;
            V3 normal = mk(0.f, 0.f, 0.f);
            int32_t material = 0;
            uint32_t face = 0xFFFFFFFFu;
            if (np >= 0) {
                const DPlane& pl = S->planes[np];
                type = 3; normal = mk(pl.nx, pl.ny, pl.nz); material = pl.material;
            } else if (ns >= 0) {
                const DSphere& sp = S->spheres[ns];
                type = 2; normal = sub(add(o, scale(d, best)), mk(sp.cx, sp.cy, sp.cz)); material = sp.material;
            } else if (nm >= 0) {
                const DModel& m = S->models[nm];
                type = 1;
                face = W.bface[r];
                const float fu = W.bu[r], fv = W.bv[r];
                const float* sh = m.shade + 9 * size_t(face);
                if (m.smooth) {
                    const V3 na = mk(sh[0], sh[1], sh[2]), nb3 = mk(sh[3], sh[4], sh[5]), nc = mk(sh[6], sh[7], sh[8]);
                    normal = add(add(scale(na, (1 - fu - fv)), scale(nb3, fu)), scale(nc, fv));
                } else {
                    const V3 v0 = mk(sh[0], sh[1], sh[2]), v1 = mk(sh[3], sh[4], sh[5]), v2 = mk(sh[6], sh[7], sh[8]);
                    normal = cross(sub(v0, v1), sub(v0, v2));
                }
                material = m.material;
            } else {
                type = 4;
            }
            if (type != 4) normal = unit(normal);
            W.traced[r] += 1;
            if (sample == 0 && bounce == 0) { W.hface[r] = face; W.ht[r] = best; }
            const DMaterial& mat = S->mats[material];
            const V3 emission = mk(mat.ex, mat.ey, mat.ez);
            V3 ret = ld3(W.ret, n, r), w = ld3(W.wt, n, r);
            bool finish = false;
            uint32_t casts_add = 0;
            if (type == 4) {
                ret = add(ret, had(w, emission));
                finish = true;
                casts_add = uint32_t(bounce);
            } else {
                float att = dot(neg(d), normal);
                if (att < 0) { normal = neg(normal); att = 0; }
                V3 pure = sub(d, scale(normal, (2 * dot(d, normal))));
                pure = unit(pure);
                uint64_t st = W.rng[r];
                const uint64_t stream = (uint64_t(W.pix[r]) << 1) | 1ULL;
                const float r0 = rand_bi(st, stream);
                const float r1 = rand_bi(st, stream);
                const float r2 = rand_bi(st, stream);
                W.rng[r] = st;
                V3 rnd = add(mk(r0, r1, r2), normal);
                rnd = unit(rnd);
                const V3 no = add(o, scale(d, best));
                const V3 nd = unit(lerp3(rnd, pure, mat.scatter));
                ret = add(ret, had(w, emission));
                w = had(w, scale(mk(mat.rx, mat.ry, mat.rz), att));
                if (bounce + 1 < limit) {
                    st3(W.ro, n, r, no);
                    st3(W.rd, n, r, nd);
                    st3(W.wt, n, r, w);
                    W.bt[r] = kMaxFloat;
                    W.bmodel[r] = -1;
                    again = true;
                } else {
                    finish = true;
                    casts_add = uint32_t(limit);
                }
            }
            st3(W.ret, n, r, ret);
            if (finish) {  // end of this sample's cast_ray: color += ret (renderer.cpp:355)
                W.col[r] = W.col[r] + ret.x;
                W.col[n + r] = W.col[n + r] + ret.y;
                W.col[2 * n + r] = W.col[2 * n + r] + ret.z;
                W.casts[r] += casts_add;
            }
        }
        const int32_t s = wave_append(&W.ctl->nact[nb], again);
        if (again) W.act[nb][s] = r;
    }
}

// bounce_limit <= 0: cast_ray returns black without tracing (renderer.cpp:222 never enters)
__global__ __launch_bounds__(kWfBlock) void wf_finish(WFParams W) {
    const atr_camera& cm = W.cam;
    const int32_t n = W.n;
    const int lane = threadIdx.x & 63;
    const int32_t iters = (n + gsize() - 1) / gsize();
    for (int32_t it = 0; it < iters; ++it) {
        const int32_t r = it * gsize() + gtid();
        uint32_t tr = 0;
        if (r < n) {
            V3 col = ld3(W.col, n, r);
            col = divs(col, float(cm.samples_per_pixel));  // :358
            const float cr = pl_max(0.0f, pl_min(col.x, 1.0f));
            const float cg = pl_max(0.0f, pl_min(col.y, 1.0f));
            const float cb = pl_max(0.0f, pl_min(col.z, 1.0f));
            const uint32_t r8 = uint32_t(cr * 255.0f) & 0xFFu, g8 = uint32_t(cg * 255.0f) & 0xFFu,
                           b8 = uint32_t(cb * 255.0f) & 0xFFu;
            const size_t o = W.layout == ATR_LAYOUT_PACKED ? size_t(r) : size_t(W.pix[r]);
            W.framebuffer[o] = b8 | (g8 << 8) | (r8 << 16);
            if (W.out_hit_face) W.out_hit_face[o] = W.hface[r];
            if (W.out_hit_t) W.out_hit_t[o] = W.ht[r];
            if (W.out_rgb) { W.out_rgb[3 * o] = col.x; W.out_rgb[3 * o + 1] = col.y; W.out_rgb[3 * o + 2] = col.z; }
            if (W.out_ray_casts) W.out_ray_casts[o] = W.casts[r];
            tr = W.traced[r];
        }
        if (W.traced_rays) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) tr += __shfl_xor(tr, off);
            if (lane == 0 && tr) atomicAdd(W.traced_rays, (unsigned long long)tr);
        }
    }
}

}  // namespace atr

// ------------------------------------------------------------------ host orchestration
namespace {
inline int grid_for(int64_t work, int cap) {
    int64_t g = (work + atr::kWfBlock - 1) / atr::kWfBlock;
    if (g < 1) g = 1;
    return int(g < cap ? g : cap);
}
}  // namespace

// Enqueue a whole render on `s`. Host syncs only to learn when a model's leaf steps are done
// (a pinned 4-byte read every `kCheck` steps).
extern "C" hipError_t atr_wf_render(const atr::WFParams& W, int32_t nmodels, const int32_t* nnodes,
                                    const int32_t* has_tree, int32_t* pinned, hipStream_t s) {
    using namespace atr;
    constexpr int kCheck = 4;
    const int cap = 4096;  // persistent grid: 4096 WGs x 256 threads
    const int gp = grid_for(W.n, cap);
    const atr_camera& cm = W.cam;
    for (uint32_t sample = 0; sample < cm.samples_per_pixel; ++sample) {
        hipLaunchKernelGGL(wf_begin, dim3(gp), dim3(kWfBlock), 0, s, W, int32_t(sample));
        int32_t abuf = 0;
        for (int32_t bounce = 0; bounce < cm.bounce_limit; ++bounce) {
            for (int32_t mi = 0; mi < nmodels; ++mi) {
                if (!has_tree[mi]) {
                    hipLaunchKernelGGL(wf_brute, dim3(gp), dim3(kWfBlock), 0, s, W, mi, abuf);
                    continue;
                }
                int32_t cur = 0;
                hipLaunchKernelGGL(wf_traverse, dim3(gp), dim3(kWfBlock), 0, s, W, mi, cur, abuf);
                for (int32_t step = 0;; ++step) {
                    hipLaunchKernelGGL(wf_scan, dim3(1), dim3(1024), 0, s, W, nnodes[mi], cur);
                    hipLaunchKernelGGL(wf_scatter, dim3(gp), dim3(kWfBlock), 0, s, W, cur);
                    hipLaunchKernelGGL(wf_process, dim3(gp), dim3(kWfBlock), 0, s, W, mi, cur);
                    hipLaunchKernelGGL(wf_rewalk, dim3(grid_for(W.n, 1024)), dim3(kWfBlock), 0, s, W, mi, cur);
                    cur ^= 1;
                    if ((step + 1) % kCheck == 0) {
                        hipError_t e = hipMemcpyAsync(pinned, &W.ctl->npend[cur], sizeof(int32_t),
                                                      hipMemcpyDeviceToHost, s);
                        if (e == hipSuccess) e = hipStreamSynchronize(s);
                        if (e != hipSuccess) return e;
                        if (*pinned == 0) break;
                    }
                }
                // leave the counters of the last (empty) step clean for the next query
                hipLaunchKernelGGL(wf_scan, dim3(1), dim3(1024), 0, s, W, nnodes[mi], cur);
            }
            hipLaunchKernelGGL(wf_shade, dim3(gp), dim3(kWfBlock), 0, s, W, bounce, int32_t(sample), abuf);
            abuf ^= 1;
            hipError_t e = hipMemsetAsync(&W.ctl->nact[abuf ^ 1], 0, sizeof(int32_t), s);
            if (e != hipSuccess) return e;
        }
    }
    hipLaunchKernelGGL(wf_finish, dim3(gp), dim3(kWfBlock), 0, s, W);
    return hipGetLastError();
}
