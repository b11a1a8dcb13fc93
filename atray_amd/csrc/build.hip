// build.hip -- f3: the octree build of prep_scene on the GPU.
//
// build_oct_kd_tree (kd_tree.cpp:67-288) splits a node with more than max_faces triangles at the
// area-weighted centroid of its triangles (kd_tree.cpp:93-114: f32 sum of centroid*area in the
// node's triangle order, f64 sum of areas) into the 8 octants of (lo, v, hi), and hands each
// triangle to every child box that contains one of its vertices (kd_tree.cpp:10-17,181-228),
// keeping the parent's order. The host restatement is atr::octree_build (host_scene.cpp).
//
// Here the build runs level by level, all nodes of a level at once:
//   prep_faces     one thread per face: the three vertices (48 B) and {centroid*area, area}
//                  (16 B), the same f32 expressions as the host build, so the same bits;
//   split_nodes    one workgroup per node to split: the node's {centroid*area, area} gathered
//                  1024 at a time into LDS, then four waves each run ONE of the four ordered
//                  sums (x, y, z in f32, the area in f64) serially from LDS -- the sums must stay
//                  sequential to give the reference's bits, so they are split by component, not
//                  by element;
//   count_children one workgroup per (node, child): vertex-in-box flags, counted;
//   fill_children  one workgroup per (node, child): the same flags compacted in order (wave
//                  ballot + mbcnt prefix, wave totals through LDS) into the next level's
//                  triangle-id buffer at the child's offset.
// The host keeps the level bookkeeping (a few hundred nodes), computes the children boxes by
// selection from (lo, v, hi) exactly as the reference does (no arithmetic), and finally numbers
// the nodes in the reference's order by replaying its LIFO work list over the finished tree
// (children appended as a block of 8 at the current tree length, kd_tree.cpp:262-270). The
// result equals atr::octree_build bit for bit (tests/test_gpu_build.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "engine.h"
#include "host_scene.h"

namespace atr {
namespace {

constexpr int kSplitThreads = 256;   // 4 waves: one per ordered sum
constexpr int kSplitChunk = 1024;    // elements gathered into LDS per round
constexpr int kPartThreads = 256;

struct Seg { float lo[3], hi[3]; uint32_t off, count; };  // a node's box and id segment

__device__ __forceinline__ bool pt_in_d(float x, float y, float z, const float* lo, const float* hi) {
    return (x >= lo[0] && x <= hi[0]) && (y >= lo[1] && y <= hi[1]) && (z >= lo[2] && z <= hi[2]);
}

__global__ void prep_faces(const V3* __restrict__ verts, const int32_t* __restrict__ fv, uint32_t nf,
                           float4_t* __restrict__ tri, float4_t* __restrict__ wsum) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nf) return;
    const V3 a = verts[fv[3 * i]], b = verts[fv[3 * i + 1]], c = verts[fv[3 * i + 2]];
    tri[3 * i] = float4_t{a.x, a.y, a.z, b.x};
    tri[3 * i + 1] = float4_t{b.y, b.z, c.x, c.y};
    tri[3 * i + 2] = float4_t{c.z, 0.f, 0.f, 0.f};
    // kd_tree.cpp:93-114 / area_of_triangle (:3-8), as atr::octree_build evaluates them
    const V3 centroid = divs(add(add(a, b), c), 3.0f);
    const V3 ab = sub(a, b), ac = sub(a, c);
    const float area = sqrtf(len2(cross(ac, ab))) / 2.0f;
    const V3 w = scale(centroid, area);
    wsum[i] = float4_t{w.x, w.y, w.z, area};
}

// out[j] = {v.xyz, 1 if v lies inside node j's box (a split) else 0}
__global__ void __launch_bounds__(kSplitThreads)
split_nodes(const Seg* __restrict__ segs, const uint32_t* __restrict__ ids,
            const float4_t* __restrict__ wsum, float4_t* __restrict__ out) {
    __shared__ float comp[4][kSplitChunk];
    __shared__ float fin[3];
    __shared__ double fin_area;
    const Seg sg = segs[blockIdx.x];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    float acc = 0.f;        // waves 0..2: one component of sum(centroid * area)
    double area_sum = 0.0;  // wave 3: sum(area) in f64
    for (uint32_t base = 0; base < sg.count; base += kSplitChunk) {
        const uint32_t n = sg.count - base < uint32_t(kSplitChunk) ? sg.count - base : uint32_t(kSplitChunk);
        for (uint32_t i = tid; i < n; i += kSplitThreads) {
            const float4_t w = wsum[ids[sg.off + base + i]];
            comp[0][i] = w.x; comp[1][i] = w.y; comp[2][i] = w.z; comp[3][i] = w.w;
        }
        __syncthreads();
        if (lane == 0) {
            const float* c = comp[wave];
            if (wave < 3) {
                for (uint32_t i = 0; i < n; ++i) acc = acc + c[i];
            } else {
                for (uint32_t i = 0; i < n; ++i) area_sum += double(c[i]);
            }
        }
        __syncthreads();
    }
    if (lane == 0) {
        if (wave < 3) fin[wave] = acc;
        else fin_area = area_sum;
    }
    __syncthreads();
    if (tid == 0) {
        const V3 v = divs(mk(fin[0], fin[1], fin[2]), float(fin_area));
        const bool inside = pt_in_d(v.x, v.y, v.z, sg.lo, sg.hi);
        out[blockIdx.x] = float4_t{v.x, v.y, v.z, inside ? 1.f : 0.f};
    }
}

__device__ __forceinline__ bool tri_in(const float4_t* __restrict__ tri, uint32_t f, const float* lo,
                                       const float* hi) {
    const float4_t t0 = tri[3 * f], t1 = tri[3 * f + 1], t2 = tri[3 * f + 2];
    return pt_in_d(t0.x, t0.y, t0.z, lo, hi) || pt_in_d(t0.w, t1.x, t1.y, lo, hi) ||
           pt_in_d(t1.z, t1.w, t2.x, lo, hi);
}

// child segment b: box = child box, off/count = the PARENT's id segment
__global__ void __launch_bounds__(kPartThreads)
count_children(const Seg* __restrict__ child, const uint32_t* __restrict__ ids,
               const float4_t* __restrict__ tri, uint32_t* __restrict__ counts) {
    const Seg sg = child[blockIdx.x];
    uint32_t n = 0;
    for (uint32_t i = threadIdx.x; i < sg.count; i += kPartThreads)
        n += tri_in(tri, ids[sg.off + i], sg.lo, sg.hi) ? 1u : 0u;
    __shared__ uint32_t tot;
    if (threadIdx.x == 0) tot = 0;
    __syncthreads();
    atomicAdd(&tot, n);
    __syncthreads();
    if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(kPartThreads)
fill_children(const Seg* __restrict__ child, const uint32_t* __restrict__ dst_off,
              const uint32_t* __restrict__ ids, const float4_t* __restrict__ tri,
              uint32_t* __restrict__ next) {
    __shared__ uint32_t wtot[kPartThreads / 64];
    const Seg sg = child[blockIdx.x];
    const int tid = threadIdx.x, wave = tid >> 6;
    uint32_t out = dst_off[blockIdx.x];
    for (uint32_t base = 0; base < sg.count; base += kPartThreads) {
        const uint32_t i = base + tid;
        uint32_t f = 0;
        bool keep = false;
        if (i < sg.count) {
            f = ids[sg.off + i];
            keep = tri_in(tri, f, sg.lo, sg.hi);
        }
        const uint64_t m = __ballot(keep);
        const uint32_t before = __builtin_amdgcn_mbcnt_hi(uint32_t(m >> 32), __builtin_amdgcn_mbcnt_lo(uint32_t(m), 0u));
        if ((tid & 63) == 0) wtot[wave] = uint32_t(__popcll(m));
        __syncthreads();
        uint32_t woff = 0, all = 0;
        for (int w = 0; w < kPartThreads / 64; ++w) {
            woff += w < wave ? wtot[w] : 0u;
            all += wtot[w];
        }
        if (keep) next[out + woff + before] = f;
        out += all;
        __syncthreads();
    }
}

__global__ void iota(uint32_t* p, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = i;
}

struct DevBuf {  // owning device allocation, move-only
    void* p = nullptr;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p) { o.p = nullptr; }
    ~DevBuf() { reset(); }
    void reset() { if (p) (void)hipFree(p); p = nullptr; }
    hipError_t alloc(size_t n) { reset(); return hipMalloc(&p, n ? n : 4); }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct Node {  // a node of the level-ordered build
    float lo[3], hi[3];
    int32_t parent = -1, first = -1;  // level-ordered indices; first child block, -1 = leaf
    int depth = 0;
    uint32_t level = 0, off = 0, count = 0;
};

#define BCHK(x)                                        \
    do {                                               \
        hipError_t e_ = (x);                           \
        if (e_ != hipSuccess) return -(1000 + int(e_)); \
    } while (0)

int build_levels(const HostMesh& m, uint32_t max_faces, hipStream_t s, std::vector<Node>& nodes,
                 std::vector<std::vector<uint32_t>>& level_ids, float* dev_ms) {
    const uint32_t nf = uint32_t(m.nfaces()), nv = uint32_t(m.vertices.size());
    DevBuf d_verts, d_fv, d_tri, d_wsum;
    BCHK(d_verts.alloc(size_t(nv) * sizeof(V3)));
    BCHK(d_fv.alloc(size_t(nf) * 12));
    BCHK(d_tri.alloc(size_t(nf) * 48));
    BCHK(d_wsum.alloc(size_t(nf) * 16));
    hipEvent_t e0, e1;
    BCHK(hipEventCreate(&e0));
    BCHK(hipEventCreate(&e1));
    struct EvGuard { hipEvent_t a, b; ~EvGuard() { (void)hipEventDestroy(a); (void)hipEventDestroy(b); } } eg{e0, e1};
    BCHK(hipMemcpyAsync(d_verts.p, m.vertices.data(), size_t(nv) * sizeof(V3), hipMemcpyHostToDevice, s));
    BCHK(hipMemcpyAsync(d_fv.p, m.face_v.data(), size_t(nf) * 12, hipMemcpyHostToDevice, s));
    BCHK(hipEventRecord(e0, s));
    if (nf) {
        prep_faces<<<(nf + 255) / 256, 256, 0, s>>>(d_verts.as<V3>(), d_fv.as<int32_t>(), nf,
                                                     d_tri.as<float4_t>(), d_wsum.as<float4_t>());
        BCHK(hipGetLastError());
    }
    std::vector<DevBuf> lvl(1);
    BCHK(lvl[0].alloc(size_t(nf) * 4));
    if (nf) {
        iota<<<(nf + 255) / 256, 256, 0, s>>>(lvl[0].as<uint32_t>(), nf);
        BCHK(hipGetLastError());
    }
    float box[6];
    mesh_aabb(m, box);
    nodes.assign(1, Node());
    std::memcpy(nodes[0].lo, box, 12);
    std::memcpy(nodes[0].hi, box + 3, 12);
    nodes[0].count = nf;
    size_t lvl_begin = 0;
    DevBuf d_seg, d_out, d_counts, d_dst;
    size_t seg_cap = 0, ch_cap = 0;
    for (uint32_t level = 0;; ++level) {
        const size_t lvl_end = nodes.size();
        std::vector<uint32_t> cand;
        std::vector<Seg> segs;
        for (size_t j = lvl_begin; j < lvl_end; ++j) {
            const Node& nd = nodes[j];
            if (nd.count <= max_faces || nd.depth >= 64) continue;  // leaf (host_scene.cpp octree_build)
            cand.push_back(uint32_t(j));
            Seg sg;
            std::memcpy(sg.lo, nd.lo, 12);
            std::memcpy(sg.hi, nd.hi, 12);
            sg.off = nd.off;
            sg.count = nd.count;
            segs.push_back(sg);
        }
        if (cand.empty()) break;
        const size_t nc = cand.size();
        if (nc > seg_cap) {
            BCHK(d_seg.alloc(nc * 8 * sizeof(Seg)));
            BCHK(d_out.alloc(nc * sizeof(float4_t)));
            seg_cap = nc;
        }
        BCHK(hipMemcpyAsync(d_seg.p, segs.data(), nc * sizeof(Seg), hipMemcpyHostToDevice, s));
        split_nodes<<<uint32_t(nc), kSplitThreads, 0, s>>>(d_seg.as<Seg>(), lvl[level].as<uint32_t>(),
                                                            d_wsum.as<float4_t>(), d_out.as<float4_t>());
        BCHK(hipGetLastError());
        std::vector<float4_t> split(nc);
        BCHK(hipMemcpyAsync(split.data(), d_out.p, nc * sizeof(float4_t), hipMemcpyDeviceToHost, s));
        BCHK(hipStreamSynchronize(s));
        // children of every node that splits: boxes by selection from (lo, v, hi) (kd_tree.cpp:116-148)
        std::vector<Seg> child;
        std::vector<uint32_t> parents;
        for (size_t q = 0; q < nc; ++q) {
            if (split[q].w == 0.f) continue;  // split point outside the box: leaf (kd_tree.cpp:112)
            const Node& nd = nodes[cand[q]];
            const float v[3] = {split[q].x, split[q].y, split[q].z};
            parents.push_back(cand[q]);
            for (int k = 0; k < 8; ++k) {
                const bool side[3] = {bool((k >> 2) & 1), bool((k >> 1) & 1), bool(k & 1)};
                Seg c;
                for (int a = 0; a < 3; ++a) {
                    c.lo[a] = side[a] ? v[a] : nd.lo[a];
                    c.hi[a] = side[a] ? nd.hi[a] : v[a];
                }
                c.off = nd.off;
                c.count = nd.count;
                child.push_back(c);
            }
        }
        if (parents.empty()) break;
        const size_t nch = child.size();
        if (nch > ch_cap) {
            BCHK(d_counts.alloc(nch * 4));
            BCHK(d_dst.alloc(nch * 4));
            ch_cap = nch;
        }
        if (nch > 8 * seg_cap) return ATR_E_INVALID;  // cannot happen: nch <= 8 * nc
        BCHK(hipMemcpyAsync(d_seg.p, child.data(), nch * sizeof(Seg), hipMemcpyHostToDevice, s));
        count_children<<<uint32_t(nch), kPartThreads, 0, s>>>(d_seg.as<Seg>(), lvl[level].as<uint32_t>(),
                                                               d_tri.as<float4_t>(), d_counts.as<uint32_t>());
        BCHK(hipGetLastError());
        std::vector<uint32_t> counts(nch), dst(nch);
        BCHK(hipMemcpyAsync(counts.data(), d_counts.p, nch * 4, hipMemcpyDeviceToHost, s));
        BCHK(hipStreamSynchronize(s));
        uint64_t total = 0;
        for (size_t b = 0; b < nch; ++b) {
            dst[b] = uint32_t(total);
            total += counts[b];
        }
        if (total > 0xFFFFFFFFull) return ATR_E_NOMEM;
        lvl.emplace_back();
        BCHK(lvl.back().alloc(size_t(total) * 4));
        BCHK(hipMemcpyAsync(d_dst.p, dst.data(), nch * 4, hipMemcpyHostToDevice, s));
        fill_children<<<uint32_t(nch), kPartThreads, 0, s>>>(d_seg.as<Seg>(), d_dst.as<uint32_t>(),
                                                              lvl[level].as<uint32_t>(), d_tri.as<float4_t>(),
                                                              lvl.back().as<uint32_t>());
        BCHK(hipGetLastError());
        lvl_begin = nodes.size();
        for (size_t q = 0; q < parents.size(); ++q) {
            const int32_t p = int32_t(parents[q]);
            nodes[p].first = int32_t(nodes.size());
            for (int k = 0; k < 8; ++k) {
                const Seg& c = child[8 * q + k];
                Node nd;
                std::memcpy(nd.lo, c.lo, 12);
                std::memcpy(nd.hi, c.hi, 12);
                nd.parent = p;
                nd.depth = nodes[p].depth + 1;
                nd.level = level + 1;
                nd.off = dst[8 * q + k];
                nd.count = counts[8 * q + k];
                nodes.push_back(nd);
            }
        }
    }
    BCHK(hipEventRecord(e1, s));
    level_ids.assign(lvl.size(), {});
    std::vector<size_t> lvl_size(lvl.size(), 0);
    for (const Node& nd : nodes) lvl_size[nd.level] = std::max<size_t>(lvl_size[nd.level], size_t(nd.off) + nd.count);
    for (size_t l = 0; l < lvl.size(); ++l) {
        level_ids[l].resize(lvl_size[l]);
        if (lvl_size[l])
            BCHK(hipMemcpyAsync(level_ids[l].data(), lvl[l].p, lvl_size[l] * 4, hipMemcpyDeviceToHost, s));
    }
    BCHK(hipStreamSynchronize(s));
    if (dev_ms) BCHK(hipEventElapsedTime(dev_ms, e0, e1));
    return ATR_OK;
}

}  // namespace

// Same contract and result as atr::octree_build; ms_out (optional): [0] wall time of the whole
// call incl. transfers and tree assembly, [1] device time from the first build kernel to the last.
int octree_build_device(const HostMesh& m, uint32_t max_faces, int device, HostTree& T, float* ms_out) {
    const auto t0 = std::chrono::steady_clock::now();
    const size_t nf = m.nfaces();
    for (size_t i = 0; i < 3 * nf; ++i)
        if (m.face_v[i] < 0 || size_t(m.face_v[i]) >= m.vertices.size()) return ATR_E_INVALID;
    if (nf >= 0xFFFFFFFFull) return ATR_E_INVALID;
    int prev = 0;
    BCHK(hipGetDevice(&prev));
    BCHK(hipSetDevice(device));
    hipStream_t s;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e != hipSuccess) { (void)hipSetDevice(prev); return -(1000 + int(e)); }
    std::vector<Node> nodes;
    std::vector<std::vector<uint32_t>> ids;
    float dev_ms = 0.f;
    int rc = build_levels(m, max_faces, s, nodes, ids, &dev_ms);
    (void)hipStreamDestroy(s);
    (void)hipSetDevice(prev);
    if (rc != ATR_OK) return rc;

    // Reference numbering: replay the LIFO work list (kd_tree.cpp:67-288 as octree_build does it).
    std::vector<int32_t> order{0};          // reference id -> level-ordered index
    std::vector<int32_t> ref_of(nodes.size(), -1);
    ref_of[0] = 0;
    std::vector<int32_t> todo{0};
    while (!todo.empty()) {
        const int32_t id = todo.back();
        todo.pop_back();
        const Node& nd = nodes[order[id]];
        if (nd.first < 0) continue;
        const int32_t first = int32_t(order.size());
        for (int k = 0; k < 8; ++k) {
            order.push_back(nd.first + k);
            ref_of[nd.first + k] = first + k;
        }
        for (int k = 0; k < 8; ++k) todo.push_back(first + k);
    }
    T = HostTree();
    const size_t n = order.size();
    T.nnodes = int32_t(n);
    T.bounds.resize(6 * n);
    T.children.resize(n);
    T.parent.resize(n);
    T.depth.resize(n);
    T.leaf_first.assign(n, 0);
    T.leaf_count.assign(n, 0);
    for (size_t i = 0; i < n; ++i) {
        const Node& nd = nodes[order[i]];
        std::memcpy(&T.bounds[6 * i], nd.lo, 12);
        std::memcpy(&T.bounds[6 * i + 3], nd.hi, 12);
        T.children[i] = nd.first < 0 ? 0 : ref_of[nd.first];
        T.parent[i] = nd.parent < 0 ? -1 : ref_of[nd.parent];
        T.depth[i] = nd.depth;
        if (nd.first >= 0) continue;
        T.leaf_first[i] = uint32_t(T.prim_face.size());
        T.leaf_count[i] = nd.count;
        const uint32_t* f = ids[nd.level].data() + nd.off;
        for (uint32_t j = 0; j < nd.count; ++j) {
            const int32_t* fv = &m.face_v[3 * size_t(f[j])];
            for (int k = 0; k < 3; ++k) {
                const V3& v = m.vertices[fv[k]];
                T.prim_vertices.push_back(v.x);
                T.prim_vertices.push_back(v.y);
                T.prim_vertices.push_back(v.z);
            }
            T.prim_face.push_back(f[j]);
        }
    }
    if (ms_out) {
        ms_out[0] = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        ms_out[1] = dev_ms;
    }
    return ATR_OK;
}

}  // namespace atr
