// trace.h -- device-side ray/box/triangle math and the exact octree traversal.
//
// Semantics are the reference's, bit for bit (kd_tree.cpp:337-465, aabb.h:29-93,
// model.h:75-103, renderer.cpp:34-160). What changes is HOW the GPU walks the tree:
//
//  * no per-ray memory: the reference's DFS hit stack becomes an 8-bit "inner children
//    still to visit" mask per tree level packed into two u64 registers (16 levels), with
//    parent indices stored in the nodes for the ascent;
//  * the reference's insertion-sorted leaf list becomes a K-entry register buffer of the
//    K smallest (entry distance, discovery index) leaves; a ray that scans K leaves without
//    a hit re-walks the tree for the next K (ties and order identical to the stable
//    insertion sort at kd_tree.cpp:392-410, whose order is exactly that key).
#pragma once
#include "engine.h"

namespace atr {

// Diagnostic work counters (compiled out unless a COUNT kernel is built): the reference-
// equivalent work (box tests of the first DFS pass + root, triangle tests, leaves scanned) and
// the engine's own extra work (re-walk passes, all box tests, wave-level triangle iterations).
struct Ctr {
    uint32_t box = 0, box_all = 0, tri = 0, leaf = 0, wave_tri = 0, pass = 0;
    uint32_t cbox = 0, screen = 0;  // clustered scan: cluster boxes tested, primitives screened
    // wave clocks (s_memtime) in the FLAT/HYBRID scan's phases: DFS passes, lane-private leaf
    // scans, dealt rounds (atr_render_phase_clocks)
    uint32_t t_pass = 0, t_lp = 0, t_deal = 0, t_prep = 0, t_scan = 0;  // per-wave deltas < 2^32
    // bounce-loop lane use (atr_render_path_counters): wave steps (counted by lane 0) and lanes
    // tracing in them, for bounce 0, bounce 1 and bounces >= 2
    uint32_t steps[3] = {0, 0, 0}, active[3] = {0, 0, 0};
    // SIMD efficiency (atr_render_simd_counters): wave-level iterations of the full-test candidate
    // loops, DFS loop iterations at wave and lane level, dealt rounds and the items they carried
    uint32_t cand_wave = 0, node_wave = 0, node_lane = 0, round_wave = 0, round_items = 0;
};

// 1 in the lowest active lane of the wavefront (counts a divergent loop's wave-level iterations)
__device__ __forceinline__ uint32_t first_active_lane() {
    return (threadIdx.x & 63) == uint32_t(__builtin_ctzll(__ballot(1))) ? 1u : 0u;
}

// Pointers into the scene's device tables are generic (loaded from memory): cast to the global
// address space, the table loads are global loads instead of flat loads. uniform_global also
// makes the value wave-uniform (readfirstlane: SGPRs) -- only for pointers every lane shares.
template <class T>
__device__ __forceinline__ T* as_global(T* p) {
    using G = __attribute__((address_space(1))) T;
    return (T*)(reinterpret_cast<G*>(reinterpret_cast<uint64_t>(p)));
}
template <class T>
__device__ __forceinline__ T* uniform_global(T* p) {
    const uint64_t v = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane(uint32_t(v)), hi = __builtin_amdgcn_readfirstlane(uint32_t(v >> 32));
    using G = __attribute__((address_space(1))) T;
    return (T*)(reinterpret_cast<G*>((uint64_t(hi) << 32) | lo));
}

struct Ray {
    V3 o, d, inv;
    int s0, s1, s2;  // inv_signs (renderer.cpp:41-44)
};

__device__ __forceinline__ Ray make_ray(V3 o, V3 d) {
    Ray r;
    r.o = o;
    r.d = d;
    r.inv = mk(1 / d.x, 1 / d.y, 1 / d.z);
    r.s0 = r.inv.x < 0;
    r.s1 = r.inv.y < 0;
    r.s2 = r.inv.z < 0;
    return r;
}

struct NodeBox { float lx, ly, lz, hx, hy, hz; int32_t children, parent; };

__device__ __forceinline__ NodeBox load_node(const DNode* __restrict__ nodes, int32_t i) {
    const float4* p = reinterpret_cast<const float4*>(nodes + i);
    const float4 a = p[0], b = p[1];
    NodeBox n;
    n.lx = a.x; n.ly = a.y; n.lz = a.z; n.hx = a.w;
    n.hy = b.x; n.hz = b.y;
    n.children = __float_as_int(b.z);
    n.parent = __float_as_int(b.w);
    return n;
}

// check_ray_AABB_intersection (aabb.h:65-93): no z merge, no t > 0 requirement.
__device__ __forceinline__ bool box_check(const Ray& r, float lx, float ly, float lz, float hx,
                                          float hy, float hz) {
    float tmin = ((r.s0 ? hx : lx) - r.o.x) * r.inv.x;
    float tmax = ((r.s0 ? lx : hx) - r.o.x) * r.inv.x;
    const float tymin = ((r.s1 ? hy : ly) - r.o.y) * r.inv.y;
    const float tymax = ((r.s1 ? ly : hy) - r.o.y) * r.inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return false;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    const float tzmin = ((r.s2 ? hz : lz) - r.o.z) * r.inv.z;
    const float tzmax = ((r.s2 ? lz : hz) - r.o.z) * r.inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return false;
    return true;
}

// get_ray_AABB_intersection (aabb.h:29-63): entry t, else exit t (origin inside), else 0.
__device__ __forceinline__ float box_entry(const Ray& r, float lx, float ly, float lz, float hx,
                                           float hy, float hz) {
    float tmin = ((r.s0 ? hx : lx) - r.o.x) * r.inv.x;
    float tmax = ((r.s0 ? lx : hx) - r.o.x) * r.inv.x;
    const float tymin = ((r.s1 ? hy : ly) - r.o.y) * r.inv.y;
    const float tymax = ((r.s1 ? ly : hy) - r.o.y) * r.inv.y;
    if ((tmin > tymax) || (tymin > tmax)) return 0;
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    const float tzmin = ((r.s2 ? hz : lz) - r.o.z) * r.inv.z;
    const float tzmax = ((r.s2 ? lz : hz) - r.o.z) * r.inv.z;
    if ((tmin > tzmax) || (tzmin > tmax)) return 0;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    if (tmin > 0) return tmin;
    if (tmax > 0) return tmax;
    return 0;
}

struct TriRec { V3 a, ab, ac; uint32_t face; };

__device__ __forceinline__ TriRec load_tri(const DTri* __restrict__ tris, uint32_t i) {
    const float4* p = reinterpret_cast<const float4*>(tris + i);
    const float4 q0 = p[0], q1 = p[1], q2 = p[2];
    TriRec t;
    t.a = mk(q0.x, q0.y, q0.z);
    t.ab = mk(q0.w, q1.x, q1.y);
    t.ac = mk(q1.z, q1.w, q2.x);
    t.face = __float_as_uint(q2.y);
    return t;
}

// 1 / x correctly rounded (the reference's f32 division, model.h:84) for the culled test's det
// (x >= kTol): the hardware reciprocal (1 ulp) and two FMA corrections, 5 VALU instead of the
// 10 of the general IEEE division expansion (scaling, denormal and overflow handling the det never
// needs). Checked equal to 1.0f / x bit for bit for every f32 in [2^-14, 2^64) on the GPU
// (tests/c/recip_check.hip, tests/test_gpu_recip.py); outside that range (and for NaN) the division.
__device__ __forceinline__ float recip_det(float x) {
#ifdef ATR_IEEE_RECIP
    return 1.0f / x;
#else
    if (!(x < 18446744073709551616.0f)) return 1.0f / x;  // 2^64
    float r = __builtin_amdgcn_rcpf(x);
    float e = __builtin_fmaf(-x, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
#endif
}

// get_triangle_ray_intersection_culled (model.h:75-103); ab/ac precomputed on the host.
__device__ __forceinline__ float tri_hit(const Ray& r, V3 a, V3 ab, V3 ac, float& u, float& v) {
    const V3 pvec = cross(r.d, ac);
    const float det = dot(ab, pvec);
    if (det < kTol) return 0;
    const float det_inv = recip_det(det);
    const V3 tvec = sub(r.o, a);
    u = dot(tvec, pvec) * det_inv;
    if (u < 0 || u > 1) return 0;
    const V3 qvec = cross(tvec, ab);
    v = dot(r.d, qvec) * det_inv;
    if (v < 0 || u + v > 1) return 0;
    return dot(qvec, ac) * det_inv;
}

struct Hit {
    float t;      // closest accepted distance (kMaxFloat = none)
    uint32_t face;
    float u, v;
};

// Scan one leaf's primitives in leaf order (kd_tree.cpp:440-456). True if `h` improved.
template <bool COUNT>
__device__ __forceinline__ bool scan_leaf(const Ray& r, const DTri* __restrict__ tris, uint32_t first,
                                          uint32_t count, Hit& h, Ctr& ct) {
    if constexpr (COUNT) { ct.tri += count; ct.leaf += 1; }
    bool improved = false;
    for (uint32_t k = 0; k < count; ++k) {
        const TriRec t = load_tri(tris, first + k);
        float u = 0.f, v = 0.f;
        const float dist = tri_hit(r, t.a, t.ab, t.ac, u, v);
        if (dist < h.t && dist > kTol) {
            h.t = dist;
            h.face = t.face;
            h.u = u;
            h.v = v;
            improved = true;
        }
    }
    return improved;
}

// ------------------------------------------------------------------ leaf order buffer
constexpr int kLeafBuf = 8;  // sorted leaves held per ray between DFS passes

// {first, count} of leaf `leaf` in a per-leaf range table (one 8-B load)
__device__ __forceinline__ uint2_t load_range(const uint32_t* __restrict__ range, int32_t leaf) {
    return reinterpret_cast<const uint2_t*>(range)[leaf];
}

template <int K>
struct LeafBuf {
    float d[K];
    int32_t leaf[K];  // leaf id = the leaf's rank in the static discovery order (inner_table)
};

template <int K>
__device__ __forceinline__ void lb_clear(LeafBuf<K>& b) {
#pragma unroll
    for (int j = 0; j < K; ++j) { b.d[j] = __builtin_inff(); b.leaf[j] = 0; }
}

// Insert a leaf discovered after every entry already held (larger discovery rank): it goes
// behind every entry with distance <= dis, as the stable insertion sort does.
template <int K>
__device__ __forceinline__ void lb_insert(LeafBuf<K>& b, float dis, int32_t leaf) {
    if (!(dis < b.d[K - 1])) return;
    b.d[K - 1] = dis;
    b.leaf[K - 1] = leaf;
#pragma unroll
    for (int j = K - 1; j > 0; --j) {
        if (b.d[j] < b.d[j - 1]) {
            const float td = b.d[j]; b.d[j] = b.d[j - 1]; b.d[j - 1] = td;
            const int32_t tl = b.leaf[j]; b.leaf[j] = b.leaf[j - 1]; b.leaf[j - 1] = tl;
        }
    }
}

// Sorted-leaf scan with a rotating head: entry 0 is always the next leaf, the buffer shifts
// down after each scanned leaf (static register moves, no dynamically indexed arrays).
template <int K>
__device__ __forceinline__ void lb_pop(LeafBuf<K>& b) {
#pragma unroll
    for (int j = 0; j + 1 < K; ++j) { b.d[j] = b.d[j + 1]; b.leaf[j] = b.leaf[j + 1]; }
    b.d[K - 1] = __builtin_inff();
}

// The same buffer held in LDS (lane-private column: entry j of lane ln at word 64 j + ln, no
// bank conflicts): registers keep only the entry count and the admission bound, so the DFS pass
// no longer carries 2K registers. An insert shifts the entries with a larger distance up one
// slot (the last drops out when full): the same order as lb_insert.
template <int K>
struct LdsLeafBuf {
    float* d;       // column base of the distances
    int32_t* leaf;  // column base of the leaf ids
    int32_t n;      // entries held
    float thr;      // d[K - 1] when full, else +inf: an insert needs dis < thr
    int32_t thr_leaf;  // leaf[K - 1] when full (near-first passes: (dis, rank) order)
};

template <int K>
__device__ __forceinline__ void lb_clear(LdsLeafBuf<K>& b) {
    b.n = 0;
    b.thr = __builtin_inff();
    b.thr_leaf = 0x7FFFFFFF;
}

// Insert in (distance, rank) order for passes that discover leaves out of rank order
// (traverse_pass_near): a leaf goes behind every entry that precedes it in that order -- the
// position the stable insertion sort (kd_tree.cpp:392-410) gives it, since its discovery order IS
// the rank order.
template <int K>
__device__ __forceinline__ void lb_insert_lex(LdsLeafBuf<K>& b, float dis, int32_t leaf) {
    if (!(dis < b.thr || (dis == b.thr && leaf < b.thr_leaf))) return;
    int j = b.n < K ? b.n : K - 1;
    for (; j > 0; --j) {
        const float pd = b.d[64 * (j - 1)];
        const int32_t pl = b.leaf[64 * (j - 1)];
        if (!(pd > dis || (pd == dis && pl > leaf))) break;
        b.d[64 * j] = pd;
        b.leaf[64 * j] = pl;
    }
    b.d[64 * j] = dis;
    b.leaf[64 * j] = leaf;
    if (b.n < K) ++b.n;
    if (b.n == K) {
        b.thr = b.d[64 * (K - 1)];
        b.thr_leaf = b.leaf[64 * (K - 1)];
    }
}

template <int K>
__device__ __forceinline__ void lb_insert(LdsLeafBuf<K>& b, float dis, int32_t leaf) {
    if (!(dis < b.thr)) return;
    int j = b.n < K ? b.n : K - 1;
    for (; j > 0; --j) {
        const float pd = b.d[64 * (j - 1)];
        if (!(pd > dis)) break;
        b.d[64 * j] = pd;
        b.leaf[64 * j] = b.leaf[64 * (j - 1)];
    }
    b.d[64 * j] = dis;
    b.leaf[64 * j] = leaf;
    if (b.n < K) ++b.n;
    if (b.n == K) b.thr = b.d[64 * (K - 1)];
}

template <int K>
__device__ __forceinline__ int32_t lb_leaf(const LeafBuf<K>& b, int j) {
    int32_t r = b.leaf[0];
#pragma unroll
    for (int q = 1; q < K; ++q) r = (j == q) ? b.leaf[q] : r;
    return r;
}

// One inner node of the derived-box table (engine.h DModel::inner).
struct Inner {
    float lx, ly, lz, vx, vy, vz, hx, hy, hz;
    int32_t leaf0;   // discovery rank of the first leaf child (leaf children are consecutive)
    int32_t parent;  // parent's inner id, -1 at the root
    uint32_t bm;     // (inner id of the first inner child << 8) | leaf-children mask
};

__device__ __forceinline__ Inner load_inner(const float4_t* __restrict__ tab, int32_t i) {
    const float4_t a = tab[3 * i], b = tab[3 * i + 1], c = tab[3 * i + 2];
    Inner n;
    n.lx = a.x; n.ly = a.y; n.lz = a.z; n.vx = a.w;
    n.vy = b.x; n.vz = b.y; n.hx = b.z; n.hy = b.w;
    n.hz = c.x;
    n.leaf0 = __float_as_int(c.y);
    n.parent = __float_as_int(c.z);
    n.bm = __float_as_uint(c.w);
    return n;
}

// The same record at a wave-uniform index, read by the scalar unit into SGPRs (one fetch per
// wavefront, no VGPRs for the record): s_load of 32 + 16 bytes. The table is read-only for the
// kernel's lifetime, so the scalar cache cannot hold a stale copy.
typedef uint32_t u32x8_t __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ Inner load_inner_uniform(const float4_t* __restrict__ tab, int32_t i) {
    const uint64_t a64 = reinterpret_cast<uint64_t>(tab + 3 * i);
    const uint64_t u64 = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int32_t(uint32_t(a64))))) |
                         (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int32_t(uint32_t(a64 >> 32))))) << 32);
    const float4_t* p = reinterpret_cast<const float4_t*>(u64);
    u32x8_t a;
    u32x4_t c;
    // early-clobber outputs ("=&s"): the first load's destination must not share registers with
    // the address the second load reads. Without them the compiler may allocate a over p (it
    // did: s_load_dwordx8 s[12:19], s[12:13] then s_load_dwordx4 ..., s[12:13]); a fast return
    // of the first load then turned the second's address into loaded data -- the rare
    // MEMORY_APERTURE_VIOLATION of rounds 4 and 5
    asm volatile("s_load_dwordx8 %0, %2, 0x0\n\ts_load_dwordx4 %1, %2, 0x20\n\ts_waitcnt lgkmcnt(0)"
                 : "=&s"(a), "=&s"(c)
                 : "s"(p));
    Inner n;
    n.lx = __uint_as_float(a[0]); n.ly = __uint_as_float(a[1]); n.lz = __uint_as_float(a[2]);
    n.vx = __uint_as_float(a[3]); n.vy = __uint_as_float(a[4]); n.vz = __uint_as_float(a[5]);
    n.hx = __uint_as_float(a[6]); n.hy = __uint_as_float(a[7]);
    n.hz = __uint_as_float(c[0]);
    n.leaf0 = int32_t(c[1]);
    n.parent = int32_t(c[2]);
    n.bm = c[3];
    return n;
}

// Examine the children of an inner node (kd_tree.cpp:370-434): box-test children in order
// until 5 have been hit; inner hits -> returned bit mask, leaf hits -> leaf order buffer.
// The children boxes are the octants of (lo, v, hi) (kd_tree.cpp:116-148), so every slab
// value a child test needs is one of three per axis, (b - o) * inv for b in {lo, v, hi}: the
// same f32 operations on the same operands as the reference's per-child slab test
// (aabb.h:29-93), hence the same bits, computed once per node instead of per child and with
// no child box loads. Child k: x half = k >> 2, y half = (k >> 1) & 1, z half = k & 1.
// Descent cull: an inner child whose exit distance (its slab exit, z merged as aabb.h:29-63
// computes it) is <= 0 or < bd holds no leaf the pass could insert -- every leaf below it is an
// octant of an octant (bitwise, checked at upload), so its slab values lie between the child's
// (b - o) * inv is monotone in b under f32 rounding) and its distance (entry, else exit, else 0)
// is <= that exit: 0 (not inserted) or below the re-walk bound. The child still counts as hit for
// the reference's 5-hit limit (kd_tree.cpp:374); only the walk into it is skipped. Valid when
// no slab value can be NaN, i.e. 1/d is finite on every axis (`cull`, per ray); the rays it
// helps are bounce rays, whose origins lie inside the tree and whose lines cross boxes behind
// them (check_ray_AABB_intersection has no t > 0 test, aabb.h:65-93).
template <int K, bool COUNT, class LB>
__device__ __forceinline__ uint32_t examine_inner(const Ray& r, const Inner& n, LB& lb,
                                                  int32_t& ncand, float bd, int32_t bi, Ctr& ct,
                                                  bool first_pass, bool cull = false) {
    const float X0 = (n.lx - r.o.x) * r.inv.x, X1 = (n.vx - r.o.x) * r.inv.x, X2 = (n.hx - r.o.x) * r.inv.x;
    const float Y0 = (n.ly - r.o.y) * r.inv.y, Y1 = (n.vy - r.o.y) * r.inv.y, Y2 = (n.hy - r.o.y) * r.inv.y;
    const float Z0 = (n.lz - r.o.z) * r.inv.z, Z1 = (n.vz - r.o.z) * r.inv.z, Z2 = (n.hz - r.o.z) * r.inv.z;
    // near/far slab value of the low (0) and high (1) half per axis: bounds[inv_signs] is the
    // max when the inverse direction is negative (aabb.h:33-34)
    const float nx0 = r.s0 ? X1 : X0, nx1 = r.s0 ? X2 : X1, fx0 = r.s0 ? X0 : X1, fx1 = r.s0 ? X1 : X2;
    const float ny0 = r.s1 ? Y1 : Y0, ny1 = r.s1 ? Y2 : Y1, fy0 = r.s1 ? Y0 : Y1, fy1 = r.s1 ? Y1 : Y2;
    const float nz0 = r.s2 ? Z1 : Z0, nz1 = r.s2 ? Z2 : Z1, fz0 = r.s2 ? Z0 : Z1, fz1 = r.s2 ? Z1 : Z2;
    uint32_t mask = 0;
    int nodes_hit = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (nodes_hit > 4) break;
        if constexpr (COUNT) { ct.box_all += 1; ct.box += first_pass ? 1u : 0u; }
        float tmin = (i >> 2) ? nx1 : nx0, tmax = (i >> 2) ? fx1 : fx0;
        const float tymin = ((i >> 1) & 1) ? ny1 : ny0, tymax = ((i >> 1) & 1) ? fy1 : fy0;
        const float tzmin = (i & 1) ? nz1 : nz0, tzmax = (i & 1) ? fz1 : fz0;
        bool in = !((tmin > tymax) || (tymin > tmax));
        if (tymin > tmin) tmin = tymin;
        if (tymax < tmax) tmax = tymax;
        in = in && !((tmin > tzmax) || (tzmin > tmax));
        if (!((n.bm >> i) & 1u)) {  // inner child: check_ray_AABB_intersection (aabb.h:65-93)
            if (in) {
                ++nodes_hit;
                const float tx = tzmax < tmax ? tzmax : tmax;
                if (!(cull && (tx <= 0.0f || tx < bd))) mask |= 1u << i;
            }
        } else {  // leaf child: get_ray_AABB_intersection (aabb.h:29-63)
            if (tzmin > tmin) tmin = tzmin;
            if (tzmax < tmax) tmax = tzmax;
            const float dis = !in ? 0.0f : (tmin > 0 ? tmin : (tmax > 0 ? tmax : 0.0f));
            if (dis > 0.0f) {
                ++nodes_hit;
                // the static discovery rank orders leaves exactly as this pass discovers them
                const int32_t id = n.leaf0 + __popc(n.bm & ((1u << i) - 1u) & 0xFFu);
                if (dis > bd || (dis == bd && id > bi)) {
                    ++ncand;
                    lb_insert<K>(lb, dis, id);
                }
            }
        }
    }
    return mask;
}

// One DFS pass over the inner nodes (the reference's hit-stack loop, kd_tree.cpp:363-435),
// keeping the K first leaves (in sorted order) strictly after (bd, bi). Returns the number of
// candidate leaves after the bound, or -1 if the tree is deeper than the mask stack.
// Per level the stack keeps only the 8-bit mask of inner children still to visit (popped
// highest first = the reference's LIFO order); a descent reads the child's 48-B record, an
// ascent the last 16 B of the parent's.
template <int K, bool COUNT, class LB>
__device__ __forceinline__ int32_t traverse_pass(const Ray& r, const float4_t* __restrict__ tab,
                                                 LB& lb, float bd, int32_t bi, Ctr& ct) {
    const bool first_pass = bi < 0;
    if constexpr (COUNT) ct.pass += 1;
    lb_clear<K>(lb);
    int32_t ncand = 0;
#ifdef ATR_NO_CULL
    const bool cull = false;  // experiment build: the round-2 walk
#else
    const bool cull = isfinite(r.inv.x) && isfinite(r.inv.y) && isfinite(r.inv.z);
#endif
    Inner cur = load_inner(tab, 0);
    uint64_t lo = examine_inner<K, COUNT>(r, cur, lb, ncand, bd, bi, ct, first_pass, cull);
    uint64_t hi = 0;
    uint32_t bm = cur.bm;
    int32_t parent = -1, lvl = 0;
    for (;;) {
        if constexpr (COUNT) { ct.node_wave += first_active_lane(); ct.node_lane += 1; }
        const uint32_t m = lvl < 8 ? uint32_t(lo >> (8 * lvl)) & 0xFFu : uint32_t(hi >> (8 * (lvl - 8))) & 0xFFu;
        if (m) {
            const int s = 31 - __clz(m);
            if (lvl < 8) lo &= ~(uint64_t(1) << (8 * lvl + s));
            else hi &= ~(uint64_t(1) << (8 * (lvl - 8) + s));
            const uint32_t innerm = ~bm & ((1u << s) - 1u);  // inner children before s
            const int32_t id = int32_t(bm >> 8) + __popc(innerm);
            cur = load_inner(tab, id);
            const uint64_t cm = examine_inner<K, COUNT>(r, cur, lb, ncand, bd, bi, ct, first_pass, cull);
            ++lvl;
            if (lvl >= kMaskLevels) return -1;
            if (lvl < 8) lo |= cm << (8 * lvl);
            else hi |= cm << (8 * (lvl - 8));
            bm = cur.bm;
            parent = cur.parent;
        } else {
            if (lvl == 0) break;
            --lvl;
            const float4_t t = tab[3 * parent + 2];
            bm = __float_as_uint(t.w);
            parent = __float_as_int(t.z);
        }
    }
    return ncand;
}

// Near-first pass (incoherent bounce rays; LDS leaf buffer): the same leaf set as traverse_pass --
// every inner child is still examined with the reference's per-node child loop and 5-hit limit
// (examine_inner) -- but a node's inner children are descended in the order the ray crosses them:
// with the child index mirrored by the direction signs (i ^ sm, sm = x, y, z sign bits), the
// octants a line crosses have increasing mirrored indices (each plane crossing sets one more bit),
// so the per-level mask is kept mirrored and popped lowest bit first. The nearest leaves then
// fill the K-entry buffer first, and once it is full a subtree whose entry distance exceeds its
// K-th distance is skipped: every leaf below it has a distance >= that entry (nested octant boxes,
// monotone f32 slab values; a leaf the origin lies in has dis = its exit > 0 >= its entry), so
// none could enter the buffer. Skipping makes the candidate count a lower bound, so a pass that
// skipped anything reports more than K candidates (the ray re-walks after its K leaves, as a pass
// with more than K candidates does). Leaves are discovered out of rank order: the buffer keeps
// (distance, rank) order (lb_insert_lex). Skips only with finite 1/d on every axis (no NaN slabs).
template <int K, bool COUNT>
__device__ __forceinline__ uint32_t examine_near(const Ray& r, const Inner& n, LdsLeafBuf<K>& lb, int32_t& ncand,
                                                 float bd, int32_t bi, Ctr& ct, bool first_pass, bool cull,
                                                 uint32_t sm, bool& skipped) {
    const float X0 = (n.lx - r.o.x) * r.inv.x, X1 = (n.vx - r.o.x) * r.inv.x, X2 = (n.hx - r.o.x) * r.inv.x;
    const float Y0 = (n.ly - r.o.y) * r.inv.y, Y1 = (n.vy - r.o.y) * r.inv.y, Y2 = (n.hy - r.o.y) * r.inv.y;
    const float Z0 = (n.lz - r.o.z) * r.inv.z, Z1 = (n.vz - r.o.z) * r.inv.z, Z2 = (n.hz - r.o.z) * r.inv.z;
    const float nx0 = r.s0 ? X1 : X0, nx1 = r.s0 ? X2 : X1, fx0 = r.s0 ? X0 : X1, fx1 = r.s0 ? X1 : X2;
    const float ny0 = r.s1 ? Y1 : Y0, ny1 = r.s1 ? Y2 : Y1, fy0 = r.s1 ? Y0 : Y1, fy1 = r.s1 ? Y1 : Y2;
    const float nz0 = r.s2 ? Z1 : Z0, nz1 = r.s2 ? Z2 : Z1, fz0 = r.s2 ? Z0 : Z1, fz1 = r.s2 ? Z1 : Z2;
    const bool full = cull && lb.n == K;
    uint32_t mask = 0;
    int nodes_hit = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (nodes_hit > 4) break;
        if constexpr (COUNT) { ct.box_all += 1; ct.box += first_pass ? 1u : 0u; }
        float tmin = (i >> 2) ? nx1 : nx0, tmax = (i >> 2) ? fx1 : fx0;
        const float tymin = ((i >> 1) & 1) ? ny1 : ny0, tymax = ((i >> 1) & 1) ? fy1 : fy0;
        const float tzmin = (i & 1) ? nz1 : nz0, tzmax = (i & 1) ? fz1 : fz0;
        bool in = !((tmin > tymax) || (tymin > tmax));
        if (tymin > tmin) tmin = tymin;
        if (tymax < tmax) tmax = tymax;
        in = in && !((tmin > tzmax) || (tzmin > tmax));
        if (!((n.bm >> i) & 1u)) {  // inner child: check_ray_AABB_intersection (aabb.h:65-93)
            if (in) {
                ++nodes_hit;
                const float tx = tzmax < tmax ? tzmax : tmax;
                const float tn = tzmin > tmin ? tzmin : tmin;  // its entry distance (z merged)
                if (cull && (tx <= 0.0f || tx < bd)) continue;  // behind the origin or the re-walk bound
                if (full && tn > lb.thr) { skipped = true; continue; }
                mask |= 1u << i;
            }
        } else {  // leaf child: get_ray_AABB_intersection (aabb.h:29-63)
            if (tzmin > tmin) tmin = tzmin;
            if (tzmax < tmax) tmax = tzmax;
            const float dis = !in ? 0.0f : (tmin > 0 ? tmin : (tmax > 0 ? tmax : 0.0f));
            if (dis > 0.0f) {
                ++nodes_hit;
                const int32_t id = n.leaf0 + __popc(n.bm & ((1u << i) - 1u) & 0xFFu);
                if (dis > bd || (dis == bd && id > bi)) {
                    ++ncand;
                    lb_insert_lex<K>(lb, dis, id);
                }
            }
        }
    }
    // bit i -> bit i ^ sm, mirrored once here (per-child shifts by (i ^ sm) were hoisted out of the
    // pass loop as eight per-lane constants, and spilled)
    if (sm & 4u) mask = ((mask & 0x0Fu) << 4) | ((mask & 0xF0u) >> 4);
    if (sm & 2u) mask = ((mask & 0x33u) << 2) | ((mask & 0xCCu) >> 2);
    if (sm & 1u) mask = ((mask & 0x55u) << 1) | ((mask & 0xAAu) >> 1);
    return mask;
}

// The pass's stack lives in registers, one 32-bit entry per level: the level's remaining inner
// children (mirrored mask, bits 0-7), the node's leaf-children mask (8-15) and its first inner
// child's id (16-31) -- everything a pop needs, so an ascent is a register shift and every loop
// iteration is one descent (the mask stack of traverse_pass re-reads the parent's record on each
// ascent: a dependent load per level climbed). A node with no inner child to visit is not pushed.
// Holds kNearLevels levels (four u64, the top entry in the low half of s0); trees deeper than that,
// or with 2^16 or more inner nodes, take traverse_pass (DModel::near_ok, set at upload).
constexpr int kNearLevels = 8;
template <int K, bool COUNT>
__device__ __forceinline__ int32_t traverse_pass_near(const Ray& r, const float4_t* __restrict__ tab,
                                                      LdsLeafBuf<K>& lb, float bd, int32_t bi, Ctr& ct) {
    const bool first_pass = bi < 0;
    if constexpr (COUNT) ct.pass += 1;
    lb_clear<K>(lb);
    int32_t ncand = 0;
    const bool cull = isfinite(r.inv.x) && isfinite(r.inv.y) && isfinite(r.inv.z);
    const uint32_t sm = (uint32_t(r.s0) << 2) | (uint32_t(r.s1) << 1) | uint32_t(r.s2);
    bool skipped = false;
    Inner cur = load_inner(tab, 0);
    const uint32_t m0 = examine_near<K, COUNT>(r, cur, lb, ncand, bd, bi, ct, first_pass, cull, sm, skipped);
    uint64_t s0 = m0 ? uint64_t(m0 | ((cur.bm & 0xFFu) << 8) | ((cur.bm >> 8) << 16)) : 0, s1 = 0, s2 = 0, s3 = 0;
    int32_t depth = m0 ? 1 : 0;
    for (;;) {
        while (depth > 0 && (uint32_t(s0) & 0xFFu) == 0) {  // ascend: pop the exhausted levels
            s0 = (s0 >> 32) | (s1 << 32);
            s1 = (s1 >> 32) | (s2 << 32);
            s2 = (s2 >> 32) | (s3 << 32);
            s3 >>= 32;
            --depth;
        }
        if (depth == 0) break;
        if constexpr (COUNT) { ct.node_wave += first_active_lane(); ct.node_lane += 1; }
        const uint32_t top = uint32_t(s0);
        const int sb = __builtin_ctz(top & 0xFFu);  // nearest remaining child (mirrored index)
        s0 &= ~uint64_t(1u << sb);
        const int s = sb ^ int(sm);
        const uint32_t innerm = ~(top >> 8) & ((1u << s) - 1u) & 0xFFu;  // inner children before s
        const int32_t id = int32_t(top >> 16) + __popc(innerm);
        cur = load_inner(tab, id);
        if (cull && lb.n == K) {  // the buffer filled since this child was pushed: its entry
            const float ex = r.s0 ? (cur.hx - r.o.x) * r.inv.x : (cur.lx - r.o.x) * r.inv.x;
            const float ey = r.s1 ? (cur.hy - r.o.y) * r.inv.y : (cur.ly - r.o.y) * r.inv.y;
            const float ez = r.s2 ? (cur.hz - r.o.z) * r.inv.z : (cur.lz - r.o.z) * r.inv.z;
            const float txy = ey > ex ? ey : ex;
            if ((ez > txy ? ez : txy) > lb.thr) { skipped = true; continue; }
        }
        const uint32_t cm = examine_near<K, COUNT>(r, cur, lb, ncand, bd, bi, ct, first_pass, cull, sm, skipped);
        if (cm) {  // push the node's level
            if (depth >= kNearLevels) return -1;
            s3 = (s3 << 32) | (s2 >> 32);
            s2 = (s2 << 32) | (s1 >> 32);
            s1 = (s1 << 32) | (s0 >> 32);
            s0 = (s0 << 32) | uint64_t(cm | ((cur.bm & 0xFFu) << 8) | ((cur.bm >> 8) << 16));
            ++depth;
        }
    }
    return skipped && ncand <= K ? K + 1 : ncand;
}

// The same pass walked by the whole wavefront (coherent primary rays): the wave visits the union
// of its lanes' DFS paths in the common order (highest inner child first, each subtree before
// the next), reading each inner record once per wave with scalar loads; a lane examines a node
// only if its own pass would visit it (the node is in the lane's own child mask), so every lane
// discovers exactly the leaves -- with the same distances and static ranks -- its lane-private
// pass discovers, in the same order. Called by every lane of the wave (converged); `part` = this
// lane runs a pass. Returns the lane's candidate count (-1: tree deeper than the mask stack).
template <int K, bool COUNT, class LB>
__device__ __forceinline__ int32_t traverse_pass_wave(const Ray& r, const float4_t* __restrict__ tab, LB& lb,
                                                      float bd, int32_t bi, Ctr& ct, bool part) {
    const bool first_pass = bi < 0;
    if constexpr (COUNT) { if (part) ct.pass += 1; }
    if (part) lb_clear<K>(lb);
    int32_t ncand = 0;
#ifdef ATR_NO_CULL
    const bool cull = false;  // experiment build: the round-2 walk
#else
    const bool cull = isfinite(r.inv.x) && isfinite(r.inv.y) && isfinite(r.inv.z);
#endif
    Inner cur = load_inner_uniform(tab, 0);
    uint64_t lo = part ? uint64_t(examine_inner<K, COUNT>(r, cur, lb, ncand, bd, bi, ct, first_pass, cull)) : 0;
    uint64_t hi = 0;
    uint32_t bm = cur.bm;  // wave-uniform walk state
    int32_t parent = -1, lvl = 0;
    for (;;) {
        if constexpr (COUNT) { ct.node_wave += (threadIdx.x & 63) == 0 ? 1u : 0u; ct.node_lane += part ? 1u : 0u; }
        const uint32_t mine = lvl < 8 ? uint32_t(lo >> (8 * lvl)) & 0xFFu : uint32_t(hi >> (8 * (lvl - 8))) & 0xFFu;
        int s = -1;  // highest child any lane still has to visit at this level
        for (int b = 7; b >= 0; --b)
            if (__ballot((mine >> b) & 1u)) { s = b; break; }
        if (s >= 0) {
            const bool act = (mine >> s) & 1u;
            if (lvl < 8) lo &= ~(uint64_t(1) << (8 * lvl + s));
            else hi &= ~(uint64_t(1) << (8 * (lvl - 8) + s));
            const uint32_t innerm = ~bm & ((1u << s) - 1u);
            const int32_t id = int32_t(bm >> 8) + __popc(innerm);
            cur = load_inner_uniform(tab, id);
            const uint64_t cm = act ? uint64_t(examine_inner<K, COUNT>(r, cur, lb, ncand, bd, bi, ct, first_pass, cull)) : 0;
            ++lvl;
            if (lvl >= kMaskLevels) return -1;
            if (lvl < 8) lo |= cm << (8 * lvl);
            else hi |= cm << (8 * (lvl - 8));
            bm = cur.bm;
            parent = cur.parent;
        } else {
            if (lvl == 0) break;
            --lvl;
            const Inner p = load_inner_uniform(tab, parent);
            bm = p.bm;
            parent = p.parent;
        }
    }
    return part ? ncand : 0;
}

}  // namespace atr
