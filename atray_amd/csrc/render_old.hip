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

#include <type_traits>

#include "cluster.h"
#include "shade.h"
#include "trace.h"

namespace atr {

// ------------------------------------------------------------------ LANE schedule
// Per-lane leaf scan over the SoA triangle streams, one triangle of prefetch: the loads of
// triangle k+1 are in flight while triangle k is tested. The hit keeps the primitive SLOT;
// its face index is read once, after the tree query.
struct TriRegs { float4_t q0, q1; float q2; };

__device__ __forceinline__ void tri_fetch(const DModel& m, uint32_t i, TriRegs& t) {
    t.q0 = m.t0[i];
    t.q1 = m.t1[i];
    t.q2 = m.t2[i];
}

__device__ __forceinline__ void tri_test(const Ray& r, const TriRegs& t, uint32_t slot, float& best_t,
                                         uint32_t& best_slot, float& bu, float& bv, bool& improved) {
    float u = 0.f, v = 0.f;
    const float dist = tri_hit(r, mk(t.q0.x, t.q0.y, t.q0.z), mk(t.q0.w, t.q1.x, t.q1.y),
                               mk(t.q1.z, t.q1.w, t.q2), u, v);
    if (dist < best_t && dist > kTol) {
        best_t = dist;
        best_slot = slot;
        bu = u;
        bv = v;
        improved = true;
    }
}

// Per-lane leaf scan over the SoA triangle streams, software-pipelined two deep with two
// register sets used alternately (no copies, so the loads of the next triangle stay in
// flight while the current one is tested). The hit keeps the primitive SLOT; its face index
// is read once, after the tree query.
template <bool COUNT>
__device__ __forceinline__ bool scan_leaf_lane(const Ray& r, const DModel& m, uint32_t first,
                                               uint32_t count, float& best_t, uint32_t& best_slot,
                                               float& bu, float& bv, Ctr& ct) {
    if constexpr (COUNT) { ct.tri += count; ct.leaf += 1; }
    bool improved = false;
    if (count == 0) return false;
    const uint32_t end = first + count;
    TriRegs A, B;
    tri_fetch(m, first, A);
    for (uint32_t k = first; k < end; k += 2) {
        const bool has_b = k + 1 < end;
        if (has_b) tri_fetch(m, k + 1, B);
        tri_test(r, A, k, best_t, best_slot, bu, bv, improved);
        if (k + 2 < end) tri_fetch(m, k + 2, A);
        if (has_b) tri_test(r, B, k + 1, best_t, best_slot, bu, bv, improved);
    }
    return improved;
}

// ------------------------------------------------------------------ clustered leaf scan
// One leaf over its clusters (cluster.h), the next cluster's record in flight while the current
// one is screened.
template <bool COUNT>
__device__ __forceinline__ bool scan_leaf_clusters(const Ray& r, const DModel& m, uint32_t cfirst,
                                                   uint32_t ccount, float& best_t, uint32_t& best_slot,
                                                   float& bu, float& bv, Ctr& ct) {
    if constexpr (COUNT) { ct.leaf += 1; ct.cbox += ccount; }
    LeafHit h;
    h.t = best_t;
    h.slot = best_slot;
    h.u = bu;
    h.v = bv;
    h.rank = -1;
    h.improved = false;
    cluster_range<COUNT>(r, m, cfirst, cfirst + ccount, h, ct);
    best_t = h.t;
    best_slot = h.slot;
    bu = h.u;
    bv = h.v;
    return h.improved;
}

template <bool COUNT, bool CL = false, int K = kLeafBuf>
__device__ __forceinline__ void tree_closest_lane(const Ray& r, const DModel& m, const float4_t* __restrict__ tab, Hit& h,
                                                  int& err, Ctr& ct) {
    h.t = kMaxFloat;
    h.face = 0;
    h.u = h.v = 0.f;
    const NodeBox root = load_node(m.nodes, 0);
    if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
    if (!box_check(r, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) return;  // :339
    uint32_t slot = 0xFFFFFFFFu;
    const uint32_t* range = CL ? m.cl_range : m.leaf_range;
    auto scan = [&](int32_t leaf) -> bool {
        if constexpr (CL) {
            const uint2_t cr = load_range(range, leaf);
            return scan_leaf_clusters<COUNT>(r, m, cr.x, cr.y, h.t, slot, h.u, h.v, ct);
        }
        else
            return scan_leaf_lane<COUNT>(r, m, range[2 * leaf], range[2 * leaf + 1], h.t, slot, h.u, h.v, ct);
    };
    if (root.children == 0) {  // :344-361
        scan(0);
    } else {
        float bd = -__builtin_inff();
        int32_t bi = -1;
        bool more = true;
        // The leaf order buffer lives in LDS (a lane-private column, 64 B per lane, 16 KB per
        // 4-wave workgroup, trace.h LdsLeafBuf): the pass inserts into it and the scan reads it,
        // so neither carries its 16 registers (94 VGPRs, no scratch at 5 waves/SIMD; the
        // register buffer copied to LDS after the pass measured 3% slower).
        __shared__ float s_lbd[4][K][64];
        __shared__ int32_t s_lbl[4][K][64];
        const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
        while (more) {
            int32_t n;
            {
                LdsLeafBuf<K> lb;
                lb.d = &s_lbd[w][0][ln];
                lb.leaf = &s_lbl[w][0][ln];
                n = traverse_pass<K, COUNT>(r, tab, lb, bd, bi, ct);
            }
            if (n < 0) { err = 1; break; }
            const int32_t nb = n < K ? n : K;
            more = n > K;
            bool hit = false;
            for (int32_t j = 0; j < nb; ++j) {
                const int32_t leaf = s_lbl[w][j][ln];
                bd = s_lbd[w][j][ln];
                bi = leaf;
                if (scan(leaf)) { hit = true; break; }
            }
            if (hit) break;
        }
    }
    if (slot != 0xFFFFFFFFu) h.face = CL ? m.cface[slot] : m.tface[slot];
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

template <bool COUNT>
__device__ __forceinline__ int32_t tq_next_leaf(TreeQuery& q, const Ray& r, const DModel& m, int& err, Ctr& ct) {
    for (;;) {
        if (q.state == 2) return -1;
        if (q.state == 0) {
            q.ncand = traverse_pass<kLeafBuf, COUNT>(r, m.inner, q.lb, q.bd, q.bi, ct);
            if (q.ncand < 0) { err = 1; q.state = 2; return -1; }
            q.pos = 0;
            q.state = 1;
        }
        const int32_t nb = q.ncand < kLeafBuf ? q.ncand : kLeafBuf;
        if (q.pos < nb) return lb_leaf<kLeafBuf>(q.lb, q.pos);
        if (q.ncand <= kLeafBuf) { q.state = 2; return -1; }
        q.bd = q.lb.d[kLeafBuf - 1];
        q.bi = q.lb.leaf[kLeafBuf - 1];
        q.state = 0;
    }
}

// Scan a wave-uniform leaf: every operand address is uniform, so the triangle records are
// fetched by the scalar unit once per wavefront instead of once per lane.
template <bool COUNT>
__device__ __forceinline__ bool scan_leaf_uniform(const Ray& r, const DTri* __restrict__ tris,
                                                  uint32_t first, uint32_t count, Hit& h, Ctr& ct) {
    bool improved = false;
    if constexpr (COUNT) { ct.tri += count; ct.leaf += 1; }
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

template <bool COUNT>
__device__ __forceinline__ void tree_closest_wave(const Ray& r, const DModel& m, bool active, Hit& h,
                                                  int& err, Ctr& ct) {
    h.t = kMaxFloat;
    h.face = 0;
    h.u = h.v = 0.f;
    TreeQuery q;
    q.state = 2;
    int32_t root_leaf_scan = 0;
    if (active) {
        const NodeBox root = load_node(m.nodes, 0);
        if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
        if (box_check(r, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) {
            if (root.children == 0) root_leaf_scan = 1;
            else { q.bd = -__builtin_inff(); q.bi = -1; q.state = 0; }
        }
    }
    int32_t leaf = -1;
    if (q.state != 2) leaf = tq_next_leaf<COUNT>(q, r, m, err, ct);
    if (root_leaf_scan) leaf = 0;
    for (;;) {
        const uint64_t want = __ballot(leaf >= 0);
        if (want == 0) break;
        const int src = __builtin_ctzll(want);
        const int32_t L = __builtin_amdgcn_readlane(leaf, src);  // uniform
        if constexpr (COUNT) { if ((threadIdx.x & 63) == 0) ct.wave_tri += m.leaf_range[2 * L + 1]; }
        if (leaf == L) {
            const uint32_t first = m.leaf_range[2 * L], count = m.leaf_range[2 * L + 1];
            const bool hit = scan_leaf_uniform<COUNT>(r, m.tris, __builtin_amdgcn_readfirstlane(first),
                                                      __builtin_amdgcn_readfirstlane(count), h, ct);
            if (root_leaf_scan || hit) { q.state = 2; leaf = -1; }
            else { ++q.pos; leaf = tq_next_leaf<COUNT>(q, r, m, err, ct); }
        }
    }
}

// ------------------------------------------------------------------ FLAT schedule
// The clustered scan with the wavefront's (ray, cluster) work flattened over its lanes
// (DESIGN.md §4e). In the lane-private scan (CLUSTER) every loop level diverges -- rays visit
// different numbers of leaves, their current leaves hold 1-20 clusters, the clusters pass the
// padded box or not -- and the wavefront executes the union: a slow 8x8 cell issued ~150 k VALU
// instructions where its rays' own work is ~7x less. Here each lane still owns a ray's query
// (traversal passes, its sorted leaves, the first-improving-leaf rule), but the clusters of all
// rays' current leaves are dealt to the 64 lanes in rounds: a round's 64 lanes each take one
// (ray, cluster) item and run the same cluster test on the owner's ray (read from the owner lane
// with a lane shuffle). Results merge per owner in LDS as the minimum (t, leaf rank) -- the
// first primitive in leaf order with the smallest t (kd_tree.cpp:440-456) -- so every output is
// CLUSTER's, bit for bit.
__device__ __forceinline__ float shfl_f(float v, int src) { return __shfl(v, src); }

// Wave-wide inclusive scans on the DPP row network (GFX9 rows of 16 lanes: shifts by 1, 2, 4, 8
// within a row, then the broadcasts of lanes 15 and 31 into the rows above): six dependent VALU
// steps, where a __shfl_up step is an LDS permute (ds_bpermute) round trip. Lanes shifted in
// from outside a row, and rows outside the mask, contribute the identity (`old`).
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xf, 0xf, false));  // row_shr:1
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xf, 0xf, false));  // row_shr:2
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xf, 0xf, false));  // row_shr:4
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xf, 0xf, false));  // row_shr:8
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xa, 0xf, false));  // row_bcast:15
    x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x143, 0xc, 0xf, false));  // row_bcast:31
    return x;
}
__device__ __forceinline__ int32_t wave_incl_max(int32_t x) {
    constexpr int32_t lo = -2147483647 - 1;
    x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x118, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x142, 0xa, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(lo, x, 0x143, 0xc, 0xf, false));
    return x;
}

// Phase clocks of the FLAT/HYBRID scans (atr_render_phase_clocks): compiled only into a diagnostic
// build (make EXTRA=-DATR_PHASE_CLOCKS). In the product build the statements vanish; even
// discarded under `if constexpr` they changed the product kernel's register allocation (3 spilled
// VGPRs).
#ifdef ATR_PHASE_CLOCKS
#define ATR_PCLK(...) __VA_ARGS__
#else
#define ATR_PCLK(...)
#endif

// LDS of the FLAT/HYBRID scans (22.5 KB per 4-wave workgroup): the leaf order buffers (lane-private
// columns), the per-owner best keys and hit records, the round's owner markers.
struct FlatLds {
    float lbd[4][kLeafBuf][64];
    int32_t lbl[4][kLeafBuf][64];
    unsigned long long key[4][64];
    uint32_t slot[4][64];
    float u[4][64], v[4][64];
    int32_t mark[4][64];
};
__device__ __forceinline__ FlatLds& flat_lds() {
    __shared__ FlatLds L;
    return L;
}

// Full tests of a round's candidates, compacted over the wavefront (CC). Each lane holds one
// (ray, cluster) item that passed the padded boxes and the screen with candidate mask `cm`
// (slots cfirst + bit, ray of lane `own`); the wave's candidates are numbered by a prefix sum of
// the masks' popcounts and dealt 64 per sub-round, one full test per lane: a cluster's
// candidates no longer run one after another in one lane (the serial chain of dependent loads
// that set the slow cells' time) while the other lanes wait. Each test lowers its owner's
// (t bits, leaf rank) key in LDS -- the minimum over the leaf in any order is the reference's
// first-in-leaf-order closest hit (kd_tree.cpp:440-456) -- and the winning test writes the slot
// and barycentrics.
template <bool COUNT, bool UO, bool NUV>
__device__ __forceinline__ void cand_rounds(const Ray& r, const DModel& m, int w, int ln, uint32_t cm,
                                            uint32_t cfirst, int32_t own, Ctr& ct, int32_t vr = 0, bool spec = false);

// HYB (the HYBRID schedule): each step the wavefront decides, uniformly, how to scan its rays'
// current leaves: lane-private (every lane scans its own leaf's clusters, as CLUSTER does: no
// per-round overhead, best when the rays' cluster counts are alike) or dealt in rounds (FLAT:
// best when one ray's leaf holds many more clusters than the rest, e.g. the few grazing rays
// left in a slow cell). It deals when the largest count exceeds a x rounds + b (RenderParams
// hyb_a / hyb_b). A leaf's result does not depend on how its clusters were visited (minimum
// (t, leaf rank)), so the choice changes no output bit. LDSB: the DFS pass inserts straight
// into the LDS columns (CLUSTER's LdsLeafBuf) instead of a register buffer copied after it.
// own: the candidates' owner slot (its key in LDS); with speculative leaf steps (spec) a slot is a
// (ray, leaf) pair and vr the ray lane of this lane's slot, so the ray comes from lane vr[own].
template <bool COUNT, bool UO, bool NUV>
__device__ __forceinline__ void cand_rounds(const Ray& r, const DModel& m, int w, int ln, uint32_t cm,
                                            uint32_t cfirst, int32_t own, Ctr& ct, int32_t vr, bool spec) {
    constexpr unsigned long long kInit = (static_cast<unsigned long long>(0x7F7FFFFFu) << 32) | 0xFFFFFFFFull;
    FlatLds& L = flat_lds();
    const uint32_t cc = uint32_t(__popc(cm));
    const uint32_t cinc = wave_incl_add(cc);
    const uint32_t total = uint32_t(__builtin_amdgcn_readlane(int(cinc), 63));
    const uint32_t cex = cinc - cc;
    int32_t carry = -1;
    for (uint32_t cb = 0; cb < total; cb += 64) {  // wave-uniform
        L.mark[w][ln] = -1;
        __builtin_amdgcn_wave_barrier();
        if (cc > 0 && cex >= cb && cex < cb + 64u) L.mark[w][cex - cb] = ln;
        __builtin_amdgcn_wave_barrier();
        int32_t src = wave_incl_max(L.mark[w][ln]);  // the lane whose candidates hold number cb + ln
        if (src < 0) src = carry;
        carry = __builtin_amdgcn_readlane(src, 63);
        const uint32_t k = cb + uint32_t(ln);
        const bool valid = k < total;
        const int32_t s2 = valid ? src : ln;
        uint32_t j = k - uint32_t(__shfl(int(cex), s2));
        uint32_t x = uint32_t(__shfl(int(cm), s2));
        uint32_t b = 0, n;  // position of the j-th set bit of the 16-bit mask x
        n = uint32_t(__popc(x & 0xFFu)); if (j >= n) { j -= n; x >>= 8; b += 8; }
        n = uint32_t(__popc(x & 0xFu)); if (j >= n) { j -= n; x >>= 4; b += 4; }
        n = uint32_t(__popc(x & 0x3u)); if (j >= n) { j -= n; x >>= 2; b += 2; }
        b += j >= (x & 1u) ? 1u : 0u;
        const uint32_t slot = uint32_t(__shfl(int(cfirst), s2)) + b;
        const int32_t ow = __shfl(own, s2);
        const int32_t rw = spec ? __shfl(vr, ow) : ow;  // the lane holding the owner's ray
        Ray q;
        q.o = UO ? r.o : mk(shfl_f(r.o.x, rw), shfl_f(r.o.y, rw), shfl_f(r.o.z, rw));
        q.d = mk(shfl_f(r.d.x, rw), shfl_f(r.d.y, rw), shfl_f(r.d.z, rw));
        unsigned long long mine = kInit;
        bool imp = false;
        float u = 0.f, v = 0.f;
        if (valid) {
            if constexpr (COUNT) { ct.tri += 1; ct.cand_wave += ln == 0 ? 1u : 0u; }
            float4_t a0, a1;
            c2_t a2;
            load_prim(m, slot, a0, a1, a2);
            const float dist = tri_hit(q, mk(a0.x, a0.y, a0.z), mk(a0.w, a1.x, a1.y), mk(a1.z, a1.w, a2.x), u, v);
            if (dist > kTol && dist < kMaxFloat) {  // accepted (model.h:75-103; kd_tree.cpp:450)
                mine = (static_cast<unsigned long long>(__float_as_uint(dist)) << 32) | uint32_t(__float_as_int(a2.y));
                if (mine < L.key[w][ow]) {
                    atomicMin(&L.key[w][ow], mine);
                    imp = true;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (imp && L.key[w][ow] == mine) {  // this sub-round's winner for its owner
            L.slot[w][ow] = slot;
            if constexpr (!NUV) {
                L.u[w][ow] = u;
                L.v[w][ow] = v;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// Speculative leaf steps (SPEC; experiment build -DATR_SPEC, not kept: DESIGN.md §4g measured it
// 4% slower on c3 and c4 with no latency gain): when at most 64 / kSpecLeaves rays of the wave are
// still scanning (the tail of a slow cell: a few grazing rays walking many leaves one dependent
// step at a time), each takes its next kSpecLeaves leaves in one step, one (ray, leaf) slot per
// lane. Every leaf is scanned from a fresh best, exactly as alone, and the ray takes the first of
// them (buffer order) that improved its hit (kd_tree.cpp:457-460), so the result is the
// sequential one; the leaves after it were speculative work on lanes that would have idled.
constexpr int kSpecLeaves = 4;
#ifdef ATR_SPEC
constexpr bool kSpecOn = true;
#else
constexpr bool kSpecOn = false;
#endif

template <bool COUNT, bool HYB = false, bool LDSB = false, bool PAIR = true, bool UO = false, bool UT = false,
          bool NUV = false, bool CC = false, bool SPEC = false>
__device__ __forceinline__ void tree_closest_flat(const Ray& r, const DModel& m, bool active, Hit& h, int& err,
                                                  Ctr& ct, int32_t hyb_a = 0, int32_t hyb_b = 0) {
    constexpr int K = kLeafBuf;
    constexpr unsigned long long kInit = (static_cast<unsigned long long>(0x7F7FFFFFu) << 32) | 0xFFFFFFFFull;
    FlatLds& L = flat_lds();  // one instance per kernel, shared by every flavour of this scan
    auto& s_lbd = L.lbd;
    auto& s_lbl = L.lbl;
    auto& s_key = L.key;
    auto& s_slot = L.slot;
    auto& s_u = L.u;
    auto& s_v = L.v;
    auto& s_mark = L.mark;
    const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
    ATR_PCLK(uint64_t tcs = clock64());
    h.t = kMaxFloat;
    h.face = 0;
    h.u = h.v = 0.f;
    bool done = true, need = false, more = false;
    int32_t j = 0, nb = 0, bi = -1;
    float bd = -__builtin_inff();
    if (active) {
        const NodeBox root = load_node(m.nodes, 0);
        if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
        if (box_check(r, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) {  // kd_tree.cpp:339
            done = false;
            if (root.children == 0) {  // :344-361: the root leaf (discovery rank 0) alone
                s_lbl[w][0][ln] = 0;
                s_lbd[w][0][ln] = 0.f;
                nb = 1;
            } else {
                need = true;
            }
        }
    }
    uint32_t res_slot = 0xFFFFFFFFu;
    float res_t = kMaxFloat, res_u = 0.f, res_v = 0.f;
#ifdef ATR_PRIO_STEPS
    int32_t nsteps = 0;  // experiment: a wave still stepping after ATR_PRIO_STEPS steps issues first
#endif
    for (;;) {
#ifdef ATR_PRIO_STEPS
        if (++nsteps == ATR_PRIO_STEPS) __builtin_amdgcn_s_setprio(2);
#endif
        ATR_PCLK(const uint64_t tc0 = clock64());
        if constexpr (UT) {  // the wave walks its passes together (traverse_pass_wave)
            if (__ballot(need)) {
                LdsLeafBuf<K> lb;
                lb.d = &s_lbd[w][0][ln];
                lb.leaf = &s_lbl[w][0][ln];
                const int32_t n = traverse_pass_wave<K, COUNT>(r, m.inner, lb, bd, bi, ct, need);
                if (need) {
                    need = false;
                    j = 0;
                    if (n < 0) { err = 1; done = true; }
                    else { nb = n < K ? n : K; more = n > K; if (nb == 0) done = true; }
                }
            }
        } else if (need) {  // one DFS pass (kd_tree.cpp:363-435); its sorted leaves wait in LDS
            int32_t n;
            if constexpr (LDSB) {
                LdsLeafBuf<K> lb;
                lb.d = &s_lbd[w][0][ln];
                lb.leaf = &s_lbl[w][0][ln];
                n = traverse_pass<K, COUNT>(r, m.inner, lb, bd, bi, ct);
            } else {  // register buffer here: the LDS one (LdsLeafBuf) measured 5% slower in FLAT at C4
                LeafBuf<K> lb;
                n = traverse_pass<K, COUNT>(r, m.inner, lb, bd, bi, ct);
#pragma unroll
                for (int q = 0; q < K; ++q) { s_lbd[w][q][ln] = lb.d[q]; s_lbl[w][q][ln] = lb.leaf[q]; }
            }
            need = false;
            j = 0;
            if (n < 0) { err = 1; done = true; }
            else { nb = n < K ? n : K; more = n > K; if (nb == 0) done = true; }
        }
        ATR_PCLK(const uint64_t tc2 = clock64());
        ATR_PCLK(ct.t_pass += uint32_t(tc2 - tc0));
        const uint64_t livem = __ballot(!done);
        if (livem == 0) break;
        // every live ray's current leaf: its clusters are this step's items
        int32_t leaf = -1;
        uint32_t cf = 0, cn = 0;
        bool spec = false;  // wave-uniform
        int32_t vr = ln;    // the ray lane of this lane's (ray, leaf) slot
        if constexpr (SPEC) spec = __popcll(livem) <= uint32_t(64 / kSpecLeaves);
        if (spec) {
            // slot q * kSpecLeaves + k: the q-th live ray's k-th next leaf
            if (!done) s_mark[w][__popcll(livem & ((uint64_t(1) << ln) - 1))] = ln;
            __builtin_amdgcn_wave_barrier();
            const int32_t qv = ln / kSpecLeaves, kv = ln % kSpecLeaves;
            vr = qv < int32_t(__popcll(livem)) ? s_mark[w][qv] : -1;
            __builtin_amdgcn_wave_barrier();
            const int32_t rs = vr >= 0 ? vr : ln;
            const int32_t jr = __shfl(j, rs) + kv, nbr = __shfl(nb, rs);
            if (vr >= 0 && jr < nbr) {
                leaf = s_lbl[w][jr][vr];
                const uint2_t cr = load_range(m.cl_range, leaf);
                cf = cr.x;
                cn = cr.y;
            }
            if (vr < 0) vr = ln;
        } else if (!done) {
            leaf = s_lbl[w][j][ln];
            const uint2_t cr = load_range(m.cl_range, leaf);
            cf = cr.x;
            cn = cr.y;
            if constexpr (COUNT) { ct.leaf += 1; ct.cbox += cn; }
        }
        const uint32_t incl = wave_incl_add(cn);  // inclusive prefix sum over the lanes
        const uint32_t excl = incl - cn;
        const uint32_t total = uint32_t(__builtin_amdgcn_readlane(int(incl), 63));
        s_key[w][ln] = kInit;
        bool deal = true;
        if constexpr (HYB) if (!spec) {
            // the largest cluster count of the step (counts are small: the signed max is exact)
            const uint32_t mx = uint32_t(__builtin_amdgcn_readlane(wave_incl_max(int32_t(cn)), 63));
            deal = int32_t(mx) > hyb_a * int32_t((total + 63u) >> 6) + hyb_b;
        }
        bool lp_imp = false;  // lane-private scan: this lane's leaf improved its hit
        ATR_PCLK(const uint64_t tc1 = clock64());
        ATR_PCLK(ct.t_prep += uint32_t(tc1 - tc2));
        if (!deal && CC) {  // every lane scans its own leaf's clusters, one per iteration; the
                            // candidates of each iteration are compacted over the wave
            const uint32_t mxc = uint32_t(__builtin_amdgcn_readlane(wave_incl_max(int32_t(cn)), 63));
            for (uint32_t i = 0; i < mxc; ++i) {
                uint32_t cm = 0;
                if (i < cn) {
                    const uint32_t c = cf + i;
                    const float bound = __uint_as_float(uint32_t(s_key[w][ln] >> 32));
                    cm = cluster_cands<COUNT>(r, m, c, m.clus[kClusterBlock * size_t(c)],
                                              m.clus[kClusterBlock * size_t(c) + 1], bound, ct);
                }
                cand_rounds<COUNT, UO, NUV>(r, m, w, ln, cm, kMaxClusterSize * (cf + i), ln, ct);
            }
        } else if (!deal) {
            if (cn > 0) {
                LeafHit lh;
                lh.t = kMaxFloat;
                lh.slot = 0xFFFFFFFFu;
                lh.u = lh.v = 0.f;
                lh.rank = -1;
                lh.improved = false;
                for (uint32_t c = cf; c < cf + cn; ++c)
                    cluster_step<COUNT>(r, m, c, m.clus[kClusterBlock * size_t(c)], m.clus[kClusterBlock * size_t(c) + 1], lh, ct);
                if (lh.improved) {
                    lp_imp = true;
                    res_t = lh.t;
                    res_slot = lh.slot;
                    if constexpr (!NUV) { res_u = lh.u; res_v = lh.v; }
                }
            }
        }
        ATR_PCLK(if (!deal) ct.t_lp += uint32_t(clock64() - tc1));
        int32_t carry = -1;
        for (uint32_t base = 0; deal && base < total; base += 64) {  // rounds of 64 items, wave-uniform
            s_mark[w][ln] = -1;
            __builtin_amdgcn_wave_barrier();
            if (cn > 0 && excl >= base && excl < base + 64u) s_mark[w][excl - base] = ln;
            __builtin_amdgcn_wave_barrier();
            int32_t own = wave_incl_max(s_mark[w][ln]);  // latest owner starting at or before this lane
            if (own < 0) own = carry;
            carry = __builtin_amdgcn_readlane(own, 63);
            const uint32_t k = base + uint32_t(ln);
            const bool valid = k < total;
            if constexpr (COUNT) { ct.round_wave += ln == 0 ? 1u : 0u; ct.round_items += valid ? 1u : 0u; }
            const int32_t src = valid ? own : ln;
            const int32_t rsrc = spec ? __shfl(vr, src) : src;  // the lane holding the owner's ray
            Ray q;  // the owner's ray
            // UO: every ray of the wave starts at the same point (primary rays: the frame's eye)
            q.o = UO ? r.o : mk(shfl_f(r.o.x, rsrc), shfl_f(r.o.y, rsrc), shfl_f(r.o.z, rsrc));
            q.d = mk(shfl_f(r.d.x, rsrc), shfl_f(r.d.y, rsrc), shfl_f(r.d.z, rsrc));
            q.inv = mk(shfl_f(r.inv.x, rsrc), shfl_f(r.inv.y, rsrc), shfl_f(r.inv.z, rsrc));
            q.s0 = q.inv.x < 0;
            q.s1 = q.inv.y < 0;
            q.s2 = q.inv.z < 0;
            const uint32_t c = uint32_t(__shfl(int(cf), src)) + (k - uint32_t(__shfl(int(excl), src)));
            if constexpr (CC) {
                uint32_t cm = 0;
                if (valid) {
                    const float bound = __uint_as_float(uint32_t(s_key[w][own] >> 32));
                    cm = cluster_cands<COUNT>(q, m, c, m.clus[kClusterBlock * size_t(c)],
                                              m.clus[kClusterBlock * size_t(c) + 1], bound, ct);
                }
                cand_rounds<COUNT, UO, NUV>(r, m, w, ln, cm, kMaxClusterSize * c, own, ct, vr, spec);
                continue;
            }
            unsigned long long mine = kInit;
            LeafHit lh;
            lh.improved = false;
            if (valid) {
                const unsigned long long cur = s_key[w][own];
                // the owner's best in this leaf so far: pruning bound, and equal t then loses only
                // to a smaller leaf rank (a fresh leaf starts from MAX_FLOAT, strict <)
                lh.t = __uint_as_float(uint32_t(cur >> 32));
                lh.rank = cur == kInit ? -1 : int32_t(uint32_t(cur));
                lh.slot = 0xFFFFFFFFu;
                lh.u = lh.v = 0.f;
                const float4_t lo = m.clus[kClusterBlock * size_t(c)], hi = m.clus[kClusterBlock * size_t(c) + 1];
                cluster_step<COUNT, PAIR>(q, m, c, lo, hi, lh, ct);
                if (lh.improved) {
                    mine = (static_cast<unsigned long long>(__float_as_uint(lh.t)) << 32) | uint32_t(lh.rank);
                    atomicMin(&s_key[w][own], mine);
                }
            }
            __builtin_amdgcn_wave_barrier();
            if (lh.improved && s_key[w][own] == mine) {  // the round's winner for this owner
                s_slot[w][own] = lh.slot;
                if constexpr (!NUV) {  // NUV: primary-only frames, u and v feed no output
                    s_u[w][own] = lh.u;
                    s_v[w][own] = lh.v;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        ATR_PCLK(if (deal) ct.t_deal += uint32_t(clock64() - tc1));
        if (spec) {
            if (!done) {  // the first of this ray's slots (buffer order) whose leaf improved the hit
                const int32_t q0 = int32_t(__popcll(livem & ((uint64_t(1) << ln) - 1))) * kSpecLeaves;
                bool imp = false;
                for (int32_t kk = 0; kk < kSpecLeaves && j + kk < nb; ++kk) {
                    const unsigned long long key = s_key[w][q0 + kk];
                    if (key != kInit) {
                        imp = true;
                        res_t = __uint_as_float(uint32_t(key >> 32));
                        res_slot = s_slot[w][q0 + kk];
                        if constexpr (!NUV) {
                            res_u = s_u[w][q0 + kk];
                            res_v = s_v[w][q0 + kk];
                        }
                        break;
                    }
                }
                if (imp) {
                    done = true;
                } else {  // none did: the re-walk bound is the last leaf scanned
                    const int32_t last = (j + kSpecLeaves < nb ? j + kSpecLeaves : nb) - 1;
                    bd = s_lbd[w][last][ln];
                    bi = s_lbl[w][last][ln];
                    j = last + 1;
                    if (j >= nb) {
                        if (more) need = true;
                        else done = true;
                    }
                }
            }
        } else if (!done) {  // stop at the first leaf that improved the hit (kd_tree.cpp:457-460)
            bool imp = lp_imp;
            if (deal || CC) {
                const unsigned long long key = s_key[w][ln];
                imp = key != kInit;
                if (imp) {
                    res_t = __uint_as_float(uint32_t(key >> 32));
                    res_slot = s_slot[w][ln];
                    if constexpr (!NUV) {
                        res_u = s_u[w][ln];
                        res_v = s_v[w][ln];
                    }
                }
            }
            if (imp) {
                done = true;
            } else {
                bd = s_lbd[w][j][ln];
                bi = leaf;
                if (++j >= nb) {
                    if (more) need = true;
                    else done = true;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (res_slot != 0xFFFFFFFFu) {
        h.t = res_t;
        h.u = res_u;
        h.v = res_v;
        h.face = m.cface[res_slot];
    }
    ATR_PCLK(ct.t_scan += uint32_t(clock64() - tcs));
}

// ------------------------------------------------------------------ TILE schedule
// The NW waves of a workgroup (NW 8x8 cells) cooperate on leaf scans. Each round elects ONE
// leaf that some ray of the workgroup wants next (at any position of its own sorted list),
// compacts the rays that want it (ballot + per-wave prefix in LDS), stages the leaf's
// triangles once in LDS (coalesced loads), and the waves process the compacted rays 64 per
// wave, each lane testing every triangle of the leaf read by LDS broadcast. Every ray still
// consumes its own leaves in its own sorted order and stops after the first leaf that
// improves its hit (kd_tree.cpp:437-462), so results are identical to LANE; what changes is
// that a leaf is fetched once per workgroup round instead of once per lane, and the triangle
// loop reads LDS (no global-memory latency inside it).
constexpr int kTileTris = 384;  // triangles staged per LDS chunk (Dragon's max leaf is 297)

template <int NW>
struct TileSmem {
    float4_t t0[kTileTris], t1[kTileTris];
    float t2[kTileTris];
    float ray[6][NW * 64];            // o.xyz, d.xyz per thread
    float rt[NW * 64], ru[NW * 64], rv[NW * 64];
    uint32_t rslot[NW * 64];
    int32_t list[NW * 64];
    int32_t cand[NW], cnt[NW];
};

template <int NW, bool COUNT>
__device__ __forceinline__ int32_t tile_next_leaf(TreeQuery& q, const Ray& r, const DModel& m, int& err,
                                                  Ctr& ct) {
    // pop the scanned head; refill with a re-walk after the bound when the buffer runs dry
    for (;;) {
        if (q.state == 2) return -1;
        if (q.state == 0) {
            q.ncand = traverse_pass<kLeafBuf, COUNT>(r, m.inner, q.lb, q.bd, q.bi, ct);
            if (q.ncand < 0) { err = 1; q.state = 2; return -1; }
            q.pos = q.ncand < kLeafBuf ? q.ncand : kLeafBuf;  // entries left in the buffer
            q.state = 1;
            if (q.pos > 0) return q.lb.leaf[0];
        }
        if (q.pos > 0) return q.lb.leaf[0];
        if (q.ncand <= kLeafBuf) { q.state = 2; return -1; }
        q.state = 0;
    }
}

template <int NW, bool COUNT>
__device__ __forceinline__ void tree_closest_tile(const Ray& r, const DModel& m, bool active, Hit& h,
                                                  int& err, Ctr& ct) {
    constexpr int NT = NW * 64;
    __shared__ TileSmem<NW> sm;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    h.t = kMaxFloat;
    h.face = 0;
    h.u = h.v = 0.f;
    TreeQuery q;
    q.state = 2;
    q.pos = 0;
    q.ncand = 0;
    bool root_scan = false;
    int32_t my_leaf = -1;
    uint32_t slot = 0xFFFFFFFFu;
    if (active) {
        const NodeBox root = load_node(m.nodes, 0);
        if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
        if (box_check(r, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) {  // :339
            if (root.children == 0) { root_scan = true; my_leaf = 0; }
            else {
                q.bd = -__builtin_inff();
                q.bi = -1;
                q.state = 0;
                my_leaf = tile_next_leaf<NW, COUNT>(q, r, m, err, ct);
            }
        }
    }
    sm.ray[0][tid] = r.o.x; sm.ray[1][tid] = r.o.y; sm.ray[2][tid] = r.o.z;
    sm.ray[3][tid] = r.d.x; sm.ray[4][tid] = r.d.y; sm.ray[5][tid] = r.d.z;
    for (;;) {
        const uint64_t want = __ballot(my_leaf >= 0);
        if (lane == 0) sm.cand[w] = want ? __builtin_amdgcn_readlane(my_leaf, __builtin_ctzll(want)) : 0x7FFFFFFF;
        __syncthreads();
        int32_t L = 0x7FFFFFFF;
#pragma unroll
        for (int i = 0; i < NW; ++i) L = sm.cand[i] < L ? sm.cand[i] : L;
        if (L == 0x7FFFFFFF) break;  // workgroup-uniform
        const bool mem = my_leaf == L;
        const uint64_t mb = __ballot(mem);
        if (lane == 0) sm.cnt[w] = __popcll(mb);
        const uint32_t first = m.leaf_range[2 * L], count = m.leaf_range[2 * L + 1];
        __syncthreads();
        int32_t base = 0, n = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) { base += i < w ? sm.cnt[i] : 0; n += sm.cnt[i]; }
        if (mem) sm.list[base + __popcll(mb & ((uint64_t(1) << lane) - 1))] = tid;
        if constexpr (COUNT) {
            if (tid == 0) ct.wave_tri += uint32_t((n + 63) / 64) * count;
        }
        for (uint32_t c0 = 0; c0 < count; c0 += kTileTris) {
            const uint32_t cc = count - c0 < uint32_t(kTileTris) ? count - c0 : uint32_t(kTileTris);
            for (uint32_t i = tid; i < cc; i += NT) {
                sm.t0[i] = m.t0[first + c0 + i];
                sm.t1[i] = m.t1[first + c0 + i];
                sm.t2[i] = m.t2[first + c0 + i];
            }
            __syncthreads();
            for (int ch = w; ch * 64 < n; ch += NW) {
                const int idx = ch * 64 + lane;
                if (idx < n) {
                    const int mt = sm.list[idx];
                    Ray rr;
                    rr.o = mk(sm.ray[0][mt], sm.ray[1][mt], sm.ray[2][mt]);
                    rr.d = mk(sm.ray[3][mt], sm.ray[4][mt], sm.ray[5][mt]);
                    float bt = kMaxFloat, bu = 0.f, bv = 0.f;
                    uint32_t bs = 0xFFFFFFFFu;
                    if (c0 > 0) { bt = sm.rt[mt]; bu = sm.ru[mt]; bv = sm.rv[mt]; bs = sm.rslot[mt]; }
                    for (uint32_t k = 0; k < cc; ++k) {
                        const float4_t a = sm.t0[k], b = sm.t1[k];
                        const float c = sm.t2[k];
                        float u = 0.f, v = 0.f;
                        const float dist = tri_hit(rr, mk(a.x, a.y, a.z), mk(a.w, b.x, b.y), mk(b.z, b.w, c), u, v);
                        if (dist < bt && dist > kTol) { bt = dist; bs = first + c0 + k; bu = u; bv = v; }
                    }
                    sm.rt[mt] = bt; sm.ru[mt] = bu; sm.rv[mt] = bv; sm.rslot[mt] = bs;
                }
            }
            __syncthreads();
        }
        if (mem) {
            if constexpr (COUNT) { ct.tri += count; ct.leaf += 1; }
            const bool improved = count > 0 && sm.rt[tid] < kMaxFloat;
            if (improved) {
                h.t = sm.rt[tid]; h.u = sm.ru[tid]; h.v = sm.rv[tid];
                slot = sm.rslot[tid];
                my_leaf = -1;
                q.state = 2;
            } else if (root_scan) {
                my_leaf = -1;
            } else {
                q.bd = q.lb.d[0];
                q.bi = q.lb.leaf[0];
                lb_pop<kLeafBuf>(q.lb);
                --q.pos;
                my_leaf = tile_next_leaf<NW, COUNT>(q, r, m, err, ct);
            }
        }
    }
    if (slot != 0xFFFFFFFFu) h.face = m.tface[slot];
}

// ------------------------------------------------------------------ get_intersection_data
enum { SCHED_LANE = 0, SCHED_WAVE = 1, SCHED_TILE4 = 2, SCHED_TILE8 = 3, SCHED_CLUSTER = 4, SCHED_CLUSTER_K4 = 5,
       SCHED_FLAT = 6, SCHED_HYBRID = 7, SCHED_FLAT_NOCC = 9, SCHED_HYBRID_NOCC = 10, SCHED_FLAT_UT = 11,
       SCHED_FLAT_REGEN = 12, SCHED_FLAT_ONE = 13 };
// The FLAT / HYBRID family (wave-wide leaf steps, LDS path stash). FLAT and HYBRID compact the full
// tests' candidates over the wavefront (cand_rounds); the _NOCC schedules are the round-2 kernels
// that test a cluster's candidates in its lane (diagnostic); FLAT_UT walks every
// bounce's DFS passes wave-wide (diagnostic).
constexpr bool sched_flat(int sc) {
    return sc == SCHED_FLAT || sc == SCHED_FLAT_NOCC || sc == SCHED_FLAT_UT || sc == SCHED_FLAT_REGEN ||
           sc == SCHED_FLAT_ONE;
}
constexpr bool sched_hyb(int sc) { return sc == SCHED_HYBRID || sc == SCHED_HYBRID_NOCC; }
constexpr bool sched_cc(int sc) { return sc != SCHED_FLAT_NOCC && sc != SCHED_HYBRID_NOCC; }
constexpr int sched_waves(int sc) { return sc == SCHED_TILE8 ? 8 : 4; }
constexpr bool sched_coop(int sc) {  // lanes must stay in lockstep loops (workgroup-wide)
    return sc != SCHED_LANE && sc != SCHED_CLUSTER && sc != SCHED_CLUSTER_K4 && !sched_flat(sc) && !sched_hyb(sc);
}

// A model's table pointers as wave-uniform GLOBAL pointers (uniform_global, trace.h): read once per
// query into SGPRs and cast to the global address space. Through the DScene reference the compiler
// re-loaded each pointer with a vector load before every use (a dependent round trip in front of
// every cluster record, candidate and leaf range) and, the pointers being generic, issued the
// table loads as flat loads.
__device__ __forceinline__ DModel uniform_model(const DModel& src) {
    DModel m = src;
    m.nodes = uniform_global(m.nodes);
    m.inner = uniform_global(m.inner);
    m.leaf_range = uniform_global(m.leaf_range);
    m.tris = uniform_global(m.tris);
    m.t0 = uniform_global(m.t0);
    m.t1 = uniform_global(m.t1);
    m.t2 = uniform_global(m.t2);
    m.tface = uniform_global(m.tface);
    m.clus = uniform_global(m.clus);
    m.cl_range = uniform_global(m.cl_range);
    m.cnrm = uniform_global(m.cnrm);
    m.c0 = uniform_global(m.c0);
    m.c1 = uniform_global(m.c1);
    m.c2 = uniform_global(m.c2);
    m.cface = uniform_global(m.cface);
    return m;
}

template <int SCHED, bool COUNT, bool PR = false>
__device__ __forceinline__ void intersect_scene(const DScene* __restrict__ S, V3 o, V3 d, bool active,
                                                Isect& id, int& err, Ctr& ct, int32_t hyb_a, int32_t hyb_b,
                                                bool first = false) {
    const Ray r = make_ray(o, d);  // renderer.cpp:41-44
    float best = kMaxFloat;
    int32_t nm = -1;
    uint32_t face = 0;
    float fu = 0.f, fv = 0.f;
    const int32_t nmodels = __builtin_amdgcn_readfirstlane(S->nmodels);  // uniform: an SGPR, not a VGPR
    for (int32_t i = 0; i < nmodels; ++i) {
        const DModel m = uniform_model(S->models[i]);
        if (m.has_tree) {  // USE_KD_TREE (:49-57)
            Hit h;
            if constexpr (SCHED == SCHED_WAVE) tree_closest_wave<COUNT>(r, m, active, h, err, ct);
            else if constexpr (sched_flat(SCHED)) {
                constexpr bool CC = sched_cc(SCHED);
                // the camera rays of a bounce loop (one origin, coherent) take HYBRID's primary flavour
                if (first && SCHED != SCHED_FLAT_ONE)  // FLAT_ONE (diagnostic): one flavour for every bounce
                    tree_closest_flat<COUNT, true, true, false, true, true, false, CC, CC && !COUNT && kSpecOn>(
                        r, m, active, h, err, ct, hyb_a, hyb_b);
                else if constexpr (SCHED == SCHED_FLAT || SCHED == SCHED_FLAT_REGEN || SCHED == SCHED_FLAT_ONE)  // LDS leaf buffer: fewer VGPRs, 5 waves/SIMD (§4d)
                    tree_closest_flat<COUNT, false, true, true, false, false, false, true, !COUNT && kSpecOn>(
                        r, m, active, h, err, ct);
                else if constexpr (SCHED == SCHED_FLAT_UT)
                    tree_closest_flat<COUNT, false, true, true, false, true, false, CC>(r, m, active, h, err, ct);
                else tree_closest_flat<COUNT, false, false, true, false, false, false, CC>(r, m, active, h, err, ct);
            }
            else if constexpr (sched_hyb(SCHED))
                // primary rays: LDS leaf buffer, one candidate test at a time (fewer VGPRs, as CLUSTER);
                // bounces: FLAT's register buffer and paired candidate loads (measured)
                tree_closest_flat<COUNT, true, PR, !PR, PR, PR, PR, sched_cc(SCHED),
                                  sched_cc(SCHED) && !COUNT && kSpecOn>(r, m, active, h, err, ct, hyb_a, hyb_b);
            else if constexpr (SCHED == SCHED_TILE4) tree_closest_tile<4, COUNT>(r, m, active, h, err, ct);
            else if constexpr (SCHED == SCHED_TILE8) tree_closest_tile<8, COUNT>(r, m, active, h, err, ct);
            else if constexpr (SCHED == SCHED_CLUSTER) {
                if (active) tree_closest_lane<COUNT, true>(r, m, m.inner, h, err, ct);
                else h.t = kMaxFloat;
            }
            else if constexpr (SCHED == SCHED_CLUSTER_K4) {  // 4-entry leaf buffer (fewer VGPRs)
                if (active) tree_closest_lane<COUNT, true, 4>(r, m, m.inner, h, err, ct);
                else h.t = kMaxFloat;
            }
            else if (active) tree_closest_lane<COUNT>(r, m, m.inner, h, err, ct);
            else h.t = kMaxFloat;
            if (h.t > kTol && h.t < best) { best = h.t; face = h.face; fu = h.u; fv = h.v; nm = i; }
        } else if (active) {  // brute force (:58-82), face-ordered triangles, uniform loads
            if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
            if (box_entry(r, m.aabb[0], m.aabb[1], m.aabb[2], m.aabb[3], m.aabb[4], m.aabb[5]) != 0) {
                if constexpr (COUNT) { ct.tri += m.nfaces; }
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
    scene_finish(S, o, d, best, face, fu, fv, nm, id);  // :86-160
}

// ------------------------------------------------------------------ cast_ray + pixel loop
// Path state parked in LDS while a ray is traced (the FLAT/HYBRID bounce kernels): the colour
// sums, throughput, PCG state and counters are dead during the tree query, so a lane-private LDS
// column holds them instead of registers the query needs (16 KB per 4-wave workgroup).
constexpr int kStash = 16;
// The stash lives in LDS (a lane-private column, stride 64 words) or, for FLAT, in the lane's
// private (scratch) memory: a volatile local array, which the compiler must keep in memory (stride
// 1), so the kernel's LDS is only the scan's 22.5 KB and more workgroups fit a CU.

template <int SCHED, bool COUNT>
__device__ __forceinline__ V3 cast_ray(const DScene* __restrict__ S, V3 o, V3 d, int32_t bounce_limit,
                                       bool active, uint64_t& st, uint64_t stream, uint32_t& casts,
                                       uint32_t& traced, bool record, uint32_t& hit_face, float& hit_t,
                                       int& err, Ctr& ct, int32_t hyb_a, int32_t hyb_b, V3& acc) {
    constexpr bool STASH = sched_flat(SCHED) || sched_hyb(SCHED);
    constexpr bool PRIV = SCHED == SCHED_FLAT || SCHED == SCHED_FLAT_ONE;  // the stash in private memory (above)
    __shared__ uint32_t s_stash[STASH && !PRIV ? 4 : 1][PRIV ? 1 : kStash][64];
    // the private stash is indexed directly (scratch loads and stores); through a generic pointer
    // every access was a flat load or store
    // (not volatile: volatile private accesses are left generic, i.e. flat loads and stores; the
    // array's address escapes into empty asm statements around the query instead, which keeps
    // its values in memory through the query)
    uint32_t pstash[PRIV ? kStash : 1];
    uint32_t* const L = &s_stash[STASH ? threadIdx.x >> 6 : 0][0][threadIdx.x & 63];
#define stash_put(k, v) do { if constexpr (PRIV) pstash[k] = (v); else L[64 * (k)] = (v); } while (0)
#define stash_get(k) (PRIV ? pstash[(PRIV ? (k) : 0)] : L[64 * (k)])
    V3 ret = mk(0.f, 0.f, 0.f), w = mk(1.f, 1.f, 1.f);
    int32_t i = 0;
    bool live = active;
    // WAVE: every lane stays in the loop until all lanes are done, so the wavefront can
    // cooperate on leaf scans inside intersect_scene.
    for (i = 0; ; ++i) {
        const bool go = live && i < bounce_limit;
        if constexpr (SCHED == SCHED_WAVE || sched_flat(SCHED) || sched_hyb(SCHED)) {
            if (__ballot(go) == 0) break;
        }
        else if constexpr (sched_coop(SCHED)) { if (!__syncthreads_or(go)) break; }
        else if (!go) break;
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
        intersect_scene<SCHED, COUNT>(S, o, d, go, id, err, ct, hyb_a, hyb_b, i == 0);
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

// FLAT_REGEN: the pixel loop of a multi-bounce render (renderer.cpp:336-357 around cast_ray
// :213-262) with path regeneration. In cast_ray's loop a lane whose path has ended (sky, or the
// bounce limit) idles until the wavefront's longest path of that sample is done; on Dragon C4 a
// path traces 1.5 rays on average and the wave's slowest lane up to 5. Here every lane runs its
// own (sample, bounce) sequence: a lane whose path ends adds the sample's colour and starts its
// next sample's camera ray in the same step, so each wave step traces a ray in every lane that
// still has samples left. A pixel's samples, its bounces and its PCG draws happen in the
// reference's order (AA jitter x then y at a sample's start, three rand_bi per non-sky hit), and
// the colour sums in sample order, so every output equals cast_ray's bit for bit. A step whose
// tracing lanes all hold camera rays (one origin: the first step, and whenever the lanes'
// samples line up) takes HYBRID's primary flavour; every other step FLAT's dealt rounds. The path
// state waits in private memory during the query, as in FLAT.
constexpr int kRegenStash = 20;
template <int SCHED, bool COUNT>
__device__ __forceinline__ V3 pixel_paths_regen(const DScene* __restrict__ S, uint32_t spp, int32_t bl, bool aa,
                                                float hpw, float hph, V3 eye, V3 fc, V3 cx, V3 cy, float film_x,
                                                float film_y, bool active, uint64_t& st, uint64_t stream,
                                                uint32_t& casts, uint32_t& traced, uint32_t& hit_face, float& hit_t,
                                                int& err, Ctr& ct, int32_t hyb_a, int32_t hyb_b) {
    // the camera's fields arrive by value (uniform: SGPRs); a reference into the kernel argument's
    // per-frame camera array made the compiler copy the whole argument to private memory
    volatile uint32_t L[kRegenStash];
    V3 col = mk(0.f, 0.f, 0.f), ret = mk(0.f, 0.f, 0.f), w = mk(1.f, 1.f, 1.f);
    uint32_t smp = 0;
    int32_t i = 0;
    bool have = active && spp > 0 && bl > 0;
    V3 o = eye, d = mk(0.f, 0.f, 1.f);
    // sample smp's camera ray (:338-351): jittered per sample with AA, else the pixel centre's
    auto camera_ray = [&]() {
        if (aa) {
            const float xo = rand_bi(st, stream) * hpw + film_x;
            const float yo = rand_bi(st, stream) * hph + film_y;
            d = unit(sub(add(add(fc, scale(cx, xo)), scale(cy, yo)), eye));
        } else {
            d = unit(sub(add(add(fc, scale(cx, film_x)), scale(cy, film_y)), eye));
        }
    };
    if (have) camera_ray();
    for (;;) {
        if (__ballot(have) == 0) break;
        // every tracing lane holds a camera ray: one origin (inactive lanes keep o = eye too)
        const bool first = __ballot(have && i != 0) == 0;
        if constexpr (COUNT) {
            const int bk = i < 2 ? i : 2;
            ct.steps[first ? 0 : 1] += (threadIdx.x & 63) == 0 ? 1u : 0u;
            ct.active[bk] += have ? 1u : 0u;
        }
        L[0] = __float_as_uint(ret.x); L[1] = __float_as_uint(ret.y); L[2] = __float_as_uint(ret.z);
        L[3] = __float_as_uint(w.x); L[4] = __float_as_uint(w.y); L[5] = __float_as_uint(w.z);
        L[6] = __float_as_uint(col.x); L[7] = __float_as_uint(col.y); L[8] = __float_as_uint(col.z);
        L[9] = uint32_t(st); L[10] = uint32_t(st >> 32);
        L[11] = casts; L[12] = traced; L[13] = hit_face; L[14] = __float_as_uint(hit_t);
        L[15] = smp; L[16] = uint32_t(i); L[17] = have ? 1u : 0u;
        L[18] = __float_as_uint(film_x); L[19] = __float_as_uint(film_y);
        Isect id;
        id.type = T_NONE;
        intersect_scene<SCHED, COUNT>(S, o, d, have, id, err, ct, hyb_a, hyb_b, first);
        auto gf = [&](int k) { return __uint_as_float(L[k]); };
        ret = mk(gf(0), gf(1), gf(2));
        w = mk(gf(3), gf(4), gf(5));
        col = mk(gf(6), gf(7), gf(8));
        st = uint64_t(L[9]) | (uint64_t(L[10]) << 32);
        casts = L[11]; traced = L[12]; hit_face = L[13]; hit_t = gf(14);
        smp = L[15]; i = int32_t(L[16]); have = L[17] != 0;
        film_x = gf(18); film_y = gf(19);
        if (!have) continue;
        ++traced;
        if (smp == 0 && i == 0) { hit_face = id.face; hit_t = id.t; }  // sample 0's camera ray
        const DMaterial& mat = S->mats[id.material];
        const V3 emission = mk(mat.ex, mat.ey, mat.ez);
        bool end;
        if (id.type == T_SKY) {  // :225-229
            ret = add(ret, had(w, emission));
            casts += uint32_t(i);
            end = true;
        } else {  // :231-258
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
            ++i;
            end = i >= bl;
            if (end) casts += uint32_t(bl);  // :260, the path ran to the bounce limit
        }
        if (end) {  // the sample's colour (:353-356), then the next sample's camera ray
            col = add(col, ret);
            ret = mk(0.f, 0.f, 0.f);
            w = mk(1.f, 1.f, 1.f);
            o = eye;
            i = 0;
            if (++smp < spp) camera_ray();
            else have = false;
        }
    }
    return col;
}

__device__ __forceinline__ int remap_xcd(int wg, int nwg, int chunk) {
    const int x = wg % 8;  // the hardware deals workgroups round-robin over the 8 XCDs
    if (chunk > 0) {
        // chunks of `chunk` consecutive workgroups dealt round-robin to the XCDs: neighbouring
        // cells still share an XCD (and its L2), every XCD gets chunks from the whole frame
        const int span = 8 * chunk, full = (nwg / span) * span;
        if (wg >= full) return wg;
        const int j = wg / 8;
        return ((j / chunk) * 8 + x) * chunk + j % chunk;
    }
    // consecutive work blocks -> same XCD (its L2 holds their shared leaves); bijective form
    const int q = nwg / 8, rm = nwg % 8;
    return (x < rm ? x * (q + 1) : rm * (q + 1) + (x - rm) * q) + wg / 8;
}

// PRIMARY: bounce_limit == 1 and no AA. Then cast_ray is one intersection whose color is the
// hit material's (or the sky's) emission; the three rand_bi draws and the bounce ray it builds
// feed only a second iteration that never runs (renderer.cpp:222-259), so they are skipped --
// output bit-identical, and far fewer live registers. Every sample re-traces the same primary
// ray in the reference (:353-356) and sums the same color, reproduced by the same f32 adds.
template <int SCHED, bool COUNT, bool PRIMARY, int OCC = 4>
__global__ __launch_bounds__(64 * sched_waves(SCHED), OCC) void render_kernel(RenderParams P) {
    constexpr int NW = sched_waves(SCHED);
    // the wave index is uniform: in an SGPR, so are the cell and frame indices derived from it
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6)), lane = threadIdx.x & 63;
    const int b = remap_xcd(blockIdx.x, gridDim.x, P.xcd_chunk) * NW + wave;
    if (SCHED != SCHED_TILE4 && SCHED != SCHED_TILE8 && b >= P.nblocks) return;  // whole wavefront
    const bool in_range = b < P.nblocks;
    // several frames per launch, interleaved: block b renders block b / nf of frame b % nf, so the
    // frames advance through the block list together (each frame's slow cells start early, and
    // neighbouring workgroups trace the same cells' rays)
    const int32_t nf = P.frame_blocks > 0 ? P.nblocks / P.frame_blocks : 1;
    const int32_t fidx = b % nf;
    // frame f's block list rotated by f / nf x frame_rotate / 1024 of the frame: the frames' slow
    // regions reach the dispatcher at different times instead of all together
    int32_t bi = b / nf;
    if (P.frame_rotate && nf > 1)
        bi = int32_t((int64_t(bi) + int64_t(P.frame_blocks) * fidx * P.frame_rotate / (1024 * int64_t(nf))) %
                     P.frame_blocks);
    DBlock blk;
    if (in_range) blk = P.blocks[bi];
    else { blk.x0 = 0; blk.y0 = 0; blk.mask_lo = 0; blk.mask_hi = 0; blk.out_base = 0; blk.flags = 0; blk.base = 0; blk.pad = 0; }
    const uint64_t mask = uint64_t(blk.mask_lo) | (uint64_t(blk.mask_hi) << 32);
    const bool active = (mask >> lane) & 1;
    const int32_t x = blk.x0 + (lane & 7), y = blk.y0 + (lane >> 3);
    if (__builtin_amdgcn_readfirstlane(blk.flags) & kBlockPrio) __builtin_amdgcn_s_setprio(2);  // cell plan
    const uint64_t clk0 = P.block_cost ? clock64() : 0;
    uint64_t clk1 = 0;
    if constexpr (COUNT) clk1 = clock64();
    const uint64_t rt0 = P.wave_trace ? __builtin_amdgcn_s_memrealtime() : 0;
    // per-frame cameras (atr_render_start_cameras): fidx is wave-uniform, so the camera comes from
    // the kernel argument with scalar loads
    const atr_camera& cm = P.nfcam > 0 ? P.fcam[__builtin_amdgcn_readfirstlane(fidx)] : P.cam;
    const DScene* S = uniform_global(P.scene);  // global loads for materials, spheres, planes, shading
    int err = 0;
    Ctr ct;
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
    if constexpr (PRIMARY) {
        Isect id;
        id.type = T_NONE;
        intersect_scene<SCHED, COUNT, true>(S, eye, dir, active, id, err, ct, P.hyb_a, P.hyb_b);
        if (active) {
            const DMaterial& mat = S->mats[id.material];
            const V3 ret = mk(mat.ex, mat.ey, mat.ez);  // weight (1,1,1) x emission
            hit_face = id.face;
            hit_t = id.t;
            const uint32_t hit = id.type == T_SKY ? 0u : 1u;
            for (uint32_t s = 0; s < cm.samples_per_pixel; ++s) {
                col = add(col, ret);
                casts += hit;
                ++traced;
            }
        }
    } else if constexpr (SCHED == SCHED_FLAT_REGEN) {
        col = pixel_paths_regen<SCHED, COUNT>(
            S, __builtin_amdgcn_readfirstlane(cm.samples_per_pixel), __builtin_amdgcn_readfirstlane(cm.bounce_limit),
            __builtin_amdgcn_readfirstlane(cm.anti_aliasing) != 0,
            __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, cm.half_pixel_width))),
            __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, cm.half_pixel_height))),
            eye, fc, cx, cy, film_x, film_y, active, st, stream, casts, traced, hit_face, hit_t, err, ct, P.hyb_a,
            P.hyb_b);
    } else
    for (uint32_t s = 0; s < cm.samples_per_pixel; ++s) {
        if (cm.anti_aliasing) {  // :338-343
            const float xo = rand_bi(st, stream) * cm.half_pixel_width + film_x;
            const float yo = rand_bi(st, stream) * cm.half_pixel_height + film_y;
            dir = unit(sub(add(add(fc, scale(cx, xo)), scale(cy, yo)), eye));
        }
        col = add(col, cast_ray<SCHED, COUNT>(S, eye, dir, cm.bounce_limit, active, st, stream, casts, traced,
                                             s == 0, hit_face, hit_t, err, ct, P.hyb_a, P.hyb_b, col));
    }
    // the output address from the cell record read again: the pixel coordinates and mask
    // then hold no registers through the trace (the asm clobber keeps the compiler from reusing
    // the first read)
    DBlock ob = blk;
    __asm__ volatile("" ::: "memory");
    if (in_range) ob = P.blocks[bi];
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
    if (P.traced_rays) {
        uint32_t t = traced;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
        // 64 counters on separate 128-B lines (atr_launch_traced_finish adds them up): one
        // address taking every wave's add serializes ~0.1 ms per frame at the L2
        if (lane == 0 && t) atomicAdd(P.traced_rays + 16 * (b & 63), (unsigned long long)t);
    }
    if (err && P.error_flag) atomicOr(P.error_flag, 1);
    // per-cell cost (calibration, the single-frame plan): a split cell's waves add up
    if (P.block_cost && lane == 0 && in_range && omask) atomicAdd(P.block_cost + ob.base, (unsigned long long)(clock64() - clk0));
    if (P.wave_trace && lane == 0 && in_range) {  // diagnostic: where and when this wave ran
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        P.wave_trace[3 * size_t(b)] = rt0;
        P.wave_trace[3 * size_t(b) + 1] = __builtin_amdgcn_s_memrealtime();
        P.wave_trace[3 * size_t(b) + 2] = uint64_t(hw) | (uint64_t(xcc) << 32);
    }
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
        if (lane == 0) { atomicAdd(C + 0, (unsigned long long)t); if (in_range) atomicAdd(C + 7, 1ull); }
        uint32_t w[2] = {ct.cbox, ct.screen};
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            uint32_t x = w[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
            if (lane == 0 && x) atomicAdd(C + 8 + k, (unsigned long long)x);
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
                uint32_t x = e[k];
#pragma unroll
                for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
                if (lane == 0 && x) atomicAdd(C + 22 + k, (unsigned long long)x);
            }
        }
        // counters[10..15]: wave clocks in DFS passes, lane-private scans, dealt rounds, whole
        // wave, per-step preparation (leaf range, prefix sums, decision), whole FLAT/HYBRID scan
        if (lane == 0 && in_range) {
            atomicAdd(C + 10, (unsigned long long)ct.t_pass);
            atomicAdd(C + 11, (unsigned long long)ct.t_lp);
            atomicAdd(C + 12, (unsigned long long)ct.t_deal);
            atomicAdd(C + 13, (unsigned long long)(clock64() - clk1));
            atomicAdd(C + 14, (unsigned long long)ct.t_prep);
            atomicAdd(C + 15, (unsigned long long)ct.t_scan);
        }
    }
}

#define ATR_INST(SC, C, PR) template __global__ void render_kernel<SC, C, PR>(RenderParams);
#define ATR_INST4(SC) ATR_INST(SC, false, false) ATR_INST(SC, true, false) ATR_INST(SC, false, true) ATR_INST(SC, true, true)
ATR_INST4(SCHED_LANE) ATR_INST4(SCHED_WAVE) ATR_INST4(SCHED_TILE4) ATR_INST4(SCHED_TILE8) ATR_INST4(SCHED_CLUSTER)
ATR_INST4(SCHED_FLAT) ATR_INST4(SCHED_HYBRID)
ATR_INST(SCHED_FLAT_NOCC, false, false) ATR_INST(SCHED_FLAT_NOCC, true, false)
ATR_INST(SCHED_FLAT_UT, false, false) ATR_INST(SCHED_FLAT_UT, true, false)
ATR_INST4(SCHED_FLAT_REGEN)
template __global__ void render_kernel<SCHED_FLAT_REGEN, false, false, 5>(RenderParams);
template __global__ void render_kernel<SCHED_FLAT_ONE, false, false, 6>(RenderParams);
template __global__ void render_kernel<SCHED_FLAT_ONE, false, false, 7>(RenderParams);
template __global__ void render_kernel<SCHED_FLAT_ONE, true, false>(RenderParams);
ATR_INST(SCHED_HYBRID_NOCC, true, true) ATR_INST(SCHED_HYBRID_NOCC, true, false)
ATR_INST(SCHED_HYBRID_NOCC, false, false)

template __global__ void render_kernel<SCHED_HYBRID_NOCC, false, true, 6>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, false, true, 5>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, false, true, 6>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, false, true, 7>(RenderParams);
template __global__ void render_kernel<SCHED_HYBRID, false, false, 5>(RenderParams);
template __global__ void render_kernel<SCHED_FLAT, false, false, 5>(RenderParams);
template __global__ void render_kernel<SCHED_FLAT, false, false, 6>(RenderParams);
template __global__ void render_kernel<SCHED_FLAT, false, false, 7>(RenderParams);
#undef ATR_INST4
#undef ATR_INST
template __global__ void render_kernel<SCHED_LANE, false, true, 5>(RenderParams);
template __global__ void render_kernel<SCHED_LANE, false, true, 6>(RenderParams);
template __global__ void render_kernel<SCHED_LANE, false, true, 8>(RenderParams);
template __global__ void render_kernel<SCHED_CLUSTER, false, true, 5>(RenderParams);
template __global__ void render_kernel<SCHED_CLUSTER, false, true, 6>(RenderParams);
template __global__ void render_kernel<SCHED_CLUSTER, false, true, 8>(RenderParams);
template __global__ void render_kernel<SCHED_CLUSTER_K4, false, true, 4>(RenderParams);
template __global__ void render_kernel<SCHED_CLUSTER_K4, false, true, 5>(RenderParams);
template __global__ void render_kernel<SCHED_CLUSTER_K4, false, true, 6>(RenderParams);
template __global__ void render_kernel<SCHED_CLUSTER_K4, false, true, 8>(RenderParams);

// Sum the 64 traced-ray counters of a cell launch into the caller's accumulator and clear them.
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

// launchers used by capi.cpp
// Default occupancy of the PRIMARY lane kernel (waves/SIMD; chosen by measurement).
constexpr int kPrimaryOcc = 5;
constexpr int kClusterOcc = 5;

template <int SC, bool C, bool PR>
static void launch_one(const atr::RenderParams& P, hipStream_t s) {
    constexpr int NW = atr::sched_waves(SC);
    const int grid = (P.nblocks + NW - 1) / NW;
    hipLaunchKernelGGL((atr::render_kernel<SC, C, PR>), dim3(grid), dim3(64 * NW), 0, s, P);
}

template <int SC>
static void launch_sched(const atr::RenderParams& P, bool count, bool prim, hipStream_t s) {
    if (count) { if (prim) launch_one<SC, true, true>(P, s); else launch_one<SC, true, false>(P, s); }
    else { if (prim) launch_one<SC, false, true>(P, s); else launch_one<SC, false, false>(P, s); }
}

// sched: 0 LANE, 1 WAVE, 2 TILE4, 3 TILE8, 4 CLUSTER; 16 + n: LANE at n waves/SIMD (diagnostic)
extern "C" hipError_t atr_launch_render(const atr::RenderParams& P, int sched, hipStream_t s) {
    if (P.nblocks <= 0) return hipSuccess;
    if (P.traced_rays && P.counters) return hipErrorInvalidValue;  // traced_rays is a ring slot (engine.h)
    const bool count = P.counters != nullptr;
    const bool prim = P.cam.bounce_limit == 1 && !P.cam.anti_aliasing;
    const dim3 g((P.nblocks + 3) / 4), b(256);
    if (sched >= 96) {  // diagnostic: 96 FLAT and 97 HYBRID without candidate compaction (round 2),
                        // 100 FLAT with wave-walked DFS passes on every bounce (FLAT at n waves/SIMD:
                        // 64 + n)
        if (sched == 96) {
            if (prim) return hipErrorInvalidValue;
            if (count) launch_one<atr::SCHED_FLAT_NOCC, true, false>(P, s);
            else launch_one<atr::SCHED_FLAT_NOCC, false, false>(P, s);
        } else if (sched == 97) {
            if (prim && !count) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_HYBRID_NOCC, false, true, 6>), g, b, 0, s, P);
            else if (count) { if (prim) launch_one<atr::SCHED_HYBRID_NOCC, true, true>(P, s); else launch_one<atr::SCHED_HYBRID_NOCC, true, false>(P, s); }
            else launch_one<atr::SCHED_HYBRID_NOCC, false, false>(P, s);
        } else if (sched == 101 || sched == 102) {  // FLAT with path regeneration (102: 5 waves/SIMD)
            if (sched == 102 && !prim && !count)
                hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_FLAT_REGEN, false, false, 5>), g, b, 0, s, P);
            else launch_sched<atr::SCHED_FLAT_REGEN>(P, count, prim, s);
        } else if (sched == 106 || sched == 107) {  // FLAT_ONE at 6 / 7 waves/SIMD (bounce loops only)
            if (prim) return hipErrorInvalidValue;
            if (count) launch_one<atr::SCHED_FLAT_ONE, true, false>(P, s);
            else if (sched == 106) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_FLAT_ONE, false, false, 6>), g, b, 0, s, P);
            else hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_FLAT_ONE, false, false, 7>), g, b, 0, s, P);
        } else if (sched == 100) {
            if (prim) return hipErrorInvalidValue;
            if (count) launch_one<atr::SCHED_FLAT_UT, true, false>(P, s);
            else launch_one<atr::SCHED_FLAT_UT, false, false>(P, s);
        } else {
            return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (sched >= 80) {  // HYBRID at 80 + n waves/SIMD (diagnostic)
        const int o = sched - 80;
        if (!count && o == 5 && prim) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_HYBRID, false, true, 5>), g, b, 0, s, P);
        else if (!count && o == 6 && prim) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_HYBRID, false, true, 6>), g, b, 0, s, P);
        else if (!count && o == 7 && prim) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_HYBRID, false, true, 7>), g, b, 0, s, P);
        else if (!count && o == 5) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_HYBRID, false, false, 5>), g, b, 0, s, P);
        else launch_sched<atr::SCHED_HYBRID>(P, count, prim, s);
        return hipGetLastError();
    }
    if (sched >= 64) {  // FLAT bounce loops at 64 + n waves/SIMD (diagnostic: 4, 5, 6, 7)
        const int o = sched - 64;
        if (!count && o == 7 && !prim) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_FLAT, false, false, 7>), g, b, 0, s, P);
        else if (!count && o == 6 && !prim) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_FLAT, false, false, 6>), g, b, 0, s, P);
        else if (!count && o == 5 && !prim) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_FLAT, false, false, 5>), g, b, 0, s, P);
        else launch_sched<atr::SCHED_FLAT>(P, count, prim, s);
        return hipGetLastError();
    }
    if (sched >= 48) {  // CLUSTER with a 4-entry leaf buffer at 48 + n waves/SIMD (diagnostic)
        const int o = sched - 48;
        if (!prim || count) return hipErrorInvalidValue;
        if (o == 5) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_CLUSTER_K4, false, true, 5>), g, b, 0, s, P);
        else if (o == 6) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_CLUSTER_K4, false, true, 6>), g, b, 0, s, P);
        else if (o == 8) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_CLUSTER_K4, false, true, 8>), g, b, 0, s, P);
        else hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_CLUSTER_K4, false, true, 4>), g, b, 0, s, P);
        return hipGetLastError();
    }
    if (sched >= 32) {  // CLUSTER at 32 + n waves/SIMD (diagnostic)
        const int o = sched - 32;
        if (prim && !count && o == 5) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_CLUSTER, false, true, 5>), g, b, 0, s, P);
        else if (prim && !count && o == 6) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_CLUSTER, false, true, 6>), g, b, 0, s, P);
        else if (prim && !count && o == 8) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_CLUSTER, false, true, 8>), g, b, 0, s, P);
        else launch_sched<atr::SCHED_CLUSTER>(P, count, prim, s);
        return hipGetLastError();
    }
    int occ = sched >= 16 ? sched - 16 : (sched == 0 ? kPrimaryOcc : 0);
    if (sched >= 16) sched = 0;
    if (sched == 0 && prim && !count && occ != 4) {
        if (occ == 5) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_LANE, false, true, 5>), g, b, 0, s, P);
        else if (occ == 6) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_LANE, false, true, 6>), g, b, 0, s, P);
        else hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_LANE, false, true, 8>), g, b, 0, s, P);
        return hipGetLastError();
    }
    switch (sched) {
        case 1: launch_sched<atr::SCHED_WAVE>(P, count, prim, s); break;
        case 6:  // bounce loops: one frame at 6 waves/SIMD (80 VGPRs; its slowest cells set the latency),
                 // frames in flight at 7 (72 VGPRs, the LDS limit: 7 x 22.5 KB per CU). The
                 // spills (54 / 83 dwords) cost less than the latency the extra waves hide: c4 1,376 ->
                 // 1,536 (6) -> 1,630 (7) Mrays/s
            if (!prim && !count && P.frame_blocks > 0)
                hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_FLAT, false, false, 7>), g, b, 0, s, P);
            else if (!prim && !count) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_FLAT, false, false, 6>), g, b, 0, s, P);
            else launch_sched<atr::SCHED_FLAT>(P, count, prim, s);
            break;
        case 7:  // primaries: one frame at 6 waves/SIMD (its slowest cells set the latency), frames in
                 // flight at 7 (72 VGPRs: throughput)
            if (prim && !count && P.frame_blocks > 0)
                hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_HYBRID, false, true, 7>), g, b, 0, s, P);
            else if (prim && !count) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_HYBRID, false, true, 6>), g, b, 0, s, P);
            else launch_sched<atr::SCHED_HYBRID>(P, count, prim, s);
            break;
        case 2: launch_sched<atr::SCHED_TILE4>(P, count, prim, s); break;
        case 3: launch_sched<atr::SCHED_TILE8>(P, count, prim, s); break;
        case 4:
            if (prim && !count) hipLaunchKernelGGL((atr::render_kernel<atr::SCHED_CLUSTER, false, true, kClusterOcc>), g, b, 0, s, P);
            else launch_sched<atr::SCHED_CLUSTER>(P, count, prim, s);
            break;
        default: launch_sched<atr::SCHED_LANE>(P, count, prim, s); break;
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
