// scan.h -- the tree queries every render kernel builds on (get_intersection_data,
// renderer.cpp:34-160 -> get_ray_kd_tree_intersection -> traverse_oct_tree_new, kd_tree.cpp:302-465).
//
// Two bit-identical schedules of the leaf scan (the hot loop, kd_tree.cpp:437-462):
//   LANE: every lane walks its own sorted leaves and tests every triangle of each (the reference's
//         exact work; per-lane SoA loads);
//   FLAT / HYBRID (tree_closest_flat): the clustered scan (cluster.h) with the
//         wavefront's (ray, cluster) work dealt over its 64 lanes, candidates compacted (§4d-§4f).
// Shared by the cell kernels (render.hip) and the sample-parallel path kernels (paths.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "cluster.h"
#include "shade.h"
#include "trace.h"

namespace atr {

// ------------------------------------------------------------------ LANE schedule
// Per-lane leaf scan over the SoA triangle streams, software-pipelined two deep with two register
// sets used alternately (the loads of the next triangle stay in flight while the current one is
// tested). The hit keeps the primitive SLOT; its face index is read once, after the tree query.
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
    if (dist < best_t && dist > kTol) {  // kd_tree.cpp:450: strict <, the first in leaf order wins
        best_t = dist;
        best_slot = slot;
        bu = u;
        bv = v;
        improved = true;
    }
}

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

// get_ray_kd_tree_intersection (kd_tree.cpp:302-335) for one lane: DFS passes into an LDS leaf
// buffer (a lane-private column, 64 B per lane), sorted leaves scanned in order, stop after the
// first leaf that improved the hit (:457-460).
template <bool COUNT, int K = kLeafBuf>
__device__ __forceinline__ void tree_closest_lane(const Ray& r, const DModel& m, Hit& h, int& err, Ctr& ct) {
    h.t = kMaxFloat;
    h.face = 0;
    h.u = h.v = 0.f;
    const NodeBox root = load_node(m.nodes, 0);
    if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
    if (!box_check(r, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) return;  // :339
    uint32_t slot = 0xFFFFFFFFu;
    auto scan = [&](int32_t leaf) -> bool {
        return scan_leaf_lane<COUNT>(r, m, m.leaf_range[2 * leaf], m.leaf_range[2 * leaf + 1], h.t, slot, h.u,
                                     h.v, ct);
    };
    if (root.children == 0) {  // :344-361
        scan(0);
    } else {
        float bd = -__builtin_inff();
        int32_t bi = -1;
        bool more = true;
        __shared__ float s_lbd[4][K][64];
        __shared__ int32_t s_lbl[4][K][64];
        const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
        while (more) {
            int32_t n;
            {
                LdsLeafBuf<K> lb;
                lb.d = &s_lbd[w][0][ln];
                lb.leaf = &s_lbl[w][0][ln];
                n = traverse_pass<K, COUNT>(r, m.inner, lb, bd, bi, ct);
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
    if (slot != 0xFFFFFFFFu) h.face = m.tface[slot];
}

// ------------------------------------------------------------------ FLAT / HYBRID schedule
// The clustered scan with the wavefront's (ray, cluster) work flattened over its lanes
// (DESIGN.md §4d-§4f). Each lane owns a ray's query (DFS passes, its sorted leaves, the
// first-improving-leaf rule); the clusters of all rays' current leaves are dealt to the 64 lanes in
// rounds, each lane running one cluster's padded boxes and screen on the owner's ray (lane
// shuffles), and the surviving candidates are compacted over the wave for the full tests. Results
// merge per owner in LDS as the minimum (t, leaf rank) -- the first primitive in leaf order with
// the smallest t (kd_tree.cpp:440-456) -- so every output is the reference's, bit for bit.
__device__ __forceinline__ float shfl_f(float v, int src) { return __shfl(v, src); }

// Wave-wide inclusive scans on the DPP row network (GFX9 rows of 16 lanes: shifts by 1, 2, 4, 8
// within a row, then the broadcasts of lanes 15 and 31 into the rows above): six dependent VALU
// steps, where a __shfl_up step is an LDS permute round trip. Lanes shifted in from outside a row,
// and rows outside the mask, contribute the identity (`old`).
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

// Phase clocks of the FLAT/HYBRID scans (atr_render_phase_clocks): compiled only into the
// diagnostic build (make DIAG=1). In the product build the statements vanish; even discarded under
// `if constexpr` they changed the product kernel's register allocation.
#ifdef ATR_PHASE_CLOCKS
#define ATR_PCLK(...) __VA_ARGS__
#else
#define ATR_PCLK(...)
#endif

// LDS of the FLAT/HYBRID scans (22.5 KB per 4-wave workgroup): the leaf order buffers (lane-private
// columns), the per-owner best keys and hit records, the round's owner markers.
// The hit's barycentrics per owner (an empty base when no output needs them: the primary-only
// kernels' LDS is then 20 KB per workgroup, so 8 of them fit a CU's 160 KB).
template <bool UV>
struct FlatUV {
    float u[4][64], v[4][64];
};
template <>
struct FlatUV<false> {};
template <int K = kLeafBuf, bool UV = true>
struct FlatLds : FlatUV<UV> {
    float lbd[4][K][64];
    int32_t lbl[4][K][64];
    unsigned long long key[4][64];
    uint32_t slot[4][64];
    int32_t mark[4][64];
};
template <int K = kLeafBuf, bool UV = true>
__device__ __forceinline__ FlatLds<K, UV>& flat_lds() {
    __shared__ FlatLds<K, UV> L;
    return L;
}

constexpr unsigned long long kKeyInit = (static_cast<unsigned long long>(0x7F7FFFFFu) << 32) | 0xFFFFFFFFull;

// One full test of candidate `slot` for the ray q of owner lane `ow`: lowers the owner's (t bits,
// leaf rank) key in LDS -- the minimum over the leaf in any order is the reference's
// first-in-leaf-order closest hit (kd_tree.cpp:440-456); true if this test lowered it.
template <bool COUNT, int K = kLeafBuf, bool UV = true>
__device__ __forceinline__ bool cand_test(const Ray& q, const DModel& m, int w, int32_t ow, uint32_t slot,
                                          unsigned long long& mine, float& u, float& v, Ctr& ct) {
    FlatLds<K, UV>& L = flat_lds<K, UV>();
    if constexpr (COUNT) ct.tri += 1;
    float4_t a0, a1, a2;
    load_prim(m, slot, a0, a1, a2);
    const float dist = tri_hit(q, mk(a0.x, a0.y, a0.z), mk(a0.w, a1.x, a1.y), mk(a1.z, a1.w, a2.x), u, v);
    if (dist > kTol && dist < kMaxFloat) {  // accepted (model.h:75-103; kd_tree.cpp:450)
        mine = (static_cast<unsigned long long>(__float_as_uint(dist)) << 32) | uint32_t(__float_as_int(a2.y));
        if (mine < L.key[w][ow]) {
            atomicMin(&L.key[w][ow], mine);
            return true;
        }
    }
    return false;
}

// Full tests of a step's candidates. Each lane holds one (ray, cluster) item that passed the padded
// boxes and the screen with candidate mask `cm` (slots cfirst + bit, ray of lane `own`; SELF: every
// lane's item is its own ray, the lane-private scan). Two schedules, chosen wave-uniformly (in place
// only with SELF: in dealt steps it measured no use and its registers spilled), same result (the minimum key
// does not depend on the order of the tests; the rank in the key makes keys unique within a leaf):
//   in place -- when no lane holds more candidates than the compacted schedule would need
//               sub-rounds, each lane tests its own candidates one per iteration (no numbering,
//               owner lookup or ray shuffles per test);
//   compacted -- the wave's candidates are numbered by a prefix sum of the masks' popcounts and
//               dealt 64 per sub-round, one full test per lane.
// The winning test of each (sub-)round writes its owner's slot and barycentrics. UO: every ray of
// the wave has the same origin (camera rays).
template <bool COUNT, bool UO, bool NUV, bool SELF = false, int K = kLeafBuf>
__device__ __forceinline__ void cand_rounds(const Ray& r, const DModel& m, int w, int ln, uint32_t cm,
                                            uint32_t cfirst, int32_t own, Ctr& ct) {
    FlatLds<K, !NUV>& L = flat_lds<K, !NUV>();
    const uint32_t cc = uint32_t(__popc(cm));
    constexpr bool kInPlace = SELF;
#ifndef ATR_INPLACE_FACTOR
#define ATR_INPLACE_FACTOR 2
#endif
    // in place while every lane holds fewer than F x (compacted sub-rounds) candidates: an
    // in-place iteration skips the numbering, owner lookup and shuffles of a sub-round (c3: in
    // place up to 1 x the sub-rounds 7,618-7,735 Mrays/s, below 2 x 7,746-7,858)
    uint32_t cinc = 0, total = 0, most;
    bool inplace;
    if (kInPlace && __ballot(cc > 1u) == 0) {  // at most one candidate per lane: in place, no scans
        most = __ballot(cc != 0u) ? 1u : 0u;    // (c3 +2%)
        inplace = true;
    } else {
        cinc = wave_incl_add(cc);
        total = uint32_t(__builtin_amdgcn_readlane(int(cinc), 63));
        most = kInPlace ? uint32_t(__builtin_amdgcn_readlane(wave_incl_max(int32_t(cc)), 63)) : 64u;
        inplace = kInPlace && most < ATR_INPLACE_FACTOR * ((total + 63u) >> 6);
    }
    if (inplace) {
        Ray q;
        q.o = r.o;
        q.d = r.d;
        uint32_t x = cm;
        for (uint32_t it = 0; it < most; ++it) {  // wave-uniform
            const bool valid = x != 0;
            const uint32_t slot = cfirst + (valid ? uint32_t(__builtin_ctz(x)) : 0u);
            x &= x - 1u;
            if constexpr (COUNT) ct.cand_wave += ln == 0 ? 1u : 0u;
            unsigned long long mine = kKeyInit;
            bool imp = false;
            float u = 0.f, v = 0.f;
            if (valid) imp = cand_test<COUNT, K, !NUV>(q, m, w, own, slot, mine, u, v, ct);
            __builtin_amdgcn_wave_barrier();
            if (imp && L.key[w][own] == mine) {  // this iteration's winner for its owner
                L.slot[w][own] = slot;
                if constexpr (!NUV) {
                    L.u[w][own] = u;
                    L.v[w][own] = v;
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        return;
    }
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
        if constexpr (kMaxClusterSize > 16) {
            n = uint32_t(__popc(x & 0xFFFFu)); if (j >= n) { j -= n; x >>= 16; b += 16; }
        }
        n = uint32_t(__popc(x & 0xFFu)); if (j >= n) { j -= n; x >>= 8; b += 8; }
        n = uint32_t(__popc(x & 0xFu)); if (j >= n) { j -= n; x >>= 4; b += 4; }
        n = uint32_t(__popc(x & 0x3u)); if (j >= n) { j -= n; x >>= 2; b += 2; }
        b += j >= (x & 1u) ? 1u : 0u;
        const uint32_t slot = uint32_t(__shfl(int(cfirst), s2)) + b;
        const int32_t ow = __shfl(own, s2);
        Ray q;
        q.o = UO ? r.o : mk(shfl_f(r.o.x, ow), shfl_f(r.o.y, ow), shfl_f(r.o.z, ow));
        q.d = mk(shfl_f(r.d.x, ow), shfl_f(r.d.y, ow), shfl_f(r.d.z, ow));
        unsigned long long mine = kKeyInit;
        bool imp = false;
        float u = 0.f, v = 0.f;
        if (valid) {
            if constexpr (COUNT) { ct.tri += 1; ct.cand_wave += ln == 0 ? 1u : 0u; }
            float4_t a0, a1;
            float4_t a2;
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

// The pieces of a clustered tree query (tree_closest_flat below; the path engine's bounce kernel
// runs them in its own loop). Per lane: `done` (no query, or the query finished), `need` (a DFS pass
// is due: the first, or a re-walk after a full buffer), j / nb / more (the current leaf of the
// buffer, its fill, whether the pass found more than fits), `rewalk` (the buffer's last entry is the
// next pass's bound). The result stays in the lane's LDS key/slot/u/v row (flat_result).

// Start a query: the root box (kd_tree.cpp:339), the root leaf alone (:344-361) or a first pass.
struct FlatQ {
    int32_t j, nb;
    bool done, need, more, rewalk;
};

template <bool COUNT, int K = kLeafBuf, bool UV = true>
__device__ __forceinline__ FlatQ flat_begin(const Ray& r, const DModel& m, bool active, int w, int ln, Ctr& ct) {
    FlatLds<K, UV>& L = flat_lds<K, UV>();
    FlatQ q{0, 0, true, false, false, false};
    L.key[w][ln] = kKeyInit;
    if (active) {
        const NodeBox root = load_node(m.nodes, 0);
        if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
        if (box_check(r, root.lx, root.ly, root.lz, root.hx, root.hy, root.hz)) {
            q.done = false;
            if (root.children == 0) {  // the root leaf (discovery rank 0) alone
                L.lbl[w][0][ln] = 0;
                L.lbd[w][0][ln] = 0.f;
                q.nb = 1;
            } else {
                q.need = true;
            }
        }
    }
    return q;
}

// One DFS pass (kd_tree.cpp:363-435) for every lane with `need`; its sorted leaves wait in LDS.
// UT: the wave walks its passes together (traverse_pass_wave: coherent rays). LDSB: the pass inserts
// straight into the LDS columns. NEAR (with LDSB): near-first passes (traverse_pass_near).
template <bool COUNT, bool LDSB, bool UT, bool NEAR, int K = kLeafBuf, bool UV = true>
__device__ __forceinline__ void flat_pass(const Ray& r, const DModel& m, int w, int ln, FlatQ& q, int& err, Ctr& ct) {
    FlatLds<K, UV>& L = flat_lds<K, UV>();
    // the re-walk bound: the last leaf of the previous pass's full buffer (entry K - 1 of the column)
    const float bd = q.rewalk ? L.lbd[w][K - 1][ln] : -__builtin_inff();
    const int32_t bi = q.rewalk ? L.lbl[w][K - 1][ln] : -1;
    auto took = [&](int32_t n) {  // the pass's leaves are the lane's buffer now
        q.need = false;
        q.j = 0;
        if (n < 0) { err = 1; q.done = true; }
        else { q.nb = n < K ? n : K; q.more = n > K; if (q.nb == 0) q.done = true; }
    };
    if constexpr (UT) {
        if (__ballot(q.need)) {
            LdsLeafBuf<K> lb;
            lb.d = &L.lbd[w][0][ln];
            lb.leaf = &L.lbl[w][0][ln];
            const int32_t n = traverse_pass_wave<K, COUNT>(r, m.inner, lb, bd, bi, ct, q.need);
            if (q.need) took(n);
        }
    } else if (q.need) {
        int32_t n;
        if constexpr (LDSB) {
            LdsLeafBuf<K> lb;
            lb.d = &L.lbd[w][0][ln];
            lb.leaf = &L.lbl[w][0][ln];
            if (NEAR && m.near_ok) n = traverse_pass_near<K, COUNT>(r, m.inner, lb, bd, bi, ct);
            else n = traverse_pass<K, COUNT>(r, m.inner, lb, bd, bi, ct);
        } else {  // register buffer: the LDS one measured 5% slower for incoherent bounce rays
            LeafBuf<K> lb;
            n = traverse_pass<K, COUNT>(r, m.inner, lb, bd, bi, ct);
#pragma unroll
            for (int t = 0; t < K; ++t) { L.lbd[w][t][ln] = lb.d[t]; L.lbl[w][t][ln] = lb.leaf[t]; }
        }
        took(n);
    }
}

// One leaf step of every lane with `live` (a query under way whose buffer is current): the
// clusters of each such lane's current leaf, scanned lane-private or dealt over the wave (HYB
// decides per step, wave-uniformly: deal when the largest cluster count exceeds hyb_a x rounds +
// hyb_b; without HYB every step deals), candidates compacted. A leaf's result does not depend on
// the visiting order (minimum (t, leaf rank)), so the choice changes no output bit. Then each live
// lane stops at the first leaf that improved its hit (kd_tree.cpp:457-460), moves to its next
// leaf, or asks for a re-walk. UO: one origin for the whole wave. NUV: u and v feed no output.
template <bool COUNT, bool HYB, bool UO, bool NUV, int K = kLeafBuf>
__device__ __forceinline__ void flat_leaf_step(const Ray& r, const DModel& m, int w, int ln, bool live, FlatQ& q,
                                               Ctr& ct, int32_t hyb_a, int32_t hyb_b) {
    FlatLds<K, !NUV>& L = flat_lds<K, !NUV>();
    // flavour of the scan (primary-only, camera, bounce rays) -> early screen normals (cluster.h)
    constexpr bool kEarly = ((NUV ? 1 : UO ? 2 : 4) & ATR_EARLY_NRM) != 0;
    ATR_PCLK(const uint64_t tc2 = clock64());
    uint32_t cf = 0, cn = 0;
    if (live) {
        const uint2_t cr = load_range(m.cl_range, L.lbl[w][q.j][ln]);
        cf = cr.x;
        cn = cr.y;
        if constexpr (COUNT) { ct.leaf += 1; ct.cbox += cn; }
    }
    const uint32_t incl = wave_incl_add(cn);  // inclusive prefix sum over the lanes
    const uint32_t excl = incl - cn;
    const uint32_t total = uint32_t(__builtin_amdgcn_readlane(int(incl), 63));
    if (live) L.key[w][ln] = kKeyInit;
    bool deal = true;
    if constexpr (HYB) {
        // the largest cluster count of the step (counts are small: the signed max is exact)
        const uint32_t mx = uint32_t(__builtin_amdgcn_readlane(wave_incl_max(int32_t(cn)), 63));
        deal = int32_t(mx) > hyb_a * int32_t((total + 63u) >> 6) + hyb_b;
    }
    ATR_PCLK(const uint64_t tc1 = clock64());
    ATR_PCLK(ct.t_prep += uint32_t(tc1 - tc2));
    if (!deal) {  // every lane scans its own leaf's clusters, one per iteration; the candidates
                  // of each iteration are compacted over the wave
        const uint32_t mxc = uint32_t(__builtin_amdgcn_readlane(wave_incl_max(int32_t(cn)), 63));
        for (uint32_t i = 0; i < mxc; ++i) {
            uint32_t cm = 0;
            if (i < cn) {
                const uint32_t c = cf + i;
                const float bound = __uint_as_float(uint32_t(L.key[w][ln] >> 32));
                cm = cluster_cands<COUNT, kEarly>(r, m, c, m.clus[kClusterBlock * size_t(c)],
                                          m.clus[kClusterBlock * size_t(c) + 1], bound, ct);
            }
            cand_rounds<COUNT, UO, NUV, true, K>(r, m, w, ln, cm, kMaxClusterSize * (cf + i), ln, ct);
        }
    }
    ATR_PCLK(if (!deal) ct.t_lp += uint32_t(clock64() - tc1));
    int32_t carry = -1;
    for (uint32_t base = 0; deal && base < total; base += 64) {  // rounds of 64 items, wave-uniform
        L.mark[w][ln] = -1;
        __builtin_amdgcn_wave_barrier();
        if (cn > 0 && excl >= base && excl < base + 64u) L.mark[w][excl - base] = ln;
        __builtin_amdgcn_wave_barrier();
        int32_t own = wave_incl_max(L.mark[w][ln]);  // latest owner starting at or before this lane
        if (own < 0) own = carry;
        carry = __builtin_amdgcn_readlane(own, 63);
        const uint32_t k = base + uint32_t(ln);
        const bool valid = k < total;
        if constexpr (COUNT) { ct.round_wave += ln == 0 ? 1u : 0u; ct.round_items += valid ? 1u : 0u; }
        const int32_t src = valid ? own : ln;
        Ray qr;  // the owner's ray
        qr.o = UO ? r.o : mk(shfl_f(r.o.x, src), shfl_f(r.o.y, src), shfl_f(r.o.z, src));
        qr.d = mk(shfl_f(r.d.x, src), shfl_f(r.d.y, src), shfl_f(r.d.z, src));
        qr.inv = mk(shfl_f(r.inv.x, src), shfl_f(r.inv.y, src), shfl_f(r.inv.z, src));
        qr.s0 = qr.inv.x < 0;
        qr.s1 = qr.inv.y < 0;
        qr.s2 = qr.inv.z < 0;
        const uint32_t c = uint32_t(__shfl(int(cf), src)) + (k - uint32_t(__shfl(int(excl), src)));
        uint32_t cm = 0;
        if (valid) {
            const float bound = __uint_as_float(uint32_t(L.key[w][own] >> 32));
            cm = cluster_cands<COUNT, kEarly>(qr, m, c, m.clus[kClusterBlock * size_t(c)], m.clus[kClusterBlock * size_t(c) + 1],
                                      bound, ct);
        }
        cand_rounds<COUNT, UO, NUV, false, K>(r, m, w, ln, cm, kMaxClusterSize * c, own, ct);
    }
    ATR_PCLK(if (deal) ct.t_deal += uint32_t(clock64() - tc1));
    if (live) {  // stop at the first leaf that improved the hit (kd_tree.cpp:457-460)
        if (L.key[w][ln] != kKeyInit) {
            q.done = true;
        } else if (++q.j >= q.nb) {
            if (q.more) q.need = q.rewalk = true;  // the next K leaves after this buffer's last
            else q.done = true;
        }
    }
    __builtin_amdgcn_wave_barrier();
}

// The lane's result from its LDS row (t = kMaxFloat: no hit).
template <bool NUV, int K = kLeafBuf>
__device__ __forceinline__ void flat_result(const DModel& m, bool active, int w, int ln, Hit& h) {
    FlatLds<K, !NUV>& L = flat_lds<K, !NUV>();
    h.t = kMaxFloat;
    h.face = 0;
    h.u = h.v = 0.f;
    const unsigned long long key = L.key[w][ln];
    if (active && key != kKeyInit) {
        h.t = __uint_as_float(uint32_t(key >> 32));
        if constexpr (!NUV) {
            h.u = L.u[w][ln];
            h.v = L.v[w][ln];
        }
        h.face = __float_as_uint(m.prim[3 * size_t(L.slot[w][ln]) + 2].z);
    }
}

// One tree query of every active lane of the wave (called by all 64 lanes, converged): passes and
// leaf steps until every lane's query is done. Flags as above.
template <bool COUNT, bool HYB = false, bool LDSB = false, bool UO = false, bool UT = false, bool NUV = false,
          bool NEAR = false, int K = kLeafBuf>
__device__ __forceinline__ void tree_closest_flat(const Ray& r, const DModel& m, bool active, Hit& h, int& err,
                                                  Ctr& ct, int32_t hyb_a = 0, int32_t hyb_b = 0) {
    const int w = threadIdx.x >> 6, ln = threadIdx.x & 63;
    ATR_PCLK(uint64_t tcs = clock64());
    FlatQ q = flat_begin<COUNT, K, !NUV>(r, m, active, w, ln, ct);
    for (;;) {
        ATR_PCLK(const uint64_t tc0 = clock64());
        flat_pass<COUNT, LDSB, UT, NEAR, K, !NUV>(r, m, w, ln, q, err, ct);
        ATR_PCLK(ct.t_pass += uint32_t(clock64() - tc0));
        if (__ballot(!q.done) == 0) break;
        flat_leaf_step<COUNT, HYB, UO, NUV, K>(r, m, w, ln, !q.done, q, ct, hyb_a, hyb_b);
    }
    flat_result<NUV, K>(m, active, w, ln, h);
    ATR_PCLK(ct.t_scan += uint32_t(clock64() - tcs));
}

// ------------------------------------------------------------------ get_intersection_data
enum { SCHED_LANE = 0, SCHED_FLAT = 6, SCHED_HYBRID = 7 };
// Flavours of the clustered scan: CAMERA rays (one origin, coherent: HYBRID's wave-walked passes,
// LDS leaf buffer), BOUNCE rays (incoherent: dealt rounds, register leaf buffer), PRIMARY-only
// frames (CAMERA without u and v).
enum { FLAV_CAMERA = 0, FLAV_BOUNCE = 1, FLAV_PRIMARY = 2, FLAV_HYB_BOUNCE = 3 };
#ifndef ATR_BOUNCE_HYB  // experiment builds: 1 = the path engine's bounce rays choose lane-private or
#define ATR_BOUNCE_HYB 0  // dealt leaf steps per step as HYBRID does (thresholds hybrid_a, hybrid_b)
#endif

// A model's table pointers as wave-uniform GLOBAL pointers (uniform_global, trace.h): read once per
// query into SGPRs and cast to the global address space (through the DScene reference the compiler
// re-loaded each pointer with a vector load before every use and issued flat loads).
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
    m.prim = uniform_global(m.prim);
    return m;
}

// The models' closest triangle (renderer.cpp:34-82): best t, face, barycentrics, model (-1: none).
struct SceneHit {
    float best, fu, fv;
    uint32_t face;
    int32_t nm;
};

// get_intersection_data (renderer.cpp:34-160) for every lane of the wave (converged call; inactive
// lanes take part in the wave-wide scans). SCHED_LANE: per-lane reference scan; otherwise the
// clustered scan in flavour FLAV. intersect_models is the models' part; scene_finish (shade.h) the
// spheres, planes and hit record, so a caller can re-read o and d between the two instead of
// holding them through the query.
template <int SCHED, int FLAV, bool COUNT, int KB = kLeafBuf>
__device__ __forceinline__ SceneHit intersect_models(const DScene* __restrict__ S, V3 o, V3 d, bool active, int& err,
                                                    Ctr& ct, int32_t hyb_a, int32_t hyb_b) {
    const Ray r = make_ray(o, d);  // renderer.cpp:41-44
    SceneHit sh{kMaxFloat, 0.f, 0.f, 0u, -1};
    const int32_t nmodels = __builtin_amdgcn_readfirstlane(S->nmodels);  // uniform: an SGPR, not a VGPR
    for (int32_t i = 0; i < nmodels; ++i) {
        const DModel m = uniform_model(S->models[i]);
        if (m.has_tree) {  // USE_KD_TREE (:49-57)
            Hit h;
            if constexpr (SCHED == SCHED_LANE) {
                if (active) tree_closest_lane<COUNT>(r, m, h, err, ct);
                else h.t = kMaxFloat;
            } else if constexpr (FLAV == FLAV_CAMERA)
                tree_closest_flat<COUNT, true, true, true, true, false>(r, m, active, h, err, ct, hyb_a, hyb_b);
            else if constexpr (FLAV == FLAV_PRIMARY)
                tree_closest_flat<COUNT, true, true, true, true, true>(r, m, active, h, err, ct, hyb_a, hyb_b);
            else if constexpr (FLAV == FLAV_HYB_BOUNCE)
                tree_closest_flat<COUNT, true, false, false, false, false>(r, m, active, h, err, ct, hyb_a, hyb_b);
            else  // bounce rays: near-first passes into the LDS leaf buffer, every step dealt
                tree_closest_flat<COUNT, ATR_BOUNCE_HYB != 0, true, false, false, false, true, KB>(r, m, active, h, err, ct,
                                                                                         hyb_a, hyb_b);
            if (h.t > kTol && h.t < sh.best) { sh.best = h.t; sh.face = h.face; sh.fu = h.u; sh.fv = h.v; sh.nm = i; }
        } else if (active) {  // brute force (:58-82), face-ordered triangles, uniform loads
            if constexpr (COUNT) { ct.box += 1; ct.box_all += 1; }
            if (box_entry(r, m.aabb[0], m.aabb[1], m.aabb[2], m.aabb[3], m.aabb[4], m.aabb[5]) != 0) {
                if constexpr (COUNT) { ct.tri += m.nfaces; }
                for (uint32_t j = 0; j < m.nfaces; ++j) {
                    const DTri* t = m.tris + j;
                    float u = 0.f, v = 0.f;
                    const float tt = tri_hit(r, mk(t->ax, t->ay, t->az), mk(t->abx, t->aby, t->abz),
                                             mk(t->acx, t->acy, t->acz), u, v);
                    if (tt > kTol && tt < sh.best) { sh.best = tt; sh.fu = u; sh.fv = v; sh.face = j; sh.nm = i; }
                }
            }
        }
    }
    return sh;
}

template <int SCHED, int FLAV, bool COUNT>
__device__ __forceinline__ void intersect_scene(const DScene* __restrict__ S, V3 o, V3 d, bool active, Isect& id,
                                                int& err, Ctr& ct, int32_t hyb_a, int32_t hyb_b) {
    const SceneHit sh = intersect_models<SCHED, FLAV, COUNT>(S, o, d, active, err, ct, hyb_a, hyb_b);
    if (!active) return;
    scene_finish(S, o, d, sh.best, sh.face, sh.fu, sh.fv, sh.nm, id);  // :86-160
}

// One non-sky bounce of cast_ray (renderer.cpp:231-258): the new ray and the path's colour and
// throughput, f32 operations in the reference's order.
__device__ __forceinline__ void bounce_shade(const DMaterial& mat, const Isect& id, V3& o, V3& d, V3& ret, V3& w,
                                             uint64_t& st, uint64_t stream) {
    const V3 emission = mk(mat.ex, mat.ey, mat.ez);
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

// Wave sum of a per-lane counter added to one of 64 counters 128 B apart (atr_launch_traced_finish
// adds them up): one address taking every wave's add serializes ~0.1 ms per frame at the L2.
__device__ __forceinline__ void add_traced(unsigned long long* slots, uint32_t t, int spread) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
    if ((threadIdx.x & 63) == 0 && t) atomicAdd(slots + 16 * (spread & 63), (unsigned long long)t);
}

}  // namespace atr
